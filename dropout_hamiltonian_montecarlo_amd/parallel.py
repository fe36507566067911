"""One process per GPU, independent chains, one collective at the end.

The reference's multi-chain layer (/root/reference/hamiltonian/inference/cpu/sghmc_multicore.py,
sgld_multicore.py, hmc_multicore.py: multiprocessing.Pool, RandomState(i) per worker,
posteriors concatenated; all broken as shipped) becomes:

* chains are sharded over ranks (chain c → rank c mod world_size); each rank samples its chains
  on its own GPU with NO communication while sampling (embarrassingly parallel);
* after sampling, ONE all-gather (RCCL over xGMI when the backend is "nccl", gloo on CPU) moves
  the per-chain traces / summaries to every rank; rank 0 computes split-R̂ and ESS.

Rendezvous: torch.distributed env:// (RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT).
"""
import os

import numpy as np
import torch
import torch.distributed as dist

from . import diagnostics


def init(backend=None):
    """Initialise the process group from the environment; returns (rank, world, local_rank).
    Backend: `backend`, else $HMCX_DIST_BACKEND, else "nccl" (RCCL) with a GPU and "gloo" without."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = os.environ.get("HMCX_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def backend_name():
    if not dist.is_initialized():
        return "none"
    b = dist.get_backend()
    return "nccl (RCCL over xGMI)" if b == "nccl" else b


def chains_of_rank(n_chains, rank, world):
    """Chain ids sampled by `rank` (round-robin, matching RandomState(i) per worker)."""
    return list(range(rank, n_chains, world))


def barrier():
    if dist.is_initialized():
        dist.barrier()


def _dev(device):
    """Collectives run on `device` with RCCL; gloo takes host tensors."""
    if dist.is_initialized() and dist.get_backend() == "gloo":
        return torch.device("cpu")
    return device


def allreduce_max(x, device=None):
    if not dist.is_initialized():
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=_dev(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allreduce_sum(x, device=None):
    if not dist.is_initialized():
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=_dev(device))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def gather_traces(local_traces, device=None):
    """All-gather per-chain traces.  local_traces: array [c_local, T, P] (same c_local, T, P on
    every rank) → array [world·c_local, T, P] ordered by (rank, local chain)."""
    x = torch.as_tensor(np.ascontiguousarray(local_traces), dtype=torch.float64)
    if not dist.is_initialized():
        return x.numpy()
    device = _dev(device)
    x = x.to(device) if device is not None else x
    out = [torch.empty_like(x) for _ in range(dist.get_world_size())]
    dist.all_gather(out, x)
    return torch.cat(out, dim=0).cpu().numpy()


def chain_diagnostics(all_traces):
    """split-R̂ and ESS per traced quantity over all gathered chains ([C, T, P])."""
    x = np.asarray(all_traces, dtype=np.float64)
    return {"rhat": diagnostics.split_rhat(x), "ess": diagnostics.ess(x)}
