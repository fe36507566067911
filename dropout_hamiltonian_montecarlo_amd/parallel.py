"""One process per GPU, independent chains, one collective at the end.

The reference's multi-chain layer (/root/reference/hamiltonian/inference/cpu/sghmc_multicore.py,
sgld_multicore.py, hmc_multicore.py: multiprocessing.Pool, RandomState(i) per worker,
posteriors concatenated; all broken as shipped) becomes:

* chains are sharded over ranks in contiguous blocks (rank r samples chains chain0 .. chain0+c−1,
  chain_block) — the samplers key their Philox streams by chain0 + c, so blocks never overlap;
  each rank samples its chains on its own GPU with NO communication while sampling
  (embarrassingly parallel);
* after sampling, ONE all-gather moves the per-chain summaries — per-parameter mean and Welford M2
  over the draws, and a thinned trace (the reference concatenates whole posteriors,
  sghmc_multicore.py:86-94) — to every rank; rank 0 computes per-parameter R̂ / split-R̂ and ESS.

Two planes:

* control — torch.distributed over gloo (env:// rendezvous: RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1,
  MASTER_PORT): barriers, the uneven-block counts, and handing rank 0's RCCL unique id to the
  other ranks.  No tensor data of the run goes through it on a GPU run;
* data — RCCL over xGMI through libhmcx's C ABI (init_rccl → hmcx_comm_init; gather_summaries /
  gather_traces → hmcx_allgather_chain_stats; allreduce_max / allreduce_sum → hmcx_allreduce_f64),
  on the hmcx context's stream.  Without a GPU (CPU tests) or with HMCX_DIST_BACKEND=gloo (several
  ranks sharing one GPU, which RCCL refuses) the same functions run over gloo.
"""
import os

import numpy as np
import torch
import torch.distributed as dist

from . import diagnostics


_rccl = None          # the data-plane communicator (RcclComm) once init_rccl has made it


def init(backend="gloo"):
    """Initialise the control-plane process group (gloo) from the environment; returns (rank, world,
    local_rank).  One rank normally runs without a process group; HMCX_DIST_FORCE=1 creates it anyway
    (world 1: the collective path of the multi-GPU run, exercised on one GPU)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    force = os.environ.get("HMCX_DIST_FORCE") == "1"
    if (world > 1 or force) and not dist.is_initialized():
        dist.init_process_group(backend)
    return rank, world, local


class RcclComm:
    """An RCCL communicator owned by libhmcx (include/hmcx.h hmcx_comm_*)."""

    def __init__(self, ctx, handle, world, rank):
        self.ctx, self.h, self.world, self.rank = ctx, handle, world, rank

    def allgather(self, x):
        """x: device float64 tensor [n] → [world, n] (rank order)."""
        from ._native import ptr
        x = x.contiguous()
        out = torch.empty((self.world,) + tuple(x.shape), dtype=torch.float64, device=x.device)
        self.ctx.bind_stream()
        self.ctx.check(self.ctx.lib.hmcx_allgather_chain_stats(self.ctx.h, self.h, ptr(x), ptr(out), x.numel()),
                       "hmcx_allgather_chain_stats")
        return out

    def allreduce(self, x, op):
        from ._native import ptr
        x = x.contiguous()
        out = torch.empty_like(x)
        self.ctx.bind_stream()
        self.ctx.check(self.ctx.lib.hmcx_allreduce_f64(self.ctx.h, self.h, ptr(x), ptr(out), x.numel(),
                                                       0 if op == "sum" else 1), "hmcx_allreduce_f64")
        return out

    def destroy(self):
        if self.h is not None and self.h.value:
            self.ctx.lib.hmcx_comm_destroy(self.h)
        self.h = None


def init_rccl(device):
    """Create the data-plane RCCL communicator through libhmcx: rank 0 makes the unique id
    (hmcx_comm_unique_id), the control plane hands it to every rank, each rank calls hmcx_comm_init
    on its own GPU.  No-op without a process group or with HMCX_DIST_BACKEND=gloo (ranks sharing a
    GPU, which RCCL refuses); returns the communicator or None."""
    global _rccl
    if _rccl is not None or not dist.is_initialized() or os.environ.get("HMCX_DIST_BACKEND") == "gloo":
        return _rccl
    import ctypes
    from . import _native as nat
    world, rank = dist.get_world_size(), dist.get_rank()
    buf = ctypes.create_string_buffer(128)
    if rank == 0:
        rc = nat.load_library().hmcx_comm_unique_id(buf)
        if rc != 0:
            raise nat.HmcxError("hmcx_comm_unique_id failed (%d)" % rc)
    obj = [buf.raw if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    buf = ctypes.create_string_buffer(obj[0], 128)
    ctx = nat.context(device)
    h = ctypes.c_void_p()
    ctx.check(ctx.lib.hmcx_comm_init(ctx.h, world, rank, buf, ctypes.byref(h)), "hmcx_comm_init")
    _rccl = RcclComm(ctx, h, world, rank)
    return _rccl


def finalize():
    """Tear down the data-plane communicator and the process group on every rank (each rank calls
    this, also when it has nothing to report)."""
    global _rccl
    if _rccl is not None:
        torch.cuda.synchronize(_rccl.ctx.device)
        _rccl.destroy()
        _rccl = None
    if dist.is_initialized():
        dist.destroy_process_group()


def backend_name():
    if _rccl is not None:
        return "RCCL over xGMI (libhmcx hmcx_allgather_chain_stats)"
    if not dist.is_initialized():
        return "none"
    return dist.get_backend()


def chain_block(n_chains, rank, world):
    """(chain0, c_local): the contiguous block of chain ids sampled by `rank` (the first
    n_chains % world ranks take one more).  Pass them as sampler(chain=chain0, chains=c_local):
    Philox keys chain0 + c are then disjoint across ranks."""
    base, extra = divmod(int(n_chains), int(world))
    c_local = base + (1 if rank < extra else 0)
    chain0 = rank * base + min(rank, extra)
    return chain0, c_local


def chains_of_rank(n_chains, rank, world):
    """Chain ids sampled by `rank`: its contiguous block (chain_block)."""
    chain0, c = chain_block(n_chains, rank, world)
    return list(range(chain0, chain0 + c))


def barrier():
    if dist.is_initialized():
        dist.barrier()


def _reduce(x, op, device):
    if not dist.is_initialized():
        return float(x)
    if _rccl is not None:
        t = torch.tensor([float(x)], dtype=torch.float64, device=_rccl.ctx.device)
        return float(_rccl.allreduce(t, op).item())
    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return float(t.item())


def allreduce_max(x, device=None):
    return _reduce(x, "max", device)


def allreduce_sum(x, device=None):
    return _reduce(x, "sum", device)


def gather_objects(obj):
    """All-gather one small picklable object per rank (list ordered by rank)."""
    if not dist.is_initialized():
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def gather_traces(local_traces, device=None, keep_device=False):
    """All-gather per-chain traces.  local_traces: array [c_local, T, P] (same T, P on every rank;
    c_local may differ, as chain_block gives the first n % world ranks one chain more) → array
    [Σ c_local, T, P] ordered by (rank, local chain).  Uneven blocks are padded to the largest
    c_local for the one all_gather (equal shapes on every rank) and the padding is dropped."""
    x = torch.as_tensor(np.ascontiguousarray(local_traces), dtype=torch.float64)
    if not dist.is_initialized():
        return x.numpy()
    world = dist.get_world_size()
    allc = gather_objects(int(x.shape[0]))                       # control plane
    cmax = max(allc)
    if x.shape[0] < cmax:
        x = torch.cat([x, x.new_zeros((cmax - x.shape[0],) + tuple(x.shape[1:]))], dim=0)
    if _rccl is not None:                                        # data plane: one RCCL all-gather
        allx = _rccl.allgather(x.to(_rccl.ctx.device).reshape(-1)).reshape((world,) + tuple(x.shape))
        if keep_device:                                          # stays where the diagnostics kernel reads it
            return torch.cat([o[:c] for o, c in zip(allx, allc)], dim=0)
        out = list(allx.cpu())
    else:
        out = [torch.empty_like(x) for _ in range(world)]
        dist.all_gather(out, x)
    return torch.cat([o[:c] for o, c in zip(out, allc)], dim=0).numpy()


class Welford:
    """Streaming per-parameter mean and M2 = Σ (x − mean)² of one or more chains' draws ([c, P]
    state per update, or a batch [c, T, P]); batches merge with Chan et al.'s pairwise update,
    so the result does not depend on how the draws were split into calls."""

    def __init__(self, shape):
        self.n = 0
        self.mean = np.zeros(shape, dtype=np.float64)
        self.M2 = np.zeros(shape, dtype=np.float64)

    def update(self, batch):
        b = np.asarray(batch, dtype=np.float64)
        if b.ndim == self.mean.ndim:
            b = b[:, None]
        nb = b.shape[1]
        if nb == 0:
            return self
        mb = b.mean(axis=1)
        M2b = ((b - mb[:, None]) ** 2).sum(axis=1)
        n = self.n + nb
        d = mb - self.mean
        self.mean = self.mean + d * (nb / n)
        self.M2 = self.M2 + M2b + d * d * (self.n * nb / n)
        self.n = n
        return self


def gather_summaries(welford, trace, device=None, keep_device=False):
    """All-gather the per-chain summaries of this rank (Welford over [c_local, P], thinned trace
    [c_local, T, P]; the same T, P on every rank, c_local may differ) in one data collective: returns
    (n, mean [C, P], M2 [C, P], trace [C, T, P]) over all C chains, ordered by rank.  keep_device: the
    three arrays are device tensors (the RCCL all-gather's own buffer; a copy of them when the gather
    ran over gloo or there is one rank) for summary_diagnostics_device."""
    c, P = welford.mean.shape
    trace = np.asarray(trace, dtype=np.float64).reshape(c, -1, P)
    T = trace.shape[1]
    packed = np.concatenate([welford.mean[:, None, :], welford.M2[:, None, :], trace], axis=1)   # [c, 2+T, P]
    allp = gather_traces(packed, device=device, keep_device=keep_device)
    if keep_device and not isinstance(allp, torch.Tensor):
        allp = torch.as_tensor(allp, dtype=torch.float64, device=device)
    n = allreduce_max(welford.n, device=device)
    if keep_device:
        return int(n), allp[:, 0, :].contiguous(), allp[:, 1, :].contiguous(), allp[:, 2:2 + T, :].contiguous()
    return int(n), allp[:, 0, :], allp[:, 1, :], allp[:, 2:2 + T, :]


def rhat_from_moments(n, means, M2):
    """Classic (non-split) R̂ per parameter from per-chain means and M2 over n draws each
    (BDA3 §11.4): W = mean_c M2/(n−1), B/n = var_c(means)."""
    means = np.asarray(means, dtype=np.float64)
    W = (np.asarray(M2, dtype=np.float64) / (n - 1)).mean(axis=0)
    B_n = means.var(axis=0, ddof=1) if means.shape[0] > 1 else np.zeros(means.shape[1:])
    var_hat = (n - 1) / n * W + B_n
    with np.errstate(divide='ignore', invalid='ignore'):
        r = np.sqrt(var_hat / W)
    return np.where(W > 0, r, np.nan)


def summary_diagnostics(n, means, M2, trace):
    """Per-parameter diagnostics on rank 0: R̂ from the moments, split-R̂ and ESS from the thinned
    traces; reported as their distribution over the parameters."""
    r = rhat_from_moments(n, means, M2)
    sr = diagnostics.split_rhat(trace)
    es = diagnostics.ess(trace)

    def q(x):
        x = np.asarray(x, dtype=np.float64).ravel()
        x = x[np.isfinite(x)]
        if x.size == 0:
            return None
        return {"min": float(x.min()), "median": float(np.median(x)), "max": float(x.max())}
    return {"chains": int(means.shape[0]), "draws_per_chain": int(n), "trace_draws_per_chain": int(trace.shape[1]),
            "params": int(means.shape[1]), "rhat": q(r), "split_rhat": q(sr), "ess": q(es)}


def summary_diagnostics_device(n, means, M2, trace):
    """summary_diagnostics with R̂ / split-R̂ / ESS computed on the device (diagnostics.device_diagnostics,
    hmcx_chain_diagnostics) from the gathered device tensors; the distribution over parameters is taken
    on the host."""
    r, sr, es = diagnostics.device_diagnostics(trace, means, M2, n)

    def q(x):
        x = np.asarray(x, dtype=np.float64).ravel()
        x = x[np.isfinite(x)]
        if x.size == 0:
            return None
        return {"min": float(x.min()), "median": float(np.median(x)), "max": float(x.max())}
    return {"chains": int(means.shape[0]), "draws_per_chain": int(n), "trace_draws_per_chain": int(trace.shape[1]),
            "params": int(means.shape[1]), "rhat": q(r), "split_rhat": q(sr), "ess": q(es),
            "computed_on": "device (hmcx_chain_diagnostics)"}


def chain_diagnostics(all_traces):
    """split-R̂ and ESS per traced quantity over all gathered chains ([C, T, P])."""
    x = np.asarray(all_traces, dtype=np.float64)
    return {"rhat": diagnostics.split_rhat(x), "ess": diagnostics.ess(x)}
