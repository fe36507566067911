"""The collective path of the multi-GPU bench on real hardware.  The data collectives are RCCL
through libhmcx's C ABI (include/hmcx.h hmcx_comm_* / hmcx_allgather_chain_stats /
hmcx_allreduce_f64); torch.distributed (gloo) is only the control plane.  bench.py launched by
torchrun with one rank and HMCX_DIST_FORCE=1 runs the timing max/sum reductions and the
per-parameter summary all-gather through that communicator on the GPU.  N > 1 RCCL ranks need one GPU
each (the driver's 8-GPU run); N > 1 here runs ranks that share cuda:0 over gloo — self-launched (2 and
4 ranks, the latter with every leg at its default) and under torch.distributed.run (the driver's
invocation form) — and the N = 2 logic is also covered by tests/test_parallel_cpu.py and
tests/test_bench_launch.py."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_comm_c_abi_world1():
    """hmcx_comm_unique_id → hmcx_comm_init (1 rank) → all-gather / sum / max → destroy, on the
    context's stream."""
    import ctypes
    import torch
    from dropout_hamiltonian_montecarlo_amd import _native as nat
    ctx = nat.context(torch.device("cuda:0"))
    buf = ctypes.create_string_buffer(128)
    assert ctx.lib.hmcx_comm_unique_id(buf) == 0
    h = ctypes.c_void_p()
    ctx.check(ctx.lib.hmcx_comm_init(ctx.h, 1, 0, buf, ctypes.byref(h)), "hmcx_comm_init")
    try:
        x = torch.arange(1000, dtype=torch.float64, device="cuda:0") * 0.5
        out = torch.empty(1000, dtype=torch.float64, device="cuda:0")
        ctx.check(ctx.lib.hmcx_allgather_chain_stats(ctx.h, h, nat.ptr(x), nat.ptr(out), 1000), "allgather")
        for op in (0, 1):
            red = torch.empty(1000, dtype=torch.float64, device="cuda:0")
            ctx.check(ctx.lib.hmcx_allreduce_f64(ctx.h, h, nat.ptr(x), nat.ptr(red), 1000, op), "allreduce")
            torch.cuda.synchronize()
            assert torch.equal(red, x)
        torch.cuda.synchronize()
        assert torch.equal(out, x)
        assert ctx.lib.hmcx_comm_init(ctx.h, 1, 3, buf, ctypes.byref(ctypes.c_void_p())) != 0   # bad rank
    finally:
        assert ctx.lib.hmcx_comm_destroy(h) == 0


def test_bench_world1_through_rccl():
    port = str(_free_port())
    env = dict(os.environ, HMCX_DIST_FORCE="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", port, "bench.py", "--gpus", "1",
           "--steps", "5", "--warmup", "2", "--cpu-seconds", "0", "--batched-chains", "0",
           "--mlp-steps", "0", "--sgld-steps", "0"]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["value"] > 0
    diag = line["diagnostics"]
    assert "hmcx_allgather_chain_stats" in diag["gather"], diag["gather"]
    pp = diag["per_parameter"]
    assert pp["chains"] == 1 and pp["params"] == 7850
    assert 0.5 < pp["rhat"]["median"] < 2.0


def test_bench_self_launch_two_ranks_shared_gpu():
    """bench.py --gpus 2 without a launcher starts its own two ranks; on the
    one-GPU box both share cuda:0 (HMCX_BENCH_SHARED_GPU) and reduce over gloo."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(HMCX_BENCH_SHARED_GPU="1", HMCX_DIST_BACKEND="gloo")
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "5", "--warmup", "2", "--cpu-seconds", "0",
           "--batched-chains", "0", "--mlp-steps", "0", "--sgld-steps", "0"]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["chains"] == 2 and line["value"] > 0
    assert line["diagnostics"]["per_parameter"]["chains"] == 2


def test_bench_four_ranks_shared_gpu_default_legs():
    """the N > 1 path at the driver's settings — every secondary leg at its
    default and rank 0 running CPU baselines while the other ranks wait in the closing barrier
    (bench.py: all ranks tear the communicator / process group down together).  Four ranks share
    cuda:0 over gloo; --path kernels, since four persistent single-chain kernels of 128 workgroups
    each would oversubscribe one GPU's 256 CUs."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(HMCX_BENCH_SHARED_GPU="1", HMCX_DIST_BACKEND="gloo")
    cmd = [sys.executable, "bench.py", "--gpus", "4", "--path", "kernels", "--steps", "20", "--warmup", "5",
           "--cpu-seconds", "1"]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=420)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["n_gpus"] == 4 and line["config"]["chains"] == 4 and line["value"] > 0
    assert line["diagnostics"]["per_parameter"]["chains"] == 4
    assert line["diagnostics"]["per_parameter"]["params"] == 7850
    assert line["cpu_baseline"]["value"] > 0 and line["cpu_baseline"]["calibration_ratio"] > 0
    for leg in ("chain_batched", "mlp", "plantvillage_sgld"):
        assert line[leg] is not None and line[leg]["value"] > 0, leg


def test_bench_torchrun_two_ranks_shared_gpu():
    """The driver's SCALE invocation form — `python -m torch.distributed.run --nproc-per-node N … bench.py
    --gpus N` — at N = 2 on one GPU (ranks share cuda:0, gloo): bench.py runs as the launcher's rank,
    rank 0 prints the one JSON line with n_gpus 2 and both chains in the diagnostics."""
    port = str(_free_port())
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(HMCX_BENCH_SHARED_GPU="1", HMCX_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", port, "bench.py", "--gpus", "2", "--path", "kernels",
           "--steps", "5", "--warmup", "2", "--cpu-seconds", "0", "--batched-chains", "0", "--mlp-steps", "0",
           "--sgld-steps", "0"]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["chains"] == 2 and line["value"] > 0
    assert line["scaling"] == "weak" and line["diagnostics"]["per_parameter"]["chains"] == 2
