#!/usr/bin/env python3
"""Headline benchmark: leapfrog-steps/sec × param-dim, MNIST-shaped softmax SGHMC (BASELINE.json).

One "step" = one SGHMC step over one minibatch (reference cpu/sghmc.py:19-39, A1 completion):
momentum draw, L−1 leapfrog iterations (each = weights sub-step + bias sub-step, i.e. one
softmax-gradient evaluation X·W → softmax → Xᵀ·diff), energies and the MH accept — all inside
libhmcx.  The reported unit counts leapfrog iterations (sghmc.py:28), summed over chains, times
the parameter dimension P = 784·10 + 10 = 7850.

Workload (BASELINE config 2 at N=1, config 4 at N=8): synthetic MNIST-shaped data
(X = rand(60000, 784), one-hot labels over 10 classes), batch 500, α = 0.01, ε = 1e-3,
λ = 1e-2 (E[L] ≈ 10.5), zero start, one chain per GPU, float64 (the reference's dtype),
device Philox noise.  Ranks run independent chains (no communication while sampling); after the
timed region an untimed diagnostics run returns every step's state, and one all-gather (RCCL) moves
each chain's per-parameter Welford mean / M2 and thinned trace to rank 0 for R̂ / split-R̂ / ESS.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...
"""
import argparse
import io
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

D, K, B, N_DATA = 784, 10, 500, 60000
P = D * K + K
ALPHA, EPS, LAMBDA = 0.01, 1e-3, 1e-2
FLOP_PER_LEAPFROG = 4.0 * B * D * K          # X·W and Xᵀ·diff: 15.68 MFLOP
DIAG_STEPS, DIAG_THIN = 240, 4               # untimed diagnostics run after the timed region
MFMA_PEAK_TFLOPS = {"f64": 78.6, "f32": 157.3}   # dense MFMA, MI355X spec (f32: MI355X_MICROARCH.md)
SEED = 20251015                              # Philox key of the headline chains (chain id = rank)
# kernel time of one persistent launch = a + b·steps + c·leapfrogs (µs), least squares over 48 calls of
# 1 … 120 steps (tools/probe_launch_fixed.py, profiles/r03_launch_fixed.txt): the model behind
# predicted_speedup
LAUNCH_FIT_US = (19.0, 11.14, 7.965)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=600, help="timed SGHMC steps per chain")
    ap.add_argument("--warmup", type=int, default=120)
    ap.add_argument("--dtype", choices=["f64", "f32"], default="f64")
    ap.add_argument("--path", choices=["auto", "kernels", "persistent"], default="auto")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="CPU-baseline time budget per baseline (0 = skip)")
    ap.add_argument("--batched-chains", type=int, default=8192,
                    help="chains per GPU of the secondary chain-batched measurement (0 = skip); the line also "
                         "reports 2048 chains (round 2's operating point) as a sweep point")
    ap.add_argument("--mlp-steps", type=int, default=40,
                    help="SGHMC steps of the secondary config-3 MLP measurement (0 = skip)")
    ap.add_argument("--sgld-steps", type=int, default=400,
                    help="SGLD steps of the secondary config-5 (D=2048, K=38) measurement (0 = skip)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check without a GPU: ranks rendezvous over gloo, reduce a dummy count "
                         "and rank 0 prints the JSON line shape (tests/test_bench_launch.py)")
    return ap.parse_args()


def aggregate_ranks(per_rank, P_dim=P):
    """The multi-GPU line from every rank's own numbers (list ordered by rank, each {"leapfrogs": lf_r,
    "seconds": t_r}): `value` is the makespan rate Σ_r lf_r ÷ max_r t_r (the contract's max-over-ranks
    clock), `value_chain_throughput` the sum of the ranks' own rates Σ_r lf_r ÷ t_r (north_star's
    "chain-throughput": independent chains, each GPU's rate counted over its own timed region).  With
    random path lengths (sghmc.py:25) the ranks do unequal work over the same steps, so the makespan
    rate is below the chain throughput by the spread of Σ L − 1 across chains."""
    lf = [float(r["leapfrogs"]) for r in per_rank]
    t = [float(r["seconds"]) for r in per_rank]
    return {"value_makespan": sum(lf) / max(t) * P_dim,
            "value_chain_throughput": sum(l_ / t_ for l_, t_ in zip(lf, t)) * P_dim,
            "per_rank_leapfrogs": lf, "per_rank_ms": [x * 1e3 for x in t]}


def predicted_scaling(warmup, steps, path_length=LAMBDA, eps=EPS, seed=SEED, worlds=(1, 2, 4, 8), fit=LAUNCH_FIT_US,
                      calls_per_rank=1):
    """What the N-GPU line should show, before any N > 1 run: the timed leapfrogs of chains 0 … N−1
    from the host twin of the device schedule (hmcx_philox_schedule — the same path lengths the kernels
    draw) and each rank's kernel time from the launch fit; speedups under both definitions of
    aggregate_ranks, relative to rank 0 alone."""
    from dropout_hamiltonian_montecarlo_amd import _native as nat
    L, n_iter, _ = nat.philox_schedule(seed, 0, max(worlds), warmup, path_length, np.full(steps, eps))
    lf = n_iter.astype(np.float64).sum(axis=0)                 # [chains]: Σ max(0, L − 1) over the timed steps
    t_us = fit[0] * calls_per_rank + fit[1] * steps + fit[2] * lf
    base = lf[0] / t_us[0]
    out = {"chain_leapfrogs": lf.tolist(), "fit_us": list(fit), "source": "hmcx_philox_schedule (host twin) + "
           "LAUNCH_FIT_US (profiles/r03_launch_fixed.txt)"}
    for n in worlds:
        out[str(n)] = {"makespan": float(lf[:n].sum() / t_us[:n].max() / base),
                       "chain_throughput": float((lf[:n] / t_us[:n]).sum() / base)}
    return out


def launch_ranks(n, argv):
    """`--gpus N` (N > 1) started without a launcher (no WORLD_SIZE in the environment): start N
    fresh rank processes of this script, one per GPU, and relay rank 0's JSON line.

    The reference's multi-chain layer starts its own workers (hamiltonian/inference/cpu/
    sghmc_multicore.py:81-99: a Pool, RandomState(i) per worker); here each rank is a child process
    with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set, exactly what
    torch.distributed.run would give it.  Called before anything touches the GPU (this process never
    imports torch); the children are started with Popen — nothing is exec'd.  Returns the exit
    code: 0 only when every rank exited 0; a failed rank stops the others (their exact PIDs)."""
    import signal
    import socket
    import subprocess
    import tempfile
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    me = os.path.abspath(__file__)
    out0 = tempfile.TemporaryFile(mode="w+")
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HMCX_BENCH_CHILD="1")
        procs.append(subprocess.Popen([sys.executable, me] + list(argv), env=env, cwd=REPO,
                                      stdout=out0 if r == 0 else subprocess.DEVNULL))
    def _term(signum, frame):
        raise SystemExit(128 + signum)
    signal.signal(signal.SIGTERM, _term)        # so the finally below runs on a SIGTERM to this parent
    rc = 0
    live = list(procs)
    deadline = time.monotonic() + float(os.environ.get("HMCX_BENCH_DEADLINE_S", "1800"))
    try:
        while live:
            time.sleep(0.2)
            if time.monotonic() > deadline:
                print("bench: ranks still running after the deadline; stopping them", file=sys.stderr)
                rc = rc or 124
                break
            for p in list(live):
                c = p.poll()
                if c is None:
                    continue
                live.remove(p)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    print("bench: rank %d exited with %d; stopping the other ranks" % (procs.index(p), c),
                          file=sys.stderr)
                    for q in live:
                        q.send_signal(signal.SIGTERM)
    finally:
        # a hung rank, a failed one or a signal to this parent: no child outlives it (exact PIDs)
        for q in procs:
            if q.poll() is None:
                q.send_signal(signal.SIGTERM)
        for q in procs:
            try:
                q.wait(timeout=20)
            except subprocess.TimeoutExpired:
                q.kill()
                q.wait()
    out0.seek(0)
    text = out0.read()
    lines = [ln for ln in text.splitlines() if ln.strip().startswith("{")]
    if rc == 0 and not lines:
        print("bench: rank 0 printed no JSON line", file=sys.stderr)
        rc = 1
    if lines:
        print(lines[-1])
    sys.stdout.flush()
    return rc


def dry_run(args):
    """--dry-run: the launch and reduction logic of a multi-rank run with no GPU work (gloo)."""
    from dropout_hamiltonian_montecarlo_amd import parallel
    rank, world, local = parallel.init("gloo")
    try:
        t = parallel.allreduce_max(0.001 * (rank + 1))
        lf = parallel.allreduce_sum(10.0 * (rank + 1))
        ranks = aggregate_ranks(parallel.gather_objects({"leapfrogs": 10.0 * (rank + 1), "seconds": 0.001 * (rank + 1)}))
        env = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
        envs = parallel.gather_objects(env)
        if rank == 0:
            print(json.dumps({"metric": "dry-run", "value": lf / t, "n_gpus": world, "steps": args.steps,
                              "warmup": args.warmup, "leapfrogs": lf, "t_max": t, "rank_env": envs, "ranks": ranks,
                              "config": {"chains": world, "local_rank_devices": [e["LOCAL_RANK"] for e in envs]}}))
    finally:
        parallel.finalize()


def synthetic_data(seed=0):
    X = np.random.RandomState(seed).rand(N_DATA, D)
    lab = np.random.RandomState(seed + 1).randint(0, K, N_DATA)
    Y = np.zeros((N_DATA, K))
    Y[np.arange(N_DATA), lab] = 1.0
    return X, Y


def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def blas_threads():
    import threadpoolctl
    blas = [i for i in threadpoolctl.threadpool_info() if i.get("user_api") == "blas"]
    return int(max((i.get("num_threads", 1) for i in blas), default=1))


def cpu_baseline(X, Y, budget_s, threads=None):
    """The oracle (NumPy float64 restatement of the reference SGHMC, bit-exact to it) on host
    cores: bounded sample of the same workload, leapfrogs counted the same way.  threads=None:
    OpenBLAS default — on the GPU box that is the job's CPU share for one GPU (the pool sets
    OMP_NUM_THREADS=16; the affinity mask lists the whole host); threads=1: one BLAS thread."""
    import threadpoolctl
    if threads is None:
        return _cpu_baseline(X, Y, budget_s)
    with threadpoolctl.threadpool_limits(limits=threads, user_api="blas"):
        return _cpu_baseline(X, Y, budget_s)


def _cpu_baseline(X, Y, budget_s):
    from oracle import models as om, samplers as osm
    threads = blas_threads()
    nb = 10
    Xs, Ys = X[:nb * B], Y[:nb * B]
    lf, t_total, steps = 0.0, 0.0, 0
    rep = 0
    while t_total < budget_s:
        s = osm.sghmc(om.softmax({"alpha": ALPHA}), {"weights": np.zeros((D, K)), "bias": np.zeros(K)},
                      path_length=LAMBDA, step_size=EPS, verbose=False)
        s.out = io.StringIO()
        s.trace = []
        np.random.seed(rep)
        t0 = time.perf_counter()
        s.sample(epochs=1, burnin=0, batch_size=B, rng=np.random.RandomState(rep), X_train=Xs, y_train=Ys)
        t_total += time.perf_counter() - t0
        lf += sum(max(0.0, t["L"] - 1) for t in s.trace)
        steps += len(s.trace)
        rep += 1
    return {"value": lf / t_total * P, "unit": "leapfrog-steps/s x param-dim", "cores": int(threads),
            "kind": "port",
            "sample": "oracle/samplers.py SGHMC (NumPy f64, bit-exact to the reference) incl. its per-10-minibatch "
                      "log-likelihood logging: %d steps / %.0f leapfrogs on minibatches of B=500 (D=784, K=10), "
                      "eps=1e-3, lambda=1e-2, %.1f s, %d BLAS threads, host %s (%d CPUs in affinity mask; "
                      "OMP_NUM_THREADS=%s is this job's CPU share, so 'all cores' = that share, not the mask)" % (
                          steps, lf, t_total, threads, cpu_model(), len(os.sched_getaffinity(0)),
                          os.environ.get("OMP_NUM_THREADS", "unset")),
            "lf_per_s": lf / t_total}


def calibrated(line):
    """Attach the committed port/reference throughput ratio (profiles/cpu_calibration.json, made by
    tools/cpu_calibration.py in the build container, where the reference exists: the oracle's SGHMC
    against the reference's own sghmc.py + softmax.py on the same loop) for the nearest BLAS thread
    count; ratio > 1 means the port is faster than the reference (the reference also evaluates the dead
    gradient of sghmc.py:26 every step)."""
    f = os.path.join(REPO, "profiles", "cpu_calibration.json")
    try:
        with open(f) as fh:
            cal = json.load(fh)["by_threads"]
    except (OSError, ValueError, KeyError):
        line["calibration_ratio"] = None
        return line
    thr = min(cal, key=lambda t: abs(int(t) - int(line["cores"])))
    line["calibration_ratio"] = cal[thr]["ratio_port_over_reference"]
    line["calibration"] = ("port/reference lf/s = %.3f at %s BLAS thread(s) in the build container "
                           "(profiles/cpu_calibration.json); reference-equivalent value = value / ratio"
                           % (cal[thr]["ratio_port_over_reference"], thr))
    line["reference_equivalent_value"] = line["value"] / cal[thr]["ratio_port_over_reference"]
    return line


def pmc_file(dtype, path):
    import glob
    fs = sorted(glob.glob(os.path.join(REPO, "profiles", "pmc_r[0-9][0-9]_%s_%s.json" % (dtype, path))))
    return os.path.relpath(fs[-1], REPO) if fs else None


def pmc_traffic(dtype, path, leapfrogs_per_launch):
    """Fabric bytes per launch of the dominant kernel, from the committed rocprofv3 PMC run of the
    driver's call shape (the newest profiles/pmc_rNN_<dtype>_<path>.json, tools/gpu_pmc_headline.sh): 2·FETCH_SIZE +
    WRITE_SIZE of the timed launches (MI355X_MICROARCH.md: FETCH_SIZE counts half of 16-byte
    streaming reads) per leapfrog of those launches, times the leapfrogs of this run's launch — the
    exchange rounds, which carry almost all of the traffic, are per leapfrog."""
    f = pmc_file(dtype, path)
    if f is None:
        return None
    f = os.path.join(REPO, f)
    with open(f) as fh:
        per_lf = json.load(fh).get("traffic_bytes_per_leapfrog")
    return None if per_lf is None else per_lf * leapfrogs_per_launch


def batched_chains(model, X, Y, data, C, n_steps, rank):
    """Secondary measurement: C independent chains on this GPU sharing every
    minibatch, i.e. the chain-batched gradient GEMMs [B×D]·[D×10C] and [D×B]·[B×10C]
    (hmcx_batch.h).  Returns throughput and the GEMM roofline of that path."""
    import torch
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu.sghmc import sghmc
    s = sghmc(model, {"weights": np.zeros((D, K)), "bias": np.zeros(K)}, path_length=LAMBDA, step_size=EPS,
              noise="philox", seed=7, chain=rank * C, chains=C)
    s.out = io.StringIO()
    state = s._init_state()
    nb = N_DATA // B
    rows = [(i % nb) * B for i in range(n_steps)]
    s.trace = []
    s._run(state, data, rows, [EPS] * n_steps, None, B)      # warm-up: same call shape (workspace, code objects)
    torch.cuda.synchronize()
    s.trace = []
    model.ctx.set_timing(True)
    t0 = time.perf_counter()
    s._run(state, data, rows, [EPS] * n_steps, None, B)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kms, kn = model.ctx.get_timing()
    model.ctx.set_timing(False)
    lf = float(sum(np.maximum(0.0, t["L"] - 1).sum() for t in s.trace))
    achieved = FLOP_PER_LEAPFROG * lf / (kms * 1e-3) / 1e12
    return {"chains_per_gpu": C, "steps": n_steps, "leapfrogs": lf, "leapfrogs_per_s": lf / dt,
            "value": lf / dt * P, "unit": "leapfrog-steps/s x param-dim", "ms": dt * 1e3,
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": MFMA_PEAK_TFLOPS["f64" if model.dtype.itemsize == 8 else "f32"],
                         "unit": "TFLOP/s", "frac": achieved / MFMA_PEAK_TFLOPS["f64" if model.dtype.itemsize == 8 else "f32"],
                         "kernel": "k_bfwd + k_bgrad + step kernels of one hmcx_sghmc_run call",
                         "device_ms": kms, "flop": FLOP_PER_LEAPFROG * lf}}


MLP_SHAPE = (784, 256, 10)                   # MyNetwork(784, 256, 10): two hidden layers (mlp.py:24-26)
MLP_P = 256 * 784 + 256 + 256 * 256 + 256 + 10 * 256 + 10          # 269,322
MLP_FLOP_PER_LEAPFROG = 1.0193e9             # SURVEY §8d "M": minimal-recompute schedule, B = 500
MLP_LAMBDA = 2e-2                            # path length: E[L] = λ/ε + ½ ≈ 20.5, inside SURVEY §8d's 10–50


def mlp_measure(X, lab, n_steps, rank, dtype="f32"):
    """Secondary measurement, BASELINE config 3: MNIST MLP 784-256-256-10 SGHMC, batch 500, one
    chain, float32 (Chainer's default dtype; dtype="f64" for the parity dtype's figure), device
    Philox noise and dropout masks, through the fused hmcx_mlp_sghmc_run."""
    import torch
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.models.gpu.mlp import mlp
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu.sghmc import sghmc
    tdt = torch.float32 if dtype == "f32" else torch.float64
    m = mlp({"alpha": ALPHA}, *MLP_SHAPE, dtype=tdt)
    s = sghmc(m, m.init_params(1), path_length=MLP_LAMBDA, step_size=EPS, noise="philox", seed=11, chain=rank)
    s.out = io.StringIO()
    state = s._init_state()
    Xd = torch.as_tensor(X).to(m.device, tdt).contiguous()
    yd = torch.as_tensor(lab).to(m.device, torch.int32).contiguous()
    nb = N_DATA // B
    rows = [(i % nb) * B for i in range(n_steps)]
    s.trace = []
    s._run(state, (Xd, yd), rows, [EPS] * n_steps, None, B)     # warm-up: same call shape
    torch.cuda.synchronize()
    # three timed calls of the same shape, the chain continuing from one to the next; the leg reports the call
    # with the median device rate (leapfrogs per device second), every call's numbers beside it
    runs = []
    for _ in range(3):
        s.trace = []
        m.ctx.set_timing(True)
        t0 = time.perf_counter()
        res = s._run(state, (Xd, yd), rows, [EPS] * n_steps, None, B)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        kms, _ = m.ctx.get_timing()
        m.ctx.set_timing(False)
        lf = float(sum(max(0.0, t["L"] - 1) for t in s.trace))
        runs.append({"device_ms": kms, "wall_s": dt, "leapfrogs": lf, "res": res, "trace": list(s.trace)})
    runs.sort(key=lambda r: r["leapfrogs"] / r["device_ms"])
    med = runs[1]
    kms, dt, res, lf = med["device_ms"], med["wall_s"], med["res"], med["leapfrogs"]
    s.trace = med["trace"]
    achieved = MLP_FLOP_PER_LEAPFROG * lf / (kms * 1e-3) / 1e12
    out = {"workload": "MNIST MLP 784-256-256-10 SGHMC, batch 500, 1 chain (BASELINE config 3)",
           "dtype": dtype, "param_dim": MLP_P, "steps": n_steps, "leapfrogs": lf, "path_length": MLP_LAMBDA,
           "mean_L": float(np.mean([t["L"] for t in s.trace])),
           "leapfrogs_per_s": lf / dt, "value": lf / dt * MLP_P, "unit": "leapfrog-steps/s x param-dim",
           "accept_rate": float(np.mean(res.accepted)),
           "roofline": {"bound": "mfma", "achieved": achieved, "peak": MFMA_PEAK_TFLOPS[dtype], "unit": "TFLOP/s",
                        "frac": achieved / MFMA_PEAK_TFLOPS[dtype], "device_ms": kms,
                        "kernel": "all kernels of one hmcx_mlp_sghmc_run call (k_mm GEMMs + step kernels)",
                        "flop_per_leapfrog": MLP_FLOP_PER_LEAPFROG},
           "runs": [{"leapfrogs": r["leapfrogs"], "device_ms": r["device_ms"], "wall_s": r["wall_s"]} for r in runs],
           "timed": "median of 3 consecutive calls by leapfrogs per device second"}
    return out


def mlp_cpu_baseline(X, lab, cpu_seconds):
    """CPU baseline of config 3: the oracle's mlp.grad (NumPy float32) six times per leapfrog — the
    reference's per-sub-step full gradient (sghmc.py:29-34), fresh dropout masks per call."""
    from oracle import models as om
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.models.gpu.mlp import init_params
    rs = np.random.RandomState(0)
    ref = om.mlp({"alpha": ALPHA}, *MLP_SHAPE)
    par = {k: v.astype(np.float32) for k, v in init_params(MLP_SHAPE, 1).items()}
    Xb, yb = X[:B].astype(np.float32), lab[:B]
    calls, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < cpu_seconds:
        ref.grad(par, masks=om.dropout_masks(rs, B, MLP_SHAPE[1]), X_train=Xb, y_train=yb)
        calls += 1
    dtc = time.perf_counter() - t0
    lfc = calls / 6.0 / dtc
    return {"value": lfc * MLP_P, "unit": "leapfrog-steps/s x param-dim", "cores": blas_threads(), "kind": "port",
            "sample": "%d oracle mlp.grad calls (NumPy f32, B=500, fresh dropout masks), 6 per leapfrog, %.1f s"
                      % (calls, dtc), "leapfrogs_per_s": lfc}


V_D, V_K, V_N = 2048, 38, 20000               # BASELINE config 5 (PlantVillage-like features; SURVEY §8 "V")
V_P = V_D * V_K + V_K
V_FLOP_PER_STEP = 4.0 * B * V_D * V_K         # 155.6 MFLOP per SGLD step


def plantvillage_data():
    return (np.random.RandomState(5).rand(V_N, V_D),
            np.eye(V_K)[np.random.RandomState(6).randint(0, V_K, V_N)])


def plantvillage_measure(n_steps, rank):
    """Secondary measurement, BASELINE config 5: softmax SGLD on conv-feature-like inputs (D=2048,
    K=38, batch 500), one chain per GPU, float64, device Philox noise, through hmcx_sgld_run (the
    wide path, hmcx_wide.hip).  Logging cadence of the reference (log-likelihood every 10
    minibatches) included."""
    import torch
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.models.gpu.softmax import softmax
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu.sgld import sgld
    Xv, Yv = plantvillage_data()
    m = softmax({"alpha": ALPHA}, dtype=torch.float64)
    s = sgld(m, {"weights": np.zeros((V_D, V_K)), "bias": np.zeros(V_K)}, step_size=1e-4, noise="philox",
             seed=17, chain=rank)
    s.out = io.StringIO()
    data = s._upload_data(Xv, Yv)
    state = s._init_state()
    nb = V_N // B
    rows = [(i % nb) * B for i in range(n_steps)]
    s._run(state, data, rows, [1e-4] * n_steps, None, B)       # warm-up: same call shape
    torch.cuda.synchronize()
    m.ctx.set_timing(True)
    t0 = time.perf_counter()
    s._run(state, data, rows, [1e-4] * n_steps, None, B)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kms, _ = m.ctx.get_timing()
    m.ctx.set_timing(False)
    tf = V_FLOP_PER_STEP * n_steps / (kms * 1e-3) / 1e12
    xbytes = 2.0 * B * V_D * 8                    # X tile read by the forward and by the gradient GEMM
    fused = os.environ.get("HMCX_WIDE_FUSE", "1") != "0"
    out = {"workload": "PlantVillage-like softmax SGLD, D=2048 features, K=38, batch 500, 1 chain (BASELINE config 5)",
           "dtype": "f64", "param_dim": V_P, "steps": n_steps, "us_per_step": kms * 1e3 / n_steps,
           "leapfrogs_per_s": n_steps / dt, "value": n_steps / dt * V_P, "unit": "leapfrog-steps/s x param-dim",
           "roofline": {"bound": "mfma", "achieved": tf, "peak": MFMA_PEAK_TFLOPS["f64"], "unit": "TFLOP/s",
                        "frac": tf / MFMA_PEAK_TFLOPS["f64"], "device_ms": kms,
                        "hbm_GBps_X": xbytes * n_steps / (kms * 1e-3) / 1e9,
                        "alg_GBps_X": xbytes / 2 * n_steps / (kms * 1e-3) / 1e9,
                        "alg_GBps_X_note": "the minibatch tile X (B x D x 8 B) counted once per step; hbm_GBps_X "
                                           "counts its two reads (forward and gradient GEMM)",
                        "kernel": ("k_wfwd_sm (forward + softmax) + k_wgrad per step" if fused else
                                   "k_wfwd + k_wsoft + k_wgrad per step") + " (+ logging forward every 10th)"}}
    return out


def plantvillage_cpu_baseline(cpu_seconds):
    """CPU baseline of config 5: the oracle's SGLD on the same shape (logging every 10 minibatches)."""
    from oracle import models as om, samplers as osm
    Xv, Yv = plantvillage_data()
    n_cpu = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < cpu_seconds:
        o = osm.sgld(om.softmax({"alpha": ALPHA}), {"weights": np.zeros((V_D, V_K)), "bias": np.zeros(V_K)},
                     step_size=1e-4, verbose=False)
        o.out = io.StringIO()
        np.random.seed(n_cpu)
        o.sample(epochs=1, burnin=0, batch_size=B, rng=np.random.RandomState(n_cpu),
                 X_train=Xv[:10 * B], y_train=Yv[:10 * B])
        n_cpu += 10
    dtc = time.perf_counter() - t0
    return {"value": n_cpu / dtc * V_P, "unit": "leapfrog-steps/s x param-dim", "cores": blas_threads(), "kind": "port",
            "sample": "%d oracle SGLD steps (NumPy f64, B=500, D=2048, K=38, logging every 10), %.1f s"
                      % (n_cpu, dtc), "leapfrogs_per_s": n_cpu / dtc}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: this process starts the N ranks itself and touches no GPU
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.dry_run:
        return dry_run(args)
    from dropout_hamiltonian_montecarlo_amd import parallel
    try:
        bench(args, parallel)
    finally:
        parallel.finalize()


def warmup_calls(warmup, chunk):
    """Step counts of the untimed warm-up calls of the headline leg: the same enqueue / collect protocol as
    the timed region, in at least two calls when there are two steps or more — the first call fills the
    sampler's argument caches, the second runs the cached steady-state path (sghmc._enqueue_quick) the
    timed calls take, so its first execution is not inside the clock.  tools/pmc_summary.py counts these
    dispatches to find the timed ones."""
    calls, done = [], 0
    first = min(chunk, max(1, warmup // 2))
    while done < warmup:
        n = min(first if done == 0 else chunk, warmup - done)
        calls.append(n)
        done += n
    return calls


def bench(args, parallel):
    import torch
    rank, world, local = parallel.init()
    if world != args.gpus and rank == 0:
        print("warning: --gpus %d but WORLD_SIZE %d" % (args.gpus, world), file=sys.stderr)
    if os.environ.get("HMCX_BENCH_SHARED_GPU") == "1":      # rehearsal: several ranks on one GPU (gloo)
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    parallel.init_rccl(dev)          # data-plane RCCL communicator through libhmcx (no-op at one rank)
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.models.gpu.softmax import softmax
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu.sghmc import sghmc

    dtype = torch.float64 if args.dtype == "f64" else torch.float32
    X, Y = synthetic_data(0)
    model = softmax({"alpha": ALPHA}, dtype=dtype, device=dev)
    model.ctx.set_sghmc_path({"auto": 0, "kernels": 1, "persistent": 2}[args.path])
    chain0, _ = parallel.chain_block(world, rank, world)     # one chain per rank: Philox key chain0
    s = sghmc(model, {"weights": np.zeros((D, K)), "bias": np.zeros(K)}, path_length=LAMBDA, step_size=EPS,
              noise="philox", seed=SEED, chain=chain0)
    s.out = io.StringIO()
    data = s._upload_data(X, Y)                      # dataset resident in HBM before timing
    state = s._init_state()
    nb = N_DATA // B

    def run(n_steps, step0):
        rows = [((step0 + i) % nb) * B for i in range(n_steps)]
        return s._run(state, data, rows, [EPS] * n_steps, None, B)

    def enqueue(n_steps, step0):
        rows = [((step0 + i) % nb) * B for i in range(n_steps)]
        return s._enqueue(state, data, rows, [EPS] * n_steps, None, B)

    CHUNK = nb                                       # one call per epoch (120 steps)
    rec0 = recoveries()
    keep_trace = os.environ.get("HMCX_BENCH_TRACE") == "1"
    s.trace = [] if keep_trace else None
    done = 0
    for n in warmup_calls(args.warmup, CHUNK):
        s._collect(enqueue(n, done))
        done += n
    torch.cuda.synchronize()

    # timed region: exactly args.steps steps per chain.  The per-step trace dicts of sample() are not
    # kept here (the leapfrog count comes from the path lengths each call returns); HMCX_BENCH_TRACE=1
    # keeps them as before (host-overhead A/B)
    s.trace = [] if keep_trace else None
    lls = []
    Ls = []
    n_calls = 0
    model.ctx.set_timing(True)        # HIP events around each run's kernels, on the launch stream
    parallel.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # calls are pipelined: call k+1 is enqueued (schedule prepared, kernel launched) before call k's
    # results are read back, so the host work overlaps the device work (sghmc._enqueue/_collect)
    done = 0
    pending = None
    while done < args.steps:
        n = min(CHUNK, args.steps - done)
        h = enqueue(n, args.warmup + done)
        if pending is not None:
            res = s._collect(pending)
            lls.append(res.ll)
            Ls.append(res.L)
        pending = h
        done += n
        n_calls += 1
    t_enq = time.perf_counter()
    # the last call: its kernel and the stores of its outputs into the pinned host block are done when
    # the stream is (synchronize below); reading those host values is bookkeeping after the clock
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    res = s._collect(pending)
    lls.append(res.ll)
    Ls.append(res.L)
    t_col = time.perf_counter()
    if os.environ.get("HMCX_BENCH_DEBUG") == "1":
        print("timed region: last enqueue returned %.1f us, sync %.1f us (last collect after it %.1f us)" % (
            (t_enq - t0) * 1e6, (t1 - t0) * 1e6, (t_col - t0) * 1e6), file=sys.stderr)
        from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu import sghmc as _sg
        m = [x for x in _sg._marks if x[1] >= t0]
        print("  enqueue phases: " + ", ".join("%s +%.1f" % (n, (t - p) * 1e6) for (n, t), (_, p) in
                                                zip(m[1:], m[:-1])), file=sys.stderr)
    parallel.barrier()
    elapsed = t1 - t0
    kern_ms, kern_n = model.ctx.get_timing()
    model.ctx.set_timing(False)

    lf_local = float(sum(np.maximum(0.0, np.asarray(L) - 1).sum() for L in Ls))
    if keep_trace:
        assert lf_local == float(sum(max(0.0, t["L"] - 1) for t in s.trace))
    t_max = parallel.allreduce_max(elapsed, device=dev)
    lf_total = parallel.allreduce_sum(lf_local, device=dev)
    value = lf_total / t_max * P
    # every rank's own leapfrogs and clock (control plane, small objects): both aggregates of the line
    per_rank = parallel.gather_objects({"leapfrogs": lf_local, "seconds": elapsed, "kernel_ms": kern_ms})
    ranks = aggregate_ranks(per_rank)
    ranks["per_rank_kernel_ms"] = [r["kernel_ms"] for r in per_rank]
    rec = {"headline": recovery_delta(rec0)}

    # cross-chain diagnostics (untimed, after the timed region): DIAG_STEPS more steps of the same
    # chain return the state after every step (out_trace); per-parameter Welford mean / M2 and a
    # thinned trace of every chain travel in ONE all-gather (RCCL over xGMI through libhmcx's
    # hmcx_allgather_chain_stats, parallel.py); rank 0 reports R̂,
    # split-R̂ and ESS per parameter.  The timed steps' log-likelihood trace is gathered too.
    s.record_steps = True
    wf = parallel.Welford((1, P))
    thin = []
    done = 0
    while done < DIAG_STEPS:
        n = min(CHUNK, DIAG_STEPS - done)
        st = run(n, args.warmup + args.steps + done).steps        # [n, 1, P]
        wf.update(st.transpose(1, 0, 2))
        thin.append(st[DIAG_THIN - 1::DIAG_THIN, 0])
        done += n
    s.record_steps = False
    # R̂ / split-R̂ / ESS per parameter on the device, where the all-gather left the summaries
    n_draws, means, M2, tr = parallel.gather_summaries(wf, np.concatenate(thin)[None], device=dev, keep_device=True)
    diag_par = parallel.summary_diagnostics_device(n_draws, means, M2, tr) if rank == 0 else None
    trace = np.concatenate(lls)[None, :, None]       # [1 chain, T, 1]
    allt = parallel.gather_traces(trace, device=dev)
    diag = parallel.chain_diagnostics(allt) if allt.shape[1] >= 4 else {"rhat": np.nan, "ess": np.nan}

    batched = None
    if args.batched_chains > 0:
        model.ctx.set_sghmc_path(0)
        r0 = recoveries()
        batched = batched_chains(model, X, Y, data, args.batched_chains, 24, rank)
        if args.batched_chains != 2048:       # round 2's operating point, for comparison
            b2 = batched_chains(model, X, Y, data, 2048, 24, rank)
            batched["sweep"] = {"2048": {"frac": b2["roofline"]["frac"], "leapfrogs_per_s": b2["leapfrogs_per_s"]},
                                str(args.batched_chains): {"frac": batched["roofline"]["frac"],
                                                           "leapfrogs_per_s": batched["leapfrogs_per_s"]}}
        batched["recoveries"] = rec["chain_batched"] = recovery_delta(r0)
        parallel.barrier()
    mlp_out = None
    if args.mlp_steps > 0:
        lab = np.argmax(Y, axis=1)
        r0 = recoveries()
        mlp_out = mlp_measure(X, lab, args.mlp_steps, rank)
        mlp_out["f64"] = mlp_measure(X, lab, args.mlp_steps, rank, dtype="f64")   # the parity dtype's cost
        mlp_out["recoveries"] = rec["mlp"] = recovery_delta(r0)
        parallel.barrier()
    v_out = None
    if args.sgld_steps > 0:
        r0 = recoveries()
        v_out = plantvillage_measure(args.sgld_steps, rank)
        v_out["recoveries"] = rec["plantvillage_sgld"] = recovery_delta(r0)
        parallel.barrier()
    # re-runs after timed-out exchanges on any rank, per leg (must all be 0: a fallback would be timed as
    # if it were the fused / persistent kernel)
    rec_all = parallel.gather_objects(rec)
    recov = {leg: sum(sum(r[leg].values()) for r in rec_all) for leg in rec}
    parallel.barrier()
    if rank == 0:
        ranks["predicted"] = predicted_scaling(args.warmup, args.steps, calls_per_rank=n_calls)
        report(args, world, value, t_max, lf_total, lf_local, n_calls, kern_ms, kern_n, diag_par, diag,
               batched, mlp_out, v_out, X, Y, ranks, recov)
    # closing barrier: every rank waits here until rank 0 has run its CPU baselines and printed, so the
    # RCCL communicator and the process group are torn down by all ranks together (main()'s finally)
    parallel.barrier()


def recoveries():
    from dropout_hamiltonian_montecarlo_amd import _native as nat
    return nat.recoveries_all()


def recovery_delta(before):
    now = recoveries()
    return {k: now[k] - before.get(k, 0) for k in now}


def report(args, world, value, t_max, lf_total, lf_local, n_calls, kern_ms, kern_n, diag_par, diag,
           batched, mlp_out, v_out, X, Y, ranks, recov):
    """Rank 0: the JSON line (and the CPU baselines, after every rank's GPU work)."""
    from dropout_hamiltonian_montecarlo_amd import parallel
    CHUNK = N_DATA // B                              # steps per call (one epoch), as in bench()
    path = "persistent" if (args.path != "kernels") else "kernels"
    assert kern_n == n_calls, (kern_n, n_calls)
    launch_ms = kern_ms / kern_n
    flop_per_launch = FLOP_PER_LEAPFROG * lf_local / n_calls
    achieved = flop_per_launch / (launch_ms * 1e-3) / 1e12
    peak = MFMA_PEAK_TFLOPS[args.dtype]
    out = {
        "metric": "leapfrog-steps/sec × param-dim, MNIST softmax SGHMC, 1/2/4/8 chains↔GPUs",
        "value": value,
        "unit": "leapfrog-steps/s x param-dim",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": t_max * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (MNIST-shaped X=rand(60000,784), one-hot y, K=10)",
        "config": {"workload": "MNIST softmax regression SGHMC, 1 chain per GPU (BASELINE configs 2/4)",
                   "global_batch": B * world, "batch_per_chain": B, "D": D, "K": K, "param_dim": P,
                   "chains": world, "step_size": EPS, "path_length": LAMBDA, "parallelism": "independent chains x%d" % world,
                   "impl": path},
        "leapfrogs_per_s": lf_total / t_max,
        "leapfrogs": lf_total,
        "value_definition": "makespan: leapfrogs of all ranks / max-over-ranks timed region x P",
        "ranks": ranks,
        "recoveries": recov,
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                     "frac": achieved / peak, "traffic": pmc_traffic(args.dtype, path, lf_local / n_calls),
                     "traffic_source": "PMC 2*FETCH_SIZE+WRITE_SIZE per leapfrog of the driver-shape launch "
                                       "(%s) x leapfrogs per launch of this run" % pmc_file(args.dtype, path),
                     "kernel": ("k_sghmc_p2<%s,10> (one launch per call: %d call(s) of <= %d steps)" % (
                         "double" if args.dtype == "f64" else "float", n_calls, CHUNK)) if path == "persistent"
                     else "kernel-per-phase sequence of each call (%d call(s) of <= %d steps)" % (n_calls, CHUNK),
                     "launch_ms": launch_ms, "flop_per_launch": flop_per_launch, "calls": n_calls,
                     "leapfrogs_per_launch": lf_local / n_calls},
        "diagnostics": {"per_parameter": diag_par,
                        "source": "%d untimed steps after the timed region, state after every step; Welford "
                                  "mean/M2 per parameter and every %dth draw, one all_gather" % (DIAG_STEPS, DIAG_THIN),
                        "note": "burn-in, not a convergence check: the chains start at zero (2.-MNIST.ipynb) and "
                                "have taken %d steps when these draws begin, so R-hat / ESS here describe the "
                                "transient; they exercise the gather path (RCCL at N > 1), not mixing"
                                % (args.warmup + args.steps),
                        "rhat_ll": float(np.ravel(diag["rhat"])[0]), "ess_ll": float(np.ravel(diag["ess"])[0]),
                        "gather": parallel.backend_name() if parallel.dist.is_initialized() else "local"},
        "cpu_baseline": None,
        "chain_batched": batched,
        "mlp": mlp_out,
        "plantvillage_sgld": v_out,
    }
    if args.cpu_seconds > 0:
        # rank 0, after every rank's GPU work (the barrier above): the oracle on host cores
        out["cpu_baseline"] = calibrated(cpu_baseline(X, Y, args.cpu_seconds))
        out["cpu_baseline_1thread"] = calibrated(cpu_baseline(X, Y, args.cpu_seconds, threads=1))
        if mlp_out is not None:
            mlp_out["cpu_baseline"] = mlp_cpu_baseline(X, np.argmax(Y, axis=1), args.cpu_seconds)
        if v_out is not None:
            v_out["cpu_baseline"] = plantvillage_cpu_baseline(args.cpu_seconds)
    print(json.dumps(out))
    sys.stdout.flush()


if __name__ == "__main__":
    main()
