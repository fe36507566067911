"""ORACLE (test infrastructure only) — ensembles of independent NumPy reference chains, for the
statistical parity tests of the device-noise (Philox) chains (tests/test_gpu_statistics.py).

Each chain is oracle/samplers.py's restatement of the reference sampler (sghmc: cpu/sghmc.py:19-39
with the A1 completion; sgld: cpu/sgld.py:31-46) driven by its own seeds, exactly like the
reference's multi-chain workers (cpu/sghmc_multicore.py:86-94 seed worker i with RandomState(i)).
With N == batch_size every epoch is one step, so ``posterior`` holds the state after every step.

Chains run in a spawn-context process pool with one BLAS thread per worker; the workers import
only NumPy and oracle/ (never torch / HIP).
"""
import io
import os

import numpy as np


def _chain(args):
    kind, cfg, seed, T, momentum_scale = args
    from oracle import inputs as gi, models as om, samplers as osm
    X, Y = gi.dataset(cfg["data_seed"], cfg["N"], cfg["D"], cfg["K"])
    cls = osm.sghmc if kind == "sghmc" else osm.sgld
    if momentum_scale != 1.0:
        # negative control only (tests/test_stats_cpu.py): a deliberately wrong momentum law
        base = cls

        class cls(base):
            def draw_momentum(self, rng, *a):
                return {k: momentum_scale * v for k, v in base.draw_momentum(self, rng, *a).items()}
    s = cls(om.softmax({"alpha": cfg["alpha"]}),
            {"weights": np.zeros((cfg["D"], cfg["K"])), "bias": np.zeros(cfg["K"])},
            path_length=cfg["path_length"], step_size=cfg["step_size"], verbose=False)
    s.out = io.StringIO()
    s.trace = []
    np.random.seed(100003 + seed)
    post, _ = s.sample(epochs=T, burnin=0, batch_size=cfg["B"], rng=np.random.RandomState(seed),
                       X_train=X, y_train=Y)
    flat = np.concatenate([post["weights"].reshape(T, -1), post["bias"].reshape(T, -1)], axis=1)
    acc = np.array([t.get("accepted", True) for t in s.trace], dtype=bool)
    return flat.astype(np.float64), acc


def default_workers():
    """The host's CPU share: at most 16 (the GPU box's share per GPU), at least 1."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def run_chains(kind, cfg, seeds, T, workers=None, momentum_scale=1.0):
    """Independent oracle chains → (draws [C, T, P] with P = D·K + K, accept flags [C, T]).
    ``momentum_scale`` ≠ 1 scales every momentum / SGLD noise draw: a deliberately wrong chain, used
    only as the negative control that shows the moment tests can fail."""
    import multiprocessing as mp
    workers = workers or default_workers()
    jobs = [(kind, cfg, int(s), int(T), float(momentum_scale)) for s in seeds]
    saved = {k: os.environ.get(k) for k in ("OPENBLAS_NUM_THREADS", "OMP_NUM_THREADS", "MKL_NUM_THREADS")}
    for k in saved:
        os.environ[k] = "1"
    try:
        with mp.get_context("spawn").Pool(workers) as pool:
            res = pool.map(_chain, jobs)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return np.stack([r[0] for r in res]), np.stack([r[1] for r in res])
