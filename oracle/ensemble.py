"""ORACLE (test infrastructure only) — ensembles of independent NumPy reference chains, for the
statistical parity tests of the device-noise (Philox) chains (tests/test_gpu_statistics.py).

Each chain is oracle/samplers.py's restatement of the reference sampler (sghmc: cpu/sghmc.py:19-39
with the A1 completion; sgld: cpu/sgld.py:31-46) driven by its own seeds, exactly like the
reference's multi-chain workers (cpu/sghmc_multicore.py:86-94 seed worker i with RandomState(i)).
With N == batch_size every epoch is one step, so ``posterior`` holds the state after every step.

The MLP ensemble (run_mlp_chains) is the same SGHMC restatement over oracle/models.py::mlp with
Chainer's train-mode dropout: fresh masks on every forward, from the chain's own RandomState.

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


def mlp_start(n_in, n_mid, n_out, seed):
    """Chainer L.Linear initialisation (W ~ N(0, 1/fan_in), b = 0) from RandomState(seed), in
    namedparams order — the start state of every chain of an MLP ensemble."""
    from oracle import models as om
    rs = np.random.RandomState(seed)
    out = {}
    for k in om.MLP_PARAM_NAMES:
        shp = om.mlp_param_shapes(n_in, n_mid, n_out)[k]
        out[k] = rs.normal(0, 1.0 / np.sqrt(shp[1]), shp) if len(shp) == 2 else np.zeros(shp)
    return out


def mlp_dataset(cfg):
    rs = np.random.RandomState(cfg["data_seed"])
    X = rs.rand(cfg["N"], cfg["n_in"])
    y = rs.randint(0, cfg["n_out"], cfg["N"])
    return X, y


class _FreshMaskMLP:
    """The reference MLP with Chainer's train-mode dropout: fresh masks on EVERY forward — each
    grad (mlp.py:47-64) and each energy evaluation of the accept test (mlp.py:80-82 through
    hmc.py:67-71) — drawn from the chain's own RandomState (F.dropout: keep iff u >= 0.1, scale
    1/0.9; oracle/models.py::dropout_masks)."""

    def __init__(self, inner, rng, dtype):
        self.inner, self.rng, self.dtype = inner, rng, dtype

    def _m(self, args):
        X = args["X_train"]
        return om_dropout(self.rng, X.shape[0], self.inner.n_mid, self.dtype)

    def grad(self, par, **args):
        return self.inner.grad(par, masks=self._m(args), **args)

    def negative_log_posterior(self, par, **args):
        return self.inner.negative_log_posterior(par, masks=self._m(args), **args)

    def log_likelihood(self, par, **args):
        return self.inner.log_likelihood(par, masks=self._m(args), **args)


def om_dropout(rng, B, n_mid, dtype):
    from oracle import models as om
    return om.dropout_masks(rng, B, n_mid, dtype=dtype)


def _mlp_chain(args):
    cfg, seed, T = args
    from oracle import models as om, samplers as osm
    dt = np.float32 if cfg["dtype"] == "f32" else np.float64
    X, y = mlp_dataset(cfg)
    X = X.astype(dt)
    start = {k: v.astype(dt) for k, v in mlp_start(cfg["n_in"], cfg["n_mid"], cfg["n_out"], cfg["start_seed"]).items()}
    model = _FreshMaskMLP(om.mlp({"alpha": cfg["alpha"]}, cfg["n_in"], cfg["n_mid"], cfg["n_out"]),
                          np.random.RandomState(300007 + seed), dt)
    s = osm.sghmc(model, start, path_length=cfg["path_length"], step_size=cfg["step_size"], verbose=False)
    s.out = io.StringIO()
    s.trace = []
    np.random.seed(100003 + seed)
    epochs = T * cfg["B"] // cfg["N"]
    with np.errstate(over="ignore"):    # exp(E_cur − E_new) overflows to inf → A = min(1, inf) = 1
        post, _ = s.sample(epochs=epochs, burnin=0, batch_size=cfg["B"], rng=np.random.RandomState(seed),
                           X_train=X, y_train=y)
    flat = np.concatenate([np.asarray(post[k]).reshape(epochs, -1) for k in om.MLP_PARAM_NAMES], axis=1)
    acc = np.array([t.get("accepted", True) for t in s.trace], dtype=bool)
    Ls = np.array([t["L"] for t in s.trace], dtype=np.int64)
    return flat.astype(np.float32), acc, Ls


def run_mlp_chains(cfg, seeds, T, workers=None):
    """Independent oracle SGHMC chains of the dropout MLP (cpu/sghmc.py:19-39 with the A1 completion
    over the mlp.py:19-96 restatement, fresh dropout masks per forward) → (draws [C, E, P] float32,
    one per epoch, P = 269,322 at 784-256-256-10; accept flags [C, T]; path lengths [C, T])."""
    return _pool(_mlp_chain, [(cfg, int(s), int(T)) for s in seeds], workers)


def _pool(fn, jobs, workers=None):
    import multiprocessing as mp
    workers = workers or default_workers()
    saved = {k: os.environ.get(k) for k in ("OPENBLAS_NUM_THREADS", "OMP_NUM_THREADS", "MKL_NUM_THREADS")}
    for k in saved:
        os.environ[k] = "1"
    try:
        with mp.get_context("spawn").Pool(workers) as pool:
            res = pool.map(fn, jobs)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return tuple(np.stack([r[i] for r in res]) for i in range(len(res[0])))


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
    jobs = [(kind, cfg, int(s), int(T), float(momentum_scale)) for s in seeds]
    return _pool(_chain, jobs, workers)
