"""GPU parity of the dropout MLP (config 3, hmcx_mlp.hip) against the NumPy restatement
oracle/models.py::mlp (itself cross-checked with torch autograd in test_oracle_golden.py; the
Chainer reference is not runnable here, so MLP parity is pinned to that restatement only).

Dropout masks are injected (the same [3, B, n_mid] arrays on both sides).  Tolerances:
float64 gradients/losses within rel 1e-9 of the largest entry (GEMM summation order only);
float32 within 2e-4 of the largest entry; SGHMC path lengths and accept flags bit-exact, float64
states within rel 1e-8."""
import io

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from oracle import models as om  # noqa: E402
from oracle import samplers as osm  # noqa: E402


def _mlp_cls():
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.models.gpu.mlp import mlp
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu.sghmc import sghmc
    return mlp, sghmc


def _problem(seed, B, n_in, n_mid, n_out, wscale=0.3):
    rs = np.random.RandomState(seed)
    par = {k: rs.normal(0, wscale, s) for k, s in om.mlp_param_shapes(n_in, n_mid, n_out).items()}
    X = rs.rand(B, n_in)
    y = rs.randint(0, n_out, B)
    masks = om.dropout_masks(rs, B, n_mid, dtype=np.float64)
    return par, X, y, masks


def _close(a, b, rel):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    scale = max(np.abs(b).max(), 1e-30)
    err = np.abs(a - b).max()
    assert err <= rel * scale, "max abs err %.3e > %.1e x %.3e" % (err, rel, scale)


SHAPES = [(32, 784, 256, 10), (19, 50, 37, 7), (500, 784, 256, 10), (1, 3, 1, 2), (70, 33, 64, 40)]


@pytest.mark.parametrize("B,n_in,n_mid,n_out", SHAPES)
@pytest.mark.parametrize("dropout", [True, False])
def test_grad_f64_matches_oracle(B, n_in, n_mid, n_out, dropout):
    mlp, _ = _mlp_cls()
    par, X, y, masks = _problem(1, B, n_in, n_mid, n_out)
    ref = om.mlp({"alpha": 0.01}, n_in, n_mid, n_out)
    mk = masks if dropout else None
    g_ref = ref.grad(par, masks=mk, X_train=X, y_train=y)
    m = mlp({"alpha": 0.01}, n_in, n_mid, n_out, dtype=torch.float64, device="cuda:0")
    g = m.grad(par, masks=(masks if dropout else 'off'), X_train=X, y_train=y)
    for k in om.MLP_PARAM_NAMES:
        assert tuple(g[k].shape) == g_ref[k].shape
        _close(g[k].cpu().numpy(), g_ref[k], 1e-9)
    l_ref = ref.log_likelihood(par, masks=mk, X_train=X, y_train=y)
    l = m.log_likelihood(par, masks=(masks if dropout else 'off'), X_train=X, y_train=y)
    assert abs(l - l_ref) <= 1e-11 * max(1.0, abs(l_ref))
    nlp_ref = ref.negative_log_posterior(par, masks=mk, X_train=X, y_train=y)
    nlp = m.negative_log_posterior(par, masks=(masks if dropout else 'off'), X_train=X, y_train=y)
    assert abs(nlp - nlp_ref) <= 1e-11 * max(1.0, abs(nlp_ref))


@pytest.mark.parametrize("B,n_in,n_mid,n_out", SHAPES[:3])
def test_grad_f32_close_to_oracle(B, n_in, n_mid, n_out):
    mlp, _ = _mlp_cls()
    par, X, y, masks = _problem(2, B, n_in, n_mid, n_out)
    # the oracle at float32-rounded inputs
    par32 = {k: v.astype(np.float32).astype(np.float64) for k, v in par.items()}
    X32 = X.astype(np.float32).astype(np.float64)
    mk32 = [mm.astype(np.float32).astype(np.float64) for mm in masks]
    g_ref = om.mlp({"alpha": 0.01}, n_in, n_mid, n_out).grad(par32, masks=mk32, X_train=X32, y_train=y)
    m = mlp({"alpha": 0.01}, n_in, n_mid, n_out, dtype=torch.float32, device="cuda:0")
    g = m.grad(par, masks=masks, X_train=X, y_train=y)
    for k in om.MLP_PARAM_NAMES:
        assert g[k].dtype == torch.float32
        _close(g[k].cpu().numpy(), g_ref[k], 2e-4)


def test_predict_matches_oracle():
    mlp, _ = _mlp_cls()
    par, X, y, masks = _problem(3, 64, 40, 24, 6)
    ref = om.mlp({"alpha": 0.01}, 40, 24, 6)
    m = mlp({"alpha": 0.01}, 40, 24, 6, dtype=torch.float64, device="cuda:0")
    np.testing.assert_array_equal(m.predict(par, X, masks='off'), ref.predict(par, X))
    np.testing.assert_allclose(m.predict(par, X, prob=True, masks='off'), ref.predict(par, X, prob=True),
                               rtol=1e-11, atol=1e-14)
    np.testing.assert_allclose(m.predict(par, X, prob=True, masks=masks),
                               ref.predict(par, X, prob=True, masks=masks), rtol=1e-11, atol=1e-14)


def test_philox_masks_properties():
    mlp, _ = _mlp_cls()
    m = mlp({"alpha": 0.01}, 784, 256, 10, dtype=torch.float32, device="cuda:0", seed=9)
    a = m.draw_masks(500).cpu().numpy()
    b = m.draw_masks(500).cpu().numpy()
    scale = np.float32(1 / 0.9)
    assert a.shape == (3, 500, 256)
    assert set(np.unique(a)) <= {np.float32(0), scale}
    assert abs(np.mean(a == 0) - 0.1) < 0.005                      # keep probability 0.9
    assert np.mean(a != b) > 0.1                                    # fresh masks per forward
    m2 = mlp({"alpha": 0.01}, 784, 256, 10, dtype=torch.float32, device="cuda:0", seed=9)
    np.testing.assert_array_equal(m2.draw_masks(500).cpu().numpy(), a)   # deterministic under the seed


# ----------------------------------------------------------------------------- SGHMC parity
def _mask_stream(B, n_mid):
    """Masks of forward f of global step k: sequential draws of RandomState(1000 + k)."""
    cache = {}

    def get(k, n):
        rs = np.random.RandomState(1000 + k)
        return np.stack([np.stack(om.dropout_masks(rs, B, n_mid, dtype=np.float64)) for _ in range(n)])

    def one(k, f):
        if k not in cache or cache[k].shape[0] <= f:
            cache[k] = get(k, max(f + 1, 2 * (f + 1)))
        return cache[k][f]
    return get, one


class _MaskedOracleMLP:
    """oracle mlp whose grad / accept energies take injected masks in the sampler's call order."""

    def __init__(self, inner, one):
        self.inner, self.one = inner, one
        self.k, self.f, self.in_step = 0, 0, False

    def grad(self, par, **args):
        m = self.one(self.k, self.f)
        self.f += 1
        return self.inner.grad(par, masks=list(m), **args)

    def negative_log_posterior(self, par, **args):
        if not self.in_step:
            return self.inner.negative_log_posterior(par, masks=None, **args)
        m = self.one(self.k, self.f)
        self.f += 1
        return self.inner.negative_log_posterior(par, masks=list(m), **args)

    def log_likelihood(self, par, **args):
        return self.inner.log_likelihood(par, masks=None, **args)


class _OracleSghmc(osm.sghmc):
    def step(self, state, momentum, rng, **args):
        self.model.in_step, self.model.f = True, 0
        out = super().step(state, momentum, rng, **args)
        self.model.in_step = False
        self.model.k += 1
        return out


@pytest.mark.parametrize("order", [list(om.MLP_PARAM_NAMES), ['/l3/b', '/l1/W', '/l2/b', '/l3/W', '/l1/b', '/l2/W']])
def test_sghmc_mlp_matches_oracle(order):
    mlp, sghmc = _mlp_cls()
    n_in, n_mid, n_out, N, B = 24, 20, 5, 120, 30
    rs = np.random.RandomState(4)
    X = rs.rand(N, n_in)
    y = rs.randint(0, n_out, N)
    start = {k: rs.normal(0, 0.2, s) for k, s in om.mlp_param_shapes(n_in, n_mid, n_out).items()}
    start = {k: start[k] for k in order}
    get, one = _mask_stream(B, n_mid)
    kw = dict(path_length=0.02, step_size=0.005, verbose=True)

    o = _OracleSghmc(_MaskedOracleMLP(om.mlp({"alpha": 0.01}, n_in, n_mid, n_out), one), start, **kw)
    o.trace, o.out = [], io.StringIO()
    np.random.seed(7)
    post_r, _ = o.sample(epochs=2, burnin=1, batch_size=B, rng=np.random.RandomState(8), X_train=X, y_train=y)

    m = mlp({"alpha": 0.01}, n_in, n_mid, n_out, dtype=torch.float64, device="cuda:0")
    s = sghmc(m, start, noise='numpy', **kw)
    s.mask_provider = get
    s.trace, s.out = [], io.StringIO()
    np.random.seed(7)
    post_g, logp_g = s.sample(epochs=2, burnin=1, batch_size=B, rng=np.random.RandomState(8), X_train=X, y_train=y)

    assert len(s.trace) == len(o.trace) == 12
    assert [t["L"] for t in s.trace] == [t["L"] for t in o.trace]
    assert max(t["L"] for t in o.trace) >= 3                       # real trajectories
    assert [t["accepted"] for t in s.trace] == [t["accepted"] for t in o.trace]
    np.testing.assert_allclose([t["A"] for t in s.trace], [t["A"] for t in o.trace], rtol=1e-8, atol=1e-12)
    for k in order:
        np.testing.assert_allclose(post_g[k], post_r[k], rtol=1e-8, atol=1e-10)
    assert np.all(np.isfinite(logp_g))


def test_sghmc_mlp_config3_philox():
    """Config 3 shape (784-256-256-10, B = 500), float32, device masks and noise: finite, mixing,
    deterministic under the seed."""
    mlp, sghmc = _mlp_cls()
    N, B = 3000, 500
    rs = np.random.RandomState(0)
    X = rs.rand(N, 784).astype(np.float32)
    y = rs.randint(0, 10, N)

    def run():
        m = mlp({"alpha": 0.01}, 784, 256, 10, dtype=torch.float32, device="cuda:0")
        s = sghmc(m, m.init_params(1), path_length=0.005, step_size=1e-3, noise='philox', seed=3)
        s.trace, s.out = [], io.StringIO()
        post, logp = s.sample(epochs=1, burnin=1, batch_size=B, X_train=X, y_train=y)
        return post, logp, s.trace

    p1, l1, t1 = run()
    p2, l2, t2 = run()
    assert all(np.all(np.isfinite(v)) for v in p1.values()) and np.all(np.isfinite(l1))
    for k in p1:
        np.testing.assert_array_equal(p1[k], p2[k])
    assert [t["L"] for t in t1] == [t["L"] for t in t2]
    assert np.mean([t["accepted"] for t in t1]) > 0.2


def test_sghmc_mlp_config3_f64_trajectory_matches_oracle():
    """Config 3 at full size — MyNetwork(784, 256, 10) (two hidden layers of 256, mlp.py:24-26),
    minibatch 500 — float64 SGHMC with injected dropout masks against the NumPy restatement of
    mlp.py:28-31,47-64 (parity unpinned vs Chainer): 4 steps of 1-3 leapfrog iterations,
    path lengths and accept flags bit-exact, state within rel 1e-8."""
    mlp, sghmc = _mlp_cls()
    n_in, n_mid, n_out, N, B = 784, 256, 10, 1000, 500
    rs = np.random.RandomState(11)
    X = rs.rand(N, n_in)
    y = rs.randint(0, n_out, N)
    start = {k: rs.normal(0, 0.05, s) for k, s in om.mlp_param_shapes(n_in, n_mid, n_out).items()}
    get, one = _mask_stream(B, n_mid)
    kw = dict(path_length=2e-3, step_size=1e-3, verbose=True)

    o = _OracleSghmc(_MaskedOracleMLP(om.mlp({"alpha": 0.01}, n_in, n_mid, n_out), one), start, **kw)
    o.trace, o.out = [], io.StringIO()
    np.random.seed(21)
    post_r, _ = o.sample(epochs=1, burnin=1, batch_size=B, rng=np.random.RandomState(22), X_train=X, y_train=y)

    m = mlp({"alpha": 0.01}, n_in, n_mid, n_out, dtype=torch.float64, device="cuda:0")
    s = sghmc(m, start, noise='numpy', **kw)
    s.mask_provider = get
    s.trace, s.out = [], io.StringIO()
    np.random.seed(21)
    post_g, logp_g = s.sample(epochs=1, burnin=1, batch_size=B, rng=np.random.RandomState(22), X_train=X, y_train=y)

    assert len(s.trace) == len(o.trace) == 4
    assert [t["L"] for t in s.trace] == [t["L"] for t in o.trace]
    assert max(t["L"] for t in o.trace) >= 2                       # at least one real trajectory
    assert [t["accepted"] for t in s.trace] == [t["accepted"] for t in o.trace]
    np.testing.assert_allclose([t["A"] for t in s.trace], [t["A"] for t in o.trace], rtol=1e-8, atol=1e-12)
    for k in start:
        np.testing.assert_allclose(post_g[k], post_r[k], rtol=1e-8, atol=1e-10)


@pytest.mark.parametrize("fwdr", ["1", "0"])
def test_sghmc_mlp_config3_f32_trajectory_matches_oracle(fwdr, monkeypatch):
    """Config 3 in float32 — the bench's dtype — through the path the bench times: the batched
    iterations with every forward of an iteration in one k_fwdr launch (HMCX_MLP_FWDR=1, default) or
    the k_mm fused forwards (=0), buffer masks injected (MK_VALS, the keep-flag kernels' twin), against
    the NumPy restatement in float64 at the float32-rounded inputs: 4 steps of 1-3 leapfrog
    iterations (iterations 0 and n−1 carry the energy forwards), path lengths and accept flags
    bit-exact, acceptance probabilities within 1e-3, the state within 2e-5 of its largest entry
    (float32 rounding through the trajectory; the kernels differ from the oracle in summation order)."""
    mlp, sghmc = _mlp_cls()
    monkeypatch.setenv("HMCX_MLP_FWDR", fwdr)
    n_in, n_mid, n_out, N, B = 784, 256, 10, 1000, 500
    rs = np.random.RandomState(11)
    X = rs.rand(N, n_in).astype(np.float32).astype(np.float64)
    y = rs.randint(0, n_out, N)
    start = {k: rs.normal(0, 0.05, s).astype(np.float32).astype(np.float64)
             for k, s in om.mlp_param_shapes(n_in, n_mid, n_out).items()}
    get, one = _mask_stream(B, n_mid)
    kw = dict(path_length=3e-3, step_size=1e-3, verbose=True)

    o = _OracleSghmc(_MaskedOracleMLP(om.mlp({"alpha": 0.01}, n_in, n_mid, n_out), one), start, **kw)
    o.trace, o.out = [], io.StringIO()
    np.random.seed(21)
    post_r, _ = o.sample(epochs=1, burnin=1, batch_size=B, rng=np.random.RandomState(22), X_train=X, y_train=y)

    m = mlp({"alpha": 0.01}, n_in, n_mid, n_out, dtype=torch.float32, device="cuda:0")
    s = sghmc(m, start, noise='numpy', **kw)
    s.mask_provider = get
    s.trace, s.out = [], io.StringIO()
    np.random.seed(21)
    post_g, _ = s.sample(epochs=1, burnin=1, batch_size=B, rng=np.random.RandomState(22), X_train=X, y_train=y)

    assert len(s.trace) == len(o.trace) == 4
    assert [t["L"] for t in s.trace] == [t["L"] for t in o.trace]
    assert max(t["L"] for t in o.trace) >= 3                       # at least one multi-iteration trajectory
    assert [t["accepted"] for t in s.trace] == [t["accepted"] for t in o.trace]
    np.testing.assert_allclose([t["A"] for t in s.trace], [t["A"] for t in o.trace], rtol=0, atol=1e-3)
    for k in start:
        _close(post_g[k], post_r[k], 2e-5)


@pytest.mark.parametrize("dtype,rtol", [(torch.float64, 1e-13), (torch.float32, 1e-6)])
def test_mlp_log_prior_device_reduction(dtype, rtol):
    """mlp.log_prior (mlp.py:40-45, −Σ_var ½·alpha·Σθ²/dim) with Σθ² from hmcx_sumsq against the
    NumPy restatement."""
    mlp, _ = _mlp_cls()
    rs = np.random.RandomState(9)
    par = {k: rs.normal(0, 0.3, s) for k, s in om.mlp_param_shapes(30, 24, 7).items()}
    m = mlp({"alpha": 0.05}, 30, 24, 7, dtype=dtype, device="cuda:0")
    ref = om.mlp({"alpha": 0.05}, 30, 24, 7).log_prior({k: v.astype(np.float32 if dtype == torch.float32 else np.float64)
                                                         for k, v in par.items()})
    assert abs(m.log_prior(par) - ref) <= rtol * abs(ref)


# ----------------------------------------------------------------------------- fused-launch timeouts
def _mlp_f64_run(monkeypatch=None, force=None):
    """The config-3 f64 trajectory of test_sghmc_mlp_config3_f64_trajectory_matches_oracle through
    the sampler, optionally with HMCX_MLP_FORCE_ABORT (the given fused layer-2/3 launch of the first
    call raises the MLP abort word and never publishes its partials)."""
    mlp, sghmc = _mlp_cls()
    n_in, n_mid, n_out, N, B = 784, 256, 10, 1000, 500
    rs = np.random.RandomState(11)
    X = rs.rand(N, n_in)
    y = rs.randint(0, n_out, N)
    start = {k: rs.normal(0, 0.05, s) for k, s in om.mlp_param_shapes(n_in, n_mid, n_out).items()}
    get, one = _mask_stream(B, n_mid)
    kw = dict(path_length=2e-3, step_size=1e-3, verbose=True)
    m = mlp({"alpha": 0.01}, n_in, n_mid, n_out, dtype=torch.float64, device="cuda:0")
    s = sghmc(m, start, noise='numpy', **kw)
    s.mask_provider = get
    s.trace, s.out = [], io.StringIO()
    if force is not None:
        monkeypatch.setenv("HMCX_MLP_FORCE_ABORT", str(force))
    try:
        np.random.seed(21)
        post, logp = s.sample(epochs=1, burnin=1, batch_size=B, rng=np.random.RandomState(22), X_train=X, y_train=y)
    finally:
        if force is not None:
            monkeypatch.delenv("HMCX_MLP_FORCE_ABORT")
    return post, logp, s.trace, m


@pytest.mark.allow_recovery
def test_mlp_fused_timeout_is_recovered_in_process(monkeypatch, capfd):
    """A fused MLP launch whose exchange times out (forced) makes its call report out_abort; the
    sampler restores the state, re-runs the call unfused and continues: the trajectory equals the
    undisturbed run's — bit-exact path lengths / accept flags, states within rel 1e-10 (the fused and
    unfused launches differ only in the summation order of the logits)."""
    ref_post, ref_logp, ref_tr, m = _mlp_f64_run()
    before = m.ctx.recoveries()["mlp_fused"]
    try:
        post, logp, tr, m = _mlp_f64_run(monkeypatch, force=3)
        err = capfd.readouterr().err
        assert "re-running the call unfused" in err
        assert not m.ctx.mlp_fuse
        # exactly the forced call is re-run (the context stays unfused after it): counted once
        assert m.ctx.recoveries()["mlp_fused"] == before + 1
        assert [t["L"] for t in tr] == [t["L"] for t in ref_tr]
        assert [t["accepted"] for t in tr] == [t["accepted"] for t in ref_tr]
        for k in ref_post:
            np.testing.assert_allclose(post[k], ref_post[k], rtol=1e-10, atol=1e-13)
        np.testing.assert_allclose(logp, ref_logp, rtol=1e-10)
    finally:
        m.ctx.set_mlp_fuse(True)


@pytest.mark.allow_recovery
def test_mlp_timeout_leaves_softmax_persistent_path_alone(monkeypatch):
    """The MLP abort word is its own: after a forced MLP timeout the persistent single-chain softmax
    SGHMC kernel (which has its own sticky word) still runs and matches the oracle."""
    from test_gpu_samplers import _run_gpu, _run_oracle
    from oracle import inputs as gi
    _, _, _, m = _mlp_f64_run(monkeypatch, force=0)
    m.ctx.set_mlp_fuse(True)
    c = gi.TRAJ_CONFIGS["sghmc_mnist"]
    post_g, logp_g, tr_g, _ = _run_gpu(c, path=2)
    m.ctx.set_sghmc_path(0)
    post_r, logp_r, tr_r, _ = _run_oracle(c)
    assert [t["accepted"] for t in tr_g] == [t["accepted"] for t in tr_r]
    np.testing.assert_allclose(post_g["weights"], post_r["weights"], rtol=1e-9, atol=1e-12)


def test_mlp_timeout_reported_through_c_abi_without_out_abort(monkeypatch):
    """Plain C callers (out_abort = NULL) get an error from the call itself.  The k_mm fused forwards
    (HMCX_MLP_FWDR=0) are the launches with an exchange that can time out; k_fwdr has none."""
    from dropout_hamiltonian_montecarlo_amd import _native as nat
    monkeypatch.setenv("HMCX_MLP_FWDR", "0")
    mlp, _ = _mlp_cls()
    n_in, n_mid, n_out, B = 784, 256, 10, 500
    m = mlp({"alpha": 0.01}, n_in, n_mid, n_out, dtype=torch.float32, device="cuda:0")
    rs = np.random.RandomState(3)
    X = torch.from_numpy(rs.rand(B, n_in)).to("cuda:0", torch.float32)
    y = torch.from_numpy(rs.randint(0, n_out, B)).to("cuda:0", torch.int32)
    par = [torch.from_numpy(v).to("cuda:0", torch.float32).contiguous() for v in m.init_params(2).values()]
    row0, eps, n_iter, u = (np.zeros(1, np.int64), np.full(1, 1e-3), np.full(1, 2, np.int32), np.full(1, 0.5))
    zoff = np.zeros(1, np.int64)
    outs = torch.zeros(8, dtype=torch.float64, device="cuda:0")
    acc = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    a = nat.MlpSghmcArgs()
    a.dtype, a.B, a.n_in, a.n_mid, a.n_out, a.n_steps = m.code, B, n_in, n_mid, n_out, 1
    for i in range(6):
        a.order[i] = i
    a.alpha = 0.01
    a.X, a.y = nat.ptr(X), nat.ptr(y)
    a.row0, a.eps = row0.ctypes.data_as(nat.c_i64p), eps.ctypes.data_as(nat.c_dblp)
    a.n_iter, a.u_accept = n_iter.ctypes.data_as(nat.c_i32p), u.ctypes.data_as(nat.c_dblp)
    a.noise_mode = a.mask_mode = nat.NOISE_PHILOX
    a.noise_off = a.mask_off = zoff.ctypes.data_as(nat.c_i64p)
    a.seed, a.chain, a.step_base = 1, 0, 0
    for i in range(6):
        a.par.p[i] = par[i].data_ptr()
    a.out_A, a.out_accepted, a.out_loss = outs.data_ptr(), acc.data_ptr(), outs.data_ptr() + 8
    monkeypatch.setenv("HMCX_MLP_FORCE_ABORT", "1")
    assert m.ctx.lib.hmcx_mlp_sghmc_run(m.ctx.h, a) != 0
    assert b"timed out" in m.ctx.lib.hmcx_last_error(m.ctx.h)
    monkeypatch.delenv("HMCX_MLP_FORCE_ABORT")
    assert m.ctx.lib.hmcx_mlp_sghmc_run(m.ctx.h, a) == 0          # the word was lowered
    torch.cuda.synchronize()


def _philox_host(c0, c1, c2, c3, seed):
    """Philox4x32-10 of counters (c0 vector, c1..c3 scalars) under key `seed`: the four output words."""
    M0, M1, m32 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57), np.uint64(0xFFFFFFFF)
    c0 = np.asarray(c0, dtype=np.uint64)
    c1, c2, c3 = (np.full(c0.shape, v & 0xFFFFFFFF, dtype=np.uint64) for v in (c1, c2, c3))
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    for _ in range(10):
        p0, p1 = M0 * c0, M1 * c2
        c0, c1, c2, c3 = (p1 >> np.uint64(32)) ^ c1 ^ np.uint64(k0), p1 & m32, \
            (p0 >> np.uint64(32)) ^ c3 ^ np.uint64(k1), p0 & m32
        k0, k1 = (k0 + 0x9E3779B9) & 0xFFFFFFFF, (k1 + 0xBB67AE85) & 0xFFFFFFFF
    return c0, c1, c2, c3


def _keep_group_host(seed, n3, slot, step, chain):
    """Host twin of hmcx_mlp.hip::keep_group, written from its definition (per-byte compares, not the
    kernel's SWAR form): the keep flags of elements 0 … n3 − 1 of one forward."""
    nG = (n3 + 63) // 64
    G = np.arange(nG, dtype=np.uint64)
    words = []                                                     # word kk = 4k + q of the group
    for k in range(4):
        words.extend(_philox_host(4 * G + k, slot, step, chain, seed))
    p = np.arange(64)
    widx = 8 * (p // 32) + p % 8                                   # element p: word, byte
    byte = np.stack([(words[w] >> np.uint64(8 * ((q // 8) % 4))) & np.uint64(0xFF)
                     for q, w in zip(p, widx)], axis=1).astype(np.int64)          # [nG, 64]
    keep = byte > 0x19
    for g in np.nonzero((byte == 0x19).any(axis=1))[0]:
        amb = np.nonzero(byte[g] == 0x19)[0]                       # ascending element order
        for a, e in enumerate(amb):
            r = _philox_host([0x80000000 | (int(g) << 3) | (a // 8)], slot, step, chain, seed)
            h = a % 8
            x = (int(r[h // 2][0]) >> (16 * (h % 2))) & 0xFFFF
            keep[g, e] = x >= 0x999A
    return keep.reshape(-1)[:n3]


@pytest.mark.parametrize("B,n_mid", [(19, 37), (500, 256)])
def test_api_masks_equal_host_keep_groups(B, n_mid):
    """hmcx_mlp_masks (and with it every Philox keep flag of the sampler, test below) is bit for bit the
    host restatement of the grouped keep-flag draw: 16 flags per Philox block, the byte == 0x19 ties
    resolved from the fallback blocks — a ragged last group (n3 = 2109) and config 3's 384,000 flags,
    among which ≈ 1,500 ties."""
    from dropout_hamiltonian_montecarlo_amd import _native as nat
    ctx = nat.context(0)
    n3 = 3 * B * n_mid
    out = torch.empty(n3, dtype=torch.float32, device="cuda:0")
    seed, chain, step, slot = 0x123456789AB, 7, 11, (nat.MLP_MASK_SLOT0 + 5) & 0xFFFFFFFF
    ctx.check(ctx.lib.hmcx_mlp_masks(ctx.h, nat.HMCX_F32, B, n_mid, seed, chain, step, slot, nat.ptr(out)),
              "hmcx_mlp_masks")
    got = out.cpu().numpy()
    want = _keep_group_host(seed, n3, slot, step, chain)
    np.testing.assert_array_equal(got != 0, want)
    assert set(np.unique(got)) <= {np.float32(0), np.float32(1 / 0.9)}


@pytest.mark.parametrize("variant", ["keep", "philox-h1"])
def test_sampler_philox_masks_equal_api_masks(variant, monkeypatch):
    """In Philox mode the sampler's dropout flags — stored once per step by k_mlp_keep (default) or
    drawn inside the kernels where they are read (HMCX_MLP_MASKS=philox, with the backward reading
    the stored h1 instead of the masks, HMCX_MLP_H1=1) — are the values hmcx_mlp_masks gives for the
    same (seed, chain, step, slot): a run fed those API masks as buffers follows the Philox-mask run
    bit for bit (float64, Philox noise in both)."""
    if variant == "philox-h1":
        monkeypatch.setenv("HMCX_MLP_MASKS", "philox")
        monkeypatch.setenv("HMCX_MLP_H1", "1")
    from dropout_hamiltonian_montecarlo_amd import _native as nat
    mlp, sghmc = _mlp_cls()
    n_in, n_mid, n_out, N, B = 784, 256, 10, 1000, 500
    rs = np.random.RandomState(5)
    X = rs.rand(N, n_in)
    y = rs.randint(0, n_out, N)
    m = mlp({"alpha": 0.01}, n_in, n_mid, n_out, dtype=torch.float64, device="cuda:0")
    start = m.init_params(4)
    kw = dict(path_length=3e-3, step_size=1e-3, verbose=False, noise='philox', seed=5, chain=3)

    def api_masks(k, n):
        out = torch.empty((n, 3, B, n_mid), dtype=torch.float64, device="cuda:0")
        for f in range(n):
            m.ctx.check(m.ctx.lib.hmcx_mlp_masks(m.ctx.h, m.code, B, n_mid, 5, 3, k & 0xFFFFFFFF,
                                                 (nat.MLP_MASK_SLOT0 + f) & 0xFFFFFFFF, nat.ptr(out[f])),
                        "hmcx_mlp_masks")
        return out.cpu().numpy()

    runs = []
    for provider in (None, api_masks):
        s = sghmc(m, start, **kw)
        s.mask_provider = provider
        s.trace, s.out = [], io.StringIO()
        post, _ = s.sample(epochs=2, burnin=1, batch_size=B, X_train=X, y_train=y)
        runs.append((post, [t["L"] for t in s.trace], [t["accepted"] for t in s.trace]))
    (p1, L1, a1), (p2, L2, a2) = runs
    assert L1 == L2 and a1 == a2 and max(L1) >= 2
    for k in p1:
        np.testing.assert_array_equal(p1[k], p2[k])


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("order", ["natural", "w1-first-permuted"])
def test_batched_iterations_equal_one_at_a_time(dtype, order, monkeypatch):
    """The sampler's batched iterations (the six sub-steps of a leapfrog iteration as one fused-forward
    launch, one layer-1-backward launch and the two weight-gradient launches: they only depend on the
    previous iteration) give the one-sub-step-at-a-time trajectory bit for bit (HMCX_MLP_BATCH=0):
    config-3 shape, Philox noise and masks, both dtypes, the natural variable order and a permuted
    one with W1 first."""
    mlp, sghmc = _mlp_cls()
    n_in, n_mid, n_out, N, B = 784, 256, 10, 1000, 500
    rs = np.random.RandomState(9)
    X = rs.rand(N, n_in)
    y = rs.randint(0, n_out, N)
    m = mlp({"alpha": 0.01}, n_in, n_mid, n_out, dtype=dtype, device="cuda:0")
    start = m.init_params(6)
    if order != "natural":
        keys = list(start)
        start = {k: start[k] for k in [keys[0], keys[4], keys[2], keys[5], keys[1], keys[3]]}
    kw = dict(path_length=4e-3, step_size=1e-3, verbose=False, noise='philox', seed=7, chain=1)
    # the k_mm fused forwards: the one-at-a-time order runs the same kernels (k_fwdr sums in another
    # order: test_batched_fwdr_close_to_one_at_a_time)
    monkeypatch.setenv("HMCX_MLP_FWDR", "0")
    runs = []
    for batch in ("1", "0"):
        monkeypatch.setenv("HMCX_MLP_BATCH", batch)
        s = sghmc(m, start, **kw)
        s.trace, s.out = [], io.StringIO()
        post, logp = s.sample(epochs=2, burnin=1, batch_size=B, X_train=X, y_train=y)
        runs.append((post, logp, [t["L"] for t in s.trace], [t["accepted"] for t in s.trace]))
    monkeypatch.delenv("HMCX_MLP_BATCH")
    (p1, l1, L1, a1), (p2, l2, L2, a2) = runs
    assert L1 == L2 and a1 == a2 and max(L1) >= 3
    for k in p1:
        np.testing.assert_array_equal(p1[k], p2[k])
    np.testing.assert_array_equal(l1, l2)


def test_batched_fwdr_close_to_one_at_a_time(monkeypatch):
    """float32 batched iterations with k_fwdr (the default: all forwards of an iteration in one launch,
    per-16-row-block partials) against the one-sub-step-at-a-time order on the same Philox noise and
    masks: the same path lengths and accept flags, states within float32 summation-order differences."""
    mlp, sghmc = _mlp_cls()
    n_in, n_mid, n_out, N, B = 784, 256, 10, 1000, 500
    rs = np.random.RandomState(9)
    X = rs.rand(N, n_in)
    y = rs.randint(0, n_out, N)
    m = mlp({"alpha": 0.01}, n_in, n_mid, n_out, dtype=torch.float32, device="cuda:0")
    start = m.init_params(6)
    kw = dict(path_length=4e-3, step_size=1e-3, verbose=False, noise='philox', seed=7, chain=1)
    monkeypatch.setenv("HMCX_MLP_FWDR", "1")
    runs = []
    for batch in ("1", "0"):
        monkeypatch.setenv("HMCX_MLP_BATCH", batch)
        s = sghmc(m, start, **kw)
        s.trace, s.out = [], io.StringIO()
        post, logp = s.sample(epochs=2, burnin=1, batch_size=B, X_train=X, y_train=y)
        runs.append((post, logp, [t["L"] for t in s.trace], [t["accepted"] for t in s.trace]))
    (p1, l1, L1, a1), (p2, l2, L2, a2) = runs
    assert L1 == L2 and a1 == a2 and max(L1) >= 3
    for k in p1:
        _close(p1[k], p2[k], 2e-5)
    np.testing.assert_allclose(l1, l2, rtol=1e-4)


# ----------------------------------------------------------------------------- full-batch HMC (generic loop)
def test_hmc_mlp_generic_loop_matches_oracle():
    """Full-batch HMC on the MLP (inference/gpu/hmc.py's generic loop: libhmcx gradients, hmcx_axpy
    kicks / drifts; the step's two energies — loss pieces, Σθ², Σp² — enqueued into one device buffer
    and read back once) against the oracle's cpu/hmc.py restatement, both fed the same dropout masks in
    call order: path lengths and accept flags bit-exact, A within rel 1e-9, states within rel 1e-8,
    losses within rel 1e-10."""
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.models.gpu.mlp import mlp
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu.hmc import hmc
    n_in, n_mid, n_out, N = 24, 20, 5, 60
    rs = np.random.RandomState(14)
    X = rs.rand(N, n_in)
    y = rs.randint(0, n_out, N)
    start = {k: rs.normal(0, 0.2, s) for k, s in om.mlp_param_shapes(n_in, n_mid, n_out).items()}
    get, one = _mask_stream(N, n_mid)
    kw = dict(path_length=0.03, step_size=0.005, verbose=True)

    class GpuMasked(mlp):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            self.k, self.f, self.in_step = 0, 0, False

        def _m(self):
            m = one(self.k, self.f)
            self.f += 1
            return list(m)

        def grad(self, par, masks=None, **args):
            return super().grad(par, masks=self._m(), **args)

        def negative_log_posterior(self, par, masks=None, **args):
            return super().negative_log_posterior(par, masks=self._m() if self.in_step else 'off', **args)

        def energy_parts_device(self, par, out, masks=None, **args):
            return super().energy_parts_device(par, out, masks=self._m() if self.in_step else 'off', **args)

    def stepping(cls):
        class S(cls):
            def step(self, state, momentum, rng, **args):
                self.model.in_step, self.model.f = True, 0
                out = super().step(state, momentum, rng, **args)
                self.model.in_step = False
                self.model.k += 1
                return out
        return S

    o = stepping(osm.hmc)(_MaskedOracleMLP(om.mlp({"alpha": 0.01}, n_in, n_mid, n_out), one), start, **kw)
    o.trace, o.out = [], io.StringIO()
    np.random.seed(3)
    post_o, loss_o, _, _ = o.sample(5, 1, np.random.RandomState(4), X_train=X, y_train=y)

    g = stepping(hmc)(GpuMasked({"alpha": 0.01}, n_in, n_mid, n_out, dtype=torch.float64, device="cuda:0"), start, **kw)
    g.trace, g.out = [], io.StringIO()
    np.random.seed(3)
    post_g, loss_g, _, _ = g.sample(5, 1, np.random.RandomState(4), X_train=X, y_train=y)

    assert [t["L"] for t in g.trace] == [t["L"] for t in o.trace]
    assert max(t["L"] for t in o.trace) >= 3                       # real trajectories
    assert [t["accepted"] for t in g.trace] == [t["accepted"] for t in o.trace]
    np.testing.assert_allclose([t["A"] for t in g.trace], [t["A"] for t in o.trace], rtol=1e-9, atol=1e-12)
    for k in start:
        np.testing.assert_allclose(np.asarray(post_g[k]), np.asarray(post_o[k]), rtol=1e-8, atol=1e-10)
    np.testing.assert_allclose(loss_g, loss_o, rtol=1e-10)


@pytest.mark.parametrize("dtype,masks", [("f64", None), ("f32", None), ("f64", "off"), ("f64", "fixed")])
def test_hmc_mlp_device_leapfrog_equals_host_loop(monkeypatch, dtype, masks):
    """hmcx_mlp_hmc_leapfrog (a step's whole trajectory in one call) against the host loop it replaces
    (HMCX_HMC_HOST_LOOP=1: model.grad + hmcx_axpy per variable, hmc.py:46-56): the same kernels in the
    same order, so path lengths, accept flags, acceptance probabilities, losses and the posterior are
    bit-identical — with Philox masks per gradient call (the same slots as the host loop's grad calls),
    without dropout, and with one injected mask set."""
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.models.gpu.mlp import mlp
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu.hmc import hmc
    n_in, n_mid, n_out, N = 24, 20, 5, 60
    rs = np.random.RandomState(21)
    X = rs.rand(N, n_in)
    y = rs.randint(0, n_out, N)
    start = {k: rs.normal(0, 0.2, s) for k, s in om.mlp_param_shapes(n_in, n_mid, n_out).items()}
    # a non-canonical start order: the sub-steps follow the caller's keys
    keys = ['/l2/W', '/l1/b', '/l3/b', '/l1/W', '/l3/W', '/l2/b']
    start = {k: start[k] for k in keys}
    args = dict(X_train=X, y_train=y)
    if masks == "off":
        args["masks"] = "off"
    elif masks == "fixed":
        args["masks"] = [(rs.rand(N, n_mid) >= 0.1) / 0.9 for _ in range(3)]
    tdt = torch.float64 if dtype == "f64" else torch.float32

    def run(host):
        if host:
            monkeypatch.setenv("HMCX_HMC_HOST_LOOP", "1")
        else:
            monkeypatch.delenv("HMCX_HMC_HOST_LOOP", raising=False)
        m = mlp({"alpha": 0.01}, n_in, n_mid, n_out, dtype=tdt, device="cuda:0", seed=5)
        s = hmc(m, start, path_length=0.03, step_size=0.005, verbose=True)
        s.trace, s.out = [], io.StringIO()
        np.random.seed(3)
        post, loss, _, _ = s.sample(4, 1, np.random.RandomState(4), **args)
        return s.trace, post, loss, m._mask_calls

    tr_h, post_h, loss_h, calls_h = run(True)
    tr_d, post_d, loss_d, calls_d = run(False)
    assert max(t["L"] for t in tr_h) >= 3
    assert tr_d == tr_h
    assert calls_d == calls_h
    np.testing.assert_array_equal(loss_d, loss_h)
    for k in start:
        np.testing.assert_array_equal(np.asarray(post_d[k]), np.asarray(post_h[k]))


@pytest.mark.parametrize("n_iter", [0, 1, 3])
@pytest.mark.parametrize("masks", ["off", "fixed"])
def test_hmc_mlp_leapfrog_returns_full_gradient_at_final_position(n_iter, masks):
    """hmcx_mlp_hmc_leapfrog's contract (include/hmcx.h): on return g holds the gradient of all six
    variables at the final position — also with n_iter = 0 — as one hmcx_mlp_grad call at that q
    with the same masks gives it (hmc.py:52 is the gradient the trajectory ends on)."""
    mlp, _ = _mlp_cls()
    n_in, n_mid, n_out, B = 24, 20, 5, 40
    par, X, y, mk = _problem(31, B, n_in, n_mid, n_out)
    m = mlp({"alpha": 0.01}, n_in, n_mid, n_out, dtype=torch.float64, device="cuda:0", seed=5)
    keys = ['/l2/W', '/l1/b', '/l3/b', '/l1/W', '/l3/W', '/l2/b']
    rs = np.random.RandomState(2)
    q = {k: torch.as_tensor(par[k], device="cuda:0").contiguous() for k in keys}
    p = {k: torch.as_tensor(rs.normal(size=par[k].shape), device="cuda:0").contiguous() for k in keys}
    margs = "off" if masks == "off" else [mk[0], mk[1], mk[2]]
    g = m.leapfrog_device(q, p, n_iter, 0.005, keys, masks=margs, X_train=X, y_train=y)
    ref = m.grad({k: q[k] for k in keys}, masks=margs, X_train=X, y_train=y)
    for k in keys:
        _close(g[k].cpu().numpy(), ref[k].cpu().numpy(), 1e-12)
