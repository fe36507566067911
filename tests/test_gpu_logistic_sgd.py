"""GPU parity of the logistic model (hmcx_logistic_*: the softmax kernels with the sigmoid link)
and of momentum SGD (hmcx_sgd_run, sgd.fit / fit_dropout) against the NumPy restatement, itself
pinned bit for bit to the reference's own outputs (tests/test_oracle_logistic.py).

Tolerances: float64 kernels differ from NumPy only by summation order → gradients within 1e-12 of
the |X|ᵀ|y − ŷ| + α|θ| scale, SGD trajectories within rel 1e-9; float32 within 2e-5 of the scale."""
import io
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from oracle import inputs as gi  # noqa: E402
from oracle import models as om  # noqa: E402
from oracle import samplers as osm  # noqa: E402


def _logistic(dtype=torch.float64, alpha=0.25):
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.models.gpu.logistic import logistic
    return logistic({"alpha": alpha}, dtype=dtype, device="cuda:0")


def _scale(X, y, W, b, alpha):
    m = om.logistic({"alpha": alpha})
    R = np.abs(y.reshape(-1, 1) - m.net({"weights": W, "bias": b}, X_train=X))
    return np.abs(X).T @ R + alpha * np.abs(W), R.sum(0) + alpha * np.abs(b)


@pytest.mark.parametrize("i", range(len(gi.LOGISTIC_CASES)))
def test_logistic_f64_vs_oracle_and_golden(golden_dir, i):
    d = np.load(os.path.join(golden_dir, "logistic.npz"))
    seed, B, D, ws = gi.LOGISTIC_CASES[i]
    X, y, W, b = gi.logistic_inputs(seed, B, D, wscale=ws)
    par = {"weights": W, "bias": b}
    ref, m = om.logistic({"alpha": 0.25}), _logistic()
    g = m.grad(par, X_train=X, y_train=y)
    r = ref.grad(par, X_train=X, y_train=y)
    sW, sb = _scale(X, y, W, b, 0.25)
    assert np.all(np.abs(g["weights"].cpu().numpy() - r["weights"]) <= 1e-12 * sW + 1e-300)
    assert np.all(np.abs(g["bias"].cpu().numpy() - r["bias"]) <= 1e-12 * sb + 1e-300)
    np.testing.assert_allclose(g["weights"].cpu().numpy(), d["c%d_gW" % i], rtol=1e-10, atol=1e-10)
    # rel error of sigmoid(z) grows like |z|·ulp (exp amplifies the GEMM summation-order error of z)
    np.testing.assert_allclose(m.net(par, X_train=X).cpu().numpy(), d["c%d_net" % i], rtol=1e-11, atol=1e-300)
    ll, nlp, lp = d["c%d_scalars" % i]
    assert abs(m.log_likelihood(par, X_train=X, y_train=y) - ll) <= 1e-12 * max(1.0, abs(ll)) * np.sqrt(B)
    assert abs(m.log_prior(par) - lp) <= 1e-12 * max(1.0, abs(lp))
    assert abs(m.negative_log_posterior(par, X_train=X, y_train=y) - nlp) <= 1e-11 * max(1.0, abs(nlp))
    bs = max(1, B // 3)
    np.testing.assert_array_equal(m.predict(par, X, prob=False, batchsize=bs), d["c%d_pred" % i])
    np.testing.assert_allclose(m.predict(par, X, prob=True, batchsize=bs), d["c%d_predp" % i], rtol=1e-11)


def test_logistic_f32_close():
    X, y, W, b = gi.logistic_inputs(1, 500, 784, wscale=0.05)
    par = {"weights": W, "bias": b}
    g = _logistic(torch.float32).grad(par, X_train=X, y_train=y)
    r = om.logistic({"alpha": 0.25}).grad(par, X_train=X, y_train=y)
    sW, sb = _scale(X, y, W, b, 0.25)
    assert np.all(np.abs(g["weights"].cpu().numpy() - r["weights"]) <= 2e-5 * (sW + 1))
    assert np.all(np.abs(g["bias"].cpu().numpy() - r["bias"]) <= 2e-5 * (sb + 1))


@pytest.mark.parametrize("C", [3, 70])
def test_logistic_parameter_sets(C):
    """C parameter sets at once (W [D][C], b [C]; e.g. posterior samples): C independent gradients
    and log-likelihoods."""
    from dropout_hamiltonian_montecarlo_amd import _native as nat
    X, y, _, _ = gi.logistic_inputs(5, 90, 12)
    rs = np.random.RandomState(C)
    Ws, bs = rs.normal(0, 0.5, (C, 12, 1)), rs.normal(0, 0.5, (C, 1))
    dev = torch.device("cuda:0")
    Wd = torch.from_numpy(np.ascontiguousarray(Ws[:, :, 0].T)).to(dev)
    bd = torch.from_numpy(bs[:, 0].copy()).to(dev)
    Xd, yd = torch.from_numpy(X).to(dev), torch.from_numpy(y).to(dev)
    gW, gb = torch.empty_like(Wd), torch.empty_like(bd)
    ll = torch.empty(C, dtype=torch.float64, device=dev)
    ctx = nat.context(0)
    ctx.check(ctx.lib.hmcx_logistic_grad(ctx.h, nat.HMCX_F64, nat.ptr(Xd), nat.ptr(yd), 90, 12, C, nat.ptr(Wd),
                                         nat.ptr(bd), 0.25, nat.ptr(gW), nat.ptr(gb)), "grad")
    ctx.check(ctx.lib.hmcx_logistic_loglik(ctx.h, nat.HMCX_F64, nat.ptr(Xd), nat.ptr(yd), 90, 12, C, nat.ptr(Wd),
                                           nat.ptr(bd), nat.ptr(ll)), "loglik")
    m = om.logistic({"alpha": 0.25})
    for c in range(C):
        par = {"weights": Ws[c], "bias": bs[c]}
        r = m.grad(par, X_train=X, y_train=y)
        np.testing.assert_allclose(gW.cpu().numpy()[:, c], r["weights"][:, 0], rtol=1e-10, atol=1e-11)
        np.testing.assert_allclose(gb.cpu().numpy()[c], r["bias"][0], rtol=1e-10, atol=1e-11)
        assert abs(ll[c].item() - m.log_likelihood(par, X_train=X, y_train=y)) < 1e-10 * abs(ll[c].item())


def _gpu_model(c, dtype=torch.float64):
    if c["model"] == "logistic":
        return _logistic(dtype, c["alpha"])
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.models.gpu.softmax import softmax
    return softmax({"alpha": c["alpha"]}, dtype=dtype, device="cuda:0")


def _fit(c, impl, **kw):
    X, Y, start = gi.sgd_problem(c)
    np.random.seed(c["np_seed"])
    fit = impl.fit_dropout if c["dropout"] else impl.fit
    extra = dict(p=c["p"]) if c["dropout"] else {}
    return fit(epochs=c["epochs"], batch_size=c["B"], gamma=c["gamma"], X_train=X, y_train=Y, **extra, **kw)


@pytest.mark.parametrize("name", sorted(gi.SGD_CONFIGS))
def test_sgd_f64_vs_oracle_and_golden(golden_dir, name):
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu.sgd import sgd
    c = gi.SGD_CONFIGS[name]
    _, _, start = gi.sgd_problem(c)
    ref_model = om.logistic({"alpha": c["alpha"]}) if c["model"] == "logistic" else om.softmax({"alpha": c["alpha"]})
    par_r, loss_r = _fit(c, osm.sgd(ref_model, start, step_size=c["step_size"]))
    g = sgd(_gpu_model(c), start, step_size=c["step_size"])
    par_g, loss_g = _fit(c, g)
    d = np.load(os.path.join(golden_dir, "sgd_%s.npz" % name))
    for v in ("weights", "bias"):
        np.testing.assert_allclose(par_g[v], par_r[v], rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(par_g[v], d[v], rtol=1e-9, atol=1e-12)
        assert par_g[v].shape == np.shape(start[v])
    np.testing.assert_allclose(loss_g, loss_r, rtol=1e-10)
    np.testing.assert_allclose(loss_g, d["loss"], rtol=1e-10)


def test_sgd_f32_close():
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu.sgd import sgd
    c = gi.SGD_CONFIGS["fit_softmax"]
    _, _, start = gi.sgd_problem(c)
    par_r, loss_r = _fit(c, osm.sgd(om.softmax({"alpha": c["alpha"]}), start, step_size=c["step_size"]))
    par_g, loss_g = _fit(c, sgd(_gpu_model(c, torch.float32), start, step_size=c["step_size"]))
    assert np.abs(par_g["weights"] - par_r["weights"]).max() <= 1e-4 * (np.abs(par_r["weights"]).max() + 1e-3)
    np.testing.assert_allclose(loss_g, loss_r, rtol=1e-4)


def test_sgd_dropout_philox_deterministic():
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu.sgd import sgd
    c = dict(gi.SGD_CONFIGS["drop_softmax"])
    _, _, start = gi.sgd_problem(c)
    runs = [_fit(c, sgd(_gpu_model(c), start, step_size=c["step_size"], noise="philox", seed=s)) for s in (3, 3, 4)]
    np.testing.assert_array_equal(runs[0][0]["weights"], runs[1][0]["weights"])
    assert not np.array_equal(runs[0][0]["weights"], runs[2][0]["weights"])
    assert np.all(np.isfinite(runs[0][1]))


def test_hmc_logistic_vs_oracle():
    """Full-batch HMC on the logistic model (benchmarks/1.-Simulated_data.ipynb's use): device
    gradients through hmc's generic loop; accept flags bit-exact, positions within rel 1e-9."""
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu.hmc import hmc
    X, y, _, _ = gi.logistic_inputs(11, 120, 2)
    start = {"weights": np.full((2, 1), 0.3), "bias": np.array([0.1])}
    kw = dict(path_length=0.05, step_size=0.01, verbose=True)
    o = osm.hmc(om.logistic({"alpha": 0.25}), start, **kw)
    o.trace, o.out = [], io.StringIO()
    np.random.seed(1)
    post_r, loss_r, _, _ = o.sample(12, 3, np.random.RandomState(2), X_train=X, y_train=y)
    h = hmc(_logistic(), start, **kw)
    h.trace, h.out = [], io.StringIO()
    np.random.seed(1)
    post_g, loss_g, _, _ = h.sample(12, 3, np.random.RandomState(2), X_train=X, y_train=y)
    assert [t["accepted"] for t in h.trace] == [t["accepted"] for t in o.trace]
    for v in ("weights", "bias"):
        np.testing.assert_allclose(np.asarray(post_g[v]).reshape(12, -1), np.asarray(post_r[v]).reshape(12, -1),
                                   rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(loss_g, loss_r, rtol=1e-10)
