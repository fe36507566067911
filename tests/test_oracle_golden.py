"""Pin the oracle: the NumPy restatement (oracle/) must reproduce, bit for bit, the
golden vectors that oracle/gen_golden.py produced by running the reference itself."""
import hashlib
import io
import json
import os

import numpy as np
import pytest

from oracle import inputs as gi
from oracle import models as om
from oracle import samplers as osm

threadpoolctl = pytest.importorskip("threadpoolctl")


@pytest.fixture(autouse=True)
def _one_blas_thread():
    """Golden vectors were produced with one BLAS thread; OpenBLAS's threaded dgemm
    partitions the reduction differently, so bit-exactness is defined at 1 thread."""
    with threadpoolctl.threadpool_limits(limits=1, user_api="blas"):
        yield


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(np.asarray(a, dtype=np.float64)).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def grad_golden(golden_dir):
    d = np.load(os.path.join(golden_dir, "softmax_grad.npz"))
    return d, json.loads(str(d["meta"]))


@pytest.mark.parametrize("i", range(len(gi.GRAD_CASES)))
def test_softmax_grad_bitexact(grad_golden, i):
    d, meta = grad_golden
    seed, B, ws = gi.GRAD_CASES[i]
    X, Y, W, b = gi.softmax_inputs(seed, B, wscale=ws)
    m = om.softmax({"alpha": 0.01})
    par = {"weights": W, "bias": b}
    g = m.grad(par, X_train=X, y_train=Y)
    assert _sha(g["weights"]) == meta["c%d" % i]["gW_sha"]
    assert _sha(g["bias"]) == meta["c%d" % i]["gb_sha"]
    np.testing.assert_array_equal(g["bias"], d["c%d_gb" % i])
    np.testing.assert_array_equal(g["weights"][:8], d["c%d_gW_slice" % i])
    sc = np.array([m.log_likelihood(par, X_train=X, y_train=Y),
                   m.negative_log_posterior(par, X_train=X, y_train=Y),
                   m.log_prior(par, X_train=X, y_train=Y)])
    np.testing.assert_array_equal(sc, d["c%d_scalars" % i])


def test_softmax_grad_closed_form():
    """grad == Xᵀ(Ŷ−Y)+αW, Σ(Ŷ−Y)+αb; finite-difference check on nlp·n."""
    X, Y, W, b = gi.softmax_inputs(9, 20, D=12, K=4)
    m = om.softmax({"alpha": 0.3})
    par = {"weights": W, "bias": b}
    g = m.grad(par, X_train=X, y_train=Y)
    Yh = m.net(par, X)
    np.testing.assert_allclose(g["weights"], X.T @ (Yh - Y) + 0.3 * W, rtol=1e-12, atol=1e-14)
    # grad is the gradient of -ll + (α/2)|θ|² (the Gaussian prior), checked by central differences
    f = lambda p: -m.log_likelihood(p, X_train=X, y_train=Y) + 0.15 * (np.sum(p["weights"] ** 2) + np.sum(p["bias"] ** 2))
    h = 1e-6
    for (var, idx) in [("weights", (3, 1)), ("weights", (0, 0)), ("bias", (2,))]:
        pp = {k: v.copy() for k, v in par.items()}
        pm = {k: v.copy() for k, v in par.items()}
        pp[var][idx] += h
        pm[var][idx] -= h
        fd = (f(pp) - f(pm)) / (2 * h)
        assert abs(fd - g[var][idx]) < 1e-6 * max(1, abs(fd))


@pytest.mark.parametrize("name", sorted(gi.TRAJ_CONFIGS))
def test_sgmcmc_trajectory_bitexact(golden_dir, name):
    c = gi.TRAJ_CONFIGS[name]
    d = np.load(os.path.join(golden_dir, "traj_%s.npz" % name))
    X, Y = gi.dataset(c["data_seed"], c["N"], c["D"], c["K"])
    model = om.softmax({"alpha": c["alpha"]})
    start = {"weights": np.zeros((c["D"], c["K"])), "bias": np.zeros(c["K"])}
    cls = osm.sghmc if c["kind"] == "sghmc" else osm.sgld
    s = cls(model, start, path_length=c["path_length"], step_size=c["step_size"], verbose=True)
    s.trace = []
    buf = io.StringIO()
    s.out = buf
    np.random.seed(c["np_seed"])
    post, logp = s.sample(epochs=c["epochs"], burnin=c["burnin"], batch_size=c["B"],
                          rng=np.random.RandomState(c["rng_seed"]), X_train=X, y_train=Y)
    np.testing.assert_array_equal(logp, d["logp"])
    for v in post:
        assert _sha(post[v]) == str(d["post_%s_sha" % v])
    tr = d["trace"]
    if c["kind"] == "sghmc":
        n_iter = np.array([max(0, t["L"] - 1) for t in s.trace])
        np.testing.assert_array_equal(n_iter, tr[:, 0])
        np.testing.assert_array_equal([t["A"] for t in s.trace], tr[:, 1])
        np.testing.assert_array_equal([t["accepted"] for t in s.trace], tr[:, 2])
        np.testing.assert_array_equal([t["eps"] for t in s.trace], tr[:, 3])
    # the reference's own log lines (printed -ll every 10 minibatches) match too
    ref_log = [l for l in str(d["log"]).splitlines() if "loss" in l]
    our_log = [l for l in buf.getvalue().splitlines() if "loss" in l]
    assert ref_log == our_log


def test_step_size_schedule_quirk():
    """ε0, ε0, ε0/(1+ε0)... within a sampling epoch (j resets per epoch)."""
    s = osm.sgld(om.softmax({"alpha": 1.0}), {"bias": np.zeros(1)}, step_size=0.1)
    nb = 4.0
    dec = 0.1 / nb
    got = [s.lr_schedule(0.1, j, dec, nb) for j in range(4)]
    np.testing.assert_allclose(got, [0.1, 0.1 / 1.1, 0.1 / 1.2, 0.1 / 1.3], rtol=1e-15)


def test_hmc_mvn_bitexact(golden_dir):
    c = gi.MVN_CONFIG
    d = np.load(os.path.join(golden_dir, "hmc_mvn.npz"))
    m = om.mvn_gaussian({"mu": np.array(c["mu"]), "cov": np.array(c["cov"])})
    h = osm.hmc(m, {"x": np.zeros(2)}, path_length=c["path_length"], step_size=c["step_size"], verbose=True)
    h.out = io.StringIO()
    h.trace = []
    np.random.seed(c["np_seed"])
    post, loss, pos, mom = h.sample(c["niter"], c["burnin"], np.random.RandomState(c["rng_seed"]))
    np.testing.assert_array_equal(post["x"], d["post_x"])
    np.testing.assert_array_equal(loss, d["loss"])
    np.testing.assert_array_equal([t["accepted"] for t in h.trace], d["trace"][:, 2])
    np.testing.assert_array_equal(np.array([p[0]["x"] for p in mom]), d["mom0"])
    # known answer (README hmc_mvn.png): correlation ≈ 0.8, unit marginals
    C = np.cov(post["x"].T)
    assert abs(C[0, 1] / np.sqrt(C[0, 0] * C[1, 1]) - 0.8) < 0.06


def test_hmc_softmax_bitexact(golden_dir):
    c = gi.HMC_SOFTMAX_CONFIG
    d = np.load(os.path.join(golden_dir, "hmc_softmax.npz"))
    X, Y = gi.dataset(c["data_seed"], c["N"], c["D"], c["K"])
    m = om.softmax({"alpha": c["alpha"]})
    h = osm.hmc(m, {"weights": np.zeros((c["D"], c["K"])), "bias": np.zeros(c["K"])},
                path_length=c["path_length"], step_size=c["step_size"], verbose=True)
    h.out = io.StringIO()
    h.trace = []
    np.random.seed(c["np_seed"])
    post, loss, _, _ = h.sample(c["niter"], c["burnin"], np.random.RandomState(c["rng_seed"]),
                                X_train=X, y_train=Y)
    np.testing.assert_array_equal(post["weights"], d["post_weights"])
    np.testing.assert_array_equal(post["bias"], d["post_bias"])
    np.testing.assert_array_equal(loss, d["loss"])
    np.testing.assert_array_equal([t["A"] for t in h.trace], d["trace"][:, 1])


def test_nan_energy_is_accepted():
    """Python min(1, nan) == 1, so a NaN energy difference is accepted."""
    assert min(1, np.exp(np.float64("nan"))) == 1
    assert min(1, np.exp(np.float64("inf"))) == 1


def test_mlp_restatement_vs_torch_autograd():
    """MLP oracle (parity UNPINNED: no runnable Chainer) cross-checked with torch CPU autograd."""
    torch = pytest.importorskip("torch")
    rs = np.random.RandomState(0)
    B, n_in, n_mid, n_out = 16, 20, 12, 5
    shapes = om.mlp_param_shapes(n_in, n_mid, n_out)
    par = {k: rs.normal(0, 0.3, s) for k, s in shapes.items()}
    X = rs.rand(B, n_in)
    y = rs.randint(0, n_out, B)
    masks = om.dropout_masks(rs, B, n_mid, dtype=np.float64)
    m = om.mlp({"alpha": 0.01}, n_in, n_mid, n_out)
    g = m.grad(par, masks=masks, X_train=X, y_train=y)
    tp = {k: torch.tensor(v, requires_grad=True) for k, v in par.items()}
    tX = torch.tensor(X)
    tm = [torch.tensor(mm) for mm in masks]
    h = torch.relu((tX @ tp["/l1/W"].T + tp["/l1/b"]) * tm[0])
    h = torch.relu((h @ tp["/l2/W"].T + tp["/l2/b"]) * tm[1])
    z = (h * tm[2]) @ tp["/l3/W"].T + tp["/l3/b"]
    loss = torch.nn.functional.cross_entropy(z, torch.tensor(y))
    loss.backward()
    for k in om.MLP_PARAM_NAMES:
        np.testing.assert_allclose(g[k], tp[k].grad.numpy() + 0.005 * par[k], rtol=1e-10, atol=1e-12)
    assert abs(m.log_likelihood(par, masks=masks, X_train=X, y_train=y) - loss.item()) < 1e-12
