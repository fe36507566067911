"""Pin the logistic-model and momentum-SGD restatements (oracle/models.py::logistic,
oracle/samplers.py::sgd) bit for bit against the fixtures oracle/gen_golden.py --logistic produced
by running the reference itself (models/cpu/logistic.py, inference/cpu/sgd.py)."""
import os

import numpy as np
import pytest

from oracle import inputs as gi
from oracle import models as om
from oracle import samplers as osm

threadpoolctl = pytest.importorskip("threadpoolctl")


@pytest.fixture(autouse=True)
def _one_blas_thread():
    with threadpoolctl.threadpool_limits(limits=1, user_api="blas"):
        yield


@pytest.mark.parametrize("i", range(len(gi.LOGISTIC_CASES)))
def test_logistic_bitexact(golden_dir, i):
    d = np.load(os.path.join(golden_dir, "logistic.npz"))
    seed, B, D, ws = gi.LOGISTIC_CASES[i]
    X, y, W, b = gi.logistic_inputs(seed, B, D, wscale=ws)
    m = om.logistic({"alpha": 0.25})
    par = {"weights": W, "bias": b}
    g = m.grad(par, X_train=X, y_train=y)
    np.testing.assert_array_equal(g["weights"], d["c%d_gW" % i])
    np.testing.assert_array_equal(g["bias"], d["c%d_gb" % i])
    np.testing.assert_array_equal(m.net(par, X_train=X), d["c%d_net" % i])
    sc = np.array([m.log_likelihood(par, X_train=X, y_train=y), m.negative_log_posterior(par, X_train=X, y_train=y),
                   m.log_prior(par)])
    np.testing.assert_array_equal(sc, d["c%d_scalars" % i])
    bs = max(1, B // 3)
    np.testing.assert_array_equal(m.predict(par, X, prob=False, batchsize=bs), d["c%d_pred" % i])
    np.testing.assert_array_equal(m.predict(par, X, prob=True, batchsize=bs), d["c%d_predp" % i])


def test_logistic_grad_finite_difference():
    """grad = ∇(−ll − log_prior) (the reference's sign convention, logistic.py:37-40)."""
    X, y, W, b = gi.logistic_inputs(7, 30, 4)
    m = om.logistic({"alpha": 0.3})
    par = {"weights": W, "bias": b}
    g = m.grad(par, X_train=X, y_train=y)
    f = lambda p: -(m.log_likelihood(p, X_train=X, y_train=y) + m.log_prior(p))
    h = 1e-6
    for var, idx in (("weights", (2, 0)), ("bias", (0,))):
        pp = {k: v.copy() for k, v in par.items()}
        pm = {k: v.copy() for k, v in par.items()}
        pp[var][idx] += h
        pm[var][idx] -= h
        assert abs((f(pp) - f(pm)) / (2 * h) - g[var][idx]) < 1e-5 * max(1.0, abs(g[var][idx]))


@pytest.mark.parametrize("name", sorted(gi.SGD_CONFIGS))
def test_sgd_bitexact(golden_dir, name):
    c = gi.SGD_CONFIGS[name]
    d = np.load(os.path.join(golden_dir, "sgd_%s.npz" % name))
    X, Y, start = gi.sgd_problem(c)
    model = om.logistic({"alpha": c["alpha"]}) if c["model"] == "logistic" else om.softmax({"alpha": c["alpha"]})
    opt = osm.sgd(model, start, step_size=c["step_size"])
    np.random.seed(c["np_seed"])
    if c["dropout"]:
        par, loss = opt.fit_dropout(epochs=c["epochs"], batch_size=c["B"], gamma=c["gamma"], p=c["p"],
                                    X_train=X, y_train=Y)
    else:
        par, loss = opt.fit(epochs=c["epochs"], batch_size=c["B"], gamma=c["gamma"], X_train=X, y_train=Y)
    np.testing.assert_array_equal(par["weights"], d["weights"])
    np.testing.assert_array_equal(par["bias"], d["bias"])
    np.testing.assert_array_equal(loss, d["loss"])
