"""A NaN energy difference is accepted on every SGHMC kernel.

The reference's accept is ``min(1, np.exp(E_cur − E_new))`` (cpu/hmc.py:67-71, used by the A1
completion of cpu/sghmc.py:36): Python's ``min(1, nan)`` returns 1, so a NaN proposal is ALWAYS
accepted and the chain carries NaN from then on.  A single NaN weight in start_p makes every logit,
gradient and energy NaN (the logit clip of softmax.py:39-41 keeps NaN).  Each kernel must then
report A = 1, accept every step, keep the oracle's path lengths, and end in the same NaN pattern:
the persistent single-chain kernel (hmcx_persist2.hip), the kernel-per-phase path (hmcx_softmax.hip)
and the chain-batched GEMMs (hmcx_batch.h, C = 16 replica chains)."""
import io

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from oracle import inputs as gi  # noqa: E402
from oracle import models as om  # noqa: E402
from oracle import samplers as osm  # noqa: E402


def _start(c):
    W = np.zeros((c["D"], c["K"]))
    W[3, 2] = np.nan
    return {"weights": W, "bias": np.zeros(c["K"])}


def _oracle(c):
    X, Y = gi.dataset(c["data_seed"], c["N"], c["D"], c["K"])
    s = osm.sghmc(om.softmax({"alpha": c["alpha"]}), _start(c), path_length=c["path_length"],
                  step_size=c["step_size"], verbose=True)
    s.trace = []
    s.out = io.StringIO()
    np.random.seed(c["np_seed"])
    with np.errstate(all="ignore"):
        post, logp = s.sample(epochs=c["epochs"], burnin=c["burnin"], batch_size=c["B"],
                              rng=np.random.RandomState(c["rng_seed"]), X_train=X, y_train=Y)
    return post, logp, s.trace


def _gpu(c, path, chains=1):
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.models.gpu.softmax import softmax
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu.sghmc import sghmc
    X, Y = gi.dataset(c["data_seed"], c["N"], c["D"], c["K"])
    m = softmax({"alpha": c["alpha"]}, dtype=torch.float64, device="cuda:0")
    m.ctx.set_sghmc_path(path)
    try:
        s = sghmc(m, _start(c), path_length=c["path_length"], step_size=c["step_size"], verbose=True,
                  noise="numpy", chains=chains)
        s.trace = []
        s.out = io.StringIO()
        np.random.seed(c["np_seed"])
        post, logp = s.sample(epochs=c["epochs"], burnin=c["burnin"], batch_size=c["B"],
                              rng=np.random.RandomState(c["rng_seed"]), X_train=X, y_train=Y)
    finally:
        m.ctx.set_sghmc_path(0)
    return post, logp, s.trace


@pytest.mark.parametrize("name,path,chains", [("sghmc_small", 1, 1), ("sghmc_small", 2, 1),
                                              ("sghmc_mnist", 2, 1), ("sghmc_small", 0, 16)])
def test_nan_energy_accepted(name, path, chains):
    c = gi.TRAJ_CONFIGS[name]
    post_r, logp_r, tr_r = _oracle(c)
    assert all(t["accepted"] for t in tr_r) and all(t["A"] == 1 for t in tr_r)    # the quirk itself
    post_g, logp_g, tr_g = _gpu(c, path, chains)
    for tg, tr in zip(tr_g, tr_r):
        assert np.all(np.asarray(tg["L"]) == tr["L"])
    assert len(tr_g) == len(tr_r)
    for t in tr_g:
        assert np.all(np.asarray(t["accepted"])) and np.all(np.asarray(t["A"]) == 1.0)
    for v in ("weights", "bias"):
        g = post_g[v] if chains == 1 else post_g[v][chains - 1]
        np.testing.assert_array_equal(np.isnan(g), np.isnan(post_r[v]))
        np.testing.assert_allclose(g, post_r[v], rtol=1e-9, atol=1e-12, equal_nan=True)
    assert np.all(np.isnan(logp_g)) and np.all(np.isnan(logp_r))
