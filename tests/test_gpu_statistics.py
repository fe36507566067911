"""Statistical parity of the device-noise (noise='philox') chains — the mode bench.py measures —
against the NumPy reference chains (oracle/samplers.py, bit-exact restatement of cpu/sghmc.py:19-39
with the A1 completion and cpu/sgld.py:31-46).

The Philox chains cannot match the reference draw for draw (the reference's NumPy streams are
replayed only in noise='numpy' mode, tests/test_gpu_samplers.py), so they are compared in law: 64
independent GPU chains against 64 independent oracle chains from the same start on the same
minibatch sequence, per parameter, on

* the ensemble's state after the last step (independent draws; SE = sd/√C), and
* the running posterior over the second half of the chains (MCSE = sd/√ESS, ESS from
  dropout_hamiltonian_montecarlo_amd.diagnostics.ess),

for both the mean and the variance.  Tolerance: 3·MCSE per parameter,
applied as "≤ 1 % of the parameters beyond 3 combined standard errors and none beyond 6" (the
chance rate of a 3σ excursion is 0.27 % per parameter; 6 bounds the largest of 77,862 t-distributed
statistics — oracle-vs-oracle ensembles reach 5.8).  The running-posterior MCSE needs ≥ 20 draws per
chain half-window: with 10, oracle-vs-oracle SGLD runs exceed 1 % (ESS overestimated), so the SGLD
test runs 40 steps.  tests/test_stats_cpu.py
shows the criterion passes for oracle-vs-oracle ensembles and fails for a chain whose momentum law
is off by 25 %.

Shapes: BASELINE config 2 (D=784, K=10, B=500, MNIST-shaped synthetic data; SGHMC ε=1e-3,
λ=1e-2 as in bench.py) and config 5 (D=2048, K=38, B=500; SGLD ε=1e-4).  N = B, so every epoch is
one step and the posterior holds the state after every step.
"""
import io

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from oracle import ensemble, inputs as gi  # noqa: E402
import _stats  # noqa: E402

C = 64
SEED = 2024

CFG2 = dict(N=500, B=500, D=784, K=10, alpha=0.01, step_size=1e-3, path_length=1e-2, data_seed=7)
CFG5 = dict(N=500, B=500, D=2048, K=38, alpha=0.01, step_size=1e-4, path_length=1.0, data_seed=9)

_ORACLE = {}


def _oracle(kind, cfg, T):
    key = (kind, tuple(sorted(cfg.items())), T)
    if key not in _ORACLE:
        _ORACLE[key] = ensemble.run_chains(kind, cfg, range(C), T)
    return _ORACLE[key]


def _flat(post, lead):
    return np.concatenate([post["weights"].reshape(lead + (-1,)), post["bias"].reshape(lead + (-1,))], axis=-1)


def _gpu(kind, cfg, T, dtype=torch.float64, path=0, batched=False):
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.models.gpu.softmax import softmax
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu.sghmc import sghmc
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu.sgld import sgld
    X, Y = gi.dataset(cfg["data_seed"], cfg["N"], cfg["D"], cfg["K"])
    cls = sghmc if kind == "sghmc" else sgld
    m = softmax({"alpha": cfg["alpha"]}, dtype=dtype, device="cuda:0")
    if kind == "sghmc":
        m.ctx.set_sghmc_path(path)
    start = {"weights": np.zeros((cfg["D"], cfg["K"])), "bias": np.zeros(cfg["K"])}

    def run(chain, chains):
        s = cls(m, start, path_length=cfg["path_length"], step_size=cfg["step_size"], verbose=False,
                noise="philox", seed=SEED, chain=chain, chains=chains)
        s.out = io.StringIO()
        s.trace = []
        post, _ = s.sample(epochs=T, burnin=0, batch_size=cfg["B"], X_train=X, y_train=Y)
        acc = np.array([t.get("accepted", True) for t in s.trace])
        return post, acc

    try:
        if batched:
            post, acc = run(0, C)
            return _flat(post, (C, T)), np.asarray(acc, dtype=bool).T
        draws, accs = [], []
        for c in range(C):
            post, acc = run(c, 1)
            draws.append(_flat(post, (T,)))
            accs.append(acc)
        return np.stack(draws), np.stack(accs).astype(bool)
    finally:
        if kind == "sghmc":
            m.ctx.set_sghmc_path(0)                     # the context is shared by later tests


def _check(gpu, ora, acc_g=None, acc_o=None):
    z = _stats.compare(gpu, ora)
    print(_stats.summary(z))
    _stats.assert_same_moments(z)
    if acc_g is not None and acc_g.size:
        # accept rates (bookkeeping in law): two-proportion z within 4
        pg, po = acc_g.mean(), acc_o.mean()
        pp = 0.5 * (pg + po)
        se = np.sqrt(pp * (1 - pp) * (1.0 / acc_g.size + 1.0 / acc_o.size))
        assert abs(pg - po) <= 4 * se + 1e-12, (pg, po)


@pytest.mark.parametrize("dtype,path,batched", [(torch.float64, 2, False),
                                                (torch.float64, 0, True),
                                                (torch.float32, 2, False)],
                         ids=["f64-persistent", "f64-batched", "f32-persistent"])
def test_sghmc_philox_moments_config2(dtype, path, batched):
    """SGHMC at BASELINE config 2's shape: the persistent single-chain kernel (the bench path) and
    the chain-batched GEMM path, f64 (and the f32 persistent path) against the NumPy chains."""
    T = 40
    ora, acc_o = _oracle("sghmc", CFG2, T)
    gpu, acc_g = _gpu("sghmc", CFG2, T, dtype=dtype, path=path, batched=batched)
    assert gpu.shape == ora.shape
    _check(gpu, ora, acc_g, acc_o)


def test_sgld_philox_moments_config5():
    """SGLD at BASELINE config 5's shape (one chain per call on the wide three-kernel path)."""
    T = 40
    ora, _ = _oracle("sgld", CFG5, T)
    gpu, _ = _gpu("sgld", CFG5, T)
    assert gpu.shape == ora.shape
    _check(gpu, ora)


# ----------------------------------------------------------------------------- MLP (config 3)
CFG3 = dict(N=500, B=500, n_in=784, n_mid=256, n_out=10, alpha=0.01, step_size=1e-3, path_length=3e-3,
            data_seed=13, start_seed=1)
C3 = 64


def _mlp_oracle(T):
    # one float32 ensemble (Chainer's default dtype, the bench's) serves both device dtypes: float32
    # rounding moves a 40-step chain by ~1e-7 relative, far below the per-parameter MCSE
    key = ("mlp", T)
    if key not in _ORACLE:
        _ORACLE[key] = ensemble.run_mlp_chains(dict(CFG3, dtype="f32"), range(C3), T)
    return _ORACLE[key]


def _mlp_gpu(T, dtype):
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.models.gpu.mlp import mlp, MLP_PARAM_NAMES
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu.sghmc import sghmc
    X, y = ensemble.mlp_dataset(CFG3)
    tdt = torch.float32 if dtype == "f32" else torch.float64
    X = X.astype(np.float32 if dtype == "f32" else np.float64)
    m = mlp({"alpha": CFG3["alpha"]}, CFG3["n_in"], CFG3["n_mid"], CFG3["n_out"], dtype=tdt, device="cuda:0")
    start = m.init_params(CFG3["start_seed"])
    ref_start = ensemble.mlp_start(CFG3["n_in"], CFG3["n_mid"], CFG3["n_out"], CFG3["start_seed"])
    for k in MLP_PARAM_NAMES:                        # both ensembles start from the same state
        np.testing.assert_array_equal(start[k], ref_start[k])
    draws, accs, Ls = [], [], []
    for c in range(C3):
        s = sghmc(m, start, path_length=CFG3["path_length"], step_size=CFG3["step_size"], verbose=False,
                  noise="philox", seed=SEED, chain=c)
        s.out = io.StringIO()
        s.trace = []
        post, _ = s.sample(epochs=T, burnin=0, batch_size=CFG3["B"], X_train=X, y_train=y)
        draws.append(np.concatenate([np.asarray(post[k]).reshape(T, -1) for k in MLP_PARAM_NAMES], axis=1)
                     .astype(np.float32))
        accs.append([t["accepted"] for t in s.trace])
        Ls.append([t["L"] for t in s.trace])
    return np.stack(draws), np.asarray(accs, dtype=bool), np.asarray(Ls)


@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_sghmc_mlp_philox_moments_config3(dtype):
    """The config-3 bench line's chains (MLP 784-256-256-10, B = 500, device Philox noise AND device
    Philox dropout masks, hmcx_mlp_sghmc_run) against 64 NumPy chains of the restated reference
    (mlp.py:19-96 with Chainer's fresh train-mode masks on every forward, sghmc.py:19-39 with the A1
    completion), per parameter over all 269,322: mean and variance within 3·MCSE (the criterion of the
    softmax tests above), accept rates within 4 standard errors, and the path-length law (the host
    schedule's ceil(2u·λ/ε)) by its mean."""
    T = 40
    ora, acc_o, L_o = _mlp_oracle(T)
    gpu, acc_g, L_g = _mlp_gpu(T, dtype)
    assert gpu.shape == ora.shape == (C3, T, 269322)
    _check(gpu, ora, acc_g, acc_o)
    # path lengths: L = ceil(2u·λ/ε) with λ/ε = 3 → uniform on {1, …, 6}: mean 3.5, var 35/12
    for L in (L_g, L_o):
        assert set(np.unique(L)) <= set(range(1, 7))
        assert abs(L.mean() - 3.5) < 4 * np.sqrt(35 / 12 / L.size)
