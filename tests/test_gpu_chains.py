"""Several chains on one GPU (``chains=C``): the chain-batched GEMM path (C >= 16, K = 10,
hmcx_batch.h) and the kernel-per-phase path (C < 16) against the NumPy oracle.

Replica mode (noise='numpy' with C chains) drives every chain with the reference's own streams, so
every chain must reproduce the oracle's single-chain trajectory: bit-exact path lengths and accept
flags, float64 states within rel 1e-9.  Philox mode checks that chain c of a batched run equals
the single-chain run keyed by chain c."""
import io

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from oracle import inputs as gi  # noqa: E402

from test_gpu_samplers import _run_oracle  # noqa: E402


def _classes():
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.models.gpu.softmax import softmax
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu.sghmc import sghmc
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu.sgld import sgld
    return softmax, sghmc, sgld


def _run_chains(c, chains, dtype=torch.float64, noise="numpy", seed=0, chain=0, path=0):
    softmax, sghmc, sgld = _classes()
    X, Y = gi.dataset(c["data_seed"], c["N"], c["D"], c["K"])
    cls = sghmc if c["kind"] == "sghmc" else sgld
    m = softmax({"alpha": c["alpha"]}, dtype=dtype, device="cuda:0")
    m.ctx.set_sghmc_path(path)
    s = cls(m, {"weights": np.zeros((c["D"], c["K"])), "bias": np.zeros(c["K"])},
            path_length=c["path_length"], step_size=c["step_size"], verbose=True, noise=noise, seed=seed,
            chain=chain, chains=chains)
    s.trace = []
    s.out = io.StringIO()
    np.random.seed(c["np_seed"])
    post, logp = s.sample(epochs=c["epochs"], burnin=c["burnin"], batch_size=c["B"],
                          rng=np.random.RandomState(c["rng_seed"]), X_train=X, y_train=Y)
    return post, logp, s.trace


@pytest.mark.parametrize("name,chains", [("sghmc_small", 16), ("sghmc_small", 4), ("sghmc_mnist", 16), ("sghmc_small", 512),
                                         ("sghmc_mnist", 1024), ("sghmc_hot", 32), ("sgld_small", 16)])
def test_replica_chains_match_oracle(name, chains):
    # ("sghmc_mnist", 1024): D = 784 with 64 chain tiles runs the wide gradient kernel k_bgradw, whose
    # last feature tile is partial (16 of 64 features: empty m-tiles skipped, dispatched last)
    c = gi.TRAJ_CONFIGS[name]
    post_r, logp_r, tr_r, _ = _run_oracle(c)
    post_g, logp_g, tr_g = _run_chains(c, chains)
    assert post_g["weights"].shape == (chains, c["epochs"], c["D"], c["K"])
    assert logp_g.shape == (chains, c["epochs"])
    if c["kind"] == "sghmc":
        for t_g, t_r in zip(tr_g, tr_r):
            assert np.all(t_g["L"] == t_r["L"])
            assert np.all(t_g["accepted"] == t_r["accepted"])
            # both energies of the accept test (E_current at the step start, E_new at the proposal):
            # A and the accept flag alone do not pin them — A is capped at 1, or ~0 on hot chains
            np.testing.assert_allclose(np.broadcast_to(t_g["A"], (chains,)), t_r["A"], rtol=1e-9, atol=1e-12)
            np.testing.assert_allclose(t_g["E"], np.broadcast_to(t_r["E"], (chains, 2)), rtol=1e-10, atol=1e-9)
    for ch in range(chains):
        for v in ("weights", "bias"):
            np.testing.assert_allclose(post_g[v][ch], post_r[v], rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(logp_g[ch], logp_r, rtol=1e-10)


def test_replica_chains_tail_64row_kernel_match_oracle(monkeypatch):
    """HMCX_BTAIL32=0: the compaction-tail forwards run the 8-wave 64-row kernel instead of 32-row tiles
    (both write the 32-row partial layout) — same oracle parity at 1024 chains."""
    monkeypatch.setenv("HMCX_BTAIL32", "0")
    test_replica_chains_match_oracle("sghmc_mnist", 1024)


def test_batched_chains_equal_single_chain_runs():
    """Philox noise: chain c of a 16-chain batched run == the single-chain run with chain=c."""
    c = dict(gi.TRAJ_CONFIGS["sghmc_small"])
    post_b, logp_b, tr_b = _run_chains(c, 16, noise="philox", seed=11, chain=3)
    for ch in (0, 5, 15):
        post_1, logp_1, tr_1 = _run_chains(c, 1, noise="philox", seed=11, chain=3 + ch, path=1)
        assert [t["L"] for t in tr_1] == [float(t["L"][ch]) for t in tr_b]
        assert [t["accepted"] for t in tr_1] == [bool(t["accepted"][ch]) for t in tr_b]
        for v in ("weights", "bias"):
            np.testing.assert_allclose(post_b[v][ch], post_1[v], rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(logp_b[ch], logp_1, rtol=1e-10)


def test_batched_chains_mnist_philox_properties():
    """MNIST shape, 64 independent chains: finite, distinct chains, deterministic under a seed."""
    c = dict(gi.TRAJ_CONFIGS["sghmc_mnist"])
    p1, l1, t1 = _run_chains(c, 64, noise="philox", seed=5)
    p2, l2, t2 = _run_chains(c, 64, noise="philox", seed=5)
    assert np.all(np.isfinite(p1["weights"])) and np.all(np.isfinite(l1))
    np.testing.assert_array_equal(p1["weights"], p2["weights"])
    np.testing.assert_array_equal(l1, l2)
    assert np.std(p1["weights"][:, -1].reshape(64, -1), axis=0).max() > 0      # chains differ
    acc = np.mean([np.mean(t["accepted"]) for t in t1])
    assert 0.05 < acc <= 1.0


def test_batched_chains_f32_equal_single_chain_runs():
    """float32 chains draw the float32 Philox normals (the f64 chains draw the f64 stream, so the two
    dtypes no longer share noise; their laws are compared in tests/test_gpu_statistics.py): chain c of
    a 16-chain batched f32 run follows the single-chain f32 run keyed by chain c (log-likelihood
    within rel 1e-4; states within 1e-3 of their scale)."""
    c = dict(gi.TRAJ_CONFIGS["sghmc_small"])
    post_b, logp_b, tr_b = _run_chains(c, 16, dtype=torch.float32, noise="philox", seed=2)
    for ch in (0, 7, 15):
        post_1, logp_1, tr_1 = _run_chains(c, 1, dtype=torch.float32, noise="philox", seed=2, chain=ch, path=1)
        assert [t["L"] for t in tr_1] == [float(t["L"][ch]) for t in tr_b]
        np.testing.assert_allclose(logp_b[ch], logp_1, rtol=1e-4)
        scale = np.abs(post_1["weights"]).max() + 1e-3
        assert np.abs(post_b["weights"][ch] - post_1["weights"]).max() <= 1e-3 * scale


SGLD_WIDE = dict(kind="sgld", N=300, B=100, D=300, K=38, alpha=0.01, step_size=1e-4, path_length=1.0,
                 burnin=1, epochs=2, data_seed=61, np_seed=2, rng_seed=3)


@pytest.mark.parametrize("chains", [2, 5])
def test_wide_sgld_replica_chains_match_oracle(chains):
    """SGLD with several chains at a config-5-like class count (K = 38): the wide path
    (hmcx_wide.hip, a chain grid dimension in every kernel) in replica mode — every chain replays the
    reference's streams, so every chain must reproduce the oracle's single-chain trajectory (float64
    within rel 1e-9) and its printed log-likelihoods."""
    c = SGLD_WIDE
    post_r, logp_r, _, _ = _run_oracle(c)
    post_g, logp_g, _ = _run_chains(c, chains)
    assert post_g["weights"].shape == (chains, c["epochs"], c["D"], c["K"])
    for ch in range(chains):
        for v in ("weights", "bias"):
            np.testing.assert_allclose(post_g[v][ch], post_r[v], rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(logp_g[ch], logp_r, rtol=1e-10)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_wide_sgld_chains_equal_single_chain_runs(dtype):
    """Philox noise: chain c of a 4-chain wide SGLD run (D = 2048, K = 38: BASELINE config 5's shape)
    equals the single-chain run keyed by chain c (f64 rel 1e-9; f32 rel 1e-4 — summation order is the
    same, only the chain layout of W differs)."""
    c = dict(SGLD_WIDE, N=1000, B=500, D=2048, burnin=0, epochs=2)
    post_b, logp_b, _ = _run_chains(c, 4, dtype=dtype, noise="philox", seed=13, chain=6)
    tol = dict(rtol=1e-9, atol=1e-12) if dtype == torch.float64 else dict(rtol=1e-4, atol=1e-6)
    for ch in (0, 3):
        post_1, logp_1, _ = _run_chains(c, 1, dtype=dtype, noise="philox", seed=13, chain=6 + ch)
        for v in ("weights", "bias"):
            np.testing.assert_allclose(post_b[v][ch], post_1[v], **tol)
        np.testing.assert_allclose(logp_b[ch], logp_1, rtol=1e-9 if dtype == torch.float64 else 1e-4)
