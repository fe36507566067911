"""ORACLE (test infrastructure only) — seeded synthetic inputs shared by the golden
generator (oracle/gen_golden.py, run in the build container against the reference)
and by tests/ (which regenerate the same inputs instead of storing large arrays).

All draws use the legacy ``np.random.RandomState`` stream, which NumPy keeps stable.
Label encoding follows utils.one_hot (/root/reference/hamiltonian/utils.py:4-8).
"""
import numpy as np


def one_hot(y, K):
    enc = np.zeros((len(y), K))
    enc[np.arange(len(y)), np.asarray(y, dtype=int)] = 1.0
    return enc


def softmax_inputs(seed, B, D=784, K=10, wscale=0.01):
    """X∈[0,1)^{B×D}, one-hot Y, W~N(0,wscale²)[D,K], b~N(0,wscale²)[K]."""
    rs = np.random.RandomState(seed)
    X = rs.rand(B, D)
    labels = rs.randint(0, K, B)
    W = rs.normal(0, wscale, (D, K))
    b = rs.normal(0, wscale, K)
    return X, one_hot(labels, K), W, b


def dataset(seed, N, D, K):
    """MNIST-shaped synthetic dataset: X=rand(N,D), Y=one_hot(randint)."""
    X = np.random.RandomState(seed).rand(N, D)
    Y = one_hot(np.random.RandomState(seed + 1).randint(0, K, N), K)
    return X, Y


# Golden trajectory configurations (kept small so fixtures stay ≤ ~200 KB).
TRAJ_CONFIGS = {
    'sgld_small':   dict(kind='sgld', N=200, B=50, D=64, K=10, alpha=0.01, step_size=1e-3,
                         path_length=1.0, burnin=1, epochs=3, data_seed=100, np_seed=0, rng_seed=1),
    'sghmc_small':  dict(kind='sghmc', N=200, B=50, D=64, K=10, alpha=0.01, step_size=1e-3,
                         path_length=1e-2, burnin=1, epochs=3, data_seed=100, np_seed=0, rng_seed=1),
    'sghmc_mnist':  dict(kind='sghmc', N=1000, B=500, D=784, K=10, alpha=0.01, step_size=1e-3,
                         path_length=1e-2, burnin=1, epochs=2, data_seed=7, np_seed=3, rng_seed=4),
    'sghmc_hot':    dict(kind='sghmc', N=120, B=40, D=32, K=10, alpha=0.01, step_size=5e-2,
                         path_length=0.25, burnin=1, epochs=2, data_seed=11, np_seed=5, rng_seed=6),
    'sgld_mnist':   dict(kind='sgld', N=1000, B=500, D=784, K=10, alpha=0.01, step_size=1e-4,
                         path_length=1.0, burnin=1, epochs=2, data_seed=7, np_seed=3, rng_seed=4),
}

MVN_CONFIG = dict(mu=[0.0, 0.0], cov=[[1.0, 0.8], [0.8, 1.0]], step_size=0.1, path_length=1.0,
                  niter=2000, burnin=100, np_seed=0, rng_seed=1)

HMC_SOFTMAX_CONFIG = dict(N=50, D=16, K=10, alpha=0.01, step_size=1e-2, path_length=0.05,
                          niter=6, burnin=2, data_seed=21, np_seed=2, rng_seed=3)

GRAD_CASES = [(seed, B, ws) for seed in (0, 1, 2) for B in (32, 500) for ws in (0.01,)] + \
             [(3, 64, 5.0), (4, 64, 50.0), (5, 1, 0.01)]
