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


def logistic_inputs(seed, B, D, wscale=0.5):
    """Two Gaussian clusters like benchmarks/1.-Simulated_data.ipynb (make_blobs, D=2 there):
    X = N(±1.5, 1)^{B×D} by label, y ∈ {0,1} (float), W~N(0,wscale²)[D,1], b~N(0,wscale²)[1]."""
    rs = np.random.RandomState(seed)
    y = rs.randint(0, 2, B).astype(np.float64)
    X = rs.normal(0, 1, (B, D)) + 1.5 * (2 * y[:, None] - 1)
    W = rs.normal(0, wscale, (D, 1))
    b = rs.normal(0, wscale, 1)
    return X, y, W, b


LOGISTIC_CASES = [(0, 50, 2, 0.5), (1, 500, 784, 0.05), (2, 1, 3, 0.5), (3, 77, 33, 2.0), (4, 64, 16, 40.0)]

# sgd.fit / fit_dropout runs (sgd.py:25-70): (name, model, N, B, D, K, alpha, eta, gamma, epochs, p, seeds)
SGD_CONFIGS = {
    'fit_logistic':  dict(model='logistic', N=750, B=50, D=2, K=1, alpha=0.25, step_size=1e-3, gamma=0.9,
                          epochs=4, data_seed=40, start_seed=41, dropout=False, p=0.5, np_seed=0),
    'fit_softmax':   dict(model='softmax', N=600, B=100, D=64, K=10, alpha=0.01, step_size=1e-4, gamma=0.9,
                          epochs=3, data_seed=42, start_seed=43, dropout=False, p=0.5, np_seed=0),
    'drop_softmax':  dict(model='softmax', N=400, B=100, D=32, K=10, alpha=0.01, step_size=1e-4, gamma=0.9,
                          epochs=2, data_seed=44, start_seed=45, dropout=True, p=0.8, np_seed=5),
    'drop_logistic': dict(model='logistic', N=300, B=50, D=8, K=1, alpha=0.25, step_size=1e-3, gamma=0.5,
                          epochs=2, data_seed=46, start_seed=47, dropout=True, p=0.5, np_seed=6),
}


# benchmarks/1.-Simulated_data.ipynb, cells 2, 6 and 10 (the reference's one live harness): blobs data,
# logistic sgd.fit and hmc.sample through the hamiltonian.models.cpu / inference.cpu import paths.
# Reduced so the reference finishes in seconds: sgd 200 epochs (notebook 1e4); hmc path_length 2e-3,
# step 1e-4, 40 samples after 10 burn-in (notebook: path 1, step 1e-5 — ≈10⁵ leapfrogs per step).
NOTEBOOK = dict(centers=[[-5, 0], [5, -1]], n_samples=1000, cluster_std=1, random_state=40, split_state=0,
                sgd=dict(epochs=200, batch_size=50, eta=1e-5, gamma=0.9, alpha=0.25, start_seed=3),
                hmc=dict(path_length=2e-3, step_size=1e-4, niter=40, burnin=10, np_seed=4, rng_seed=5))


def notebook_data():
    """Cell 2: make_blobs → standardise → train_test_split (needs scikit-learn)."""
    from sklearn.datasets import make_blobs
    from sklearn.model_selection import train_test_split
    c = NOTEBOOK
    X, y = make_blobs(n_samples=c['n_samples'], centers=c['centers'], cluster_std=c['cluster_std'],
                      random_state=c['random_state'])
    X = (X - X.mean(axis=0)) / X.std(axis=0)
    return train_test_split(X, y, random_state=c['split_state'])


def sgd_problem(c):
    """Dataset and start point of an SGD_CONFIGS entry."""
    if c['model'] == 'logistic':
        X, y, _, _ = logistic_inputs(c['data_seed'], c['N'], c['D'])
        rs = np.random.RandomState(c['start_seed'])
        start = {'weights': 2 * rs.random_sample((c['D'], 1)), 'bias': 2 * rs.random_sample(1)}   # notebook :269
        return X, y, start
    X, Y = dataset(c['data_seed'], c['N'], c['D'], c['K'])
    rs = np.random.RandomState(c['start_seed'])
    start = {'weights': rs.normal(0, 0.01, (c['D'], c['K'])), 'bias': rs.normal(0, 0.01, c['K'])}
    return X, Y, start
