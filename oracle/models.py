"""ORACLE (test infrastructure only) — NumPy float64 restatement of the reference models.

softmax        ← /root/reference/hamiltonian/models/cpu/softmax.py
mvn_gaussian   ← /root/reference/hamiltonian/models/cpu/mvn_gaussian.py
logistic       ← /root/reference/hamiltonian/models/cpu/logistic.py
mlp            ← /root/reference/hamiltonian/models/gpu/mlp.py (Chainer; restated with
                 injected dropout masks — parity UNPINNED, cross-checked vs torch autograd)
one_hot        ← /root/reference/hamiltonian/utils.py:4-8

Arithmetic is written in the same NumPy op order as the reference so that the
golden vectors in tests/golden (produced by the reference itself) match bit for bit.
"""
import numpy as np
from scipy.special import logsumexp

# Clip bounds of softmax.py:40-41 (np.finfo(float) == float64).
CLIP_HI = -np.log(np.finfo(float).eps)                 # 36.04365338911715
CLIP_LO = -np.log(1. / np.finfo(float).tiny - 1.0)     # -708.3964185322641


def one_hot(y, num_classes):
    """utils.py:4-8 (``np.int`` → ``int``)."""
    encoding = np.zeros((len(y), num_classes))
    for i, val in enumerate(y):
        encoding[i, int(val)] = 1.0
    return encoding


def _batch(args):
    X = y = None
    for k, v in args.items():
        if k == 'X_train':
            X = v
        elif k == 'y_train':
            y = v
    return X, y


class softmax:
    """models/cpu/softmax.py:12-100 — softmax regression, float64."""

    def __init__(self, _hyper, prior='cpu'):
        self.hyper = _hyper                                              # :14-15
        self.prior = prior       # 'gpu': the CuPy file's log_prior (models/gpu/softmax.py:29-39)

    def cross_entropy(self, y_linear, y):                                # :17-20
        lse = logsumexp(y_linear, axis=1)
        y_hat = y_linear - np.repeat(lse[:, np.newaxis], y.shape[1]).reshape(y.shape)
        return np.sum(y * y_hat, axis=1)

    def log_prior(self, par, **args):                                    # :22-30 (constant in par)
        K = 0
        if self.prior == 'gpu':                                          # gpu/softmax.py:29-39
            for var in par.keys():
                dim = (np.asarray(par[var])).size
                K -= 0.5 * self.hyper['alpha'] * np.sum(np.square(par[var])) / dim
            return K
        for var in par.keys():
            dim = (np.array(par[var])).size
            K -= 0.5 * dim * np.log(2 * np.pi) - 0.5 * dim * np.log(self.hyper['alpha'])
        return K

    def softmax(self, y_linear):                                         # :32-36
        exp = np.exp(y_linear - np.max(y_linear, axis=1).reshape((-1, 1)))
        norms = np.sum(exp, axis=1).reshape((-1, 1))
        return exp / norms

    def logits(self, par, X):                                            # :39-41 (net before softmax)
        y_linear = np.dot(X, par['weights']) + par['bias']
        y_linear = np.minimum(y_linear, CLIP_HI)
        y_linear = np.maximum(y_linear, CLIP_LO)
        return y_linear

    def net(self, par, X):                                               # :38-43
        return self.softmax(self.logits(par, X))

    def grad(self, par, **args):                                         # :45-61
        X, y = _batch(args)
        yhat = self.net(par, X)
        diff = y - yhat
        grad_w = np.dot(X.T, diff)
        grad_b = np.sum(diff, axis=0)
        grad = {}
        grad['weights'] = grad_w - self.hyper['alpha'] * par['weights']
        grad['weights'] = -1.0 * grad['weights']
        grad['bias'] = grad_b - self.hyper['alpha'] * par['bias']
        grad['bias'] = -1.0 * grad['bias']
        return grad

    def log_likelihood(self, par, **args):                               # :63-72
        X, y = _batch(args)
        return np.sum(self.cross_entropy(self.logits(par, X), y))

    def negative_log_posterior(self, par, **args):                       # :74-79
        n_data = np.asarray(args['X_train']).shape[0]
        return (-1.0 / n_data) * (self.log_likelihood(par, **args) + self.log_prior(par, **args))

    # north-star surface name: loss ≡ the sampler energy U.
    def loss(self, par, **args):
        return self.negative_log_posterior(par, **args)

    def predict(self, par, X, prob=False):                               # :82-89
        yhat = self.net(par, X)
        return yhat if prob else yhat.argmax(axis=1)

    def predict_stochastic(self, par, X, prob=False, p=0.5, Z=None):     # :91-100 (mask injectable)
        if Z is None:
            Z = np.random.binomial(1, p, size=X.shape)
        yhat = self.net(par, np.multiply(X, Z))
        return yhat if prob else yhat.argmax(axis=1)


class logistic:
    """models/cpu/logistic.py:10-87 — logistic regression (K = 1, sigmoid link), float64."""

    def __init__(self, _hyper):
        self.hyper = {var: np.asarray(_hyper[var]) for var in _hyper.keys()}     # :12-13

    def log_prior(self, par, **args):                                    # :15-21
        K = 0
        for var in par.keys():
            dim = (np.asarray(par[var])).size
            K += dim * 0.5 * np.log(self.hyper['alpha'] / (2 * np.pi))
            K -= 0.5 * self.hyper['alpha'] * np.sum(np.square(par[var]))
        return K

    def grad(self, par, **args):                                         # :24-41
        X, y = _batch(args)
        X = np.asarray(X)
        y = np.asarray(y)
        yhat = self.net(par, **args)
        diff = y.reshape(-1, 1) - yhat
        grad_w = np.dot(X.T, diff)
        grad_b = np.sum(diff, axis=0)
        grad = {}
        grad['weights'] = grad_w - self.hyper['alpha'] * par['weights']
        grad['weights'] = -1.0 * grad['weights']
        grad['bias'] = grad_b - self.hyper['alpha'] * par['bias']
        grad['bias'] = -1.0 * grad['bias']
        return grad

    def net(self, par, **args):                                          # :43-51
        X, _ = _batch(args)
        y_linear = np.dot(np.asarray(X), par['weights']) + par['bias']
        y_linear = np.minimum(y_linear, CLIP_HI)
        y_linear = np.maximum(y_linear, CLIP_LO)
        return self.sigmoid(y_linear)

    def sigmoid(self, y_linear):                                         # :53-55
        norms = (1.0 + np.exp(-y_linear))
        return 1.0 / norms

    def negative_log_posterior(self, par, **args):                       # :57-62
        n_data = np.asarray(args['X_train']).shape[0]
        return (-1.0 / n_data) * (self.log_likelihood(par, **args) + self.log_prior(par, **args))

    def log_likelihood(self, par, **args):                               # :64-72
        X, y = _batch(args)
        y = np.asarray(y)
        y_pred = np.squeeze(self.net(par, **args), axis=1)
        return np.sum(np.multiply(y, np.log(y_pred)) + np.multiply((1.0 - y), np.log(1.0 - y_pred)))

    def loss(self, par, **args):
        return self.negative_log_posterior(par, **args)

    def predict(self, par, X, prob=False, batchsize=32):                 # :75-87
        results = []
        for start_idx in range(0, X.shape[0] - batchsize + 1, batchsize):
            yhat = self.net(par, X_train=X[start_idx:start_idx + batchsize])
            results.append(yhat if prob else (yhat > 0.5).astype(int).flatten())
        return np.asarray(results).flatten()


class mvn_gaussian:
    """models/cpu/mvn_gaussian.py:9-31."""

    def __init__(self, _hyper):
        self.hyper = _hyper

    def grad(self, par, **args):                                         # :14-20
        cov = self.hyper['cov']
        mu = self.hyper['mu']
        x = par['x']
        return {'x': np.dot(x - mu, np.linalg.inv(cov))}

    def negative_log_posterior(self, par, **args):                       # :22-31
        dim = self.hyper['mu'].shape[0]
        sigma = self.hyper['cov']
        mu = self.hyper['mu']
        x = par['x']
        log_loss = dim * np.log(2 * np.pi)
        log_loss += np.log(np.linalg.det(sigma))
        log_loss += np.dot(np.dot((x - mu).T, np.linalg.inv(sigma)), x - mu)
        log_loss *= 0.5
        return log_loss

    def loss(self, par, **args):
        return self.negative_log_posterior(par, **args)


# ---------------------------------------------------------------------------
# MLP — models/gpu/mlp.py:19-96 restated without Chainer.
# Parameter names follow Chainer's sorted ``namedparams`` order (mlp.py:54,62):
MLP_PARAM_NAMES = ('/l1/W', '/l1/b', '/l2/W', '/l2/b', '/l3/W', '/l3/b')
DROPOUT_RATIO = 0.1                                                      # mlp.py:29-31


def mlp_param_shapes(n_in, n_mid, n_out):
    """L.Linear stores W as [out, in] (mlp.py:24-26)."""
    return {'/l1/W': (n_mid, n_in), '/l1/b': (n_mid,),
            '/l2/W': (n_mid, n_mid), '/l2/b': (n_mid,),
            '/l3/W': (n_out, n_mid), '/l3/b': (n_out,)}


def dropout_masks(rng, B, n_mid, dtype=np.float32, ratio=DROPOUT_RATIO):
    """Chainer F.dropout train-mode mask: ``scale * (rand >= ratio)``, scale = 1/(1-ratio).

    Three masks per forward (mlp.py:29,30,31), all of shape [B, n_mid].
    """
    scale = dtype(1. / (1 - ratio))
    return [scale * (rng.rand(B, n_mid) >= ratio).astype(dtype) for _ in range(3)]


class mlp:
    """mlp.py:33-96 with explicit masks ``masks=[m1,m2,m3]`` (None → no dropout)."""

    def __init__(self, _hyper, n_in, n_mid_units, n_out):
        self.hyper = _hyper
        self.n_in, self.n_mid, self.n_out = n_in, n_mid_units, n_out

    def _forward(self, par, X, masks):                                   # mlp.py:28-31
        m1, m2, m3 = masks if masks is not None else (1, 1, 1)
        a1 = X.dot(par['/l1/W'].T) + par['/l1/b']
        h1 = np.maximum(a1 * m1, 0)
        a2 = h1.dot(par['/l2/W'].T) + par['/l2/b']
        h2 = np.maximum(a2 * m2, 0)
        d3 = h2 * m3
        z = d3.dot(par['/l3/W'].T) + par['/l3/b']
        return z, (a1, h1, a2, h2, d3)

    @staticmethod
    def _ce(z, t):                                                       # F.softmax_cross_entropy, mean
        zm = z - z.max(axis=1, keepdims=True)
        logp = zm - np.log(np.exp(zm).sum(axis=1, keepdims=True))
        return -logp[np.arange(z.shape[0]), t].mean(), logp

    def log_prior(self, par, **args):                                    # mlp.py:40-45
        K = 0
        for var in par.keys():
            dim = np.asarray(par[var]).size
            K -= 0.5 * self.hyper['alpha'] * np.sum(np.square(par[var])) / dim
        return K

    def grad(self, par, masks=None, **args):                             # mlp.py:47-64
        X, y = _batch(args)
        t = np.asarray(y).astype(int)
        z, (a1, h1, a2, h2, d3) = self._forward(par, X, masks)
        m1, m2, m3 = masks if masks is not None else (1, 1, 1)
        _, logp = self._ce(z, t)
        B = z.shape[0]
        gz = np.exp(logp)
        gz[np.arange(B), t] -= 1
        gz = (gz / B).astype(z.dtype)
        g = {}
        g['/l3/W'] = gz.T.dot(d3)
        g['/l3/b'] = gz.sum(axis=0)
        gh2 = gz.dot(par['/l3/W']) * m3
        ga2 = gh2 * (a2 * m2 > 0) * m2
        g['/l2/W'] = ga2.T.dot(h1)
        g['/l2/b'] = ga2.sum(axis=0)
        gh1 = ga2.dot(par['/l2/W'])
        ga1 = gh1 * (a1 * m1 > 0) * m1
        g['/l1/W'] = ga1.T.dot(X)
        g['/l1/b'] = ga1.sum(axis=0)
        return {k: g[k] + 0.5 * self.hyper['alpha'] * par[k] for k in MLP_PARAM_NAMES}

    def log_likelihood(self, par, masks=None, **args):                   # mlp.py:66-78 (returns the loss)
        X, y = _batch(args)
        z, _ = self._forward(par, X, masks)
        return self._ce(z, np.asarray(y).astype(int))[0]

    def negative_log_posterior(self, par, masks=None, **args):           # mlp.py:80-82
        return self.log_likelihood(par, masks=masks, **args) + self.log_prior(par, **args)

    def loss(self, par, masks=None, **args):
        return self.negative_log_posterior(par, masks=masks, **args)

    def predict(self, par, X_test, prob=False, masks=None):             # mlp.py:84-96
        z, _ = self._forward(par, X_test, masks)
        if prob:
            e = np.exp(z - z.max(axis=1, keepdims=True))
            return e / e.sum(axis=1, keepdims=True)
        return z.argmax(axis=1)
