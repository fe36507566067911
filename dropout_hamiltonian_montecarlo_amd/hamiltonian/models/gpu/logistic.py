"""HIP-backed logistic regression — drop-in for the reference's logistic model.

Reference: /root/reference/hamiltonian/models/cpu/logistic.py:10-87 (NumPy, the parity target;
models/gpu/logistic.py is its CuPy twin).  K = 1: ``weights`` [D, 1], ``bias`` [1], labels
y ∈ {0, 1} of shape [B] (or [B, 1]).  grad / log_likelihood / net run in libhmcx (the k_fwd /
k_grad MFMA kernels of the softmax model with the sigmoid link, hmcx_logistic_*); log_prior's
Σθ² is a device reduction (hmcx_sumsq).  Results of grad are torch tensors on the model's device.
"""
import numpy as np
import torch

from dropout_hamiltonian_montecarlo_amd._native import HmcxError, context, dtype_code, ptr

from .softmax import _batch, as_device



def _log0(x):
    """np.log without the divide-by-zero RuntimeWarning at α = 0 (−inf, as the reference computes it:
    its model files silence warnings, models/cpu/softmax.py:1-2)."""
    with np.errstate(divide="ignore"):
        return np.log(x)

class logistic:
    _hmcx_model = 'logistic'

    def __init__(self, _hyper, dtype=torch.float64, device=None):
        self.hyper = {var: np.asarray(_hyper[var]) for var in _hyper.keys()}     # logistic.py:12-13
        self.alpha = float(self.hyper['alpha'])
        self.dtype = dtype
        self.code = dtype_code(dtype)
        self.ctx = context(device)
        self.device = self.ctx.device

    # -------------------------------------------------------------- helpers
    def _dev(self, a):
        return as_device(a, self.dtype, self.device)

    def _par(self, par):
        W = self._dev(par['weights'])
        b = self._dev(par['bias']).reshape(-1)
        if W.dim() != 2 or W.shape[1] != 1 or b.numel() != 1:
            raise HmcxError("logistic: weights must be [D,1] and bias [1]")
        return W.contiguous(), b.contiguous()

    def _x(self, X):
        X = self._dev(X)
        if X.dim() != 2:
            raise HmcxError("logistic: X_train [B,D] expected")
        return X

    def _xy(self, args):
        X, y = _batch(args)
        X = self._x(X)
        y = self._dev(y).reshape(-1).contiguous()                           # y.reshape(-1,1) (:32)
        if y.shape[0] != X.shape[0]:
            raise HmcxError("logistic: y_train must hold one label per row of X_train")
        return X, y

    # -------------------------------------------------------------- model surface
    def log_prior(self, par, **args):                                     # logistic.py:15-21
        K = 0
        ctx = context(self.device)
        for var in par.keys():
            v = self._dev(par[var]).reshape(-1).contiguous()
            dim = v.numel()
            ss = torch.empty(1, dtype=torch.float64, device=self.device)
            ctx.check(ctx.lib.hmcx_sumsq(ctx.h, self.code, ptr(v), dim, ptr(ss)), "hmcx_sumsq")
            K += dim * 0.5 * _log0(self.hyper['alpha'] / (2 * np.pi))
            K -= 0.5 * self.hyper['alpha'] * ss.item()
        return K

    def grad(self, par, **args):                                          # logistic.py:24-41
        X, y = self._xy(args)
        W, b = self._par(par)
        B, D = X.shape
        if W.shape[0] != D:
            raise HmcxError("logistic.grad: shape mismatch")
        gW = torch.empty_like(W)
        gb = torch.empty_like(b)
        ctx = context(self.device)
        ctx.check(ctx.lib.hmcx_logistic_grad(ctx.h, self.code, ptr(X), ptr(y), B, D, 1, ptr(W), ptr(b),
                                             self.alpha, ptr(gW), ptr(gb)), "hmcx_logistic_grad")
        return {'weights': gW, 'bias': gb}

    def net(self, par, **args):                                           # logistic.py:43-51
        return self._net_device(par, **args)

    def _net_device(self, par, **args):
        X, _ = _batch(args)
        X = self._x(X)
        W, b = self._par(par)
        B, D = X.shape
        prob = torch.empty((B, 1), dtype=self.dtype, device=self.device)
        ctx = context(self.device)
        ctx.check(ctx.lib.hmcx_logistic_predict(ctx.h, self.code, ptr(X), B, D, 1, ptr(W), ptr(b), ptr(prob)),
                  "hmcx_logistic_predict")
        return prob

    def log_likelihood_device(self, par, **args):
        X, y = self._xy(args)
        W, b = self._par(par)
        B, D = X.shape
        ll = torch.empty(1, dtype=torch.float64, device=self.device)
        ctx = context(self.device)
        ctx.check(ctx.lib.hmcx_logistic_loglik(ctx.h, self.code, ptr(X), ptr(y), B, D, 1, ptr(W), ptr(b),
                                               ptr(ll)), "hmcx_logistic_loglik")
        return ll

    def log_likelihood(self, par, **args):                                # logistic.py:64-72
        return np.float64(self.log_likelihood_device(par, **args).item())

    def negative_log_posterior(self, par, **args):                        # logistic.py:57-62
        n_data = args['X_train'].shape[0]
        return (-1.0 / n_data) * (self.log_likelihood(par, **args) + self.log_prior(par, **args))

    def loss(self, par, **args):
        """North-star surface name: the sampler energy U = negative_log_posterior."""
        return self.negative_log_posterior(par, **args)

    def predict(self, par, X, prob=False, batchsize=32):                  # logistic.py:75-87
        """Whole batches only, as the reference (rows past the last full batch are dropped)."""
        n = (X.shape[0] // batchsize) * batchsize
        if n == 0:
            return np.asarray([]).flatten()
        yhat = self._net_device(par, X_train=X[:n]).cpu().numpy()
        if prob:
            return yhat.flatten()
        return (yhat > 0.5).astype(int).flatten()
