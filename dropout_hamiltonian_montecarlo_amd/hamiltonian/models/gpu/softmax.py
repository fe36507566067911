"""HIP-backed softmax regression — drop-in for the reference's softmax model.

Reference: /root/reference/hamiltonian/models/cpu/softmax.py:12-100 (NumPy, the parity
target) and models/gpu/softmax.py:12-121 (CuPy; the slot this class fills).
Every compute call goes through libhmcx (k_fwd / k_grad MFMA kernels); arrays may be
NumPy or torch, results are torch tensors on the model's HIP device.

Semantics follow the CPU file (the NumPy oracle): ``log_prior`` is the constant of
softmax.py:22-30.  ``prior='gpu'`` selects the CuPy file's −½α·Σθ²/dim (gpu/softmax.py:29-39).
"""
import numpy as np
import torch

from dropout_hamiltonian_montecarlo_amd._native import HmcxError, context, dtype_code, ptr


def as_device(a, dtype, device):
    if isinstance(a, torch.Tensor):
        t = a.to(device=device, dtype=dtype)
    else:
        t = torch.as_tensor(np.asarray(a), dtype=dtype).to(device)
    return t.contiguous()


def _batch(args):
    X = y = None
    for k, v in args.items():
        if k == 'X_train':
            X = v
        elif k == 'y_train':
            y = v
    return X, y



def _log0(x):
    """np.log without the divide-by-zero RuntimeWarning at α = 0 (−inf, as the reference computes it:
    its model files silence warnings, models/cpu/softmax.py:1-2)."""
    with np.errstate(divide="ignore"):
        return np.log(x)

class softmax:
    _hmcx_model = 'softmax'

    def __init__(self, _hyper, dtype=torch.float64, device=None, prior='cpu'):
        self.hyper = _hyper
        self.alpha = float(np.asarray(_hyper['alpha']))
        self.dtype = dtype
        self.code = dtype_code(dtype)
        self.ctx = context(device)
        self.device = self.ctx.device
        if prior not in ('cpu', 'gpu'):
            raise ValueError("prior must be 'cpu' or 'gpu'")
        self.prior = prior

    # -------------------------------------------------------------- helpers
    def _dev(self, a):
        return as_device(a, self.dtype, self.device)

    def _par(self, par):
        W = self._dev(par['weights'])
        b = self._dev(par['bias'])
        if W.dim() != 2 or b.dim() != 1 or W.shape[1] != b.shape[0]:
            raise HmcxError("softmax: weights must be [D,K] and bias [K]")
        return W, b

    def _xy(self, args):
        X, y = _batch(args)
        X = self._dev(X)
        Y = self._dev(y)
        if X.dim() != 2 or Y.dim() != 2 or X.shape[0] != Y.shape[0]:
            raise HmcxError("softmax: X_train [B,D] and one-hot y_train [B,K] expected")
        return X, Y

    # -------------------------------------------------------------- model surface
    def grad(self, par, **args):                                          # softmax.py:45-61
        X, Y = self._xy(args)
        W, b = self._par(par)
        B, D = X.shape
        K = W.shape[1]
        if W.shape[0] != D or Y.shape[1] != K:
            raise HmcxError("softmax.grad: shape mismatch")
        gW = torch.empty_like(W)
        gb = torch.empty_like(b)
        ctx = context(self.device)
        ctx.check(ctx.lib.hmcx_softmax_grad(ctx.h, self.code, ptr(X), ptr(Y), B, D, K, 1, ptr(W), ptr(b),
                                            self.alpha, ptr(gW), ptr(gb)), "hmcx_softmax_grad")
        return {'weights': gW, 'bias': gb}

    def log_likelihood_device(self, par, **args):
        X, Y = self._xy(args)
        W, b = self._par(par)
        B, D = X.shape
        K = W.shape[1]
        ll = torch.empty(1, dtype=torch.float64, device=self.device)
        ctx = context(self.device)
        ctx.check(ctx.lib.hmcx_softmax_loglik(ctx.h, self.code, ptr(X), ptr(Y), B, D, K, 1, ptr(W), ptr(b),
                                              ptr(ll)), "hmcx_softmax_loglik")
        return ll

    def log_likelihood(self, par, **args):                                # softmax.py:63-72
        return np.float64(self.log_likelihood_device(par, **args).item())

    def log_prior(self, par, **args):                                     # softmax.py:22-30
        K = 0
        if self.prior == 'cpu':
            for var in par.keys():
                dim = int(np.prod(tuple(par[var].shape)))
                K -= 0.5 * dim * np.log(2 * np.pi) - 0.5 * dim * _log0(self.hyper['alpha'])
            return K
        ctx = context(self.device)
        for var in par.keys():                                            # gpu/softmax.py:29-39
            v = self._dev(par[var]).reshape(-1)
            ss = torch.empty(1, dtype=torch.float64, device=self.device)   # Σθ² on the device (hmcx_sumsq)
            ctx.check(ctx.lib.hmcx_sumsq(ctx.h, self.code, ptr(v), v.numel(), ptr(ss)), "hmcx_sumsq")
            K -= 0.5 * self.alpha * ss.item() / v.numel()
        return K

    def log_prior_const(self, shapes):
        """Constant CPU-semantics log prior for parameter shapes (used by the fused samplers)."""
        if self.prior != 'cpu':
            raise HmcxError("fused samplers implement the CPU (constant) log prior only")
        K = 0
        for shp in shapes:
            dim = int(np.prod(shp))
            K -= 0.5 * dim * np.log(2 * np.pi) - 0.5 * dim * _log0(self.hyper['alpha'])
        return K

    def negative_log_posterior(self, par, **args):                        # softmax.py:74-79
        n_data = args['X_train'].shape[0]
        return (-1.0 / n_data) * (self.log_likelihood(par, **args) + self.log_prior(par, **args))

    def loss(self, par, **args):
        """North-star surface name: the sampler energy U = negative_log_posterior."""
        return self.negative_log_posterior(par, **args)

    def net(self, par, X):                                                # softmax.py:38-43
        return self._net_device(par, X)

    def _net_device(self, par, X):
        X = self._dev(X)
        W, b = self._par(par)
        B, D = X.shape
        K = W.shape[1]
        prob = torch.empty((B, K), dtype=self.dtype, device=self.device)
        ctx = context(self.device)
        ctx.check(ctx.lib.hmcx_softmax_predict(ctx.h, self.code, ptr(X), B, D, K, 1, ptr(W), ptr(b), ptr(prob)),
                  "hmcx_softmax_predict")
        return prob

    def predict(self, par, X, prob=False, batchsize=None):                # softmax.py:82-89
        """CPU semantics (cpu/softmax.py:82-89) by default; with ``batchsize`` the GPU file's
        batching (gpu/softmax.py:90-102): whole batches only, and prob=True returns the
        probabilities flattened to 1-D (its ``results.reshape(-1,)``)."""
        if batchsize:
            n = (X.shape[0] // batchsize) * batchsize
            yhat = self._net_device(par, X[:n])
            out = yhat if prob else yhat.argmax(dim=1)
            return out.cpu().numpy().reshape(-1)
        yhat = self._net_device(par, X)
        out = yhat if prob else yhat.argmax(dim=1)
        return out.cpu().numpy()

    def predict_stochastic(self, par, X, prob=False, p=0.5, Z=None, batchsize=None):   # softmax.py:91-100
        """Input dropout X ⊙ Z, Z ~ Bernoulli(p) (``Z`` may be given).  With ``batchsize`` the GPU
        file's batching (gpu/softmax.py:105-121): whole batches, output reshaped to
        (-1, last dimension) as there."""
        X = self._dev(X)
        if batchsize:
            n = (X.shape[0] // batchsize) * batchsize
            X = X[:n]
            Z = Z[:n] if Z is not None else None
        if Z is None:
            Z = torch.bernoulli(torch.full_like(X, p))
        else:
            Z = self._dev(Z)
        yhat = self._net_device(par, X * Z)
        out = (yhat if prob else yhat.argmax(dim=1)).cpu().numpy()
        if batchsize:
            out = out.reshape(-1, out.shape[-1]) if prob else out.reshape(-1, batchsize)
        return out

    def predict_posterior(self, posterior, X, prob=False):
        """Posterior predictive over S samples (extension): mean over s of softmax(X·W_s + b_s), all
        S parameter sets in ONE launch (the chain-interleaved layout W[D][S][K] of hmcx_softmax_predict).
        ``posterior``: {'weights': [S, D, K], 'bias': [S, K]} as returned by ``sample``."""
        Ws = np.asarray(posterior['weights'])
        bs = np.asarray(posterior['bias'])
        S, D, K = Ws.shape
        Xd = self._dev(X)
        B = Xd.shape[0]
        W = self._dev(np.ascontiguousarray(Ws.transpose(1, 0, 2)).reshape(D, S * K))
        b = self._dev(bs.reshape(S * K))
        prob_all = torch.empty((B, S * K), dtype=self.dtype, device=self.device)
        ctx = context(self.device)
        ctx.check(ctx.lib.hmcx_softmax_predict(ctx.h, self.code, ptr(Xd), B, D, K, S, ptr(W), ptr(b),
                                               ptr(prob_all)), "hmcx_softmax_predict")
        mean = prob_all.cpu().numpy().reshape(B, S, K).mean(axis=1)
        return mean if prob else mean.argmax(axis=1)
