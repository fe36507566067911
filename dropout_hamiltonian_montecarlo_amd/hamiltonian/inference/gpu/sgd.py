"""Momentum SGD — drop-in for hamiltonian/inference/{cpu,gpu}/sgd.py.

Reference: /root/reference/hamiltonian/inference/cpu/sgd.py:11-70.  ``fit`` runs, per minibatch,
g = model.grad(θ); m = γ·m − η·g; θ += m (sgd.py:36-41) and records negative_log_posterior on the
epoch's last minibatch (:42); ``fit_dropout`` multiplies each minibatch by a fresh Bernoulli(p)
mask Z first (:59-63) and records −log_likelihood on the undropped last minibatch (:67).

One epoch is ONE libhmcx call (hmcx_sgd_run: per minibatch one k_fwd + one k_grad launch, the
momentum update fused into the gradient epilogue); the dataset is resident in HBM for the whole
fit.  Models: the libhmcx softmax and logistic models.

Masks of fit_dropout: ``noise='numpy'`` (default) draws Z on the host with the reference's own
call, ``np.random.binomial(1, p, size=X_batch.shape)`` per minibatch in minibatch order, so a
float64 fit matches the reference's up to GEMM summation order; ``noise='philox'`` draws Z on
the device (Philox keyed by (seed, global minibatch index, element)).
"""
import sys

import numpy as np
import torch

from dropout_hamiltonian_montecarlo_amd import _native as nat
from dropout_hamiltonian_montecarlo_amd._native import HmcxError, ptr


class sgd:

    def __init__(self, model, start_p, step_size=0.1, noise='numpy', seed=0):   # sgd.py:13-16
        self.start = start_p
        self.step_size = step_size
        self.model = model
        if noise not in ('numpy', 'philox'):
            raise ValueError("noise must be 'numpy' or 'philox'")
        self.noise, self.seed = noise, int(seed)
        self.global_step = 0
        self.out = sys.stdout
        kind = getattr(model, '_hmcx_model', None)
        if kind not in ('softmax', 'logistic'):
            raise HmcxError("sgd: libhmcx implements sgd for the softmax and logistic models")
        if list(start_p.keys()) != ['weights', 'bias']:
            raise HmcxError("sgd: start_p keys must be ['weights', 'bias']")

    def iterate_minibatches(self, X, y, batchsize):                       # sgd.py:19-23
        assert X.shape[0] == y.shape[0]
        for start_idx in range(0, X.shape[0] - batchsize + 1, batchsize):
            excerpt = slice(start_idx, start_idx + batchsize)
            yield X[excerpt], y[excerpt]

    # ------------------------------------------------------------------ device state
    def _setup(self, args, batch_size):
        m = self.model
        X = args['X_train']
        y = args['y_train']
        N = X.shape[0]
        rows = list(range(0, N - batch_size + 1, batch_size))
        if not rows:
            raise ValueError("batch_size larger than the dataset: no minibatch (sgd.py:21)")
        Xd = m._dev(X)
        Yd = m._dev(y)
        if m._hmcx_model == 'logistic':
            Yd = Yd.reshape(-1).contiguous()
            K = 1
        else:
            K = Yd.shape[1]
        par = {var: m._dev(np.asarray(self.start[var])).clone() for var in self.start}
        if m._hmcx_model == 'logistic':
            par['bias'] = par['bias'].reshape(-1).contiguous()
        mom = {var: torch.zeros_like(par[var]) for var in par}            # sgd.py:35
        return Xd, Yd, K, rows, par, mom

    def _run(self, Xd, Yd, K, rows, par, mom, batch_size, gamma, dropout=False, p=0.5):
        m = self.model
        n_steps = len(rows)
        B, D = batch_size, Xd.shape[1]
        keep_d, keep_off = None, np.zeros(n_steps, dtype=np.int64)
        if dropout and self.noise == 'numpy':
            # sgd.py:61: Z = np.random.binomial(1, p, size=X_batch.shape), one draw per minibatch
            Z = np.stack([np.random.binomial(1, p, size=(B, D)) for _ in range(n_steps)]).astype(np.uint8)
            keep_d = torch.from_numpy(Z.reshape(-1)).to(m.device)
            keep_off = np.arange(n_steps, dtype=np.int64) * (B * D)
        row0 = np.asarray(rows, dtype=np.int64)
        a = nat.SgdArgs()
        a.dtype = m.code
        a.model = nat.MODEL_LOGISTIC if m._hmcx_model == 'logistic' else nat.MODEL_SOFTMAX
        a.B, a.D, a.K, a.n_steps = B, D, K, n_steps
        a.alpha, a.step_size, a.gamma = m.alpha, float(self.step_size), float(gamma)
        a.X, a.Y = ptr(Xd), ptr(Yd)
        a.row0 = row0.ctypes.data_as(nat.c_i64p)
        a.dropout = 1 if dropout else 0
        a.keep_p = float(p)
        a.mask_mode = nat.NOISE_BUFFER if self.noise == 'numpy' else nat.NOISE_PHILOX
        a.keep = ptr(keep_d)
        a.keep_off = keep_off.ctypes.data_as(nat.c_i64p)
        a.seed, a.step_base = self.seed, self.global_step & 0xFFFFFFFF
        a.W, a.b, a.mW, a.mb = ptr(par['weights']), ptr(par['bias']), ptr(mom['weights']), ptr(mom['bias'])
        ctx = nat.context(m.device)
        ctx.check(ctx.lib.hmcx_sgd_run(ctx.h, a), "hmcx_sgd_run")
        self.global_step += n_steps
        del keep_d

    def _host(self, par):
        out = {}
        for var in self.start:
            out[var] = par[var].detach().cpu().numpy().astype(np.float64).reshape(np.shape(self.start[var]))
        return out

    # ------------------------------------------------------------------ reference surface
    def fit(self, epochs=1, batch_size=1, gamma=0.9, **args):            # sgd.py:25-45
        verbose = args.get('verbose', None)
        epochs = int(epochs)
        loss_val = np.zeros(epochs)
        Xd, Yd, K, rows, par, mom = self._setup(args, batch_size)
        last = slice(rows[-1], rows[-1] + batch_size)
        for i in range(epochs):
            self._run(Xd, Yd, K, rows, par, mom, batch_size, gamma)
            loss_val[i] = self.model.negative_log_posterior(par, X_train=Xd[last], y_train=Yd[last])
            if verbose and (i % (epochs / 10) == 0):
                print('loss: {0:.4f}'.format(loss_val[i]), file=self.out)
        self.last_state = par
        return self._host(par), loss_val

    def fit_dropout(self, epochs=1, batch_size=1, gamma=0.9, p=0.5, **args):   # sgd.py:47-70
        verbose = args.get('verbose', None)
        epochs = int(epochs)
        loss_val = np.zeros(epochs)
        Xd, Yd, K, rows, par, mom = self._setup(args, batch_size)
        last = slice(rows[-1], rows[-1] + batch_size)
        for i in range(epochs):
            self._run(Xd, Yd, K, rows, par, mom, batch_size, gamma, dropout=True, p=p)
            loss_val[i] = -1. * self.model.log_likelihood(par, X_train=Xd[last], y_train=Yd[last])
            if verbose and (i % (epochs / 10) == 0):
                print('loss: {0:.4f}'.format(loss_val[i]), file=self.out)
        self.last_state = par
        return self._host(par), loss_val
