"""Multivariate Gaussian target — drop-in for hamiltonian/models/{cpu,gpu}/mvn_gaussian.py.

Reference: /root/reference/hamiltonian/models/cpu/mvn_gaussian.py:9-31.
The HMC hot path for this model is the fused device kernel behind hmcx_hmc_mvn_run
(hamiltonian.inference.gpu.hmc); ``grad``/``negative_log_posterior`` here are the per-call
surface, one hmcx_mvn_eval launch each (the same device functions as the fused kernel).
"""
import numpy as np
import torch

from dropout_hamiltonian_montecarlo_amd._native import context, ptr


class mvn_gaussian:
    _hmcx_model = 'mvn_gaussian'

    def __init__(self, _hyper, device=None):
        self.hyper = _hyper
        self.dtype = torch.float64
        self.ctx = context(device)
        self.device = self.ctx.device
        mu = np.asarray(_hyper['mu'], dtype=np.float64)
        cov = np.asarray(_hyper['cov'], dtype=np.float64)
        self.dim = mu.shape[0]
        self.prec_np = np.linalg.inv(cov)                                    # mvn_gaussian.py:19
        # mvn_gaussian.py:27-28: dim·log2π + log det Σ (then + quad form, then ×0.5)
        self.nlp_const = self.dim * np.log(2 * np.pi) + np.log(np.linalg.det(cov))
        self.mu = torch.as_tensor(mu).to(self.device)
        self.prec = torch.as_tensor(self.prec_np).to(self.device).contiguous()

    def _x(self, par):
        x = par['x']
        x = torch.as_tensor(np.asarray(x) if not isinstance(x, torch.Tensor) else x)
        return x.to(self.device, torch.float64).reshape(-1).contiguous()

    def _eval(self, par, want_grad):
        x = self._x(par)
        g = torch.empty_like(x) if want_grad else None
        nlp = None if want_grad else torch.empty(1, dtype=torch.float64, device=self.device)
        ctx = context(self.device)
        ctx.check(ctx.lib.hmcx_mvn_eval(ctx.h, self.dim, 1, ptr(self.mu), ptr(self.prec), float(self.nlp_const),
                                        ptr(x), ptr(g), ptr(nlp)), "hmcx_mvn_eval")
        return g if want_grad else nlp

    def grad(self, par, **args):                                            # :14-20
        return {'x': self._eval(par, True)}

    def negative_log_posterior(self, par, **args):                          # :22-31
        return float(self._eval(par, False).item())

    def loss(self, par, **args):
        return self.negative_log_posterior(par, **args)
