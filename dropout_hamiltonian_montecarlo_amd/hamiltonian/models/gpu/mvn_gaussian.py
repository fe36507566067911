"""Multivariate Gaussian target — drop-in for hamiltonian/models/{cpu,gpu}/mvn_gaussian.py.

Reference: /root/reference/hamiltonian/models/cpu/mvn_gaussian.py:9-31.
The HMC hot path for this model is the fused device kernel behind hmcx_hmc_mvn_run
(hamiltonian.inference.gpu.hmc); ``grad``/``negative_log_posterior`` here are the per-call
surface (tiny dim-vector algebra on the device tensors).
"""
import numpy as np
import torch

from dropout_hamiltonian_montecarlo_amd._native import context


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

    def grad(self, par, **args):                                            # :14-20
        x = torch.as_tensor(np.asarray(par['x']) if not isinstance(par['x'], torch.Tensor) else par['x'])
        x = x.to(self.device, torch.float64)
        return {'x': (x - self.mu) @ self.prec}

    def negative_log_posterior(self, par, **args):                          # :22-31
        x = torch.as_tensor(np.asarray(par['x']) if not isinstance(par['x'], torch.Tensor) else par['x'])
        d = x.to(self.device, torch.float64) - self.mu
        return float((self.nlp_const + float((d @ self.prec) @ d)) * 0.5)

    def loss(self, par, **args):
        return self.negative_log_posterior(par, **args)
