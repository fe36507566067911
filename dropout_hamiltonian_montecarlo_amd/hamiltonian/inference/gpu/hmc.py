"""Full-batch HMC — drop-in for hamiltonian/inference/{cpu,gpu}/hmc.py.

Reference: /root/reference/hamiltonian/inference/cpu/hmc.py:11-176.
step (hmc.py:39-64): per var  p −= ½ε·g;  q += ε·p;  g = ∇U(q);  p −= ε·g;  then p ← −p and
MH accept min(1, exp(E_cur − E_new)).  sample (hmc.py:90-119) draws one discarded momentum
first (hmc.py:93), runs burn-in, updates DualAveragingStepSize once and prints it (the value
is not used, hmc.py:101-102), then samples.

For the MVN model (config 1) every step of a burn-in / sampling phase runs in ONE device
launch (hmcx_hmc_mvn_run, one thread per chain).  Other libhmcx models run the reference's
loop with device gradients (model.grad → libhmcx kernels).
"""
import sys
from copy import deepcopy

import numpy as np
import torch

from dropout_hamiltonian_montecarlo_amd import _native as nat
from dropout_hamiltonian_montecarlo_amd._native import HmcxError, ptr

from .sghmc import _n_iter


class hmc:
    def __init__(self, model, start_p, path_length=1.0, step_size=0.1, verbose=True,
                 noise='numpy', seed=0, chain=0):
        self.start = start_p
        self.step_size = step_size
        self.path_length = path_length
        self.model = model
        self.verbose = verbose
        self.noise = noise
        self.seed, self.chain = int(seed), int(chain)
        self.global_step = 0
        self.trace = None
        self.out = sys.stdout
        if getattr(model, '_hmcx_model', None) is None:
            raise HmcxError("hmc needs a libhmcx model (hamiltonian.models.gpu.*)")

    def draw_momentum(self, rng):                                           # hmc.py:82-87
        return {var: rng.normal(0, 1, size=np.shape(self.start[var])) for var in self.start.keys()}

    # ------------------------------------------------------------------ MVN fused path
    def _mvn_run(self, x, n_steps, rng):
        m = self.model
        dim = m.dim
        eps = np.full(n_steps, self.step_size, dtype=np.float64)
        n_iter = np.empty(n_steps, dtype=np.int32)
        u = np.empty(n_steps, dtype=np.float64)
        noise = np.empty((n_steps, dim), dtype=np.float64)
        for s in range(n_steps):
            g = (self.global_step + s) & 0xFFFFFFFF
            if self.noise == 'numpy':
                noise[s] = rng.normal(0, 1, size=dim)                          # hmc.py:41 (draw_momentum)
                L = np.ceil(2 * np.random.rand() * self.path_length / self.step_size)  # :46
                u[s] = np.random.rand()                                        # :61
            else:
                noise[s] = nat.philox_normals(self.seed, self.chain, g, 0, 0, dim)
                L = np.ceil(2 * nat.philox_uniforms(self.seed, self.chain, g, nat.SLOT_PATH, 1)[0]
                            * self.path_length / self.step_size)
                u[s] = nat.philox_uniforms(self.seed, self.chain, g, nat.SLOT_ACCEPT, 1)[0]
            n_iter[s] = _n_iter(L)
        dev = m.device
        noise_d = torch.from_numpy(noise.ravel()).to(dev)
        noff = np.arange(n_steps, dtype=np.int64) * dim
        out_A = torch.empty(n_steps, dtype=torch.float64, device=dev)
        out_acc = torch.empty(n_steps, dtype=torch.int32, device=dev)
        out_nlp = torch.empty(n_steps, dtype=torch.float64, device=dev)
        out_tr = torch.empty(n_steps * dim, dtype=torch.float64, device=dev)
        a = nat.MvnArgs()
        a.dim, a.C, a.n_steps = dim, 1, n_steps
        a.mu, a.prec, a.nlp_const = ptr(m.mu), ptr(m.prec), m.nlp_const
        a.eps = eps.ctypes.data_as(nat.c_dblp)
        a.n_iter = n_iter.ctypes.data_as(nat.c_i32p)
        a.u_accept = u.ctypes.data_as(nat.c_dblp)
        a.noise_mode = nat.NOISE_BUFFER if self.noise == 'numpy' else nat.NOISE_PHILOX
        a.noise = ptr(noise_d)
        a.noise_off = noff.ctypes.data_as(nat.c_i64p)
        a.seed, a.chain0, a.step_base = self.seed, self.chain, self.global_step & 0xFFFFFFFF
        a.x = ptr(x)
        a.out_A, a.out_accepted, a.out_nlp, a.out_trace = ptr(out_A), ptr(out_acc), ptr(out_nlp), ptr(out_tr)
        ctx = nat.context(dev)
        ctx.check(ctx.lib.hmcx_hmc_mvn_run(ctx.h, a), "hmcx_hmc_mvn_run")
        self.global_step += n_steps
        A = out_A.cpu().numpy()
        acc = out_acc.cpu().numpy().astype(bool)
        if self.trace is not None:
            self.trace.extend({'L': float(n + 1), 'A': float(A[s]), 'accepted': bool(acc[s]),
                               'eps': self.step_size} for s, n in enumerate(n_iter))
        return A, acc, out_nlp.cpu().numpy(), out_tr.cpu().numpy().reshape(n_steps, dim), noise

    def sample(self, niter=1e4, burnin=1e3, rng=None, **args):              # hmc.py:90-119
        if rng is None:
            rng = np.random.RandomState()
        niter, nburn = int(niter), int(burnin)
        if self.noise == 'numpy':
            self.draw_momentum(rng)                                          # hmc.py:93 consumes RNG
        step_size_tuning = DualAveragingStepSize(self.step_size)
        if self.model._hmcx_model == 'mvn_gaussian':
            return self._sample_fused(niter, nburn, burnin, rng, step_size_tuning)
        return self._sample_generic(niter, nburn, burnin, rng, step_size_tuning, args)

    def _sample_fused(self, niter, nburn, burnin, rng, tuning):
        x = torch.as_tensor(np.asarray(self.start['x'], dtype=np.float64)).to(self.model.device).contiguous().clone()
        p_accept = None
        if nburn > 0:
            A, acc, nlp, tr, _ = self._mvn_run(x, nburn, rng)
            for i in range(nburn):
                if self.verbose is not None and (i % (burnin / 10) == 0):
                    print('loss: {0:.4f}'.format(nlp[i]), file=self.out)
            p_accept = A[-1]
        _, avg_step_size = tuning.update(p_accept)
        print('adapted step size : ', avg_step_size, file=self.out)
        x_before = x.cpu().numpy().copy()
        A, acc, nlp, tr, mom = self._mvn_run(x, niter, rng)
        positions = [[{'x': (x_before if i == 0 else tr[i - 1]).copy()}] for i in range(niter)]
        momentums = [[{'x': mom[i].copy()}] for i in range(niter)]
        for i in range(niter):
            if self.verbose and (i % (niter / 10) == 0):
                print('loss: {0:.4f}'.format(nlp[i]), file=self.out)
        return {'x': tr}, nlp, positions, momentums

    # ------------------------------------------------------------------ generic path (device grads)
    def _K(self, p):
        K = 0
        for var in p.keys():
            K += 0.5 * float(torch.sum(p[var] * p[var]))
        return K

    def step(self, state, momentum, rng, **args):                           # hmc.py:39-64
        m = self.model
        dev, dt = m.device, m.dtype
        q = {k: torch.as_tensor(np.asarray(v) if not isinstance(v, torch.Tensor) else v).to(dev, dt)
             for k, v in state.items()}
        p = {k: torch.as_tensor(v).to(dev, dt) for k, v in self.draw_momentum(rng).items()}
        q_new = {k: v.clone() for k, v in q.items()}
        p_new = {k: v.clone() for k, v in p.items()}
        positions, momentums = [deepcopy(state)], [{k: v.cpu().numpy() for k, v in p.items()}]
        epsilon = self.step_size
        path_length = np.ceil(2 * np.random.rand() * self.path_length / epsilon)
        grad_q = m.grad(q, **args)
        for _ in range(_n_iter(path_length)):
            for var in self.start.keys():
                p_new[var] -= (0.5 * epsilon) * grad_q[var]
                q_new[var] += epsilon * p_new[var]
                grad_q = m.grad(q_new, **args)
                p_new[var] -= epsilon * grad_q[var]
        for var in self.start.keys():
            p_new[var] = -p_new[var]
        E_new = m.negative_log_posterior(q_new, **args) + self._K(p_new)
        E_cur = m.negative_log_posterior(q, **args) + self._K(p)
        acceptprob = min(1, np.exp(E_cur - E_new))
        accepted = bool(np.isfinite(acceptprob) and (np.random.rand() < acceptprob))
        if accepted:
            q, p = q_new, p_new
        if self.trace is not None:
            self.trace.append({'L': float(path_length), 'A': float(acceptprob), 'accepted': accepted,
                               'eps': float(epsilon)})
        return q, p, positions, momentums, acceptprob

    def _sample_generic(self, niter, nburn, burnin, rng, tuning, args):
        q, p = self.start, None
        p_accept = None
        for i in range(nburn):
            q, p, positions, momentums, p_accept = self.step(q, p, rng, **args)
            if self.verbose is not None and (i % (burnin / 10) == 0):
                print('loss: {0:.4f}'.format(self.model.negative_log_posterior(q, **args)), file=self.out)
        _, avg_step_size = tuning.update(p_accept)
        print('adapted step size : ', avg_step_size, file=self.out)
        loss = np.zeros(niter)
        sample_positions, sample_momentums = [], []
        posterior = {var: [] for var in self.start.keys()}
        for i in range(niter):
            q, p, positions, momentums, _ = self.step(q, p, rng, **args)
            sample_positions.append(positions)
            sample_momentums.append(momentums)
            loss[i] = self.model.negative_log_posterior(q, **args)
            for var in self.start.keys():
                posterior[var].append(q[var].cpu().numpy() if isinstance(q[var], torch.Tensor) else q[var])
            if self.verbose and (i % (niter / 10) == 0):
                print('loss: {0:.4f}'.format(loss[i]), file=self.out)
        for var in self.start.keys():
            posterior[var] = np.array(posterior[var])
        return posterior, loss, sample_positions, sample_momentums

    def backend_mean(self, multi_backend, niter, ncores=None):               # hmc.py:132-138
        """Posterior mean from HDF5 backend files (h5trace: the image's HDF5 C library)."""
        from dropout_hamiltonian_montecarlo_amd import h5trace
        return h5trace.backend_mean(self.start, multi_backend, niter)


class DualAveragingStepSize:                                                # hmc.py:141-176
    def __init__(self, initial_step_size, target_accept=0.8, gamma=0.05, t0=10.0, kappa=0.75):
        self.mu = np.log(10 * initial_step_size)
        self.target_accept = target_accept
        self.gamma = gamma
        self.t = t0
        self.kappa = kappa
        self.error_sum = 0
        self.log_averaged_step = 0

    def update(self, p_accept):
        if p_accept is None:
            return np.nan, np.nan
        self.error_sum += self.target_accept - p_accept
        log_step = self.mu - self.error_sum / (np.sqrt(self.t) * self.gamma)
        eta = self.t ** -self.kappa
        self.log_averaged_step = eta * log_step + (1 - eta) * self.log_averaged_step
        self.t += 1
        return np.exp(log_step), np.exp(self.log_averaged_step)
