"""Full-batch HMC — drop-in for hamiltonian/inference/{cpu,gpu}/hmc.py.

Reference: /root/reference/hamiltonian/inference/cpu/hmc.py:11-176.
step (hmc.py:39-64): per var  p −= ½ε·g;  q += ε·p;  g = ∇U(q);  p −= ε·g;  then p ← −p and
MH accept min(1, exp(E_cur − E_new)).  sample (hmc.py:90-119) draws one discarded momentum
first (hmc.py:93), runs burn-in, updates DualAveragingStepSize once and prints it (the value
is not used, hmc.py:101-102), then samples.

Device paths:

* MVN model (config 1): every step of a burn-in / sampling phase runs in ONE device launch
  (hmcx_hmc_mvn_run, one thread per chain);
* softmax (CPU prior) and logistic models: a burn-in / sampling phase is ONE hmcx_hmc_run call —
  momentum, every kick/drift (fused into the gradient kernels' epilogues), the energies, the MH
  accept and the commit run on the device; the host only draws the schedule (path lengths, accept
  uniforms and, in noise='numpy' mode, the momenta) in the reference's order;
* the MLP: a step's whole leapfrog trajectory is ONE hmcx_mlp_hmc_leapfrog call (device gradients,
  kicks and drifts enqueued from C in the reference's order); the energies go out as device pieces
  read back once.  A model that overrides grad (or HMCX_HMC_HOST_LOOP=1) runs the reference's loop
  with device gradients (model.grad) and hmcx_axpy / hmcx_sumsq from the host instead.
"""
import os
import sys
from copy import deepcopy

import numpy as np
import torch

from dropout_hamiltonian_montecarlo_amd import _native as nat
from dropout_hamiltonian_montecarlo_amd._native import HmcxError, ptr

from .sghmc import _n_iter


def _host_loop():
    return os.environ.get("HMCX_HMC_HOST_LOOP", "0") == "1"


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
                noise[s] = nat.philox_normals(self.seed, self.chain, g, 0, 0, dim, dtype="f64")
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
        # both modes hand the device the host-drawn momenta (philox: the f64 Philox stream's host twin),
        # so the returned momentums are exactly the ones used (dim = 2: nothing to save on the device)
        a.noise_mode = nat.NOISE_BUFFER
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
        if self._linear_fused():
            return self._sample_linear(niter, nburn, burnin, rng, step_size_tuning, args)
        return self._sample_generic(niter, nburn, burnin, rng, step_size_tuning, args)

    # ------------------------------------------------------------------ softmax / logistic fused path
    def _linear_fused(self):
        m = self.model
        return (m._hmcx_model in ('softmax', 'logistic') and getattr(m, 'prior', 'cpu') == 'cpu'
                and list(self.start.keys()) == ['weights', 'bias'])

    def _linear_data(self, args):
        m = self.model
        X, y = m._xy(args)
        return X.contiguous(), y.contiguous()

    def _linear_run(self, W, b, data, n_steps, rng, record):
        """n_steps HMC steps in one hmcx_hmc_run call.  Host work: the schedule in the reference's
        draw order (hmc.py:41 momentum from rng, :46 path length and :61 accept uniform from the
        global np.random) or, with noise='philox', path lengths / uniforms from the Philox twin."""
        m = self.model
        Xd, Yd = data
        D, K = W.shape
        P = D * K + K
        eps = np.full(n_steps, self.step_size, dtype=np.float64)
        n_iter = np.empty(n_steps, dtype=np.int32)
        u = np.empty(n_steps, dtype=np.float64)
        noise = np.empty((n_steps, P), dtype=np.float64) if self.noise == 'numpy' else None
        for s in range(n_steps):
            g = (self.global_step + s) & 0xFFFFFFFF
            if self.noise == 'numpy':
                mom = self.draw_momentum(rng)                                  # hmc.py:41
                noise[s, :D * K] = mom['weights'].reshape(-1)
                noise[s, D * K:] = mom['bias'].reshape(-1)
                L = np.ceil(2 * np.random.rand() * self.path_length / self.step_size)   # hmc.py:46
                n_iter[s] = _n_iter(L)
                u[s] = np.random.rand()                                        # hmc.py:61
            else:
                L = np.ceil(2 * nat.philox_uniforms(self.seed, self.chain, g, nat.SLOT_PATH, 1)[0]
                            * self.path_length / self.step_size)
                n_iter[s] = _n_iter(L)
                u[s] = nat.philox_uniforms(self.seed, self.chain, g, nat.SLOT_ACCEPT, 1)[0]
        dev = m.device
        noise_d = torch.from_numpy(noise.ravel()).to(dev) if noise is not None else None
        noff = np.arange(n_steps, dtype=np.int64) * P
        out_f = torch.empty(4 * n_steps, dtype=torch.float64, device=dev)        # A, nlp, E (2)
        out_acc = torch.empty(n_steps, dtype=torch.int32, device=dev)
        tr = torch.empty((n_steps, P), dtype=m.dtype, device=dev) if record else None
        mo = torch.empty((n_steps, P), dtype=m.dtype, device=dev) if (record and noise is None) else None
        a = nat.HmcArgs()
        a.dtype, a.model = m.code, nat.MODEL_LOGISTIC if m._hmcx_model == 'logistic' else nat.MODEL_SOFTMAX
        a.B, a.D, a.K, a.n_steps = Xd.shape[0], D, K, n_steps
        a.alpha = m.alpha
        if m._hmcx_model == 'logistic':                                        # logistic.py:15-21
            for i, var in enumerate(('weights', 'bias')):
                dim = int(np.prod(np.shape(self.start[var])))
                a.lp_const[i] = dim * 0.5 * np.log(m.hyper['alpha'] / (2 * np.pi))
        else:
            a.log_prior = m.log_prior_const([np.shape(self.start[v]) for v in self.start])
        a.X, a.Y = ptr(Xd), ptr(Yd)
        a.eps = eps.ctypes.data_as(nat.c_dblp)
        a.n_iter = n_iter.ctypes.data_as(nat.c_i32p)
        a.u_accept = u.ctypes.data_as(nat.c_dblp)
        a.noise_mode = nat.NOISE_BUFFER if noise is not None else nat.NOISE_PHILOX
        a.noise = ptr(noise_d)
        a.noise_off = noff.ctypes.data_as(nat.c_i64p)
        a.seed, a.chain, a.step_base = self.seed, self.chain, self.global_step & 0xFFFFFFFF
        a.W, a.b = ptr(W), ptr(b)
        a.out_A, a.out_nlp, a.out_E = ptr(out_f[:n_steps]), ptr(out_f[n_steps:2 * n_steps]), ptr(out_f[2 * n_steps:])
        a.out_accepted = ptr(out_acc)
        a.out_trace, a.out_mom = ptr(tr), ptr(mo)
        ctx = nat.context(dev)
        ctx.check(ctx.lib.hmcx_hmc_run(ctx.h, a), "hmcx_hmc_run")
        self.global_step += n_steps
        f = out_f.cpu().numpy()
        A, nlp = f[:n_steps], f[n_steps:2 * n_steps]
        acc = out_acc.cpu().numpy().astype(bool)
        if self.trace is not None:
            self.trace.extend({'L': float(n + 1), 'A': float(A[s]), 'accepted': bool(acc[s]), 'eps': self.step_size}
                              for s, n in enumerate(n_iter))
        trace = tr.cpu().numpy().astype(np.float64) if tr is not None else None
        mom = (noise if noise is not None else mo.cpu().numpy().astype(np.float64)) if record else None
        return A, acc, nlp, trace, mom

    def _split(self, flat):
        D, K = np.shape(self.start['weights'])
        return {'weights': flat[:D * K].reshape(D, K).copy(), 'bias': flat[D * K:].reshape(np.shape(self.start['bias'])).copy()}

    def _sample_linear(self, niter, nburn, burnin, rng, tuning, args):
        m = self.model
        data = self._linear_data(args)
        W = m._dev(self.start['weights']).clone()
        b = m._dev(np.reshape(self.start['bias'], -1)).clone()
        p_accept = None
        if nburn > 0:
            A, _, nlp, _, _ = self._linear_run(W, b, data, nburn, rng, False)
            for i in range(nburn):
                if self.verbose is not None and (i % (burnin / 10) == 0):
                    print('loss: {0:.4f}'.format(nlp[i]), file=self.out)
            p_accept = A[-1]
        _, avg_step_size = tuning.update(p_accept)
        print('adapted step size : ', avg_step_size, file=self.out)
        before = np.concatenate([W.cpu().numpy().reshape(-1), b.cpu().numpy().reshape(-1)]).astype(np.float64)
        if niter == 0:
            return {v: np.zeros((0,) + np.shape(self.start[v])) for v in self.start}, np.zeros(0), [], []
        A, acc, nlp, tr, mom = self._linear_run(W, b, data, niter, rng, True)
        positions = [[self._split(before if i == 0 else tr[i - 1])] for i in range(niter)]
        momentums = [[self._split(mom[i])] for i in range(niter)]
        for i in range(niter):
            if self.verbose and (i % (niter / 10) == 0):
                print('loss: {0:.4f}'.format(nlp[i]), file=self.out)
        D, K = np.shape(self.start['weights'])
        posterior = {'weights': tr[:, :D * K].reshape((niter,) + np.shape(self.start['weights'])),
                     'bias': tr[:, D * K:].reshape((niter,) + np.shape(self.start['bias']))}
        self.last_state = {'weights': W, 'bias': b}
        return posterior, nlp, positions, momentums

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
    def _K(self, p):                                                         # hmc.py:74-79
        """Σ_var ½·Σp²: one device reduction per variable into one buffer, one readback (the per-variable
        sums are added on the host in the reference's variable order)."""
        K = 0
        ctx = nat.context(self.model.device)
        ss = torch.empty(len(p), dtype=torch.float64, device=self.model.device)
        keep = []
        for i, var in enumerate(p.keys()):
            v = p[var].reshape(-1)
            keep.append(v)
            ctx.check(ctx.lib.hmcx_sumsq(ctx.h, self.model.code, ptr(v), v.numel(), ptr(ss[i:i + 1])), "hmcx_sumsq")
        for s2 in ss.cpu().numpy():
            K += 0.5 * float(s2)
        return K

    def _sumsq_into(self, p, out):
        """Σp² of each variable of p into out[i] (device, no readback)."""
        ctx = nat.context(self.model.device)
        keep = []
        for i, var in enumerate(p.keys()):
            v = p[var].reshape(-1)
            keep.append(v)
            ctx.check(ctx.lib.hmcx_sumsq(ctx.h, self.model.code, ptr(v), v.numel(), ptr(out[i:i + 1])), "hmcx_sumsq")
        return keep

    @staticmethod
    def _K_from(sums):                                                      # hmc.py:74-79
        K = 0
        for s2 in sums:
            K += 0.5 * float(s2)
        return K

    def _energies(self, q_new, p_new, q, p, args):
        """E_new, E_cur (hmc.py:57-58).  A model with energy_parts_device (the MLP) gets all four terms
        enqueued into one device buffer and read back once, in the reference's order of evaluation;
        otherwise through negative_log_posterior and _K."""
        m = self.model
        if not hasattr(m, "energy_parts_device"):
            E_new = m.negative_log_posterior(q_new, **args) + self._K(p_new)
            E_cur = m.negative_log_posterior(q, **args) + self._K(p)
            return E_new, E_cur
        nq, npv = len(q_new), len(p_new)
        buf = torch.empty(2 * (1 + nq + npv), dtype=torch.float64, device=m.device)
        o = [0, 1 + nq, 1 + nq + npv, 2 + 2 * nq + npv, 2 * (1 + nq + npv)]
        keep = [m.energy_parts_device(q_new, buf[o[0]:o[1]], **args), self._sumsq_into(p_new, buf[o[1]:o[2]]),
                m.energy_parts_device(q, buf[o[2]:o[3]], **args), self._sumsq_into(p, buf[o[3]:o[4]])]
        h = buf.cpu().numpy()
        del keep
        E_new = m.nlp_from_parts(h[o[0]:o[1]], q_new) + self._K_from(h[o[1]:o[2]])
        E_cur = m.nlp_from_parts(h[o[2]:o[3]], q) + self._K_from(h[o[3]:o[4]])
        return E_new, E_cur

    def _axpy(self, mode, a, x, y):
        """y −= a·x (mode 0) / y += a·x (mode 1) on the device (hmcx_axpy)."""
        ctx = nat.context(self.model.device)
        ctx.check(ctx.lib.hmcx_axpy(ctx.h, self.model.code, mode, y.numel(), float(a), ptr(x), ptr(y)), "hmcx_axpy")

    def step(self, state, momentum, rng, **args):                           # hmc.py:39-64
        m = self.model
        dev, dt = m.device, m.dtype
        q = {k: torch.as_tensor(np.asarray(v) if not isinstance(v, torch.Tensor) else v).to(dev, dt).contiguous()
             for k, v in state.items()}
        p_host = self.draw_momentum(rng)
        p = {k: torch.as_tensor(v).to(dev, dt).contiguous() for k, v in p_host.items()}
        q_new = {k: v.clone() for k, v in q.items()}
        p_new = {k: v.clone() for k, v in p.items()}
        # the recorded momentum is the host draw in the model's dtype (what a device round trip returns)
        npdt = torch.empty(0, dtype=dt).numpy().dtype
        positions, momentums = [deepcopy(state)], [{k: np.asarray(v).astype(npdt) for k, v in p_host.items()}]
        epsilon = self.step_size
        path_length = np.ceil(2 * np.random.rand() * self.path_length / epsilon)
        if hasattr(m, "leapfrog_device") and m.leapfrog_device_ok() and not _host_loop():
            # the whole trajectory in one libhmcx call (hmcx_mlp_hmc_leapfrog): the same kernels in the
            # same order as the loop below, enqueued from C
            m.leapfrog_device(q_new, p_new, _n_iter(path_length), epsilon, list(self.start.keys()), **args)
        else:
            grad_q = m.grad(q, **args)
            for _ in range(_n_iter(path_length)):
                for var in self.start.keys():
                    self._axpy(0, 0.5 * epsilon, grad_q[var], p_new[var])      # hmc.py:50
                    self._axpy(1, epsilon, p_new[var], q_new[var])             # hmc.py:51
                    grad_q = m.grad(q_new, **args)
                    self._axpy(0, epsilon, grad_q[var], p_new[var])            # hmc.py:53
            for var in self.start.keys():
                self._axpy(0, 2.0, p_new[var], p_new[var])                     # hmc.py:55-56: p − 2p = −p
        E_new, E_cur = self._energies(q_new, p_new, q, p, args)
        acceptprob = min(1, np.exp(E_cur - E_new))
        accepted = bool(np.isfinite(acceptprob) and (np.random.rand() < acceptprob))
        if accepted:
            q, p = q_new, p_new
        if self.trace is not None:
            self.trace.append({'L': float(path_length), 'A': float(acceptprob), 'accepted': accepted,
                               'eps': float(epsilon)})
        return q, p, positions, momentums, acceptprob

    def _loss_and_state(self, q, args):
        """negative_log_posterior(q) (hmc.py:113) and q on the host.  With energy_parts_device and a
        device state: the loss pieces and the state (widened to float64, exactly) in one buffer, one
        readback."""
        m = self.model
        keys = list(self.start.keys())
        if not (hasattr(m, "energy_parts_device") and all(isinstance(q[v], torch.Tensor) for v in keys)):
            loss = m.negative_log_posterior(q, **args)
            return loss, {v: q[v].cpu().numpy() if isinstance(q[v], torch.Tensor) else q[v] for v in keys}
        nq = len(q)
        sizes = [q[v].numel() for v in keys]
        buf = torch.empty(1 + nq + sum(sizes), dtype=torch.float64, device=m.device)
        keep = m.energy_parts_device(q, buf[:1 + nq], **args)
        buf[1 + nq:].copy_(torch.cat([q[v].reshape(-1) for v in keys]))
        h = buf.cpu().numpy()
        del keep
        npdt = torch.empty(0, dtype=m.dtype).numpy().dtype
        qh, o = {}, 1 + nq
        for v, n in zip(keys, sizes):
            qh[v] = h[o:o + n].astype(npdt).reshape(tuple(q[v].shape))
            o += n
        return m.nlp_from_parts(h[:1 + nq], q), qh

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
            loss[i], qh = self._loss_and_state(q, args)
            for var in self.start.keys():
                posterior[var].append(qh[var])
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
