"""ORACLE (test infrastructure only) — NumPy restatement of the reference samplers.

sgmcmc  ← /root/reference/hamiltonian/inference/cpu/sgmcmc.py:14-89
sghmc   ← /root/reference/hamiltonian/inference/cpu/sghmc.py:16-39  + the A1 completion
          (SURVEY §8a): draw_momentum/accept/potential_energy from cpu/hmc.py:67-87 and
          ``sample`` consuming the first two entries of step()'s 3-tuple.
sgld    ← /root/reference/hamiltonian/inference/cpu/sgld.py:13-46
hmc     ← /root/reference/hamiltonian/inference/cpu/hmc.py:11-176
sgd     ← /root/reference/hamiltonian/inference/cpu/sgd.py:11-70

Random streams are used exactly as in the reference: the sampler's ``rng``
(RandomState) for momenta/noise and the GLOBAL ``np.random`` for the path
length and the accept uniform.  ``trace`` (optional list) records per-step
integers (path length L, accept flag) and the accept probability A.
"""
import sys
from copy import deepcopy

import numpy as np


class sgmcmc:
    def __init__(self, model, start_p, path_length=1.0, step_size=0.1, verbose=True):  # :16-29
        self.start = {var: np.asarray(start_p[var]) for var in start_p.keys()}
        self.step_size = step_size
        self.path_length = path_length
        self.model = model
        self.verbose = verbose
        self.trace = None
        self.out = sys.stdout

    def iterate_minibatches(self, X, y, batchsize):                       # :34-38
        assert X.shape[0] == y.shape[0]
        for start_idx in range(0, X.shape[0] - batchsize + 1, batchsize):
            excerpt = slice(start_idx, start_idx + batchsize)
            yield X[excerpt], y[excerpt]

    def sample(self, epochs=1, burnin=1, batch_size=1, rng=None, **args):  # :40-86
        if rng is None:
            rng = np.random.RandomState()
        X = args['X_train']
        y = args['y_train']
        verbose = args.get('verbose', None)
        epochs = int(epochs)
        num_batches = np.ceil(y[:].shape[0] / float(batch_size))
        decay_factor = self.step_size / num_batches
        q, p = self.start, {var: np.zeros_like(self.start[var]) for var in self.start.keys()}
        print('start burnin', file=self.out)
        for i in range(int(burnin)):
            j = 0
            for X_batch, y_batch in self.iterate_minibatches(X, y, batch_size):
                kwargs = {'X_train': X_batch, 'y_train': y_batch, 'verbose': verbose}
                out = self.step(q, p, rng, **kwargs)
                q, p = out[0], out[1]
                if (j % 10) == 0:
                    ll = -1.0 * self.model.log_likelihood(q, **kwargs)
                    print('burnin {0}, loss: {1:.4f}, mini-batch update : {2}'.format(i, ll, j),
                          file=self.out)
                j = j + 1
        logp_samples = np.zeros(epochs)
        posterior = {var: [] for var in self.start.keys()}
        print('start sampling', file=self.out)
        initial_step_size = self.step_size
        for i in range(epochs):
            j = 0
            for X_batch, y_batch in self.iterate_minibatches(X, y, batch_size):
                kwargs = {'X_train': X_batch, 'y_train': y_batch, 'verbose': verbose}
                out = self.step(q, p, rng, **kwargs)
                q, p = out[0], out[1]
                self.step_size = self.lr_schedule(initial_step_size, j, decay_factor, num_batches)
                if (j % 10) == 0:
                    ll = -1.0 * self.model.log_likelihood(q, **kwargs)
                    print('epoch {0}, loss: {1:.4f}, mini-batch update : {2}'.format(i, ll, j),
                          file=self.out)
                j = j + 1
            logp_samples[i] = self.model.negative_log_posterior(q, **kwargs)
            for var in self.start.keys():
                posterior[var].append(q[var])
            if self.verbose and (i % (epochs / 10) == 0):
                print('loss: {0:.4f}'.format(logp_samples[i]), file=self.out)
        for var in self.start.keys():
            posterior[var] = np.array(posterior[var])
        return posterior, logp_samples

    def lr_schedule(self, initial_step_size, step, decay_factor, num_batches):  # :88-89
        return initial_step_size * (1.0 / (1.0 + step * decay_factor * num_batches))


class sghmc(sgmcmc):
    def step(self, state, momentum, rng, **args):                         # sghmc.py:19-39
        q = state.copy()
        p = self.draw_momentum(rng)
        q_new = deepcopy(q)
        p_new = deepcopy(p)
        epsilon = self.step_size
        path_length = np.ceil(2 * np.random.rand() * self.path_length / epsilon)
        # sghmc.py:26 computes grad(q) and discards it (dead; no RNG use) — omitted.
        for _ in np.arange(path_length - 1):
            for var in self.start.keys():
                dim = (np.array(q_new[var])).size
                rvar = rng.normal(0, 2 * epsilon, dim).reshape(q[var].shape)
                q_new[var] += epsilon * p_new[var]
                grad_q = self.model.grad(q_new, **args)
                p_new[var] = (1 - epsilon) * p_new[var] + epsilon * grad_q[var] + rvar
        acceptprob = self.accept(q, q_new, p, p_new, **args)
        accepted = bool(np.isfinite(acceptprob) and (np.random.rand() < acceptprob))
        if accepted:
            q = q_new.copy()
            p = p_new.copy()
        if self.trace is not None:
            self.trace.append({'L': float(path_length), 'A': float(acceptprob),
                               'accepted': accepted, 'eps': float(epsilon), 'E': self._E})
        return q, p, acceptprob

    # --- A1 completion: cpu/hmc.py:67-87 -------------------------------------
    def accept(self, current_q, proposal_q, current_p, proposal_p, **args):  # hmc.py:67-71
        E_new = (self.model.negative_log_posterior(proposal_q, **args) + self.potential_energy(proposal_p))
        E_current = (self.model.negative_log_posterior(current_q, **args) + self.potential_energy(current_p))
        A = min(1, np.exp(E_current - E_new))
        self._E = (float(E_current), float(E_new))        # test-side record for the trace (no effect on A)
        return A

    def potential_energy(self, p):                                        # hmc.py:74-79
        K = 0
        for var in p.keys():
            K += 0.5 * (np.sum(np.square(p[var])))
        return K

    def draw_momentum(self, rng):                                         # hmc.py:82-87
        momentum = {}
        for var in self.start.keys():
            momentum[var] = rng.normal(0, 1, size=self.start[var].shape)
        return momentum


class sgld(sgmcmc):
    def step(self, state, momentum, rng, **args):                         # sgld.py:31-39
        epsilon = self.step_size
        q = deepcopy(state)
        p = self.draw_momentum(rng, epsilon)
        grad_q = self.model.grad(q, **args)
        for var in p.keys():
            p[var] += - 0.5 * epsilon * grad_q[var]
            q[var] += p[var]
        return q, p

    def draw_momentum(self, rng, epsilon):                                # sgld.py:41-46
        noise_scale = 2.0 * epsilon
        return {var: rng.normal(0, noise_scale, size=self.start[var].shape) for var in self.start.keys()}


class sgld_gpu_variant(sgld):
    """gpu/sgld.py:11-20 — the GPU file's different update p = ν⊙p_prev − ½ε∇U."""

    def step(self, state, momentum, rng, **args):
        epsilon = self.step_size
        q = deepcopy(state)
        nu = self.draw_momentum(rng, epsilon)
        p = deepcopy(momentum)
        grad_q = self.model.grad(q, **args)
        for var in p.keys():
            p[var] = nu[var] * p[var] - 0.5 * epsilon * grad_q[var]
            q[var] += p[var]
        return q, p


class hmc:
    """cpu/hmc.py:11-138 (full-batch HMC)."""

    def __init__(self, model, start_p, path_length=1.0, step_size=0.1, verbose=True):  # :12-36
        self.start = start_p
        self.step_size = step_size
        self.path_length = path_length
        self.model = model
        self.verbose = verbose
        self.trace = None
        self.out = sys.stdout

    def step(self, state, momentum, rng, **args):                         # :39-64
        q = state.copy()
        p = self.draw_momentum(rng)
        q_new = deepcopy(q)
        p_new = deepcopy(p)
        positions, momentums = [deepcopy(q)], [deepcopy(p)]
        epsilon = self.step_size
        path_length = np.ceil(2 * np.random.rand() * self.path_length / epsilon)
        grad_q = self.model.grad(q, **args)
        for _ in np.arange(path_length - 1):
            for var in self.start.keys():
                p_new[var] -= (0.5 * epsilon) * grad_q[var]
                q_new[var] += epsilon * p_new[var]
                grad_q = self.model.grad(q_new, **args)
                p_new[var] -= epsilon * grad_q[var]
        for var in self.start.keys():
            p_new[var] = -p_new[var]
        acceptprob = self.accept(q, q_new, p, p_new, **args)
        accepted = bool(np.isfinite(acceptprob) and (np.random.rand() < acceptprob))
        if accepted:
            q = q_new.copy()
            p = p_new.copy()
        if self.trace is not None:
            self.trace.append({'L': float(path_length), 'A': float(acceptprob),
                               'accepted': accepted, 'eps': float(epsilon)})
        return q, p, positions, momentums, acceptprob

    accept = sghmc.accept
    potential_energy = sghmc.potential_energy
    draw_momentum = sghmc.draw_momentum

    def sample(self, niter=1e4, burnin=1e3, rng=None, **args):           # :90-119
        if rng is None:
            rng = np.random.RandomState()
        q, p = self.start, self.draw_momentum(rng)
        step_size_tuning = DualAveragingStepSize(self.step_size)
        p_accept = None
        for i in range(int(burnin)):
            q, p, positions, momentums, p_accept = self.step(q, p, rng, **args)
            if self.verbose is not None and (i % (burnin / 10) == 0):
                ll = self.model.negative_log_posterior(q, **args)
                print('loss: {0:.4f}'.format(ll), file=self.out)
        _, avg_step_size = step_size_tuning.update(p_accept)
        print('adapted step size : ', avg_step_size, file=self.out)
        loss = np.zeros(int(niter))
        sample_positions, sample_momentums = [], []
        posterior = {var: [] for var in self.start.keys()}
        for i in range(int(niter)):
            q, p, positions, momentums, _ = self.step(q, p, rng, **args)
            sample_positions.append(positions)
            sample_momentums.append(momentums)
            loss[i] = self.model.negative_log_posterior(q, **args)
            for var in self.start.keys():
                posterior[var].append(q[var])
            if self.verbose and (i % (niter / 10) == 0):
                print('loss: {0:.4f}'.format(loss[i]), file=self.out)
        for var in self.start.keys():
            posterior[var] = np.array(posterior[var])
        return posterior, loss, sample_positions, sample_momentums


class DualAveragingStepSize:                                              # hmc.py:141-176
    def __init__(self, initial_step_size, target_accept=0.8, gamma=0.05, t0=10.0, kappa=0.75):
        self.mu = np.log(10 * initial_step_size)
        self.target_accept = target_accept
        self.gamma = gamma
        self.t = t0
        self.kappa = kappa
        self.error_sum = 0
        self.log_averaged_step = 0

    def update(self, p_accept):
        self.error_sum += self.target_accept - p_accept
        log_step = self.mu - self.error_sum / (np.sqrt(self.t) * self.gamma)
        eta = self.t ** -self.kappa
        self.log_averaged_step = eta * log_step + (1 - eta) * self.log_averaged_step
        self.t += 1
        return np.exp(log_step), np.exp(self.log_averaged_step)


class sgd:
    """cpu/sgd.py:11-70 — momentum SGD (fit) and input-dropout SGD (fit_dropout).  The tqdm
    progress bar of the reference (:36,58) is omitted (display only)."""

    def __init__(self, model, start_p, step_size=0.1):                  # :13-16
        self.start = start_p
        self.step_size = step_size
        self.model = model
        self.out = sys.stdout

    iterate_minibatches = sgmcmc.iterate_minibatches                    # :19-23

    def fit(self, epochs=1, batch_size=1, gamma=0.9, **args):           # :25-45
        X = args['X_train']
        y = args['y_train']
        verbose = args.get('verbose', None)
        epochs = int(epochs)
        loss_val = np.zeros(epochs)
        par = deepcopy(self.start)
        momentum = {var: np.zeros_like(par[var]) for var in par.keys()}
        for i in range(epochs):
            for X_batch, y_batch in self.iterate_minibatches(X, y, batch_size):
                grad_p = self.model.grad(par, X_train=X_batch, y_train=y_batch)
                for var in par.keys():
                    momentum[var] = gamma * momentum[var] - self.step_size * grad_p[var]
                    par[var] += momentum[var]
            loss_val[i] = self.model.negative_log_posterior(par, X_train=X_batch, y_train=y_batch)
            if verbose and (i % (epochs / 10) == 0):
                print('loss: {0:.4f}'.format(loss_val[i]), file=self.out)
        return par, loss_val

    def fit_dropout(self, epochs=1, batch_size=1, gamma=0.9, p=0.5, **args):   # :47-70
        X = args['X_train']
        y = args['y_train']
        verbose = args.get('verbose', None)
        epochs = int(epochs)
        loss_val = np.zeros(epochs)
        par = deepcopy(self.start)
        momentum = {var: np.zeros_like(par[var]) for var in par.keys()}
        for i in range(epochs):
            for X_batch, y_batch in self.iterate_minibatches(X, y, batch_size):
                Z = np.random.binomial(1, p, size=X_batch.shape)
                X_batch_dropout = np.multiply(X_batch, Z)
                grad_p = self.model.grad(par, X_train=X_batch_dropout, y_train=y_batch)
                for var in par.keys():
                    momentum[var] = gamma * momentum[var] - self.step_size * grad_p[var]
                    par[var] += momentum[var]
            loss_val[i] = -1. * self.model.log_likelihood(par, X_train=X_batch, y_train=y_batch)
            if verbose and (i % (epochs / 10) == 0):
                print('loss: {0:.4f}'.format(loss_val[i]), file=self.out)
        return par, loss_val


def backend_mean_arrays(start, backends, niter):
    """cpu/hmc.py:132-138 (backend_mean) over in-memory stand-ins of the backend files: each
    element of ``backends`` maps dataset name → float32 array (the file's contents)."""
    aux = []
    for f in backends:
        aux.append({var: np.sum(f[var], axis=0) for var in f.keys()})
    return {var: ((np.sum([r[var] for r in aux], axis=0).reshape(start[var].shape)) / niter) for var in start.keys()}


def multicore_steps(sampler, X, y, niter_w, burnin_w, batch_size, rng):
    """One worker of cpu/sghmc_multicore.py:19-53 / gpu/sgld_multicore.py:21-47 fed the minibatches
    in order: burnin_w passes, then niter_w passes recording the state after every step (the rows
    appended to the backend).  Returns {var: [T, *shape]} float64 and the per-pass logp of the last
    minibatch (negative_log_posterior)."""
    q = {var: np.array(sampler.start[var], dtype=np.float64) for var in sampler.start}
    p = {var: np.zeros_like(q[var]) for var in q}
    rows = {var: [] for var in q}
    logp = np.zeros(niter_w)
    for i in range(burnin_w + niter_w):
        for X_b, y_b in sampler.iterate_minibatches(X, y, batch_size):
            out = sampler.step(q, p, rng, X_train=X_b, y_train=y_b)
            q, p = out[0], out[1]
            if i >= burnin_w:
                for var in q:
                    rows[var].append(np.array(q[var]))
        if i >= burnin_w:
            logp[i - burnin_w] = sampler.model.negative_log_posterior(q, X_train=X_b, y_train=y_b)
    return {var: np.array(rows[var]) for var in rows}, logp
