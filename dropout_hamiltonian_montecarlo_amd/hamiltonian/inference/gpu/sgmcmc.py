"""SG-MCMC outer loop — drop-in for hamiltonian/inference/{cpu,gpu}/sgmcmc.py.

Reference: /root/reference/hamiltonian/inference/cpu/sgmcmc.py:14-89 (semantics followed)
and gpu/sgmcmc.py:14-87.  Differences are in WHERE the work runs, not in what is computed:

* the dataset is made resident in HBM once per ``sample`` call (the CuPy version copies every
  minibatch host→device, gpu/sgmcmc.py:38);
* one epoch (or burn-in epoch) is ONE call into libhmcx: the per-step schedule (step sizes,
  path lengths, accept uniforms, noise) is prepared on the host first, then every leapfrog
  iteration, energy and accept decision runs on the device; the host reads back the per-step
  log-likelihoods afterwards to print the reference's log lines (every 10 minibatches,
  sgmcmc.py:60-62,74-76) — the logging forward pass is free, it reuses the accept kernel's
  energies.

Random streams.  ``noise='numpy'`` (default) draws every random number on the host from the
same streams, in the same order, as the reference (``rng`` RandomState for momenta/noise,
the global ``np.random`` for path lengths and accept uniforms), so a float64 run reproduces
the NumPy reference's integer bookkeeping bit for bit.  ``noise='philox'`` generates all noise
on the device (counter-based, keyed by (seed, chain, step)) — the fast mode.

Several chains on one device (``chains=C``, an extension; the reference runs one chain per
process).  The chains share every minibatch and run in one libhmcx call; with C ≥ 16 the
gradient GEMMs are chain-batched ([B×D]·[D×10C]).  ``noise='philox'`` gives
independent chains (Philox key chain + c); ``noise='numpy'`` drives all C chains with the SAME
reference streams (replicas — a parity test mode).  With C > 1, ``posterior[var]`` is
[C, epochs, *shape] and ``logp`` is [C, epochs].
"""
import sys

import numpy as np
import torch

from dropout_hamiltonian_montecarlo_amd import _native as nat
from dropout_hamiltonian_montecarlo_amd._native import HmcxError, ptr


class RunResult:
    """Per-step outputs of one libhmcx run call (host numpy arrays)."""

    def __init__(self, A, accepted, ll, E=None, nlp=None, steps=None, L=None):
        self.A, self.accepted, self.ll, self.E, self.nlp = A, accepted, ll, E, nlp
        self.L = L              # path length of every step ([n_steps] or [n_steps, C]) when known
        self.steps = steps      # [n_steps, C, P] state after every step (record_steps), else None
        self.mom = None         # device [C, P] momentum returned by the last step (sghmc.step), else None


class sgmcmc:
    def __init__(self, model, start_p, path_length=1.0, step_size=0.1, verbose=True,
                 noise='numpy', seed=0, chain=0, chains=1):
        self.start = {var: np.asarray(start_p[var]) for var in start_p.keys()}   # sgmcmc.py:17
        self.step_size = step_size
        self.path_length = path_length
        self.model = model
        self.verbose = verbose
        if noise not in ('numpy', 'philox'):
            raise ValueError("noise must be 'numpy' or 'philox'")
        self.noise = noise
        self.seed = int(seed)
        self.chain = int(chain)
        self.chains = int(chains)
        if self.chains < 1:
            raise ValueError("chains must be >= 1")
        self.global_step = 0
        self.record_steps = False  # _run also returns the state after every step (RunResult.steps)
        self.trace = None          # optional list: per-step dict(L, A, accepted, eps)
        self.out = sys.stdout
        self.log_every = 10
        if getattr(model, '_hmcx_model', None) is None:
            raise HmcxError("sampler needs a libhmcx model (hamiltonian.models.gpu.*)")
        self._check_vars()

    def _check_vars(self):
        pass

    # ------------------------------------------------------------------ reference helpers
    def iterate_minibatches(self, X, y, batchsize):                       # sgmcmc.py:34-38
        assert X.shape[0] == y.shape[0]
        for start_idx in range(0, X.shape[0] - batchsize + 1, batchsize):
            excerpt = slice(start_idx, start_idx + batchsize)
            yield X[excerpt], y[excerpt]

    def lr_schedule(self, initial_step_size, step, decay_factor, num_batches):  # sgmcmc.py:88-89
        return initial_step_size * (1.0 / (1.0 + step * decay_factor * num_batches))

    # ------------------------------------------------------------------ device state
    def _upload_data(self, X, y):
        dt, dev = self.model.dtype, self.model.device
        Xd = torch.as_tensor(np.asarray(X) if not isinstance(X, torch.Tensor) else X).to(dev, dt).contiguous()
        if self.model._hmcx_model == 'mlp':                 # integer labels (mlp.py:52)
            dt = torch.int32
        Yd = torch.as_tensor(np.asarray(y) if not isinstance(y, torch.Tensor) else y).to(dev, dt).contiguous()
        return Xd, Yd

    def _state_to_host(self, state):
        C = self.chains
        out = {}
        for var in self.start:
            h = state[var].detach().cpu().numpy().astype(np.float64)
            shape = self.start[var].shape
            if C == 1:
                out[var] = h.reshape(shape)
            elif len(shape) == 2:                      # [D, C·K] chain-interleaved → [C, D, K]
                out[var] = h.reshape(shape[0], C, shape[1]).transpose(1, 0, 2).copy()
            else:                                      # [C·K] → [C, K]
                out[var] = h.reshape(C, *shape)
        return out

    def _init_state(self):
        dt, dev = self.model.dtype, self.model.device
        C = self.chains
        st = {}
        for var in self.start:
            a = self.start[var]
            if C > 1:
                a = np.tile(a, (1, C)) if a.ndim == 2 else np.tile(a, C)
            st[var] = torch.as_tensor(a).to(dev, dt).contiguous().clone()
        return st

    # ------------------------------------------------------------------ outer loop (sgmcmc.py:40-86)
    def sample(self, epochs=1, burnin=1, batch_size=1, rng=None, **args):
        if rng is None:
            rng = np.random.RandomState()
        X = args['X_train']
        y = args['y_train']
        epochs = int(epochs)
        N = y[:].shape[0]
        num_batches = np.ceil(N / float(batch_size))
        decay_factor = self.step_size / num_batches
        rows = list(range(0, X.shape[0] - batch_size + 1, batch_size))
        if not rows:
            raise ValueError("batch_size larger than the dataset: no minibatch (sgmcmc.py:36)")
        data = self._upload_data(X, y)
        state = self._init_state()
        # Epoch calls are pipelined where the sampler supports it (_enqueue/_collect): epoch i+1 is
        # enqueued before epoch i is read back, and a device copy of the state taken right after
        # epoch i stands in for the state itself.  Printed lines and results are unchanged.
        pipelined = hasattr(self, '_enqueue') and self.model._hmcx_model != 'mlp'

        def launch(eps):
            if not pipelined:
                return self._run(state, data, rows, eps, rng, batch_size)
            return self._enqueue(state, data, rows, eps, rng, batch_size)

        def finish(h):
            return self._collect(h) if pipelined else h

        print('start burnin', file=self.out)

        def burnin_log(i, res):
            for j in range(len(rows)):
                if (j % self.log_every) == 0:
                    ll = -1.0 * np.ravel(res.ll[j])[0]
                    print('burnin {0}, loss: {1:.4f}, mini-batch update : {2}'.format(i, ll, j), file=self.out)

        pend = None
        for i in range(int(burnin)):
            h = launch([self.step_size] * len(rows))
            if pend is not None:
                burnin_log(i - 1, finish(pend))
            pend = h
        if pend is not None:
            burnin_log(int(burnin) - 1, finish(pend))
        logp_samples = np.zeros(epochs) if self.chains == 1 else np.zeros((epochs, self.chains))
        posterior = {var: [] for var in self.start.keys()}
        print('start sampling', file=self.out)
        initial_step_size = self.step_size

        def epoch_done(i, res, snap):
            for j in range(len(rows)):
                if (j % self.log_every) == 0:
                    ll = -1.0 * np.ravel(res.ll[j])[0]
                    print('epoch {0}, loss: {1:.4f}, mini-batch update : {2}'.format(i, ll, j), file=self.out)
            # sgmcmc.py:79 — negative_log_posterior(q, last minibatch) from the device energies
            if res.nlp is not None:
                logp_samples[i] = res.nlp[-1]
            else:
                logp_samples[i] = (-1.0 / batch_size) * (res.ll[-1] + self._log_prior())
            host = self._state_to_host(snap)
            for var in self.start.keys():
                posterior[var].append(host[var])
            if self.verbose and (i % (epochs / 10) == 0):
                print('loss: {0:.4f}'.format(np.ravel(logp_samples[i])[0]), file=self.out)

        pend = None
        for i in range(epochs):
            eps = []
            for j in range(len(rows)):
                eps.append(self.step_size)
                self.step_size = self.lr_schedule(initial_step_size, j, decay_factor, num_batches)
            h = launch(eps)
            if not pipelined:                       # _run has already completed the epoch
                epoch_done(i, h, state)
                continue
            snap = {var: state[var].clone() for var in state}   # stream-ordered copy of the epoch's state
            if pend is not None:
                epoch_done(i - 1, finish(pend[0]), pend[1])
            pend = (h, snap)
        if pend is not None:
            epoch_done(epochs - 1, finish(pend[0]), pend[1])
        for var in self.start.keys():
            posterior[var] = np.array(posterior[var])
            if self.chains > 1:
                posterior[var] = np.moveaxis(posterior[var], 1, 0)     # [C, epochs, *shape]
        if self.chains > 1:
            logp_samples = logp_samples.T.copy()
        self.last_state = state
        return posterior, logp_samples

    def _log_prior(self):
        return self.model.log_prior_const([self.start[v].shape for v in self.start])

    def _run(self, state, data, rows, eps, rng, batch_size):
        raise NotImplementedError
