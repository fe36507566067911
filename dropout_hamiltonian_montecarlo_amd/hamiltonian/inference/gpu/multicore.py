"""Multi-chain sampling with per-step traces — the reference's ``*_multicore`` samplers.

Reference: /root/reference/hamiltonian/inference/cpu/sghmc_multicore.py:19-98 and
gpu/sgld_multicore.py:19-90.  There, ``multicore_sample`` forks ``ncores`` worker processes fed
minibatches from one shared queue; worker i draws from ``RandomState(i)``, runs
``int(burnin/ncores)`` burn-in passes and ``int(niter/ncores)`` sampling passes over the
minibatches and records the state after EVERY step — appended to its HDF5 file
``backend + "_%i.h5" % i`` (one float32 dataset per variable, first row the zero fill value,
sghmc_multicore.py:36-53) or kept in memory as flattened rows.  It returns
``(multi_backend, logp)`` or ``(posterior, logp)`` with the workers' results concatenated.

Here the ncores workers are ncores chains of ONE libhmcx call per pass (chain-batched GEMMs for
ncores ≥ 16; or spread over GPUs by ``parallel.py``), each chain seeing every minibatch in order
(the reference's shared queue hands each minibatch to whichever worker is free, which is not
reproducible).  The per-step states come back from the device in one buffer per pass
(hmcx_sampler_args.out_trace) and are appended to the backend files in one write per pass.
Chains are independent with ``noise='philox'`` (the default of these classes); with
``noise='numpy'`` every chain replays one RandomState(0) stream (replicas — with ncores = 1 this
is the reference worker 0's stream exactly).  ``logp[i]`` of a chain is the negative log
posterior of the last minibatch after pass i (sghmc_multicore.py:46).
"""
import os

import numpy as np

from dropout_hamiltonian_montecarlo_amd._native import HmcxError
from dropout_hamiltonian_montecarlo_amd import h5trace


class multicore_mixin:

    def multicore_sample(self, X_train, y_train, niter=1e4, burnin=1e3, batch_size=20, backend=None,
                         ncores=None):
        """ncores: number of chains (default: the sampler's ``chains``)."""
        if self.model._hmcx_model == 'mlp':
            raise HmcxError("multicore_sample: softmax model only")
        ncores = int(self.chains if ncores is None else ncores)
        if ncores < 1:
            raise ValueError("ncores must be >= 1")
        niter_w, burnin_w = int(niter / ncores), int(burnin / ncores)       # sghmc_multicore.py:94
        rows = list(range(0, X_train.shape[0] - batch_size + 1, batch_size))
        if not rows:
            raise ValueError("batch_size larger than the dataset: no minibatch")
        saved_chains, self.chains = self.chains, ncores
        try:
            data = self._upload_data(X_train, y_train)
            state = self._init_state()
            rng = np.random.RandomState(0)
            eps = [self.step_size] * len(rows)
            for _ in range(burnin_w):
                self._run(state, data, rows, eps, rng, batch_size)
            shapes = {var: self.start[var].shape for var in self.start}
            multi_backend = [backend + "_%i.h5" % i for i in range(ncores)] if backend else None
            writers = [h5trace.TraceFile(f, shapes) for f in multi_backend] if backend else None
            mem = {var: [[] for _ in range(ncores)] for var in self.start} if not backend else None
            logp = np.zeros((ncores, niter_w))
            sizes = [int(np.prod(shapes[v])) for v in self.start]
            offs = np.concatenate([[0], np.cumsum(sizes)])
            self.record_steps = True
            try:
                for i in range(niter_w):
                    res = self._run(state, data, rows, eps, rng, batch_size)
                    steps = res.steps                                        # [n_steps, C, P]
                    for c in range(ncores):
                        for j, var in enumerate(self.start):
                            block = steps[:, c, offs[j]:offs[j + 1]]
                            if writers:
                                writers[c].append(var, block.reshape((-1,) + shapes[var]))
                            else:
                                mem[var][c].append(block.copy())
                        if writers:
                            writers[c].flush()                               # sghmc_multicore.py:52
                    ll_last = np.ravel(res.ll[-1])
                    logp[:, i] = (-1.0 / batch_size) * (ll_last + self._log_prior())
            finally:
                self.record_steps = False
                if writers:
                    for w in writers:
                        w.close()
            self.last_state = state
            logp_samples = logp.reshape(-1)                                  # workers concatenated
            if backend:
                return multi_backend, logp_samples
            posterior = {var: np.concatenate([np.concatenate(mem[var][c], axis=0) if mem[var][c]
                                              else np.zeros((0, sizes[j]))
                                              for c in range(ncores)], axis=0)
                         for j, var in enumerate(self.start)}
            return posterior, logp_samples
        finally:
            self.chains = saved_chains

    def backend_mean(self, multi_backend, niter, ncores=None):
        """cpu/hmc.py:132-138 over the files multicore_sample wrote."""
        return h5trace.backend_mean(self.start, multi_backend, niter)


def _default_philox(kwargs):
    kwargs.setdefault('noise', 'philox')
    return kwargs


def cpu_count():
    return len(os.sched_getaffinity(0))
