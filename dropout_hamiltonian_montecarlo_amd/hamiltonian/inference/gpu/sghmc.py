"""SGHMC sampler — drop-in for hamiltonian/inference/{cpu,gpu}/sghmc.py.

Reference step: /root/reference/hamiltonian/inference/cpu/sghmc.py:19-39, run with the A1
completion: momentum ~ N(0,1) (cpu/hmc.py:82-87), MH accept
A = min(1, exp(E_cur − E_new)) with E = negative_log_posterior + ½Σp² (cpu/hmc.py:67-79),
the ``+ε·∇U`` momentum sign and 2ε noise std (sghmc.py:31,34), no momentum negation, and a
NaN energy difference accepted (Python ``min``).  The dead ``grad(q)`` of sghmc.py:26 is not
executed (it has no effect and consumes no randomness).

The whole trajectory of every step runs inside libhmcx (hmcx_sghmc_run): per leapfrog
iteration one k_fwd + one k_grad launch; the host only prepares the per-step schedule.
"""
import numpy as np
import torch

from dropout_hamiltonian_montecarlo_amd import _native as nat
from dropout_hamiltonian_montecarlo_amd._native import HmcxError, ptr

from .sgmcmc import RunResult, sgmcmc


def _n_iter(path_length):
    """len(np.arange(path_length - 1)) for the float path length of sghmc.py:25,28."""
    if not np.isfinite(path_length):
        raise HmcxError("non-finite path length (step size 0?)")
    return max(0, int(np.ceil(path_length - 1)))


class sghmc(sgmcmc):

    mask_provider = None    # MLP parity hook: f(global_step, n_forwards) -> [n_fwd, 3, B, n_mid] masks

    def _check_vars(self):
        if self.model._hmcx_model == 'mlp':
            from dropout_hamiltonian_montecarlo_amd.hamiltonian.models.gpu.mlp import MLP_PARAM_NAMES
            if sorted(self.start.keys()) != sorted(MLP_PARAM_NAMES):
                raise HmcxError("sghmc(mlp): start_p must hold exactly %s" % (MLP_PARAM_NAMES,))
            if self.chains != 1:
                raise HmcxError("sghmc(mlp): one chain per sampler (chains=1)")
            self._order = [MLP_PARAM_NAMES.index(k) for k in self.start.keys()]
            return
        if self.model._hmcx_model != 'softmax' or list(self.start.keys()) != ['weights', 'bias']:
            raise HmcxError("sghmc: libhmcx implements the softmax model with start_p keys "
                            "['weights', 'bias'] (in that order, sghmc.py:29)")

    # ------------------------------------------------------------------ schedule
    def _schedule(self, n_steps, eps, rng, P):
        """Host-side randomness of n_steps steps, in the reference's draw order.  Arrays are
        [n_steps, C] (step-major) for C = self.chains."""
        C = self.chains
        n_iter = np.empty((n_steps, C), dtype=np.int32)
        u = np.empty((n_steps, C), dtype=np.float64)
        noise_off = np.zeros((n_steps, C), dtype=np.int64)
        chunks = []
        off = 0
        Ls = np.empty((n_steps, C))
        if self.noise == 'philox':
            # per-step path-length and accept uniforms of every chain, all steps in one pass
            g = ((self.global_step + np.arange(n_steps)) & 0xFFFFFFFF)[:, None]
            chain_ids = (self.chain + np.arange(C))[None, :]
            uL = nat.philox_uniforms_chains(self.seed, chain_ids, g, nat.SLOT_PATH)
            Ls[:] = np.ceil(2 * uL * self.path_length / np.asarray(eps, dtype=np.float64)[:, None])
            if not np.all(np.isfinite(Ls)):
                raise HmcxError("non-finite path length (step size 0?)")
            n_iter[:] = np.maximum(0, np.ceil(Ls - 1)).astype(np.int32)
            u[:] = nat.philox_uniforms_chains(self.seed, chain_ids, g, nat.SLOT_ACCEPT)
        for s in range(n_steps):
            e = eps[s]
            if self.noise == 'numpy':
                # sghmc.py:21 momentum (rng) → :25 path length (global np.random) → :31 per-iteration
                # noise rng.normal(0, 2ε) = 2ε·N(0,1) (scaled on the device) → :36 accept uniform.
                # With C > 1 every chain replays the same streams (replicas).
                L = np.ceil(2 * np.random.rand() * self.path_length / e)
                ni = _n_iter(L)
                z = rng.standard_normal(P * (1 + ni))
                chunks.append(z)
                noise_off[s, :] = off
                off += z.size
                Ls[s, :] = L
                n_iter[s, :] = ni
                u[s, :] = np.random.rand()
            if self.trace is not None:
                self.trace.append({'L': float(Ls[s, 0]) if C == 1 else Ls[s].copy(), 'eps': float(e)})
        noise = np.concatenate(chunks) if chunks else None
        return n_iter, u, noise, noise_off

    def _run(self, state, data, rows, eps, rng, batch_size):
        if self.model._hmcx_model == 'mlp':
            return self._run_mlp(state, data, rows, eps, rng, batch_size)
        return self._collect(self._enqueue(state, data, rows, eps, rng, batch_size))

    def _enqueue(self, state, data, rows, eps, rng, batch_size):
        """Prepare the schedule of len(rows) steps and enqueue them (one hmcx_sghmc_run call) without
        waiting: the returned handle is read back by _collect.  A caller may enqueue the next call
        before collecting this one — the state stays on the device and stream order keeps the calls
        in sequence — so the host work of one call overlaps the device work of the previous one."""
        Xd, Yd = data
        W, b = state['weights'], state['bias']
        C = self.chains
        D, K = W.shape[0], W.shape[1] // C
        P = D * K + K
        n_steps = len(rows)
        t0 = len(self.trace) if self.trace is not None else 0
        n_iter, u, noise, noise_off = self._schedule(n_steps, eps, rng, P)
        n_iter, u, noise_off = (np.ascontiguousarray(x.reshape(-1)) for x in (n_iter, u, noise_off))
        dev = self.model.device
        noise_d = torch.from_numpy(noise).to(dev) if noise is not None else None
        out_f = torch.empty(4 * n_steps * C, dtype=torch.float64, device=dev)     # A, ll, E (2)
        out_acc = torch.empty(n_steps * C, dtype=torch.int32, device=dev)
        out_A, out_ll, out_E = out_f[:n_steps * C], out_f[n_steps * C:2 * n_steps * C], out_f[2 * n_steps * C:]
        row0 = np.asarray(rows, dtype=np.int64)
        eps_a = np.asarray(eps, dtype=np.float64)
        a = nat.SamplerArgs()
        a.dtype = self.model.code
        a.B, a.D, a.K, a.C = batch_size, D, K, C
        a.n_steps = n_steps
        a.alpha = self.model.alpha
        a.log_prior = self._log_prior()
        a.X, a.Y = ptr(Xd), ptr(Yd)
        a.row0 = row0.ctypes.data_as(nat.c_i64p)
        a.eps = eps_a.ctypes.data_as(nat.c_dblp)
        a.n_iter = n_iter.ctypes.data_as(nat.c_i32p)
        a.u_accept = u.ctypes.data_as(nat.c_dblp)
        a.noise_mode = nat.NOISE_BUFFER if self.noise == 'numpy' else nat.NOISE_PHILOX
        a.noise = ptr(noise_d)
        a.noise_off = noise_off.ctypes.data_as(nat.c_i64p)
        a.seed, a.chain0, a.step_base = self.seed, self.chain, self.global_step & 0xFFFFFFFF
        a.W, a.b = ptr(W), ptr(b)
        a.out_A, a.out_accepted, a.out_ll, a.out_E = ptr(out_A), ptr(out_acc), ptr(out_ll), ptr(out_E)
        out_steps = None
        if self.record_steps:
            out_steps = torch.empty((n_steps, C, P), dtype=self.model.dtype, device=dev)
            a.out_trace = ptr(out_steps)
        ctx = nat.context(dev)
        ctx.check(ctx.lib.hmcx_sghmc_run(ctx.h, a), "hmcx_sghmc_run")
        self.global_step += n_steps
        return dict(out_f=out_f, out_acc=out_acc, noise_d=noise_d, n_steps=n_steps, C=C, t0=t0, ctx=ctx,
                    out_steps=out_steps)

    def _collect(self, h):
        """Read back one enqueued call (waits for it) and fill the trace entries of its steps."""
        n_steps, C = h['n_steps'], h['C']
        f = h['out_f'].cpu().numpy()
        acc = h['out_acc'].cpu().numpy().astype(bool)
        ctx = h['ctx']
        ctx.check(ctx.lib.hmcx_synchronize(ctx.h), "hmcx_sghmc_run")        # deferred abort check
        nsc = n_steps * C
        A, ll, E = f[:nsc], f[nsc:2 * nsc], f[2 * nsc:]
        steps = h['out_steps'].cpu().numpy() if h.get('out_steps') is not None else None
        if C == 1:
            res = RunResult(A, acc, ll, E.reshape(n_steps, 2), steps=steps)
        else:
            res = RunResult(A.reshape(n_steps, C), acc.reshape(n_steps, C), ll.reshape(n_steps, C),
                            E.reshape(n_steps, C, 2), steps=steps)
        if self.trace is not None:
            for s in range(n_steps):
                t = self.trace[h['t0'] + s]
                t['A'] = float(res.A[s]) if C == 1 else res.A[s].copy()
                t['accepted'] = bool(res.accepted[s]) if C == 1 else res.accepted[s].copy()
        return res

    def _run_mlp(self, state, data, rows, eps, rng, batch_size):
        """MLP steps through hmcx_mlp_sghmc_run (hmcx_mlp.hip): same schedule and noise layout as the
        softmax path; dropout masks from Philox on the device, or from ``mask_provider`` (parity)."""
        from dropout_hamiltonian_montecarlo_amd.hamiltonian.models.gpu.mlp import MLP_PARAM_NAMES
        m = self.model
        Xd, yd = data
        P = sum(int(np.prod(self.start[k].shape)) for k in self.start)
        n_steps = len(rows)
        n_iter, u, noise, noise_off = self._schedule(n_steps, eps, rng, P)
        n_iter, u, noise_off = (np.ascontiguousarray(x.reshape(-1)) for x in (n_iter, u, noise_off))
        dev = m.device
        noise_d = torch.from_numpy(noise).to(dev) if noise is not None else None
        masks_d, mask_off = None, np.zeros(n_steps, dtype=np.int64)
        if self.mask_provider is not None:
            chunks, off = [], 0
            for s in range(n_steps):
                mk = np.asarray(self.mask_provider(self.global_step + s, 6 * int(n_iter[s]) + 2))
                chunks.append(mk.reshape(-1))
                mask_off[s] = off
                off += chunks[-1].size
            masks_d = torch.from_numpy(np.concatenate(chunks)).to(dev, m.dtype)
        outs = {k: torch.empty(n_steps * w, dtype=torch.float64, device=dev)
                for k, w in (('A', 1), ('loss', 1), ('nlp', 1), ('E', 2))}
        out_acc = torch.empty(n_steps, dtype=torch.int32, device=dev)
        row0 = np.asarray(rows, dtype=np.int64)
        eps_a = np.asarray(eps, dtype=np.float64)
        a = nat.MlpSghmcArgs()
        a.dtype = m.code
        a.B, a.n_in, a.n_mid, a.n_out, a.n_steps = batch_size, m.n_in, m.n_mid, m.n_out, n_steps
        for i, v in enumerate(self._order):
            a.order[i] = v
        a.alpha = m.alpha
        a.X, a.y = ptr(Xd), ptr(yd)
        a.row0 = row0.ctypes.data_as(nat.c_i64p)
        a.eps = eps_a.ctypes.data_as(nat.c_dblp)
        a.n_iter = n_iter.ctypes.data_as(nat.c_i32p)
        a.u_accept = u.ctypes.data_as(nat.c_dblp)
        a.noise_mode = nat.NOISE_BUFFER if self.noise == 'numpy' else nat.NOISE_PHILOX
        a.noise = ptr(noise_d)
        a.noise_off = noise_off.ctypes.data_as(nat.c_i64p)
        a.mask_mode = nat.NOISE_BUFFER if masks_d is not None else nat.NOISE_PHILOX
        a.masks = ptr(masks_d)
        a.mask_off = mask_off.ctypes.data_as(nat.c_i64p)
        a.seed, a.chain, a.step_base = self.seed, self.chain, self.global_step & 0xFFFFFFFF
        for i, k in enumerate(MLP_PARAM_NAMES):
            a.par.p[i] = state[k].data_ptr()
        a.out_A, a.out_accepted = ptr(outs['A']), ptr(out_acc)
        a.out_loss, a.out_nlp, a.out_E = ptr(outs['loss']), ptr(outs['nlp']), ptr(outs['E'])
        ctx = nat.context(dev)
        ctx.check(ctx.lib.hmcx_mlp_sghmc_run(ctx.h, a), "hmcx_mlp_sghmc_run")
        self.global_step += n_steps
        h = {k: v.cpu().numpy() for k, v in outs.items()}
        res = RunResult(h['A'], out_acc.cpu().numpy().astype(bool), h['loss'], h['E'].reshape(n_steps, 2),
                        nlp=h['nlp'])
        del noise_d, masks_d
        if self.trace is not None:
            for s in range(n_steps):
                t = self.trace[len(self.trace) - n_steps + s]
                t['A'] = float(res.A[s])
                t['accepted'] = bool(res.accepted[s])
        return res

    # ------------------------------------------------------------------ single step (API parity)
    def step(self, state, momentum, rng, **args):                         # sghmc.py:19-39
        """One SGHMC step on the given minibatch; returns (q, None, acceptprob).

        q is a dict of device tensors.  The final momentum stays on the device (the reference
        returns it but ``sample`` discards it; draw_momentum redraws it every step)."""
        if self.chains != 1:
            raise HmcxError("step() is the reference's single-chain API; use sample() for chains > 1")
        X, y = args['X_train'], args['y_train']
        data = self._upload_data(X, y)
        st = {var: torch.as_tensor(np.asarray(state[var]) if not isinstance(state[var], torch.Tensor)
                                   else state[var]).to(self.model.device, self.model.dtype).contiguous().clone()
              for var in self.start}
        res = self._run(st, data, [0], [self.step_size], rng, data[0].shape[0])
        return st, None, float(res.A[0])
