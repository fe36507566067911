"""SGHMC sampler — drop-in for hamiltonian/inference/{cpu,gpu}/sghmc.py.

Reference step: /root/reference/hamiltonian/inference/cpu/sghmc.py:19-39, run with the A1
completion: momentum ~ N(0,1) (cpu/hmc.py:82-87), MH accept
A = min(1, exp(E_cur − E_new)) with E = negative_log_posterior + ½Σp² (cpu/hmc.py:67-79),
the ``+ε·∇U`` momentum sign and 2ε noise std (sghmc.py:31,34), no momentum negation, and a
NaN energy difference accepted (Python ``min``).  The dead ``grad(q)`` of sghmc.py:26 is not
executed (it has no effect and consumes no randomness).

The whole trajectory of every step runs inside libhmcx (hmcx_sghmc_run): one chain — one
persistent launch per call (csrc/hmcx_persist2.hip); C ≥ 16 chains — the chain-batched GEMMs
(csrc/hmcx_batch.h); otherwise one k_fwd + one k_grad launch per leapfrog iteration.  The host only
prepares the per-step schedule and reads back the per-step scalars.
"""
import os
import time

import numpy as np
import torch

from dropout_hamiltonian_montecarlo_amd import _native as nat
from dropout_hamiltonian_montecarlo_amd._native import HmcxError, ptr

from .sgmcmc import RunResult, sgmcmc


_HOST_PROF = os.environ.get("HMCX_HOST_PROF") == "1"     # phase timestamps of _enqueue (tools/)
_marks = []


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
            # per-step path lengths and accept uniforms of every chain: one host C call
            Ls, n_iter, u = nat.philox_schedule(self.seed, self.chain, C, self.global_step, self.path_length, eps)
            if self.trace is not None:
                if C == 1:
                    self.trace.extend({'L': float(l), 'eps': float(e)} for l, e in zip(Ls[:, 0], eps))
                else:
                    self.trace.extend({'L': Ls[s].copy(), 'eps': float(eps[s])} for s in range(n_steps))
            return n_iter, u, None, noise_off
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

    _IO_SLOTS = 4          # output buffers in rotation (at most two calls are in flight in sample/bench)

    def _io_slot(self, nbytes, dev):
        """A device output buffer and its pinned host mirror, reused round-robin across calls (all
        slots are allocated by the first call, so later calls allocate nothing)."""
        ring = self.__dict__.get('_io_ring')
        if ring is None:
            self._io_ring = ring = [{'dev': None, 'host': None, 'busy': None, 'cap': 0}
                                    for _ in range(self._IO_SLOTS)]
        i = self.__dict__.get('_io_next', 0)
        self._io_next = i + 1
        slot = ring[i % self._IO_SLOTS]
        if slot['busy'] is not None:    # an uncollected call keeps its buffers; the slot gets new ones
            slot.update(dev=None, host=None, busy=None, cap=0)
        if slot['cap'] < nbytes:
            cap = max(1 << 16, 1 << (int(nbytes) - 1).bit_length())
            for sl in ring:                          # busy slots grow when their turn comes
                if sl['busy'] is None and sl['cap'] < cap:
                    sl['dev'] = torch.empty(cap, dtype=torch.uint8, device=dev)
                    sl['host'] = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
                    sl['base'], sl['hptr'], sl['cap'] = sl['dev'].data_ptr(), sl['host'].data_ptr(), cap
                    sl['hnp'] = sl['host'].numpy()
        return slot

    def _call_template(self, Xd, Yd, W, b, batch_size, D, K, C):
        """hmcx_sampler_args fields that stay fixed from call to call (cached per data/state)."""
        key = (Xd.data_ptr(), Yd.data_ptr(), W.data_ptr(), b.data_ptr(), batch_size, C, self.path_length,
               self.seed, self.chain, self.model.alpha)
        tpl = self.__dict__.get('_tpl')
        if tpl is None or tpl[0] != key:
            a = nat.SamplerArgs()
            a.dtype = self.model.code
            a.B, a.D, a.K, a.C = batch_size, D, K, C
            a.alpha = self.model.alpha
            a.log_prior = self._log_prior()
            a.X, a.Y = ptr(Xd), ptr(Yd)
            a.noise_mode = nat.NOISE_BUFFER if self.noise == 'numpy' else nat.NOISE_PHILOX
            a.seed, a.chain0 = self.seed, self.chain
            a.path_length = self.path_length
            a.W, a.b = ptr(W), ptr(b)
            self._tpl = tpl = (key, a)
        return tpl[1]

    def _enqueue(self, state, data, rows, eps, rng, batch_size):
        # the steady state of a Philox-mode sampler (what sample() and bench.py repeat): same data, state
        # and step count as the previous call on this output slot — refill the rows / step sizes and go
        q = self.__dict__.get('_quick')
        if q is not None and not _HOST_PROF and self.noise == 'philox' and not self.record_steps \
                and not self.__dict__.get('_want_mom'):
            h = self._enqueue_quick(q, state, data, rows, eps, batch_size)
            if h is not None:
                return h
        return self._enqueue_full(state, data, rows, eps, rng, batch_size)

    def _enqueue_quick(self, q, state, data, rows, eps, batch_size):
        """The cached fast path of _enqueue_full (same struct, same host arrays, same slot rotation):
        only valid when the data / state tensors, the step count and every sampler setting baked into
        the cached argument struct (batch size, chains, path length, seed, chain id, alpha) are those the
        cache was made for — anything else takes the full path, which rebuilds the struct."""
        n_steps = len(rows)
        W, b = state['weights'], state['bias']
        if (data[0] is not q['X'] or data[1] is not q['Y'] or W is not q['W'] or b is not q['b']
                or self.trace is not None or q['tkey'][4:] != (batch_size, self.chains, self.path_length,
                                                               self.seed, self.chain, self.model.alpha)):
            return None
        ring = self._io_ring
        i = self._io_next
        slot = ring[i % self._IO_SLOTS]
        ac = slot.get('acache')
        if slot['busy'] is not None or ac is None or ac[1] is not slot['dev'] or n_steps > ac[6] \
                or ac[0] != q['tkey'] or 36 * n_steps + 4 > slot['cap']:
            return None
        self._io_next = i + 1
        _, _, a, r0b, epb, Lb, _, last_n = ac
        r0b[:n_steps] = rows
        epb[:n_steps] = eps
        base = slot['base']
        if last_n[0] != n_steps:
            a.n_steps = n_steps
            a.out_A, a.out_ll, a.out_E = base, base + 8 * n_steps, base + 16 * n_steps
            a.out_accepted = base + 32 * n_steps
            last_n[0] = n_steps
        a.out_abort = base + 36 * n_steps
        a.step_base = self.global_step & 0xFFFFFFFF
        ctx = q['ctx']
        ctx.bind_stream()
        ctx.check(ctx.lib.hmcx_sghmc_run(ctx.h, a), "hmcx_sghmc_run")
        self.global_step += n_steps
        h = dict(slot=slot, dev=slot['dev'], host=slot['host'], hnp=slot['hnp'], hptr=slot['hptr'],
                 nbytes=32 * n_steps + 4 * n_steps + 4, n_steps=n_steps, C=1, t0=0, ctx=ctx, out_steps=None,
                 out_mom=None, args=a, keep=(r0b, epb, None, None, None, None, Lb[:n_steps]))
        slot['busy'] = h
        self._inflight.append(h)
        return h

    def _enqueue_full(self, state, data, rows, eps, rng, batch_size):
        """Prepare the schedule of len(rows) steps and enqueue them (one hmcx_sghmc_run call) without
        waiting: the call copies its outputs into a pinned host buffer behind its kernels (out_host,
        stream-ordered) and records an event behind them; _collect waits on that event only (hmcx_host_wait), so a caller may
        enqueue the next call before collecting this one — the state stays on the device, stream
        order keeps the calls in sequence, and the host work of call k+1 overlaps the device work of
        call k."""
        mark = _marks if _HOST_PROF else None
        if mark is not None:
            mark.append(('start', time.perf_counter()))
        Xd, Yd = data
        W, b = state['weights'], state['bias']
        C = self.chains
        D, K = W.shape[0], W.shape[1] // C
        P = D * K + K
        n_steps = len(rows)
        t0 = len(self.trace) if self.trace is not None else 0
        nsc = n_steps * C
        philox = self.noise == 'philox'
        if philox:                      # the C call draws the Philox schedule itself (out_L: the L's)
            L_out = n_iter = u = noise = noise_off = None
        else:
            n_iter, u, noise, noise_off = self._schedule(n_steps, eps, rng, P)
            n_iter, u, noise_off = (np.ascontiguousarray(x.reshape(-1)) for x in (n_iter, u, noise_off))
        if mark is not None:
            mark.append(('schedule', time.perf_counter()))
        dev = self.model.device
        noise_d = torch.from_numpy(noise).to(dev) if noise is not None else None
        nbytes = 32 * nsc + 4 * nsc + 4                  # A, ll, E (2) f64 | accepted i32 | abort i32
        slot = self._io_slot(nbytes, dev)
        base = slot['base']
        if mark is not None:
            mark.append(('io slot', time.perf_counter()))
        fast = philox and not self.record_steps and not self.__dict__.get('_want_mom')
        if fast:
            # every slot keeps an argument struct and host schedule arrays (sized for up to `cap` steps)
            # between calls: a call only refills the step rows / sizes, the step count and the output
            # offsets.  A miss rebuilds the caches of ALL slots at once, so the first call on each slot
            # (and a call with a new step count) costs no more than the others.
            tkey = (Xd.data_ptr(), Yd.data_ptr(), W.data_ptr(), b.data_ptr(), batch_size, C, self.path_length,
                    self.seed, self.chain, self.model.alpha)
            ac = slot.get('acache')
            if ac is None or ac[0] != tkey or ac[1] is not slot['dev'] or n_steps > ac[6]:
                cap = max(128, 1 << (n_steps - 1).bit_length())
                tpl = self._call_template(Xd, Yd, W, b, batch_size, D, K, C)
                for sl in self._io_ring:
                    if sl['dev'] is None or (sl is not slot and sl['busy'] is not None):
                        continue
                    a = nat.SamplerArgs.from_buffer_copy(tpl)
                    r0b, epb, Lb = np.empty(cap, np.int64), np.empty(cap), np.empty(cap * C)
                    a.row0, a.eps, a.out_L = nat.addr(r0b), nat.addr(epb), nat.addr(Lb)
                    a.out_host = sl['hptr']
                    sl['acache'] = (tkey, sl['dev'], a, r0b, epb, Lb, cap, [0])
                ac = slot['acache']
            _, _, a, r0b, epb, Lb, _, last_n = ac
            row0, eps_a, L_out = r0b[:n_steps], epb[:n_steps], Lb[:nsc]
            row0[:] = rows
            eps_a[:] = eps
            if last_n[0] != n_steps:
                a.n_steps = n_steps
                a.out_A, a.out_ll, a.out_E = base, base + 8 * nsc, base + 16 * nsc
                a.out_accepted = base + 32 * nsc
                last_n[0] = n_steps
            a.out_abort = base + 36 * nsc
        else:
            if philox:                  # the C call draws the Philox schedule itself (out_L: the L's)
                L_out = np.empty(nsc)
            row0 = np.asarray(rows, dtype=np.int64)
            eps_a = np.asarray(eps, dtype=np.float64)
            a = nat.SamplerArgs.from_buffer_copy(self._call_template(Xd, Yd, W, b, batch_size, D, K, C))
            a.n_steps = n_steps
            a.row0 = nat.addr(row0)
            a.eps = nat.addr(eps_a)
            if philox:
                a.out_L = nat.addr(L_out)
            else:
                a.n_iter = nat.addr(n_iter)
                a.u_accept = nat.addr(u)
                a.noise = ptr(noise_d)
                a.noise_off = nat.addr(noise_off)
            a.out_A, a.out_ll, a.out_E = base, base + 8 * nsc, base + 16 * nsc
            a.out_accepted, a.out_abort = base + 32 * nsc, base + 36 * nsc
            a.out_host = slot['hptr']                 # outputs + abort word land here (include/hmcx.h)
        if mark is not None:
            mark.append(('template', time.perf_counter()))
        a.step_base = self.global_step & 0xFFFFFFFF
        out_steps = None
        if self.record_steps:
            out_steps = torch.empty((n_steps, C, P), dtype=self.model.dtype, device=dev)
            a.out_trace = ptr(out_steps)
        out_mom = None
        if self.__dict__.get('_want_mom'):
            out_mom = torch.empty((C, P), dtype=self.model.dtype, device=dev)
            a.out_mom = ptr(out_mom)
        if mark is not None:
            mark.append(('args', time.perf_counter()))
        cc = self.__dict__.get('_ctx_of')
        if cc is None or cc[0] != dev:
            self._ctx_of = cc = (dev, nat.context(dev))
        ctx = cc[1]
        ctx.bind_stream()                              # follow torch's current stream
        if mark is not None:
            mark.append(('context', time.perf_counter()))
        ctx.check(ctx.lib.hmcx_sghmc_run(ctx.h, a), "hmcx_sghmc_run")     # records the out_host event
        if mark is not None:
            mark.append(('c call', time.perf_counter()))
        if philox and self.trace is not None:                 # while the launch runs
            if C == 1:
                self.trace += [{'L': l, 'eps': float(e)} for l, e in zip(L_out.tolist(), eps)]
            else:
                Ls = L_out.reshape(n_steps, C)
                self.trace.extend({'L': Ls[i].copy(), 'eps': float(eps[i])} for i in range(n_steps))
        self.global_step += n_steps
        h = dict(slot=slot, dev=slot['dev'], host=slot['host'], hnp=slot['hnp'], hptr=slot['hptr'], nbytes=nbytes,
                 n_steps=n_steps,
                 C=C, t0=t0, ctx=ctx, out_steps=out_steps, out_mom=out_mom,
                 args=a, keep=(row0, eps_a, n_iter, u, noise_off, noise_d, L_out if philox else None))
        slot['busy'] = h
        self.__dict__.setdefault('_inflight', []).append(h)
        if fast and C == 1 and out_steps is None and out_mom is None:
            self._quick = dict(X=Xd, Y=Yd, W=W, b=b, ctx=ctx,
                               tkey=tkey)
        return h

    def _collect(self, h):
        """Wait for one enqueued call (its own event, not the stream) and read its outputs; a call
        whose persistent launch timed out is re-run first (_recover)."""
        n_steps, C = h['n_steps'], h['C']
        slot = h['slot']
        ctx = h['ctx']
        ctx.check(ctx.lib.hmcx_host_wait(ctx.h, h['hptr']), "hmcx_host_wait")
        nsc = n_steps * C
        raw = h['hnp'][:h['nbytes']]
        if raw[36 * nsc:36 * nsc + 4].view(np.int32)[0] and not h.get('recovered'):
            self._recover(h)
        raw = raw.copy()
        if slot['busy'] is h:
            slot['busy'] = None
        self._inflight.remove(h)
        f = raw[:32 * nsc].view(np.float64)
        acc = raw[32 * nsc:36 * nsc].view(np.int32).astype(bool)
        A, ll, E = f[:nsc], f[nsc:2 * nsc], f[2 * nsc:]
        steps = h['out_steps'].cpu().numpy() if h.get('out_steps') is not None else None
        if C == 1:
            res = RunResult(A, acc, ll, E.reshape(n_steps, 2), steps=steps)
        else:
            res = RunResult(A.reshape(n_steps, C), acc.reshape(n_steps, C), ll.reshape(n_steps, C),
                            E.reshape(n_steps, C, 2), steps=steps)
        res.mom = h.get('out_mom')
        Lk = h['keep'][-1]
        if Lk is not None:                       # Philox: the path lengths the C call drew
            res.L = Lk[:nsc].copy() if C == 1 else Lk[:nsc].reshape(n_steps, C).copy()
        if self.trace is not None:
            t0 = h['t0']
            if C == 1:                       # Python floats / bools straight from tolist()
                for t, a_, c_, e_ in zip(self.trace[t0:t0 + n_steps], A.tolist(), acc.tolist(), res.E.tolist()):
                    t['A'] = a_
                    t['accepted'] = c_
                    t['E'] = e_                      # (E_current, E_new) of the accept test
            else:
                for s in range(n_steps):
                    t = self.trace[t0 + s]
                    t['A'] = res.A[s].copy()
                    t['accepted'] = res.accepted[s].copy()
                    t['E'] = res.E[s].copy()
        return res

    def _recover(self, h):
        """The persistent launch of call h timed out in a hand-off (include/hmcx.h hmcx_clear_abort):
        it, and every call enqueued after it, left W/b untouched.  Lower the abort word and re-run
        those calls in order, in this process, on the kernel-per-phase path — same schedule, same
        noise, so the results are those the persistent kernel would have produced.  The context
        stays on that path afterwards (a misplacement that happened once is likely to recur)."""
        import sys
        ctx = h['ctx']
        torch.cuda.synchronize()
        ctx.clear_abort()
        print("hmcx: persistent SGHMC hand-off timed out; re-running %d call(s) on the kernel-per-phase "
              "path" % (len(self._inflight) - self._inflight.index(h)), file=sys.stderr)
        ctx.set_sghmc_path(1)
        for x in self._inflight[self._inflight.index(h):]:
            a = x['args']
            a.out_abort = None
            ctx.check(ctx.lib.hmcx_sghmc_run(ctx.h, a), "hmcx_sghmc_run (recovery)")
            ctx.note_recovery("persistent_sghmc")                  # one per re-run call (hmcx_get_recoveries)
            x['host'][:x['nbytes']].copy_(x['dev'][:x['nbytes']])
            x['host'][36 * x['n_steps'] * x['C']:x['nbytes']].zero_()
            x['recovered'] = True
        torch.cuda.synchronize()

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
        out_abort = torch.zeros(1, dtype=torch.int32, device=dev)
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
        a.out_abort = ptr(out_abort)
        ctx = nat.context(dev)
        # the state before the call: a call whose fused exchange timed out leaves it invalid (below)
        saved = [state[k].clone() for k in MLP_PARAM_NAMES] if ctx.mlp_fuse else None
        ctx.check(ctx.lib.hmcx_mlp_sghmc_run(ctx.h, a), "hmcx_mlp_sghmc_run")
        if saved is not None and int(out_abort.item()):
            # a fused layer-2/3 launch timed out in its exchange (include/hmcx.h out_abort): restore the
            # state and re-run the call unfused — same schedule, noise and masks, so the results are
            # those the fused launches would have given; the context stays unfused afterwards
            import sys
            print("hmcx: fused MLP layer-2/3 exchange timed out; re-running the call unfused", file=sys.stderr)
            for k, t in zip(MLP_PARAM_NAMES, saved):
                state[k].copy_(t)
            ctx.set_mlp_fuse(False)
            ctx.note_recovery("mlp_fused")
            ctx.check(ctx.lib.hmcx_mlp_sghmc_run(ctx.h, a), "hmcx_mlp_sghmc_run (unfused re-run)")
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
        """One SGHMC step on the given minibatch; returns (q, p, acceptprob) like the reference:
        q and p are dicts of device tensors — p is the final momentum when the proposal was
        accepted, else the momentum drawn at the start of the step (sghmc.py:36-39; the argument
        `momentum` is ignored there too, the step draws its own)."""
        if self.chains != 1:
            raise HmcxError("step() is the reference's single-chain API; use sample() for chains > 1")
        X, y = args['X_train'], args['y_train']
        data = self._upload_data(X, y)
        st = {var: torch.as_tensor(np.asarray(state[var]) if not isinstance(state[var], torch.Tensor)
                                   else state[var]).to(self.model.device, self.model.dtype).contiguous().clone()
              for var in self.start}
        self._want_mom = True
        try:
            res = self._run(st, data, [0], [self.step_size], rng, data[0].shape[0])
        finally:
            self._want_mom = False
        W = st['weights']
        D, K = W.shape
        mom = res.mom.reshape(-1)
        p = {'weights': mom[:D * K].reshape(D, K), 'bias': mom[D * K:]}
        return st, p, float(res.A[0])
