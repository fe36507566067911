"""SGLD sampler — drop-in for hamiltonian/inference/cpu/sgld.py.

Reference step: /root/reference/hamiltonian/inference/cpu/sgld.py:31-46:
    p = N(0, (2ε)²)  (draw_momentum, noise_scale = 2ε);  p += −½ε·∇U(q);  q += p.
The CuPy file's variant (gpu/sgld.py:11-20) is the named mode ``variant='gpu'``:
p = ν⊙p_prev − ½ε∇U(q) with ν ~ N(0, (2ε)²) and p carried from step to step (zeros at the start
of ``sample``, gpu/sgmcmc.py:48), q += p.  The momentum lives on the device next to the state
(hmcx_sampler_args.pW/pb); the kernels fuse the extra multiply and store.  Default
``variant='cpu'``: the NumPy semantics, the parity target.

One SGLD step = one k_fwd + one k_grad launch (hmcx_sgld_run); the log-likelihood the
reference prints every 10 minibatches costs one extra forward launch on those steps only.
"""
import numpy as np
import torch

from dropout_hamiltonian_montecarlo_amd import _native as nat
from dropout_hamiltonian_montecarlo_amd._native import HmcxError, ptr

from .sgmcmc import RunResult, sgmcmc


class sgld(sgmcmc):

    def __init__(self, model, start_p, path_length=1.0, step_size=0.1, verbose=True,
                 noise='numpy', seed=0, chain=0, chains=1, variant='cpu'):
        if variant not in ('cpu', 'gpu'):
            raise ValueError("variant must be 'cpu' (cpu/sgld.py) or 'gpu' (gpu/sgld.py)")
        self.variant = variant
        self._mom = None
        super().__init__(model, start_p, path_length=path_length, step_size=step_size, verbose=verbose,
                         noise=noise, seed=seed, chain=chain, chains=chains)

    def sample(self, epochs=1, burnin=1, batch_size=1, rng=None, **args):
        self._mom = None                       # p = zeros (gpu/sgmcmc.py:48)
        return super().sample(epochs=epochs, burnin=burnin, batch_size=batch_size, rng=rng, **args)

    def _momentum(self, state):
        if self._mom is None or any(self._mom[v].shape != state[v].shape for v in state):
            self._mom = {v: torch.zeros_like(state[v]) for v in state}
        return self._mom

    def _check_vars(self):
        if self.model._hmcx_model != 'softmax' or list(self.start.keys()) != ['weights', 'bias']:
            raise HmcxError("sgld: libhmcx implements the softmax model with start_p keys ['weights', 'bias']")

    def _run(self, state, data, rows, eps, rng, batch_size):
        Xd, Yd = data
        W, b = state['weights'], state['bias']
        C = self.chains
        D, K = W.shape[0], W.shape[1] // C
        P = D * K + K
        n_steps = len(rows)
        dev = self.model.device
        # noise offsets [n_steps, C]; numpy mode: every chain replays the same stream (replicas)
        noise_off = np.repeat(np.arange(n_steps, dtype=np.int64) * P, C)
        noise_d = None
        if self.noise == 'numpy':
            # sgld.py:45: rng.normal(0, 2ε, shape) per var = 2ε·N(0,1) (scaled on the device)
            noise_d = torch.from_numpy(rng.standard_normal(P * n_steps)).to(dev)
        want = np.zeros(n_steps, dtype=np.uint8)
        want[::self.log_every] = 1
        want[-1] = 1
        out_ll = torch.zeros(n_steps * C, dtype=torch.float64, device=dev)
        row0 = np.asarray(rows, dtype=np.int64)
        eps_a = np.asarray(eps, dtype=np.float64)
        a = nat.SamplerArgs()
        a.dtype = self.model.code
        a.B, a.D, a.K, a.C = batch_size, D, K, C
        a.n_steps = n_steps
        a.alpha = self.model.alpha
        a.log_prior = self._log_prior()
        a.X, a.Y = ptr(Xd), ptr(Yd)
        a.row0 = nat.addr(row0)
        a.eps = nat.addr(eps_a)
        a.want_ll = nat.addr(want)
        a.noise_mode = nat.NOISE_BUFFER if self.noise == 'numpy' else nat.NOISE_PHILOX
        a.noise = ptr(noise_d)
        a.noise_off = nat.addr(noise_off)
        a.seed, a.chain0, a.step_base = self.seed, self.chain, self.global_step & 0xFFFFFFFF
        a.W, a.b = ptr(W), ptr(b)
        if self.variant == 'gpu':
            mom = self._momentum(state)
            a.pW, a.pb = ptr(mom['weights']), ptr(mom['bias'])
        a.out_ll = ptr(out_ll)
        out_steps = None
        if self.record_steps:
            out_steps = torch.empty((n_steps, C, P), dtype=self.model.dtype, device=dev)
            a.out_trace = ptr(out_steps)
        ctx = nat.context(dev)
        # the call's verdict (include/hmcx.h out_abort): a fused wide-SGLD call that timed out in a team
        # round leaves W / b invalid; the start state is kept here and the call re-run on the three
        # launches — same noise, same result — so the call itself never waits for its stream
        out_abort = torch.zeros(1, dtype=torch.int32, device=dev)
        a.out_abort = ptr(out_abort)
        saved = [t.clone() for t in ((W, b) if self.variant != 'gpu' else (W, b, mom['weights'], mom['bias']))]
        ctx.check(ctx.lib.hmcx_sgld_run(ctx.h, a), "hmcx_sgld_run")
        ll = out_ll.cpu().numpy()
        if int(out_abort.item()):
            import sys
            print("[hmcx] wide SGLD: a team round timed out; call re-run on the three-launch path", file=sys.stderr)
            for t, s0 in zip((W, b) if self.variant != 'gpu' else (W, b, mom['weights'], mom['bias']), saved):
                t.copy_(s0)
            ctx.set_sgld_fuse(False)
            try:
                ctx.check(ctx.lib.hmcx_sgld_run(ctx.h, a), "hmcx_sgld_run (unfused re-run)")
            finally:
                ctx.set_sgld_fuse(True)
            ctx.note_recovery("sgld_wide_fused")
            ll = out_ll.cpu().numpy()
        del saved
        self.global_step += n_steps
        if C > 1:
            ll = ll.reshape(n_steps, C)
        if self.trace is not None:
            self.trace.extend({'L': 1.0, 'A': 1.0, 'accepted': True, 'eps': float(e)} for e in eps)
        return RunResult(np.ones(n_steps), np.ones(n_steps, dtype=bool), ll,
                         steps=out_steps.cpu().numpy() if out_steps is not None else None)

    def step(self, state, momentum, rng, **args):                         # sgld.py:31-39
        """variant='cpu': returns (q, None) — the drawn momentum is not part of the result the
        reference's loop uses.  variant='gpu' (gpu/sgld.py:11-20): ``momentum`` is p_prev (None =
        zeros) and (q, p) is returned."""
        if self.chains != 1:
            raise HmcxError("step() is the reference's single-chain API; use sample() for chains > 1")
        X, y = args['X_train'], args['y_train']
        data = self._upload_data(X, y)
        dev, dt = self.model.device, self.model.dtype

        def dev_copy(v):
            return torch.as_tensor(np.asarray(v) if not isinstance(v, torch.Tensor) else v) \
                .to(dev, dt).contiguous().clone()

        st = {var: dev_copy(state[var]) for var in self.start}
        if self.variant == 'gpu':
            self._mom = {var: (dev_copy(momentum[var]).reshape(st[var].shape) if momentum is not None
                               else torch.zeros_like(st[var])) for var in self.start}
        self._run(st, data, [0], [self.step_size], rng, data[0].shape[0])
        return st, (self._mom if self.variant == 'gpu' else None)
