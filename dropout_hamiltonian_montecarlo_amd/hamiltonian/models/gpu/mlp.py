"""HIP-backed dropout MLP — drop-in for the reference's Chainer MLP (config 3).

Reference: /root/reference/hamiltonian/models/gpu/mlp.py:19-96.  ``MyNetwork`` (:19-31) is
l1 (n_in→n_mid) → dropout(.1) → relu → l2 (n_mid→n_mid) → dropout → relu → dropout → l3
(n_mid→n_out); ``grad`` (:47-64) returns ∇ mean softmax-CE + ½α·θ per parameter,
``log_likelihood`` (:66-78) returns the mean CE *loss*, ``log_prior`` (:40-45) is
−Σ_var ½α·Σθ²/dim and ``negative_log_posterior`` (:80-82) is loss + log_prior.

Parameters use Chainer's ``namedparams`` names and [out, in] weight layout ('/l1/W' [n_mid, n_in],
'/l1/b', '/l2/W', '/l2/b', '/l3/W' [n_out, n_mid], '/l3/b').  Labels are integers (mlp.py:52).
Every compute call goes through libhmcx (k_mm MFMA GEMMs with fused bias/dropout/relu/gradient
epilogues, hmcx_mlp.hip).

Dropout.  Chainer draws fresh masks on every forward (train mode).  Here ``masks=None`` draws them
on the device from Philox (hmcx_mlp_masks, keyed by the model's seed and a call counter);
``masks='off'`` disables dropout; an explicit ``masks=[m1, m2, m3]`` (each [B, n_mid]) injects
them — the parity mode against oracle/models.py::mlp.
"""
import ctypes

import numpy as np
import torch

from dropout_hamiltonian_montecarlo_amd._native import (HmcxError, MlpLeapfrogArgs, MlpParams, MLP_MASK_SLOT0,
                                                        MLP_MASKS_FIXED, MLP_MASKS_NONE, MLP_MASKS_PHILOX, context,
                                                        dtype_code, ptr)

from .softmax import _batch, as_device

MLP_PARAM_NAMES = ('/l1/W', '/l1/b', '/l2/W', '/l2/b', '/l3/W', '/l3/b')


def mlp_param_shapes(n_in, n_mid, n_out):
    return {'/l1/W': (n_mid, n_in), '/l1/b': (n_mid,), '/l2/W': (n_mid, n_mid), '/l2/b': (n_mid,),
            '/l3/W': (n_out, n_mid), '/l3/b': (n_out,)}


def init_params(shape, seed=0):
    """Chainer L.Linear defaults for MyNetwork(n_in, n_mid, n_out): W ~ LeCunNormal (N(0, 1/fan_in)),
    b = 0 (host numpy, float64).  Needs no device."""
    shapes = mlp_param_shapes(*shape)
    rs = np.random.RandomState(seed)
    out = {}
    for k in MLP_PARAM_NAMES:
        shp = shapes[k]
        out[k] = rs.normal(0, 1.0 / np.sqrt(shp[1]), shp) if len(shp) == 2 else np.zeros(shp)
    return out


class mlp:
    _hmcx_model = 'mlp'

    def __init__(self, _hyper, n_in, n_mid_units, n_out, dtype=torch.float32, device=None, seed=0):
        self.hyper = _hyper
        self.alpha = float(np.asarray(_hyper['alpha']))
        self.n_in, self.n_mid, self.n_out = int(n_in), int(n_mid_units), int(n_out)
        self.dtype = dtype
        self.code = dtype_code(dtype)
        self.ctx = context(device)
        self.device = self.ctx.device
        self.seed = int(seed)
        self._mask_calls = 0
        self.shapes = mlp_param_shapes(self.n_in, self.n_mid, self.n_out)

    # -------------------------------------------------------------- helpers
    def init_params(self, seed=0):
        """Chainer L.Linear defaults: W ~ LeCunNormal (N(0, 1/fan_in)), b = 0 (host numpy, float64)."""
        return init_params((self.n_in, self.n_mid, self.n_out), seed)

    def _dev(self, a):
        return as_device(a, self.dtype, self.device)

    def _params(self, par):
        ts = []
        for k in MLP_PARAM_NAMES:
            if k not in par:
                raise HmcxError("mlp: missing parameter %r (expected %s)" % (k, MLP_PARAM_NAMES))
            t = self._dev(par[k])
            if tuple(t.shape) != self.shapes[k]:
                raise HmcxError("mlp: %s has shape %s, expected %s" % (k, tuple(t.shape), self.shapes[k]))
            ts.append(t)
        mp = MlpParams()
        for i, t in enumerate(ts):
            mp.p[i] = t.data_ptr()
        return ts, mp

    def _xy(self, args, need_y=True):
        X, y = _batch(args)
        X = self._dev(X)
        if X.dim() != 2 or X.shape[1] != self.n_in:
            raise HmcxError("mlp: X_train must be [B, %d]" % self.n_in)
        if not need_y:
            return X, None
        yt = y if isinstance(y, torch.Tensor) else torch.as_tensor(np.asarray(y))
        yt = yt.to(self.device, torch.int32).contiguous()
        if yt.dim() != 1 or yt.shape[0] != X.shape[0]:
            raise HmcxError("mlp: y_train must be integer labels [B] (mlp.py:52)")
        return X, yt

    def draw_masks(self, B):
        """Fresh Philox dropout masks [3, B, n_mid] on the device (one forward's worth)."""
        out = torch.empty((3, B, self.n_mid), dtype=self.dtype, device=self.device)
        slot = (MLP_MASK_SLOT0 + self._mask_calls) & 0xFFFFFFFF
        self._mask_calls += 1
        ctx = context(self.device)
        ctx.check(ctx.lib.hmcx_mlp_masks(ctx.h, self.code, B, self.n_mid, self.seed, 0, 0xFFFFFFFF, slot, ptr(out)),
                  "hmcx_mlp_masks")
        return out

    def _masks(self, masks, B):
        if masks is None:
            return self.draw_masks(B)
        if isinstance(masks, str):
            if masks != 'off':
                raise ValueError("masks must be None, 'off' or [m1, m2, m3]")
            return None
        m = torch.stack([self._dev(x) for x in masks]) if isinstance(masks, (list, tuple)) else self._dev(masks)
        if tuple(m.shape) != (3, B, self.n_mid):
            raise HmcxError("mlp: masks must be 3 x [B, n_mid]")
        return m.contiguous()

    # -------------------------------------------------------------- model surface
    def grad(self, par, masks=None, **args):                              # mlp.py:47-64
        X, y = self._xy(args)
        B = X.shape[0]
        ts, mp = self._params(par)
        m = self._masks(masks, B)
        gs = [torch.empty_like(t) for t in ts]
        gp = MlpParams()
        for i, g in enumerate(gs):
            gp.p[i] = g.data_ptr()
        ctx = context(self.device)
        ctx.check(ctx.lib.hmcx_mlp_grad(ctx.h, self.code, ptr(X), ptr(y), B, self.n_in, self.n_mid, self.n_out, mp,
                                        ptr(m), self.alpha, gp, None), "hmcx_mlp_grad")
        return {k: g for k, g in zip(MLP_PARAM_NAMES, gs)}

    def leapfrog_device_ok(self):
        """hmc.step may hand the whole trajectory to leapfrog_device only when grad is this class's own
        (a subclass that overrides grad, e.g. to inject masks per call, keeps the host loop)."""
        return type(self).grad is mlp.grad

    def leapfrog_device(self, q, p, n_iter, eps, keys, masks=None, **args):
        """hmc.py:46-56 for the MLP in one libhmcx call (hmcx_mlp_hmc_leapfrog): q and p (dicts of device
        tensors of the model's dtype, keyed in the sampler's start order `keys`) are advanced in place
        and p is negated at the end.  The 1 + 6·n_iter gradient calls take their masks as grad() would:
        masks=None draws fresh Philox masks per call (the same slots as that many grad() calls),
        'off' disables dropout, explicit masks are used by every call.  Returns the gradient at the
        final position."""
        X, y = self._xy(args)
        B = X.shape[0]
        order = [MLP_PARAM_NAMES.index(k) for k in keys]
        if sorted(order) != list(range(6)):
            raise HmcxError("mlp: leapfrog keys must be the six parameters, got %s" % (list(keys),))
        a = MlpLeapfrogArgs()
        a.dtype, a.B, a.n_in, a.n_mid, a.n_out, a.n_iter = self.code, B, self.n_in, self.n_mid, self.n_out, int(n_iter)
        for i, v in enumerate(order):
            a.order[i] = v
        a.eps, a.alpha = float(eps), self.alpha
        a.X, a.y = X.data_ptr(), y.data_ptr()
        gs = {}
        for k in MLP_PARAM_NAMES:
            for t in (q[k], p[k]):
                if not (isinstance(t, torch.Tensor) and t.device == self.device and t.dtype == self.dtype
                        and t.is_contiguous() and tuple(t.shape) == self.shapes[k]):
                    raise HmcxError("mlp: leapfrog state %s must be a contiguous %s device tensor of shape %s"
                                    % (k, self.dtype, self.shapes[k]))
            i = MLP_PARAM_NAMES.index(k)
            gs[k] = torch.empty_like(q[k])
            a.q.p[i], a.p.p[i], a.g.p[i] = q[k].data_ptr(), p[k].data_ptr(), gs[k].data_ptr()
        keep = None
        if masks is None:
            keep = torch.empty((3, B, self.n_mid), dtype=self.dtype, device=self.device)
            a.mask_mode, a.masks = MLP_MASKS_PHILOX, keep.data_ptr()
            a.seed, a.chain, a.step = self.seed, 0, 0xFFFFFFFF
            a.slot0 = (MLP_MASK_SLOT0 + self._mask_calls) & 0xFFFFFFFF
            self._mask_calls += 1 + 6 * int(n_iter)
        else:
            keep = self._masks(masks, B)
            a.mask_mode = MLP_MASKS_NONE if keep is None else MLP_MASKS_FIXED
            a.masks = None if keep is None else keep.data_ptr()
        ctx = context(self.device)
        ctx.check(ctx.lib.hmcx_mlp_hmc_leapfrog(ctx.h, ctypes.byref(a)), "hmcx_mlp_hmc_leapfrog")
        del keep                                        # stream-ordered: the allocator reuses it after the launches
        return gs

    def loss_device(self, par, masks=None, **args):
        X, y = self._xy(args)
        B = X.shape[0]
        _, mp = self._params(par)
        m = self._masks(masks, B)
        out = torch.empty(1, dtype=torch.float64, device=self.device)
        ctx = context(self.device)
        ctx.check(ctx.lib.hmcx_mlp_loss(ctx.h, self.code, ptr(X), ptr(y), B, self.n_in, self.n_mid, self.n_out, mp,
                                        ptr(m), ptr(out), None), "hmcx_mlp_loss")
        return out

    def log_likelihood(self, par, masks=None, **args):                    # mlp.py:66-78 (returns the loss)
        return np.float64(self.loss_device(par, masks=masks, **args).item())

    def log_prior(self, par, **args):                                     # mlp.py:40-45
        """−Σ_var ½·alpha·Σθ²/dim, with Σθ² a float64 device reduction (hmcx_sumsq)."""
        ctx = context(self.device)
        ss = torch.empty(len(par), dtype=torch.float64, device=self.device)
        keep = []
        for i, var in enumerate(par.keys()):
            v = self._dev(par[var]).contiguous()
            keep.append(v)
            ctx.check(ctx.lib.hmcx_sumsq(ctx.h, self.code, ptr(v), v.numel(), ptr(ss[i:i + 1])), "hmcx_sumsq")
        sums = ss.cpu().numpy()
        K = 0.0
        for v, s2 in zip(keep, sums):
            K -= 0.5 * self.alpha * float(s2) / v.numel()
        return K

    def negative_log_posterior(self, par, masks=None, **args):           # mlp.py:80-82
        return self.log_likelihood(par, masks=masks, **args) + self.log_prior(par, **args)

    def energy_parts_device(self, par, out, masks=None, **args):
        """The device pieces of negative_log_posterior without a readback: out[0] = the loss
        (log_likelihood), out[1 + i] = Σθ² of the i-th variable of par.  nlp_from_parts adds them up on
        the host exactly as negative_log_posterior does, so a sampler can enqueue several energies and
        read them back once.  Returns the device tensors the launches read (keep them until then)."""
        X, y = self._xy(args)
        B = X.shape[0]
        _, mp = self._params(par)
        m = self._masks(masks, B)
        ctx = context(self.device)
        ctx.check(ctx.lib.hmcx_mlp_loss(ctx.h, self.code, ptr(X), ptr(y), B, self.n_in, self.n_mid, self.n_out, mp,
                                        ptr(m), ptr(out[0:1]), None), "hmcx_mlp_loss")
        keep = [m]
        for i, var in enumerate(par.keys()):
            v = self._dev(par[var]).contiguous()
            keep.append(v)
            ctx.check(ctx.lib.hmcx_sumsq(ctx.h, self.code, ptr(v), v.numel(), ptr(out[1 + i:2 + i])), "hmcx_sumsq")
        return keep

    def nlp_from_parts(self, parts, par):
        """negative_log_posterior from energy_parts_device's values (same float64 operations, same order)."""
        ll = np.float64(parts[0])
        K = 0.0
        for i, var in enumerate(par.keys()):
            K -= 0.5 * self.alpha * float(parts[1 + i]) / int(np.prod(np.shape(par[var])))
        return ll + K

    def loss(self, par, masks=None, **args):
        """North-star surface name: the sampler energy U = negative_log_posterior."""
        return self.negative_log_posterior(par, masks=masks, **args)

    def logits(self, par, X, masks='off'):
        X = self._dev(X)
        B = X.shape[0]
        _, mp = self._params(par)
        m = self._masks(masks, B)
        z = torch.empty((B, self.n_out), dtype=self.dtype, device=self.device)
        ctx = context(self.device)
        ctx.check(ctx.lib.hmcx_mlp_loss(ctx.h, self.code, ptr(X), None, B, self.n_in, self.n_mid, self.n_out, mp,
                                        ptr(m), None, ptr(z)), "hmcx_mlp_loss")
        return z

    def predict(self, par, X_test, prob=False, masks=None):              # mlp.py:84-96
        """Chainer runs the net in train mode here too, so dropout is on by default (masks=None);
        pass masks='off' for the deterministic network."""
        z = self.logits(par, X_test, masks=masks).cpu().numpy()
        if prob:                                                          # F.softmax on the host (:92)
            e = np.exp(z - z.max(axis=1, keepdims=True))
            return e / e.sum(axis=1, keepdims=True)
        return z.argmax(axis=1)
