"""ctypes binding of libhmcx.so (include/hmcx.h).

The HIP library is the only compute path of this package: if it is missing or no
HIP device is visible, every entry point raises — there is no CPU fallback.
torch is imported first so that the process has exactly one HIP runtime (torch's
libamdhip64.so.7 satisfies libhmcx.so's NEEDED entry by soname).
"""
import atexit
import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", os.environ.get("HMCX_LIB", "libhmcx.so"))   # HMCX_LIB: A/B builds

HMCX_F32, HMCX_F64 = 0, 1
NOISE_BUFFER, NOISE_PHILOX = 0, 1

c_int, c_double, c_void_p = ctypes.c_int, ctypes.c_double, ctypes.c_void_p
c_i64p = ctypes.POINTER(ctypes.c_int64)
c_i32p = ctypes.POINTER(ctypes.c_int32)
c_dblp = ctypes.POINTER(ctypes.c_double)
c_u8p = ctypes.POINTER(ctypes.c_uint8)


class SamplerArgs(ctypes.Structure):
    # host-array fields are plain addresses here (same layout as the typed pointers of include/hmcx.h):
    # assigning addr(ndarray) costs far less than ndarray.ctypes.data_as on the per-call path
    _fields_ = [("dtype", c_int), ("B", c_int), ("D", c_int), ("K", c_int), ("C", c_int),
                ("n_steps", c_int), ("alpha", c_double), ("log_prior", c_double),
                ("X", c_void_p), ("Y", c_void_p), ("row0", c_void_p), ("eps", c_void_p),
                ("n_iter", c_void_p), ("u_accept", c_void_p), ("want_ll", c_void_p),
                ("noise_mode", c_int), ("noise", c_void_p), ("noise_off", c_void_p),
                ("seed", ctypes.c_uint64), ("chain0", ctypes.c_uint32), ("step_base", ctypes.c_uint32),
                ("W", c_void_p), ("b", c_void_p), ("out_A", c_void_p), ("out_accepted", c_void_p),
                ("out_ll", c_void_p), ("out_E", c_void_p), ("pW", c_void_p), ("pb", c_void_p),
                ("out_trace", c_void_p), ("out_abort", c_void_p), ("path_length", c_double),
                ("out_L", c_void_p), ("out_mom", c_void_p), ("out_host", c_void_p)]


class MvnArgs(ctypes.Structure):
    _fields_ = [("dim", c_int), ("C", c_int), ("n_steps", c_int), ("mu", c_void_p), ("prec", c_void_p),
                ("nlp_const", c_double), ("eps", c_dblp), ("n_iter", c_i32p), ("u_accept", c_dblp),
                ("noise_mode", c_int), ("noise", c_void_p), ("noise_off", c_i64p),
                ("seed", ctypes.c_uint64), ("chain0", ctypes.c_uint32), ("step_base", ctypes.c_uint32),
                ("x", c_void_p), ("out_A", c_void_p), ("out_accepted", c_void_p), ("out_nlp", c_void_p),
                ("out_trace", c_void_p)]


class MlpParams(ctypes.Structure):
    _fields_ = [("p", c_void_p * 6)]


class MlpSghmcArgs(ctypes.Structure):
    _fields_ = [("dtype", c_int), ("B", c_int), ("n_in", c_int), ("n_mid", c_int), ("n_out", c_int),
                ("n_steps", c_int), ("order", c_int * 6), ("alpha", c_double),
                ("X", c_void_p), ("y", c_void_p), ("row0", c_i64p), ("eps", c_dblp),
                ("n_iter", c_i32p), ("u_accept", c_dblp),
                ("noise_mode", c_int), ("noise", c_void_p), ("noise_off", c_i64p),
                ("mask_mode", c_int), ("masks", c_void_p), ("mask_off", c_i64p),
                ("seed", ctypes.c_uint64), ("chain", ctypes.c_uint32), ("step_base", ctypes.c_uint32),
                ("par", MlpParams), ("out_A", c_void_p), ("out_accepted", c_void_p),
                ("out_loss", c_void_p), ("out_nlp", c_void_p), ("out_E", c_void_p), ("out_abort", c_void_p)]


class MlpLeapfrogArgs(ctypes.Structure):
    _fields_ = [("dtype", c_int), ("B", c_int), ("n_in", c_int), ("n_mid", c_int), ("n_out", c_int),
                ("n_iter", c_int), ("order", c_int * 6), ("eps", c_double), ("alpha", c_double),
                ("X", c_void_p), ("y", c_void_p), ("q", MlpParams), ("p", MlpParams), ("g", MlpParams),
                ("mask_mode", c_int), ("masks", c_void_p), ("seed", ctypes.c_uint64), ("chain", ctypes.c_uint32),
                ("step", ctypes.c_uint32), ("slot0", ctypes.c_uint32)]


class SgdArgs(ctypes.Structure):
    _fields_ = [("dtype", c_int), ("model", c_int), ("B", c_int), ("D", c_int), ("K", c_int), ("n_steps", c_int),
                ("alpha", c_double), ("step_size", c_double), ("gamma", c_double),
                ("X", c_void_p), ("Y", c_void_p), ("row0", c_i64p),
                ("dropout", c_int), ("keep_p", c_double), ("mask_mode", c_int), ("keep", c_void_p),
                ("keep_off", c_i64p), ("seed", ctypes.c_uint64), ("step_base", ctypes.c_uint32),
                ("W", c_void_p), ("b", c_void_p), ("mW", c_void_p), ("mb", c_void_p)]


class HmcArgs(ctypes.Structure):
    _fields_ = [("dtype", c_int), ("model", c_int), ("B", c_int), ("D", c_int), ("K", c_int), ("n_steps", c_int),
                ("alpha", c_double), ("log_prior", c_double), ("lp_const", c_double * 2),
                ("X", c_void_p), ("Y", c_void_p), ("eps", c_dblp), ("n_iter", c_i32p), ("u_accept", c_dblp),
                ("noise_mode", c_int), ("noise", c_void_p), ("noise_off", c_i64p),
                ("seed", ctypes.c_uint64), ("chain", ctypes.c_uint32), ("step_base", ctypes.c_uint32),
                ("W", c_void_p), ("b", c_void_p), ("out_A", c_void_p), ("out_accepted", c_void_p),
                ("out_nlp", c_void_p), ("out_E", c_void_p), ("out_trace", c_void_p), ("out_mom", c_void_p)]


MODEL_SOFTMAX, MODEL_LOGISTIC = 0, 1
MLP_MASK_SLOT0 = 0x80000000
MLP_MASKS_NONE, MLP_MASKS_FIXED, MLP_MASKS_PHILOX = 0, 1, 2


# Every symbol include/hmcx.h declares (checked by tests/test_capi.py).
EXPORTS = ("hmcx_version", "hmcx_create", "hmcx_destroy", "hmcx_last_error", "hmcx_set_stream",
           "hmcx_synchronize", "hmcx_set_graph_mode", "hmcx_set_sghmc_path", "hmcx_set_timing", "hmcx_get_timing",
           "hmcx_philox_uniforms", "hmcx_philox_normals", "hmcx_philox_normals_f64",
           "hmcx_softmax_grad", "hmcx_softmax_loglik", "hmcx_softmax_predict", "hmcx_sghmc_run",
           "hmcx_sgld_run", "hmcx_hmc_mvn_run", "hmcx_mlp_masks", "hmcx_mlp_grad", "hmcx_mlp_loss",
           "hmcx_mlp_sghmc_run", "hmcx_mlp_hmc_leapfrog", "hmcx_logistic_grad", "hmcx_logistic_loglik", "hmcx_logistic_predict",
           "hmcx_sumsq", "hmcx_sgd_run", "hmcx_hmc_run", "hmcx_axpy", "hmcx_mvn_eval",
           "hmcx_clear_abort", "hmcx_get_recoveries", "hmcx_note_recovery", "hmcx_set_sgld_fuse", "hmcx_philox_schedule", "hmcx_host_wait", "hmcx_set_mlp_fuse",
           "hmcx_comm_unique_id", "hmcx_comm_init", "hmcx_comm_destroy", "hmcx_allgather_chain_stats",
           "hmcx_allreduce_f64", "hmcx_chain_diagnostics")

_lib = None
_lock = threading.Lock()


class HmcxError(RuntimeError):
    pass


def load_library():
    """Load libhmcx.so (no GPU needed); raise if it has not been built."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise HmcxError("libhmcx.so not built (%s): run `python -c 'import __graft_entry__ as g; g.build()'`"
                            % LIB_PATH)
        lib = ctypes.CDLL(LIB_PATH)
        lib.hmcx_version.restype = c_int
        lib.hmcx_create.argtypes = [c_int, ctypes.POINTER(c_void_p)]
        lib.hmcx_destroy.argtypes = [c_void_p]
        lib.hmcx_last_error.argtypes = [c_void_p]
        lib.hmcx_last_error.restype = ctypes.c_char_p
        lib.hmcx_set_stream.argtypes = [c_void_p, c_void_p]
        lib.hmcx_synchronize.argtypes = [c_void_p]
        lib.hmcx_set_graph_mode.argtypes = [c_void_p, c_int]
        lib.hmcx_set_sghmc_path.argtypes = [c_void_p, c_int]
        lib.hmcx_set_timing.argtypes = [c_void_p, c_int]
        lib.hmcx_get_timing.argtypes = [c_void_p, c_dblp, ctypes.POINTER(ctypes.c_longlong)]
        lib.hmcx_philox_uniforms.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                             ctypes.c_uint32, c_dblp]
        lib.hmcx_philox_uniforms.restype = None
        lib.hmcx_philox_normals.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_uint32, ctypes.c_uint32, c_dblp]
        lib.hmcx_philox_normals.restype = None
        lib.hmcx_philox_normals_f64.argtypes = lib.hmcx_philox_normals.argtypes
        lib.hmcx_philox_normals_f64.restype = None
        lib.hmcx_softmax_grad.argtypes = [c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                          c_void_p, c_void_p, c_double, c_void_p, c_void_p]
        lib.hmcx_softmax_loglik.argtypes = [c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                            c_void_p, c_void_p, c_void_p]
        lib.hmcx_softmax_predict.argtypes = [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int,
                                             c_void_p, c_void_p, c_void_p]
        lib.hmcx_sghmc_run.argtypes = [c_void_p, ctypes.POINTER(SamplerArgs)]
        lib.hmcx_clear_abort.argtypes = [c_void_p]
        if hasattr(lib, "hmcx_get_recoveries"):        # absent in older builds loaded for A/B runs
            lib.hmcx_get_recoveries.argtypes = [c_void_p, c_i64p]
            lib.hmcx_note_recovery.argtypes = [c_void_p, c_int]
        lib.hmcx_host_wait.argtypes = [c_void_p, c_void_p]
        lib.hmcx_philox_schedule.argtypes = [ctypes.c_uint64, ctypes.c_uint32, c_int, ctypes.c_uint32, c_int,
                                             c_double, c_dblp, c_dblp, c_i32p, c_dblp]
        lib.hmcx_sgld_run.argtypes = [c_void_p, ctypes.POINTER(SamplerArgs)]
        lib.hmcx_hmc_mvn_run.argtypes = [c_void_p, ctypes.POINTER(MvnArgs)]
        u32, u64 = ctypes.c_uint32, ctypes.c_uint64
        lib.hmcx_mlp_masks.argtypes = [c_void_p, c_int, c_int, c_int, u64, u32, u32, u32, c_void_p]
        lib.hmcx_mlp_grad.argtypes = [c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                      ctypes.POINTER(MlpParams), c_void_p, c_double, ctypes.POINTER(MlpParams),
                                      c_void_p]
        lib.hmcx_mlp_loss.argtypes = [c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                      ctypes.POINTER(MlpParams), c_void_p, c_void_p, c_void_p]
        lib.hmcx_mlp_sghmc_run.argtypes = [c_void_p, ctypes.POINTER(MlpSghmcArgs)]
        if hasattr(lib, "hmcx_mlp_hmc_leapfrog"):
            lib.hmcx_mlp_hmc_leapfrog.argtypes = [c_void_p, ctypes.POINTER(MlpLeapfrogArgs)]
        if hasattr(lib, "hmcx_set_mlp_fuse"):          # absent in older builds loaded for A/B runs
            lib.hmcx_set_mlp_fuse.argtypes = [c_void_p, c_int]
        if hasattr(lib, "hmcx_set_sgld_fuse"):
            lib.hmcx_set_sgld_fuse.argtypes = [c_void_p, c_int]
        if hasattr(lib, "hmcx_comm_init"):
            lib.hmcx_comm_unique_id.argtypes = [c_void_p]
            lib.hmcx_comm_init.argtypes = [c_void_p, c_int, c_int, c_void_p, ctypes.POINTER(c_void_p)]
            lib.hmcx_comm_destroy.argtypes = [c_void_p]
            lib.hmcx_allgather_chain_stats.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_uint64]
            lib.hmcx_allreduce_f64.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_uint64, c_int]
        if hasattr(lib, "hmcx_chain_diagnostics"):
            lib.hmcx_chain_diagnostics.argtypes = [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                                   ctypes.c_int64, c_void_p]
        lib.hmcx_logistic_grad.argtypes = [c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int,
                                           c_void_p, c_void_p, c_double, c_void_p, c_void_p]
        lib.hmcx_logistic_loglik.argtypes = [c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int,
                                             c_void_p, c_void_p, c_void_p]
        lib.hmcx_logistic_predict.argtypes = [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                                              c_void_p]
        lib.hmcx_sumsq.argtypes = [c_void_p, c_int, c_void_p, ctypes.c_int64, c_void_p]
        lib.hmcx_sgd_run.argtypes = [c_void_p, ctypes.POINTER(SgdArgs)]
        lib.hmcx_hmc_run.argtypes = [c_void_p, ctypes.POINTER(HmcArgs)]
        lib.hmcx_axpy.argtypes = [c_void_p, c_int, c_int, ctypes.c_int64, c_double, c_void_p, c_void_p]
        lib.hmcx_mvn_eval.argtypes = [c_void_p, c_int, c_int, c_void_p, c_void_p, c_double, c_void_p, c_void_p,
                                      c_void_p]
        _lib = lib
        return lib


class Context:
    """One hmcx context per HIP device; calls run on torch's current stream."""

    def __init__(self, device):
        lib = load_library()
        if not torch.cuda.is_available():
            raise HmcxError("no HIP device visible: the HIP engine has no CPU fallback")
        self.lib = lib
        self.device = torch.device("cuda", device if isinstance(device, int) else (device.index or 0))
        h = c_void_p()
        with torch.cuda.device(self.device):
            rc = lib.hmcx_create(self.device.index, ctypes.byref(h))
        if rc != 0:
            raise HmcxError("hmcx_create failed (%d)" % rc)
        self.h = h

    _bound = None

    def bind_stream(self):
        """Run on torch's current stream of this device (set again only when it has changed)."""
        try:
            raw = torch._C._cuda_getCurrentRawStream(self.device.index)
        except AttributeError:
            raw = torch.cuda.current_stream(self.device).cuda_stream
        if raw != self._bound:
            self.lib.hmcx_set_stream(self.h, c_void_p(raw))
            self._bound = raw

    def check(self, rc, what):
        if rc != 0:
            msg = self.lib.hmcx_last_error(self.h)
            raise HmcxError("%s failed (%d): %s" % (what, rc, msg.decode() if msg else ""))

    path = 0

    def set_sghmc_path(self, path):
        """0 auto, 1 kernel-per-phase, 2 persistent (see include/hmcx.h)."""
        self.check(self.lib.hmcx_set_sghmc_path(self.h, int(path)), "hmcx_set_sghmc_path")
        self.path = int(path)

    def clear_abort(self):
        """Lower the context's persistent-launch abort word (include/hmcx.h hmcx_clear_abort)."""
        self.check(self.lib.hmcx_clear_abort(self.h), "hmcx_clear_abort")

    RECOVERY_KINDS = ("persistent_sghmc", "mlp_fused", "sgld_wide_fused")   # include/hmcx.h hmcx_recovery

    def recoveries(self):
        """Re-runs after timed-out exchanges since this context was created, by kind
        (include/hmcx.h hmcx_get_recoveries): all zero unless a fallback path ran.  None when the
        loaded library predates the counters (an older build loaded through HMCX_LIB for an A/B run)."""
        if not hasattr(self.lib, "hmcx_get_recoveries"):
            return None
        out = (ctypes.c_int64 * len(self.RECOVERY_KINDS))()
        self.check(self.lib.hmcx_get_recoveries(self.h, out), "hmcx_get_recoveries")
        return dict(zip(self.RECOVERY_KINDS, (int(v) for v in out)))

    def note_recovery(self, kind):
        """Record a re-run the host layer performed (include/hmcx.h hmcx_note_recovery)."""
        self.check(self.lib.hmcx_note_recovery(self.h, self.RECOVERY_KINDS.index(kind)), "hmcx_note_recovery")

    mlp_fuse = True

    def set_sgld_fuse(self, on):
        """Fused forward + softmax of the wide SGLD path (include/hmcx.h hmcx_set_sgld_fuse)."""
        self.check(self.lib.hmcx_set_sgld_fuse(self.h, 1 if on else 0), "hmcx_set_sgld_fuse")

    def set_mlp_fuse(self, on):
        """Fused layer-2/3 MLP launches in the sampler (include/hmcx.h hmcx_set_mlp_fuse)."""
        self.check(self.lib.hmcx_set_mlp_fuse(self.h, 1 if on else 0), "hmcx_set_mlp_fuse")
        self.mlp_fuse = bool(on)

    def set_timing(self, on):
        """Bracket every sampler run's kernels with HIP events on the launch stream (resets totals)."""
        self.check(self.lib.hmcx_set_timing(self.h, 1 if on else 0), "hmcx_set_timing")

    def get_timing(self):
        """(summed kernel milliseconds, number of timed runs) since set_timing(True)."""
        ms, n = c_double(), ctypes.c_longlong()
        self.check(self.lib.hmcx_get_timing(self.h, ctypes.byref(ms), ctypes.byref(n)), "hmcx_get_timing")
        return ms.value, n.value

    def set_graph_mode(self, on):
        self.check(self.lib.hmcx_set_graph_mode(self.h, 1 if on else 0), "hmcx_set_graph_mode")

    def __del__(self):
        try:
            if getattr(self, "h", None) and self.h.value:
                self.lib.hmcx_destroy(self.h)
        except Exception:
            pass


_ctxs = {}


def context(device=None):
    """Context for `device` (default: torch's current device)."""
    if device is None:
        device = torch.cuda.current_device() if torch.cuda.is_available() else 0
    idx = device if isinstance(device, int) else (
        device.index or 0 if isinstance(device, torch.device) else torch.device(device).index or 0)
    ctx = _ctxs.get(idx)
    if ctx is None:
        with _lock:
            ctx = _ctxs.get(idx)
        if ctx is None:
            ctx = Context(idx)
            with _lock:
                _ctxs[idx] = ctx
    ctx.bind_stream()
    return ctx


@atexit.register
def _release_contexts():
    """Destroy contexts while the HIP runtime (and any profiler tool) is still alive."""
    with _lock:
        ctxs = list(_ctxs.values())
        _ctxs.clear()
    for c in ctxs:
        if getattr(c, "h", None) and c.h.value:
            c.lib.hmcx_destroy(c.h)
            c.h = c_void_p()


def recoveries_all():
    """Summed recovery counts over every context of this process (zeros when none exists)."""
    tot = dict.fromkeys(Context.RECOVERY_KINDS, 0)
    with _lock:
        ctxs = list(_ctxs.values())
    for c in ctxs:
        for k, v in (c.recoveries() or {}).items():
            tot[k] += v
    return tot


def ptr(t):
    return c_void_p(t.data_ptr()) if t is not None else c_void_p()


def addr(a):
    """Address of a host ndarray's data (None for None)."""
    return a.__array_interface__['data'][0] if a is not None else None


def dtype_code(dt):
    if dt == torch.float64:
        return HMCX_F64
    if dt == torch.float32:
        return HMCX_F32
    raise HmcxError("unsupported dtype %s (float32/float64)" % dt)


def philox_uniforms(seed, chain, step, slot, n):
    import numpy as np
    lib = load_library()
    out = np.empty(n, dtype=np.float64)
    lib.hmcx_philox_uniforms(seed, chain, step, slot, n, out.ctypes.data_as(c_dblp))
    return out


def philox_normals(seed, chain, step, slot, e0, n, dtype="f32"):
    """Host twin of the device noise stream: dtype 'f32' (float Box–Muller, f32 chains) or 'f64'
    (53-bit uniforms, double Box–Muller, f64 chains)."""
    import numpy as np
    lib = load_library()
    out = np.empty(n, dtype=np.float64)
    fn = lib.hmcx_philox_normals_f64 if dtype == "f64" else lib.hmcx_philox_normals
    fn(seed, chain, step, slot, e0, n, out.ctypes.data_as(c_dblp))
    return out


SLOT_PATH = 0xFFFFFFFE
SLOT_ACCEPT = 0xFFFFFFFD


def philox_schedule(seed, chain0, C, step_base, path_length, eps):
    """Path lengths L, iterations max(0, L − 1) and accept uniforms of len(eps) Philox-mode steps
    for C chains, [n_steps, C] each (hmcx_philox_schedule; one host C call)."""
    import numpy as np
    eps = np.ascontiguousarray(eps, dtype=np.float64)
    n = eps.shape[0]
    L = np.empty((n, C), dtype=np.float64)
    n_iter = np.empty((n, C), dtype=np.int32)
    u = np.empty((n, C), dtype=np.float64)
    rc = load_library().hmcx_philox_schedule(seed & 0xFFFFFFFFFFFFFFFF, chain0 & 0xFFFFFFFF, C,
                                             step_base & 0xFFFFFFFF, n, float(path_length),
                                             eps.ctypes.data_as(c_dblp), L.ctypes.data_as(c_dblp),
                                             n_iter.ctypes.data_as(c_i32p), u.ctypes.data_as(c_dblp))
    if rc != 0:
        raise HmcxError("non-finite path length (step size 0?)")
    return L, n_iter, u


def philox_uniforms_chains(seed, chains, step, slot, idx=0):
    """Philox4x32-10 uniform of element `idx` for every (step, chain): `chains` and `step` broadcast
    against each other (vectorised host twin of hmcx_common.h::philox_uniform, bit-identical to
    hmcx_philox_uniforms)."""
    import numpy as np
    M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
    mask = np.uint64(0xFFFFFFFF)
    ch, st = np.broadcast_arrays(np.asarray(chains, dtype=np.uint64) & mask,
                                 np.asarray(step, dtype=np.uint64) & mask)
    c0 = np.full(ch.shape, idx, dtype=np.uint64)
    c1 = np.full(ch.shape, slot & 0xFFFFFFFF, dtype=np.uint64)
    c2 = st.copy()
    c3 = ch.copy()
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        c0, c1, c2, c3 = ((p1 >> np.uint64(32)) ^ c1 ^ np.uint64(k0)), p1 & mask, \
                         ((p0 >> np.uint64(32)) ^ c3 ^ np.uint64(k1)), p0 & mask
        k0 = (k0 + 0x9E3779B9) & 0xFFFFFFFF
        k1 = (k1 + 0xBB67AE85) & 0xFFFFFFFF
    return ((c0 << np.uint64(21)) ^ (c1 >> np.uint64(11))).astype(np.float64) * (1.0 / 9007199254740992.0)
