"""Posterior traces in the reference's HDF5 backend format (ctypes over lib/libhmcx_trace.so).

Reference writer: /root/reference/hamiltonian/inference/cpu/sghmc_multicore.py:36-53 (and
gpu/sgld_multicore.py:30-47): per worker file ``backend_i.h5``, one root dataset per variable,
float32, created (1,)+shape with maxshape (None,)+shape — row 0 is the zero fill value — and
grown by one row per sampler step.  Reference reader: cpu/hmc.py:132-138 (``backend_mean``).

h5py is not available in this image; the native library (include/hmcx_trace.h) writes and reads
the same files through the HDF5 C library.  It raises if that library is missing — there is no
other storage fallback.
"""
import ctypes
import os

import numpy as np

_LIB_PATH = os.environ.get("HMCX_TRACE_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib",
                                                              "libhmcx_trace.so")
EXPORTS = ["hmcx_trace_create", "hmcx_trace_append", "hmcx_trace_rows", "hmcx_trace_flush", "hmcx_trace_close",
           "hmcx_h5_list", "hmcx_h5_info", "hmcx_h5_read_f32", "hmcx_h5_read_f64", "hmcx_h5_write",
           "hmcx_trace_last_error"]
_H5_TYPES = {np.dtype(np.uint8): 0, np.dtype(np.int64): 1, np.dtype(np.float32): 2, np.dtype(np.float64): 3}
_lib = None


class TraceError(RuntimeError):
    pass


def load_library():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        raise TraceError("libhmcx_trace.so not built (%s): run __graft_entry__.build() on a machine with "
                         "the HDF5 C library" % _LIB_PATH)
    lib = ctypes.CDLL(_LIB_PATH)
    vp, i64, c_int = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    lib.hmcx_trace_create.restype = vp
    lib.hmcx_trace_create.argtypes = [ctypes.c_char_p, c_int, ctypes.POINTER(ctypes.c_char_p),
                                      ctypes.POINTER(c_int), ctypes.POINTER(i64)]
    lib.hmcx_trace_append.argtypes = [vp, c_int, vp, i64]
    lib.hmcx_trace_rows.restype = i64
    lib.hmcx_trace_rows.argtypes = [vp, c_int]
    lib.hmcx_trace_flush.argtypes = [vp]
    lib.hmcx_trace_close.argtypes = [vp]
    lib.hmcx_h5_list.argtypes = [ctypes.c_char_p, ctypes.c_char_p, i64]
    lib.hmcx_h5_info.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(i64), c_int]
    lib.hmcx_h5_read_f32.argtypes = [ctypes.c_char_p, ctypes.c_char_p, vp, i64]
    lib.hmcx_h5_read_f64.argtypes = [ctypes.c_char_p, ctypes.c_char_p, vp, i64]
    lib.hmcx_h5_write.argtypes = [ctypes.c_char_p, ctypes.c_char_p, c_int, c_int, ctypes.POINTER(i64), vp, c_int]
    lib.hmcx_trace_last_error.restype = ctypes.c_char_p
    lib.hmcx_trace_last_error.argtypes = []
    _lib = lib
    return lib


def _check(rc, what):
    if rc < 0:
        raise TraceError("%s: %s" % (what, load_library().hmcx_trace_last_error().decode()))
    return rc


class TraceFile:
    """One backend file: ``TraceFile(path, {var: param_shape})`` creates the datasets
    ((1,)+shape, float32, unlimited rows); ``append(var, rows)`` adds rows [n, *shape]."""

    def __init__(self, path, shapes):
        lib = load_library()
        self.path = str(path)
        self.vars = list(shapes.keys())
        self.shapes = {v: tuple(int(d) for d in shapes[v]) for v in self.vars}
        names = (ctypes.c_char_p * len(self.vars))(*[v.encode() for v in self.vars])
        ranks = (ctypes.c_int * len(self.vars))(*[len(self.shapes[v]) for v in self.vars])
        flat = [d for v in self.vars for d in self.shapes[v]] or [0]
        dims = (ctypes.c_int64 * len(flat))(*flat)
        self._h = lib.hmcx_trace_create(self.path.encode(), len(self.vars), names, ranks, dims)
        if not self._h:
            raise TraceError("trace_create: " + lib.hmcx_trace_last_error().decode())

    def append(self, var, rows):
        shape = self.shapes[var]
        a = np.ascontiguousarray(rows, dtype=np.float32).reshape((-1,) + shape)
        _check(load_library().hmcx_trace_append(self._h, self.vars.index(var), a.ctypes.data, a.shape[0]),
               "trace_append")

    def rows(self, var):
        return _check(load_library().hmcx_trace_rows(self._h, self.vars.index(var)), "trace_rows")

    def flush(self):
        _check(load_library().hmcx_trace_flush(self._h), "trace_flush")

    def close(self):
        if self._h:
            h, self._h = self._h, None
            _check(load_library().hmcx_trace_close(h), "trace_close")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def list_datasets(path):
    """Root names in name order (h5py ``File.keys()``)."""
    lib = load_library()
    size = 1 << 16
    while True:
        buf = ctypes.create_string_buffer(size)
        n = lib.hmcx_h5_list(str(path).encode(), buf, size)
        if n >= 0:
            return [s for s in buf.value.decode().split("\n") if s][:n]
        if "too small" not in lib.hmcx_trace_last_error().decode() or size > (1 << 26):
            _check(n, "h5_list")
        size *= 4


def dataset_shape(path, name):
    lib = load_library()
    dims = (ctypes.c_int64 * 32)()
    r = _check(lib.hmcx_h5_info(str(path).encode(), name.encode(), dims, 32), "h5_info")
    return tuple(dims[i] for i in range(r))


def read_dataset(path, name, dtype=np.float32):
    """The whole dataset (``f[name][...]``) converted to float32 (default) or float64."""
    lib = load_library()
    dtype = np.dtype(dtype)
    if dtype not in (np.dtype(np.float32), np.dtype(np.float64)):
        raise ValueError("read_dataset: dtype float32 or float64")
    out = np.empty(dataset_shape(path, name), dtype=dtype)
    fn = lib.hmcx_h5_read_f32 if dtype == np.float32 else lib.hmcx_h5_read_f64
    _check(fn(str(path).encode(), name.encode(), out.ctypes.data, out.size), "h5_read")
    return out


def write_dataset(path, name, data, truncate=False):
    """Write ``data`` (uint8, int64, float32 or float64) as the fixed-shape dataset ``name``."""
    a = np.ascontiguousarray(data)
    if a.dtype not in _H5_TYPES:
        raise ValueError("write_dataset: unsupported dtype %s" % a.dtype)
    dims = (ctypes.c_int64 * max(1, a.ndim))(*a.shape)
    _check(load_library().hmcx_h5_write(str(path).encode(), name.encode(), _H5_TYPES[a.dtype], a.ndim, dims,
                                        a.ctypes.data, 1 if truncate else 0), "h5_write")


def backend_mean(start, multi_backend, niter):
    """cpu/hmc.py:132-138: per file {var: np.sum(f[var], axis=0)} over every root dataset, summed
    over files, divided by niter and reshaped to the start shape (float32 arithmetic, as there)."""
    aux = []
    for filename in multi_backend:
        aux.append({var: np.sum(read_dataset(filename, var), axis=0) for var in list_datasets(filename)})
    return {var: ((np.sum([r[var] for r in aux], axis=0).reshape(np.shape(start[var]))) / niter)
            for var in start.keys()}
