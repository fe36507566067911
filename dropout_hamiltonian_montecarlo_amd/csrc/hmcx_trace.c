/* HDF5 posterior-trace backend (include/hmcx_trace.h).  Host C over the HDF5 1.10 C API.
 *
 * Layout written per file (reference: inference/cpu/sghmc_multicore.py:36-53): one root dataset
 * per variable, float32 LE, dims (rows,)+param_shape with rows starting at 1 (the fill value 0)
 * and growing by the appended steps, maxdims (H5S_UNLIMITED,)+param_shape.  Chunks hold whole
 * rows, about 1 MiB each, so appending a block of steps touches each chunk once. */
#include "hmcx_trace.h"

#include <hdf5.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define TR_MAX_VARS 64
#define TR_MAX_RANK 7

struct hmcx_trace {
  hid_t file;
  int n;
  hid_t ds[TR_MAX_VARS];
  int rank[TR_MAX_VARS];                       /* param rank; dataset rank is rank + 1 */
  hsize_t dims[TR_MAX_VARS][TR_MAX_RANK + 1];  /* current dataset dims */
};

static __thread char g_err[512];

static int fail(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  return -1;
}

const char* hmcx_trace_last_error(void) { return g_err; }

static void quiet(void) { H5Eset_auto2(H5E_DEFAULT, NULL, NULL); }

static void close_all(hmcx_trace* t) {
  for (int v = 0; v < t->n; ++v)
    if (t->ds[v] >= 0) H5Dclose(t->ds[v]);
  if (t->file >= 0) H5Fclose(t->file);
}

hmcx_trace* hmcx_trace_create(const char* path, int n_vars, const char* const* names, const int* ranks,
                              const int64_t* shapes) {
  quiet();
  if (!path || !names || !ranks || n_vars < 1 || n_vars > TR_MAX_VARS) {
    fail("trace_create: bad arguments (1 <= n_vars <= %d)", TR_MAX_VARS);
    return NULL;
  }
  hmcx_trace* t = (hmcx_trace*)calloc(1, sizeof(hmcx_trace));
  if (!t) { fail("trace_create: out of memory"); return NULL; }
  t->file = -1;
  for (int v = 0; v < TR_MAX_VARS; ++v) t->ds[v] = -1;
  t->file = H5Fcreate(path, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT);
  if (t->file < 0) { fail("trace_create: cannot create %s", path); free(t); return NULL; }
  int64_t off = 0;
  for (int v = 0; v < n_vars; ++v) {
    const int r = ranks[v];
    if (r < 0 || r > TR_MAX_RANK || !names[v] || (r > 0 && !shapes)) {
      fail("trace_create: bad rank/name for variable %d", v);
      t->n = v; close_all(t); free(t); return NULL;
    }
    hsize_t dims[TR_MAX_RANK + 1], maxd[TR_MAX_RANK + 1], chunk[TR_MAX_RANK + 1];
    dims[0] = 1; maxd[0] = H5S_UNLIMITED;
    hsize_t row = 1;
    for (int i = 0; i < r; ++i) {
      if (shapes[off + i] < 1) { fail("trace_create: zero-sized dim in %s", names[v]); t->n = v; close_all(t); free(t); return NULL; }
      dims[i + 1] = maxd[i + 1] = chunk[i + 1] = (hsize_t)shapes[off + i];
      row *= (hsize_t)shapes[off + i];
    }
    off += r;
    hsize_t rows_per_chunk = (hsize_t)((1u << 20) / 4) / row;
    if (rows_per_chunk < 1) rows_per_chunk = 1;
    if (rows_per_chunk > 4096) rows_per_chunk = 4096;
    chunk[0] = rows_per_chunk;
    hid_t space = H5Screate_simple(r + 1, dims, maxd);
    hid_t dcpl = H5Pcreate(H5P_DATASET_CREATE);
    const float zero = 0.0f;
    int bad = space < 0 || dcpl < 0 || H5Pset_chunk(dcpl, r + 1, chunk) < 0 ||
              H5Pset_fill_value(dcpl, H5T_NATIVE_FLOAT, &zero) < 0 ||
              H5Pset_fill_time(dcpl, H5D_FILL_TIME_ALLOC) < 0;
    hid_t ds = bad ? -1 : H5Dcreate2(t->file, names[v], H5T_IEEE_F32LE, space, H5P_DEFAULT, dcpl, H5P_DEFAULT);
    if (dcpl >= 0) H5Pclose(dcpl);
    if (space >= 0) H5Sclose(space);
    t->n = v + 1;
    if (ds < 0) { fail("trace_create: cannot create dataset %s", names[v]); close_all(t); free(t); return NULL; }
    t->ds[v] = ds;
    t->rank[v] = r;
    memcpy(t->dims[v], dims, sizeof(hsize_t) * (size_t)(r + 1));
  }
  return t;
}

int hmcx_trace_append(hmcx_trace* t, int var, const float* rows, int64_t n_rows) {
  quiet();
  if (!t || var < 0 || var >= t->n) return fail("trace_append: bad handle or variable");
  if (n_rows < 0 || (n_rows > 0 && !rows)) return fail("trace_append: bad rows");
  if (n_rows == 0) return 0;
  const int R = t->rank[var] + 1;
  hsize_t nd[TR_MAX_RANK + 1], start[TR_MAX_RANK + 1], count[TR_MAX_RANK + 1];
  for (int i = 0; i < R; ++i) { nd[i] = t->dims[var][i]; start[i] = 0; count[i] = t->dims[var][i]; }
  start[0] = t->dims[var][0];
  count[0] = (hsize_t)n_rows;
  nd[0] = t->dims[var][0] + (hsize_t)n_rows;
  if (H5Dset_extent(t->ds[var], nd) < 0) return fail("trace_append: resize failed");
  hid_t fs = H5Dget_space(t->ds[var]);
  hid_t ms = H5Screate_simple(R, count, NULL);
  int rc = 0;
  if (fs < 0 || ms < 0 || H5Sselect_hyperslab(fs, H5S_SELECT_SET, start, NULL, count, NULL) < 0 ||
      H5Dwrite(t->ds[var], H5T_NATIVE_FLOAT, ms, fs, H5P_DEFAULT, rows) < 0)
    rc = fail("trace_append: write failed");
  if (ms >= 0) H5Sclose(ms);
  if (fs >= 0) H5Sclose(fs);
  if (rc == 0) t->dims[var][0] = nd[0];
  return rc;
}

int64_t hmcx_trace_rows(const hmcx_trace* t, int var) {
  if (!t || var < 0 || var >= t->n) return fail("trace_rows: bad handle or variable");
  return (int64_t)t->dims[var][0];
}

int hmcx_trace_flush(hmcx_trace* t) {
  quiet();
  if (!t) return fail("trace_flush: null handle");
  return H5Fflush(t->file, H5F_SCOPE_LOCAL) < 0 ? fail("trace_flush failed") : 0;
}

int hmcx_trace_close(hmcx_trace* t) {
  quiet();
  if (!t) return fail("trace_close: null handle");
  int rc = 0;
  for (int v = 0; v < t->n; ++v)
    if (t->ds[v] >= 0 && H5Dclose(t->ds[v]) < 0) rc = -1;
  if (t->file >= 0 && H5Fclose(t->file) < 0) rc = -1;
  free(t);
  return rc ? fail("trace_close failed") : 0;
}

/* ------------------------------------------------------------------------------ readers */
typedef struct { char* buf; int64_t len, used; int count, overflow; } name_acc;

static herr_t collect_name(hid_t g, const char* name, const H5L_info_t* info, void* op) {
  (void)g; (void)info;
  name_acc* a = (name_acc*)op;
  const int64_t n = (int64_t)strlen(name);
  if (a->used + n + 1 > a->len) { a->overflow = 1; return 1; }
  memcpy(a->buf + a->used, name, (size_t)n);
  a->used += n;
  a->buf[a->used++] = '\n';
  a->count++;
  return 0;
}

int hmcx_h5_list(const char* path, char* buf, int64_t buf_len) {
  quiet();
  if (!path || !buf || buf_len < 1) return fail("h5_list: bad arguments");
  hid_t f = H5Fopen(path, H5F_ACC_RDONLY, H5P_DEFAULT);
  if (f < 0) return fail("h5_list: cannot open %s", path);
  name_acc a = {buf, buf_len - 1, 0, 0, 0};
  hsize_t idx = 0;
  herr_t r = H5Literate(f, H5_INDEX_NAME, H5_ITER_INC, &idx, collect_name, &a);
  H5Fclose(f);
  if (a.overflow) return fail("h5_list: name buffer too small");
  if (r < 0) return fail("h5_list: iteration failed");
  buf[a.used] = '\0';
  return a.count;
}

static hid_t open_ds(const char* path, const char* name, hid_t* f) {
  *f = H5Fopen(path, H5F_ACC_RDONLY, H5P_DEFAULT);
  if (*f < 0) { fail("h5: cannot open %s", path); return -1; }
  hid_t ds = H5Dopen2(*f, name, H5P_DEFAULT);
  if (ds < 0) { fail("h5: no dataset %s in %s", name, path); H5Fclose(*f); return -1; }
  return ds;
}

int hmcx_h5_info(const char* path, const char* name, int64_t* dims, int max_rank) {
  quiet();
  if (!path || !name || !dims || max_rank < 0) return fail("h5_info: bad arguments");
  hid_t f, ds = open_ds(path, name, &f);
  if (ds < 0) return -1;
  hid_t sp = H5Dget_space(ds);
  int r = sp < 0 ? -1 : H5Sget_simple_extent_ndims(sp);
  hsize_t d[32];
  int rc = r;
  if (r < 0 || r > 32) rc = fail("h5_info: bad dataspace");
  else if (r > max_rank) rc = fail("h5_info: rank %d exceeds %d", r, max_rank);
  else {
    H5Sget_simple_extent_dims(sp, d, NULL);
    for (int i = 0; i < r; ++i) dims[i] = (int64_t)d[i];
  }
  if (sp >= 0) H5Sclose(sp);
  H5Dclose(ds);
  H5Fclose(f);
  return rc;
}

static int read_as(const char* path, const char* name, hid_t mtype, void* out, int64_t n_elems);

int hmcx_h5_read_f32(const char* path, const char* name, float* out, int64_t n_elems) {
  return read_as(path, name, H5T_NATIVE_FLOAT, out, n_elems);
}

int hmcx_h5_read_f64(const char* path, const char* name, double* out, int64_t n_elems) {
  return read_as(path, name, H5T_NATIVE_DOUBLE, out, n_elems);
}

static int read_as(const char* path, const char* name, hid_t mtype, void* out, int64_t n_elems) {
  quiet();
  if (!path || !name || (n_elems > 0 && !out)) return fail("h5_read: bad arguments");
  hid_t f, ds = open_ds(path, name, &f);
  if (ds < 0) return -1;
  hid_t sp = H5Dget_space(ds);
  const hssize_t n = sp < 0 ? -1 : H5Sget_simple_extent_npoints(sp);
  int rc = 0;
  if (n < 0) rc = fail("h5_read: bad dataspace");
  else if ((int64_t)n != n_elems) rc = fail("h5_read: %s has %lld elements, buffer %lld", name, (long long)n,
                                           (long long)n_elems);
  else if (n > 0 && H5Dread(ds, mtype, H5S_ALL, H5S_ALL, H5P_DEFAULT, out) < 0)
    rc = fail("h5_read: read of %s failed", name);
  if (sp >= 0) H5Sclose(sp);
  H5Dclose(ds);
  H5Fclose(f);
  return rc;
}

int hmcx_h5_write(const char* path, const char* name, int type, int rank, const int64_t* dims, const void* data,
                  int truncate) {
  quiet();
  if (!path || !name || rank < 0 || rank > 32 || (rank > 0 && !dims)) return fail("h5_write: bad arguments");
  hid_t ftype, mtype;
  switch (type) {
    case HMCX_H5_U8: ftype = H5T_STD_U8LE; mtype = H5T_NATIVE_UINT8; break;
    case HMCX_H5_I64: ftype = H5T_STD_I64LE; mtype = H5T_NATIVE_INT64; break;
    case HMCX_H5_F32: ftype = H5T_IEEE_F32LE; mtype = H5T_NATIVE_FLOAT; break;
    case HMCX_H5_F64: ftype = H5T_IEEE_F64LE; mtype = H5T_NATIVE_DOUBLE; break;
    default: return fail("h5_write: bad type %d", type);
  }
  hsize_t d[32], n = 1;
  for (int i = 0; i < rank; ++i) {
    if (dims[i] < 0) return fail("h5_write: negative dim");
    d[i] = (hsize_t)dims[i];
    n *= d[i];
  }
  if (n > 0 && !data) return fail("h5_write: null data");
  hid_t f;
  if (truncate) f = H5Fcreate(path, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT);
  else {
    f = H5Fopen(path, H5F_ACC_RDWR, H5P_DEFAULT);
    if (f < 0) f = H5Fcreate(path, H5F_ACC_EXCL, H5P_DEFAULT, H5P_DEFAULT);
  }
  if (f < 0) return fail("h5_write: cannot open %s", path);
  hid_t sp = H5Screate_simple(rank, d, NULL);
  hid_t ds = sp < 0 ? -1 : H5Dcreate2(f, name, ftype, sp, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
  int rc = 0;
  if (ds < 0) rc = fail("h5_write: cannot create dataset %s", name);
  else if (n > 0 && H5Dwrite(ds, mtype, H5S_ALL, H5S_ALL, H5P_DEFAULT, data) < 0) rc = fail("h5_write: write failed");
  if (ds >= 0) H5Dclose(ds);
  if (sp >= 0) H5Sclose(sp);
  if (H5Fclose(f) < 0 && rc == 0) rc = fail("h5_write: close failed");
  return rc;
}
