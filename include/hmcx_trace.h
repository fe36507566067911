/* hmcx_trace — posterior trace storage in the reference's HDF5 backend format.
 *
 * Replaces the h5py backend of the reference's multi-chain samplers:
 *   writer  hamiltonian/inference/cpu/sghmc_multicore.py:36-53 and
 *           hamiltonian/inference/gpu/sgld_multicore.py:30-47 —
 *           one file per worker, one root dataset per variable, float32, created with shape
 *           (1,)+param_shape and maxshape (None,)+param_shape (so row 0 is the zero fill value),
 *           grown by one row per sampler step, flushed after each step;
 *   reader  hamiltonian/inference/cpu/hmc.py:132-138 (backend_mean: every root dataset of every
 *           file, summed over axis 0).
 * Host-only C library over the HDF5 C API (libhdf5, 1.10.x); no device code and no torch.
 * Every function returns 0 (or a count / rank) on success and -1 on failure; the message of the
 * last failure on this thread is hmcx_trace_last_error(). */
#ifndef HMCX_TRACE_H
#define HMCX_TRACE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hmcx_trace hmcx_trace;

/* Create (truncate) `path` with n_vars root datasets: names[v], param rank ranks[v] (0..7) and
 * param shape shapes[off_v .. off_v+ranks[v]) where off_v = Σ_{u<v} ranks[u].  Each dataset is
 * float32 (IEEE LE), shape (1,)+param_shape, maxshape (unlimited,)+param_shape, chunked, fill 0
 * (h5py create_dataset(var, (1,)+shape, maxshape=(None,)+shape, dtype=float32),
 * sghmc_multicore.py:40).  Returns NULL on failure. */
hmcx_trace* hmcx_trace_create(const char* path, int n_vars, const char* const* names, const int* ranks,
                              const int64_t* shapes);

/* Append n_rows rows (host float32, row-major [n_rows][param_shape]) to dataset `var`: the
 * resize-then-write of sghmc_multicore.py:49-51, n_rows steps at once. */
int hmcx_trace_append(hmcx_trace* t, int var, const float* rows, int64_t n_rows);

/* Current number of rows of dataset `var` (initial zero row included). */
int64_t hmcx_trace_rows(const hmcx_trace* t, int var);

int hmcx_trace_flush(hmcx_trace* t);                     /* sghmc_multicore.py:52 */
int hmcx_trace_close(hmcx_trace* t);                     /* sghmc_multicore.py:53; frees t */

/* Readers (hmc.py:132-138).  hmcx_h5_list writes the root link names in name order (h5py's
 * File.keys()) separated by '\n' into buf and returns their count. */
int hmcx_h5_list(const char* path, char* buf, int64_t buf_len);
/* Rank of dataset `name` (≤ max_rank) with its dims in dims[]. */
int hmcx_h5_info(const char* path, const char* name, int64_t* dims, int max_rank);
/* Whole dataset converted to float32 into out[n_elems] (n_elems must equal its element count). */
int hmcx_h5_read_f32(const char* path, const char* name, float* out, int64_t n_elems);

/* Same, converted to float64 (integer and uint8 image data convert exactly). */
int hmcx_h5_read_f64(const char* path, const char* name, double* out, int64_t n_elems);

/* Write one fixed-shape dataset `name` of element type `type` (HMCX_H5_U8, _I64, _F32, _F64) and
 * dims[rank] from host `data` into `path` (truncate != 0: create/truncate the file; else open it
 * read-write, creating it if absent).  For data files such as the MNIST HDF5 files the
 * reference's notebooks read (benchmarks/2.-MNIST.ipynb cell 2: X_train [N,28,28], y_train [N]). */
enum { HMCX_H5_U8 = 0, HMCX_H5_I64 = 1, HMCX_H5_F32 = 2, HMCX_H5_F64 = 3 };
int hmcx_h5_write(const char* path, const char* name, int type, int rank, const int64_t* dims, const void* data,
                  int truncate);

const char* hmcx_trace_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
