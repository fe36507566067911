// hmcx_internal.h — context, workspace, kernel argument blocks (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <vector>
#include <algorithm>
#include "hmcx.h"

struct hmcx_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  std::string err;
  int graph_mode = 0;
  int sghmc_path = 0;          // 0 auto (persistent when eligible), 1 kernel-per-phase, 2 persistent only
  int num_cus = 256;
  size_t lds_max = 160 * 1024;
  // device workspace (grows; freed only after a stream sync)
  char* ws = nullptr;
  size_t ws_cap = 0;
  // pinned host staging for per-call schedules: two slots used by alternate calls, so a call only
  // waits (begin_call) for the uploads of the call before the previous one, never for the stream
  char* stage_buf[2] = {nullptr, nullptr};
  size_t stage_capv[2] = {0, 0};
  hipEvent_t stage_evv[2] = {nullptr, nullptr};
  bool stage_pend[2] = {false, false};
  int stage_cur = 0;
  size_t stage_off = 0;
  // tagged-granule arena of the fused launches (MLP MM_L23, wide SGLD forward+softmax): zeroed once,
  // one epoch per launch from a single counter, so no launch can match another's granules
  char* gx_arena = nullptr;
  size_t gx_bytes = 0;
  unsigned gx_epoch = 0;
  std::vector<int64_t> rs_poff, rs_nzo;   // row-space SGHMC: per-step projection / noise offsets
  // host schedule of the calls that draw their own (PHILOX, n_iter == u_accept == NULL)
  std::vector<double> sched_L, sched_u;
  std::vector<int32_t> sched_n;
  // launch attributes already applied (dynamic-LDS limit) and the occupancy they gave, per kernel
  std::vector<std::pair<std::pair<const void*, int>, int>> occ_cache;
  // hipGraph mode: capture happens on own_stream (the legacy default stream cannot be captured)
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  std::vector<std::pair<hipGraphExec_t, hipEvent_t>> graveyard;   // executed graphs awaiting release
  // device timing of sampler launches (hmcx_set_timing): an event pair brackets the kernels of each
  // run; pairs are collected lazily (hmcx_get_timing), so timing never serialises consecutive calls
  int timing = 0;
  hipEvent_t t_open = nullptr;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> t_pend;
  double t_ms = 0.0;
  long long t_n = 0;
  std::vector<hipEvent_t> ev_pool;     // recycled timing-capable events
  // deferred abort checks of persistent launches: the abort word is copied into a pinned slot and
  // checked once the launch's event has completed (next call, hmcx_synchronize), not by a per-call sync
  int* abort_host = nullptr;           // pinned [ABORT_SLOTS]
  int* abort_dev = nullptr;            // device word: raised by a timed-out persistent launch, sticky
  void* zeros_dev = nullptr;           // 256 zero bytes: a valid target for loads whose value is discarded
                                       // until hmcx_clear_abort (later launches return at once)
  std::vector<std::pair<hipEvent_t, int>> abort_pend;
  std::vector<std::pair<const void*, hipEvent_t>> host_marks;   // out_host block -> its latest copy's event
  std::vector<hipEvent_t> host_mark_pool;                        // spare events for new out_host blocks
  unsigned abort_next = 0;
  // fused MLP launches (hmcx_mlp.hip MM_L23): their own abort word, reported per call (out_abort)
  int* mlp_abort_dev = nullptr;
  int mlp_nofuse = 0;                  // hmcx_set_mlp_fuse(ctx, 0): the sampler runs unfused
  int wide_nofuse = 0;                 // hmcx_set_sgld_fuse(ctx, 0): wide SGLD on the three launches
  // fused wide-SGLD forward + softmax (hmcx_wide.hip k_wfwd_sm): its own abort word, never the
  // persistent SGHMC kernels' sticky one — read and lowered only by the wide call that raised it
  int* wide_abort_dev = nullptr;
  // re-runs after timed-out exchanges, by hmcx_recovery kind (hmcx_get_recoveries)
  int64_t recoveries[HMCX_RECOVERY_KINDS] = {0, 0, 0};
};
constexpr int ABORT_SLOTS = 64;
constexpr int ABORT_WORDS = 4;       // abort_dev: the word, then workgroup / granule base / epoch of the first timeout

namespace hmcx {

// softmax.py:40-41 clip bounds, exact float64 values (-log(eps), -log(1/tiny - 1)).
constexpr double CLIP_HI = 0x1.205966f2b4f12p+5;    //  36.04365338911715
constexpr double CLIP_LO = -0x1.6232bdd7abcd2p+9;   // -708.3964185322641

int set_error(hmcx_ctx* ctx, int code, const std::string& msg);

// Kernel timing: timing_begin/timing_end record events on `st` around a run's kernels;
// timing_collect folds a finished interval into (t_ms, t_n).  No-ops while timing is off.
int timing_begin(hmcx_ctx* ctx, hipStream_t st);
int timing_end(hmcx_ctx* ctx, hipStream_t st);
int timing_collect(hmcx_ctx* ctx);
// Deferred abort check of a persistent launch: copy the device abort word into a pinned slot after
// the launch (stream-ordered) and remember it; abort_poll folds completed checks (block: wait for all)
// and returns an error if any launch had aborted.
int abort_defer(hmcx_ctx* ctx, const int* dev_flag, hipStream_t st);
int abort_poll(hmcx_ctx* ctx, bool block);
int abort_precheck(hmcx_ctx* ctx);
// Grow the fused launches' granule arena to `bytes` (zeroed; stream-synchronising when it grows) and
// return the next launch epoch (never 0).
int gx_reserve(hmcx_ctx* ctx, size_t bytes);
unsigned gx_next_epoch(hmcx_ctx* ctx);
int gx_epochs(hmcx_ctx* ctx, unsigned count, unsigned* first);   // count consecutive epochs

#define HMCX_HIP(ctx, expr)                                                                  \
  do {                                                                                       \
    hipError_t e_ = (expr);                                                                  \
    if (e_ != hipSuccess)                                                                    \
      return ::hmcx::set_error((ctx), HMCX_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

// Sub-allocates one call's buffers from the context workspace (256-B aligned):
//   Workspace ws(ctx); do { ws.reset(); p = ws.take<T>(n); ... } while (ws.retry());
// retry() grows the workspace (after a stream sync) when the takes overflowed it.
struct Workspace {
  hmcx_ctx* ctx;
  size_t off = 0;
  bool failed = false;
  explicit Workspace(hmcx_ctx* c) : ctx(c) {}
  void reset() { off = 0; }
  template <typename T> T* take(size_t n) {
    const size_t bytes = ((n * sizeof(T) + 255) / 256) * 256 + 256;
    T* p = (off + bytes <= ctx->ws_cap) ? reinterpret_cast<T*>(ctx->ws + off) : nullptr;
    off += bytes;
    return p;
  }
  bool retry();
};

struct Tiling {
  int CB, NBLK, nCT, nRB, nDB;
};
Tiling make_tiling(int B, int D, int K, int C);

enum FwdMode { FWD_GRAD = 0, FWD_SGHMC = 1, FWD_LL = 2, FWD_PRED = 3 };
// GRAD_SGLD_GPU: the CuPy file's SGLD update p = ν⊙p_prev − ½ε∇U, q += p (gpu/sgld.py:11-20, A2g)
// GRAD_HMC: full-batch HMC sub-steps (cpu/hmc.py:49-54) fused into the gradient epilogue, per hmc_flags
enum GradMode { GRAD_OUT = 0, GRAD_SGHMC = 1, GRAD_SGLD = 2, GRAD_SGD = 3, GRAD_SGLD_GPU = 4, GRAD_HMC = 5 };
// After gradient evaluation k of an HMC trajectory: full kick of the variable drifted before it
// (p_v −= ε·g_v) and the half kick + drift of the next one (p_v −= ½ε·g_v; q_v += ε·p_v).
enum HmcFlags { HMC_KICK_W = 1, HMC_KICK_B = 2, HMC_HALF_W = 4, HMC_HALF_B = 8 };
// Output link of the linear model: softmax over K classes (models/cpu/softmax.py) or the
// sigmoid of K = 1 logistic regression (models/cpu/logistic.py:43-55).
enum Link { LINK_SOFTMAX = 0, LINK_SIGMOID = 1 };
// Philox slot of the input-dropout masks of sgd.fit_dropout (below the SGHMC path/accept slots).
constexpr uint32_t SLOT_DROPX = 0xFFFFFFFCu;

template <typename T> struct FwdArgs {
  const T* X; const T* Y; const T* W; const T* b; const T* pb;
  int B, D, K, C, N, CB;
  int mode;
  int link;                  // Link (FWD_SGHMC: softmax only)
  T eps, clip_hi, clip_lo;
  int iter;
  const int32_t* n_iter;
  T* diff; T* colsum_part; double* ll_part; T* prob;
  // split-K forward (few, deep tiles): slab_mode 1 = write the XW partial of D slice blockIdx.z to
  // slab[z][B][N] and stop; 2 = skip the GEMM, XW = Σ_z slab[z] (fixed order), then the epilogue
  int slab_mode, nslab;
  T* slab;
};

template <typename T> struct GradArgs {
  const T* X; const T* diff; const T* colsum_part;
  int B, D, K, C, N, CB, nRB, nDB, P;
  int mode;
  T alpha, eps, one_minus_eps, noise_scale, m_half_eps;
  T gamma, lr;               // GRAD_SGD: momentum decay and step size (sgd.py:40)
  T half_eps;                // GRAD_HMC: 0.5·ε (hmc.py:50)
  int hmc_flags;             // GRAD_HMC: HmcFlags
  int iter;
  const int32_t* n_iter;
  const T* Wsrc; const T* bsrc;
  T* W; T* b; T* pW; T* pb; T* gW; T* gb;
  double* kin_part;   // SGHMC: [nDB][C] Σ pW² of the block at the chain's last iteration
  double* kinb;       // SGHMC: [C] Σ pb² at the chain's last iteration
  int noise_mode; const double* noise; const int64_t* noff;
  uint64_t seed; uint32_t chain0, step, slot;
  T* trace;           // SGLD: out_trace row of this step ([C][P]), or null
};

// SGHMC step start: commit the previous step's accepted proposal, draw momentum, first drift.
template <typename T> struct InitArgs {
  int D, K, C, N, nDB;
  T eps;
  const int32_t* n_iter;
  const int32_t* prev_acc;   // [C] accept flags of the previous step of this call, or null
  int noise_mode; const double* noise; const int64_t* noff;
  uint64_t seed; uint32_t chain0, step;
  T* W; T* b;
  T* Wwork; T* bwork; T* pW; T* pb;
  double* kin0_part;         // [nDB][C]
  double* kin0b;             // [C]
  T* trace; int P;           // out_trace row of the PREVIOUS step ([C][P]), stored from the state it kept, or null
};

template <typename T> struct CommitArgs {
  int D, K, C, N;
  const int32_t* acc;
  const T* Wwork; const T* bwork; T* W; T* b;
  T* trace; int P;           // out_trace row of the call's last step ([C][P]), or null
};

template <typename T> struct AcceptArgs {
  int C, nRB, nDB, nDB1;     // nDB: blocks of kin0_part, nDB1: blocks of kin1_part
  const int32_t* n_iter; const double* u;
  double neg_inv_n, log_prior;
  const double* kin0_part; const double* kin0b; const double* kin1_part; const double* kin1b;
  const double* ll0_part; const double* ll1_part;
  double* out_A; int32_t* out_acc; double* out_ll; double* out_E;
};

// Copy a host array to device through the context's pinned staging buffer (stream-ordered).
int upload(hmcx_ctx* ctx, void* dst, const void* src, size_t bytes);
void begin_call(hmcx_ctx* ctx);
// Several host arrays in ONE host-to-device copy: item i lands at dst + packed_offset(i) (256-B
// aligned pieces); dst must hold packed_bytes(n, bytes).  Null / empty items are skipped.
size_t packed_bytes(int n, const size_t* bytes);
int upload_packed(hmcx_ctx* ctx, char* dst, int n, const void* const* src, const size_t* bytes, char** dev);
// hipFuncSetAttribute(max dynamic LDS) once per (kernel, lds) and the occupancy it gives (cached).
int kernel_occupancy(hmcx_ctx* ctx, const void* kfn, int threads, int lds, int* per_cu);

// Optional hipGraph capture of one run call (hmcx_set_graph_mode).
struct GraphScope {
  hmcx_ctx* ctx;
  bool capturing = false;
  hipStream_t user_stream = nullptr;
  explicit GraphScope(hmcx_ctx* c);
  int finish();
  ~GraphScope();
};

template <typename T> int softmax_grad_t(hmcx_ctx*, const void*, const void*, int, int, int, int, const void*,
                                         const void*, double, void*, void*, int link = LINK_SOFTMAX);
template <typename T> int softmax_loglik_t(hmcx_ctx*, const void*, const void*, int, int, int, int, const void*,
                                           const void*, double*, int link = LINK_SOFTMAX);
template <typename T> int softmax_predict_t(hmcx_ctx*, const void*, int, int, int, int, const void*, const void*,
                                            void*, int link = LINK_SOFTMAX);
template <typename T> int sgd_run_t(hmcx_ctx*, const hmcx_sgd_args*);
template <typename T> int sumsq_t(hmcx_ctx*, const void*, int64_t, double*);
template <typename T> int sghmc_run_t(hmcx_ctx*, const hmcx_sampler_args*);
template <typename T> int hmc_run_t(hmcx_ctx*, const hmcx_hmc_args*);
template <typename T> int axpy_t(hmcx_ctx*, int, int64_t, double, const void*, void*);
bool sghmc_p2_selected(hmcx_ctx*, const hmcx_sampler_args*);   // hmcx_softmax.hip
template <typename T> int sgld_run_t(hmcx_ctx*, const hmcx_sampler_args*);
bool sgld_wide_eligible(const hmcx_sampler_args*);       // hmcx_wide.hip: K ≤ 64 (C > 1: K > 16)
template <typename T> int sgld_wide_t(hmcx_ctx*, const hmcx_sampler_args*);
int hmc_mvn_run(hmcx_ctx*, const hmcx_hmc_mvn_args*);
int mvn_eval(hmcx_ctx*, int, int, const double*, const double*, double, const double*, double*, double*);
template <typename T> int mlp_grad_t(hmcx_ctx*, const void*, const int32_t*, int, int, int, int,
                                     const hmcx_mlp_params*, const void*, double, hmcx_mlp_params*, double*);
template <typename T> int mlp_loss_t(hmcx_ctx*, const void*, const int32_t*, int, int, int, int,
                                     const hmcx_mlp_params*, const void*, double*, void*);
template <typename T> int mlp_sghmc_t(hmcx_ctx*, const hmcx_mlp_sghmc_args*);
template <typename T> int mlp_leapfrog_t(hmcx_ctx*, const hmcx_mlp_leapfrog_args*);
template <typename T> int mlp_masks_t(hmcx_ctx*, int, int, uint64_t, uint32_t, uint32_t, uint32_t, void*);

}  // namespace hmcx
