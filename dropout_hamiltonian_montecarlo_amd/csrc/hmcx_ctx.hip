// hmcx_ctx.hip — context, workspace, staging, hipGraph capture, the C ABI (include/hmcx.h),
// and the full-batch HMC kernel for the MVN model (config 1).
#include "hmcx_common.h"
#include "hmcx_internal.h"
#include <new>
#include <cstdio>
#include <cstring>
#include <cmath>

namespace hmcx {

int set_error(hmcx_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

bool Workspace::retry() {
  if (off <= ctx->ws_cap) return false;
  if (ctx->ws) {
    if (hipDeviceSynchronize() != hipSuccess) { failed = true; return false; }
    (void)hipFree(ctx->ws);
    ctx->ws = nullptr;
    ctx->ws_cap = 0;
  }
  const size_t want = off + off / 4 + (1 << 20);
  if (hipMalloc((void**)&ctx->ws, want) != hipSuccess) {
    ctx->ws = nullptr;
    failed = true;
    set_error(ctx, HMCX_ENOMEM, "hipMalloc workspace failed");
    return false;
  }
  ctx->ws_cap = want;
  return true;
}

static int ev_take(hmcx_ctx* ctx, hipEvent_t* ev) {
  if (!ctx->ev_pool.empty()) {
    *ev = ctx->ev_pool.back();
    ctx->ev_pool.pop_back();
    return HMCX_OK;
  }
  HMCX_HIP(ctx, hipEventCreate(ev));
  return HMCX_OK;
}

int timing_collect(hmcx_ctx* ctx) {
  for (auto& pr : ctx->t_pend) {
    HMCX_HIP(ctx, hipEventSynchronize(pr.second));
    float ms = 0.f;
    HMCX_HIP(ctx, hipEventElapsedTime(&ms, pr.first, pr.second));
    ctx->t_ms += ms;
    ctx->t_n += 1;
    ctx->ev_pool.push_back(pr.first);
    ctx->ev_pool.push_back(pr.second);
  }
  ctx->t_pend.clear();
  return HMCX_OK;
}

int timing_begin(hmcx_ctx* ctx, hipStream_t st) {
  if (!ctx->timing) return HMCX_OK;
  int rc = ev_take(ctx, &ctx->t_open);
  if (rc) return rc;
  HMCX_HIP(ctx, hipEventRecord(ctx->t_open, st));
  return HMCX_OK;
}

int timing_end(hmcx_ctx* ctx, hipStream_t st) {
  if (!ctx->timing || !ctx->t_open) return HMCX_OK;
  hipEvent_t e1 = nullptr;
  int rc = ev_take(ctx, &e1);
  if (rc) return rc;
  HMCX_HIP(ctx, hipEventRecord(e1, st));
  ctx->t_pend.emplace_back(ctx->t_open, e1);
  ctx->t_open = nullptr;
  return HMCX_OK;
}

int abort_poll(hmcx_ctx* ctx, bool block) {
  bool aborted = false;
  size_t keep = 0;
  for (size_t i = 0; i < ctx->abort_pend.size(); ++i) {
    auto pr = ctx->abort_pend[i];
    hipError_t e = block ? hipEventSynchronize(pr.first) : hipEventQuery(pr.first);
    if (e == hipErrorNotReady) {
      ctx->abort_pend[keep++] = pr;
      continue;
    }
    if (e != hipSuccess) return set_error(ctx, HMCX_EHIP, std::string("abort check: ") + hipGetErrorString(e));
    if (ctx->abort_host[pr.second]) aborted = true;
    ctx->ev_pool.push_back(pr.first);
  }
  ctx->abort_pend.resize(keep);
  if (aborted) return set_error(ctx, HMCX_EHIP, "persistent SGHMC: hand-off timed out (workgroups not co-resident?)");
  return HMCX_OK;
}

int abort_precheck(hmcx_ctx* ctx) {
  // earlier launches that have finished (all of them when too many checks are in flight): an abort
  // is reported here, before the caller enqueues anything
  return abort_poll(ctx, ctx->abort_pend.size() >= (size_t)ABORT_SLOTS / 2);
}

int abort_defer(hmcx_ctx* ctx, const int* dev_flag, hipStream_t st) {
  if (!ctx->abort_host) HMCX_HIP(ctx, hipHostMalloc((void**)&ctx->abort_host, ABORT_SLOTS * sizeof(int), hipHostMallocDefault));
  const int slot = (int)(ctx->abort_next++ % ABORT_SLOTS);
  hipEvent_t ev = nullptr;
  int rc = ev_take(ctx, &ev);
  if (rc) return rc;
  HMCX_HIP(ctx, hipMemcpyAsync(ctx->abort_host + slot, dev_flag, sizeof(int), hipMemcpyDeviceToHost, st));
  HMCX_HIP(ctx, hipEventRecord(ev, st));
  ctx->abort_pend.emplace_back(ev, slot);
  return HMCX_OK;          // checked before the next launch (abort_precheck) or by hmcx_synchronize
}

int gx_reserve(hmcx_ctx* ctx, size_t bytes) {
  if (ctx->gx_bytes >= bytes) return HMCX_OK;
  HMCX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (ctx->gx_arena) (void)hipFree(ctx->gx_arena);
  ctx->gx_arena = nullptr;
  ctx->gx_bytes = 0;
  HMCX_HIP(ctx, hipMalloc((void**)&ctx->gx_arena, bytes));
  HMCX_HIP(ctx, hipMemset(ctx->gx_arena, 0, bytes));          // epoch 0 never matches a launch
  ctx->gx_bytes = bytes;
  return HMCX_OK;
}

// Epochs are unique over the arena's life: a launch polls only for epochs no earlier launch wrote,
// so the arena needs no clearing between launches.  When the 32-bit counter would wrap, the arena is
// cleared on the stream (behind every earlier user) and the count restarts at 1.
int gx_epochs(hmcx_ctx* ctx, unsigned count, unsigned* first) {
  if (count == 0) count = 1;
  if ((uint64_t)ctx->gx_epoch + count > 0xffffffffull) {
    if (ctx->gx_arena) HMCX_HIP(ctx, hipMemsetAsync(ctx->gx_arena, 0, ctx->gx_bytes, ctx->stream));
    ctx->gx_epoch = 0;
  }
  *first = ctx->gx_epoch + 1;
  ctx->gx_epoch += count;
  return HMCX_OK;
}

unsigned gx_next_epoch(hmcx_ctx* ctx) {
  unsigned ep = 1;
  (void)gx_epochs(ctx, 1, &ep);
  return ep;
}

void begin_call(hmcx_ctx* ctx) {
  ctx->stage_cur ^= 1;
  const int c = ctx->stage_cur;
  if (ctx->stage_pend[c]) {                     // uploads of the call before the previous one
    (void)hipEventSynchronize(ctx->stage_evv[c]);
    ctx->stage_pend[c] = false;
  }
  ctx->stage_off = 0;
}

static int stage_reserve(hmcx_ctx* ctx, size_t bytes, char** h) {
  const int c = ctx->stage_cur;
  const size_t need = ctx->stage_off + ((bytes + 255) / 256) * 256;
  if (need > ctx->stage_capv[c]) {
    // a grown staging buffer invalidates earlier offsets of this call: drain the stream first.  Both
    // slots grow together (pinned allocations cost hundreds of µs: not inside the next call too)
    HMCX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    const size_t cap = std::max(need * 2, (size_t)1 << 20);
    for (int i = 0; i < 2; ++i) {
      if (ctx->stage_capv[i] >= cap) continue;
      if (ctx->stage_pend[i]) {
        HMCX_HIP(ctx, hipEventSynchronize(ctx->stage_evv[i]));
        ctx->stage_pend[i] = false;
      }
      char* nb = nullptr;
      HMCX_HIP(ctx, hipHostMalloc((void**)&nb, cap, hipHostMallocDefault));
      if (ctx->stage_buf[i]) (void)hipHostFree(ctx->stage_buf[i]);
      ctx->stage_buf[i] = nb;
      ctx->stage_capv[i] = cap;
      if (!ctx->stage_evv[i]) HMCX_HIP(ctx, hipEventCreateWithFlags(&ctx->stage_evv[i], hipEventDisableTiming));
    }
    ctx->stage_off = 0;
  }
  *h = ctx->stage_buf[c] + ctx->stage_off;
  ctx->stage_off += ((bytes + 255) / 256) * 256;
  return HMCX_OK;
}

static int stage_copy(hmcx_ctx* ctx, void* dst, const char* h, size_t bytes) {
  const int c = ctx->stage_cur;
  HMCX_HIP(ctx, hipMemcpyAsync(dst, h, bytes, hipMemcpyHostToDevice, ctx->stream));
  HMCX_HIP(ctx, hipEventRecord(ctx->stage_evv[c], ctx->stream));
  ctx->stage_pend[c] = true;
  return HMCX_OK;
}

int upload(hmcx_ctx* ctx, void* dst, const void* src, size_t bytes) {
  if (bytes == 0) return HMCX_OK;
  if (!src) return set_error(ctx, HMCX_EINVAL, "upload: null host array");
  char* h = nullptr;
  int rc = stage_reserve(ctx, bytes, &h);
  if (rc) return rc;
  std::memcpy(h, src, bytes);
  return stage_copy(ctx, dst, h, bytes);
}

size_t packed_bytes(int n, const size_t* bytes) {
  size_t t = 0;
  for (int i = 0; i < n; ++i) t += ((bytes[i] + 255) / 256) * 256;
  return t;
}

int upload_packed(hmcx_ctx* ctx, char* dst, int n, const void* const* src, const size_t* bytes, char** dev) {
  const size_t total = packed_bytes(n, bytes);
  size_t off = 0;
  for (int i = 0; i < n; ++i) {
    dev[i] = dst + off;
    off += ((bytes[i] + 255) / 256) * 256;
  }
  if (total == 0) return HMCX_OK;
  char* h = nullptr;
  int rc = stage_reserve(ctx, total, &h);
  if (rc) return rc;
  for (int i = 0; i < n; ++i)
    if (bytes[i] && src[i]) std::memcpy(h + (dev[i] - dst), src[i], bytes[i]);
  return stage_copy(ctx, dst, h, total);
}

int kernel_occupancy(hmcx_ctx* ctx, const void* kfn, int threads, int lds, int* per_cu) {
  for (auto& e : ctx->occ_cache)
    if (e.first.first == kfn && e.first.second == lds) { *per_cu = e.second; return HMCX_OK; }
  HMCX_HIP(ctx, hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  int occ = 0;
  HMCX_HIP(ctx, hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kfn, threads, lds));
  ctx->occ_cache.push_back({{kfn, lds}, occ});
  *per_cu = occ;
  return HMCX_OK;
}

GraphScope::GraphScope(hmcx_ctx* c) : ctx(c) {
  if (!ctx->graph_mode) return;
  // fork: own_stream waits for everything already queued on the caller's stream
  user_stream = ctx->stream;
  if (hipEventRecord(ctx->ev_in, user_stream) != hipSuccess) return;
  if (hipStreamWaitEvent(ctx->own_stream, ctx->ev_in, 0) != hipSuccess) return;
  if (hipStreamBeginCapture(ctx->own_stream, hipStreamCaptureModeThreadLocal) != hipSuccess) return;
  ctx->stream = ctx->own_stream;
  capturing = true;
}

static void sweep_graveyard(hmcx_ctx* ctx) {
  auto& g = ctx->graveyard;
  for (size_t i = 0; i < g.size();) {
    if (hipEventQuery(g[i].second) == hipSuccess) {
      (void)hipGraphExecDestroy(g[i].first);
      (void)hipEventDestroy(g[i].second);
      g[i] = g.back();
      g.pop_back();
    } else {
      ++i;
    }
  }
}

int GraphScope::finish() {
  if (!capturing) return HMCX_OK;
  capturing = false;
  ctx->stream = user_stream;
  hipGraph_t graph = nullptr;
  HMCX_HIP(ctx, hipStreamEndCapture(ctx->own_stream, &graph));
  hipGraphExec_t exec = nullptr;
  hipError_t e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
  (void)hipGraphDestroy(graph);
  if (e != hipSuccess) return set_error(ctx, HMCX_EHIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(e));
  e = hipGraphLaunch(exec, ctx->own_stream);
  if (e != hipSuccess) {
    (void)hipGraphExecDestroy(exec);
    return set_error(ctx, HMCX_EHIP, std::string("hipGraphLaunch: ") + hipGetErrorString(e));
  }
  // join: the caller's stream waits for the graph; the exec is released once it has run
  hipEvent_t done = nullptr;
  HMCX_HIP(ctx, hipEventCreateWithFlags(&done, hipEventDisableTiming));
  HMCX_HIP(ctx, hipEventRecord(done, ctx->own_stream));
  HMCX_HIP(ctx, hipStreamWaitEvent(user_stream, done, 0));
  ctx->graveyard.emplace_back(exec, done);
  sweep_graveyard(ctx);
  return HMCX_OK;
}

GraphScope::~GraphScope() {
  if (capturing) {
    hipGraph_t g = nullptr;
    (void)hipStreamEndCapture(ctx->own_stream, &g);
    if (g) (void)hipGraphDestroy(g);
    ctx->stream = user_stream;
  }
}

// ------------------------------------------------------------------ MVN full-batch HMC
// cpu/hmc.py:39-71 with mvn_gaussian.py:14-31, one thread per chain, all steps in one launch.
struct MvnArgs {
  int dim, C, n_steps;
  const double* mu; const double* prec; double nlp_const;
  const double* eps; const int32_t* n_iter; const double* u;
  int noise_mode; const double* noise; const int64_t* noff;
  uint64_t seed; uint32_t chain0, step_base;
  double* x; double* out_A; int32_t* out_acc; double* out_nlp; double* out_trace;
};
constexpr int MVN_MAXDIM = 16;

__device__ inline void mvn_grad(const MvnArgs& a, const double* x, double* g) {
  double dm[MVN_MAXDIM];
  for (int i = 0; i < a.dim; ++i) dm[i] = x[i] - a.mu[i];
  for (int j = 0; j < a.dim; ++j) {                     // np.dot(x - mu, inv(cov))
    double s = dm[0] * a.prec[j];
    for (int i = 1; i < a.dim; ++i) s = s + dm[i] * a.prec[i * a.dim + j];
    g[j] = s;
  }
}

__device__ inline double mvn_nlp(const MvnArgs& a, const double* x) {
  double dm[MVN_MAXDIM], v[MVN_MAXDIM];
  for (int i = 0; i < a.dim; ++i) dm[i] = x[i] - a.mu[i];
  for (int j = 0; j < a.dim; ++j) {
    double s = dm[0] * a.prec[j];
    for (int i = 1; i < a.dim; ++i) s = s + dm[i] * a.prec[i * a.dim + j];
    v[j] = s;
  }
  double q = v[0] * dm[0];
  for (int j = 1; j < a.dim; ++j) q = q + v[j] * dm[j];
  return (a.nlp_const + q) * 0.5;                        // mvn_gaussian.py:27-30
}

__global__ void k_hmc_mvn(MvnArgs a) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.C) return;
  double x[MVN_MAXDIM], xn[MVN_MAXDIM], p[MVN_MAXDIM], p0[MVN_MAXDIM], g[MVN_MAXDIM];
  for (int j = 0; j < a.dim; ++j) x[j] = a.x[c * a.dim + j];
  for (int s = 0; s < a.n_steps; ++s) {
    const double eps = a.eps[s];
    const int n = a.n_iter[(size_t)s * a.C + c];
    for (int j = 0; j < a.dim; ++j) {
      double z;
      if (a.noise_mode == HMCX_NOISE_BUFFER) z = a.noise[a.noff[(size_t)s * a.C + c] + j];
      else z = philox_normal_d(a.seed, a.chain0 + c, a.step_base + s, 0u, (uint32_t)j);
      p0[j] = z; p[j] = z; xn[j] = x[j];
    }
    mvn_grad(a, x, g);                                   // hmc.py:47
    const double half = 0.5 * eps;
    for (int it = 0; it < n; ++it) {                     // hmc.py:49-54 (one var)
      for (int j = 0; j < a.dim; ++j) p[j] = p[j] - half * g[j];
      for (int j = 0; j < a.dim; ++j) xn[j] = xn[j] + eps * p[j];
      mvn_grad(a, xn, g);
      for (int j = 0; j < a.dim; ++j) p[j] = p[j] - eps * g[j];
    }
    double k1 = 0.0, k0 = 0.0;
    for (int j = 0; j < a.dim; ++j) { p[j] = -p[j]; k1 += p[j] * p[j]; k0 += p0[j] * p0[j]; }
    const double Enew = mvn_nlp(a, xn) + (0.0 + 0.5 * k1);
    const double Ecur = mvn_nlp(a, x) + (0.0 + 0.5 * k0);
    const double ex = exp(Ecur - Enew);
    const double A = (ex < 1.0) ? ex : 1.0;
    const int acc = a.u[(size_t)s * a.C + c] < A;
    if (acc) for (int j = 0; j < a.dim; ++j) x[j] = xn[j];
    a.out_A[(size_t)s * a.C + c] = A;
    a.out_acc[(size_t)s * a.C + c] = acc;
    if (a.out_nlp) a.out_nlp[(size_t)s * a.C + c] = mvn_nlp(a, x);
    if (a.out_trace)
      for (int j = 0; j < a.dim; ++j) a.out_trace[((size_t)s * a.C + c) * a.dim + j] = x[j];
  }
  for (int j = 0; j < a.dim; ++j) a.x[c * a.dim + j] = x[j];
}

// Per-call MVN surface (mvn_gaussian.py:14-31): one thread per parameter set.
__global__ void k_mvn_eval(MvnArgs a, const double* x, double* g, double* nlp) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.C) return;
  double xv[MVN_MAXDIM], gv[MVN_MAXDIM];
  for (int j = 0; j < a.dim; ++j) xv[j] = x[c * a.dim + j];
  if (g) {
    mvn_grad(a, xv, gv);
    for (int j = 0; j < a.dim; ++j) g[c * a.dim + j] = gv[j];
  }
  if (nlp) nlp[c] = mvn_nlp(a, xv);
}

int mvn_eval(hmcx_ctx* ctx, int dim, int C, const double* mu, const double* prec, double nlp_const, const double* x,
             double* g, double* nlp) {
  if (dim < 1 || dim > MVN_MAXDIM) return set_error(ctx, HMCX_EUNSUPPORTED, "mvn: dim must be 1..16");
  MvnArgs a{};
  a.dim = dim; a.C = C; a.mu = mu; a.prec = prec; a.nlp_const = nlp_const;
  hipLaunchKernelGGL(k_mvn_eval, dim3((C + 63) / 64), dim3(64), 0, ctx->stream, a, x, g, nlp);
  HMCX_HIP(ctx, hipGetLastError());
  return HMCX_OK;
}

int hmc_mvn_run(hmcx_ctx* ctx, const hmcx_hmc_mvn_args* s) {
  if (s->dim < 1 || s->dim > MVN_MAXDIM) return set_error(ctx, HMCX_EUNSUPPORTED, "mvn: dim must be 1..16");
  const size_t nsc = (size_t)s->n_steps * s->C;
  Workspace ws(ctx);
  double *d_eps, *d_u;
  int32_t* d_n;
  int64_t* d_off;
  do {
    ws.reset();
    d_eps = ws.take<double>(s->n_steps);
    d_u = ws.take<double>(nsc);
    d_n = ws.take<int32_t>(nsc);
    d_off = ws.take<int64_t>(nsc);
  } while (ws.retry());
  if (ws.failed) return HMCX_ENOMEM;
  begin_call(ctx);
  int rc;
  if ((rc = upload(ctx, d_eps, s->eps, s->n_steps * sizeof(double)))) return rc;
  if ((rc = upload(ctx, d_u, s->u_accept, nsc * sizeof(double)))) return rc;
  if ((rc = upload(ctx, d_n, s->n_iter, nsc * sizeof(int32_t)))) return rc;
  if (s->noise_mode == HMCX_NOISE_BUFFER && (rc = upload(ctx, d_off, s->noise_off, nsc * sizeof(int64_t))))
    return rc;
  MvnArgs a{};
  a.dim = s->dim; a.C = s->C; a.n_steps = s->n_steps;
  a.mu = s->mu; a.prec = s->prec; a.nlp_const = s->nlp_const;
  a.eps = d_eps; a.n_iter = d_n; a.u = d_u;
  a.noise_mode = s->noise_mode; a.noise = s->noise; a.noff = d_off;
  a.seed = s->seed; a.chain0 = s->chain0; a.step_base = s->step_base;
  a.x = s->x; a.out_A = s->out_A; a.out_acc = s->out_accepted; a.out_nlp = s->out_nlp; a.out_trace = s->out_trace;
  hipLaunchKernelGGL(k_hmc_mvn, dim3((s->C + 63) / 64), dim3(64), 0, ctx->stream, a);
  HMCX_HIP(ctx, hipGetLastError());
  return HMCX_OK;
}

// An event behind the copies into an out_host block (one reusable, non-timing event per block).
static int host_mark(hmcx_ctx* ctx, const void* out_host) {
  hipEvent_t ev = nullptr;
  for (auto& m : ctx->host_marks)
    if (m.first == out_host) { ev = m.second; break; }
  if (!ev) {
    // events for the next blocks are created with the first one (a caller's first call on each of
    // its output blocks then creates nothing inside its timed region)
    if (ctx->host_marks.empty())
      for (int i = 0; i < 8; ++i) {
        hipEvent_t e = nullptr;
        HMCX_HIP(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ctx->host_mark_pool.push_back(e);
      }
    if (!ctx->host_mark_pool.empty()) {
      ev = ctx->host_mark_pool.back();
      ctx->host_mark_pool.pop_back();
    } else {
      HMCX_HIP(ctx, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    }
    ctx->host_marks.emplace_back(out_host, ev);
  }
  HMCX_HIP(ctx, hipEventRecord(ev, ctx->stream));
  return HMCX_OK;
}

}  // namespace hmcx

// =================================================================== C ABI
using namespace hmcx;

#define HMCX_GUARD_CTX(ctx) \
  if (!(ctx)) return HMCX_EINVAL;

extern "C" {

int hmcx_version(void) { return 10000; }

int hmcx_create(int device, hmcx_ctx** out) {
  if (!out) return HMCX_EINVAL;
  *out = nullptr;
  hmcx_ctx* c = new (std::nothrow) hmcx_ctx();
  if (!c) return HMCX_ENOMEM;
  c->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming) != hipSuccess) {
    delete c;
    return HMCX_EHIP;
  }
  c->stream = c->own_stream;
  // the abort word and, after it, where the first timeout happened (hmcx_p2x.h p2_timeout)
  if (hipMalloc((void**)&c->abort_dev, ABORT_WORDS * sizeof(int)) != hipSuccess ||
      hipMemset(c->abort_dev, 0, ABORT_WORDS * sizeof(int)) != hipSuccess) {
    delete c;
    return HMCX_EHIP;
  }
  if (hipMalloc(&c->zeros_dev, 256) != hipSuccess || hipMemset(c->zeros_dev, 0, 256) != hipSuccess) {
    (void)hipFree(c->abort_dev);
    delete c;
    return HMCX_EHIP;
  }
  int ncu = 0, lds = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0)
    c->num_cus = ncu;
  if (hipDeviceGetAttribute(&lds, hipDeviceAttributeSharedMemPerBlockOptin, device) == hipSuccess && lds > 0)
    c->lds_max = (size_t)lds;
  // the Philox schedule of a call is drawn into these: sized for a whole epoch of steps up front, so
  // a call does not reallocate them (the first call of a new, larger step count did)
  c->sched_L.reserve(4096);
  c->sched_n.reserve(4096);
  c->sched_u.reserve(4096);
  *out = c;
  return HMCX_OK;
}

int hmcx_destroy(hmcx_ctx* ctx) {
  HMCX_GUARD_CTX(ctx);
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  if (ctx->ws) (void)hipFree(ctx->ws);
  for (int i = 0; i < 2; ++i) {
    if (ctx->stage_buf[i]) (void)hipHostFree(ctx->stage_buf[i]);
    if (ctx->stage_evv[i]) (void)hipEventDestroy(ctx->stage_evv[i]);
  }
  if (ctx->ev_in) (void)hipEventDestroy(ctx->ev_in);
  for (auto& pr : ctx->t_pend) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
  if (ctx->t_open) (void)hipEventDestroy(ctx->t_open);
  for (auto& pr : ctx->abort_pend) (void)hipEventDestroy(pr.first);
  for (auto e : ctx->ev_pool) (void)hipEventDestroy(e);
  for (auto& m : ctx->host_marks) (void)hipEventDestroy(m.second);
  for (auto e : ctx->host_mark_pool) (void)hipEventDestroy(e);
  if (ctx->abort_host) (void)hipHostFree(ctx->abort_host);
  if (ctx->abort_dev) (void)hipFree(ctx->abort_dev);
  if (ctx->mlp_abort_dev) (void)hipFree(ctx->mlp_abort_dev);
  if (ctx->wide_abort_dev) (void)hipFree(ctx->wide_abort_dev);
  if (ctx->zeros_dev) (void)hipFree(ctx->zeros_dev);
  if (ctx->gx_arena) (void)hipFree(ctx->gx_arena);
  for (auto& g : ctx->graveyard) {
    (void)hipGraphExecDestroy(g.first);
    (void)hipEventDestroy(g.second);
  }
  if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
  delete ctx;
  return HMCX_OK;
}

const char* hmcx_last_error(const hmcx_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int hmcx_set_stream(hmcx_ctx* ctx, void* stream) {
  HMCX_GUARD_CTX(ctx);
  ctx->stream = (hipStream_t)stream;   // NULL = the legacy default stream (torch's default)
  return HMCX_OK;
}

int hmcx_synchronize(hmcx_ctx* ctx) {
  HMCX_GUARD_CTX(ctx);
  HMCX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return abort_poll(ctx, true);                    // reports an aborted persistent launch
}

int hmcx_clear_abort(hmcx_ctx* ctx) {
  HMCX_GUARD_CTX(ctx);
  for (auto& pr : ctx->abort_pend) ctx->ev_pool.push_back(pr.first);
  ctx->abort_pend.clear();
  static const bool dbg = getenv("HMCX_P2_DEBUG") && getenv("HMCX_P2_DEBUG")[0] == '1';
  if (dbg) {                                        // where the first timeout happened
    int w[ABORT_WORDS];
    HMCX_HIP(ctx, hipMemcpyAsync(w, ctx->abort_dev, sizeof(w), hipMemcpyDeviceToHost, ctx->stream));
    HMCX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    fprintf(stderr, "[hmcx] abort word %d; first timeout: workgroup %d, granule base %d, epoch %d\n", w[0], w[1] - 1,
            w[2], w[3]);
  }
  HMCX_HIP(ctx, hipMemsetAsync(ctx->abort_dev, 0, ABORT_WORDS * sizeof(int), ctx->stream));
  return HMCX_OK;                                   // the re-runs themselves are counted by the caller
}

int hmcx_get_recoveries(const hmcx_ctx* ctx, int64_t* counts) {
  if (!ctx || !counts) return HMCX_EINVAL;
  for (int k = 0; k < HMCX_RECOVERY_KINDS; ++k) counts[k] = ctx->recoveries[k];
  return HMCX_OK;
}

int hmcx_note_recovery(hmcx_ctx* ctx, int kind) {
  HMCX_GUARD_CTX(ctx);
  if (kind < 0 || kind >= HMCX_RECOVERY_KINDS) return set_error(ctx, HMCX_EINVAL, "unknown recovery kind");
  ++ctx->recoveries[kind];
  return HMCX_OK;
}

int hmcx_set_sghmc_path(hmcx_ctx* ctx, int path) {
  HMCX_GUARD_CTX(ctx);
  if (path < 0 || path > 2)
    return set_error(ctx, HMCX_EINVAL, "path must be 0 (auto), 1 (kernels), 2 (persistent)");
  ctx->sghmc_path = path;
  return HMCX_OK;
}

int hmcx_set_mlp_fuse(hmcx_ctx* ctx, int on) {
  HMCX_GUARD_CTX(ctx);
  ctx->mlp_nofuse = on ? 0 : 1;
  return HMCX_OK;
}

int hmcx_set_sgld_fuse(hmcx_ctx* ctx, int on) {
  HMCX_GUARD_CTX(ctx);
  ctx->wide_nofuse = on ? 0 : 1;
  return HMCX_OK;
}

int hmcx_set_graph_mode(hmcx_ctx* ctx, int enabled) {
  HMCX_GUARD_CTX(ctx);
  ctx->graph_mode = enabled ? 1 : 0;
  return HMCX_OK;
}

int hmcx_set_timing(hmcx_ctx* ctx, int enabled) {
  HMCX_GUARD_CTX(ctx);
  int rc = timing_collect(ctx);                    // drain (and discard) pending intervals
  if (rc) return rc;
  ctx->timing = enabled ? 1 : 0;
  ctx->t_ms = 0.0;
  ctx->t_n = 0;
  // event creation costs tens of µs: create the timed runs' events here, not inside the first run
  while (enabled && ctx->ev_pool.size() < 8) {
    hipEvent_t ev = nullptr;
    HMCX_HIP(ctx, hipEventCreate(&ev));
    ctx->ev_pool.push_back(ev);
  }
  return HMCX_OK;
}

int hmcx_get_timing(hmcx_ctx* ctx, double* kernel_ms, long long* launches) {
  HMCX_GUARD_CTX(ctx);
  if (!kernel_ms || !launches) return set_error(ctx, HMCX_EINVAL, "hmcx_get_timing: null output");
  int rc = timing_collect(ctx);
  if (rc) return rc;
  *kernel_ms = ctx->t_ms;
  *launches = ctx->t_n;
  return HMCX_OK;
}

void hmcx_philox_uniforms(uint64_t seed, uint32_t chain, uint32_t step, uint32_t slot, uint32_t n, double* out) {
  for (uint32_t i = 0; i < n; ++i) out[i] = philox_uniform(seed, chain, step, slot, i);
}

void hmcx_philox_normals(uint64_t seed, uint32_t chain, uint32_t step, uint32_t slot, uint32_t e0, uint32_t n,
                         double* out) {
  for (uint32_t i = 0; i < n; ++i) out[i] = philox_normal(seed, chain, step, slot, e0 + i);
}

void hmcx_philox_normals_f64(uint64_t seed, uint32_t chain, uint32_t step, uint32_t slot, uint32_t e0, uint32_t n,
                             double* out) {
  for (uint32_t i = 0; i < n; ++i) out[i] = philox_normal_d(seed, chain, step, slot, e0 + i);
}

int hmcx_philox_schedule(uint64_t seed, uint32_t chain0, int C, uint32_t step_base, int n_steps, double path_length,
                         const double* eps, double* L, int32_t* n_iter, double* u) {
  if (C < 1 || n_steps < 0 || !eps || !L || !n_iter || !u) return HMCX_EINVAL;
  for (int s = 0; s < n_steps; ++s) {
    const uint32_t st = step_base + (uint32_t)s;
    for (int c = 0; c < C; ++c) {
      const size_t i = (size_t)s * C + c;
      const double l = std::ceil(2.0 * philox_uniform(seed, chain0 + (uint32_t)c, st, SLOT_PATH, 0) *
                                 path_length / eps[s]);
      if (!std::isfinite(l) || l > 2147483647.0) return HMCX_EINVAL;
      L[i] = l;
      n_iter[i] = l - 1.0 > 0.0 ? (int32_t)std::ceil(l - 1.0) : 0;
      u[i] = philox_uniform(seed, chain0 + (uint32_t)c, st, SLOT_ACCEPT, 0);
    }
  }
  return HMCX_OK;
}

static int check_dims(hmcx_ctx* ctx, int dtype, int B, int D, int K, int C) {
  if (dtype != HMCX_F32 && dtype != HMCX_F64) return set_error(ctx, HMCX_EINVAL, "dtype must be HMCX_F32/HMCX_F64");
  if (B < 1 || D < 1 || K < 1 || C < 1) return set_error(ctx, HMCX_EINVAL, "B, D, K, C must be >= 1");
  if (K > 64) return set_error(ctx, HMCX_EUNSUPPORTED, "K > 64 classes not built");
  return HMCX_OK;
}

int hmcx_softmax_grad(hmcx_ctx* ctx, int dtype, const void* X, const void* Y, int B, int D, int K, int C,
                      const void* W, const void* b, double alpha, void* gW, void* gb) {
  HMCX_GUARD_CTX(ctx);
  int rc = check_dims(ctx, dtype, B, D, K, C);
  if (rc) return rc;
  if (!X || !Y || !W || !b || !gW || !gb) return set_error(ctx, HMCX_EINVAL, "null pointer");
  return dtype == HMCX_F64 ? softmax_grad_t<double>(ctx, X, Y, B, D, K, C, W, b, alpha, gW, gb)
                           : softmax_grad_t<float>(ctx, X, Y, B, D, K, C, W, b, alpha, gW, gb);
}

int hmcx_softmax_loglik(hmcx_ctx* ctx, int dtype, const void* X, const void* Y, int B, int D, int K, int C,
                        const void* W, const void* b, double* ll) {
  HMCX_GUARD_CTX(ctx);
  int rc = check_dims(ctx, dtype, B, D, K, C);
  if (rc) return rc;
  if (!X || !Y || !W || !b || !ll) return set_error(ctx, HMCX_EINVAL, "null pointer");
  return dtype == HMCX_F64 ? softmax_loglik_t<double>(ctx, X, Y, B, D, K, C, W, b, ll)
                           : softmax_loglik_t<float>(ctx, X, Y, B, D, K, C, W, b, ll);
}

int hmcx_softmax_predict(hmcx_ctx* ctx, int dtype, const void* X, int B, int D, int K, int C, const void* W,
                         const void* b, void* prob) {
  HMCX_GUARD_CTX(ctx);
  int rc = check_dims(ctx, dtype, B, D, K, C);
  if (rc) return rc;
  if (!X || !W || !b || !prob) return set_error(ctx, HMCX_EINVAL, "null pointer");
  return dtype == HMCX_F64 ? softmax_predict_t<double>(ctx, X, B, D, K, C, W, b, prob)
                           : softmax_predict_t<float>(ctx, X, B, D, K, C, W, b, prob);
}

int hmcx_logistic_grad(hmcx_ctx* ctx, int dtype, const void* X, const void* y, int B, int D, int C,
                       const void* W, const void* b, double alpha, void* gW, void* gb) {
  HMCX_GUARD_CTX(ctx);
  int rc = check_dims(ctx, dtype, B, D, 1, C);
  if (rc) return rc;
  if (!X || !y || !W || !b || !gW || !gb) return set_error(ctx, HMCX_EINVAL, "null pointer");
  return dtype == HMCX_F64 ? softmax_grad_t<double>(ctx, X, y, B, D, 1, C, W, b, alpha, gW, gb, LINK_SIGMOID)
                           : softmax_grad_t<float>(ctx, X, y, B, D, 1, C, W, b, alpha, gW, gb, LINK_SIGMOID);
}

int hmcx_logistic_loglik(hmcx_ctx* ctx, int dtype, const void* X, const void* y, int B, int D, int C,
                         const void* W, const void* b, double* ll) {
  HMCX_GUARD_CTX(ctx);
  int rc = check_dims(ctx, dtype, B, D, 1, C);
  if (rc) return rc;
  if (!X || !y || !W || !b || !ll) return set_error(ctx, HMCX_EINVAL, "null pointer");
  return dtype == HMCX_F64 ? softmax_loglik_t<double>(ctx, X, y, B, D, 1, C, W, b, ll, LINK_SIGMOID)
                           : softmax_loglik_t<float>(ctx, X, y, B, D, 1, C, W, b, ll, LINK_SIGMOID);
}

int hmcx_logistic_predict(hmcx_ctx* ctx, int dtype, const void* X, int B, int D, int C, const void* W,
                          const void* b, void* prob) {
  HMCX_GUARD_CTX(ctx);
  int rc = check_dims(ctx, dtype, B, D, 1, C);
  if (rc) return rc;
  if (!X || !W || !b || !prob) return set_error(ctx, HMCX_EINVAL, "null pointer");
  return dtype == HMCX_F64 ? softmax_predict_t<double>(ctx, X, B, D, 1, C, W, b, prob, LINK_SIGMOID)
                           : softmax_predict_t<float>(ctx, X, B, D, 1, C, W, b, prob, LINK_SIGMOID);
}

int hmcx_sumsq(hmcx_ctx* ctx, int dtype, const void* x, int64_t n, double* out) {
  HMCX_GUARD_CTX(ctx);
  if (dtype != HMCX_F32 && dtype != HMCX_F64) return set_error(ctx, HMCX_EINVAL, "dtype must be HMCX_F32/HMCX_F64");
  if (n < 0 || (n > 0 && !x) || !out) return set_error(ctx, HMCX_EINVAL, "hmcx_sumsq: bad arguments");
  return dtype == HMCX_F64 ? sumsq_t<double>(ctx, x, n, out) : sumsq_t<float>(ctx, x, n, out);
}

int hmcx_hmc_run(hmcx_ctx* ctx, const hmcx_hmc_args* a) {
  HMCX_GUARD_CTX(ctx);
  if (!a) return set_error(ctx, HMCX_EINVAL, "null args");
  if (a->model != HMCX_MODEL_SOFTMAX && a->model != HMCX_MODEL_LOGISTIC)
    return set_error(ctx, HMCX_EINVAL, "hmc: model must be HMCX_MODEL_SOFTMAX or HMCX_MODEL_LOGISTIC");
  if (a->model == HMCX_MODEL_LOGISTIC && a->K != 1) return set_error(ctx, HMCX_EINVAL, "hmc: logistic needs K = 1");
  int rc = check_dims(ctx, a->dtype, a->B, a->D, a->K, 1);
  if (rc) return rc;
  if (a->n_steps < 0) return set_error(ctx, HMCX_EINVAL, "n_steps < 0");
  if (a->n_steps == 0) return HMCX_OK;
  if (!a->X || !a->Y || !a->W || !a->b || !a->eps || !a->n_iter || !a->u_accept || !a->out_A || !a->out_accepted ||
      !a->out_nlp)
    return set_error(ctx, HMCX_EINVAL, "null pointer");
  if (a->noise_mode == HMCX_NOISE_BUFFER && (!a->noise || !a->noise_off))
    return set_error(ctx, HMCX_EINVAL, "BUFFER noise needs noise and noise_off");
  if (a->noise_mode != HMCX_NOISE_BUFFER && a->noise_mode != HMCX_NOISE_PHILOX)
    return set_error(ctx, HMCX_EINVAL, "bad noise_mode");
  for (int i = 0; i < a->n_steps; ++i)
    if (a->n_iter[i] < 0) return set_error(ctx, HMCX_EINVAL, "n_iter < 0");
  return a->dtype == HMCX_F64 ? hmc_run_t<double>(ctx, a) : hmc_run_t<float>(ctx, a);
}

int hmcx_mvn_eval(hmcx_ctx* ctx, int dim, int C, const double* mu, const double* prec, double nlp_const,
                  const double* x, double* g, double* nlp) {
  HMCX_GUARD_CTX(ctx);
  if (C < 1 || !mu || !prec || !x || (!g && !nlp)) return set_error(ctx, HMCX_EINVAL, "hmcx_mvn_eval: bad arguments");
  return mvn_eval(ctx, dim, C, mu, prec, nlp_const, x, g, nlp);
}

int hmcx_axpy(hmcx_ctx* ctx, int dtype, int mode, int64_t n, double a, const void* x, void* y) {
  HMCX_GUARD_CTX(ctx);
  if (dtype != HMCX_F32 && dtype != HMCX_F64) return set_error(ctx, HMCX_EINVAL, "dtype must be HMCX_F32/HMCX_F64");
  if (mode != 0 && mode != 1) return set_error(ctx, HMCX_EINVAL, "hmcx_axpy: mode must be 0 or 1");
  if (n < 0 || (n > 0 && (!x || !y))) return set_error(ctx, HMCX_EINVAL, "hmcx_axpy: bad arguments");
  return dtype == HMCX_F64 ? axpy_t<double>(ctx, mode, n, a, x, y) : axpy_t<float>(ctx, mode, n, a, x, y);
}

int hmcx_sgd_run(hmcx_ctx* ctx, const hmcx_sgd_args* a) {
  HMCX_GUARD_CTX(ctx);
  if (!a) return set_error(ctx, HMCX_EINVAL, "null args");
  if (a->model != HMCX_MODEL_SOFTMAX && a->model != HMCX_MODEL_LOGISTIC)
    return set_error(ctx, HMCX_EINVAL, "sgd: model must be HMCX_MODEL_SOFTMAX or HMCX_MODEL_LOGISTIC");
  if (a->model == HMCX_MODEL_LOGISTIC && a->K != 1) return set_error(ctx, HMCX_EINVAL, "sgd: logistic needs K = 1");
  int rc = check_dims(ctx, a->dtype, a->B, a->D, a->K, 1);
  if (rc) return rc;
  if (a->n_steps < 0) return set_error(ctx, HMCX_EINVAL, "n_steps < 0");
  if (!a->X || !a->Y || !a->row0 || !a->W || !a->b || !a->mW || !a->mb)
    return set_error(ctx, HMCX_EINVAL, "null pointer");
  if (a->dropout) {
    if (a->mask_mode == HMCX_NOISE_BUFFER && (!a->keep || !a->keep_off))
      return set_error(ctx, HMCX_EINVAL, "sgd: BUFFER dropout needs keep and keep_off");
    if (a->mask_mode != HMCX_NOISE_BUFFER && a->mask_mode != HMCX_NOISE_PHILOX)
      return set_error(ctx, HMCX_EINVAL, "bad mask_mode");
  }
  if (a->n_steps == 0) return HMCX_OK;
  return a->dtype == HMCX_F64 ? sgd_run_t<double>(ctx, a) : sgd_run_t<float>(ctx, a);
}

static int check_sampler(hmcx_ctx* ctx, const hmcx_sampler_args* a, bool sghmc) {
  if (!a) return set_error(ctx, HMCX_EINVAL, "null args");
  int rc = check_dims(ctx, a->dtype, a->B, a->D, a->K, a->C);
  if (rc) return rc;
  if (a->n_steps < 0) return set_error(ctx, HMCX_EINVAL, "n_steps < 0");
  if (!a->X || !a->Y || !a->W || !a->b || !a->row0 || !a->eps) return set_error(ctx, HMCX_EINVAL, "null pointer");
  if (sghmc && (!a->n_iter || !a->u_accept || !a->out_A || !a->out_accepted || !a->out_ll))
    return set_error(ctx, HMCX_EINVAL, "sghmc: n_iter/u_accept/out_* required");
  if (a->noise_mode == HMCX_NOISE_BUFFER && (!a->noise || !a->noise_off))
    return set_error(ctx, HMCX_EINVAL, "BUFFER noise mode needs noise and noise_off");
  if (a->noise_mode != HMCX_NOISE_BUFFER && a->noise_mode != HMCX_NOISE_PHILOX)
    return set_error(ctx, HMCX_EINVAL, "bad noise_mode");
  if ((long long)a->D * a->K + a->K > 0x7fffffffLL) return set_error(ctx, HMCX_EUNSUPPORTED, "too many parameters");
  return HMCX_OK;
}


int hmcx_sghmc_run(hmcx_ctx* ctx, const hmcx_sampler_args* a_in) {
  HMCX_GUARD_CTX(ctx);
  if (!a_in) return set_error(ctx, HMCX_EINVAL, "null args");
  const hmcx_sampler_args* a = a_in;
  hmcx_sampler_args own;
  if (a_in->noise_mode == HMCX_NOISE_PHILOX && !a_in->n_iter && !a_in->u_accept && a_in->n_steps > 0 && a_in->C > 0) {
    // the call draws its own Philox schedule (one pass here instead of one by the caller)
    const size_t nsc = (size_t)a_in->n_steps * a_in->C;
    if (!a_in->eps) return set_error(ctx, HMCX_EINVAL, "null pointer");
    ctx->sched_L.resize(nsc);
    ctx->sched_n.resize(nsc);
    ctx->sched_u.resize(nsc);
    if (hmcx_philox_schedule(a_in->seed, a_in->chain0, a_in->C, a_in->step_base, a_in->n_steps, a_in->path_length,
                             a_in->eps, ctx->sched_L.data(), ctx->sched_n.data(), ctx->sched_u.data()))
      return set_error(ctx, HMCX_EINVAL, "non-finite path length (step size 0?)");
    if (a_in->out_L) std::memcpy(a_in->out_L, ctx->sched_L.data(), nsc * sizeof(double));
    own = *a_in;
    own.n_iter = ctx->sched_n.data();
    own.u_accept = ctx->sched_u.data();
    a = &own;
  }
  int rc = check_sampler(ctx, a, true);
  if (rc) return rc;
  if (a->pW || a->pb) return set_error(ctx, HMCX_EINVAL, "sghmc: pW/pb are SGLD-only fields");
  if (a->n_steps == 0) return HMCX_OK;
  const bool p2 = sghmc_p2_selected(ctx, a);
  // the 2-D persistent path fills out_host itself (no device abort copy); the others are copied here
  const bool host_by_kernel = p2;
  if (a->out_abort && !p2) HMCX_HIP(ctx, hipMemsetAsync(a->out_abort, 0, sizeof(int32_t), ctx->stream));
  // every SGHMC path stores the per-step state rows (out_trace) itself: the persistent kernel after each
  // accept, the chain-batched and kernel-per-phase paths in the next step's init launch (the state the
  // step kept) and in the closing commit launch — one call, no one-step sub-calls or snapshot launches
  rc = a->dtype == HMCX_F64 ? sghmc_run_t<double>(ctx, a) : sghmc_run_t<float>(ctx, a);
  if (rc || !a->out_host) return rc;
  if (!host_by_kernel) {
    const size_t nsc = (size_t)a->n_steps * a->C;
    char* h = reinterpret_cast<char*>(a->out_host);
    HMCX_HIP(ctx, hipMemcpyAsync(h, a->out_A, 36 * nsc, hipMemcpyDeviceToHost, ctx->stream));
    if (a->out_abort)
      HMCX_HIP(ctx, hipMemcpyAsync(h + 36 * nsc, a->out_abort, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
    else
      reinterpret_cast<int32_t*>(h + 36 * nsc)[0] = 0;
  }
  return host_mark(ctx, a->out_host);
}

int hmcx_host_wait(hmcx_ctx* ctx, const void* out_host) {
  HMCX_GUARD_CTX(ctx);
  for (auto& m : ctx->host_marks)
    if (m.first == out_host) {
      HMCX_HIP(ctx, hipEventSynchronize(m.second));
      return HMCX_OK;
    }
  return HMCX_OK;
}

int hmcx_sgld_run(hmcx_ctx* ctx, const hmcx_sampler_args* a) {
  HMCX_GUARD_CTX(ctx);
  int rc = check_sampler(ctx, a, false);
  if (rc) return rc;
  if (!a->pW != !a->pb) return set_error(ctx, HMCX_EINVAL, "sgld: pW and pb must both be set or both NULL");
  if (a->n_steps == 0) return HMCX_OK;
  // both SGLD paths store the per-step state rows (out_trace) in their update kernels: one call
  if (sgld_wide_eligible(a))
    return a->dtype == HMCX_F64 ? sgld_wide_t<double>(ctx, a) : sgld_wide_t<float>(ctx, a);
  return a->dtype == HMCX_F64 ? sgld_run_t<double>(ctx, a) : sgld_run_t<float>(ctx, a);
}

int hmcx_hmc_mvn_run(hmcx_ctx* ctx, const hmcx_hmc_mvn_args* a) {
  HMCX_GUARD_CTX(ctx);
  if (!a || !a->mu || !a->prec || !a->x || !a->eps || !a->n_iter || !a->u_accept || !a->out_A || !a->out_accepted)
    return set_error(ctx, HMCX_EINVAL, "hmc_mvn: null pointer");
  if (a->C < 1 || a->n_steps < 0) return set_error(ctx, HMCX_EINVAL, "hmc_mvn: bad sizes");
  if (a->noise_mode == HMCX_NOISE_BUFFER && (!a->noise || !a->noise_off))
    return set_error(ctx, HMCX_EINVAL, "BUFFER noise mode needs noise and noise_off");
  if (a->n_steps == 0) return HMCX_OK;
  return hmc_mvn_run(ctx, a);
}

static int check_mlp(hmcx_ctx* ctx, int dtype, int B, int n_in, int n_mid, int n_out) {
  if (dtype != HMCX_F32 && dtype != HMCX_F64) return set_error(ctx, HMCX_EINVAL, "dtype must be HMCX_F32/HMCX_F64");
  if (B < 1 || n_in < 1 || n_mid < 1 || n_out < 1) return set_error(ctx, HMCX_EINVAL, "mlp: sizes must be >= 1");
  if ((long long)B * n_mid * 3 > 0x7fffffffLL || (long long)n_mid * n_in > 0x7fffffffLL ||
      (long long)n_mid * n_mid > 0x7fffffffLL)
    return set_error(ctx, HMCX_EUNSUPPORTED, "mlp: layer too large");
  return HMCX_OK;
}

static bool mlp_par_ok(const hmcx_mlp_params* p) {
  if (!p) return false;
  for (int v = 0; v < 6; ++v)
    if (!p->p[v]) return false;
  return true;
}

int hmcx_mlp_masks(hmcx_ctx* ctx, int dtype, int B, int n_mid, uint64_t seed, uint32_t chain, uint32_t step,
                   uint32_t slot, void* out) {
  HMCX_GUARD_CTX(ctx);
  int rc = check_mlp(ctx, dtype, B, 1, n_mid, 1);
  if (rc) return rc;
  if (!out) return set_error(ctx, HMCX_EINVAL, "null pointer");
  return dtype == HMCX_F64 ? mlp_masks_t<double>(ctx, B, n_mid, seed, chain, step, slot, out)
                           : mlp_masks_t<float>(ctx, B, n_mid, seed, chain, step, slot, out);
}

int hmcx_mlp_grad(hmcx_ctx* ctx, int dtype, const void* X, const int32_t* y, int B, int n_in, int n_mid, int n_out,
                  const hmcx_mlp_params* par, const void* masks, double alpha, hmcx_mlp_params* grads,
                  double* loss) {
  HMCX_GUARD_CTX(ctx);
  int rc = check_mlp(ctx, dtype, B, n_in, n_mid, n_out);
  if (rc) return rc;
  if (!X || !y || !mlp_par_ok(par) || !mlp_par_ok(grads)) return set_error(ctx, HMCX_EINVAL, "null pointer");
  return dtype == HMCX_F64 ? mlp_grad_t<double>(ctx, X, y, B, n_in, n_mid, n_out, par, masks, alpha, grads, loss)
                           : mlp_grad_t<float>(ctx, X, y, B, n_in, n_mid, n_out, par, masks, alpha, grads, loss);
}

int hmcx_mlp_loss(hmcx_ctx* ctx, int dtype, const void* X, const int32_t* y, int B, int n_in, int n_mid, int n_out,
                  const hmcx_mlp_params* par, const void* masks, double* loss, void* logits) {
  HMCX_GUARD_CTX(ctx);
  int rc = check_mlp(ctx, dtype, B, n_in, n_mid, n_out);
  if (rc) return rc;
  if (!X || !mlp_par_ok(par)) return set_error(ctx, HMCX_EINVAL, "null pointer");
  if (!y && !logits) return set_error(ctx, HMCX_EINVAL, "mlp_loss: need labels or a logits output");
  return dtype == HMCX_F64 ? mlp_loss_t<double>(ctx, X, y, B, n_in, n_mid, n_out, par, masks, loss, logits)
                           : mlp_loss_t<float>(ctx, X, y, B, n_in, n_mid, n_out, par, masks, loss, logits);
}

int hmcx_mlp_sghmc_run(hmcx_ctx* ctx, const hmcx_mlp_sghmc_args* a) {
  HMCX_GUARD_CTX(ctx);
  if (!a) return set_error(ctx, HMCX_EINVAL, "null args");
  int rc = check_mlp(ctx, a->dtype, a->B, a->n_in, a->n_mid, a->n_out);
  if (rc) return rc;
  if (a->n_steps < 0) return set_error(ctx, HMCX_EINVAL, "n_steps < 0");
  if (!a->X || !a->y || !a->row0 || !a->eps || !a->n_iter || !a->u_accept || !mlp_par_ok(&a->par) || !a->out_A ||
      !a->out_accepted || !a->out_loss)
    return set_error(ctx, HMCX_EINVAL, "mlp sghmc: null pointer");
  if (a->noise_mode != HMCX_NOISE_BUFFER && a->noise_mode != HMCX_NOISE_PHILOX)
    return set_error(ctx, HMCX_EINVAL, "bad noise_mode");
  if (a->mask_mode != HMCX_NOISE_BUFFER && a->mask_mode != HMCX_NOISE_PHILOX)
    return set_error(ctx, HMCX_EINVAL, "bad mask_mode");
  if (a->noise_mode == HMCX_NOISE_BUFFER && (!a->noise || !a->noise_off))
    return set_error(ctx, HMCX_EINVAL, "BUFFER noise mode needs noise and noise_off");
  if (a->mask_mode == HMCX_NOISE_BUFFER && (!a->masks || !a->mask_off))
    return set_error(ctx, HMCX_EINVAL, "BUFFER mask mode needs masks and mask_off");
  if (a->n_steps == 0) return HMCX_OK;
  return a->dtype == HMCX_F64 ? mlp_sghmc_t<double>(ctx, a) : mlp_sghmc_t<float>(ctx, a);
}

int hmcx_mlp_hmc_leapfrog(hmcx_ctx* ctx, const hmcx_mlp_leapfrog_args* a) {
  HMCX_GUARD_CTX(ctx);
  if (!a) return set_error(ctx, HMCX_EINVAL, "null args");
  int rc = check_mlp(ctx, a->dtype, a->B, a->n_in, a->n_mid, a->n_out);
  if (rc) return rc;
  if (a->n_iter < 0) return set_error(ctx, HMCX_EINVAL, "mlp leapfrog: n_iter < 0");
  if (!a->X || !a->y || !mlp_par_ok(&a->q) || !mlp_par_ok(&a->p) || !mlp_par_ok(&a->g))
    return set_error(ctx, HMCX_EINVAL, "mlp leapfrog: null pointer");
  if (a->mask_mode != HMCX_MLP_MASKS_NONE && a->mask_mode != HMCX_MLP_MASKS_FIXED &&
      a->mask_mode != HMCX_MLP_MASKS_PHILOX)
    return set_error(ctx, HMCX_EINVAL, "mlp leapfrog: bad mask_mode");
  if (a->mask_mode != HMCX_MLP_MASKS_NONE && !a->masks)
    return set_error(ctx, HMCX_EINVAL, "mlp leapfrog: masks required for FIXED / PHILOX");
  int seen = 0;
  for (int i = 0; i < 6; ++i) {
    const int v = a->order[i];
    if (v < 0 || v > 5 || ((seen >> v) & 1))
      return set_error(ctx, HMCX_EINVAL, "mlp leapfrog: order must be a permutation of 0..5");
    seen |= 1 << v;
  }
  return a->dtype == HMCX_F64 ? mlp_leapfrog_t<double>(ctx, a) : mlp_leapfrog_t<float>(ctx, a);
}

}  // extern "C"
