// hmcx_comm.cpp — the cross-rank gather of the multi-GPU run over RCCL (include/hmcx.h, "cross-rank
// gather").  Host code only: an RCCL communicator per rank, created from a unique id handed out by
// the launcher, and the two collectives the run needs (one all-gather of the per-chain summaries,
// the timing max / leapfrog sum), enqueued on the hmcx context's stream.
//
// Reference: the multi-chain layer collects worker results through multiprocessing
// (hamiltonian/inference/cpu/sghmc_multicore.py:81-99, Pool.map + concatenation); here the chains
// never communicate while sampling and the result collection is one collective over xGMI.
//
// RCCL is loaded lazily (dlopen on the first hmcx_comm_* call), so the single-GPU paths neither link
// nor load it: preferred is the copy the process already has (torch's bundled librccl.so, or a
// librccl.so.1 loaded by someone else — one RCCL per process), else the system librccl.so.1.  Without
// any, the hmcx_comm_* entry points return HMCX_EUNSUPPORTED.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <dlfcn.h>
#include <cstring>
#include <mutex>
#include <string>
#include "hmcx_internal.h"

struct hmcx_comm {
  ncclComm_t nc = nullptr;
  int nranks = 0, rank = 0, device = 0;
};

namespace {
struct Rccl {
  bool ok = false;
  std::string from;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = nullptr;
    const char* loaded[] = {"librccl.so.1", "librccl.so"};            // already in the process
    for (const char* n : loaded)
      if (!h && (h = dlopen(n, RTLD_NOW | RTLD_LOCAL | RTLD_NOLOAD))) r.from = n;
    const char* fresh[] = {"librccl.so.1", "/opt/rocm/lib/librccl.so.1"};
    for (const char* n : fresh)
      if (!h && (h = dlopen(n, RTLD_NOW | RTLD_LOCAL))) r.from = n;
    if (!h) return;
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    r.all_gather = reinterpret_cast<decltype(r.all_gather)>(dlsym(h, "ncclAllGather"));
    r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(dlsym(h, "ncclAllReduce"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
    r.ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.all_gather && r.all_reduce && r.error_string;
  });
  return r;
}

int nccl_error(hmcx_ctx* ctx, const char* what, ncclResult_t r) {
  return hmcx::set_error(ctx, HMCX_EHIP, std::string(what) + ": " + rccl().error_string(r));
}
int no_rccl(hmcx_ctx* ctx) {
  return ctx ? hmcx::set_error(ctx, HMCX_EUNSUPPORTED, "comm: RCCL (librccl.so.1) could not be loaded")
             : HMCX_EUNSUPPORTED;
}
}  // namespace

extern "C" {

int hmcx_comm_unique_id(void* id) {
  if (!id) return HMCX_EINVAL;
  static_assert(sizeof(ncclUniqueId) == HMCX_COMM_ID_BYTES, "RCCL unique id size");
  if (!rccl().ok) return no_rccl(nullptr);
  ncclUniqueId u;
  if (rccl().get_unique_id(&u) != ncclSuccess) return HMCX_EHIP;
  std::memcpy(id, &u, sizeof(u));
  return HMCX_OK;
}

int hmcx_comm_init(hmcx_ctx* ctx, int nranks, int rank, const void* id, hmcx_comm** out) {
  if (!ctx || !out || !id) return HMCX_EINVAL;
  if (nranks < 1 || rank < 0 || rank >= nranks) return hmcx::set_error(ctx, HMCX_EINVAL, "comm: bad rank / size");
  if (!rccl().ok) return no_rccl(ctx);
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  HMCX_HIP(ctx, hipSetDevice(ctx->device));
  auto* c = new hmcx_comm();
  c->nranks = nranks;
  c->rank = rank;
  c->device = ctx->device;
  const ncclResult_t r = rccl().comm_init_rank(&c->nc, nranks, u, rank);
  if (r != ncclSuccess) {
    delete c;
    return nccl_error(ctx, "ncclCommInitRank", r);
  }
  *out = c;
  return HMCX_OK;
}

int hmcx_comm_destroy(hmcx_comm* comm) {
  if (!comm) return HMCX_OK;
  (void)hipSetDevice(comm->device);
  if (comm->nc) (void)rccl().comm_destroy(comm->nc);
  delete comm;
  return HMCX_OK;
}

int hmcx_allgather_chain_stats(hmcx_ctx* ctx, hmcx_comm* comm, const double* send, double* recv, uint64_t count) {
  if (!ctx || !comm || (count && (!send || !recv))) return HMCX_EINVAL;
  if (comm->device != ctx->device) return hmcx::set_error(ctx, HMCX_EINVAL, "comm: other device than the context");
  const ncclResult_t r = rccl().all_gather(send, recv, (size_t)count, ncclDouble, comm->nc, ctx->stream);
  return r == ncclSuccess ? HMCX_OK : nccl_error(ctx, "ncclAllGather", r);
}

int hmcx_allreduce_f64(hmcx_ctx* ctx, hmcx_comm* comm, const double* send, double* recv, uint64_t count, int op) {
  if (!ctx || !comm || (count && (!send || !recv)) || (op != 0 && op != 1)) return HMCX_EINVAL;
  if (comm->device != ctx->device) return hmcx::set_error(ctx, HMCX_EINVAL, "comm: other device than the context");
  const ncclResult_t r = rccl().all_reduce(send, recv, (size_t)count, ncclDouble, op == 0 ? ncclSum : ncclMax,
                                           comm->nc, ctx->stream);
  return r == ncclSuccess ? HMCX_OK : nccl_error(ctx, "ncclAllReduce", r);
}

}  // extern "C"
