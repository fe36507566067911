// hmcx_comm.cpp — the cross-rank gather of the multi-GPU run over RCCL (include/hmcx.h, "cross-rank
// gather").  Host code only: an RCCL communicator per rank, created from a unique id handed out by
// the launcher, and the two collectives the run needs (one all-gather of the per-chain summaries,
// the timing max / leapfrog sum), enqueued on the hmcx context's stream.
//
// Reference: the multi-chain layer collects worker results through multiprocessing
// (hamiltonian/inference/cpu/sghmc_multicore.py:81-99, Pool.map + concatenation); here the chains
// never communicate while sampling and the result collection is one collective over xGMI.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <cstring>
#include <string>
#include "hmcx_internal.h"

struct hmcx_comm {
  ncclComm_t nc = nullptr;
  int nranks = 0, rank = 0, device = 0;
};

namespace {
int nccl_error(hmcx_ctx* ctx, const char* what, ncclResult_t r) {
  return hmcx::set_error(ctx, HMCX_EHIP, std::string(what) + ": " + ncclGetErrorString(r));
}
}  // namespace

extern "C" {

int hmcx_comm_unique_id(void* id) {
  if (!id) return HMCX_EINVAL;
  static_assert(sizeof(ncclUniqueId) == HMCX_COMM_ID_BYTES, "RCCL unique id size");
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return HMCX_EHIP;
  std::memcpy(id, &u, sizeof(u));
  return HMCX_OK;
}

int hmcx_comm_init(hmcx_ctx* ctx, int nranks, int rank, const void* id, hmcx_comm** out) {
  if (!ctx || !out || !id) return HMCX_EINVAL;
  if (nranks < 1 || rank < 0 || rank >= nranks) return hmcx::set_error(ctx, HMCX_EINVAL, "comm: bad rank / size");
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  HMCX_HIP(ctx, hipSetDevice(ctx->device));
  auto* c = new hmcx_comm();
  c->nranks = nranks;
  c->rank = rank;
  c->device = ctx->device;
  const ncclResult_t r = ncclCommInitRank(&c->nc, nranks, u, rank);
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
  if (comm->nc) (void)ncclCommDestroy(comm->nc);
  delete comm;
  return HMCX_OK;
}

int hmcx_allgather_chain_stats(hmcx_ctx* ctx, hmcx_comm* comm, const double* send, double* recv, uint64_t count) {
  if (!ctx || !comm || (count && (!send || !recv))) return HMCX_EINVAL;
  if (comm->device != ctx->device) return hmcx::set_error(ctx, HMCX_EINVAL, "comm: other device than the context");
  const ncclResult_t r = ncclAllGather(send, recv, (size_t)count, ncclDouble, comm->nc, ctx->stream);
  return r == ncclSuccess ? HMCX_OK : nccl_error(ctx, "ncclAllGather", r);
}

int hmcx_allreduce_f64(hmcx_ctx* ctx, hmcx_comm* comm, const double* send, double* recv, uint64_t count, int op) {
  if (!ctx || !comm || (count && (!send || !recv)) || (op != 0 && op != 1)) return HMCX_EINVAL;
  if (comm->device != ctx->device) return hmcx::set_error(ctx, HMCX_EINVAL, "comm: other device than the context");
  const ncclResult_t r = ncclAllReduce(send, recv, (size_t)count, ncclDouble, op == 0 ? ncclSum : ncclMax, comm->nc,
                                       ctx->stream);
  return r == ncclSuccess ? HMCX_OK : nccl_error(ctx, "ncclAllReduce", r);
}

}  // extern "C"
