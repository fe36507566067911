// hmcx_persist.h — argument block and launch plan of the persistent SGHMC kernel.
#pragma once
#include "hmcx_internal.h"

namespace hmcx {

template <typename T> struct PersistArgs {
  const T* X; const T* Y;
  int B, D, K, P, n_steps;
  int Gr, Gf, Br, Bf, BFP;
  T alpha;
  double neg_inv_n, log_prior;
  const double* eps; const double* u; const int64_t* row0; const int32_t* n_iter;
  int noise_mode; const double* noise; const int64_t* noff;
  uint64_t seed; uint32_t chain0, step_base;
  T* W; T* b;
  T* exA; T* exB; T* exBcs; double* exBll; double* exG; double* exL;
  unsigned* rowc; unsigned* featc; unsigned* globc; int* abort_flag;
  double* out_A; int32_t* out_acc; double* out_ll; double* out_E;
  unsigned long long* prof;   // HMCX_PERSIST_PROF=1: per-phase s_memtime totals of block 0
};

struct PersistPlan {
  bool ok;
  int Gr, Gf, Br, Bf, BFP;
  size_t lds;
  double cost;
};

// hmcx_persist2.hip: reduce-scatter / all-gather teams over tagged-granule hand-offs.
struct PersistPlan2 {
  bool ok;
  int Gr, Gf, Br, Bf, BfP, BFP, Ro, Fo;
  size_t lds;
  double cost;
};
PersistPlan2 plan_p2(int B, int D, int K, size_t tsize, int num_cus, size_t lds_max);
template <typename T> int sghmc_p2_t(hmcx_ctx*, const hmcx_sampler_args*, const PersistPlan2&);

PersistPlan plan_persist(int B, int D, int K, size_t tsize, int num_cus, size_t lds_max);
template <typename T> int sghmc_persist_t(hmcx_ctx*, const hmcx_sampler_args*, const PersistPlan&);

}  // namespace hmcx
