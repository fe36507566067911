// hmcx_persist.h — launch plan of the persistent single-chain SGHMC kernel (hmcx_persist2.hip).
#pragma once
#include "hmcx_internal.h"

namespace hmcx {

// hmcx_persist2.hip: reduce-scatter / all-gather teams over tagged-granule hand-offs.
struct PersistPlan2 {
  bool ok;
  int Gr, Gf, Br, Bf, BfP, BFP, Ro, Fo;
  size_t lds;
  double cost;
};
PersistPlan2 plan_p2(int B, int D, int K, size_t tsize, int num_cus, size_t lds_max);
template <typename T> int sghmc_p2_t(hmcx_ctx*, const hmcx_sampler_args*, const PersistPlan2&);

}  // namespace hmcx
