// hmcx_granule.h — tagged-granule hand-off between the workgroups of one launch (the R2 recipe of
// MI355X_MICROARCH.md, as in hmcx_persist2.hip): a value travels as one 16-byte granule
// {lo32, epoch, hi32, epoch} written by one write-through (sc1) store and re-read with sc1 loads until
// both epoch words equal the launch's epoch.  Used by the fused launches whose workgroups exchange a
// small partial once (MLP layer 2 + 3, wide SGLD forward + softmax); the arena and the per-launch
// epoch come from the context (gx_reserve / gx_next_epoch).
#pragma once
#include "hmcx_common.h"

namespace hmcx {

__device__ inline __amdgpu_buffer_rsrc_t gx_rsrc(char* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(base, 0, bytes, 0x00020000);
}

__device__ inline void gx_put(__amdgpu_buffer_rsrc_t rs, int g, double v, unsigned ep) {
  typedef unsigned int g4 __attribute__((ext_vector_type(4)));
  const unsigned long long x = __builtin_bit_cast(unsigned long long, v);
  const g4 w = {(unsigned)x, ep, (unsigned)(x >> 32), ep};
  __builtin_amdgcn_raw_buffer_store_b128(w, rs, g * 16, 0, 16 /* sc1 */);
}

// Granule poll of one item over `np` producers (stride `pstride` granules): sum in producer order.
// Bounded (2 s of s_memrealtime): on timeout the context's abort word is raised and the item reads
// 0 — the host reports the launch as failed (abort_defer), it never returns a stale value silently.
__device__ inline bool gx_poll_sum(__amdgpu_buffer_rsrc_t rs, int g0, int pstride, int np, unsigned ep, int* abort_flag,
                                double* sum) {
  typedef unsigned int g4 __attribute__((ext_vector_type(4)));
  constexpr int NPMAX = 16;
  unsigned pend = (np >= 32) ? 0xffffffffu : ((1u << np) - 1u);
  double val[NPMAX];
#pragma unroll
  for (int p = 0; p < NPMAX; ++p) val[p] = 0.0;
  unsigned long long t0 = 0;
  for (int spins = 0; pend; ++spins) {
    g4 v[NPMAX];
#pragma unroll
    for (int p = 0; p < NPMAX; ++p)
      v[p] = __builtin_amdgcn_raw_buffer_load_b128(rs, (g0 + (p < np ? p : 0) * pstride) * 16, 0, 16 /* sc1 */);
#pragma unroll
    for (int p = 0; p < NPMAX; ++p)
      if (((pend >> p) & 1u) && v[p].y == ep && v[p].w == ep) {
        val[p] = __builtin_bit_cast(double, (unsigned long long)v[p].x | ((unsigned long long)v[p].z << 32));
        pend &= ~(1u << p);
      }
    if (!pend) break;
    if (spins == 0) t0 = __builtin_amdgcn_s_memrealtime();
    if ((spins & 63) == 63 && (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull ||
                               __hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
      __hip_atomic_store(abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *sum = 0.0;
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  double acc = val[0];
#pragma unroll
  for (int p = 1; p < NPMAX; ++p)
    if (p < np) acc += val[p];
  *sum = acc;
  return true;
}

}  // namespace hmcx
