// hmcx_p2x.h — tagged-granule exchange of the persistent single-chain SGHMC kernel
// (hmcx_persist2.hip: 2-D teams) and shared DPP reductions.  Every value travels as
// one 16-byte granule {lo32, epoch, hi32, epoch} written by ONE buffer_store_dwordx4 and re-read
// until both epoch words match (cdna_hip_programming.md §6 G16, recipe R2); spins are bounded
// (QTIMEOUT) and raise the context's sticky abort word.
#pragma once
#include "hmcx_common.h"

namespace hmcx {

constexpr int QTH = 256;                 // threads per workgroup (4 waves)
constexpr int QNW = QTH / 64;
constexpr int QNPM = 16;                 // largest team (producers per gather)
#ifndef HMCX_P2_SLEEP
#define HMCX_P2_SLEEP 1
#endif
constexpr unsigned long long QTIMEOUT = 400000000ull;   // s_memrealtime ticks (100 MHz): 4 s

typedef unsigned int gran_t __attribute__((ext_vector_type(4)));
__host__ __device__ inline int p2_pad(int n, int pad) { return pad ? (n + 7) & ~7 : n; }

// The thread index as a value the compiler cannot see through: index arithmetic derived from it is
// recomputed where it is used instead of being hoisted out of the step loop and kept live (the
// hoisted offsets of every gather and load batch exceeded the register file and spilled).
// A uniform 64-bit value the compiler must re-read at this point (kept scalar): derived constants
// (the Philox key schedule of a seed) are recomputed per use instead of being hoisted and spilled.
__device__ inline uint64_t opaque_s64(uint64_t x) {
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  asm volatile("" : "+s"(lo), "+s"(hi));
  return ((uint64_t)hi << 32) | lo;
}
__device__ inline int opaque(int x) {
  asm volatile("" : "+v"(x));
  return x;
}

// ---------------------------------------------------------------- granule transport
__device__ inline __amdgpu_buffer_rsrc_t arena_rsrc(char* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(base, 0, bytes, 0x00020000);
}
__device__ inline void put(__amdgpu_buffer_rsrc_t rs, int g, double v, unsigned ep) {
  const unsigned long long x = __builtin_bit_cast(unsigned long long, v);
  gran_t w = {(unsigned)x, ep, (unsigned)(x >> 32), ep};
  __builtin_amdgcn_raw_buffer_store_b128(w, rs, g * 16, 0, 16 /* sc1 */);
}
// XCD-local team regions (fl2): plain store, kept in the XCD's L2
__device__ inline void put_t(bool l2, __amdgpu_buffer_rsrc_t rs, int g, double v, unsigned ep) {
  const unsigned long long x = __builtin_bit_cast(unsigned long long, v);
  gran_t w = {(unsigned)x, ep, (unsigned)(x >> 32), ep};
  if (l2) __builtin_amdgcn_raw_buffer_store_b128(w, rs, g * 16, 0, 0);
  else __builtin_amdgcn_raw_buffer_store_b128(w, rs, g * 16, 0, 16 /* sc1 */);
}
__device__ inline double decode(gran_t w) {
  return __builtin_bit_cast(double, (unsigned long long)w.x | ((unsigned long long)w.z << 32));
}

// A timed-out poll raises the sticky abort word; the first timeout also records where it happened
// (abort_flag[1] = workgroup + 1, [2] = the round's granule base, [3] = its epoch) for diagnosis
// (hmcx_clear_abort prints them under HMCX_P2_DEBUG=1).  A poll that sees the word already raised
// only leaves.
__device__ inline void p2_timeout(int* abort_flag, int where, unsigned ep) {
  int z = 0;
  if (__hip_atomic_compare_exchange_strong(abort_flag + 1, &z, (int)blockIdx.x + 1, __ATOMIC_RELAXED,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
    __hip_atomic_store(abort_flag + 2, where, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(abort_flag + 3, (int)ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __hip_atomic_store(abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline bool p2_spin_over(unsigned long long t0, int* abort_flag, int where, unsigned ep) {
  if (__builtin_amdgcn_s_memrealtime() - t0 > QTIMEOUT) {
    p2_timeout(abort_flag, where, ep);
    return true;
  }
  if (__hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return true;
  return false;
}

// Polls one granule per producer p < np (p != pskip) at base0 + p·pstride + off until both epoch
// words match.  Loads go out unpredicated in one batch of 8·NB (absent producers clamped to a
// valid address and ignored); a pass re-reads the batch while any granule is missing.
// SUM: *sum = v_0 + v_1 + … in producer order; else v_p → dst[p·dstride].  false on timeout/abort.
template <int NB, bool SUM, typename V, int AUX = 16>
__device__ inline bool poll_nb(__amdgpu_buffer_rsrc_t rs, int base0, int pstride, int np, int pskip, int off,
                               bool valid, unsigned ep, double* sum, int* abort_flag, V* dst, int dstride) {
  constexpr int N = 8 * NB;
  unsigned pend = 0;
  int o[N];
#pragma unroll
  for (int u = 0; u < N; ++u) {
    const bool want = valid && u < np && u != pskip;
    pend |= want ? 1u << u : 0u;
    o[u] = (base0 + (want ? u * pstride + off : 0)) * 16;
  }
  double val[N];
#pragma unroll
  for (int u = 0; u < N; ++u) val[u] = 0.0;
  unsigned long long t0 = 0;
  for (int spins = 0; pend; ++spins) {
    gran_t v[N];
#pragma unroll
    for (int u = 0; u < N; ++u) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, o[u], 0, AUX /* 16: sc1 */);
#pragma unroll
    for (int u = 0; u < N; ++u)
      if (((pend >> u) & 1u) && v[u].y == ep && v[u].w == ep) {
        val[u] = decode(v[u]);
        pend &= ~(1u << u);
      }
    if (!pend) break;
    if (spins == 0) t0 = __builtin_amdgcn_s_memrealtime();
    if ((spins & 63) == 63 && p2_spin_over(t0, abort_flag, base0, ep)) return false;
    if (HMCX_P2_SLEEP) __builtin_amdgcn_s_sleep(1);
  }
  if (!valid) return true;
  if (SUM) {
    double acc = val[0];
#pragma unroll
    for (int u = 1; u < N; ++u)
      if (u < np && u != pskip) acc += val[u];
    *sum = acc;
  } else {
#pragma unroll
    for (int u = 0; u < N; ++u)
      if (u < np && u != pskip) dst[u * dstride] = (V)val[u];
  }
  return true;
}
// AUX = 1 (sc0: coherent at the XCD's L2) is used only for teams whose members share an XCD; the
// L2 is invalidated at launch, and every round's epoch is new within the launch.
template <bool SUM, typename V = double, int AUX = 16>
__device__ inline bool poll(__amdgpu_buffer_rsrc_t rs, int base0, int pstride, int np, int pskip, int off, bool valid,
                            unsigned ep, double* /*unused*/, int /*unused*/, double* sum, int* abort_flag,
                            V* dst = nullptr, int dstride = 0) {
  return np <= 8 ? poll_nb<1, SUM, V, AUX>(rs, base0, pstride, np, pskip, off, valid, ep, sum, abort_flag, dst, dstride)
                 : poll_nb<2, SUM, V, AUX>(rs, base0, pstride, np, pskip, off, valid, ep, sum, abort_flag, dst, dstride);
}

// NI items per thread (item j at granule offset off[j] of every producer block, valid bit j of vmask),
// each summed over producers p < np in producer order: NI·8·NB loads per pass in one batch.
// false on timeout/abort.
// `work()` runs once while the first batch of loads is in flight (independent work hidden behind the
// round's latency).
template <int NI, int NB, typename Work>
__device__ inline bool polln_nb(__amdgpu_buffer_rsrc_t rs, int base0, int pstride, int np, const int* off,
                                unsigned vmask, unsigned ep, double* sum, int* abort_flag, Work work) {
  constexpr int N = 8 * NB, M = NI * N;
  static_assert(M <= 64, "pending mask");
  unsigned long long pend = 0;
  int o[M];
#pragma unroll
  for (int u = 0; u < M; ++u) {
    const int j = u / N, p = u - j * N;
    const bool want = ((vmask >> j) & 1u) && p < np;
    pend |= want ? 1ull << u : 0ull;
    o[u] = (base0 + (want ? p * pstride + off[j] : 0)) * 16;
  }
  double val[M];
#pragma unroll
  for (int u = 0; u < M; ++u) val[u] = 0.0;
  unsigned long long t0 = 0;
  bool worked = false;
  for (int spins = 0; pend; ++spins) {
    gran_t v[M];
#pragma unroll
    for (int u = 0; u < M; ++u) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, o[u], 0, 16 /* sc1 */);
    if (spins == 0) work();
    worked = true;
#pragma unroll
    for (int u = 0; u < M; ++u)
      if (((pend >> u) & 1ull) && v[u].y == ep && v[u].w == ep) {
        val[u] = decode(v[u]);
        pend &= ~(1ull << u);
      }
    if (!pend) break;
    if (spins == 0) t0 = __builtin_amdgcn_s_memrealtime();
    if ((spins & 63) == 63 && p2_spin_over(t0, abort_flag, base0, ep)) return false;
    if (HMCX_P2_SLEEP) __builtin_amdgcn_s_sleep(1);
  }
  if (!worked) work();
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    double acc = val[j * N];
#pragma unroll
    for (int p = 1; p < N; ++p)
      if (p < np) acc += val[j * N + p];
    sum[j] = acc;
  }
  return true;
}
template <int NI, typename Work>
__device__ inline bool polln(__amdgpu_buffer_rsrc_t rs, int base0, int pstride, int np, const int* off, unsigned vmask,
                             unsigned ep, double* sum, int* abort_flag, Work work) {
  return np <= 8 ? polln_nb<NI, 1>(rs, base0, pstride, np, off, vmask, ep, sum, abort_flag, work)
                 : polln_nb<NI, 2>(rs, base0, pstride, np, off, vmask, ep, sum, abort_flag, work);
}

// Spread gather: the (producer, item) pairs of a round are dealt over ALL threads of the workgroup
// (at most 4 granules per thread, where the per-item polls above put up to 16 on a few lanes of
// one wave) and land in LDS as stage[p·nitems + i]; the caller combines them in producer order
// after the barrier, so sums are bit-identical to poll<true>.  Item i of producer p is granule
// base0 + p·pstride + ioff(i); pairs with want(p, i) false are skipped.
constexpr int QSTAGE = 4 * QTH;             // staged pairs per round (LDS doubles)
template <int U, typename Off, typename Want>
__device__ inline bool gather_u(__amdgpu_buffer_rsrc_t rs, int base0, int pstride, int np, int nitems, Off ioff,
                                Want want, unsigned ep, int* abort_flag, double* stage) {
  unsigned pend = 0;
  int o[U], qi[U];
  const int t0i = opaque((int)threadIdx.x);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int q = t0i + u * QTH;
    const int p = q / nitems, i = q - p * nitems;
    const bool w = q < np * nitems && want(p, i);
    pend |= w ? 1u << u : 0u;
    o[u] = (base0 + (w ? p * pstride + ioff(i) : 0)) * 16;
    qi[u] = q;
  }
  unsigned long long t0 = 0;
  for (int spins = 0; pend; ++spins) {
    gran_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, o[u], 0, 16 /* sc1 */);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (((pend >> u) & 1u) && v[u].y == ep && v[u].w == ep) {
        stage[qi[u]] = decode(v[u]);
        pend &= ~(1u << u);
      }
    if (!pend) break;
    if (spins == 0) t0 = __builtin_amdgcn_s_memrealtime();
    if ((spins & 63) == 63 && p2_spin_over(t0, abort_flag, base0, ep)) return false;
    if (HMCX_P2_SLEEP) __builtin_amdgcn_s_sleep(1);
  }
  return true;
}
// gather_u with the destination chosen per pair: store(q, v) for pair q = p·nitems + i (e.g. straight
// into the consumer's LDS layout, saving a staging copy and its barrier).
template <int U, typename Off, typename Store>
__device__ inline bool gather_st_u(__amdgpu_buffer_rsrc_t rs, int base0, int pstride, int np, int nitems, Off ioff,
                                   unsigned ep, int* abort_flag, Store store) {
  unsigned pend = 0;
  int o[U], qi[U];
  const int t0i = opaque((int)threadIdx.x);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int q = t0i + u * QTH;
    const int p = q / nitems, i = q - p * nitems;
    const bool w = q < np * nitems;
    pend |= w ? 1u << u : 0u;
    o[u] = (base0 + (w ? p * pstride + ioff(i) : 0)) * 16;
    qi[u] = q;
  }
  unsigned long long t0 = 0;
  for (int spins = 0; pend; ++spins) {
    gran_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, o[u], 0, 16 /* sc1 */);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (((pend >> u) & 1u) && v[u].y == ep && v[u].w == ep) {
        store(qi[u], decode(v[u]));
        pend &= ~(1u << u);
      }
    if (!pend) break;
    if (spins == 0) t0 = __builtin_amdgcn_s_memrealtime();
    if ((spins & 63) == 63 && p2_spin_over(t0, abort_flag, base0, ep)) return false;
    if (HMCX_P2_SLEEP) __builtin_amdgcn_s_sleep(1);
  }
  return true;
}
template <typename Off, typename Store>
__device__ inline bool gather_st(__amdgpu_buffer_rsrc_t rs, int base0, int pstride, int np, int nitems, Off ioff,
                                 unsigned ep, int* abort_flag, Store store) {
  const int u = (np * nitems + QTH - 1) / QTH;
  if (u <= 1) return gather_st_u<1>(rs, base0, pstride, np, nitems, ioff, ep, abort_flag, store);
  if (u == 2) return gather_st_u<2>(rs, base0, pstride, np, nitems, ioff, ep, abort_flag, store);
  if (u == 3) return gather_st_u<3>(rs, base0, pstride, np, nitems, ioff, ep, abort_flag, store);
  return gather_st_u<4>(rs, base0, pstride, np, nitems, ioff, ep, abort_flag, store);
}

template <typename Off, typename Want>
__device__ inline bool gather(__amdgpu_buffer_rsrc_t rs, int base0, int pstride, int np, int nitems, Off ioff,
                              Want want, unsigned ep, int* abort_flag, double* stage) {
  const int u = (np * nitems + QTH - 1) / QTH;
  if (u <= 1) return gather_u<1>(rs, base0, pstride, np, nitems, ioff, want, ep, abort_flag, stage);
  if (u == 2) return gather_u<2>(rs, base0, pstride, np, nitems, ioff, want, ep, abort_flag, stage);
  if (u == 3) return gather_u<3>(rs, base0, pstride, np, nitems, ioff, want, ep, abort_flag, stage);
  return gather_u<4>(rs, base0, pstride, np, nitems, ioff, want, ep, abort_flag, stage);
}

// ---------------------------------------------------------------- commit decision
// One 64-bit word per launch decides whether the launch commits: (epoch << 2) | d, d = 1 commit,
// d = 2 abort, set ONCE by a compare-and-swap (vector global atomic; words of earlier launches carry
// older epochs).  Whoever swaps first decides; every other proposer, and every waiter, adopts that
// value — so all workgroups that read a decision read the same one, whatever their timeouts.
constexpr int P2_COMMIT = 1, P2_ABORT = 2;
__device__ inline int p2_decide(unsigned long long* w, unsigned ep, int d) {
  const unsigned long long mine = ((unsigned long long)ep << 2) | (unsigned)d;
  unsigned long long cur = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  while ((cur >> 2) != (unsigned long long)ep) {
    if (__hip_atomic_compare_exchange_strong(w, &cur, mine, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT))
      return d;
  }
  return (int)(cur & 3ull);
}
// Waits (bounded) for the launch's decision; on timeout or a raised abort word it proposes abort —
// and adopts whatever was decided first.  Only a decided abort raises the context's sticky abort word
// (and records where): a COMMIT that lands between the last load and the swap leaves the word down,
// so the next launch is not stopped for nothing.
__device__ inline int p2_wait_decision(unsigned long long* w, unsigned ep, int* abort_flag) {
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int spins = 0;; ++spins) {
    const unsigned long long cur = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((cur >> 2) == (unsigned long long)ep) return (int)(cur & 3ull);
    if ((spins & 63) == 63 &&
        (__builtin_amdgcn_s_memrealtime() - t0 > QTIMEOUT ||
         __hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
      const int d = p2_decide(w, ep, P2_ABORT);
      if (d == P2_ABORT) p2_timeout(abort_flag, -1, ep);
      return d;
    }
    if (HMCX_P2_SLEEP) __builtin_amdgcn_s_sleep(1);
  }
}

// Workgroup-uniform verdict after a gather (also the barrier that publishes dst).
__device__ inline bool all_ok(bool ok, int* sh_fail) {
  if (!ok) *sh_fail = 1;
  __syncthreads();
  return *sh_fail == 0;
}

// Deterministic workgroup sum (fixed butterfly + fixed wave order).
__device__ inline double wsum(double v, double* sh) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = sh[0];
#pragma unroll
  for (int w = 1; w < QNW; ++w) r += sh[w];
  __syncthreads();
  return r;
}

// All-reduce over a 16-lane row with DPP (xor 1, xor 2, half-row mirror, row mirror): every lane
// of the row ends with the same bits (each step combines a symmetric pair).
template <int CTRL> __device__ inline double dpp64(double v) {
  const unsigned long long x = __builtin_bit_cast(unsigned long long, v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)x, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(x >> 32), CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, (unsigned long long)(unsigned)lo | ((unsigned long long)(unsigned)hi << 32));
}
template <int CTRL> __device__ inline float dpp64(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
constexpr int DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_HMIRROR = 0x141, DPP_MIRROR = 0x140;
template <typename T> __device__ inline T g16_max2(T v) {
  v = max_nan(v, dpp64<DPP_XOR1>(v));
  v = max_nan(v, dpp64<DPP_XOR2>(v));
  v = max_nan(v, dpp64<DPP_HMIRROR>(v));
  v = max_nan(v, dpp64<DPP_MIRROR>(v));
  return v;
}
template <typename T> __device__ inline T g16_sum2(T v) {
  v = v + dpp64<DPP_XOR1>(v);
  v = v + dpp64<DPP_XOR2>(v);
  v = v + dpp64<DPP_HMIRROR>(v);
  v = v + dpp64<DPP_MIRROR>(v);
  return v;
}

// Integer quotient e / d for small non-negative e (e·d < 2^22) via a float reciprocal.
__device__ inline int qdiv(int e, float inv) { return (int)(((float)e + 0.5f) * inv); }

}  // namespace hmcx
