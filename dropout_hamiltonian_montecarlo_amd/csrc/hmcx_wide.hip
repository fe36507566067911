// hmcx_wide.hip — SGLD for wide softmax shapes (K ≤ 64 classes; designed for BASELINE config 5:
// PlantVillage-like conv features, D = 2048, K = 38, batch 500), one or several chains: two launches
// per step (k_wfwd_sm, k_wgrad) where the forward grid is co-resident, else three (k_wfwd, k_wsoft,
// k_wgrad).
//
// Mathematics and op order: cpu/sgld.py:31-46 (p = N(0,(2ε)²) then p += −½ε·g, q += p) with the
// gradient of cpu/softmax.py:38-61 (clip, softmax, diff = y − ŷ, g = −(Xᵀ·diff − αW)), as in the
// kernel-per-phase path of hmcx_softmax.hip; only the tiling differs.  C chains share the minibatch
// (W [D][C·K] chain-interleaved, b [C][K], as at the C ABI); every kernel has a chain grid dimension.
//
//   k_wfwd   grid (row blocks of 32, D slices of ≤ 128, chains): operands straight into registers
//            (no LDS staging): wave w owns 32 features of the slice, in k-step j lane (lr, lg) holds
//            feature 32w + 8lg + j of its rows — one batch of loads, then 2·KB·8 MFMAs; the four
//            waves' partials are summed in wave order into slab[z][c][B][16·KB].
//   k_wsoft  one wave per minibatch row and chain, lane = class: Σ_z slab (fixed order), + b, clip,
//            softmax by DPP row reductions + two cross-row shuffles (every lane ends with identical
//            bits), diff = y − ŷ (gradient pass) or the log-likelihood partial per 4-row block
//            (logging pass).
//   k_wgrad  grid (G·⌈D/16⌉, chains): block g·ntile + t owns feature tile t × class group g
//            (16 × ⌈K/2⌉ weights; one group when K ≤ 16) and computes its Xᵀ·diff over the whole
//            minibatch (8 waves split the rows, summed in wave order) — no cross-workgroup
//            reduction — then updates those weights in place; feature tile 0 of each group also
//            sums its diff columns and updates the group's biases.  Its loads are issued before the
//            Philox noise is drawn, so the noise hides in their latency.
//   k_wfwd_sm k_wfwd + k_wsoft in one launch: the row team's partial logits travel as tagged granules.
// Measured (config 5, f64, one chain, MI355X): 20.6 µs per step fused, 21.9 on the three launches,
// 29.1 for the round-2 LDS-staged forward + one-workgroup-per-feature-tile gradient.
#include "hmcx_common.h"
#include "hmcx_internal.h"
#include "hmcx_p2x.h"
#include "hmcx_granule.h"
#include <algorithm>
#include <cstdio>
#include <vector>

namespace hmcx {

constexpr int WTH = 256;        // threads per workgroup of k_wfwd / k_wsoft (4 waves)
constexpr int WRB = 32;         // forward row block
constexpr int WDZ = 128;        // forward D slice (max): 4 waves × 32 features
constexpr int WSR = 4;          // rows per k_wsoft workgroup (one per wave)
constexpr int GNW = 8;          // k_wgrad waves (rows of the minibatch split over them)
constexpr int GTH = GNW * 64;

template <typename T> struct WideArgs {
  const T* X; const T* Y; T* W; T* b;
  T* pW; T* pb;                          // non-null: GPU-file momentum update (gpu/sgld.py:11-20)
  int B, D, K, KP, S, Dz, nSB, C;        // nSB: k_wsoft blocks per chain; C: chains
  T* slab; T* diff; double* llp;
  T alpha, noise_scale, m_half_eps, clip_hi, clip_lo;
  int want_diff;                         // k_wsoft: 1 = diff + colsum (gradient), 0 = ll only
  int noise_mode; const double* noise; const int64_t* noff;   // BUFFER: noise[noff[c] + e]
  uint64_t seed; uint32_t chain, step;   // PHILOX: keyed by chain + c
  unsigned long long* prof;              // HMCX_WIDE_PROF: per-workgroup s_memrealtime stamps (WPH each)
  int wt;                                // slab / diff stored write-through (sc1; HMCX_WIDE_WT=0: plain)
  // fused forward + softmax (k_wfwd_sm): the row team's partial logits travel as tagged granules
  char* gx; int gx_bytes; unsigned ep;   // the context's granule arena and this launch's epoch
  int* abort_flag;                       // the wide forward's own abort word (raised on a timed-out poll)
  int force_abort;                       // test knob (HMCX_WIDE_FORCE_ABORT): workgroup 0 raises the word
  T* trace; int P;                       // out_trace row of this step ([C][P]: W of chain c as [D][K], then b), or null
};

// a store that leaves the XCD's L2 (sc1: written through, the line dropped) or a plain one: the
// slab and diff are read by the next launch on other XCDs, so writing them through shortens the
// end-of-kernel write-back (1.79 vs 2.22 µs between k_wfwd and k_wsoft)
template <typename T> __device__ inline void wstore(T* p, T v, int wt) {
  if (wt) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}

constexpr int WPH = 8;                   // stamps per workgroup and launch (one chain only)
#define WSTAMP(ph)                                                                                  \
  do {                                                                                              \
    if (a.prof && threadIdx.x == 0)                                                                 \
      a.prof[(size_t)(blockIdx.y * gridDim.x + blockIdx.x) * WPH + (ph)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

// ---------------------------------------------------------------- partial logits, register operands
template <typename T, int KB>
__global__ __launch_bounds__(WTH) void k_wfwd(WideArgs<T> a) {
  using M = mfma16<T>;
  constexpr int KP = 16 * KB;
  __shared__ __align__(16) T red[4 * WRB * KP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  const int m0 = blockIdx.x * WRB, z = blockIdx.y, ch = blockIdx.z;
  const int dlo = min(a.D, z * a.Dz), dhi = min(a.D, dlo + a.Dz);
  const int nrow = min(WRB, a.B - m0), K = a.K, NW = a.C * K;
  const T* Wc = a.W + (size_t)ch * K;                        // chain ch's columns of W [D][C·K]
  WSTAMP(0);
  const int f0 = dlo + 32 * wave + 8 * lg;
  const int fsafe = dlo < a.D ? dlo : 0;
  T xa[2][8], wb[8][KB];
  // every load unconditional (clamped address, zeroed after the batch): one memory round trip
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int i = mt * 16 + lr;
    const T* xr = a.X + (size_t)m0 * a.D + (size_t)(i < nrow ? i : 0) * a.D;
#pragma unroll
    for (int j = 0; j < 8; ++j) xa[mt][j] = xr[f0 + j < dhi ? f0 + j : fsafe];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int nb = 0; nb < KB; ++nb) {
      const int c = nb * 16 + lr;
      wb[j][nb] = Wc[(f0 + j < dhi && c < K) ? (size_t)(f0 + j) * NW + c : 0];
    }
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (!(mt * 16 + lr < nrow && f0 + j < dhi)) xa[mt][j] = T(0);
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int nb = 0; nb < KB; ++nb)
      if (!(f0 + j < dhi && nb * 16 + lr < K)) wb[j][nb] = T(0);
  WSTAMP(1);
  typename M::acc_t acc[2][KB];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nb = 0; nb < KB; ++nb) acc[mt][nb] = M::zero();
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int nb = 0; nb < KB; ++nb) {
      acc[0][nb] = M::fma(xa[0][j], wb[j][nb], acc[0][nb]);
      acc[1][nb] = M::fma(xa[1][j], wb[j][nb], acc[1][nb]);
    }
  WSTAMP(2);
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nb = 0; nb < KB; ++nb)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        red[(wave * WRB + mt * 16 + M::row(lane, q)) * KP + nb * 16 + lr] = acc[mt][nb][q];
  WSTAMP(3);
  __syncthreads();
  WSTAMP(4);
  T* out = a.slab + (((size_t)z * a.C + ch) * a.B + m0) * KP;
  for (int e = tid; e < nrow * KP; e += WTH) {
    const T v = ((red[e] + red[WRB * KP + e]) + red[2 * WRB * KP + e]) + red[3 * WRB * KP + e];
    wstore(out + e, v, a.wt);
  }
  WSTAMP(5);
  WSTAMP(6);
}

// Wave-wide all-reductions: every step combines a symmetric pair of lanes, so all lanes hold the
// same bits and the result is deterministic.  Within each 16-lane row by DPP (g16_*: xor 1, xor 2,
// half mirror, mirror), then across the four rows by two shuffles (xor 16, xor 32).
template <typename T> __device__ inline T wave_sum(T v) {
  v = g16_sum2(v);
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}
template <typename T> __device__ inline T wave_max(T v) {                  // NaN on either side wins
  v = g16_max2(v);
  v = max_nan(v, __shfl_xor(v, 16, 64));
  v = max_nan(v, __shfl_xor(v, 32, 64));
  return v;
}

// ---------------------------------------------------------------- softmax rows
template <typename T>
__global__ __launch_bounds__(WTH) void k_wsoft(WideArgs<T> a) {
  __shared__ double ll[WSR];
  const int tid = threadIdx.x, k = tid & 63, wave = tid >> 6, ch = blockIdx.y;
  const int row = blockIdx.x * WSR + wave, K = a.K, KP = a.KP;
  const bool rv = row < a.B, kv = rv && k < K;
  WSTAMP(0);
  T d = T(0);
  double t = 0.0;
  if (rv) {
    // Σ_z slab[z] in slab order; the slab loads go out in batches of 16 (unconditional: lanes
    // k ≥ K read their row's padding columns, which exist in every slab)
    const size_t zstride = (size_t)a.C * a.B * KP;
    const T* sp = a.slab + ((size_t)ch * a.B + row) * KP + min(k, KP - 1);
    T xw = T(0);
    for (int s0 = 0; s0 < a.S; s0 += 16) {
      T v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = sp[(size_t)min(s0 + q, a.S - 1) * zstride];
#pragma unroll
      for (int q = 0; q < 16; ++q)
        if (s0 + q < a.S) xw = (s0 + q == 0) ? v[q] : xw + v[q];
    }
    if (wave == 0) WSTAMP(1);
    const int kc = min(k, K - 1);
    const T bk = a.b[ch * K + kc], yk = a.Y[(size_t)row * K + kc];                        // unconditional loads
    const T zz = kv ? clipz(xw + bk, a.clip_hi, a.clip_lo) : (T)-__builtin_inf();          // softmax.py:39-41
    const T m = wave_max(zz);
    const T e = kv ? exp(zz - m) : T(0);                                                  // softmax.py:34
    const T s = wave_sum(e);
    const T y = kv ? yk : T(0);
    if (a.want_diff) {
      d = kv ? y - e / s : T(0);                                                          // softmax.py:52
      if (k < KP) wstore(a.diff + ((size_t)ch * a.B + row) * KP + k, d, a.wt);
    } else {
      const T lse = log(s) + m;                                                           // softmax.py:18-20
      t = kv ? (double)(y * (zz - lse)) : 0.0;
      t = wave_sum(t);
    }
  }
  WSTAMP(2);
  if (!a.want_diff) {                  // the logging pass: ll partial of the block's rows
    if (k == 0) ll[wave] = t;
    __syncthreads();
    if (tid == 0) a.llp[(size_t)ch * a.nSB + blockIdx.x] = ((ll[0] + ll[1]) + ll[2]) + ll[3];
  }
  WSTAMP(3);
}

// One softmax row (lane = class): Σ_z of the row's partials in slice order (the caller's sum), + b,
// clip, softmax by wave reductions; the diff row (gradient pass) or the row's log-likelihood term.
template <typename T>
__device__ inline double wide_softmax_row(const WideArgs<T>& a, int ch, int row, int k, T xw, T bk, T yk) {
  const int K = a.K;
  const bool kv = k < K;
  const T zz = kv ? clipz(xw + bk, a.clip_hi, a.clip_lo) : (T)-__builtin_inf();            // softmax.py:39-41
  const T m = wave_max(zz);
  const T e = kv ? exp(zz - m) : T(0);                                                    // softmax.py:34
  const T s = wave_sum(e);
  const T y = kv ? yk : T(0);
  if (a.want_diff) {
    const T d = kv ? y - e / s : T(0);                                                    // softmax.py:52
    if (k < a.KP) wstore(a.diff + ((size_t)ch * a.B + row) * a.KP + k, d, a.wt);
    return 0.0;
  }
  const T lse = log(s) + m;                                                               // softmax.py:18-20
  return wave_sum(kv ? (double)(y * (zz - lse)) : 0.0);
}

template <typename T> __device__ inline T wide_ld(__amdgpu_buffer_rsrc_t rs, int off) {
  if constexpr (sizeof(T) == 8)
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0));
  else
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
}

// ---------------------------------------------------------------- fused forward + softmax
// k_wfwd's partial logits, then ONE team round instead of a kernel boundary and k_wsoft: the S
// workgroups of a row block (its D slices) publish their 32 × K partials as tagged granules
// (hmcx_granule.h), workgroup z owns rows [z·R, z·R + R) (R = ⌈32/S⌉), gathers their S partials
// (pairs dealt over all threads, landing in LDS), sums them in slice order — the order k_wsoft sums
// the slab in, so the logits are bit-identical — and runs the softmax rows.  The grid must be
// co-resident (checked on the host); polls are bounded (2 s) and raise the wide abort word.
constexpr int WSM_STAGE = 8 * WTH;       // gathered (slice, row, class) partials per workgroup (LDS)
template <typename T, int KB>
__global__ __launch_bounds__(WTH) void k_wfwd_sm(WideArgs<T> a) {
  using M = mfma16<T>;
  constexpr int KP = 16 * KB;
  __shared__ __align__(16) T red[4 * WRB * KP];
  __shared__ double stage[WSM_STAGE];
  __shared__ double llw[4];
  __shared__ int fail;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  const int m0 = blockIdx.x * WRB, z = blockIdx.y, ch = blockIdx.z;
  const int dlo = min(a.D, z * a.Dz), dhi = min(a.D, dlo + a.Dz);
  const int nrow = min(WRB, a.B - m0), K = a.K, NW = a.C * K, S = a.S;
  WSTAMP(0);
  if (tid == 0) fail = 0;
  const int f0 = dlo + 32 * wave + 8 * lg;
  // operands by buffer loads issued k-step by k-step: an element outside the tile (row past the
  // minibatch, feature past the slice, class past K) gets an out-of-range offset and reads 0 with no
  // memory request, so nothing is masked after the batch and the MFMAs of step j wait only for the
  // loads of steps ≤ j (the loads of the later steps are still landing)
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<T*>(a.X) + (size_t)m0 * a.D, 0, nrow * a.D * (int)sizeof(T), 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      a.W + (size_t)ch * K, 0, (a.D * NW - ch * K) * (int)sizeof(T), 0x00020000);
  constexpr int OOB = 0x7fffffff;
  T xa[2][8], wb[8][KB];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const bool fok = f0 + j < dhi;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int off = fok ? ((mt * 16 + lr) * a.D + f0 + j) * (int)sizeof(T) : OOB;
      xa[mt][j] = wide_ld<T>(xrs, off);
    }
#pragma unroll
    for (int nb = 0; nb < KB; ++nb) {
      const int c = nb * 16 + lr;
      const int off = (fok && c < K) ? ((f0 + j) * NW + c) * (int)sizeof(T) : OOB;
      wb[j][nb] = wide_ld<T>(wrs, off);
    }
  }
  // softmax operands of this wave's first owned row (b and the labels), loaded while the partials travel
  const int R = (WRB + S - 1) / S;
  const int r0 = min(nrow, z * R), r1 = min(nrow, r0 + R);
  const int kc = min(lane, K - 1);
  const T bk = a.b[ch * K + kc];
  const T yk0 = a.Y[(size_t)(m0 + min(r0 + wave, nrow - 1)) * K + kc];
  WSTAMP(1);
  typename M::acc_t acc[2][KB];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nb = 0; nb < KB; ++nb) acc[mt][nb] = M::zero();
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int nb = 0; nb < KB; ++nb) {
      acc[0][nb] = M::fma(xa[0][j], wb[j][nb], acc[0][nb]);
      acc[1][nb] = M::fma(xa[1][j], wb[j][nb], acc[1][nb]);
    }
  WSTAMP(2);
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nb = 0; nb < KB; ++nb)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        red[(wave * WRB + mt * 16 + M::row(lane, q)) * KP + nb * 16 + lr] = acc[mt][nb][q];
  __syncthreads();
  // publish the workgroup's partial (the 4 waves summed in wave order, as k_wfwd's slab entry)
  const __amdgpu_buffer_rsrc_t rs = gx_rsrc(a.gx, a.gx_bytes);
  const int blk = WRB * K;                                       // granules per producer
  const int team = (ch * gridDim.x + blockIdx.x) * S;            // first producer block of my team
  for (int e = tid; e < nrow * K; e += WTH) {
    const int i = e / K, k = e - (e / K) * K, x = i * KP + k;
    const T v = ((red[x] + red[WRB * KP + x]) + red[2 * WRB * KP + x]) + red[3 * WRB * KP + x];
    gx_put(rs, (team + z) * blk + e, (double)v, a.ep);
  }
  if (a.force_abort && blockIdx.x == 0 && z == 0 && ch == 0 && tid == 0)
    __hip_atomic_store(a.abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  WSTAMP(3);
  // gather my rows' partials from the S producers: pair q = p·nit + it, it = row-in-slice·K + class
  const int nit = (r1 - r0) * K, npair = S * nit;
  {
    typedef unsigned int g4 __attribute__((ext_vector_type(4)));
    constexpr int U = WSM_STAGE / WTH;
    unsigned pend = 0;
    int o[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = tid + u * WTH;
      const int p = q / max(nit, 1), it = q - p * max(nit, 1);
      const bool w = q < npair;
      pend |= w ? 1u << u : 0u;
      o[u] = w ? ((team + p) * blk + r0 * K + it) * 16 : 0;
    }
    unsigned long long t0 = 0;
    bool ok = true;
    for (int spins = 0; pend; ++spins) {
      g4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, o[u], 0, 16 /* sc1 */);
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (((pend >> u) & 1u) && v[u].y == a.ep && v[u].w == a.ep) {
          stage[tid + u * WTH] = __builtin_bit_cast(double, (unsigned long long)v[u].x | ((unsigned long long)v[u].z << 32));
          pend &= ~(1u << u);
        }
      if (!pend) break;
      if (spins == 0) t0 = __builtin_amdgcn_s_memrealtime();
      if ((spins & 63) == 63 && (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull ||
                                 __hip_atomic_load(a.abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
        __hip_atomic_store(a.abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (!ok) fail = 1;
  }
  __syncthreads();
  WSTAMP(4);
  if (fail) return;                    // the host sees the abort word and re-runs the call unfused
  double t = 0.0;
  for (int row = r0 + wave; row < r1; row += 4) {
    const int ri = (row - r0) * K + kc;
    T xw = (T)stage[ri];
    // Σ over the S slices in slice order (k_wsoft's slab order), the LDS reads of 16 slices at a time
    // issued together (a runtime-length loop waited for each read before the next add)
    for (int p0 = 1; p0 < S; p0 += 16) {
      double v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = stage[min(p0 + q, S - 1) * nit + ri];
#pragma unroll
      for (int q = 0; q < 16; ++q)
        if (p0 + q < S) xw = xw + (T)v[q];
    }
    const T yk = row == r0 + wave ? yk0 : a.Y[(size_t)(m0 + row) * K + kc];
    t += wide_softmax_row(a, ch, m0 + row, lane, xw, bk, yk);
  }
  WSTAMP(5);
  if (!a.want_diff) {                  // the logging pass: ll partial of my rows (waves in order)
    if (lane == 0) llw[wave] = t;
    __syncthreads();
    if (tid == 0) a.llp[((size_t)ch * gridDim.x + blockIdx.x) * S + z] = ((llw[0] + llw[1]) + llw[2]) + llw[3];
  }
  WSTAMP(6);
}

template <typename T>
__device__ inline double wide_noise(const WideArgs<T>& a, int ch, uint32_t e) {
  if (a.noise_mode == HMCX_NOISE_BUFFER) return a.noise[a.noff[ch] + e];
  return (double)philox_normal_t<T>(a.seed, a.chain + (uint32_t)ch, a.step, 0u, e);
}

// ---------------------------------------------------------------- Xᵀ·diff + SGLD update
// Class grouping of k_wgrad: K ≤ 16 → one group; otherwise two groups of ⌈K/2⌉ classes (config 5:
// 2 × 19), each NT = ⌈group/16⌉ MFMA column tiles.  One workgroup per (feature tile, group): 256 of
// them at config 5, one per CU, with the same bytes and MFMAs each (three 16-class tiles gave 385
// workgroups, 129 CUs with two and twice the load traffic and MFMA issue of the others).  The bias
// gradient Σ_rows diff falls out of the same diff loads; feature tile 0 of each group applies it (no
// bias block, no column-sum partials from k_wsoft).
// Group widths are even (config 5: 20 + 18), so a group's first class starts a 16-byte pair: the f64
// kernel with two column tiles loads its diff operands as class PAIRS (one 16-byte load per lane and
// row: classes c0 + 2·lr and c0 + 2·lr + 1), and its two accumulators hold the even and the odd classes
// of the group — one load instruction per k-step instead of two, and fewer, fuller L2 requests
// (the gradient's load phase is bound by the requests a CU keeps in flight).
struct WGroups { int G, GW, NT; };
__host__ __device__ inline WGroups wide_groups(int K) {
  if (K <= 16) return {1, K, 1};
  const int gw = ((K + 1) / 2 + 1) & ~1;
  return {2, gw, (gw + 15) / 16};
}

template <typename T, int NT, int U>
__global__ __launch_bounds__(GTH) void k_wgrad(WideArgs<T> a) {
  using M = mfma16<T>;
  constexpr bool PAIR = NT == 2 && sizeof(T) == 8;    // class-pair operands (wide_groups)
  __shared__ T red[GNW][16][NT * 16 + 1];
  __shared__ T cs[GNW][NT * 16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  const int ch = blockIdx.y;
  WSTAMP(0);
  const int ntile = (a.D + 15) / 16;
  const WGroups gr = wide_groups(a.K);
  const int grp = blockIdx.x / ntile, t = blockIdx.x - grp * ntile;
  const int d0 = t * 16, K = a.K, B = a.B, KP = a.KP, NW = a.C * K;
  const int c0 = grp * gr.GW, c1 = min(K, c0 + gr.GW);        // my classes [c0, c1)
  const bool dok = d0 + lr < a.D;
  const int dcol = dok ? d0 + lr : 0;
  const int nks = (B + 3) / 4, Q = (nks + GNW - 1) / GNW;
  const int kb0 = wave * Q, kb1 = min(nks, kb0 + Q);
  // diff [C][B][KP] read through a range-checked buffer: a column outside [c0, c1) or a row past the
  // minibatch gets an out-of-range offset and reads 0 without a memory request (the padded classes of
  // a group cost no bytes)
  const __amdgpu_buffer_rsrc_t drs = __builtin_amdgcn_make_buffer_rsrc(
      a.diff + (size_t)ch * B * KP, 0, B * KP * (int)sizeof(T), 0x00020000);
  int col[NT];
  bool cok[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    col[j] = PAIR ? c0 + 2 * lr + j : c0 + j * 16 + lr;      // PAIR: col[0] even, col[1] = col[0] + 1
    cok[j] = PAIR ? c0 + 2 * lr < c1 : col[j] < c1;
  }
  // my epilogue element: feature d0 + tid / GW, class c0 + tid % GW (threads 0 … 16·GW − 1)
  const int ei = tid / gr.GW, ek = c0 + (tid - (tid / gr.GW) * gr.GW);
  const bool eok = tid < 16 * gr.GW && d0 + ei < a.D && ek < c1;
  const uint32_t el = eok ? (uint32_t)((d0 + ei) * K + ek) : 0u;            // element of the chain's P
  const size_t wi = eok ? (size_t)(d0 + ei) * NW + (size_t)ch * K + ek : 0;  // its place in W [D][C·K]
  const bool gpu_var = a.pW != nullptr;
  const T* psrc = gpu_var ? a.pW : a.W;
  typename M::acc_t acc[NT];
  T csum[NT];                          // Σ_rows diff of my columns (the bias gradient, softmax.py:59)
#pragma unroll
  for (int j = 0; j < NT; ++j) { acc[j] = M::zero(); csum[j] = T(0); }
  T wv = T(0), pv = T(0), zv = T(0);
  bool first = true;
  for (int ks = kb0; ks < kb1 || first; ks += U) {
    T av[U], bv[U][NT];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = (ks + u) * 4 + lg;
      const bool ok = ks + u < kb1 && row < B;
      const size_t rr = ok ? (size_t)row : 0;
      av[u] = a.X[rr * a.D + dcol];
      if constexpr (PAIR) {
        // classes c0 + 2·lr, c0 + 2·lr + 1 (the odd one may be the padding past c1: its column is unused)
        const int off = (ok && cok[0]) ? (row * KP + col[0]) * (int)sizeof(T) : 0x7fffffff;
        typedef double dd2 __attribute__((ext_vector_type(2)));
        const dd2 q = __builtin_bit_cast(dd2, __builtin_amdgcn_raw_buffer_load_b128(drs, off, 0, 0));
        bv[u][0] = (T)q.x;
        bv[u][1] = (T)q.y;
      } else {
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int off = (ok && cok[j]) ? (row * KP + col[j]) * (int)sizeof(T) : 0x7fffffff;
          if constexpr (sizeof(T) == 8)
            bv[u][j] = __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(drs, off, 0, 0));
          else
            bv[u][j] = __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(drs, off, 0, 0));
        }
      }
      if (!(ok && dok)) av[u] = T(0);
    }
    if (first) {                       // epilogue operands and noise while the first batch is in flight
      first = false;
      wv = a.W[wi];
      pv = psrc[wi];
      zv = (T)wide_noise(a, ch, el);
      WSTAMP(1);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        acc[j] = M::fma(av[u], bv[u][j], acc[j]);
        csum[j] += bv[u][j];
      }
  }
  WSTAMP(2);
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int cc = PAIR ? 2 * lr + j : j * 16 + lr;     // class of accumulator column lr, within the group
#pragma unroll
    for (int q = 0; q < 4; ++q) red[wave][M::row(lane, q)][cc] = acc[j][q];
    // the four row groups of a column (lanes lr, lr + 16, lr + 32, lr + 48), symmetric pairs
    T v = csum[j];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    if (lg == 0) cs[wave][cc] = v;
  }
  __syncthreads();
  WSTAMP(3);
  if (t == 0 && tid < c1 - c0) {       // feature tile 0 of each group also finishes the group's biases
    const int c = c0 + tid, bi = ch * K + c;
    T colsum = cs[0][tid];
#pragma unroll
    for (int w = 1; w < GNW; ++w) colsum += cs[w][tid];
    const T bb = a.b[bi];
    const T gb = -(colsum - a.alpha * bb);                                   // softmax.py:55,59-60
    T p = a.noise_scale * (T)wide_noise(a, ch, (uint32_t)(a.D * K + c));     // sgld.py:43-46
    if (gpu_var) p = p * a.pb[bi];                                           // gpu/sgld.py:18
    p = p + a.m_half_eps * gb;                                               // sgld.py:37
    if (gpu_var) a.pb[bi] = p;
    a.b[bi] = bb + p;                                                        // sgld.py:38
    if (a.trace) a.trace[(size_t)ch * a.P + (size_t)a.D * K + c] = bb + p;  // the step's state row
  }
  if (eok) {
    const int cc = ek - c0;
    T dot = red[0][ei][cc];
#pragma unroll
    for (int w = 1; w < GNW; ++w) dot += red[w][ei][cc];
    const T gr_ = -(dot - a.alpha * wv);                                       // softmax.py:57-58
    T p = a.noise_scale * zv;                                                  // sgld.py:43-46
    if (gpu_var) p = p * pv;                                                   // gpu/sgld.py:18
    p = p + a.m_half_eps * gr_;                                                // sgld.py:37
    if (gpu_var) a.pW[wi] = p;
    a.W[wi] = wv + p;                                                          // sgld.py:38
    if (a.trace) a.trace[(size_t)ch * a.P + el] = wv + p;
  }
  WSTAMP(4);
  WSTAMP(5);
}

__global__ void k_wreduce_ll(const double* llp, int n, double* out) {   // block = chain
  __shared__ double sh[256];
  const double* p = llp + (size_t)blockIdx.x * n;
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) s += p[i];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int m = 128; m > 0; m >>= 1) {
    if ((int)threadIdx.x < m) sh[threadIdx.x] += sh[threadIdx.x + m];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = sh[0];
}

// ---------------------------------------------------------------- host
bool sgld_wide_eligible(const hmcx_sampler_args* s) {
  const char* env = getenv("HMCX_SGLD_WIDE");
  if (env && env[0] == '0') return false;        // 0: kernel-per-phase path
  if (s->K > 64 || s->K < 1 || s->B < 1 || s->D < 1 || s->C < 1 || s->C > 65535) return false;
  // one chain: faster than the kernel-per-phase path for every shape measured (MNIST D=784, K=10:
  // 18.0 vs 20.5 µs per f64 step; config 5: 22.8 vs 35.1 µs).  Several chains: when a chain's K
  // classes fill most of the 16-wide class tiles (K > 16); at K = 10 the kernel-per-phase path packs
  // the chains' columns together instead
  return s->C == 1 || s->K > 16 || (env && env[0] == '1');
}

template <typename T, int KB>
static void launch_fwd_kb(const WideArgs<T>& a, hipStream_t st) {
  hipLaunchKernelGGL((k_wfwd<T, KB>), dim3((a.B + WRB - 1) / WRB, a.S, a.C), dim3(WTH), 0, st, a);
}
template <typename T>
static void launch_fwd(const WideArgs<T>& a, hipStream_t st) {
  switch (a.KP / 16) {
    case 1: launch_fwd_kb<T, 1>(a, st); break;
    case 2: launch_fwd_kb<T, 2>(a, st); break;
    case 3: launch_fwd_kb<T, 3>(a, st); break;
    default: launch_fwd_kb<T, 4>(a, st); break;
  }
}

template <typename T, int KB>
static void launch_fwd_sm_kb(const WideArgs<T>& a, hipStream_t st) {
  hipLaunchKernelGGL((k_wfwd_sm<T, KB>), dim3((a.B + WRB - 1) / WRB, a.S, a.C), dim3(WTH), 0, st, a);
}
template <typename T>
static void launch_fwd_sm(const WideArgs<T>& a, hipStream_t st) {
  switch (a.KP / 16) {
    case 1: launch_fwd_sm_kb<T, 1>(a, st); break;
    case 2: launch_fwd_sm_kb<T, 2>(a, st); break;
    case 3: launch_fwd_sm_kb<T, 3>(a, st); break;
    default: launch_fwd_sm_kb<T, 4>(a, st); break;
  }
}
template <typename T>
static const void* fwd_sm_fn(int KP) {
  switch (KP / 16) {
    case 1: return (const void*)k_wfwd_sm<T, 1>;
    case 2: return (const void*)k_wfwd_sm<T, 2>;
    case 3: return (const void*)k_wfwd_sm<T, 3>;
    default: return (const void*)k_wfwd_sm<T, 4>;
  }
}

template <typename T>
static int sgld_wide_impl(hmcx_ctx* ctx, const hmcx_sampler_args* s, bool allow_fuse);

template <typename T>
int sgld_wide_t(hmcx_ctx* ctx, const hmcx_sampler_args* s) {
  return sgld_wide_impl<T>(ctx, s, true);
}

template <typename T>
static int sgld_wide_impl(hmcx_ctx* ctx, const hmcx_sampler_args* s, bool allow_fuse) {
  const int B = s->B, D = s->D, K = s->K, C = s->C, KP = (K + 15) / 16 * 16;
  const int S = (D + WDZ - 1) / WDZ, Dz = ((D + S - 1) / S + 3) / 4 * 4;
  const int nSB = (B + WSR - 1) / WSR;
  const int nRB = (B + WRB - 1) / WRB;
  const int ntile = (D + 15) / 16;
  const size_t nsc = (size_t)s->n_steps * C;
  // fused forward + softmax (k_wfwd_sm: one team round instead of k_wsoft and a kernel boundary) when
  // the whole forward grid is co-resident and a workgroup's gathered partials fit its LDS stage;
  // HMCX_WIDE_FUSE=0 keeps the three launches
  const int fuse_env = getenv("HMCX_WIDE_FUSE") ? atoi(getenv("HMCX_WIDE_FUSE")) : 1;     // read per call (tests)
  bool fuse = allow_fuse && !ctx->wide_nofuse && fuse_env != 0 && S * ((WRB + S - 1) / S) * K <= WSM_STAGE;
  // out_abort set: the call's verdict is stream-ordered into it and the caller, which keeps the start
  // state, re-runs a timed-out call itself — no snapshot here and no wait for the stream
  const bool defer = s->out_abort != nullptr;
  if (fuse) {
    int per_cu = 0, rc0 = kernel_occupancy(ctx, fwd_sm_fn<T>(KP), WTH, 0, &per_cu);
    if (rc0) return rc0;
    fuse = (long)per_cu * ctx->num_cus >= (long)nRB * S * C;
  }
  // HMCX_WIDE_PROF=<file> (one chain): stamps of the first 64 steps' launches, appended to <file> after
  // the call (header: steps, workgroups of k_wfwd(_sm), k_wsoft, k_wgrad, WPH; tools/wide_prof_summary.py)
  static const char* prof_path = getenv("HMCX_WIDE_PROF");
  const WGroups wg = wide_groups(K);
  const int GF = nRB * S, GS = nSB, GG = wg.G * ntile, GALL = GF + GS + GG;
  const int nprof = (prof_path && C == 1) ? std::min(s->n_steps, 64) : 0;
  const bool buf = s->noise_mode == HMCX_NOISE_BUFFER;
  Workspace ws(ctx);
  T *slab, *diff;
  double* llp;
  int64_t* d_noff = nullptr;
  unsigned long long* prof = nullptr;
  T *snapW = nullptr, *snapb = nullptr, *snappW = nullptr, *snappb = nullptr;
  const size_t nW = (size_t)D * C * K, nb = (size_t)C * K;
  do {
    ws.reset();
    slab = fuse ? nullptr : ws.take<T>((size_t)S * C * B * KP);
    diff = ws.take<T>((size_t)C * B * KP);
    llp = ws.take<double>((size_t)C * std::max(nSB, nRB * S));
    if (fuse && !defer) {              // the call's start state, for the unfused re-run after a timeout
      snapW = ws.take<T>(nW);
      snapb = ws.take<T>(nb);
      if (s->pW) { snappW = ws.take<T>(nW); snappb = ws.take<T>(nb); }
    }
    if (buf) d_noff = ws.take<int64_t>(nsc);
    if (nprof) prof = ws.take<unsigned long long>((size_t)nprof * GALL * WPH);
  } while (ws.retry());
  if (ws.failed) return HMCX_ENOMEM;
  int rc;
  unsigned ep0 = 0;
  if (fuse) {
    if (!ctx->wide_abort_dev) {        // its own word (hmcx_internal.h), allocated on first use
      HMCX_HIP(ctx, hipMalloc((void**)&ctx->wide_abort_dev, sizeof(int)));
      HMCX_HIP(ctx, hipMemsetAsync(ctx->wide_abort_dev, 0, sizeof(int), ctx->stream));
    }
    unsigned nfwd = 0;
    for (int i = 0; i < s->n_steps; ++i) nfwd += 1u + ((s->want_ll && s->want_ll[i] && s->out_ll) ? 1u : 0u);
    if ((rc = gx_reserve(ctx, (size_t)nRB * S * C * WRB * K * 16))) return rc;
    if ((rc = gx_epochs(ctx, nfwd, &ep0))) return rc;
  }
  begin_call(ctx);
  if (buf && (rc = upload(ctx, d_noff, s->noise_off, nsc * sizeof(int64_t)))) return rc;
  if (fuse && !defer) {
    HMCX_HIP(ctx, hipMemcpyAsync(snapW, s->W, nW * sizeof(T), hipMemcpyDeviceToDevice, ctx->stream));
    HMCX_HIP(ctx, hipMemcpyAsync(snapb, s->b, nb * sizeof(T), hipMemcpyDeviceToDevice, ctx->stream));
    if (snappW) {
      HMCX_HIP(ctx, hipMemcpyAsync(snappW, s->pW, nW * sizeof(T), hipMemcpyDeviceToDevice, ctx->stream));
      HMCX_HIP(ctx, hipMemcpyAsync(snappb, s->pb, nb * sizeof(T), hipMemcpyDeviceToDevice, ctx->stream));
    }
  }
  const int force_abort = getenv("HMCX_WIDE_FORCE_ABORT") ? atoi(getenv("HMCX_WIDE_FORCE_ABORT")) : -1;
  WideArgs<T> a{};
  a.gx = ctx->gx_arena; a.gx_bytes = (int)std::min<size_t>(ctx->gx_bytes, 0x7fffffff);
  a.abort_flag = ctx->wide_abort_dev;        // polled only by k_wfwd_sm (null before the first fused call)
  a.W = (T*)s->W; a.b = (T*)s->b; a.pW = (T*)s->pW; a.pb = (T*)s->pb;
  a.B = B; a.D = D; a.K = K; a.KP = KP; a.S = S; a.Dz = Dz; a.nSB = nSB; a.C = C;
  a.slab = slab; a.diff = diff; a.llp = llp;
  a.alpha = (T)s->alpha;
  a.clip_hi = (T)CLIP_HI; a.clip_lo = (T)CLIP_LO;
  a.noise_mode = s->noise_mode; a.noise = s->noise;
  a.seed = s->seed; a.chain = s->chain0;
  static const int wt_env = getenv("HMCX_WIDE_WT") ? atoi(getenv("HMCX_WIDE_WT")) : 1;
  a.wt = wt_env;
  if ((rc = timing_begin(ctx, ctx->stream))) return rc;
  GraphScope gs(ctx);
  hipStream_t st = ctx->stream;
  const dim3 ggrid(GG, C), sgrid(nSB, C);
  for (int i = 0; i < s->n_steps; ++i) {
    a.X = (const T*)s->X + (size_t)s->row0[i] * D;
    a.Y = (const T*)s->Y + (size_t)s->row0[i] * K;
    const double eps = s->eps[i];
    a.noise_scale = (T)(2.0 * eps);                                   // sgld.py:43
    a.m_half_eps = (T)(-0.5 * eps);                                   // sgld.py:37
    a.step = s->step_base + (uint32_t)i;
    a.noff = buf ? d_noff + (size_t)i * C : nullptr;
    a.want_diff = 1;
    // sghmc_multicore.py:49-51's per-step state row, stored by k_wgrad's update itself
    a.trace = s->out_trace ? (T*)s->out_trace + (size_t)i * C * (D * K + K) : nullptr;
    a.P = D * K + K;
    unsigned long long* pr = i < nprof ? prof + (size_t)i * GALL * WPH : nullptr;
    a.prof = pr;
    if (fuse) {
      a.ep = ep0++;
      a.force_abort = i == force_abort;
      launch_fwd_sm<T>(a, st);
      a.force_abort = 0;
    } else {
      launch_fwd<T>(a, st);
      a.prof = pr ? pr + (size_t)GF * WPH : nullptr;
      hipLaunchKernelGGL(k_wsoft<T>, sgrid, dim3(WTH), 0, st, a);
    }
    a.prof = pr ? pr + (size_t)(GF + GS) * WPH : nullptr;
    // one chain: 16 k-steps of loads per batch (one batch at B = 500, one workgroup per CU);
    // several chains: 8 per batch, so that two workgroups fit on a CU (C = 8 at config 5: 92.7 → see
    // DESIGN §5.4)
    if (wg.NT == 1) {
      if (C == 1) hipLaunchKernelGGL((k_wgrad<T, 1, 16>), ggrid, dim3(GTH), 0, st, a);
      else hipLaunchKernelGGL((k_wgrad<T, 1, 8>), ggrid, dim3(GTH), 0, st, a);
    } else {
      if (C == 1) hipLaunchKernelGGL((k_wgrad<T, 2, 16>), ggrid, dim3(GTH), 0, st, a);
      else hipLaunchKernelGGL((k_wgrad<T, 2, 8>), ggrid, dim3(GTH), 0, st, a);
    }
    a.prof = nullptr;
    HMCX_HIP(ctx, hipGetLastError());
    if (s->want_ll && s->want_ll[i] && s->out_ll) {                   // sgmcmc.py:61 logging
      a.want_diff = 0;
      if (fuse) {
        a.ep = ep0++;
        launch_fwd_sm<T>(a, st);
        hipLaunchKernelGGL(k_wreduce_ll, dim3(C), dim3(256), 0, st, (const double*)llp, nRB * S,
                           s->out_ll + (size_t)i * C);
      } else {
        launch_fwd<T>(a, st);
        hipLaunchKernelGGL(k_wsoft<T>, sgrid, dim3(WTH), 0, st, a);
        hipLaunchKernelGGL(k_wreduce_ll, dim3(C), dim3(256), 0, st, (const double*)llp, nSB, s->out_ll + (size_t)i * C);
      }
      HMCX_HIP(ctx, hipGetLastError());
    }
  }
  if ((rc = gs.finish())) return rc;
  if ((rc = timing_end(ctx, ctx->stream))) return rc;
  if (defer) {
    // the verdict (1: a team round timed out, W / b are invalid) into the caller's slot and the word
    // lowered, both stream-ordered: the call returns without waiting for its kernels
    if (fuse) {
      HMCX_HIP(ctx, hipMemcpyAsync(s->out_abort, ctx->wide_abort_dev, sizeof(int), hipMemcpyDeviceToDevice, ctx->stream));
      HMCX_HIP(ctx, hipMemsetAsync(ctx->wide_abort_dev, 0, sizeof(int), ctx->stream));
    } else {
      HMCX_HIP(ctx, hipMemsetAsync(s->out_abort, 0, sizeof(int32_t), ctx->stream));
    }
  } else if (fuse) {
    // a timed-out team round raised the wide abort word (the launch's workgroups then stopped early): put
    // the call's start state back, lower the word and run the call again on the three-launch path — same
    // operands, same noise, so the result is the one the fused call would have given.  The check waits
    // for the stream, so a fused hmcx_sgld_run call returns only when its kernels are done (one wait
    // per call: sample() makes one call per epoch); the re-run is counted (hmcx_get_recoveries)
    int flag = 0;
    HMCX_HIP(ctx, hipMemcpyAsync(&flag, ctx->wide_abort_dev, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    HMCX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (flag) {
      HMCX_HIP(ctx, hipMemsetAsync(ctx->wide_abort_dev, 0, sizeof(int), ctx->stream));
      ++ctx->recoveries[HMCX_RECOVERY_WIDE_FUSED];
      HMCX_HIP(ctx, hipMemcpyAsync(s->W, snapW, nW * sizeof(T), hipMemcpyDeviceToDevice, ctx->stream));
      HMCX_HIP(ctx, hipMemcpyAsync(s->b, snapb, nb * sizeof(T), hipMemcpyDeviceToDevice, ctx->stream));
      if (snappW) {
        HMCX_HIP(ctx, hipMemcpyAsync(s->pW, snappW, nW * sizeof(T), hipMemcpyDeviceToDevice, ctx->stream));
        HMCX_HIP(ctx, hipMemcpyAsync(s->pb, snappb, nb * sizeof(T), hipMemcpyDeviceToDevice, ctx->stream));
      }
      HMCX_HIP(ctx, hipStreamSynchronize(ctx->stream));     // the snapshot lives in the workspace
      fprintf(stderr, "[hmcx] wide SGLD: a team round timed out; call re-run on the three-launch path\n");
      return sgld_wide_impl<T>(ctx, s, false);
    }
  }
  if (nprof) {
    std::vector<unsigned long long> h((size_t)nprof * GALL * WPH);
    HMCX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    HMCX_HIP(ctx, hipMemcpy(h.data(), prof, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    if (FILE* f = fopen(prof_path, "ab")) {
      const int hdr[5] = {nprof, GF, GS, GG, WPH};
      fwrite(hdr, sizeof(int), 5, f);
      fwrite(h.data(), sizeof(unsigned long long), h.size(), f);
      fclose(f);
    }
  }
  return HMCX_OK;
}

template int sgld_wide_t<float>(hmcx_ctx*, const hmcx_sampler_args*);
template int sgld_wide_t<double>(hmcx_ctx*, const hmcx_sampler_args*);

}  // namespace hmcx
