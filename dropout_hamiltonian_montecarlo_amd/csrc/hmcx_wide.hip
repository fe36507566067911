// hmcx_wide.hip — single-chain SGLD (any K ≤ 64; designed for BASELINE config 5: PlantVillage-like
// conv features, D = 2048, K = 38, batch 500), three launches per step.
//
// Mathematics and op order: cpu/sgld.py:31-46 (p = N(0,(2ε)²) then p += −½ε·g, q += p) with the
// gradient of cpu/softmax.py:38-61 (clip, softmax, diff = y − ŷ, g = −(Xᵀ·diff − αW)), as in the
// kernel-per-phase path of hmcx_softmax.hip; only the tiling differs.
//
//   k_wfwd   grid (row blocks of 32, D slices of ≤128): the X tile [32 × Dz] and the weight slice
//            [Dz × 16·KB] are staged through LDS with 16-byte loads, every wave runs all 2·KB MFMA
//            tiles over a quarter of the slice, the four partials are summed in wave order and the
//            slice's partial logits go to slab[z][B][16·KB].
//   k_wsoft  one wave per minibatch row, lane = class: Σ_z slab (fixed order), + b, clip, softmax
//            by wave butterflies (every lane ends with identical bits), diff = y − ŷ, column-sum and
//            log-likelihood partials per 4-row block.
//   k_wgrad  grid = 16-feature tiles: Xᵀ·diff over the whole minibatch on MFMA (rows split over the
//            four waves, summed in wave order), then the fused SGLD update of the tile's weights;
//            block 0 also finishes the bias from the column-sum partials.
// The kernel-per-phase path served this shape with 16-row forward tiles whose epilogue walks the
// K = 38 classes serially; here the class dimension lives in the lanes.
#include "hmcx_common.h"
#include "hmcx_internal.h"
#include "hmcx_p2x.h"
#include <algorithm>
#include <cstdio>
#include <vector>

namespace hmcx {

constexpr int WTH = 256;        // threads per workgroup (4 waves)
constexpr int WRB = 32;         // forward row block
#ifndef HMCX_WDZ
#define HMCX_WDZ 128
#endif
#ifndef HMCX_GNW
#define HMCX_GNW 8
#endif
constexpr int WDZ = HMCX_WDZ;   // forward D slice (max)
constexpr int WSR = 4;          // rows per k_wsoft workgroup (one per wave)
constexpr int GNW = HMCX_GNW;   // k_wgrad waves: 8 so that its D/16 workgroups cover every SIMD
constexpr int GTH = GNW * 64;

template <typename T> struct WideArgs {
  const T* X; const T* Y; T* W; T* b;
  T* pW; T* pb;                          // non-null: GPU-file momentum update (gpu/sgld.py:11-20)
  int B, D, K, KP, S, Dz, nSB;           // nSB: k_wsoft blocks
  T* slab; T* diff; T* csp; double* llp;
  T alpha, noise_scale, m_half_eps, clip_hi, clip_lo;
  int want_diff;                         // k_wsoft: 1 = diff + colsum (gradient), 0 = ll only
  int noise_mode; const double* noise; int64_t noff; int P;
  uint64_t seed; uint32_t chain, step;
  unsigned long long* prof;              // HMCX_WIDE_PROF: per-workgroup s_memrealtime stamps (WPH each)
  int wt;                                // slab / diff stored write-through (sc1; HMCX_WIDE_WT=0: plain)
};

// a store that leaves the XCD's L2 (sc1: written through, the line dropped) or a plain one
template <typename T> __device__ inline void wstore(T* p, T v, int wt) {
  if (wt) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}

constexpr int WPH = 8;                   // stamps per workgroup and launch
#define WSTAMP(ph)                                                                                  \
  do {                                                                                              \
    if (a.prof && threadIdx.x == 0)                                                                 \
      a.prof[(size_t)(blockIdx.y * gridDim.x + blockIdx.x) * WPH + (ph)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

// ---------------------------------------------------------------- partial logits
template <typename T, int KB>
__global__ __launch_bounds__(WTH) void k_wfwd(WideArgs<T> a) {
  using M = mfma16<T>;
  constexpr int KP = 16 * KB;
  constexpr int XP = WDZ + (sizeof(T) == 8 ? 2 : 1);       // conflict-free row pitches
  constexpr int WP = KP + (sizeof(T) == 8 ? 2 : 1);
  __shared__ __align__(16) T Xs[WRB * XP];
  constexpr int WSN = WDZ * WP > 4 * WRB * KP ? WDZ * WP : 4 * WRB * KP;   // also the reduction area
  __shared__ __align__(16) T Ws[WSN];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  const int m0 = blockIdx.x * WRB, z = blockIdx.y;
  const int dlo = min(a.D, z * a.Dz), dhi = min(a.D, dlo + a.Dz), nd = dhi - dlo;
  const int nrow = min(WRB, a.B - m0), K = a.K;
  WSTAMP(0);

  // ---- stage X[m0:+32, dlo:dhi] and W[dlo:dhi, 0:K], zero padded to [32][WDZ] / [WDZ][KP].
  // Every load is unconditional (out-of-range slots read a clamped valid address and are zeroed
  // afterwards) and all of a thread's loads are issued before the first LDS store: one memory
  // round trip for the whole tile (a load under a branch makes hipcc wait for each one).
  constexpr int NXE = WRB * WDZ / WTH;                       // X elements per thread
  constexpr int NWE = WDZ * KP / WTH;                        // W elements per thread
  const T* xsrc = a.X + (size_t)m0 * a.D + dlo;
  const T* wsrc = a.W + (size_t)dlo * K;                     // the slice is contiguous: nd·K values
  T xr[NXE], wr[NWE];
#pragma unroll
  for (int u = 0; u < NXE; ++u) {
    const int e = tid + u * WTH, i = e / WDZ, j = e % WDZ;
    const bool ok = i < nrow && j < nd;
    xr[u] = xsrc[ok ? (size_t)i * a.D + j : 0];
    if (!ok) xr[u] = T(0);
  }
#pragma unroll
  for (int u = 0; u < NWE; ++u) {
    const int e = tid + u * WTH, i = e / KP, k = e % KP;
    const bool ok = i < nd && k < K;
    wr[u] = wsrc[ok ? i * K + k : 0];
    if (!ok) wr[u] = T(0);
  }
  WSTAMP(1);
#pragma unroll
  for (int u = 0; u < NXE; ++u) {
    const int e = tid + u * WTH;
    Xs[(e / WDZ) * XP + e % WDZ] = xr[u];
  }
#pragma unroll
  for (int u = 0; u < NWE; ++u) {
    const int e = tid + u * WTH;
    Ws[(e / KP) * WP + e % KP] = wr[u];
  }
  WSTAMP(2);
  __syncthreads();
  WSTAMP(3);

  // ---- MFMA: wave w takes k-steps [w·Q, (w+1)·Q) of the slice for all 2·KB tiles
  const int nks = (nd + 3) / 4, Q = (nks + 3) / 4;
  const int k0 = wave * Q, k1 = min(nks, k0 + Q);
  typename M::acc_t acc[2][KB];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nb = 0; nb < KB; ++nb) acc[mt][nb] = M::zero();
  for (int ks = k0; ks < k1; ++ks) {
    const int kk = ks * 4 + lg;
    const T a0 = Xs[lr * XP + kk], a1 = Xs[(16 + lr) * XP + kk];
    T bv[KB];
#pragma unroll
    for (int nb = 0; nb < KB; ++nb) bv[nb] = Ws[kk * WP + nb * 16 + lr];
#pragma unroll
    for (int nb = 0; nb < KB; ++nb) {
      acc[0][nb] = M::fma(a0, bv[nb], acc[0][nb]);
      acc[1][nb] = M::fma(a1, bv[nb], acc[1][nb]);
    }
  }
  WSTAMP(4);
  __syncthreads();                                           // staging buffers become the reduction area
  T* red = Ws;                                               // [4][32][KP] ⊂ Ws
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nb = 0; nb < KB; ++nb)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        red[(wave * WRB + mt * 16 + M::row(lane, q)) * KP + nb * 16 + lr] = acc[mt][nb][q];
  __syncthreads();
  WSTAMP(5);
  T* out = a.slab + ((size_t)z * a.B + m0) * KP;
  for (int e = tid; e < nrow * KP; e += WTH) {
    const T v = ((red[e] + red[WRB * KP + e]) + red[2 * WRB * KP + e]) + red[3 * WRB * KP + e];
    out[e] = v;
  }
  WSTAMP(6);
}

// ---------------------------------------------------------------- partial logits, register operands
// Same grid and slab as k_wfwd, no LDS staging: wave w owns features [dlo + 32w, dlo + 32w + 32) of
// the slice, and in k-step j lane (lr, lg) holds feature 32w + 8lg + j (A and B use the same
// permutation of the k index, so the product is unchanged up to summation order).  Each lane's
// operands are its rows' 8 consecutive features and those features' weight rows: one batch of
// loads straight into registers, then 2·KB·8 MFMAs back to back.
template <typename T, int KB>
__global__ __launch_bounds__(WTH) void k_wfwd2(WideArgs<T> a) {
  using M = mfma16<T>;
  constexpr int KP = 16 * KB;
  __shared__ __align__(16) T red[4 * WRB * KP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  const int m0 = blockIdx.x * WRB, z = blockIdx.y;
  const int dlo = min(a.D, z * a.Dz), dhi = min(a.D, dlo + a.Dz);
  const int nrow = min(WRB, a.B - m0), K = a.K;
  WSTAMP(0);
  const int f0 = dlo + 32 * wave + 8 * lg;
  const int fsafe = dlo < a.D ? dlo : 0;
  T xa[2][8], wb[8][KB];
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
      wb[j][nb] = a.W[(f0 + j < dhi && c < K) ? (size_t)(f0 + j) * K + c : 0];
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
  T* out = a.slab + ((size_t)z * a.B + m0) * KP;
  for (int e = tid; e < nrow * KP; e += WTH) {
    const T v = ((red[e] + red[WRB * KP + e]) + red[2 * WRB * KP + e]) + red[3 * WRB * KP + e];
    wstore(out + e, v, a.wt);
  }
  WSTAMP(5);
  WSTAMP(6);
}

// Wave-wide all-reductions: every step combines a symmetric pair of lanes, so all lanes hold the
// same bits and the result is deterministic.
// Within each 16-lane row by DPP (g16_*: xor 1, xor 2, half mirror, mirror), then across the four
// rows by two shuffles (xor 16, xor 32): 2 cross-lane permutes per value instead of 6.
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
  __shared__ T cs[WSR][64];
  __shared__ double ll[WSR];
  const int tid = threadIdx.x, k = tid & 63, wave = tid >> 6;
  const int row = blockIdx.x * WSR + wave, K = a.K, KP = a.KP;
  const bool rv = row < a.B, kv = rv && k < K;
  WSTAMP(0);
  T d = T(0);
  double t = 0.0;
  if (rv) {
    // Σ_z slab[z] in slab order; the slab loads go out in batches of 16 (unconditional: lanes
    // k ≥ K read their row's padding columns, which exist in every slab)
    const T* sp = a.slab + (size_t)row * KP + min(k, KP - 1);
    T xw = T(0);
    for (int s0 = 0; s0 < a.S; s0 += 16) {
      T v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = sp[(size_t)min(s0 + q, a.S - 1) * a.B * KP];
#pragma unroll
      for (int q = 0; q < 16; ++q)
        if (s0 + q < a.S) xw = (s0 + q == 0) ? v[q] : xw + v[q];
    }
    if (wave == 0) WSTAMP(1);
    const int kc = min(k, K - 1);
    const T bk = a.b[kc], yk = a.Y[(size_t)row * K + kc];                                 // unconditional loads
    const T zz = kv ? clipz(xw + bk, a.clip_hi, a.clip_lo) : (T)-__builtin_inf();          // softmax.py:39-41
    const T m = wave_max(zz);
    const T e = kv ? exp(zz - m) : T(0);                                                  // softmax.py:34
    const T s = wave_sum(e);
    const T y = kv ? yk : T(0);
    if (a.want_diff) {
      d = kv ? y - e / s : T(0);                                                          // softmax.py:52
      if (k < KP) wstore(a.diff + (size_t)row * KP + k, d, a.wt);
    } else {
      const T lse = log(s) + m;                                                           // softmax.py:18-20
      t = kv ? (double)(y * (zz - lse)) : 0.0;
      t = wave_sum(t);
    }
  }
  cs[wave][k] = d;
  if (k == 0) ll[wave] = t;
  WSTAMP(2);
  __syncthreads();
  if (a.want_diff) {
    if (tid < K) {
      const T v = ((cs[0][tid] + cs[1][tid]) + cs[2][tid]) + cs[3][tid];
      a.csp[(size_t)blockIdx.x * K + tid] = v;
    }
  } else if (tid == 0) {
    a.llp[blockIdx.x] = ((ll[0] + ll[1]) + ll[2]) + ll[3];
  }
  WSTAMP(3);
}

template <typename T>
__device__ inline double wide_noise(const WideArgs<T>& a, uint32_t e) {
  if (a.noise_mode == HMCX_NOISE_BUFFER) return a.noise[a.noff + e];
  return (double)philox_normal_t<T>(a.seed, a.chain, a.step, 0u, e);
}

// ---------------------------------------------------------------- Xᵀ·diff + SGLD update
template <typename T, int KB>
__global__ __launch_bounds__(GTH) void k_wgrad(WideArgs<T> a) {
  using M = mfma16<T>;
  constexpr int KP = 16 * KB;
  constexpr int EPT = (16 * KP + GTH - 1) / GTH;
  __shared__ T red[GNW][16][KP + 1];
  __shared__ T csh[GTH];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  const int d0 = blockIdx.x * 16, K = a.K, B = a.B;
  const bool dok = d0 + lr < a.D;
  WSTAMP(0);

  // epilogue operands and noise first: their latency overlaps the GEMM
  T wreg[EPT], zreg[EPT], preg[EPT];
  const bool gpu_var = a.pW != nullptr;
  const T* psrc = gpu_var ? a.pW : a.W;                      // pointer-selected: no load under a branch
#pragma unroll
  for (int q = 0; q < EPT; ++q) {
    const int e = tid + q * GTH, i = e / KP, k = e - (e / KP) * KP;
    const bool ok = e < 16 * KP && d0 + i < a.D && k < K;
    const uint32_t el = ok ? (uint32_t)((d0 + i) * K + k) : 0u;
    wreg[q] = a.W[el];                                       // unconditional (clamped) load
    preg[q] = psrc[el];
    zreg[q] = (T)wide_noise(a, el);
    if (!ok) wreg[q] = zreg[q] = preg[q] = T(0);
  }
  WSTAMP(1);

  // rows [w·Bw, (w+1)·Bw) of the minibatch on wave w, 16 k-steps of operands in flight; loads are
  // unconditional (clamped row / feature, zeroed after the load) so they all go out together.
  // Even and odd k-steps accumulate separately (2·KB independent MFMA chains), summed at the end.
  constexpr int U = 16;
  const int nks = (B + 3) / 4, Q = (nks + GNW - 1) / GNW;
  const int kb0 = wave * Q, kb1 = min(nks, kb0 + Q);
  const int dcol = dok ? d0 + lr : 0;
  typename M::acc_t acc[2][KB];
#pragma unroll
  for (int nb = 0; nb < KB; ++nb) acc[0][nb] = acc[1][nb] = M::zero();
  for (int ks = kb0; ks < kb1; ks += U) {
    T av[U], bv[U][KB];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = (ks + u) * 4 + lg;
      const bool ok = ks + u < kb1 && row < B;
      const size_t rr = ok ? (size_t)row : 0;
      av[u] = a.X[rr * a.D + dcol];
#pragma unroll
      for (int nb = 0; nb < KB; ++nb) bv[u][nb] = a.diff[rr * KP + nb * 16 + lr];
      if (!(ok && dok)) av[u] = T(0);
      if (!ok)
#pragma unroll
        for (int nb = 0; nb < KB; ++nb) bv[u][nb] = T(0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int nb = 0; nb < KB; ++nb) acc[u & 1][nb] = M::fma(av[u], bv[u][nb], acc[u & 1][nb]);
  }
  WSTAMP(2);
#pragma unroll
  for (int nb = 0; nb < KB; ++nb)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[0][nb][q] = acc[0][nb][q] + acc[1][nb][q];
#pragma unroll
  for (int nb = 0; nb < KB; ++nb)
#pragma unroll
    for (int q = 0; q < 4; ++q) red[wave][M::row(lane, q)][nb * 16 + lr] = acc[0][nb][q];
  __syncthreads();
  WSTAMP(3);

#pragma unroll
  for (int q = 0; q < EPT; ++q) {
    const int e = tid + q * GTH, i = e / KP, k = e - (e / KP) * KP;
    if (e >= 16 * KP || d0 + i >= a.D || k >= K) continue;
    T dot = red[0][i][k];
#pragma unroll
    for (int w = 1; w < GNW; ++w) dot += red[w][i][k];
    const T gr = -(dot - a.alpha * wreg[q]);                                  // softmax.py:57-58
    T p = a.noise_scale * zreg[q];                                            // sgld.py:43-46
    if (gpu_var) p = p * preg[q];                                             // gpu/sgld.py:18
    p = p + a.m_half_eps * gr;                                                // sgld.py:37
    if (gpu_var) a.pW[(size_t)(d0 + i) * K + k] = p;
    a.W[(size_t)(d0 + i) * K + k] = wreg[q] + p;                              // sgld.py:38
  }
  WSTAMP(4);

  if (blockIdx.x == 0) {   // bias: Σ_rows(y − ŷ) from the k_wsoft partials (softmax.py:55,59-60)
    // group g sums row blocks g, g+4, … in order; 16 loads in flight per batch
    const int j = tid % 64, g = min(tid / 64, 3), jc = min(j, K - 1);   // groups 0-3 (threads ≥ 256 idle)
    T s = T(0);
    for (int r0 = g; r0 < a.nSB; r0 += 64) {
      T v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = a.csp[(size_t)min(r0 + 4 * q, a.nSB - 1) * K + jc];
#pragma unroll
      for (int q = 0; q < 16; ++q)
        if (r0 + 4 * q < a.nSB) s = (r0 + 4 * q == g) ? v[q] : s + v[q];
    }
    if (j >= K || tid >= 256) s = T(0);
    csh[tid] = s;
    __syncthreads();
    if (tid < K) {
      const T cs = ((csh[tid] + csh[64 + tid]) + csh[128 + tid]) + csh[192 + tid];
      const T bb = a.b[tid];
      const T gr = -(cs - a.alpha * bb);
      T p = a.noise_scale * (T)wide_noise(a, (uint32_t)(a.D * K + tid));
      if (gpu_var) p = p * a.pb[tid];                                         // gpu/sgld.py:18
      p = p + a.m_half_eps * gr;
      if (gpu_var) a.pb[tid] = p;
      a.b[tid] = bb + p;
    }
  }
  WSTAMP(5);
}

// ---------------------------------------------------------------- Xᵀ·diff per (feature tile, class tile) + SGLD update
// grid = 1 + KB·⌈D/16⌉: block 0 does the bias from the k_wsoft column sums; block 1 + c·ntile + t owns
// feature tile t × class tile c (16 × 16 weights) and computes its Xᵀ·diff over the WHOLE minibatch —
// no cross-workgroup reduction; 8 waves split the rows (summed in wave order) and the tile's weights
// are updated in place (cpu/sgld.py:31-46).  The blocks of one feature tile are ntile apart, so they
// share an XCD (and the X columns in its L2) when ntile % 8 == 0.  Every load a thread needs is
// issued before the Philox noise is drawn, so the noise hides in their latency.
template <typename T>
__device__ inline void wide_bias(const WideArgs<T>& a, T* csh) {
  const int tid = threadIdx.x;
  const int K = a.K;
  const int j = tid % 64, g = min(tid / 64, 3), jc = min(j, K - 1);
  T s = T(0);
  for (int r0 = g; r0 < a.nSB; r0 += 64) {
    T v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = a.csp[(size_t)min(r0 + 4 * q, a.nSB - 1) * K + jc];
#pragma unroll
    for (int q = 0; q < 16; ++q)
      if (r0 + 4 * q < a.nSB) s = (r0 + 4 * q == g) ? v[q] : s + v[q];
  }
  if (j >= K || tid >= 256) s = T(0);
  csh[tid] = s;
  __syncthreads();
  if (tid < K) {
    const T cs = ((csh[tid] + csh[64 + tid]) + csh[128 + tid]) + csh[192 + tid];
    const T bb = a.b[tid];
    const T gr = -(cs - a.alpha * bb);                                       // softmax.py:55,59-60
    T p = a.noise_scale * (T)wide_noise(a, (uint32_t)(a.D * K + tid));
    if (a.pW != nullptr) p = p * a.pb[tid];                                  // gpu/sgld.py:18
    p = p + a.m_half_eps * gr;
    if (a.pW != nullptr) a.pb[tid] = p;
    a.b[tid] = bb + p;
  }
}

template <typename T>
__global__ __launch_bounds__(GTH) void k_wgrad2(WideArgs<T> a) {
  using M = mfma16<T>;
  __shared__ T red[GNW][16][17];
  __shared__ T csh[GTH];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  WSTAMP(0);
  if (blockIdx.x == 0) {
    wide_bias(a, csh);
    WSTAMP(1); WSTAMP(2); WSTAMP(3); WSTAMP(4); WSTAMP(5);
    return;
  }
  const int ntile = (a.D + 15) / 16;
  const int c = (blockIdx.x - 1) / ntile, t = (blockIdx.x - 1) - c * ntile;
  const int d0 = t * 16, K = a.K, B = a.B, KP = a.KP;
  const bool dok = d0 + lr < a.D;
  const int dcol = dok ? d0 + lr : 0;
  const int nks = (B + 3) / 4, Q = (nks + GNW - 1) / GNW;
  const int kb0 = wave * Q, kb1 = min(nks, kb0 + Q);
  // my epilogue element: feature d0 + tid / 16, class 16c + tid % 16 (threads 0-255)
  const int ei = tid >> 4, ek = c * 16 + (tid & 15);
  const bool eok = tid < 256 && d0 + ei < a.D && ek < K;
  const uint32_t el = eok ? (uint32_t)((d0 + ei) * K + ek) : 0u;
  const bool gpu_var = a.pW != nullptr;
  const T* psrc = gpu_var ? a.pW : a.W;
  constexpr int U = 16;
  typename M::acc_t acc0 = M::zero(), acc1 = M::zero();
  T wv = T(0), pv = T(0), zv = T(0);
  bool first = true;
  for (int ks = kb0; ks < kb1 || first; ks += U) {
    T av[U], bv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = (ks + u) * 4 + lg;
      const bool ok = ks + u < kb1 && row < B;
      const size_t rr = ok ? (size_t)row : 0;
      av[u] = a.X[rr * a.D + dcol];
      bv[u] = a.diff[rr * KP + c * 16 + lr];
      if (!(ok && dok)) av[u] = T(0);
      if (!ok) bv[u] = T(0);
    }
    if (first) {                       // epilogue operands and noise while the first batch is in flight
      first = false;
      wv = a.W[el];
      pv = psrc[el];
      zv = (T)wide_noise(a, el);
      WSTAMP(1);
    }
#pragma unroll
    for (int u = 0; u < U; u += 2) {
      acc0 = M::fma(av[u], bv[u], acc0);
      acc1 = M::fma(av[u + 1], bv[u + 1], acc1);
    }
  }
  WSTAMP(2);
#pragma unroll
  for (int q = 0; q < 4; ++q) red[wave][M::row(lane, q)][lr] = acc0[q] + acc1[q];
  __syncthreads();
  WSTAMP(3);
  if (eok) {
    T dot = red[0][ei][tid & 15];
#pragma unroll
    for (int w = 1; w < GNW; ++w) dot += red[w][ei][tid & 15];
    const T gr = -(dot - a.alpha * wv);                                        // softmax.py:57-58
    T p = a.noise_scale * zv;                                                  // sgld.py:43-46
    if (gpu_var) p = p * pv;                                                   // gpu/sgld.py:18
    p = p + a.m_half_eps * gr;                                                 // sgld.py:37
    if (gpu_var) a.pW[el] = p;
    a.W[el] = wv + p;                                                          // sgld.py:38
  }
  WSTAMP(4);
  WSTAMP(5);
}

__global__ void k_wreduce_ll(const double* llp, int n, double* out) {
  __shared__ double sh[256];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) s += llp[i];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int m = 128; m > 0; m >>= 1) {
    if ((int)threadIdx.x < m) sh[threadIdx.x] += sh[threadIdx.x + m];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = sh[0];
}

// ---------------------------------------------------------------- host
bool sgld_wide_eligible(const hmcx_sampler_args* s) {
  const char* env = getenv("HMCX_SGLD_WIDE");
  if (env && env[0] == '0') return false;        // 0: kernel-per-phase; 1: this path; 2: persistent
  if (s->C != 1 || s->K > 64 || s->K < 1 || s->B < 1 || s->D < 1) return false;
  // faster than the kernel-per-phase path for every single-chain shape measured (MNIST D=784,
  // K=10: 18.0 vs 20.5 µs per f64 step; config 5 D=2048, K=38: 26.4 vs 35.1 µs)
  return true;
}

// kernel generation: 2 (default) = k_wfwd2 / k_wgrad2, 1 = k_wfwd / k_wgrad (HMCX_WIDE_V=1)
static int wide_version() {
  static const int v = getenv("HMCX_WIDE_V") ? atoi(getenv("HMCX_WIDE_V")) : 2;
  return v == 1 ? 1 : 2;
}

template <typename T, int KB>
static void launch_wide(const WideArgs<T>& a, hipStream_t st, int which) {
  const dim3 gf((a.B + WRB - 1) / WRB, a.S);
  if (wide_version() == 1) {
    if (which == 0) hipLaunchKernelGGL((k_wfwd<T, KB>), gf, dim3(WTH), 0, st, a);
    else hipLaunchKernelGGL((k_wgrad<T, KB>), dim3((a.D + 15) / 16), dim3(GTH), 0, st, a);
  } else {
    if (which == 0) hipLaunchKernelGGL((k_wfwd2<T, KB>), gf, dim3(WTH), 0, st, a);
    else hipLaunchKernelGGL((k_wgrad2<T>), dim3(1 + KB * ((a.D + 15) / 16)), dim3(GTH), 0, st, a);
  }
}
template <typename T>
static void launch_wide_kb(const WideArgs<T>& a, hipStream_t st, int which) {
  switch (a.KP / 16) {
    case 1: launch_wide<T, 1>(a, st, which); break;
    case 2: launch_wide<T, 2>(a, st, which); break;
    case 3: launch_wide<T, 3>(a, st, which); break;
    default: launch_wide<T, 4>(a, st, which); break;
  }
}

template <typename T>
int sgld_wide_t(hmcx_ctx* ctx, const hmcx_sampler_args* s) {
  const int B = s->B, D = s->D, K = s->K, KP = (K + 15) / 16 * 16;
  const int S = (D + WDZ - 1) / WDZ, Dz = ((D + S - 1) / S + 3) / 4 * 4;
  const int nSB = (B + WSR - 1) / WSR;
  // HMCX_WIDE_PROF=<file>: stamps of the first PROF_CAP steps' three launches, appended to <file>
  // after the call (header: steps, workgroups of k_wfwd, k_wsoft, k_wgrad, WPH; tools/wide_prof_summary.py)
  static const char* prof_path = getenv("HMCX_WIDE_PROF");
  const int ntile = (D + 15) / 16;
  const int GF = ((B + WRB - 1) / WRB) * S, GS = nSB, GG = wide_version() == 1 ? ntile : 1 + (KP / 16) * ntile,
            GALL = GF + GS + GG;
  const int nprof = prof_path ? std::min(s->n_steps, 64) : 0;
  Workspace ws(ctx);
  T *slab, *diff, *csp;
  double* llp;
  unsigned long long* prof = nullptr;
  do {
    ws.reset();
    slab = ws.take<T>((size_t)S * B * KP);
    diff = ws.take<T>((size_t)B * KP);
    csp = ws.take<T>((size_t)nSB * K);
    llp = ws.take<double>((size_t)nSB);
    if (nprof) prof = ws.take<unsigned long long>((size_t)nprof * GALL * WPH);
  } while (ws.retry());
  if (ws.failed) return HMCX_ENOMEM;
  int rc;
  begin_call(ctx);
  WideArgs<T> a{};
  a.W = (T*)s->W; a.b = (T*)s->b; a.pW = (T*)s->pW; a.pb = (T*)s->pb;
  a.B = B; a.D = D; a.K = K; a.KP = KP; a.S = S; a.Dz = Dz; a.nSB = nSB;
  a.slab = slab; a.diff = diff; a.csp = csp; a.llp = llp;
  a.alpha = (T)s->alpha;
  a.clip_hi = (T)CLIP_HI; a.clip_lo = (T)CLIP_LO;
  a.noise_mode = s->noise_mode; a.noise = s->noise; a.P = D * K + K;
  a.seed = s->seed; a.chain = s->chain0;
  static const int wt_env = getenv("HMCX_WIDE_WT") ? atoi(getenv("HMCX_WIDE_WT")) : 1;
  a.wt = wt_env;
  if ((rc = timing_begin(ctx, ctx->stream))) return rc;
  GraphScope gs(ctx);
  hipStream_t st = ctx->stream;
  for (int i = 0; i < s->n_steps; ++i) {
    a.X = (const T*)s->X + (size_t)s->row0[i] * D;
    a.Y = (const T*)s->Y + (size_t)s->row0[i] * K;
    const double eps = s->eps[i];
    a.noise_scale = (T)(2.0 * eps);                                   // sgld.py:43
    a.m_half_eps = (T)(-0.5 * eps);                                   // sgld.py:37
    a.step = s->step_base + (uint32_t)i;
    a.noff = s->noise_mode == HMCX_NOISE_BUFFER ? s->noise_off[i] : 0;
    a.want_diff = 1;
    unsigned long long* pr = i < nprof ? prof + (size_t)i * GALL * WPH : nullptr;
    a.prof = pr;
    launch_wide_kb<T>(a, st, 0);
    a.prof = pr ? pr + (size_t)GF * WPH : nullptr;
    hipLaunchKernelGGL(k_wsoft<T>, dim3(nSB), dim3(WTH), 0, st, a);
    a.prof = pr ? pr + (size_t)(GF + GS) * WPH : nullptr;
    launch_wide_kb<T>(a, st, 1);
    a.prof = nullptr;
    HMCX_HIP(ctx, hipGetLastError());
    if (s->want_ll && s->want_ll[i] && s->out_ll) {                   // sgmcmc.py:61 logging
      a.want_diff = 0;
      launch_wide_kb<T>(a, st, 0);
      hipLaunchKernelGGL(k_wsoft<T>, dim3(nSB), dim3(WTH), 0, st, a);
      hipLaunchKernelGGL(k_wreduce_ll, dim3(1), dim3(256), 0, st, (const double*)llp, nSB, s->out_ll + i);
      HMCX_HIP(ctx, hipGetLastError());
    }
  }
  if ((rc = gs.finish())) return rc;
  if ((rc = timing_end(ctx, ctx->stream))) return rc;
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
