// hmcx_softmax.hip — softmax-regression gradient + SGHMC / SGLD leapfrog kernels (gfx950).
//
// Reference hot path:
//   softmax.grad          /root/reference/hamiltonian/models/cpu/softmax.py:38-61   (A6)
//   softmax.log_likelihood                                         softmax.py:63-72 (A7)
//   sghmc.step            /root/reference/hamiltonian/inference/cpu/sghmc.py:19-39  (A1)
//   sgld.step             /root/reference/hamiltonian/inference/cpu/sgld.py:31-46   (A2)
//
// One SGHMC leapfrog iteration (sghmc.py:28-34, vars in order weights, bias) is two kernels:
//   k_fwd  (16-row x chain tile):  Z = X·W on v_mfma_*_16x16x4 (d split over the block's
//          waves, 4 k-chunks of loads in flight per wave), then, element-parallel from LDS:
//          z = clip(Z+b), softmax, diff = y − ŷ (weights sub-step), and the bias sub-step
//          b' = b + ε·pb, z' = clip(Z+b'): Σ_rows(y − ŷ') and log-likelihood partials at (W,b')
//          — the bias sub-step reuses X·W (W is unchanged by it).
//   k_grad (16-feature x chain tile):  Xᵀ·diff on MFMA (minibatch split over waves), fused
//          epilogue g = −(Xᵀdiff − αW);  p = (1−ε)p + εg + 2ε·ξ;  W += ε·p (next drift);
//          the tile-column-0 blocks finish the bias sub-step from the row partials.
// Per step: k_sghmc_init (commit previous accept, momentum, first drift, kinetic partials),
// k_fwd(LL) at q0, n_iter × (k_fwd, k_grad), k_sghmc_accept (energies, MH decision).
// Rules followed for latency: no serial loop over global loads anywhere (all reductions are
// parallel loads + fixed-order LDS trees, so results are deterministic run to run).
// Elementwise arithmetic follows the reference's NumPy op order with FP contraction off
// (-ffp-contract=off), so float64 runs differ from NumPy only through summation order.
#include "hmcx_common.h"
#include "hmcx_internal.h"
#include "hmcx_persist.h"
#include "hmcx_batch.h"
#include <algorithm>
#include <numeric>
#include <vector>

namespace hmcx {

// ------------------------------------------------------------------ forward (logits) kernel
template <typename T, int NBLK, bool VEC, int NW>
__global__ __launch_bounds__(NW * 64) void k_fwd(FwdArgs<T> a) {
  using M = mfma16<T>;
  constexpr int NT = NBLK * 16, NTH = NW * 64, LD = NT + 1;
  constexpr int YPT = (16 * NT + NTH - 1) / NTH;   // Y values prefetched per thread
  __shared__ T red[NW][16][NT];
  __shared__ T zA[16][LD], eA[16][LD], zB[16][LD], eB[16][LD], yt[16][LD];
  __shared__ T bt[NT], bpt[NT];
  __shared__ T mA[16][NT], sA[16][NT], mB[16][NT], sB[16][NT];
  __shared__ double lrow[16][NT];
  __shared__ int act[NT];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int m0 = blockIdx.x * 16;
  const int c0 = blockIdx.y * a.CB;
  const int ncb = min(a.CB, a.C - c0);
  const int n0 = c0 * a.K;
  const int ncols = ncb * a.K;
  const int K = a.K;
  const int mode = a.mode;
  const bool sghmc = mode == FWD_SGHMC;
  const bool sig = a.link == LINK_SIGMOID;                 // logistic.py:43-55 (K = 1)
  const int nrow = min(16, a.B - m0);

  // ---- prefetch epilogue operands into registers (their latency overlaps the GEMM)
  T breg = T(0), bpreg = T(0);
  int actreg = 1;
  if (tid < ncols) {
    breg = a.b[n0 + tid];
    if (sghmc) bpreg = breg + a.eps * a.pb[n0 + tid];                  // b' = b + ε·pb (sghmc.py:32)
  }
  if (sghmc && tid < ncb) actreg = a.iter < a.n_iter[c0 + tid];
  T yreg[YPT];
#pragma unroll
  for (int q = 0; q < YPT; ++q) {
    const int e = tid + q * NTH;
    const int i = e / NT, j = e - (e / NT) * NT;
    yreg[q] = (mode != FWD_PRED && e < 16 * NT && i < nrow && j < ncols) ? a.Y[(size_t)(m0 + i) * K + j % K] : T(0);
  }

  // ---- Z = X·W : wave w owns d in [w·Dw, (w+1)·Dw), 4 chunks of 16 loaded before their MFMAs
  typename M::acc_t acc0[NBLK], acc1[NBLK];
#pragma unroll
  for (int nb = 0; nb < NBLK; ++nb) { acc0[nb] = M::zero(); acc1[nb] = M::zero(); }
  int dlo = 0, dhi = a.D;
  if (a.slab_mode == 1) {                                  // D slice blockIdx.z of gridDim.z
    const int Dz = ((a.D + (int)gridDim.z * 16 - 1) / ((int)gridDim.z * 16)) * 16;
    dlo = min(a.D, (int)blockIdx.z * Dz);
    dhi = min(a.D, dlo + Dz);
  }
  const int Dw = ((dhi - dlo + NW * 16 - 1) / (NW * 16)) * 16;
  const int kbeg = dlo + wave * Dw, kend = a.slab_mode == 2 ? kbeg : min(dhi, kbeg + Dw);
  const bool rok = r < nrow;
  const T* xrow = a.X + (size_t)(m0 + (rok ? r : 0)) * a.D;
  for (int kc = kbeg; kc < kend; kc += 64) {
    T av[4][4], bv[4][NBLK][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int kb = kc + 16 * u + 4 * g;
      if (VEC && kb + 3 < kend && rok) {
        if constexpr (sizeof(T) == 8) {
          const double2* p2 = reinterpret_cast<const double2*>(xrow + kb);
          const double2 x0 = p2[0], x1 = p2[1];
          av[u][0] = x0.x; av[u][1] = x0.y; av[u][2] = x1.x; av[u][3] = x1.y;
        } else {
          const float4 x0 = *reinterpret_cast<const float4*>(xrow + kb);
          av[u][0] = x0.x; av[u][1] = x0.y; av[u][2] = x0.z; av[u][3] = x0.w;
        }
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) av[u][s] = (rok && kb + s < kend) ? xrow[kb + s] : T(0);
      }
#pragma unroll
      for (int nb = 0; nb < NBLK; ++nb) {
        const int col = nb * 16 + r;
        const bool cok = col < ncols;
#pragma unroll
        for (int s = 0; s < 4; ++s)
          bv[u][nb][s] = (cok && kb + s < kend) ? a.W[(size_t)(kb + s) * a.N + n0 + col] : T(0);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int nb = 0; nb < NBLK; ++nb) {
        acc0[nb] = M::fma(av[u][0], bv[u][nb][0], acc0[nb]);
        acc1[nb] = M::fma(av[u][1], bv[u][nb][1], acc1[nb]);
        acc0[nb] = M::fma(av[u][2], bv[u][nb][2], acc0[nb]);
        acc1[nb] = M::fma(av[u][3], bv[u][nb][3], acc1[nb]);
      }
  }
#pragma unroll
  for (int nb = 0; nb < NBLK; ++nb)
#pragma unroll
    for (int q = 0; q < 4; ++q) red[wave][M::row(lane, q)][nb * 16 + r] = acc0[nb][q] + acc1[nb][q];
  if (tid < NT) { bt[tid] = breg; bpt[tid] = bpreg; }
  if (tid < NT) act[tid] = actreg;
#pragma unroll
  for (int q = 0; q < YPT; ++q) {
    const int e = tid + q * NTH;
    if (e < 16 * NT) yt[e / NT][e - (e / NT) * NT] = yreg[q];
  }
  __syncthreads();
  if (a.slab_mode == 1) {                                  // split-K partial: XW of this D slice
    for (int e = tid; e < 16 * NT; e += NTH) {
      const int i = e / NT, j = e - (e / NT) * NT;
      if (i >= nrow || j >= ncols) continue;
      T xw = red[0][i][j];
#pragma unroll
      for (int w = 1; w < NW; ++w) xw += red[w][i][j];
      a.slab[((size_t)blockIdx.z * a.B + m0 + i) * a.N + n0 + j] = xw;
    }
    return;
  }
  if (a.slab_mode == 2) {                                  // XW = Σ_z slab[z]; the waves' partials are 0
    for (int e = tid; e < 16 * NT; e += NTH) {
      const int i = e / NT, j = e - (e / NT) * NT;
      T xw = T(0);
      if (i < nrow && j < ncols) {
        const T* sp = a.slab + (size_t)(m0 + i) * a.N + n0 + j;
        xw = sp[0];
        for (int z = 1; z < a.nslab; ++z) xw += sp[(size_t)z * a.B * a.N];
      }
      red[0][i][j] = xw;
    }
    __syncthreads();
  }

  // ---- pass 1 (element): XW (fixed wave order), z = clip(XW + b), z' = clip(XW + b')
  const T hi = a.clip_hi, lo = a.clip_lo;
  for (int e = tid; e < 16 * NT; e += NTH) {
    const int i = e / NT, j = e - (e / NT) * NT;
    T xw = red[0][i][j];
#pragma unroll
    for (int w = 1; w < NW; ++w) xw += red[w][i][j];
    zA[i][j] = clipz(xw + bt[j], hi, lo);                                  // softmax.py:39-41
    if (sghmc) zB[i][j] = clipz(xw + bpt[j], hi, lo);
  }
  __syncthreads();
  // ---- pass 2 (row, chain): row max (np.max semantics: NaN propagates); softmax link only
  for (int p = tid; p < (sig ? 0 : 16 * ncb); p += NTH) {
    const int i = p & 15, cb = (p >> 4) * K;
    T m = zA[i][cb];
    for (int k = 1; k < K; ++k) m = max_nan(m, zA[i][cb + k]);
    mA[i][p >> 4] = m;
    if (sghmc) {
      T mb = zB[i][cb];
      for (int k = 1; k < K; ++k) mb = max_nan(mb, zB[i][cb + k]);
      mB[i][p >> 4] = mb;
    }
  }
  __syncthreads();
  // ---- pass 3 (element): exponentials
  for (int e = tid; e < 16 * NT; e += NTH) {
    const int i = e / NT, j = e - (e / NT) * NT;
    if (j >= ncols) continue;
    const int cc = j / K;
    if (sig) {
      eA[i][j] = T(1) / (T(1) + exp(-zA[i][j]));                          // logistic.py:54-55
      continue;
    }
    eA[i][j] = exp(zA[i][j] - mA[i][cc]);                                 // softmax.py:34
    if (sghmc) eB[i][j] = exp(zB[i][j] - mB[i][cc]);
  }
  __syncthreads();
  // ---- pass 4 (row, chain): normalisers (softmax link)
  for (int p = tid; p < (sig ? 0 : 16 * ncb); p += NTH) {
    const int i = p & 15, cc = p >> 4, cb = cc * K;
    T s = T(0);
    for (int k = 0; k < K; ++k) s += eA[i][cb + k];
    sA[i][cc] = s;
    if (sghmc) {
      T sb = T(0);
      for (int k = 0; k < K; ++k) sb += eB[i][cb + k];
      sB[i][cc] = sb;
    }
  }
  __syncthreads();
  // ---- pass 5 (element): ŷ, diff, colsum terms, log-likelihood terms (written in place)
  for (int e = tid; e < 16 * NT; e += NTH) {
    const int i = e / NT, j = e - (e / NT) * NT;
    if (j >= ncols || i >= nrow) continue;
    const int cc = j / K;
    const size_t gidx = (size_t)(m0 + i) * a.N + n0 + j;
    const T yh = sig ? eA[i][j] : eA[i][j] / sA[i][cc];                   // softmax.py:35-36
    if (mode == FWD_PRED) { a.prob[gidx] = yh; continue; }
    const T y = yt[i][j];
    if (mode == FWD_GRAD || sghmc) {
      const T d = y - yh;                                                 // softmax.py:52
      if (act[cc]) a.diff[gidx] = d;
      if (mode == FWD_GRAD) eA[i][j] = d;
    }
    if (sghmc) {
      const T lse = log(sB[i][cc]) + mB[i][cc];                           // logsumexp (softmax.py:18)
      const T yb = eB[i][j] / sB[i][cc];
      zA[i][j] = y - yb;                                                  // bias sub-step colsum term
      eB[i][j] = y * (zB[i][j] - lse);                                    // softmax.py:19-20
    } else if (mode == FWD_LL) {
      if (sig) {
        eA[i][j] = y * log(yh) + (T(1) - y) * log(T(1) - yh);             // logistic.py:71
      } else {
        const T lse = log(sA[i][cc]) + mA[i][cc];
        eA[i][j] = y * (zA[i][j] - lse);
      }
    }
  }
  __syncthreads();
  // ---- pass 6: column sums of diff (→ gb partial) and row log-likelihoods
  if (mode == FWD_GRAD || sghmc) {
    const T(*src)[LD] = sghmc ? zA : eA;
    for (int j = tid; j < ncols; j += NTH) {
      if (!act[j / K]) continue;
      T s = T(0);
      for (int i = 0; i < nrow; ++i) s += src[i][j];
      a.colsum_part[(size_t)blockIdx.x * a.N + n0 + j] = s;
    }
  }
  if (sghmc || mode == FWD_LL) {
    const T(*src)[LD] = sghmc ? eB : eA;
    for (int p = tid; p < nrow * ncb; p += NTH) {
      const int i = p % nrow, cc = p / nrow, cb = cc * K;
      double s = 0.0;
      for (int k = 0; k < K; ++k) s += (double)src[i][cb + k];
      lrow[i][cc] = s;
    }
    __syncthreads();
    for (int cc = tid; cc < ncb; cc += NTH) {
      if (!act[cc]) continue;
      double s = 0.0;
      for (int i = 0; i < nrow; ++i) s += lrow[i][cc];
      a.ll_part[(size_t)blockIdx.x * a.C + c0 + cc] = s;
    }
  }
}

// ------------------------------------------------------------------ noise
template <typename T>
__device__ inline double noise_at(const GradArgs<T>& a, int c, uint32_t e) {
  if (a.noise_mode == HMCX_NOISE_BUFFER) return a.noise[a.noff[c] + (int64_t)a.slot * a.P + e];
  return (double)philox_normal_t<T>(a.seed, a.chain0 + c, a.step, a.slot, e);
}

// ------------------------------------------------------------------ gradient (Xᵀ·diff) kernel
template <typename T, int NBLK, int NW>
__global__ __launch_bounds__(NW * 64) void k_grad(GradArgs<T> a) {
  using M = mfma16<T>;
  constexpr int NT = NBLK * 16, NTH = NW * 64;
  constexpr int EPT = (16 * NT + NTH - 1) / NTH;    // epilogue elements per thread
  __shared__ T red[NW][16][NT];
  __shared__ T csr[NTH];
  __shared__ double ksh[NTH];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int d0 = blockIdx.x * 16;
  const int c0 = blockIdx.y * a.CB;
  const int ncb = min(a.CB, a.C - c0);
  const int n0 = c0 * a.K;
  const int ncols = ncb * a.K;
  const int K = a.K;
  const int mode = a.mode;

  // ---- prefetch the epilogue's per-element operands and noise (overlaps the GEMM)
  T wreg[EPT], preg[EPT], zreg[EPT];
  int ok[EPT];
#pragma unroll
  for (int q = 0; q < EPT; ++q) {
    const int e = tid + q * NTH;
    const int i = e / NT, j = e - (e / NT) * NT;
    const int d = d0 + i;
    ok[q] = e < 16 * NT && d < a.D && j < ncols;
    if (ok[q] && mode == GRAD_SGHMC) ok[q] = a.iter < a.n_iter[c0 + j / K];
    wreg[q] = preg[q] = zreg[q] = T(0);
    if (ok[q]) {
      const size_t idx = (size_t)d * a.N + n0 + j;
      const int cc = j / K, k = j - cc * K;
      if (mode == GRAD_OUT) {
        wreg[q] = a.Wsrc[idx];
      } else {
        wreg[q] = a.W[idx];
        if (mode == GRAD_SGHMC || mode == GRAD_SGD || mode == GRAD_SGLD_GPU || mode == GRAD_HMC) preg[q] = a.pW[idx];
        if (mode != GRAD_SGD && mode != GRAD_HMC) zreg[q] = (T)noise_at(a, c0 + cc, (uint32_t)(d * K + k));
      }
    }
  }

  // ---- Xᵀ·diff : wave w owns minibatch rows [w·Bw, (w+1)·Bw)
  typename M::acc_t acc0[NBLK], acc1[NBLK];
#pragma unroll
  for (int nb = 0; nb < NBLK; ++nb) { acc0[nb] = M::zero(); acc1[nb] = M::zero(); }
  const int Bw = ((a.B + NW * 16 - 1) / (NW * 16)) * 16;
  const int kbeg = wave * Bw, kend = min(a.B, kbeg + Bw);
  const bool dok = d0 + r < a.D;
  for (int kc = kbeg; kc < kend; kc += 64) {
    T av[4][4], bv[4][NBLK][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int kb = kc + 16 * u + 4 * g;
#pragma unroll
      for (int s = 0; s < 4; ++s) av[u][s] = (dok && kb + s < kend) ? a.X[(size_t)(kb + s) * a.D + d0 + r] : T(0);
#pragma unroll
      for (int nb = 0; nb < NBLK; ++nb) {
        const int col = nb * 16 + r;
        const bool cok = col < ncols;
#pragma unroll
        for (int s = 0; s < 4; ++s)
          bv[u][nb][s] = (cok && kb + s < kend) ? a.diff[(size_t)(kb + s) * a.N + n0 + col] : T(0);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int nb = 0; nb < NBLK; ++nb) {
        acc0[nb] = M::fma(av[u][0], bv[u][nb][0], acc0[nb]);
        acc1[nb] = M::fma(av[u][1], bv[u][nb][1], acc1[nb]);
        acc0[nb] = M::fma(av[u][2], bv[u][nb][2], acc0[nb]);
        acc1[nb] = M::fma(av[u][3], bv[u][nb][3], acc1[nb]);
      }
  }
#pragma unroll
  for (int nb = 0; nb < NBLK; ++nb)
#pragma unroll
    for (int q = 0; q < 4; ++q) red[wave][M::row(lane, q)][nb * 16 + r] = acc0[nb][q] + acc1[nb][q];
  __syncthreads();

  // ---- epilogue (element): gradient, momentum, drift (sghmc.py:31-34 / sgld.py:34-38)
  T pnew[EPT];
#pragma unroll
  for (int q = 0; q < EPT; ++q) {
    pnew[q] = T(0);
    if (!ok[q]) continue;
    const int e = tid + q * NTH;
    const int i = e / NT, j = e - (e / NT) * NT;
    const size_t idx = (size_t)(d0 + i) * a.N + n0 + j;
    T dot = red[0][i][j];
#pragma unroll
    for (int w = 1; w < NW; ++w) dot += red[w][i][j];
    const T gr = -(dot - a.alpha * wreg[q]);                              // softmax.py:57-58
    if (mode == GRAD_OUT) {
      a.gW[idx] = gr;
    } else if (mode == GRAD_SGHMC) {
      const T p = (a.one_minus_eps * preg[q] + a.eps * gr) + a.noise_scale * zreg[q];
      a.pW[idx] = p;
      pnew[q] = p;
      if (a.iter < a.n_iter[c0 + j / K] - 1) a.W[idx] = wreg[q] + a.eps * p;   // next drift
    } else if (mode == GRAD_SGD) {
      const T m = a.gamma * preg[q] - a.lr * gr;                          // sgd.py:40
      a.pW[idx] = m;
      a.W[idx] = wreg[q] + m;                                             // sgd.py:41
    } else if (mode == GRAD_HMC) {
      T p = preg[q];
      if (a.hmc_flags & HMC_KICK_W) p = p - a.eps * gr;                   // hmc.py:53
      if (a.hmc_flags & HMC_HALF_W) {
        p = p - a.half_eps * gr;                                          // hmc.py:50
        a.W[idx] = wreg[q] + a.eps * p;                                   // hmc.py:51
      }
      a.pW[idx] = p;
    } else if (mode == GRAD_SGLD_GPU) {
      T p = (a.noise_scale * zreg[q]) * preg[q];                          // gpu/sgld.py:18 ν⊙p
      p = p + a.m_half_eps * gr;
      a.pW[idx] = p;
      a.W[idx] = wreg[q] + p;                                             // gpu/sgld.py:19
      if (a.trace) a.trace[(size_t)(c0 + j / K) * a.P + (size_t)(d0 + i) * K + j % K] = wreg[q] + p;
    } else {
      T p = a.noise_scale * zreg[q];
      p = p + a.m_half_eps * gr;
      a.W[idx] = wreg[q] + p;
      if (a.trace) a.trace[(size_t)(c0 + j / K) * a.P + (size_t)(d0 + i) * K + j % K] = wreg[q] + p;   // sghmc_multicore.py:49-51
    }
  }
  if (mode == GRAD_SGHMC) {
    // Σ pW² of this block, per chain whose trajectory ends at this iteration (E_new, hmc.py:74-79)
    for (int cc = 0; cc < ncb; ++cc) {
      if (a.iter != a.n_iter[c0 + cc] - 1) continue;
      double v = 0.0;
#pragma unroll
      for (int q = 0; q < EPT; ++q) {
        const int e = tid + q * NTH;
        const int j = e - (e / NT) * NT;
        if (ok[q] && j / K == cc) v += (double)pnew[q] * (double)pnew[q];
      }
      ksh[tid] = v;
      __syncthreads();
      for (int s = NTH / 2; s > 0; s >>= 1) {
        if (tid < s) ksh[tid] += ksh[tid + s];
        __syncthreads();
      }
      if (tid == 0) a.kin_part[(size_t)blockIdx.x * a.C + c0 + cc] = ksh[0];
      __syncthreads();
    }
  }

  if (blockIdx.x == 0) {  // bias: Σ_rows(y−ŷ) from the k_fwd row partials (softmax.py:55,59-60)
    constexpr int G = NTH / NT;
    const int j = tid % NT, grp = tid / NT;
    T s = T(0);
    if (j < ncols && grp < G) {
      const T* src = a.colsum_part + n0 + j;
      int rb = grp;
      for (; rb + 3 * G < a.nRB; rb += 4 * G) {
        const T v0 = src[(size_t)rb * a.N], v1 = src[(size_t)(rb + G) * a.N];
        const T v2 = src[(size_t)(rb + 2 * G) * a.N], v3 = src[(size_t)(rb + 3 * G) * a.N];
        s += ((v0 + v1) + v2) + v3;
      }
      for (; rb < a.nRB; rb += G) s += src[(size_t)rb * a.N];
    }
    csr[tid] = s;
    __syncthreads();
    T pb_new = T(0);
    if (tid < ncols) {
      const int cc = tid / K, k = tid - cc * K, c = c0 + cc, col = n0 + tid;
      const bool active = mode != GRAD_SGHMC || a.iter < a.n_iter[c];
      if (active) {
        T cs = csr[tid];
        for (int q = 1; q < G; ++q) cs += csr[q * NT + tid];
        const int DK = a.D * K;
        if (mode == GRAD_OUT) {
          a.gb[col] = -(cs - a.alpha * a.bsrc[col]);
        } else if (mode == GRAD_SGHMC) {
          const T bb = a.b[col];
          T p = a.pb[col];
          const T bp = bb + a.eps * p;
          const T gr = -(cs - a.alpha * bp);
          const T z = (T)noise_at(a, c, (uint32_t)(DK + k));
          p = (a.one_minus_eps * p + a.eps * gr) + a.noise_scale * z;
          a.pb[col] = p;
          a.b[col] = bp;
          pb_new = p;
        } else if (mode == GRAD_SGD) {
          const T bb = a.b[col];
          const T gr = -(cs - a.alpha * bb);
          const T m = a.gamma * a.pb[col] - a.lr * gr;                      // sgd.py:40-41
          a.pb[col] = m;
          a.b[col] = bb + m;
        } else if (mode == GRAD_HMC) {
          const T bb = a.b[col];
          const T gr = -(cs - a.alpha * bb);
          T p = a.pb[col];
          if (a.hmc_flags & HMC_KICK_B) p = p - a.eps * gr;                 // hmc.py:53
          if (a.hmc_flags & HMC_HALF_B) {
            p = p - a.half_eps * gr;                                        // hmc.py:50
            a.b[col] = bb + a.eps * p;                                      // hmc.py:51
          }
          a.pb[col] = p;
        } else {
          const T bb = a.b[col];
          const T gr = -(cs - a.alpha * bb);
          const T z = (T)noise_at(a, c, (uint32_t)(DK + k));
          T p = a.noise_scale * z;
          if (mode == GRAD_SGLD_GPU) p = p * a.pb[col];                     // gpu/sgld.py:18
          p = p + a.m_half_eps * gr;
          if (mode == GRAD_SGLD_GPU) a.pb[col] = p;
          a.b[col] = bb + p;
          if (a.trace) a.trace[(size_t)c * a.P + DK + k] = bb + p;
        }
      }
    }
    if (mode == GRAD_SGHMC) {
      __syncthreads();
      csr[tid] = pb_new;      // reuse as staging for Σ pb² of finished chains
      __syncthreads();
      if (tid < ncb && a.iter == a.n_iter[c0 + tid] - 1) {
        double v = 0.0;
        for (int k = 0; k < K; ++k) {
          const double p = (double)csr[tid * K + k];
          v += p * p;
        }
        a.kinb[c0 + tid] = v;
      }
    }
  }
}

// ------------------------------------------------------------------ SGHMC step init / commit / accept
// grid (nDB, C): block x handles features [16x, 16x+16) of chain y; block 0 also the bias.
template <typename T>
__global__ __launch_bounds__(256) void k_sghmc_init(InitArgs<T> a) {
  __shared__ double ksh[256];
  const int c = blockIdx.y, tid = threadIdx.x;
  const int K = a.K;
  const int d0 = blockIdx.x * 16;
  const bool take = a.prev_acc && a.prev_acc[c];
  const bool drift = a.n_iter[c] >= 1;
  double kin = 0.0;
  for (int e = tid; e < 16 * K; e += 256) {
    const int i = e / K, k = e - (e / K) * K, d = d0 + i;
    if (d >= a.D) continue;
    const size_t w = (size_t)d * a.N + c * K + k;
    double z;
    if (a.noise_mode == HMCX_NOISE_BUFFER) z = a.noise[a.noff[c] + d * K + k];
    else z = (double)philox_normal_t<T>(a.seed, a.chain0 + c, a.step, 0u, (uint32_t)(d * K + k));
    const T p = (T)z;                                                     // hmc.py:86 N(0,1)
    T q = a.W[w];
    if (take) { q = a.Wwork[w]; a.W[w] = q; }                             // commit (sghmc.py:37)
    if (a.trace) a.trace[(size_t)c * a.P + d * K + k] = q;                // sghmc_multicore.py:49-51 row
    a.pW[w] = p;
    a.Wwork[w] = drift ? q + a.eps * p : q;                               // sghmc.py:32 (iteration 0)
    kin += (double)p * (double)p;
  }
  ksh[tid] = kin;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) ksh[tid] += ksh[tid + s];
    __syncthreads();
  }
  if (tid == 0) a.kin0_part[(size_t)blockIdx.x * a.C + c] = ksh[0];
  if (blockIdx.x == 0) {
    __syncthreads();
    double kb = 0.0;
    if (tid < K) {
      const int col = c * K + tid;
      double z;
      if (a.noise_mode == HMCX_NOISE_BUFFER) z = a.noise[a.noff[c] + a.D * K + tid];
      else z = (double)philox_normal_t<T>(a.seed, a.chain0 + c, a.step, 0u, (uint32_t)(a.D * K + tid));
      const T p = (T)z;
      T q = a.b[col];
      if (take) { q = a.bwork[col]; a.b[col] = q; }
      if (a.trace) a.trace[(size_t)c * a.P + a.D * K + tid] = q;
      a.pb[col] = p;
      a.bwork[col] = q;
      kb = (double)p * (double)p;
    }
    ksh[tid] = kb;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
      if (tid < s) ksh[tid] += ksh[tid + s];
      __syncthreads();
    }
    if (tid == 0) a.kin0b[c] = ksh[0];
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_sghmc_commit(CommitArgs<T> a) {
  const int c = blockIdx.y, tid = threadIdx.x;
  const bool acc = a.acc[c];
  if (!acc && !a.trace) return;
  const int K = a.K, d0 = blockIdx.x * 16;
  for (int e = tid; e < 16 * K; e += 256) {
    const int i = e / K, k = e - (e / K) * K, d = d0 + i;
    if (d >= a.D) continue;
    const size_t w = (size_t)d * a.N + c * K + k;
    const T q = acc ? a.Wwork[w] : a.W[w];
    if (acc) a.W[w] = q;
    if (a.trace) a.trace[(size_t)c * a.P + d * K + k] = q;               // the last step's row
  }
  if (blockIdx.x == 0 && tid < K) {
    const T q = acc ? a.bwork[c * K + tid] : a.b[c * K + tid];
    if (acc) a.b[c * K + tid] = q;
    if (a.trace) a.trace[(size_t)c * a.P + a.D * K + tid] = q;
  }
}

// Deterministic parallel sum of a[i*stride] for i < n over a 64-thread block.
__device__ inline double block_sum64(const double* a, int n, int stride, double* sh) {
  const int t = threadIdx.x;
  double s = 0.0;
  for (int i = t; i < n; i += 64) s += a[(size_t)i * stride];
  sh[t] = s;
  __syncthreads();
  for (int w = 32; w > 0; w >>= 1) {
    if (t < w) sh[t] += sh[t + w];
    __syncthreads();
  }
  const double r = sh[0];
  __syncthreads();
  return r;
}

template <typename T>
__global__ __launch_bounds__(64) void k_sghmc_accept(AcceptArgs<T> a) {
  __shared__ double sh[64];
  const int c = blockIdx.x;
  const int n = a.n_iter[c];
  // hmc.py:67-79: E = nlp + ½Σp² (vars in order weights, bias); A = min(1, exp(E_cur − E_new))
  const double ll0 = block_sum64(a.ll0_part + c, a.nRB, a.C, sh);
  const double S0W = block_sum64(a.kin0_part + c, a.nDB, a.C, sh);
  double ll1 = 0.0, S1W = 0.0;
  if (n > 0) {
    ll1 = block_sum64(a.ll1_part + c, a.nRB, a.C, sh);
    S1W = block_sum64(a.kin1_part + c, a.nDB1, a.C, sh);
  }
  if (threadIdx.x == 0) {
    const double K0 = (0.0 + 0.5 * S0W) + 0.5 * a.kin0b[c];
    const double Ecur = a.neg_inv_n * (ll0 + a.log_prior) + K0;
    double A, Enew, llq;
    int acc;
    if (n <= 0) {
      A = 1.0; Enew = Ecur; llq = ll0;
      acc = a.u[c] < A;
    } else {
      const double K1 = (0.0 + 0.5 * S1W) + 0.5 * a.kin1b[c];
      Enew = a.neg_inv_n * (ll1 + a.log_prior) + K1;
      const double x = exp(Ecur - Enew);
      A = (x < 1.0) ? x : 1.0;                                    // Python min(1, x): NaN -> 1
      acc = a.u[c] < A;
      llq = acc ? ll1 : ll0;
    }
    a.out_A[c] = A;
    // n == 0: q_new is q (sghmc.py:22), nothing to commit; k_fix_acc reports the flag at the end
    a.out_acc[c] = acc && n > 0;
    a.out_ll[c] = llq;
    if (a.out_E) { a.out_E[2 * c] = Ecur; a.out_E[2 * c + 1] = Enew; }
  }
}

// Momentum returned by the call's last step (sghmc.py:36-39): p_new (pW/pb after the last iteration)
// when accepted with at least one iteration, else the momentum drawn at step start (slot 0, as
// k_sghmc_init draws it).  out [C][D·K + K] (weights row-major, then bias).
template <typename T>
__global__ void k_mom_out(InitArgs<T> a, const int32_t* acc, const T* pW, const T* pb, T* out) {
  const int c = blockIdx.y, K = a.K;
  const long long P = (long long)a.D * K + K, DK = (long long)a.D * K;
  const bool keep_new = acc[c] && a.n_iter[c] >= 1;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < P; e += (long long)gridDim.x * blockDim.x) {
    T v;
    if (keep_new) {
      v = e < DK ? pW[(size_t)(e / K) * a.N + c * K + e % K] : pb[c * K + (e - DK)];
    } else if (a.noise_mode == HMCX_NOISE_BUFFER) {
      v = (T)a.noise[a.noff[c] + e];
    } else {
      v = philox_normal_t<T>(a.seed, a.chain0 + c, a.step, 0u, (uint32_t)e);
    }
    out[(size_t)c * P + e] = v;
  }
}

__global__ void k_fix_acc(const int32_t* n_iter, const double* u, int32_t* acc, int n) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < n && n_iter[c] <= 0) acc[c] = u[c] < 1.0;
}

__global__ void k_reduce_ll(const double* ll_part, int nRB, int C, double* out) {
  __shared__ double sh[64];
  const int c = blockIdx.x;
  const double s = block_sum64(ll_part + c, nRB, C, sh);
  if (threadIdx.x == 0) out[c] = s;
}

// ------------------------------------------------------------------ host-side launchers
template <typename T>
static hipError_t launch_fwd(const FwdArgs<T>& a, const Tiling& t, hipStream_t st) {
  const int nz = a.slab_mode == 1 ? a.nslab : 1;
  dim3 grid(t.nRB, t.nCT, nz);
  const bool vec = (a.D % 4) == 0;
#define HMCX_FWD(NB, NW)                                                                          \
  if (vec) hipLaunchKernelGGL((k_fwd<T, NB, true, NW>), grid, dim3(NW * 64), 0, st, a);           \
  else hipLaunchKernelGGL((k_fwd<T, NB, false, NW>), grid, dim3(NW * 64), 0, st, a);
  // few, deep tiles (one chain, large D: config 5) split D over 8 waves instead of 4
  const bool deep = (size_t)t.nRB * t.nCT * nz <= 512 && a.D / nz >= 1024 && a.slab_mode != 2;
  switch (t.NBLK) {
    case 1: HMCX_FWD(1, 8) break;
    case 2: HMCX_FWD(2, 8) break;
    case 3: if (deep) { HMCX_FWD(3, 8) } else { HMCX_FWD(3, 4) } break;
    default: if (deep) { HMCX_FWD(4, 8) } else { HMCX_FWD(4, 4) } break;
  }
#undef HMCX_FWD
  return hipGetLastError();
}

template <typename T>
static hipError_t launch_grad(const GradArgs<T>& a, const Tiling& t, hipStream_t st) {
  dim3 grid(t.nDB, t.nCT);
  const bool deep = (size_t)t.nDB * t.nCT <= 512;
  switch (t.NBLK) {
    case 1: hipLaunchKernelGGL((k_grad<T, 1, 8>), grid, dim3(512), 0, st, a); break;
    case 2: hipLaunchKernelGGL((k_grad<T, 2, 8>), grid, dim3(512), 0, st, a); break;
    case 3:
      if (deep) hipLaunchKernelGGL((k_grad<T, 3, 8>), grid, dim3(512), 0, st, a);
      else hipLaunchKernelGGL((k_grad<T, 3, 4>), grid, dim3(256), 0, st, a);
      break;
    default:
      if (deep) hipLaunchKernelGGL((k_grad<T, 4, 8>), grid, dim3(512), 0, st, a);
      else hipLaunchKernelGGL((k_grad<T, 4, 4>), grid, dim3(256), 0, st, a);
      break;
  }
  return hipGetLastError();
}

// Forward with the D reduction split over S workgroups per tile (S > 1): one launch writes the
// partial XW slabs, a second sums them in a fixed order and runs the epilogue.
template <typename T>
static hipError_t launch_fwd_split(FwdArgs<T> a, const Tiling& t, hipStream_t st, int S, T* slab) {
  if (S <= 1) return launch_fwd<T>(a, t, st);
  a.slab = slab; a.nslab = S;
  a.slab_mode = 1;
  hipError_t e = launch_fwd<T>(a, t, st);
  if (e != hipSuccess) return e;
  a.slab_mode = 2;
  return launch_fwd<T>(a, t, st);
}

Tiling make_tiling(int B, int D, int K, int C) {
  Tiling t;
  t.CB = K >= 64 ? 1 : (64 / K < C ? 64 / K : C);
  if (t.CB < 1) t.CB = 1;
  const int NT = ((t.CB * K + 15) / 16) * 16;
  t.NBLK = NT / 16;
  t.nCT = (C + t.CB - 1) / t.CB;
  t.nRB = (B + 15) / 16;
  t.nDB = (D + 15) / 16;
  return t;
}

template <typename T>
static FwdArgs<T> fwd_args(const void* X, const void* Y, const void* W, const void* b, int B, int D, int K,
                           int C, const Tiling& t, int mode) {
  FwdArgs<T> a{};
  a.X = (const T*)X; a.Y = (const T*)Y; a.W = (const T*)W; a.b = (const T*)b;
  a.B = B; a.D = D; a.K = K; a.C = C; a.N = C * K; a.CB = t.CB;
  a.mode = mode;
  a.clip_hi = (T)CLIP_HI; a.clip_lo = (T)CLIP_LO;
  return a;
}

template <typename T>
static GradArgs<T> grad_args(const T* X, const T* diff, const T* csp, int B, int D, int K, int C, const Tiling& t,
                             int mode, double alpha) {
  GradArgs<T> g{};
  g.X = X; g.diff = diff; g.colsum_part = csp;
  g.B = B; g.D = D; g.K = K; g.C = C; g.N = C * K; g.CB = t.CB; g.nRB = t.nRB; g.nDB = t.nDB; g.P = D * K + K;
  g.mode = mode; g.alpha = (T)alpha;
  return g;
}

// ------------------------------------------------------------------ entry points (typed)
template <typename T>
int softmax_grad_t(hmcx_ctx* ctx, const void* X, const void* Y, int B, int D, int K, int C, const void* W,
                   const void* b, double alpha, void* gW, void* gb, int link) {
  const Tiling t = make_tiling(B, D, K, C);
  const int N = C * K;
  Workspace ws(ctx);
  T *diff, *csp;
  do {
    ws.reset();
    diff = ws.take<T>((size_t)B * N);
    csp = ws.take<T>((size_t)t.nRB * N);
  } while (ws.retry());
  if (ws.failed) return HMCX_ENOMEM;
  FwdArgs<T> f = fwd_args<T>(X, Y, W, b, B, D, K, C, t, FWD_GRAD);
  f.link = link;
  f.diff = diff; f.colsum_part = csp;
  HMCX_HIP(ctx, launch_fwd<T>(f, t, ctx->stream));
  GradArgs<T> g = grad_args<T>((const T*)X, diff, csp, B, D, K, C, t, GRAD_OUT, alpha);
  g.Wsrc = (const T*)W; g.bsrc = (const T*)b; g.gW = (T*)gW; g.gb = (T*)gb;
  HMCX_HIP(ctx, launch_grad<T>(g, t, ctx->stream));
  return HMCX_OK;
}

template <typename T>
int softmax_loglik_t(hmcx_ctx* ctx, const void* X, const void* Y, int B, int D, int K, int C, const void* W,
                     const void* b, double* ll, int link) {
  const Tiling t = make_tiling(B, D, K, C);
  Workspace ws(ctx);
  double* llp;
  do {
    ws.reset();
    llp = ws.take<double>((size_t)t.nRB * C);
  } while (ws.retry());
  if (ws.failed) return HMCX_ENOMEM;
  FwdArgs<T> f = fwd_args<T>(X, Y, W, b, B, D, K, C, t, FWD_LL);
  f.link = link;
  f.ll_part = llp;
  HMCX_HIP(ctx, launch_fwd<T>(f, t, ctx->stream));
  hipLaunchKernelGGL(k_reduce_ll, dim3(C), dim3(64), 0, ctx->stream, llp, t.nRB, C, ll);
  HMCX_HIP(ctx, hipGetLastError());
  return HMCX_OK;
}

template <typename T>
int softmax_predict_t(hmcx_ctx* ctx, const void* X, int B, int D, int K, int C, const void* W, const void* b,
                      void* prob, int link) {
  const Tiling t = make_tiling(B, D, K, C);
  FwdArgs<T> f = fwd_args<T>(X, nullptr, W, b, B, D, K, C, t, FWD_PRED);
  f.link = link;
  f.prob = (T*)prob;
  HMCX_HIP(ctx, launch_fwd<T>(f, t, ctx->stream));
  return HMCX_OK;
}

// ------------------------------------------------------------------ momentum SGD (sgd.py:25-70)
// X_s ⊙ Z for sgd.fit_dropout (sgd.py:61-62): Z from the host's binomial draws or from Philox.
template <typename T>
__global__ void k_xdrop(const T* X, T* Xd, int64_t n, const uint8_t* keep, int mode, double p, uint64_t seed,
                        uint32_t step) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool z = mode == HMCX_NOISE_BUFFER ? keep[i] != 0 : philox_uniform(seed, 0u, step, SLOT_DROPX, (uint32_t)i) < p;
  Xd[i] = X[i] * (z ? T(1) : T(0));                                      // np.multiply(X_batch, Z)
}

// One k_fwd (gradient mode, softmax or sigmoid link) + one k_grad (GRAD_SGD epilogue) per minibatch.
template <typename T>
int sgd_run_t(hmcx_ctx* ctx, const hmcx_sgd_args* s) {
  const int B = s->B, D = s->D, K = s->K;
  const Tiling t = make_tiling(B, D, K, 1);
  const int link = s->model == HMCX_MODEL_LOGISTIC ? LINK_SIGMOID : LINK_SOFTMAX;
  Workspace ws(ctx);
  T *diff, *csp, *xd = nullptr;
  do {
    ws.reset();
    diff = ws.take<T>((size_t)B * K);
    csp = ws.take<T>((size_t)t.nRB * K);
    if (s->dropout) xd = ws.take<T>((size_t)B * D);
  } while (ws.retry());
  if (ws.failed) return HMCX_ENOMEM;
  begin_call(ctx);
  int rc;
  if ((rc = timing_begin(ctx, ctx->stream))) return rc;
  GraphScope gs(ctx);
  hipStream_t st = ctx->stream;
  for (int i = 0; i < s->n_steps; ++i) {
    const T* Xs = (const T*)s->X + (size_t)s->row0[i] * D;
    const T* Ys = (const T*)s->Y + (size_t)s->row0[i] * K;
    if (s->dropout) {
      const int64_t n = (int64_t)B * D;
      const uint8_t* kp = s->mask_mode == HMCX_NOISE_BUFFER ? s->keep + s->keep_off[i] : nullptr;
      hipLaunchKernelGGL(k_xdrop<T>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, Xs, xd, n, kp,
                         s->mask_mode, s->keep_p, s->seed, s->step_base + (uint32_t)i);
      HMCX_HIP(ctx, hipGetLastError());
      Xs = xd;
    }
    FwdArgs<T> f = fwd_args<T>(Xs, Ys, s->W, s->b, B, D, K, 1, t, FWD_GRAD);
    f.link = link;
    f.diff = diff; f.colsum_part = csp;
    HMCX_HIP(ctx, launch_fwd<T>(f, t, st));
    GradArgs<T> g = grad_args<T>(Xs, diff, csp, B, D, K, 1, t, GRAD_SGD, s->alpha);
    g.gamma = (T)s->gamma; g.lr = (T)s->step_size;
    g.W = (T*)s->W; g.b = (T*)s->b; g.pW = (T*)s->mW; g.pb = (T*)s->mb;
    HMCX_HIP(ctx, launch_grad<T>(g, t, st));
  }
  if ((rc = gs.finish())) return rc;
  return timing_end(ctx, ctx->stream);
}

// Σ x² in float64, fixed order (logistic.py:20's np.sum(np.square(θ))).  Up to SQ_ONE elements one workgroup
// (lane t sums elements t, t + 256, …, then a fixed tree); above, SQ_NB workgroups each sum a contiguous slice
// that way into part[b] and one more launch adds the SQ_NB partials in block order — one workgroup streaming
// a 200,704-element W1 alone took 37.8 µs (one CU's pull rate), a quarter of the full-batch MLP accept.
constexpr int64_t SQ_ONE = 16384;
constexpr int SQ_NB = 64;
template <typename T>
__device__ inline double sumsq_slice(const T* x, int64_t i0, int64_t i1) {
  __shared__ double sh[256];
  double acc = 0.0;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += 256) {
    const double v = (double)x[i];
    acc += v * v;
  }
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
    __syncthreads();
  }
  return sh[0];
}
template <typename T>
__global__ __launch_bounds__(256) void k_sumsq(const T* x, int64_t n, double* out) {
  const int64_t per = (n + gridDim.x - 1) / gridDim.x, i0 = (int64_t)blockIdx.x * per;
  const double v = sumsq_slice<T>(x, i0, i0 + per < n ? i0 + per : n);
  if (threadIdx.x == 0) out[blockIdx.x] = v;
}
__global__ void k_sumsq_fin(const double* part, int nb, double* out) {
  double s = part[0];
  for (int b = 1; b < nb; ++b) s += part[b];
  *out = s;
}

template <typename T>
int sumsq_t(hmcx_ctx* ctx, const void* x, int64_t n, double* out) {
  if (n <= SQ_ONE) {
    hipLaunchKernelGGL(k_sumsq<T>, dim3(1), dim3(256), 0, ctx->stream, (const T*)x, n, out);
  } else {
    Workspace ws(ctx);
    double* part;
    do { ws.reset(); part = ws.take<double>(SQ_NB); } while (ws.retry());
    if (ws.failed) return set_error(ctx, HMCX_ENOMEM, "sumsq: workspace");
    hipLaunchKernelGGL(k_sumsq<T>, dim3(SQ_NB), dim3(256), 0, ctx->stream, (const T*)x, n, part);
    hipLaunchKernelGGL(k_sumsq_fin, dim3(1), dim3(1), 0, ctx->stream, (const double*)part, SQ_NB, out);
  }
  HMCX_HIP(ctx, hipGetLastError());
  return HMCX_OK;
}

// ------------------------------------------------------------------ leapfrog axpy (hmc.py:50-53)
template <typename T>
__global__ __launch_bounds__(256) void k_axpy(int mode, int64_t n, T a, const T* x, T* y) {   // x may alias y
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const T ax = a * x[i];
    y[i] = mode == 0 ? y[i] - ax : y[i] + ax;
  }
}

template <typename T>
int axpy_t(hmcx_ctx* ctx, int mode, int64_t n, double a, const void* x, void* y) {
  if (n == 0) return HMCX_OK;
  const int64_t nb = std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_axpy<T>, dim3((unsigned)nb), dim3(256), 0, ctx->stream, mode, n, (T)a, (const T*)x, (T*)y);
  HMCX_HIP(ctx, hipGetLastError());
  return HMCX_OK;
}

// ------------------------------------------------------------------ full-batch HMC, linear models
// hmc.py:39-64 with the softmax / logistic model, one chain.  State: q = (W, b) (caller's buffers),
// the proposal (Wn, bn) and its momentum (pW, pb) in the workspace.  Per step:
//   k_hmc_init     p0 (hmc.py:41), proposal := q, Σp0² partials
//   [n_iter ≥ 1]   1 + 2·n_iter gradient evaluations at the proposal: k_fwd(FWD_GRAD) + k_grad(GRAD_HMC)
//                  whose epilogue applies the kicks/drifts that follow that evaluation (HmcFlags)
//   k_fwd(FWD_LL)  log-likelihood of the proposal
//   k_hmc_accept   energies (hmc.py:67-79), MH decision, nlp of the kept state (carried to the next
//                  step as its E_current's nlp: the same kernel output, so no recomputation)
//   k_hmc_commit   q := proposal if accepted; trace row of the kept state
struct HmcState {
  double ll, sW, sb;   // log-likelihood and Σθ² (weights, bias) of the current state q
};

template <typename T>
struct HmcInitArgs {
  int D, K, P, nDB;
  int noise_mode; const double* noise; int64_t noff;
  uint64_t seed; uint32_t chain, step;
  const T* W; const T* b; T* Wn; T* bn; T* pW; T* pb; T* mom;
  double* kin0_part;   // [nDB + 1]: Σ pW0² per block, then Σ pb0²
};

template <typename T>
__global__ __launch_bounds__(256) void k_hmc_init(HmcInitArgs<T> a) {
  __shared__ double ksh[256];
  const int tid = threadIdx.x, K = a.K;
  const int e0 = blockIdx.x * 16 * K, ne = min(16 * K, a.D * K - e0);
  double kin = 0.0;
  for (int e = tid; e < ne; e += 256) {
    const int i = e0 + e;
    const T p = a.noise_mode == HMCX_NOISE_BUFFER ? (T)a.noise[a.noff + i]
                                                  : philox_normal_t<T>(a.seed, a.chain, a.step, 0u, (uint32_t)i);
    a.pW[i] = p;
    a.Wn[i] = a.W[i];
    if (a.mom) a.mom[i] = p;
    kin += (double)p * (double)p;
  }
  ksh[tid] = kin;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) ksh[tid] += ksh[tid + s];
    __syncthreads();
  }
  if (tid == 0) a.kin0_part[blockIdx.x] = ksh[0];
  if (blockIdx.x == 0) {
    __syncthreads();
    double kb = 0.0;
    if (tid < K) {
      const int i = a.D * K + tid;
      const T p = a.noise_mode == HMCX_NOISE_BUFFER ? (T)a.noise[a.noff + i]
                                                    : philox_normal_t<T>(a.seed, a.chain, a.step, 0u, (uint32_t)i);
      a.pb[tid] = p;
      a.bn[tid] = a.b[tid];
      if (a.mom) a.mom[i] = p;
      kb = (double)p * (double)p;
    }
    ksh[tid] = kb;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
      if (tid < s) ksh[tid] += ksh[tid + s];
      __syncthreads();
    }
    if (tid == 0) a.kin0_part[a.nDB] = ksh[0];
  }
}

template <typename T>
struct HmcAcceptArgs {
  int D, K, nRB, nDB, n_iter, first, logistic;
  double u, neg_inv_n, log_prior, lpc0, lpc1, half_alpha;
  const double* kin0_part; const double* ll0_part; const double* ll1_part;
  const T* W; const T* b; const T* Wn; const T* bn; const T* pW; const T* pb;
  HmcState* st;
  double* out_A; int32_t* out_acc; double* out_nlp; double* out_E;
};

// Fixed-order Σ f(i) for i < n over the 256 threads of the block.
template <typename F>
__device__ inline double block_sum256(int n, F f, double* sh) {
  const int t = threadIdx.x;
  double s = 0.0;
  for (int i = t; i < n; i += 256) s += f(i);
  sh[t] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) sh[t] += sh[t + w];
    __syncthreads();
  }
  const double r = sh[0];
  __syncthreads();
  return r;
}

template <typename T>
__global__ __launch_bounds__(256) void k_hmc_accept(HmcAcceptArgs<T> a) {
  __shared__ double sh[256];
  const int DK = a.D * a.K;
  const bool moved = a.n_iter > 0;
  // current state: computed at the call's first step, carried afterwards
  double ll0, sW0, sb0;
  if (a.first) {
    ll0 = block_sum256(a.nRB, [&](int i) { return a.ll0_part[i]; }, sh);
    sW0 = a.logistic ? block_sum256(DK, [&](int i) { const double v = (double)a.W[i]; return v * v; }, sh) : 0.0;
    sb0 = a.logistic ? block_sum256(a.K, [&](int i) { const double v = (double)a.b[i]; return v * v; }, sh) : 0.0;
  } else {
    ll0 = a.st->ll; sW0 = a.st->sW; sb0 = a.st->sb;
  }
  const double S0W = block_sum256(a.nDB, [&](int i) { return a.kin0_part[i]; }, sh);
  double ll1 = ll0, sW1 = sW0, sb1 = sb0, S1W = 0.0, S1b = 0.0;
  if (moved) {
    ll1 = block_sum256(a.nRB, [&](int i) { return a.ll1_part[i]; }, sh);
    if (a.logistic) {
      sW1 = block_sum256(DK, [&](int i) { const double v = (double)a.Wn[i]; return v * v; }, sh);
      sb1 = block_sum256(a.K, [&](int i) { const double v = (double)a.bn[i]; return v * v; }, sh);
    }
    S1W = block_sum256(DK, [&](int i) { const double v = (double)a.pW[i]; return v * v; }, sh);
    S1b = block_sum256(a.K, [&](int i) { const double v = (double)a.pb[i]; return v * v; }, sh);
  }
  if (threadIdx.x == 0) {
    auto nlp = [&](double ll, double sW, double sb) {
      double lp = a.log_prior;                                   // softmax.py:22-30 (constant)
      if (a.logistic) lp = (((0.0 + a.lpc0) - a.half_alpha * sW) + a.lpc1) - a.half_alpha * sb;   // logistic.py:15-21
      return a.neg_inv_n * (ll + lp);
    };
    const double K0 = (0.0 + 0.5 * S0W) + 0.5 * a.kin0_part[a.nDB];
    const double nlp0 = nlp(ll0, sW0, sb0);
    const double Ecur = nlp0 + K0;
    double Enew = Ecur, A = 1.0;
    if (moved) {
      const double K1 = (0.0 + 0.5 * S1W) + 0.5 * S1b;           // ½Σ(−p)² = ½Σp² (hmc.py:55-56)
      Enew = nlp(ll1, sW1, sb1) + K1;
      const double x = exp(Ecur - Enew);
      A = (x < 1.0) ? x : 1.0;                                   // Python min(1, x): NaN → 1
    }
    const int acc = a.u < A;
    a.out_A[0] = A;
    a.out_acc[0] = acc;
    if (a.out_E) { a.out_E[0] = Ecur; a.out_E[1] = Enew; }
    HmcState s;
    if (acc && moved) { s.ll = ll1; s.sW = sW1; s.sb = sb1; }
    else { s.ll = ll0; s.sW = sW0; s.sb = sb0; }
    *a.st = s;
    a.out_nlp[0] = (acc && moved) ? nlp(ll1, sW1, sb1) : nlp0;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_hmc_commit(int DK, int K, const int32_t* acc, const T* Wn, const T* bn,
                                                    T* W, T* b, T* trace) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const bool take = *acc != 0;
  if (i < DK) {
    T v = W[i];
    if (take) { v = Wn[i]; W[i] = v; }
    if (trace) trace[i] = v;
  } else if (i < DK + K) {
    T v = b[i - DK];
    if (take) { v = bn[i - DK]; b[i - DK] = v; }
    if (trace) trace[i] = v;
  }
}

template <typename T>
int hmc_run_t(hmcx_ctx* ctx, const hmcx_hmc_args* s) {
  const int B = s->B, D = s->D, K = s->K, DK = D * K, P = DK + K;
  const bool logistic = s->model == HMCX_MODEL_LOGISTIC;
  const int link = logistic ? LINK_SIGMOID : LINK_SOFTMAX;
  const Tiling t = make_tiling(B, D, K, 1);
  Workspace ws(ctx);
  T *Wn, *bn, *pW, *pb, *diff, *csp;
  double *kin0, *ll0p, *ll1p;
  HmcState* st;
  do {
    ws.reset();
    Wn = ws.take<T>(DK); bn = ws.take<T>(K); pW = ws.take<T>(DK); pb = ws.take<T>(K);
    diff = ws.take<T>((size_t)B * K); csp = ws.take<T>((size_t)t.nRB * K);
    kin0 = ws.take<double>(t.nDB + 1); ll0p = ws.take<double>(t.nRB); ll1p = ws.take<double>(t.nRB);
    st = ws.take<HmcState>(1);
  } while (ws.retry());
  if (ws.failed) return HMCX_ENOMEM;
  begin_call(ctx);
  int rc;
  if ((rc = timing_begin(ctx, ctx->stream))) return rc;
  GraphScope gs(ctx);
  hipStream_t st_ = ctx->stream;
  T* W = (T*)s->W;
  T* b = (T*)s->b;
  // log-likelihood of the call's starting state (its nlp enters step 0's E_current)
  {
    FwdArgs<T> f = fwd_args<T>(s->X, s->Y, W, b, B, D, K, 1, t, FWD_LL);
    f.link = link;
    f.ll_part = ll0p;
    HMCX_HIP(ctx, launch_fwd<T>(f, t, st_));
  }
  for (int i = 0; i < s->n_steps; ++i) {
    const double eps = s->eps[i];
    const int n = s->n_iter[i];
    HmcInitArgs<T> ia{};
    ia.D = D; ia.K = K; ia.P = P; ia.nDB = t.nDB;
    ia.noise_mode = s->noise_mode; ia.noise = s->noise;
    ia.noff = s->noise_mode == HMCX_NOISE_BUFFER ? s->noise_off[i] : 0;
    ia.seed = s->seed; ia.chain = s->chain; ia.step = s->step_base + (uint32_t)i;
    ia.W = W; ia.b = b; ia.Wn = Wn; ia.bn = bn; ia.pW = pW; ia.pb = pb;
    ia.mom = s->out_mom ? (T*)s->out_mom + (size_t)i * P : nullptr;
    ia.kin0_part = kin0;
    hipLaunchKernelGGL(k_hmc_init<T>, dim3(t.nDB), dim3(256), 0, st_, ia);
    HMCX_HIP(ctx, hipGetLastError());
    const int n_eval = n > 0 ? 1 + 2 * n : 0;
    for (int e = 0; e < n_eval; ++e) {
      FwdArgs<T> f = fwd_args<T>(s->X, s->Y, Wn, bn, B, D, K, 1, t, FWD_GRAD);
      f.link = link;
      f.diff = diff; f.colsum_part = csp;
      HMCX_HIP(ctx, launch_fwd<T>(f, t, st_));
      GradArgs<T> g = grad_args<T>((const T*)s->X, diff, csp, B, D, K, 1, t, GRAD_HMC, s->alpha);
      g.eps = (T)eps; g.half_eps = (T)(0.5 * eps);
      g.W = Wn; g.b = bn; g.pW = pW; g.pb = pb;
      int fl;
      if (e == 0) fl = HMC_HALF_W;                               // hmc.py:47 then it 0, weights
      else if (e & 1) fl = HMC_KICK_W | HMC_HALF_B;              // after the weights' drift
      else fl = HMC_KICK_B | (e < 2 * n ? HMC_HALF_W : 0);       // after the bias' drift
      g.hmc_flags = fl;
      HMCX_HIP(ctx, launch_grad<T>(g, t, st_));
    }
    if (n > 0) {
      FwdArgs<T> f = fwd_args<T>(s->X, s->Y, Wn, bn, B, D, K, 1, t, FWD_LL);
      f.link = link;
      f.ll_part = ll1p;
      HMCX_HIP(ctx, launch_fwd<T>(f, t, st_));
    }
    HmcAcceptArgs<T> aa{};
    aa.D = D; aa.K = K; aa.nRB = t.nRB; aa.nDB = t.nDB; aa.n_iter = n; aa.first = i == 0; aa.logistic = logistic;
    aa.u = s->u_accept[i]; aa.neg_inv_n = -1.0 / (double)B; aa.log_prior = s->log_prior;
    aa.lpc0 = s->lp_const[0]; aa.lpc1 = s->lp_const[1]; aa.half_alpha = 0.5 * s->alpha;
    aa.kin0_part = kin0; aa.ll0_part = ll0p; aa.ll1_part = ll1p;
    aa.W = W; aa.b = b; aa.Wn = Wn; aa.bn = bn; aa.pW = pW; aa.pb = pb;
    aa.st = st;
    aa.out_A = s->out_A + i; aa.out_acc = s->out_accepted + i; aa.out_nlp = s->out_nlp + i;
    aa.out_E = s->out_E ? s->out_E + 2 * i : nullptr;
    hipLaunchKernelGGL(k_hmc_accept<T>, dim3(1), dim3(256), 0, st_, aa);
    HMCX_HIP(ctx, hipGetLastError());
    T* tr = s->out_trace ? (T*)s->out_trace + (size_t)i * P : nullptr;
    if (n > 0 || tr) {
      hipLaunchKernelGGL(k_hmc_commit<T>, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, st_, DK, K,
                         s->out_accepted + i, Wn, bn, W, b, tr);
      HMCX_HIP(ctx, hipGetLastError());
    }
  }
  if ((rc = gs.finish())) return rc;
  return timing_end(ctx, ctx->stream);
}

// k_sghmc_init for the chain-batched path: same arithmetic, but the working copy Wwork and the
// momentum pW are chain-major [C][D][K] (each chain's block contiguous, so every tile of the batched
// kernels owns whole cache lines); W stays in the caller's [D][C·K] layout.  One workgroup per
// (16 features, 16 chains): 16 lanes per chain, each taking element pairs (k, k+1) of one feature —
// one Box–Muller per pair (both normals of the Philox block are used), the chain-major writes
// contiguous per chain, the kinetic partial summed over the chain's 16 lanes (fixed DPP order).
template <typename T>
__device__ inline void philox_pair_t(uint64_t seed, uint32_t chain, uint32_t step, uint32_t slot, uint32_t e, T& z0,
                                     T& z1) {   // elements e, e + 1 (e even) of philox_normal_t<T>
  if constexpr (sizeof(T) == sizeof(double)) {
    double a, b;
    philox_pair_d(seed, chain, step, slot, e >> 1, a, b);
    z0 = (T)a; z1 = (T)b;
  } else {
    u32x4 c = {{e >> 2, slot, step, chain}};
    u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    float a, b;
    if (e & 2u) box_muller(r.v[2], r.v[3], a, b);
    else box_muller(r.v[0], r.v[1], a, b);
    z0 = (T)a; z1 = (T)b;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_binit(InitArgs<T> a) {
  const int tid = threadIdx.x, K = a.K, KP = K / 2;                 // K even (batched path: K = 10)
  const int cl = tid >> 4, j = tid & 15;
  const int c = blockIdx.y * 16 + cl, d0 = blockIdx.x * 16;
  const bool cv = c < a.C;
  const int cc = cv ? c : a.C - 1;
  const bool take = cv && a.prev_acc && a.prev_acc[cc];
  const bool drift = cv && a.n_iter[cc] >= 1;
  double kin = 0.0;
  for (int r = j; r < 16 * KP; r += 16) {                            // pair r: feature r / KP, classes 2·(r % KP) + {0, 1}
    const int dl = r / KP, k = 2 * (r - dl * KP), d = d0 + dl;
    if (!cv || d >= a.D) continue;
    const size_t w = (size_t)d * a.N + c * K + k;
    const size_t wc = ((size_t)c * a.D + d) * K + k;
    T p0, p1;
    if (a.noise_mode == HMCX_NOISE_BUFFER) {
      p0 = (T)a.noise[a.noff[c] + d * K + k];
      p1 = (T)a.noise[a.noff[c] + d * K + k + 1];
    } else {
      philox_pair_t<T>(a.seed, a.chain0 + c, a.step, 0u, (uint32_t)(d * K + k), p0, p1);   // hmc.py:86
    }
    T q0, q1;
    if (take) {                                                       // commit (sghmc.py:37)
      q0 = a.Wwork[wc]; q1 = a.Wwork[wc + 1];
      a.W[w] = q0; a.W[w + 1] = q1;
    } else {
      q0 = a.W[w]; q1 = a.W[w + 1];
    }
    if (a.trace) {                                                    // sghmc_multicore.py:49-51 row
      a.trace[(size_t)c * a.P + d * K + k] = q0;
      a.trace[(size_t)c * a.P + d * K + k + 1] = q1;
    }
    a.pW[wc] = p0; a.pW[wc + 1] = p1;
    a.Wwork[wc] = drift ? q0 + a.eps * p0 : q0;                       // sghmc.py:32 (iteration 0)
    a.Wwork[wc + 1] = drift ? q1 + a.eps * p1 : q1;
    kin += (double)p0 * (double)p0;
    kin += (double)p1 * (double)p1;
  }
  // the chain's 16 lanes (one DPP row): symmetric pairs, every lane ends with the same bits
  kin += __shfl_xor(kin, 1, 16);
  kin += __shfl_xor(kin, 2, 16);
  kin += __shfl_xor(kin, 4, 16);
  kin += __shfl_xor(kin, 8, 16);
  if (j == 0 && cv) a.kin0_part[(size_t)blockIdx.x * a.C + c] = kin;
  if (blockIdx.x == 0 && cv) {                                        // the bias of chain c
    double kb = 0.0;
    if (j < K) {
      const int col = c * K + j;
      double z;
      if (a.noise_mode == HMCX_NOISE_BUFFER) z = a.noise[a.noff[c] + a.D * K + j];
      else z = (double)philox_normal_t<T>(a.seed, a.chain0 + c, a.step, 0u, (uint32_t)(a.D * K + j));
      const T p = (T)z;
      T q = a.b[col];
      if (take) { q = a.bwork[col]; a.b[col] = q; }
      if (a.trace) a.trace[(size_t)c * a.P + a.D * K + j] = q;
      a.pb[col] = p;
      a.bwork[col] = q;
      kb = (double)p * (double)p;
    }
    kb += __shfl_xor(kb, 1, 16);
    kb += __shfl_xor(kb, 2, 16);
    kb += __shfl_xor(kb, 4, 16);
    kb += __shfl_xor(kb, 8, 16);
    if (j == 0) a.kin0b[c] = kb;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_bcommit(CommitArgs<T> a) {
  const int c = blockIdx.y, tid = threadIdx.x;
  const bool acc = a.acc[c];
  if (!acc && !a.trace) return;
  const int K = a.K, d0 = blockIdx.x * 16;
  for (int e = tid; e < 16 * K; e += 256) {
    const int i = e / K, k = e - (e / K) * K, d = d0 + i;
    if (d >= a.D) continue;
    const size_t w = (size_t)d * a.N + c * K + k;
    const T q = acc ? a.Wwork[((size_t)c * a.D + d) * K + k] : a.W[w];
    if (acc) a.W[w] = q;
    if (a.trace) a.trace[(size_t)c * a.P + d * K + k] = q;               // the last step's row
  }
  if (blockIdx.x == 0 && tid < K) {
    const T q = acc ? a.bwork[c * K + tid] : a.b[c * K + tid];
    if (acc) a.b[c * K + tid] = q;
    if (a.trace) a.trace[(size_t)c * a.P + a.D * K + tid] = q;
  }
}

// C chains, K = 10: per step k_sghmc_init, k_bfwd(LL) at q0, then per leapfrog iteration k_bfwd +
// k_bgrad over the chains still moving (ranks < c_act(it), ranks = chains by path length
// descending), k_sghmc_accept; the last step's proposal is committed by k_sghmc_commit.
template <typename T>
int sghmc_batch_t(hmcx_ctx* ctx, const hmcx_sampler_args* s) {
  const int B = s->B, D = s->D, K = s->K, C = s->C, N = C * K;
  // row tiles of 64 (k_bfwd<T,2>) whenever the step's first iteration has >= 32 tiles of chains;
  // colsum/ll partials are laid out per 32-row block (a 64-row tile writes its sums and a zero block)
  const bool big = C >= 512;
  const int nX64 = (B + 63) / 64, nRB = big ? 2 * nX64 : (B + 31) / 32;
  const int nDB = (D + BRW - 1) / BRW, nDB16 = (D + 15) / 16;
  // compaction-tail launches (< one workgroup per CU at 64-row tiles): 32-row tiles, twice the workgroups
  // (HMCX_BTAIL32=0: the 8-wave 64-row kernel, round 3)
  const bool tail32 = !(getenv("HMCX_BTAIL32") && getenv("HMCX_BTAIL32")[0] == '0');
  const int nDB2 = (D + BRW2 - 1) / BRW2;            // k_bgradw<T, 4> feature tiles
  // dynamic LDS of the wide gradient kernel (set once per kernel)
  const size_t lds4 = BGW<T, 4>::lds();
  static bool bgw_attr = false;
  if (!bgw_attr) {
    HMCX_HIP(ctx, hipFuncSetAttribute((const void*)k_bgradw<T, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds4));
    bgw_attr = true;
  }
  const size_t nsc = (size_t)s->n_steps * C;
  // host: chain order per step (path length descending, stable) and active counts per iteration
  std::vector<int32_t> perm(nsc);
  for (int st = 0; st < s->n_steps; ++st) {
    int32_t* pr = perm.data() + (size_t)st * C;
    std::iota(pr, pr + C, 0);
    const int32_t* ni = s->n_iter + (size_t)st * C;
    std::stable_sort(pr, pr + C, [&](int32_t x, int32_t y) { return ni[x] > ni[y]; });
  }
  Workspace ws(ctx);
  T *Wwork, *bwork, *pW, *pb, *diff, *csp;
  double *ll0, *ll1, *k0p, *k0b, *k1p, *k1b, *d_u;
  int32_t *d_niter, *d_perm;
  int64_t* d_noff;
  do {
    ws.reset();
    Wwork = ws.take<T>((size_t)D * N);
    bwork = ws.take<T>(N);
    pW = ws.take<T>((size_t)D * N);
    pb = ws.take<T>(N);
    diff = ws.take<T>((size_t)B * N);
    csp = ws.take<T>((size_t)nRB * N);
    ll0 = ws.take<double>((size_t)nRB * C);
    ll1 = ws.take<double>((size_t)nRB * C);
    k0p = ws.take<double>((size_t)nDB16 * C);
    k1p = ws.take<double>((size_t)nDB * C);
    k0b = ws.take<double>(C);
    k1b = ws.take<double>(C);
    d_niter = ws.take<int32_t>(nsc);
    d_perm = ws.take<int32_t>(nsc);
    d_u = ws.take<double>(nsc);
    d_noff = ws.take<int64_t>(nsc);
  } while (ws.retry());
  if (ws.failed) return HMCX_ENOMEM;
  begin_call(ctx);
  int rc = upload(ctx, d_niter, s->n_iter, nsc * sizeof(int32_t));
  if (rc) return rc;
  if ((rc = upload(ctx, d_perm, perm.data(), nsc * sizeof(int32_t)))) return rc;
  if ((rc = upload(ctx, d_u, s->u_accept, nsc * sizeof(double)))) return rc;
  if (s->noise_mode == HMCX_NOISE_BUFFER && (rc = upload(ctx, d_noff, s->noise_off, nsc * sizeof(int64_t))))
    return rc;

  const T* X = (const T*)s->X;
  const T* Y = (const T*)s->Y;
  if ((rc = timing_begin(ctx, ctx->stream))) return rc;
  GraphScope gs(ctx);
  hipStream_t st = ctx->stream;
  for (int st_i = 0; st_i < s->n_steps; ++st_i) {
    const T* Xs = X + (size_t)s->row0[st_i] * D;
    const T* Ys = Y + (size_t)s->row0[st_i] * K;
    const double eps = s->eps[st_i];
    const int32_t* ni_h = s->n_iter + (size_t)st_i * C;
    int maxit = 0;
    for (int c = 0; c < C; ++c) maxit = std::max(maxit, (int)ni_h[c]);
    const int32_t* niter = d_niter + (size_t)st_i * C;
    const int32_t* prm = d_perm + (size_t)st_i * C;
    const int64_t* noff = d_noff + (size_t)st_i * C;
    const uint32_t step_id = s->step_base + (uint32_t)st_i;

    InitArgs<T> ia{};
    ia.D = D; ia.K = K; ia.C = C; ia.N = N; ia.nDB = nDB16;
    ia.eps = (T)eps; ia.n_iter = niter;
    ia.prev_acc = st_i > 0 ? s->out_accepted + (size_t)(st_i - 1) * C : nullptr;
    ia.noise_mode = s->noise_mode; ia.noise = s->noise; ia.noff = noff;
    ia.seed = s->seed; ia.chain0 = s->chain0; ia.step = step_id;
    ia.W = (T*)s->W; ia.b = (T*)s->b;
    ia.Wwork = Wwork; ia.bwork = bwork; ia.pW = pW; ia.pb = pb;
    ia.kin0_part = k0p; ia.kin0b = k0b;
    ia.P = D * K + K;
    ia.trace = s->out_trace && st_i > 0 ? (T*)s->out_trace + (size_t)(st_i - 1) * C * ia.P : nullptr;
    hipLaunchKernelGGL((k_binit<T>), dim3(nDB16, (C + 15) / 16), dim3(256), 0, st, ia);
    HMCX_HIP(ctx, hipGetLastError());

    BFwdArgs<T> f{};
    f.X = Xs; f.Y = Ys; f.B = B; f.D = D; f.C = C; f.N = N; f.eps = (T)eps;
    f.n_iter = niter; f.perm = prm;
    f.mode = FWD_LL; f.iter = -1; f.c_act = C;                      // E_current at q0 (all chains)
    f.W = (const T*)s->W; f.b = (const T*)s->b; f.pb = pb;
    f.ll_part = ll0;
    f.nX = big ? nX64 : nRB; f.nCT = (C + BCT - 1) / BCT;
    f.nRB_all = nRB;
    if (big) hipLaunchKernelGGL((k_bfwd<T, 2, 0>), dim3(xcd_grid(f.nX, f.nCT)), dim3(256), 0, st, f);
    else hipLaunchKernelGGL((k_bfwd<T, 1, 0>), dim3(xcd_grid(f.nX, f.nCT)), dim3(256), 0, st, f);
    HMCX_HIP(ctx, hipGetLastError());

    f.mode = FWD_SGHMC; f.W = Wwork; f.b = bwork;
    f.diff = diff; f.colsum_part = csp; f.ll_part = ll1;
    BGradArgs<T> g{};
    g.X = Xs; g.diff = diff; g.colsum_part = csp;
    g.B = B; g.D = D; g.C = C; g.N = N; g.nRB = nRB; g.P = D * K + K;
    g.alpha = (T)s->alpha; g.eps = (T)eps; g.one_minus_eps = (T)(1.0 - eps); g.noise_scale = (T)(2.0 * eps);
    g.n_iter = niter; g.perm = prm;
    g.W = Wwork; g.b = bwork; g.pW = pW; g.pb = pb;
    g.kin_part = k1p; g.kinb = k1b; g.nDB_all = nDB;
    g.noise_mode = s->noise_mode; g.noise = s->noise; g.noff = noff;
    g.seed = s->seed; g.chain0 = s->chain0; g.step = step_id;
    for (int it = 0; it < maxit; ++it) {
      int c_act = 0;
      while (c_act < C && ni_h[perm[(size_t)st_i * C + c_act]] > it) ++c_act;
      f.iter = it; f.c_act = c_act;
      f.nX = big ? nX64 : nRB; f.nCT = (c_act + BCT - 1) / BCT;
      // launches that leave CUs without a second workgroup: 32-row tiles (or the 8-wave 64-row kernel)
      static const bool bf8_off = getenv("HMCX_BFWD8") && getenv("HMCX_BFWD8")[0] == '0';
      // HMCX_BTAIL_WG / HMCX_BGW_MIN: tile-height and feature-tile switch points (measurement knobs)
      static const int tail_wg = getenv("HMCX_BTAIL_WG") ? atoi(getenv("HMCX_BTAIL_WG")) : ctx->num_cus;
      const bool tail = big && f.nX * f.nCT <= tail_wg;
      if (tail && tail32) {
        f.nX = (B + 31) / 32;
        hipLaunchKernelGGL((k_bfwd<T, 1, 1>), dim3(xcd_grid(f.nX, f.nCT)), dim3(256), 0, st, f);
      } else if (tail && !bf8_off)
        hipLaunchKernelGGL((k_bfwd<T, 2, 1, 8>), dim3(xcd_grid(f.nX, f.nCT)), dim3(512), 0, st, f);
      else if (big) hipLaunchKernelGGL((k_bfwd<T, 2, 1>), dim3(xcd_grid(f.nX, f.nCT)), dim3(256), 0, st, f);
      else hipLaunchKernelGGL((k_bfwd<T, 1, 1>), dim3(xcd_grid(f.nX, f.nCT)), dim3(256), 0, st, f);
      HMCX_HIP(ctx, hipGetLastError());
      g.iter = it; g.c_act = c_act; g.slot = (uint32_t)(it + 1);
      // 64-feature tiles while they fill the chip's 2 workgroups per CU, 32-feature tiles after
      const int ctiles = (c_act + BCT - 1) / BCT;
      g.nCT = ctiles;
      static const int bgw_min = getenv("HMCX_BGW_MIN") ? atoi(getenv("HMCX_BGW_MIN")) : 2 * ctx->num_cus;
      if (nDB2 * ctiles >= bgw_min) {
        g.nX = nDB2;
        static const bool tail_off = getenv("HMCX_BGW_TAIL") && getenv("HMCX_BGW_TAIL")[0] == '0';
        g.tail_last = !tail_off && nDB2 > 1 && D % BRW2 != 0 && D % BRW2 <= BRW2 / 2;
        hipLaunchKernelGGL((k_bgradw<T, 4>), dim3(xcd_grid(g.nX, g.nCT)), dim3(256), lds4, st, g);
      } else {
        g.nX = nDB;
        hipLaunchKernelGGL((k_bgrad<T>), dim3(xcd_grid(g.nX, g.nCT)), dim3(256), 0, st, g);
      }
      HMCX_HIP(ctx, hipGetLastError());
    }
    AcceptArgs<T> aa{};
    aa.C = C; aa.nRB = nRB; aa.nDB = nDB16; aa.nDB1 = nDB;
    aa.n_iter = niter; aa.u = d_u + (size_t)st_i * C;
    aa.neg_inv_n = -1.0 / (double)B; aa.log_prior = s->log_prior;
    aa.kin0_part = k0p; aa.kin0b = k0b; aa.kin1_part = k1p; aa.kin1b = k1b;
    aa.ll0_part = ll0; aa.ll1_part = ll1;
    aa.out_A = s->out_A + (size_t)st_i * C;
    aa.out_acc = s->out_accepted + (size_t)st_i * C;
    aa.out_ll = s->out_ll + (size_t)st_i * C;
    aa.out_E = s->out_E ? s->out_E + (size_t)st_i * C * 2 : nullptr;
    hipLaunchKernelGGL((k_sghmc_accept<T>), dim3(C), dim3(64), 0, st, aa);
    HMCX_HIP(ctx, hipGetLastError());
  }
  CommitArgs<T> ca{};
  ca.D = D; ca.K = K; ca.C = C; ca.N = N;
  ca.acc = s->out_accepted + (size_t)(s->n_steps - 1) * C;
  ca.Wwork = Wwork; ca.bwork = bwork; ca.W = (T*)s->W; ca.b = (T*)s->b;
  ca.P = D * K + K;
  ca.trace = s->out_trace ? (T*)s->out_trace + (size_t)(s->n_steps - 1) * C * ca.P : nullptr;
  hipLaunchKernelGGL((k_bcommit<T>), dim3(nDB16, C), dim3(256), 0, st, ca);
  HMCX_HIP(ctx, hipGetLastError());
  hipLaunchKernelGGL(k_fix_acc, dim3((unsigned)((nsc + 255) / 256)), dim3(256), 0, st, d_niter, d_u,
                     s->out_accepted, (int)nsc);
  HMCX_HIP(ctx, hipGetLastError());
  if ((rc = gs.finish())) return rc;
  return timing_end(ctx, ctx->stream);
}

// True when sghmc_run_t serves this call with k_sghmc_p2, which writes out_trace itself.
bool sghmc_p2_selected(hmcx_ctx* ctx, const hmcx_sampler_args* s) {
  if (s->C != 1 || ctx->sghmc_path == 1) return false;
  const size_t ts = s->dtype == HMCX_F64 ? sizeof(double) : sizeof(float);
  return plan_p2(s->B, s->D, s->K, ts, ctx->num_cus, ctx->lds_max).ok;
}

template <typename T>
int sghmc_run_t(hmcx_ctx* ctx, const hmcx_sampler_args* s) {
  const int B = s->B, D = s->D, K = s->K, C = s->C, N = C * K;
  if (C == 1 && ctx->sghmc_path != 1) {   // single chain: persistent kernels
    const PersistPlan2 p2 = plan_p2(B, D, K, sizeof(T), ctx->num_cus, ctx->lds_max);
    if (p2.ok) return sghmc_p2_t<T>(ctx, s, p2);
    if (ctx->sghmc_path == 2) return set_error(ctx, HMCX_EUNSUPPORTED, "persistent SGHMC: shape not supported");
  } else if (ctx->sghmc_path >= 2) {
    return set_error(ctx, HMCX_EUNSUPPORTED, "persistent SGHMC needs C == 1");
  }
  static const bool no_batch = getenv("HMCX_NO_BATCH") && getenv("HMCX_NO_BATCH")[0] == '1';
  if (C >= 16 && K == BKC && D % 2 == 0 && !no_batch) {                                // chain-batched GEMMs
    if (s->out_mom) return set_error(ctx, HMCX_EUNSUPPORTED, "out_mom: single-chain / C < 16 paths only");
    return sghmc_batch_t<T>(ctx, s);
  }
  const Tiling t = make_tiling(B, D, K, C);
  const size_t nsc = (size_t)s->n_steps * C;
  Workspace ws(ctx);
  T *Wwork, *bwork, *pW, *pb, *diff, *csp;
  double *ll0, *ll1, *k0p, *k0b, *k1p, *k1b, *d_u;
  int32_t* d_niter;
  int64_t* d_noff;
  do {
    ws.reset();
    Wwork = ws.take<T>((size_t)D * N);
    bwork = ws.take<T>(N);
    pW = ws.take<T>((size_t)D * N);
    pb = ws.take<T>(N);
    diff = ws.take<T>((size_t)B * N);
    csp = ws.take<T>((size_t)t.nRB * N);
    ll0 = ws.take<double>((size_t)t.nRB * C);
    ll1 = ws.take<double>((size_t)t.nRB * C);
    k0p = ws.take<double>((size_t)t.nDB * C);
    k1p = ws.take<double>((size_t)t.nDB * C);
    k0b = ws.take<double>(C);
    k1b = ws.take<double>(C);
    d_niter = ws.take<int32_t>(nsc);
    d_u = ws.take<double>(nsc);
    d_noff = ws.take<int64_t>(nsc);
  } while (ws.retry());
  if (ws.failed) return HMCX_ENOMEM;
  begin_call(ctx);
  int rc = upload(ctx, d_niter, s->n_iter, nsc * sizeof(int32_t));
  if (rc) return rc;
  if ((rc = upload(ctx, d_u, s->u_accept, nsc * sizeof(double)))) return rc;
  if (s->noise_mode == HMCX_NOISE_BUFFER && (rc = upload(ctx, d_noff, s->noise_off, nsc * sizeof(int64_t))))
    return rc;

  const T* X = (const T*)s->X;
  const T* Y = (const T*)s->Y;
  if ((rc = timing_begin(ctx, ctx->stream))) return rc;
  GraphScope gs(ctx);
  hipStream_t st = ctx->stream;
  for (int st_i = 0; st_i < s->n_steps; ++st_i) {
    const T* Xs = X + (size_t)s->row0[st_i] * D;
    const T* Ys = Y + (size_t)s->row0[st_i] * K;
    const double eps = s->eps[st_i];
    int maxit = 0;
    for (int c = 0; c < C; ++c) maxit = std::max(maxit, (int)s->n_iter[(size_t)st_i * C + c]);
    const int32_t* niter = d_niter + (size_t)st_i * C;
    const int64_t* noff = d_noff + (size_t)st_i * C;
    const uint32_t step_id = s->step_base + (uint32_t)st_i;

    InitArgs<T> ia{};
    ia.D = D; ia.K = K; ia.C = C; ia.N = N; ia.nDB = t.nDB;
    ia.eps = (T)eps; ia.n_iter = niter;
    ia.prev_acc = st_i > 0 ? s->out_accepted + (size_t)(st_i - 1) * C : nullptr;
    ia.noise_mode = s->noise_mode; ia.noise = s->noise; ia.noff = noff;
    ia.seed = s->seed; ia.chain0 = s->chain0; ia.step = step_id;
    ia.W = (T*)s->W; ia.b = (T*)s->b;
    ia.Wwork = Wwork; ia.bwork = bwork; ia.pW = pW; ia.pb = pb;
    ia.kin0_part = k0p; ia.kin0b = k0b;
    ia.P = D * K + K;
    ia.trace = s->out_trace && st_i > 0 ? (T*)s->out_trace + (size_t)(st_i - 1) * C * ia.P : nullptr;
    hipLaunchKernelGGL((k_sghmc_init<T>), dim3(t.nDB, C), dim3(256), 0, st, ia);
    HMCX_HIP(ctx, hipGetLastError());

    FwdArgs<T> f0 = fwd_args<T>(Xs, Ys, s->W, s->b, B, D, K, C, t, FWD_LL);
    f0.ll_part = ll0;
    HMCX_HIP(ctx, launch_fwd<T>(f0, t, st));

    FwdArgs<T> f = fwd_args<T>(Xs, Ys, Wwork, bwork, B, D, K, C, t, FWD_SGHMC);
    f.pb = pb; f.eps = (T)eps; f.n_iter = niter;
    f.diff = diff; f.colsum_part = csp; f.ll_part = ll1;
    GradArgs<T> g = grad_args<T>(Xs, diff, csp, B, D, K, C, t, GRAD_SGHMC, s->alpha);
    g.eps = (T)eps; g.one_minus_eps = (T)(1.0 - eps); g.noise_scale = (T)(2.0 * eps);
    g.n_iter = niter;
    g.W = Wwork; g.b = bwork; g.pW = pW; g.pb = pb;
    g.kin_part = k1p; g.kinb = k1b;
    g.noise_mode = s->noise_mode; g.noise = s->noise; g.noff = noff;
    g.seed = s->seed; g.chain0 = s->chain0; g.step = step_id;
    for (int it = 0; it < maxit; ++it) {
      f.iter = it;
      HMCX_HIP(ctx, launch_fwd<T>(f, t, st));
      g.iter = it;
      g.slot = (uint32_t)(it + 1);
      HMCX_HIP(ctx, launch_grad<T>(g, t, st));
    }
    AcceptArgs<T> aa{};
    aa.C = C; aa.nRB = t.nRB; aa.nDB = t.nDB; aa.nDB1 = t.nDB;
    aa.n_iter = niter; aa.u = d_u + (size_t)st_i * C;
    aa.neg_inv_n = -1.0 / (double)B; aa.log_prior = s->log_prior;
    aa.kin0_part = k0p; aa.kin0b = k0b; aa.kin1_part = k1p; aa.kin1b = k1b;
    aa.ll0_part = ll0; aa.ll1_part = ll1;
    aa.out_A = s->out_A + (size_t)st_i * C;
    aa.out_acc = s->out_accepted + (size_t)st_i * C;
    aa.out_ll = s->out_ll + (size_t)st_i * C;
    aa.out_E = s->out_E ? s->out_E + (size_t)st_i * C * 2 : nullptr;
    hipLaunchKernelGGL((k_sghmc_accept<T>), dim3(C), dim3(64), 0, st, aa);
    HMCX_HIP(ctx, hipGetLastError());
  }
  // commit the last step's proposal, then report n_iter == 0 steps as accepted (A = 1 > u)
  CommitArgs<T> ca{};
  ca.D = D; ca.K = K; ca.C = C; ca.N = N;
  ca.acc = s->out_accepted + (size_t)(s->n_steps - 1) * C;
  ca.Wwork = Wwork; ca.bwork = bwork; ca.W = (T*)s->W; ca.b = (T*)s->b;
  ca.P = D * K + K;
  ca.trace = s->out_trace ? (T*)s->out_trace + (size_t)(s->n_steps - 1) * C * ca.P : nullptr;
  hipLaunchKernelGGL((k_sghmc_commit<T>), dim3(t.nDB, C), dim3(256), 0, st, ca);
  HMCX_HIP(ctx, hipGetLastError());
  hipLaunchKernelGGL(k_fix_acc, dim3((unsigned)((nsc + 255) / 256)), dim3(256), 0, st, d_niter, d_u,
                     s->out_accepted, (int)nsc);
  HMCX_HIP(ctx, hipGetLastError());
  if (s->out_mom) {
    const int last = s->n_steps - 1;
    InitArgs<T> ma{};
    ma.D = D; ma.K = K; ma.C = C; ma.N = N;
    ma.n_iter = d_niter + (size_t)last * C;
    ma.noise_mode = s->noise_mode; ma.noise = s->noise; ma.noff = d_noff + (size_t)last * C;
    ma.seed = s->seed; ma.chain0 = s->chain0; ma.step = s->step_base + (uint32_t)last;
    const unsigned gx = (unsigned)std::min<long long>(((long long)D * K + K + 255) / 256, 1024);
    hipLaunchKernelGGL((k_mom_out<T>), dim3(gx, C), dim3(256), 0, st, ma, s->out_accepted + (size_t)last * C,
                       (const T*)pW, (const T*)pb, (T*)s->out_mom);
    HMCX_HIP(ctx, hipGetLastError());
  }
  if ((rc = gs.finish())) return rc;
  return timing_end(ctx, ctx->stream);
}

template <typename T>
int sgld_run_t(hmcx_ctx* ctx, const hmcx_sampler_args* s) {
  const int B = s->B, D = s->D, K = s->K, C = s->C, N = C * K;
  const Tiling t = make_tiling(B, D, K, C);
  const size_t nsc = (size_t)s->n_steps * C;
  // few, deep forward tiles (one chain, large D: config 5): split D over S workgroups per tile
  int S = 1;
  if ((size_t)t.nRB * t.nCT < 128 && D >= 1024)
    S = std::max(1, std::min(std::min(256 / (t.nRB * t.nCT), D / 256), 16));
  Workspace ws(ctx);
  T *diff, *csp, *slab = nullptr;
  double* llp;
  int64_t* d_noff;
  do {
    ws.reset();
    diff = ws.take<T>((size_t)B * N);
    csp = ws.take<T>((size_t)t.nRB * N);
    llp = ws.take<double>((size_t)t.nRB * C);
    d_noff = ws.take<int64_t>(nsc);
    if (S > 1) slab = ws.take<T>((size_t)S * B * N);
  } while (ws.retry());
  if (ws.failed) return HMCX_ENOMEM;
  begin_call(ctx);
  int rc;
  if (s->noise_mode == HMCX_NOISE_BUFFER && (rc = upload(ctx, d_noff, s->noise_off, nsc * sizeof(int64_t))))
    return rc;
  const T* X = (const T*)s->X;
  const T* Y = (const T*)s->Y;
  if ((rc = timing_begin(ctx, ctx->stream))) return rc;
  GraphScope gs(ctx);
  hipStream_t st = ctx->stream;
  for (int st_i = 0; st_i < s->n_steps; ++st_i) {
    const T* Xs = X + (size_t)s->row0[st_i] * D;
    const T* Ys = Y + (size_t)s->row0[st_i] * K;
    const double eps = s->eps[st_i];
    FwdArgs<T> f = fwd_args<T>(Xs, Ys, s->W, s->b, B, D, K, C, t, FWD_GRAD);
    f.diff = diff; f.colsum_part = csp;
    HMCX_HIP(ctx, launch_fwd_split<T>(f, t, st, S, slab));
    GradArgs<T> g = grad_args<T>(Xs, diff, csp, B, D, K, C, t, s->pW ? GRAD_SGLD_GPU : GRAD_SGLD, s->alpha);
    g.eps = (T)eps;
    g.noise_scale = (T)(2.0 * eps);                               // sgld.py:43
    g.m_half_eps = (T)(-0.5 * eps);                               // sgld.py:37
    g.W = (T*)s->W; g.b = (T*)s->b; g.pW = (T*)s->pW; g.pb = (T*)s->pb;
    g.noise_mode = s->noise_mode; g.noise = s->noise; g.noff = d_noff + (size_t)st_i * C;
    g.seed = s->seed; g.chain0 = s->chain0; g.step = s->step_base + (uint32_t)st_i; g.slot = 0;
    g.trace = s->out_trace ? (T*)s->out_trace + (size_t)st_i * C * g.P : nullptr;
    HMCX_HIP(ctx, launch_grad<T>(g, t, st));
    if (s->want_ll && s->want_ll[st_i] && s->out_ll) {
      FwdArgs<T> fl = fwd_args<T>(Xs, Ys, s->W, s->b, B, D, K, C, t, FWD_LL);
      fl.ll_part = llp;
      HMCX_HIP(ctx, launch_fwd_split<T>(fl, t, st, S, slab));
      hipLaunchKernelGGL(k_reduce_ll, dim3(C), dim3(64), 0, st, llp, t.nRB, C, s->out_ll + (size_t)st_i * C);
      HMCX_HIP(ctx, hipGetLastError());
    }
  }
  if ((rc = gs.finish())) return rc;
  return timing_end(ctx, ctx->stream);
}

template int softmax_grad_t<float>(hmcx_ctx*, const void*, const void*, int, int, int, int, const void*,
                                   const void*, double, void*, void*, int);
template int softmax_grad_t<double>(hmcx_ctx*, const void*, const void*, int, int, int, int, const void*,
                                    const void*, double, void*, void*, int);
template int softmax_loglik_t<float>(hmcx_ctx*, const void*, const void*, int, int, int, int, const void*,
                                     const void*, double*, int);
template int softmax_loglik_t<double>(hmcx_ctx*, const void*, const void*, int, int, int, int, const void*,
                                      const void*, double*, int);
template int softmax_predict_t<float>(hmcx_ctx*, const void*, int, int, int, int, const void*, const void*, void*,
                                      int);
template int softmax_predict_t<double>(hmcx_ctx*, const void*, int, int, int, int, const void*, const void*, void*,
                                       int);
template int sgd_run_t<float>(hmcx_ctx*, const hmcx_sgd_args*);
template int sgd_run_t<double>(hmcx_ctx*, const hmcx_sgd_args*);
template int hmc_run_t<float>(hmcx_ctx*, const hmcx_hmc_args*);
template int hmc_run_t<double>(hmcx_ctx*, const hmcx_hmc_args*);
template int axpy_t<float>(hmcx_ctx*, int, int64_t, double, const void*, void*);
template int axpy_t<double>(hmcx_ctx*, int, int64_t, double, const void*, void*);
template int sumsq_t<float>(hmcx_ctx*, const void*, int64_t, double*);
template int sumsq_t<double>(hmcx_ctx*, const void*, int64_t, double*);
template int sghmc_run_t<float>(hmcx_ctx*, const hmcx_sampler_args*);
template int sghmc_run_t<double>(hmcx_ctx*, const hmcx_sampler_args*);
template int sgld_run_t<float>(hmcx_ctx*, const hmcx_sampler_args*);
template int sgld_run_t<double>(hmcx_ctx*, const hmcx_sampler_args*);

}  // namespace hmcx
