// hmcx_softmax.hip — softmax-regression gradient + SGHMC / SGLD leapfrog kernels (gfx950).
//
// Reference hot path:
//   softmax.grad          /root/reference/hamiltonian/models/cpu/softmax.py:38-61   (A6)
//   softmax.log_likelihood                                         softmax.py:63-72 (A7)
//   sghmc.step            /root/reference/hamiltonian/inference/cpu/sghmc.py:19-39  (A1)
//   sgld.step             /root/reference/hamiltonian/inference/cpu/sgld.py:31-46   (A2)
//
// One SGHMC leapfrog iteration (sghmc.py:28-34, vars in order weights, bias) is two kernels:
//   k_fwd  (rows x chain-tile):  Z = X·W (MFMA), then per (row, chain): z = clip(Z+b),
//          softmax, diff = y − ŷ  (for the weights sub-step), and the bias sub-step
//          b' = b + ε·pb, z' = clip(Z+b'), Σ_rows(y − ŷ') partials and log-likelihood
//          partials at (W, b') — the bias sub-step reuses X·W (W is unchanged by it).
//   k_grad (features x chain-tile):  Xᵀ·diff (MFMA), fused epilogue
//          g = −(Xᵀdiff − αW);  p = (1−ε)p + εg + 2ε·ξ;  W += ε·p (next drift);
//          tile-column 0 also finishes the bias sub-step from the row partials.
// Elementwise arithmetic follows the reference's NumPy op order with FP contraction off
// (-ffp-contract=off), so float64 runs differ from NumPy only through GEMM summation order.
#include "hmcx_common.h"
#include "hmcx_internal.h"

namespace hmcx {

// ------------------------------------------------------------------ forward (logits) kernel
template <typename T, int NBLK, bool VEC>
__global__ __launch_bounds__(256) void k_fwd(FwdArgs<T> a) {
  using M = mfma16<T>;
  constexpr int NT = NBLK * 16;
  __shared__ T red[4][16][NT];
  __shared__ T zt[16][NT + 1];
  __shared__ T dt[16][NT + 1];
  __shared__ double llt[16][NT];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int m0 = blockIdx.x * 16;
  const int c0 = blockIdx.y * a.CB;
  const int ncb = min(a.CB, a.C - c0);
  const int n0 = c0 * a.K;
  const int ncols = ncb * a.K;

  typename M::acc_t acc0[NBLK], acc1[NBLK];
#pragma unroll
  for (int nb = 0; nb < NBLK; ++nb) { acc0[nb] = M::zero(); acc1[nb] = M::zero(); }

  const int Dq = ((a.D + 63) / 64) * 16;
  const int kbeg = wave * Dq, kend = min(a.D, kbeg + Dq);
  const int row = m0 + r;
  const bool rok = row < a.B;
  const T* xrow = a.X + (size_t)(rok ? row : 0) * a.D;

  for (int kc = kbeg; kc < kend; kc += 16) {
    const int kb = kc + 4 * g;
    T av[4];
    if (VEC && kc + 16 <= kend) {
      if (rok) {
        if constexpr (sizeof(T) == 8) {
          const double2* p2 = reinterpret_cast<const double2*>(xrow + kb);
          double2 u = p2[0], v = p2[1];
          av[0] = u.x; av[1] = u.y; av[2] = v.x; av[3] = v.y;
        } else {
          float4 u = *reinterpret_cast<const float4*>(xrow + kb);
          av[0] = u.x; av[1] = u.y; av[2] = u.z; av[3] = u.w;
        }
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) av[s] = T(0);
      }
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s) av[s] = (rok && kb + s < kend) ? xrow[kb + s] : T(0);
    }
#pragma unroll
    for (int nb = 0; nb < NBLK; ++nb) {
      const int col = nb * 16 + r;
      const bool cok = col < ncols;
      T bv[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int kk = kb + s;
        bv[s] = (cok && kk < kend) ? a.W[(size_t)kk * a.N + n0 + col] : T(0);
      }
      acc0[nb] = M::fma(av[0], bv[0], acc0[nb]);
      acc1[nb] = M::fma(av[1], bv[1], acc1[nb]);
      acc0[nb] = M::fma(av[2], bv[2], acc0[nb]);
      acc1[nb] = M::fma(av[3], bv[3], acc1[nb]);
    }
  }
#pragma unroll
  for (int nb = 0; nb < NBLK; ++nb)
#pragma unroll
    for (int q = 0; q < 4; ++q) red[wave][M::row(lane, q)][nb * 16 + r] = acc0[nb][q] + acc1[nb][q];
  __syncthreads();
  for (int e = tid; e < 16 * NT; e += 256) {
    const int i = e / NT, j = e % NT;
    zt[i][j] = ((red[0][i][j] + red[1][i][j]) + red[2][i][j]) + red[3][i][j];
  }
  __syncthreads();

  // ---- epilogue: one thread per (row, chain)
  const T hi = a.clip_hi, lo = a.clip_lo;
  for (int p = tid; p < 16 * ncb; p += 256) {
    const int i = p & 15, cc = p >> 4;
    const int rw = m0 + i;
    const int cb = cc * a.K;
    const int c = c0 + cc;
    if (rw >= a.B) continue;
    const bool active = (a.mode != FWD_SGHMC) || (a.iter < a.n_iter[c]);
    const T* y = a.Y + (size_t)rw * a.K;
    const T* bb = a.b + n0 + cb;
    if (a.mode == FWD_GRAD || a.mode == FWD_SGHMC || a.mode == FWD_PRED) {
      // softmax.py:39-43 at (W, b)
      T m = np_max(np_min(zt[i][cb] + bb[0], hi), lo);
      for (int k = 1; k < a.K; ++k) m = max_nan(m, np_max(np_min(zt[i][cb + k] + bb[k], hi), lo));
      T s = T(0);
      for (int k = 0; k < a.K; ++k) s += exp(np_max(np_min(zt[i][cb + k] + bb[k], hi), lo) - m);
      for (int k = 0; k < a.K; ++k) {
        const T yh = exp(np_max(np_min(zt[i][cb + k] + bb[k], hi), lo) - m) / s;
        if (a.mode == FWD_PRED) {
          a.prob[(size_t)rw * a.N + n0 + cb + k] = yh;
        } else {
          const T d = y[k] - yh;                                  // softmax.py:52
          if (active) a.diff[(size_t)rw * a.N + n0 + cb + k] = d;
          if (a.mode == FWD_GRAD) dt[i][cb + k] = d;
        }
      }
    }
    if (a.mode == FWD_SGHMC) {
      // bias sub-step (sghmc.py:32-33 for var 'bias'): b' = b + ε·pb, grad at (W, b')
      const T* pb = a.pb + n0 + cb;
      T m = np_max(np_min(zt[i][cb] + (bb[0] + a.eps * pb[0]), hi), lo);
      for (int k = 1; k < a.K; ++k)
        m = max_nan(m, np_max(np_min(zt[i][cb + k] + (bb[k] + a.eps * pb[k]), hi), lo));
      T s = T(0);
      for (int k = 0; k < a.K; ++k) s += exp(np_max(np_min(zt[i][cb + k] + (bb[k] + a.eps * pb[k]), hi), lo) - m);
      const T lse = log(s) + m;
      double ll = 0.0;
      for (int k = 0; k < a.K; ++k) {
        const T z = np_max(np_min(zt[i][cb + k] + (bb[k] + a.eps * pb[k]), hi), lo);
        dt[i][cb + k] = y[k] - exp(z - m) / s;
        ll += (double)(y[k] * (z - lse));                         // softmax.py:17-20
      }
      llt[i][cc] = ll;
    } else if (a.mode == FWD_LL) {
      T m = np_max(np_min(zt[i][cb] + bb[0], hi), lo);
      for (int k = 1; k < a.K; ++k) m = max_nan(m, np_max(np_min(zt[i][cb + k] + bb[k], hi), lo));
      T s = T(0);
      for (int k = 0; k < a.K; ++k) s += exp(np_max(np_min(zt[i][cb + k] + bb[k], hi), lo) - m);
      const T lse = log(s) + m;
      double ll = 0.0;
      for (int k = 0; k < a.K; ++k) {
        const T z = np_max(np_min(zt[i][cb + k] + bb[k], hi), lo);
        ll += (double)(y[k] * (z - lse));
      }
      llt[i][cc] = ll;
    }
  }
  __syncthreads();
  if (a.mode == FWD_GRAD || a.mode == FWD_SGHMC) {
    for (int j = tid; j < ncols; j += 256) {
      const int c = c0 + j / a.K;
      if (a.mode == FWD_SGHMC && a.iter >= a.n_iter[c]) continue;
      T s = T(0);
      for (int i = 0; i < 16 && m0 + i < a.B; ++i) s += dt[i][j];
      a.colsum_part[(size_t)blockIdx.x * a.N + n0 + j] = s;
    }
  }
  if (a.mode == FWD_SGHMC || a.mode == FWD_LL) {
    for (int cc = tid; cc < ncb; cc += 256) {
      const int c = c0 + cc;
      if (a.mode == FWD_SGHMC && a.iter >= a.n_iter[c]) continue;
      double s = 0.0;
      for (int i = 0; i < 16 && m0 + i < a.B; ++i) s += llt[i][cc];
      a.ll_part[(size_t)blockIdx.x * a.C + c] = s;
    }
  }
}

// ------------------------------------------------------------------ noise
template <typename T>
__device__ inline double noise_at(const GradArgs<T>& a, int c, uint32_t e) {
  if (a.noise_mode == HMCX_NOISE_BUFFER) return a.noise[a.noff[c] + (int64_t)a.slot * a.P + e];
  return philox_normal(a.seed, a.chain0 + c, a.step, a.slot, e);
}

// ------------------------------------------------------------------ gradient (Xᵀ·diff) kernel
template <typename T, int NBLK>
__global__ __launch_bounds__(256) void k_grad(GradArgs<T> a) {
  using M = mfma16<T>;
  constexpr int NT = NBLK * 16;
  __shared__ T red[4][16][NT];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int d0 = blockIdx.x * 16;
  const int c0 = blockIdx.y * a.CB;
  const int ncb = min(a.CB, a.C - c0);
  const int n0 = c0 * a.K;
  const int ncols = ncb * a.K;

  typename M::acc_t acc0[NBLK], acc1[NBLK];
#pragma unroll
  for (int nb = 0; nb < NBLK; ++nb) { acc0[nb] = M::zero(); acc1[nb] = M::zero(); }

  const int Bq = ((a.B + 63) / 64) * 16;
  const int kbeg = wave * Bq, kend = min(a.B, kbeg + Bq);
  const bool dok = d0 + r < a.D;
  for (int kc = kbeg; kc < kend; kc += 16) {
    const int kb = kc + 4 * g;
    T av[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int kk = kb + s;
      av[s] = (dok && kk < kend) ? a.X[(size_t)kk * a.D + d0 + r] : T(0);
    }
#pragma unroll
    for (int nb = 0; nb < NBLK; ++nb) {
      const int col = nb * 16 + r;
      const bool cok = col < ncols;
      T bv[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int kk = kb + s;
        bv[s] = (cok && kk < kend) ? a.diff[(size_t)kk * a.N + n0 + col] : T(0);
      }
      acc0[nb] = M::fma(av[0], bv[0], acc0[nb]);
      acc1[nb] = M::fma(av[1], bv[1], acc1[nb]);
      acc0[nb] = M::fma(av[2], bv[2], acc0[nb]);
      acc1[nb] = M::fma(av[3], bv[3], acc1[nb]);
    }
  }
#pragma unroll
  for (int nb = 0; nb < NBLK; ++nb)
#pragma unroll
    for (int q = 0; q < 4; ++q) red[wave][M::row(lane, q)][nb * 16 + r] = acc0[nb][q] + acc1[nb][q];
  __syncthreads();

  const int DK = a.D * a.K;
  for (int e = tid; e < 16 * NT; e += 256) {
    const int i = e / NT, j = e % NT;
    const int d = d0 + i;
    if (d >= a.D || j >= ncols) continue;
    const T dot = ((red[0][i][j] + red[1][i][j]) + red[2][i][j]) + red[3][i][j];
    const int cc = j / a.K, k = j - cc * a.K, c = c0 + cc;
    const size_t idx = (size_t)d * a.N + n0 + j;
    if (a.mode == GRAD_OUT) {
      a.gW[idx] = -(dot - a.alpha * a.Wsrc[idx]);                 // softmax.py:57-58
    } else if (a.mode == GRAD_SGHMC) {
      if (a.iter >= a.n_iter[c]) continue;
      const T w = a.W[idx];
      const T gr = -(dot - a.alpha * w);
      T p = a.pW[idx];
      const T z = (T)noise_at(a, c, (uint32_t)(d * a.K + k));
      p = (a.one_minus_eps * p + a.eps * gr) + a.noise_scale * z;  // sghmc.py:31,34
      a.pW[idx] = p;
      if (a.iter < a.n_iter[c] - 1) a.W[idx] = w + a.eps * p;     // next iteration's drift :32
    } else {  // GRAD_SGLD (sgld.py:34-38)
      const T w = a.W[idx];
      const T gr = -(dot - a.alpha * w);
      const T z = (T)noise_at(a, c, (uint32_t)(d * a.K + k));
      T p = a.noise_scale * z;
      p = p + a.m_half_eps * gr;
      a.W[idx] = w + p;
    }
  }

  if (blockIdx.x == 0) {  // bias: Σ_rows(y−ŷ) from the k_fwd row partials (softmax.py:55,59-60)
    for (int j = tid; j < ncols; j += 256) {
      const int cc = j / a.K, k = j - cc * a.K, c = c0 + cc;
      const int col = n0 + j;
      if (a.mode == GRAD_SGHMC && a.iter >= a.n_iter[c]) continue;
      T cs = T(0);
      for (int rb = 0; rb < a.nRB; ++rb) cs += a.colsum_part[(size_t)rb * a.N + col];
      if (a.mode == GRAD_OUT) {
        a.gb[col] = -(cs - a.alpha * a.bsrc[col]);
      } else if (a.mode == GRAD_SGHMC) {
        const T bb = a.b[col];
        T p = a.pb[col];
        const T bp = bb + a.eps * p;
        const T gr = -(cs - a.alpha * bp);
        const T z = (T)noise_at(a, c, (uint32_t)(DK + k));
        p = (a.one_minus_eps * p + a.eps * gr) + a.noise_scale * z;
        a.pb[col] = p;
        a.b[col] = bp;
      } else {
        const T bb = a.b[col];
        const T gr = -(cs - a.alpha * bb);
        const T z = (T)noise_at(a, c, (uint32_t)(DK + k));
        T p = a.noise_scale * z;
        p = p + a.m_half_eps * gr;
        a.b[col] = bb + p;
      }
    }
  }
}

// ------------------------------------------------------------------ SGHMC step init / accept
template <typename T>
__global__ __launch_bounds__(256) void k_sghmc_init(InitArgs<T> a) {
  const int P = a.D * a.K + a.K;
  const int DK = a.D * a.K;
  const int total = a.C * P;
  for (int idx = blockIdx.x * 256 + threadIdx.x; idx < total; idx += gridDim.x * 256) {
    const int c = idx / P, e = idx - c * P;
    double z;
    if (a.noise_mode == HMCX_NOISE_BUFFER) z = a.noise[a.noff[c] + e];
    else z = philox_normal(a.seed, a.chain0 + c, a.step, 0u, (uint32_t)e);
    const T p = (T)z;                                             // hmc.py:86 N(0,1)
    if (e < DK) {
      const int d = e / a.K, k = e - d * a.K;
      const size_t w = (size_t)d * a.N + c * a.K + k;
      a.p0W[w] = p;
      a.pW[w] = p;
      const T q = a.W[w];
      a.Wwork[w] = (a.n_iter[c] >= 1) ? q + a.eps * p : q;        // sghmc.py:32 (iteration 0)
    } else {
      const int col = c * a.K + (e - DK);
      a.p0b[col] = p;
      a.pb[col] = p;
      a.bwork[col] = a.b[col];
    }
  }
}

__device__ inline double block_sum256(double v, double* sh) {
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (t < s) sh[t] = sh[t] + sh[t + s];
    __syncthreads();
  }
  const double r = sh[0];
  __syncthreads();
  return r;
}

template <typename T>
__global__ __launch_bounds__(256) void k_sghmc_accept(AcceptArgs<T> a) {
  __shared__ double sh[256];
  const int c = blockIdx.x, t = threadIdx.x;
  const int DK = a.D * a.K;
  const int n = a.n_iter[c];
  double s0 = 0.0, s1 = 0.0;
  for (int e = t; e < DK; e += 256) {
    const int d = e / a.K, k = e - d * a.K;
    const size_t w = (size_t)d * a.N + c * a.K + k;
    const double x0 = (double)a.p0W[w], x1 = (double)a.pW[w];
    s0 += x0 * x0;
    s1 += x1 * x1;
  }
  const double S0W = block_sum256(s0, sh), S1W = block_sum256(s1, sh);
  s0 = 0.0; s1 = 0.0;
  for (int k = t; k < a.K; k += 256) {
    const double x0 = (double)a.p0b[c * a.K + k], x1 = (double)a.pb[c * a.K + k];
    s0 += x0 * x0;
    s1 += x1 * x1;
  }
  const double S0b = block_sum256(s0, sh), S1b = block_sum256(s1, sh);
  __shared__ int acc_sh;
  if (t == 0) {
    // hmc.py:67-79: E = nlp + ½Σp² (vars in order weights, bias); A = min(1, exp(E_cur − E_new))
    double ll0 = 0.0;
    for (int rb = 0; rb < a.nRB; ++rb) ll0 += a.ll0_part[(size_t)rb * a.C + c];
    const double K0 = (0.0 + 0.5 * S0W) + 0.5 * S0b;
    const double Ecur = a.neg_inv_n * (ll0 + a.log_prior) + K0;
    double A, Enew, llq;
    int acc;
    if (n <= 0) {
      A = 1.0; Enew = Ecur; llq = ll0;
      acc = a.u[c] < A;
    } else {
      double ll1 = 0.0;
      for (int rb = 0; rb < a.nRB; ++rb) ll1 += a.ll1_part[(size_t)rb * a.C + c];
      const double K1 = (0.0 + 0.5 * S1W) + 0.5 * S1b;
      Enew = a.neg_inv_n * (ll1 + a.log_prior) + K1;
      const double x = exp(Ecur - Enew);
      A = (x < 1.0) ? x : 1.0;                                    // Python min(1, x): NaN -> 1
      acc = a.u[c] < A;
      llq = acc ? ll1 : ll0;
    }
    a.out_A[c] = A;
    a.out_acc[c] = acc;
    a.out_ll[c] = llq;
    if (a.out_E) { a.out_E[2 * c] = Ecur; a.out_E[2 * c + 1] = Enew; }
    acc_sh = acc && (n > 0);
  }
  __syncthreads();
  if (acc_sh) {                                                  // sghmc.py:36-38
    for (int e = t; e < DK; e += 256) {
      const int d = e / a.K, k = e - d * a.K;
      const size_t w = (size_t)d * a.N + c * a.K + k;
      a.W[w] = a.Wwork[w];
    }
    for (int k = t; k < a.K; k += 256) a.b[c * a.K + k] = a.bwork[c * a.K + k];
  }
}

__global__ void k_reduce_ll(const double* ll_part, int nRB, int C, double* out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0;
  for (int rb = 0; rb < nRB; ++rb) s += ll_part[(size_t)rb * C + c];
  out[c] = s;
}

// ------------------------------------------------------------------ host-side launchers
template <typename T>
static hipError_t launch_fwd(const FwdArgs<T>& a, const Tiling& t, hipStream_t st) {
  dim3 grid(t.nRB, t.nCT), block(256);
  const bool vec = (a.D % 4) == 0;
#define HMCX_FWD(NB)                                                                   \
  if (vec) hipLaunchKernelGGL((k_fwd<T, NB, true>), grid, block, 0, st, a);            \
  else hipLaunchKernelGGL((k_fwd<T, NB, false>), grid, block, 0, st, a);
  switch (t.NBLK) {
    case 1: HMCX_FWD(1) break;
    case 2: HMCX_FWD(2) break;
    case 3: HMCX_FWD(3) break;
    default: HMCX_FWD(4) break;
  }
#undef HMCX_FWD
  return hipGetLastError();
}

template <typename T>
static hipError_t launch_grad(const GradArgs<T>& a, const Tiling& t, hipStream_t st) {
  dim3 grid(t.nDB, t.nCT), block(256);
  switch (t.NBLK) {
    case 1: hipLaunchKernelGGL((k_grad<T, 1>), grid, block, 0, st, a); break;
    case 2: hipLaunchKernelGGL((k_grad<T, 2>), grid, block, 0, st, a); break;
    case 3: hipLaunchKernelGGL((k_grad<T, 3>), grid, block, 0, st, a); break;
    default: hipLaunchKernelGGL((k_grad<T, 4>), grid, block, 0, st, a); break;
  }
  return hipGetLastError();
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
                           int C, const Tiling& t, int mode, double clip_hi, double clip_lo) {
  FwdArgs<T> a{};
  a.X = (const T*)X; a.Y = (const T*)Y; a.W = (const T*)W; a.b = (const T*)b;
  a.B = B; a.D = D; a.K = K; a.C = C; a.N = C * K; a.CB = t.CB;
  a.mode = mode;
  a.clip_hi = (T)clip_hi; a.clip_lo = (T)clip_lo;
  return a;
}

// ------------------------------------------------------------------ entry points (typed)
template <typename T>
int softmax_grad_t(hmcx_ctx* ctx, const void* X, const void* Y, int B, int D, int K, int C, const void* W,
                   const void* b, double alpha, void* gW, void* gb) {
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
  FwdArgs<T> f = fwd_args<T>(X, Y, W, b, B, D, K, C, t, FWD_GRAD, CLIP_HI, CLIP_LO);
  f.diff = diff; f.colsum_part = csp;
  HMCX_HIP(ctx, launch_fwd<T>(f, t, ctx->stream));
  GradArgs<T> g{};
  g.X = (const T*)X; g.diff = diff; g.colsum_part = csp;
  g.B = B; g.D = D; g.K = K; g.C = C; g.N = N; g.CB = t.CB; g.nRB = t.nRB; g.P = D * K + K;
  g.mode = GRAD_OUT; g.alpha = (T)alpha;
  g.Wsrc = (const T*)W; g.bsrc = (const T*)b; g.gW = (T*)gW; g.gb = (T*)gb;
  HMCX_HIP(ctx, launch_grad<T>(g, t, ctx->stream));
  return HMCX_OK;
}

template <typename T>
int softmax_loglik_t(hmcx_ctx* ctx, const void* X, const void* Y, int B, int D, int K, int C, const void* W,
                     const void* b, double* ll) {
  const Tiling t = make_tiling(B, D, K, C);
  Workspace ws(ctx);
  double* llp;
  do {
    ws.reset();
    llp = ws.take<double>((size_t)t.nRB * C);
  } while (ws.retry());
  if (ws.failed) return HMCX_ENOMEM;
  FwdArgs<T> f = fwd_args<T>(X, Y, W, b, B, D, K, C, t, FWD_LL, CLIP_HI, CLIP_LO);
  f.ll_part = llp;
  HMCX_HIP(ctx, launch_fwd<T>(f, t, ctx->stream));
  hipLaunchKernelGGL(k_reduce_ll, dim3((C + 63) / 64), dim3(64), 0, ctx->stream, llp, t.nRB, C, ll);
  HMCX_HIP(ctx, hipGetLastError());
  return HMCX_OK;
}

template <typename T>
int softmax_predict_t(hmcx_ctx* ctx, const void* X, int B, int D, int K, int C, const void* W, const void* b,
                      void* prob) {
  const Tiling t = make_tiling(B, D, K, C);
  FwdArgs<T> f = fwd_args<T>(X, nullptr, W, b, B, D, K, C, t, FWD_PRED, CLIP_HI, CLIP_LO);
  f.prob = (T*)prob;
  HMCX_HIP(ctx, launch_fwd<T>(f, t, ctx->stream));
  return HMCX_OK;
}

template <typename T>
int sghmc_run_t(hmcx_ctx* ctx, const hmcx_sampler_args* s) {
  const int B = s->B, D = s->D, K = s->K, C = s->C, N = C * K, P = D * K + K;
  const Tiling t = make_tiling(B, D, K, C);
  const size_t nsc = (size_t)s->n_steps * C;
  Workspace ws(ctx);
  T *Wwork, *bwork, *pW, *pb, *p0W, *p0b, *diff, *csp;
  double *ll0, *ll1, *d_u;
  int32_t* d_niter;
  int64_t* d_noff;
  do {
    ws.reset();
    Wwork = ws.take<T>((size_t)D * N);
    bwork = ws.take<T>(N);
    pW = ws.take<T>((size_t)D * N);
    pb = ws.take<T>(N);
    p0W = ws.take<T>((size_t)D * N);
    p0b = ws.take<T>(N);
    diff = ws.take<T>((size_t)B * N);
    csp = ws.take<T>((size_t)t.nRB * N);
    ll0 = ws.take<double>((size_t)t.nRB * C);
    ll1 = ws.take<double>((size_t)t.nRB * C);
    d_niter = ws.take<int32_t>(nsc);
    d_u = ws.take<double>(nsc);
    d_noff = ws.take<int64_t>(nsc);
  } while (ws.retry());
  if (ws.failed) return HMCX_ENOMEM;
  begin_call(ctx);
  // per-call schedule -> device
  int rc = upload(ctx, d_niter, s->n_iter, nsc * sizeof(int32_t));
  if (rc) return rc;
  if ((rc = upload(ctx, d_u, s->u_accept, nsc * sizeof(double)))) return rc;
  if (s->noise_mode == HMCX_NOISE_BUFFER && (rc = upload(ctx, d_noff, s->noise_off, nsc * sizeof(int64_t))))
    return rc;

  const T* X = (const T*)s->X;
  const T* Y = (const T*)s->Y;
  const int init_grid = (int)std::min<long>(1024, ((long)C * P + 255) / 256);
  hipStream_t st = ctx->stream;
  GraphScope gs(ctx);
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
    ia.D = D; ia.K = K; ia.C = C; ia.N = N;
    ia.eps = (T)eps; ia.n_iter = niter;
    ia.noise_mode = s->noise_mode; ia.noise = s->noise; ia.noff = noff;
    ia.seed = s->seed; ia.chain0 = s->chain0; ia.step = step_id;
    ia.W = (const T*)s->W; ia.b = (const T*)s->b;
    ia.Wwork = Wwork; ia.bwork = bwork; ia.pW = pW; ia.pb = pb; ia.p0W = p0W; ia.p0b = p0b;
    hipLaunchKernelGGL((k_sghmc_init<T>), dim3(init_grid), dim3(256), 0, st, ia);
    HMCX_HIP(ctx, hipGetLastError());

    FwdArgs<T> f0 = fwd_args<T>(Xs, Ys, s->W, s->b, B, D, K, C, t, FWD_LL, CLIP_HI, CLIP_LO);
    f0.ll_part = ll0;
    HMCX_HIP(ctx, launch_fwd<T>(f0, t, st));

    FwdArgs<T> f = fwd_args<T>(Xs, Ys, Wwork, bwork, B, D, K, C, t, FWD_SGHMC, CLIP_HI, CLIP_LO);
    f.pb = pb; f.eps = (T)eps; f.n_iter = niter;
    f.diff = diff; f.colsum_part = csp; f.ll_part = ll1;
    GradArgs<T> g{};
    g.X = Xs; g.diff = diff; g.colsum_part = csp;
    g.B = B; g.D = D; g.K = K; g.C = C; g.N = N; g.CB = t.CB; g.nRB = t.nRB; g.P = P;
    g.mode = GRAD_SGHMC;
    g.alpha = (T)s->alpha; g.eps = (T)eps; g.one_minus_eps = (T)(1.0 - eps); g.noise_scale = (T)(2.0 * eps);
    g.n_iter = niter;
    g.W = Wwork; g.b = bwork; g.pW = pW; g.pb = pb;
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
    aa.D = D; aa.K = K; aa.C = C; aa.N = N; aa.nRB = t.nRB;
    aa.n_iter = niter; aa.u = d_u + (size_t)st_i * C;
    aa.neg_inv_n = -1.0 / (double)B; aa.log_prior = s->log_prior;
    aa.p0W = p0W; aa.p0b = p0b; aa.pW = pW; aa.pb = pb;
    aa.ll0_part = ll0; aa.ll1_part = ll1;
    aa.Wwork = Wwork; aa.bwork = bwork; aa.W = (T*)s->W; aa.b = (T*)s->b;
    aa.out_A = s->out_A + (size_t)st_i * C;
    aa.out_acc = s->out_accepted + (size_t)st_i * C;
    aa.out_ll = s->out_ll + (size_t)st_i * C;
    aa.out_E = s->out_E ? s->out_E + (size_t)st_i * C * 2 : nullptr;
    hipLaunchKernelGGL((k_sghmc_accept<T>), dim3(C), dim3(256), 0, st, aa);
    HMCX_HIP(ctx, hipGetLastError());
  }
  return gs.finish();
}

template <typename T>
int sgld_run_t(hmcx_ctx* ctx, const hmcx_sampler_args* s) {
  const int B = s->B, D = s->D, K = s->K, C = s->C, N = C * K, P = D * K + K;
  const Tiling t = make_tiling(B, D, K, C);
  const size_t nsc = (size_t)s->n_steps * C;
  Workspace ws(ctx);
  T *diff, *csp;
  double* llp;
  int64_t* d_noff;
  do {
    ws.reset();
    diff = ws.take<T>((size_t)B * N);
    csp = ws.take<T>((size_t)t.nRB * N);
    llp = ws.take<double>((size_t)t.nRB * C);
    d_noff = ws.take<int64_t>(nsc);
  } while (ws.retry());
  if (ws.failed) return HMCX_ENOMEM;
  begin_call(ctx);
  int rc;
  if (s->noise_mode == HMCX_NOISE_BUFFER && (rc = upload(ctx, d_noff, s->noise_off, nsc * sizeof(int64_t))))
    return rc;
  const T* X = (const T*)s->X;
  const T* Y = (const T*)s->Y;
  hipStream_t st = ctx->stream;
  GraphScope gs(ctx);
  for (int st_i = 0; st_i < s->n_steps; ++st_i) {
    const T* Xs = X + (size_t)s->row0[st_i] * D;
    const T* Ys = Y + (size_t)s->row0[st_i] * K;
    const double eps = s->eps[st_i];
    FwdArgs<T> f = fwd_args<T>(Xs, Ys, s->W, s->b, B, D, K, C, t, FWD_GRAD, CLIP_HI, CLIP_LO);
    f.diff = diff; f.colsum_part = csp;
    HMCX_HIP(ctx, launch_fwd<T>(f, t, st));
    GradArgs<T> g{};
    g.X = Xs; g.diff = diff; g.colsum_part = csp;
    g.B = B; g.D = D; g.K = K; g.C = C; g.N = N; g.CB = t.CB; g.nRB = t.nRB; g.P = P;
    g.mode = GRAD_SGLD;
    g.alpha = (T)s->alpha; g.eps = (T)eps;
    g.noise_scale = (T)(2.0 * eps);                               // sgld.py:43
    g.m_half_eps = (T)(-0.5 * eps);                               // sgld.py:37
    g.W = (T*)s->W; g.b = (T*)s->b;
    g.noise_mode = s->noise_mode; g.noise = s->noise; g.noff = d_noff + (size_t)st_i * C;
    g.seed = s->seed; g.chain0 = s->chain0; g.step = s->step_base + (uint32_t)st_i; g.slot = 0;
    HMCX_HIP(ctx, launch_grad<T>(g, t, st));
    if (s->want_ll && s->want_ll[st_i] && s->out_ll) {
      FwdArgs<T> fl = fwd_args<T>(Xs, Ys, s->W, s->b, B, D, K, C, t, FWD_LL, CLIP_HI, CLIP_LO);
      fl.ll_part = llp;
      HMCX_HIP(ctx, launch_fwd<T>(fl, t, st));
      hipLaunchKernelGGL(k_reduce_ll, dim3((C + 63) / 64), dim3(64), 0, st, llp, t.nRB, C,
                         s->out_ll + (size_t)st_i * C);
      HMCX_HIP(ctx, hipGetLastError());
    }
  }
  return gs.finish();
}

template int softmax_grad_t<float>(hmcx_ctx*, const void*, const void*, int, int, int, int, const void*,
                                   const void*, double, void*, void*);
template int softmax_grad_t<double>(hmcx_ctx*, const void*, const void*, int, int, int, int, const void*,
                                    const void*, double, void*, void*);
template int softmax_loglik_t<float>(hmcx_ctx*, const void*, const void*, int, int, int, int, const void*,
                                     const void*, double*);
template int softmax_loglik_t<double>(hmcx_ctx*, const void*, const void*, int, int, int, int, const void*,
                                      const void*, double*);
template int softmax_predict_t<float>(hmcx_ctx*, const void*, int, int, int, int, const void*, const void*, void*);
template int softmax_predict_t<double>(hmcx_ctx*, const void*, int, int, int, int, const void*, const void*, void*);
template int sghmc_run_t<float>(hmcx_ctx*, const hmcx_sampler_args*);
template int sghmc_run_t<double>(hmcx_ctx*, const hmcx_sampler_args*);
template int sgld_run_t<float>(hmcx_ctx*, const hmcx_sampler_args*);
template int sgld_run_t<double>(hmcx_ctx*, const hmcx_sampler_args*);

}  // namespace hmcx
