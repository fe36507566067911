// hmcx_mlp.hip — the reference's dropout MLP (config 3) on gfx950: gradient, loss and fused SGHMC.
//
// Reference: hamiltonian/models/gpu/mlp.py:19-31 (MyNetwork: relu(dropout(l1 x)) → relu(dropout(l2 ·))
// → l3(dropout(·)), dropout ratio 0.1 in train mode) and :47-82 (grad = ∇ mean softmax-CE + ½αθ,
// log_likelihood returns the mean CE, nlp = loss + log_prior).  Chainer/CuPy are not available, so
// the arithmetic follows the NumPy restatement in oracle/models.py::mlp (parity with injected masks).
//
// Names: a1 = X·W1ᵀ + b1, h1 = max(a1·m0, 0), h2 = max((h1·W2ᵀ + b2)·m1, 0), d3 = h2·m2,
// z = d3·W3ᵀ + b3; m0, m1, m2 are the three dropout masks of one forward ([B][n_mid] each).
//
// Kernels:
//  * k_mm<T, EPI, AOP, BOP>: C = op(A)·op(B) on v_mfma_*_16x16x4, 32x32 output tile per workgroup,
//    K split over its 8 waves (three k chunks in flight per wave, 16-byte vector loads along k for
//    k-contiguous operands, fixed-order LDS combine).
//    Operand transform OP_H1 builds h1 = max(a1·m0, 0) on the fly, so h1 is never stored.  Fused
//    epilogues: bias (a1, logits), layer 2 (bias, dropout, relu, next dropout → h2, d3), layer 3
//    with the softmax cross-entropy (gz = (softmax − onehot)/B and per-row-block loss partials),
//    the two relu/dropout backward gates (ga2, ga1), gradient + prior, and the SGHMC update of one
//    variable (sghmc.py:31,34) which also writes the NEXT iteration's drifted position (sghmc.py:32)
//    into the other half of a double buffer — no separate drift launch.
//  * k_colsum: bias gradients Σ_rows (fixed order) with the same gradient / SGHMC epilogues.
//  * k_mlp_keep: the keep flags of every dropout mask of one SGHMC step (Philox, one launch/step).
//  * k_mlp_init / k_sumsq12 / k_mlp_accept / k_mlp_commit: momentum draw + first drift + energy
//    partials, end-of-trajectory energy partials, MH accept (hmc.py:67-79), commit on accept.
// Per leapfrog iteration at order (W1, b1, W2, b2, W3, b3): 26 launches, ≈1.2 GFLOP at
// 784-256-256-10, B = 500 (layer 1 is recomputed only after W1 or b1 moved).
#include "hmcx_common.h"
#include "hmcx_internal.h"
#include <algorithm>
#include <vector>

namespace hmcx {

// Mask slots live above the noise slots (0 = momentum, it+1 = iteration it) of the same counter space.
constexpr uint32_t MASK_SLOT0 = 0x80000000u;
constexpr int NPART = 32;   // blocks per variable in the energy partial sums

// Dropout masks of one forward: m0, m1, m2 at offsets 0, mn, 2·mn.
template <typename T> struct MaskSrc {
  const T* vals;          // explicit mask values (API / BUFFER mode), or
  const uint8_t* keep;    // keep flags (PHILOX mode): value = keep ? scale : 0;  both null: no dropout
  T scale;
  int mn;
};
template <typename T> __device__ inline T mval(const MaskSrc<T>& s, int which, size_t i) {
  const size_t e = (size_t)which * s.mn + i;
  if (s.vals) return s.vals[e];
  if (s.keep) return s.keep[e] ? s.scale : T(0);
  return T(1);
}

__device__ inline bool keep_flag(uint32_t w) {                // Chainer dropout: keep iff u >= ratio
  return (float)(w >> 8) * 5.9604644775390625e-08f >= 0.1f;
}

enum MMEpi { MM_BIAS = 0, MM_L2 = 1, MM_L3CE = 2, MM_GA2 = 3, MM_GA1 = 4, MM_GRAD = 5, MM_SGHMC = 6 };
enum MMOp { OP_PLAIN = 0, OP_H1 = 1 };

template <typename T> struct MMArgs {
  int M, N, K;
  const T* A; int lda, ta;           // A(m,k) = ta ? A[k·lda + m] : A[m·lda + k]
  const T* B; int ldb, tb;           // B(k,n) = tb ? B[n·ldb + k] : B[k·ldb + n]
  T* C; int ldc;                     // output [M][ldc]
  const T* bias;                     // [N]
  MaskSrc<T> ms;
  const T* H;                        // GA2: h2, GA1: a1 (the relu gate)
  T* C2;                             // L2: d3
  double* lpart;                     // L3CE: Σ −log p[label] of each 32-row block
  const int32_t* y;                  // L3CE: labels
  const T* W; T* P; T* Qn;           // GRAD/SGHMC: θ of the variable, momentum, next drifted θ
  T half_alpha, eps, one_minus_eps, noise_scale;
  int noise_mode; const double* noise;
  uint64_t seed; uint32_t chain, step, slot, e0;
};

template <typename T, int EPI>
__device__ inline void mm_epilogue(const MMArgs<T>& a, int m, int n, T v) {
  const size_t i = (size_t)m * a.ldc + n;
  if constexpr (EPI == MM_BIAS) {
    a.C[i] = v + a.bias[n];
  } else if constexpr (EPI == MM_L2) {                          // mlp.py:30-31
    const T t = (v + a.bias[n]) * mval(a.ms, 1, i);
    const T h = t > T(0) ? t : T(0);
    a.C[i] = h;
    a.C2[i] = h * mval(a.ms, 2, i);
  } else if constexpr (EPI == MM_GA2) {                         // ((gz·W3)·m2)·[h2>0]·m1
    T t = v * mval(a.ms, 2, i);
    t = t * (a.H[i] > T(0) ? T(1) : T(0));
    a.C[i] = t * mval(a.ms, 1, i);
  } else if constexpr (EPI == MM_GA1) {                         // (ga2·W2)·[a1·m0>0]·m0
    const T m0 = mval(a.ms, 0, i);
    a.C[i] = (v * (a.H[i] * m0 > T(0) ? T(1) : T(0))) * m0;
  } else if constexpr (EPI == MM_GRAD) {                        // mlp.py:63 grad + ½αθ
    a.C[i] = v + a.half_alpha * a.W[i];
  } else if constexpr (EPI == MM_SGHMC) {                       // sghmc.py:31-34
    const T g = v + a.half_alpha * a.W[i];
    const T z = a.noise_mode == HMCX_NOISE_BUFFER ? (T)a.noise[i]
                                                  : (T)philox_normal(a.seed, a.chain, a.step, a.slot, a.e0 + (uint32_t)i);
    const T p = (a.one_minus_eps * a.P[i] + a.eps * g) + a.noise_scale * z;
    a.P[i] = p;
    if (a.Qn) a.Qn[i] = a.W[i] + a.eps * p;
  }
}

// Softmax cross-entropy of the rows of one 32-row block held in LDS (F.softmax_cross_entropy, mean):
// gz = (softmax − onehot)/B, lpart[block] = Σ_rows −log p[label] (fixed order).
template <typename T>
__device__ inline void ce_rows(T (*zt)[33], double* rowl, int m0, int M, int N, const int32_t* y, T* gz, int ldg,
                               double* lpart, int blk) {
  const int t = threadIdx.x;
  if (t < 32) {
    const int m = m0 + t;
    double l = 0.0;
    if (m < M) {
      T mx = zt[t][0];
      for (int k = 1; k < N; ++k) mx = zt[t][k] > mx ? zt[t][k] : mx;
      T s = T(0);
      for (int k = 0; k < N; ++k) s += exp(zt[t][k] - mx);
      const T ls = log(s);
      const int lab = y[m];
      l = -(double)((zt[t][lab] - mx) - ls);
      for (int k = 0; k < N; ++k) {
        T g = exp((zt[t][k] - mx) - ls);
        if (k == lab) g -= T(1);
        gz[(size_t)m * ldg + k] = g / (T)M;
      }
    }
    rowl[t] = l;
  }
  __syncthreads();
  if (t == 0) {
    double s = 0.0;
    for (int r = 0; r < 32; ++r) s += rowl[r];
    lpart[blk] = s;
  }
}

// k offset, inside a 16-wide k chunk, of MFMA step u (0..3) for lane group lg: each lane's k values
// are contiguous (4 floats / 2+2 doubles), so a k-contiguous operand is one or two 16-byte loads.
template <typename T> __device__ inline int kmap(int u, int lg);
template <> __device__ inline int kmap<float>(int u, int lg) { return 4 * lg + u; }
template <> __device__ inline int kmap<double>(int u, int lg) { return ((u >> 1) << 3) + 2 * lg + (u & 1); }

template <typename T, int OP>
__device__ inline T op_apply(T x, size_t idx, const MaskSrc<T>& ms) {
  if constexpr (OP == OP_H1) {
    const T t = x * mval(ms, 0, idx);
    return t > T(0) ? t : T(0);
  }
  return x;
}

// Operand values of one 16-k chunk for rows (A) / columns (B) r0 + 16·i + lr, i = 0, 1:
// x[u][i] = Op(r, k0 + kmap(u, lg)).  TR: element (r, k) at P[k·ld + r], else P[r·ld + k].
// VEC (requires !TR, ld % (16/sizeof T) == 0 and a 16-byte aligned P): 16-byte vector loads along k.
template <typename T, int OP, int TR, int VEC>
__device__ inline void load_chunk(T (&x)[4][2], const T* P, int ld, int r0, int R, int k0, int ke, int lr, int lg,
                                  const MaskSrc<T>& ms) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = r0 + 16 * i + lr;
    const bool rok = r < R;
    if constexpr (VEC) {
      constexpr int V = 16 / sizeof(T);
#pragma unroll
      for (int h = 0; h < 4 / V; ++h) {                        // f32: one float4; f64: two double2
        const int kv = k0 + (sizeof(T) == 8 ? 8 * h + 2 * lg : 4 * lg);
        const size_t base = (size_t)r * ld + kv;
        if (rok && kv + V <= ke) {
          if constexpr (V == 4) {
            const float4 v = *reinterpret_cast<const float4*>(P + base);
            x[0][i] = op_apply<T, OP>(v.x, base, ms); x[1][i] = op_apply<T, OP>(v.y, base + 1, ms);
            x[2][i] = op_apply<T, OP>(v.z, base + 2, ms); x[3][i] = op_apply<T, OP>(v.w, base + 3, ms);
          } else {
            const double2 v = *reinterpret_cast<const double2*>(P + base);
            x[2 * h][i] = op_apply<T, OP>(v.x, base, ms);
            x[2 * h + 1][i] = op_apply<T, OP>(v.y, base + 1, ms);
          }
        } else {
#pragma unroll
          for (int q = 0; q < V; ++q)
            x[h * V + q][i] = (rok && kv + q < ke) ? op_apply<T, OP>(P[base + q], base + q, ms) : T(0);
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = k0 + kmap<T>(u, lg);
        const size_t idx = TR ? (size_t)k * ld + r : (size_t)r * ld + k;
        x[u][i] = (rok && k < ke) ? op_apply<T, OP>(P[idx], idx, ms) : T(0);
      }
    }
  }
}

constexpr int MM_NW = 8;   // waves per workgroup; the K range is split over them

template <typename T, int EPI, int AOP, int BOP, int TA, int TB, int AV, int BV>
__global__ __launch_bounds__(MM_NW * 64) void k_mm(MMArgs<T> a) {
  using M = mfma16<T>;
  __shared__ T red[MM_NW][32][33];
  __shared__ double rowl[32];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  const int m0 = blockIdx.x * 32, n0 = blockIdx.y * 32;
  const int Kq = ((a.K + 16 * MM_NW - 1) / (16 * MM_NW)) * 16;   // k range per wave (multiple of 16)
  const int kb = wave * Kq, ke = min(a.K, kb + Kq);
  typename M::acc_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = M::zero();
  // three chunks in flight (register ring), then one MFMA batch per chunk
  T av[3][4][2], bv[3][4][2];
  auto load = [&](int s, int k0) {
    load_chunk<T, AOP, TA, AV>(av[s], a.A, a.lda, m0, a.M, k0, ke, lr, lg, a.ms);
    load_chunk<T, BOP, !TB, BV>(bv[s], a.B, a.ldb, n0, a.N, k0, ke, lr, lg, a.ms);
  };
  auto mfma = [&](int s) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = M::fma(av[s][u][i], bv[s][u][j], acc[i][j]);
  };
  if (kb < ke) load(0, kb);
  if (kb + 16 < ke) load(1, kb + 16);
  if (kb + 32 < ke) load(2, kb + 32);
  for (int k0 = kb; k0 < ke; k0 += 48) {
    mfma(0);
    if (k0 + 48 < ke) load(0, k0 + 48);
    if (k0 + 16 < ke) {
      mfma(1);
      if (k0 + 64 < ke) load(1, k0 + 64);
    }
    if (k0 + 32 < ke) {
      mfma(2);
      if (k0 + 80 < ke) load(2, k0 + 80);
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) red[wave][16 * i + M::row(lane, q)][16 * j + lr] = acc[i][j][q];
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 1024 / (MM_NW * 64); ++u) {
    const int e = tid + MM_NW * 64 * u, mm = e >> 5, nn = e & 31;
    const int m = m0 + mm, n = n0 + nn;
    T v = red[0][mm][nn];
#pragma unroll
    for (int w = 1; w < MM_NW; ++w) v += red[w][mm][nn];
    if constexpr (EPI == MM_L3CE) {
      red[0][mm][nn] = (n < a.N) ? v + a.bias[n] : T(0);     // logits of the block (one writer each)
    } else {
      if (m < a.M && n < a.N) mm_epilogue<T, EPI>(a, m, n, v);
    }
  }
  if constexpr (EPI == MM_L3CE) {
    __syncthreads();
    ce_rows<T>(red[0], rowl, m0, a.M, a.N, a.y, a.C, a.ldc, a.lpart, blockIdx.x);
  }
}

// Cross-entropy for n_out > 32 (logits z already stored): one 32-row block per workgroup.
template <typename T>
__global__ __launch_bounds__(256) void k_mlp_ce(const T* z, const int32_t* y, int B, int K, T* gz, double* lpart) {
  __shared__ double rowl[32];
  const int t = threadIdx.x, m0 = blockIdx.x * 32;
  if (t < 32) {
    const int m = m0 + t;
    double l = 0.0;
    if (m < B) {
      const T* zr = z + (size_t)m * K;
      T mx = zr[0];
      for (int k = 1; k < K; ++k) mx = zr[k] > mx ? zr[k] : mx;
      T s = T(0);
      for (int k = 0; k < K; ++k) s += exp(zr[k] - mx);
      const T ls = log(s);
      const int lab = y[m];
      l = -(double)((zr[lab] - mx) - ls);
      for (int k = 0; k < K; ++k) {
        T g = exp((zr[k] - mx) - ls);
        if (k == lab) g -= T(1);
        gz[(size_t)m * K + k] = g / (T)B;
      }
    }
    rowl[t] = l;
  }
  __syncthreads();
  if (t == 0) {
    double s = 0.0;
    for (int r = 0; r < 32; ++r) s += rowl[r];
    lpart[blockIdx.x] = s;
  }
}

// Bias gradient Σ_rows g[m][n] (rows split over 8 groups, fixed combine order) + epilogue at (0, n).
template <typename T, int EPI>
__global__ __launch_bounds__(256) void k_colsum(const T* g, int rows, int N, MMArgs<T> a) {
  __shared__ T part[8][32];
  const int c = threadIdx.x & 31, grp = threadIdx.x >> 5, n = blockIdx.x * 32 + c;
  T s = T(0);
  if (n < N) {
#pragma unroll 4
    for (int m = grp; m < rows; m += 8) s += g[(size_t)m * N + n];
  }
  part[grp][c] = s;
  __syncthreads();
  if (grp == 0 && n < N) {
    T t = part[0][c];
#pragma unroll
    for (int j = 1; j < 8; ++j) t += part[j][c];
    mm_epilogue<T, EPI>(a, 0, n, t);
  }
}

// Keep flags of F forwards (blockIdx.y = forward f, Philox slot MASK_SLOT0 + f), 3·mn per forward.
__global__ void k_mlp_keep(uint8_t* keep, int n3, uint64_t seed, uint32_t chain, uint32_t step) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x, f = blockIdx.y;
  if (4 * g >= n3) return;
  u32x4 c = {{(uint32_t)g, MASK_SLOT0 + (uint32_t)f, step, chain}};
  const u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  uint8_t* out = keep + (size_t)f * n3;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (4 * g + q < n3) out[4 * g + q] = keep_flag(r.v[q]) ? 1 : 0;
}

// Mask values of one forward (the API twin of k_mlp_keep: same counters, value = keep·(1/0.9)).
template <typename T>
__global__ void k_mlp_masks(T* masks, int n3, uint64_t seed, uint32_t chain, uint32_t step, uint32_t slot) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (4 * g >= n3) return;
  u32x4 c = {{(uint32_t)g, slot, step, chain}};
  const u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const T scale = (T)(1.0 / 0.9);
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (4 * g + q < n3) masks[4 * g + q] = keep_flag(r.v[q]) ? scale : T(0);
}

// Six variables in the caller's order (position i of `order`).
struct VarTab {
  void* q[6]; void* qn[6]; void* p[6];
  int n[6], e0[6];
};

__device__ inline void block_sum2(double a, double b, double* out_a, double* out_b) {
  __shared__ double sa[256], sb[256];
  const int t = threadIdx.x;
  sa[t] = a;
  sb[t] = b;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) { sa[t] += sa[t + w]; sb[t] += sb[t + w]; }
    __syncthreads();
  }
  if (t == 0) { *out_a = sa[0]; if (out_b) *out_b = sb[0]; }
}

// Momentum draw (hmc.py:82-87) + first drift q' = q + ε·p + partials of Σp², Σq² (part [2][6][NPART]).
template <typename T>
__global__ __launch_bounds__(256) void k_mlp_init(VarTab vt, T eps, int drift, int noise_mode, const double* noise,
                                                  uint64_t seed, uint32_t chain, uint32_t step, double* part) {
  const int v = blockIdx.y, n = vt.n[v];
  const T* q = (const T*)vt.q[v];
  T* qn = (T*)vt.qn[v];
  T* p = (T*)vt.p[v];
  double sp = 0.0, sq = 0.0;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += NPART * 256) {
    const uint32_t e = (uint32_t)(vt.e0[v] + i);
    const T z = noise_mode == HMCX_NOISE_BUFFER ? (T)noise[e] : (T)philox_normal(seed, chain, step, 0u, e);
    const T qv = q[i];
    p[i] = z;
    if (drift) qn[i] = qv + eps * z;
    sp += (double)z * (double)z;
    sq += (double)qv * (double)qv;
  }
  block_sum2(sp, sq, part + v * NPART + blockIdx.x, part + (6 + v) * NPART + blockIdx.x);
}

// End-of-trajectory partials: part[0][i] = Σp², part[1][i] = Σq² per variable (same layout as init).
template <typename T>
__global__ __launch_bounds__(256) void k_sumsq12(VarTab vt, double* part) {
  const int v = blockIdx.y, n = vt.n[v];
  const T* q = (const T*)vt.q[v];
  const T* p = (const T*)vt.p[v];
  double sp = 0.0, sq = 0.0;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += NPART * 256) {
    const double pv = (double)p[i], qv = (double)q[i];
    sp += pv * pv;
    sq += qv * qv;
  }
  block_sum2(sp, sq, part + v * NPART + blockIdx.x, part + (6 + v) * NPART + blockIdx.x);
}

// MH accept (hmc.py:67-79): E = nlp + ½Σp², nlp = loss + log_prior, log_prior = −Σ_v ½α·Σθ²/dim.
struct MlpAccept {
  const double* part_cur; const double* part_new;   // [2][6][NPART]
  const double* lp_cur; const double* lp_new;       // loss partials [nlb]
  int nlb, B;
  int dim[6];
  double alpha, u;
  double* out_A; int32_t* out_acc; double* out_loss; double* out_nlp; double* out_E;
  int32_t* acc_flag;
};
// One workgroup of 26 × 32 threads: group g < 24 sums the NPART partials of (state g/12, kind, variable),
// groups 24/25 the loss partials of the current / proposed state — each by a fixed-order tree.
__global__ __launch_bounds__(1024) void k_mlp_accept(MlpAccept a) {
  __shared__ double sh[26][32];
  const int t = threadIdx.x, g = t >> 5, j = t & 31;
  double x = 0.0;
  if (g < 24) {
    x = (g < 12 ? a.part_cur : a.part_new)[(g % 12) * NPART + j];
  } else if (g < 26) {
    const double* lp = g == 24 ? a.lp_cur : a.lp_new;
    for (int b = j; b < a.nlb; b += 32) x += lp[b];
  }
  if (g < 26) sh[g][j] = x;
  __syncthreads();
  for (int w = 16; w > 0; w >>= 1) {
    if (g < 26 && j < w) sh[g][j] += sh[g][j + w];
    __syncthreads();
  }
  if (t != 0) return;
  const double lc = sh[24][0] / (double)a.B, ln = sh[25][0] / (double)a.B;
  double pri_c = 0.0, pri_n = 0.0, kc = 0.0, kn = 0.0;
  for (int v = 0; v < 6; ++v) {                                // variables in the caller's order
    pri_c -= 0.5 * a.alpha * sh[6 + v][0] / (double)a.dim[v];
    pri_n -= 0.5 * a.alpha * sh[18 + v][0] / (double)a.dim[v];
    kc += 0.5 * sh[v][0];
    kn += 0.5 * sh[12 + v][0];
  }
  const double Enew = (ln + pri_n) + kn;
  const double Ecur = (lc + pri_c) + kc;
  const double e = exp(Ecur - Enew);
  const double A = (e < 1.0) ? e : 1.0;                       // Python min(1, x)
  const int acc = (A == A) && (A - A == 0.0) && a.u < A;      // isfinite(A) and u < A
  *a.out_A = A;
  *a.out_acc = acc;
  *a.out_loss = acc ? ln : lc;
  if (a.out_nlp) *a.out_nlp = acc ? (ln + pri_n) : (lc + pri_c);
  if (a.out_E) { a.out_E[0] = Ecur; a.out_E[1] = Enew; }
  *a.acc_flag = acc;
}

// state ← proposal where accepted
template <typename T>
__global__ void k_mlp_commit(VarTab vt, const int32_t* acc) {
  const int v = blockIdx.y, n = vt.n[v];
  if (!*acc || vt.q[v] == vt.qn[v]) return;
  const T* src = (const T*)vt.q[v];
  T* dst = (T*)vt.qn[v];
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) dst[i] = src[i];
}

__global__ void k_loss_final(const double* lpart, int nlb, int B, double* out) {
  double s = 0.0;
  for (int b = 0; b < nlb; ++b) s += lpart[b];
  *out = s / (double)B;
}

// ------------------------------------------------------------------ host side
namespace {

template <typename T>
struct MlpNet {
  int B, n_in, n_mid, n_out, nlb;
  const T* X; const int32_t* y;
  T *a1, *h2, *d3, *z, *gz, *ga2, *ga1;
  hipStream_t st;
  bool a1_valid = false;
  int nvar(int v) const {
    switch (v) {
      case 0: return n_mid * n_in;  case 1: return n_mid;
      case 2: return n_mid * n_mid; case 3: return n_mid;
      case 4: return n_out * n_mid; default: return n_out;
    }
  }
};

inline bool vec_ok(const void* p, int ld, int elt) {
  return ((uintptr_t)p % 16 == 0) && ((size_t)ld * elt) % 16 == 0;
}

// Launch k_mm for a call site with compile-time operand layouts (TA: A stored [K][M], TB: B stored
// [N][K]); k-contiguous operands take the 16-byte vector path when aligned.
template <typename T, int EPI, int TA, int TB, int AOP = OP_PLAIN, int BOP = OP_PLAIN>
hipError_t mm(const MMArgs<T>& a, hipStream_t st) {
  if (a.ta != TA || a.tb != TB) return hipErrorInvalidValue;
  dim3 grid((a.M + 31) / 32, (a.N + 31) / 32), blk(MM_NW * 64);
  const bool av = !TA && vec_ok(a.A, a.lda, sizeof(T)), bv = TB && vec_ok(a.B, a.ldb, sizeof(T));
  if (av && bv) hipLaunchKernelGGL((k_mm<T, EPI, AOP, BOP, TA, TB, !TA, TB>), grid, blk, 0, st, a);
  else if (av) hipLaunchKernelGGL((k_mm<T, EPI, AOP, BOP, TA, TB, !TA, 0>), grid, blk, 0, st, a);
  else if (bv) hipLaunchKernelGGL((k_mm<T, EPI, AOP, BOP, TA, TB, 0, TB>), grid, blk, 0, st, a);
  else hipLaunchKernelGGL((k_mm<T, EPI, AOP, BOP, TA, TB, 0, 0>), grid, blk, 0, st, a);
  return hipGetLastError();
}

template <typename T>
void mm_set(MMArgs<T>& a, int M, int N, int K, const T* A, int lda, int ta, const T* B, int ldb, int tb, T* C, int ldc) {
  a.M = M; a.N = N; a.K = K; a.A = A; a.lda = lda; a.ta = ta; a.B = B; a.ldb = ldb; a.tb = tb; a.C = C; a.ldc = ldc;
}

// Forward with masks `ms` at parameters q; loss partials into lpart.  Layer 1 only when a1 is stale.
template <typename T>
hipError_t mlp_forward(MlpNet<T>& net, T* const* q, const MaskSrc<T>& ms, double* lpart, T* logits = nullptr) {
  const int B = net.B, nm = net.n_mid;
  hipError_t e;
  if (!net.a1_valid) {                                        // a1 = X·W1ᵀ + b1
    MMArgs<T> a{};
    mm_set<T>(a, B, nm, net.n_in, net.X, net.n_in, 0, q[0], net.n_in, 1, net.a1, nm);
    a.bias = q[1];
    if ((e = mm<T, MM_BIAS, 0, 1>(a, net.st))) return e;
    net.a1_valid = true;
  }
  {                                                           // h2, d3 from h1 = max(a1·m0, 0) on the fly
    MMArgs<T> a{};
    mm_set<T>(a, B, nm, nm, net.a1, nm, 0, q[2], nm, 1, net.h2, nm);
    a.bias = q[3]; a.ms = ms; a.C2 = net.d3;
    if ((e = mm<T, MM_L2, 0, 1, OP_H1>(a, net.st))) return e;
  }
  if (logits) {
    MMArgs<T> a{};
    mm_set<T>(a, B, net.n_out, nm, net.d3, nm, 0, q[4], nm, 1, logits, net.n_out);
    a.bias = q[5];
    if ((e = mm<T, MM_BIAS, 0, 1>(a, net.st))) return e;
  }
  if (!lpart) return hipSuccess;
  MMArgs<T> a{};
  if (net.n_out <= 32) {                                      // z and the cross-entropy in one kernel
    mm_set<T>(a, B, net.n_out, nm, net.d3, nm, 0, q[4], nm, 1, net.gz, net.n_out);
    a.bias = q[5]; a.y = net.y; a.lpart = lpart;
    return mm<T, MM_L3CE, 0, 1>(a, net.st);
  }
  mm_set<T>(a, B, net.n_out, nm, net.d3, nm, 0, q[4], nm, 1, net.z, net.n_out);
  a.bias = q[5];
  if ((e = mm<T, MM_BIAS, 0, 1>(a, net.st))) return e;
  hipLaunchKernelGGL(k_mlp_ce<T>, dim3(net.nlb), dim3(256), 0, net.st, net.z, net.y, B, net.n_out, net.gz, lpart);
  return hipGetLastError();
}

template <typename T>
hipError_t mlp_ga2(MlpNet<T>& net, T* const* q, const MaskSrc<T>& ms) {
  MMArgs<T> a{};
  mm_set<T>(a, net.B, net.n_mid, net.n_out, net.gz, net.n_out, 0, q[4], net.n_mid, 0, net.ga2, net.n_mid);
  a.ms = ms; a.H = net.h2;
  return mm<T, MM_GA2, 0, 0>(a, net.st);
}
template <typename T>
hipError_t mlp_ga1(MlpNet<T>& net, T* const* q, const MaskSrc<T>& ms) {
  MMArgs<T> a{};
  mm_set<T>(a, net.B, net.n_mid, net.n_mid, net.ga2, net.n_mid, 0, q[2], net.n_mid, 0, net.ga1, net.n_mid);
  a.ms = ms; a.H = net.a1;
  return mm<T, MM_GA1, 0, 0>(a, net.st);
}

// Gradient of variable v into the epilogue `a` (GRAD: a.C = output; SGHMC: a.P / a.Qn / noise).
template <typename T, int EPI>
hipError_t mlp_var_grad(MlpNet<T>& net, const MaskSrc<T>& ms, int v, MMArgs<T> a) {
  const int B = net.B, nm = net.n_mid;
  T* out = a.C;
  switch (v) {
    case 4: mm_set<T>(a, net.n_out, nm, B, net.gz, net.n_out, 1, net.d3, nm, 0, out, nm);      // gzᵀ·d3
            return mm<T, EPI, 1, 0>(a, net.st);
    case 2: mm_set<T>(a, nm, nm, B, net.ga2, nm, 1, net.a1, nm, 0, out, nm);                   // ga2ᵀ·h1
            a.ms = ms;
            return mm<T, EPI, 1, 0, OP_PLAIN, OP_H1>(a, net.st);
    case 0: mm_set<T>(a, nm, net.n_in, B, net.ga1, nm, 1, net.X, net.n_in, 0, out, net.n_in);  // ga1ᵀ·X
            return mm<T, EPI, 1, 0>(a, net.st);
    default: {                                                 // biases: Σ_rows of gz / ga2 / ga1
      const T* g = v == 5 ? net.gz : (v == 3 ? net.ga2 : net.ga1);
      const int N = v == 5 ? net.n_out : nm;
      a.ldc = N;
      hipLaunchKernelGGL((k_colsum<T, EPI>), dim3((N + 31) / 32), dim3(256), 0, net.st, g, B, N, a);
      return hipGetLastError();
    }
  }
}

template <typename T>
void mlp_workspace(Workspace& ws, MlpNet<T>& net) {
  const size_t mn = (size_t)net.B * net.n_mid;
  net.a1 = ws.take<T>(mn); net.h2 = ws.take<T>(mn); net.d3 = ws.take<T>(mn);
  net.ga2 = ws.take<T>(mn); net.ga1 = ws.take<T>(mn);
  net.z = ws.take<T>((size_t)net.B * net.n_out); net.gz = ws.take<T>((size_t)net.B * net.n_out);
}

}  // namespace

template <typename T>
int mlp_masks_t(hmcx_ctx* ctx, int B, int n_mid, uint64_t seed, uint32_t chain, uint32_t step, uint32_t slot,
                void* out) {
  const int n3 = 3 * B * n_mid;
  hipLaunchKernelGGL(k_mlp_masks<T>, dim3((unsigned)(((n3 + 3) / 4 + 255) / 256)), dim3(256), 0, ctx->stream,
                     (T*)out, n3, seed, chain, step, slot);
  HMCX_HIP(ctx, hipGetLastError());
  return HMCX_OK;
}

template <typename T>
int mlp_grad_t(hmcx_ctx* ctx, const void* X, const int32_t* y, int B, int n_in, int n_mid, int n_out,
               const hmcx_mlp_params* par, const void* masks, double alpha, hmcx_mlp_params* grads, double* loss) {
  MlpNet<T> net{};
  net.B = B; net.n_in = n_in; net.n_mid = n_mid; net.n_out = n_out; net.nlb = (B + 31) / 32;
  net.X = (const T*)X; net.y = y; net.st = ctx->stream;
  Workspace ws(ctx);
  double* lpart;
  do { ws.reset(); mlp_workspace<T>(ws, net); lpart = ws.take<double>(net.nlb); } while (ws.retry());
  if (ws.failed) return HMCX_ENOMEM;
  const MaskSrc<T> ms{(const T*)masks, nullptr, T(1), B * n_mid};
  T* q[6];
  for (int v = 0; v < 6; ++v) q[v] = (T*)par->p[v];
  HMCX_HIP(ctx, mlp_forward<T>(net, q, ms, lpart));
  HMCX_HIP(ctx, mlp_ga2<T>(net, q, ms));
  HMCX_HIP(ctx, mlp_ga1<T>(net, q, ms));
  MMArgs<T> a{};
  a.half_alpha = (T)(0.5 * alpha);
  for (int v = 0; v < 6; ++v) {
    a.C = (T*)grads->p[v];
    a.W = q[v];
    HMCX_HIP(ctx, (mlp_var_grad<T, MM_GRAD>(net, ms, v, a)));
  }
  if (loss) {
    hipLaunchKernelGGL(k_loss_final, dim3(1), dim3(1), 0, ctx->stream, lpart, net.nlb, B, loss);
    HMCX_HIP(ctx, hipGetLastError());
  }
  return HMCX_OK;
}

template <typename T>
int mlp_loss_t(hmcx_ctx* ctx, const void* X, const int32_t* y, int B, int n_in, int n_mid, int n_out,
               const hmcx_mlp_params* par, const void* masks, double* loss, void* logits) {
  MlpNet<T> net{};
  net.B = B; net.n_in = n_in; net.n_mid = n_mid; net.n_out = n_out; net.nlb = (B + 31) / 32;
  net.X = (const T*)X; net.y = y; net.st = ctx->stream;
  Workspace ws(ctx);
  double* lpart;
  do { ws.reset(); mlp_workspace<T>(ws, net); lpart = ws.take<double>(net.nlb); } while (ws.retry());
  if (ws.failed) return HMCX_ENOMEM;
  const MaskSrc<T> ms{(const T*)masks, nullptr, T(1), B * n_mid};
  T* q[6];
  for (int v = 0; v < 6; ++v) q[v] = (T*)par->p[v];
  HMCX_HIP(ctx, mlp_forward<T>(net, q, ms, y ? lpart : nullptr, (T*)logits));
  if (y && loss) {
    hipLaunchKernelGGL(k_loss_final, dim3(1), dim3(1), 0, ctx->stream, lpart, net.nlb, B, loss);
    HMCX_HIP(ctx, hipGetLastError());
  }
  return HMCX_OK;
}

template <typename T>
int mlp_sghmc_t(hmcx_ctx* ctx, const hmcx_mlp_sghmc_args* s) {
  MlpNet<T> net{};
  net.B = s->B; net.n_in = s->n_in; net.n_mid = s->n_mid; net.n_out = s->n_out; net.st = ctx->stream;
  net.nlb = (s->B + 31) / 32;
  const int mn = s->B * s->n_mid, n3 = 3 * mn;
  int off_v[6], dim[6], P = 0;                                // element offset of each variable in `order`
  for (int i = 0; i < 6; ++i) {
    const int v = s->order[i];
    if (v < 0 || v > 5) return set_error(ctx, HMCX_EINVAL, "mlp sghmc: order must be a permutation of 0..5");
    off_v[v] = P;
    dim[v] = net.nvar(v);
    P += dim[v];
  }
  {
    int seen = 0;
    for (int i = 0; i < 6; ++i) seen |= 1 << s->order[i];
    if (seen != 63) return set_error(ctx, HMCX_EINVAL, "mlp sghmc: order must be a permutation of 0..5");
  }
  int maxF = 2;
  for (int si = 0; si < s->n_steps; ++si) {
    if (s->n_iter[si] < 0) return set_error(ctx, HMCX_EINVAL, "mlp sghmc: n_iter < 0");
    maxF = std::max(maxF, 6 * s->n_iter[si] + 2);
  }
  const bool philox_masks = s->mask_mode == HMCX_NOISE_PHILOX;
  Workspace ws(ctx);
  T *pv[6], *qa[6], *qb[6];
  double *part_cur, *part_new, *lp_cur, *lp_new, *lp_scr;
  uint8_t* keep = nullptr;
  int32_t* accf;
  do {
    ws.reset();
    mlp_workspace<T>(ws, net);
    for (int v = 0; v < 6; ++v) { pv[v] = ws.take<T>(dim[v]); qa[v] = ws.take<T>(dim[v]); qb[v] = ws.take<T>(dim[v]); }
    part_cur = ws.take<double>(12 * NPART);
    part_new = ws.take<double>(12 * NPART);
    lp_cur = ws.take<double>(net.nlb);
    lp_new = ws.take<double>(net.nlb);
    lp_scr = ws.take<double>(net.nlb);
    if (philox_masks) keep = ws.take<uint8_t>((size_t)maxF * n3);
    accf = ws.take<int32_t>(1);
  } while (ws.retry());
  if (ws.failed) return HMCX_ENOMEM;
  begin_call(ctx);
  int rc = timing_begin(ctx, ctx->stream);
  if (rc) return rc;
  GraphScope gs(ctx);
  hipStream_t st = ctx->stream;
  net.st = st;
  T* par[6];
  for (int v = 0; v < 6; ++v) par[v] = (T*)s->par.p[v];
  const T* Xall = (const T*)s->X;
  const T scale = (T)(1.0 / 0.9);

  for (int si = 0; si < s->n_steps; ++si) {
    net.X = Xall + (size_t)s->row0[si] * s->n_in;
    net.y = s->y + s->row0[si];
    net.a1_valid = false;
    const double eps = s->eps[si];
    const int n = s->n_iter[si], F = 6 * n + 2;
    const uint32_t step_id = s->step_base + (uint32_t)si;
    const double* nz = s->noise_mode == HMCX_NOISE_BUFFER ? s->noise + s->noise_off[si] : nullptr;
    if (philox_masks) {
      hipLaunchKernelGGL(k_mlp_keep, dim3((unsigned)(((n3 + 3) / 4 + 255) / 256), (unsigned)F), dim3(256), 0, st, keep,
                         n3, s->seed, s->chain, step_id);
    }
    auto masks_for = [&](int f) -> MaskSrc<T> {
      if (philox_masks) return MaskSrc<T>{nullptr, keep + (size_t)f * n3, scale, mn};
      return MaskSrc<T>{(const T*)s->masks + s->mask_off[si] + (size_t)f * n3, nullptr, scale, mn};
    };
    // momentum (hmc.py:82-87), first drift into qa, Σp², Σθ² of the current state
    VarTab vt{};
    for (int i = 0; i < 6; ++i) {
      const int v = s->order[i];
      vt.q[i] = par[v]; vt.qn[i] = qa[v]; vt.p[i] = pv[v]; vt.n[i] = dim[v]; vt.e0[i] = off_v[v];
    }
    hipLaunchKernelGGL(k_mlp_init<T>, dim3(NPART, 6), dim3(256), 0, st, vt, (T)eps, n > 0 ? 1 : 0, s->noise_mode,
                       nz, s->seed, s->chain, step_id, part_cur);
    T* cur[6];
    for (int v = 0; v < 6; ++v) cur[v] = par[v];
    int fwd = 0;
    for (int it = 0; it < n; ++it) {
      for (int i = 0; i < 6; ++i) {
        const int v = s->order[i];
        cur[v] = (it & 1) ? qb[v] : qa[v];                    // drifted position of this iteration
        if (v <= 1) net.a1_valid = false;
        const MaskSrc<T> ms = masks_for(fwd++);
        HMCX_HIP(ctx, mlp_forward<T>(net, cur, ms, lp_scr));
        if (v <= 3) HMCX_HIP(ctx, mlp_ga2<T>(net, cur, ms));
        if (v <= 1) HMCX_HIP(ctx, mlp_ga1<T>(net, cur, ms));
        MMArgs<T> a{};
        a.W = cur[v]; a.P = pv[v];
        a.Qn = it + 1 < n ? ((it & 1) ? qa[v] : qb[v]) : nullptr;
        a.half_alpha = (T)(0.5 * s->alpha); a.eps = (T)eps; a.one_minus_eps = (T)(1.0 - eps);
        a.noise_scale = (T)(2.0 * eps);
        a.noise_mode = s->noise_mode;
        a.noise = nz ? nz + (size_t)P * (it + 1) + off_v[v] : nullptr;   // BUFFER: one block of P per iteration
        a.seed = s->seed; a.chain = s->chain; a.step = step_id; a.slot = (uint32_t)(it + 1);
        a.e0 = (uint32_t)off_v[v];
        HMCX_HIP(ctx, (mlp_var_grad<T, MM_SGHMC>(net, ms, v, a)));
      }
    }
    // energies (hmc.py:67-71: E_new first, then E_current), each with fresh masks
    HMCX_HIP(ctx, mlp_forward<T>(net, cur, masks_for(fwd++), lp_new));
    net.a1_valid = false;
    HMCX_HIP(ctx, mlp_forward<T>(net, par, masks_for(fwd++), lp_cur));
    VarTab ve{};
    for (int i = 0; i < 6; ++i) {
      const int v = s->order[i];
      ve.q[i] = cur[v]; ve.qn[i] = par[v]; ve.p[i] = pv[v]; ve.n[i] = dim[v];
    }
    hipLaunchKernelGGL(k_sumsq12<T>, dim3(NPART, 6), dim3(256), 0, st, ve, part_new);
    MlpAccept ac{};
    ac.part_cur = part_cur; ac.part_new = part_new; ac.lp_cur = lp_cur; ac.lp_new = lp_new;
    ac.nlb = net.nlb; ac.B = s->B;
    for (int i = 0; i < 6; ++i) ac.dim[i] = dim[s->order[i]];
    ac.alpha = s->alpha; ac.u = s->u_accept[si];
    ac.out_A = s->out_A + si; ac.out_acc = s->out_accepted + si; ac.out_loss = s->out_loss + si;
    ac.out_nlp = s->out_nlp ? s->out_nlp + si : nullptr;
    ac.out_E = s->out_E ? s->out_E + 2 * si : nullptr;
    ac.acc_flag = accf;
    hipLaunchKernelGGL(k_mlp_accept, dim3(1), dim3(26 * 32), 0, st, ac);
    if (n > 0) hipLaunchKernelGGL(k_mlp_commit<T>, dim3(NPART, 6), dim3(256), 0, st, ve, accf);
    HMCX_HIP(ctx, hipGetLastError());
  }
  if ((rc = gs.finish())) return rc;
  return timing_end(ctx, ctx->stream);
}

template int mlp_masks_t<float>(hmcx_ctx*, int, int, uint64_t, uint32_t, uint32_t, uint32_t, void*);
template int mlp_masks_t<double>(hmcx_ctx*, int, int, uint64_t, uint32_t, uint32_t, uint32_t, void*);
template int mlp_grad_t<float>(hmcx_ctx*, const void*, const int32_t*, int, int, int, int, const hmcx_mlp_params*,
                               const void*, double, hmcx_mlp_params*, double*);
template int mlp_grad_t<double>(hmcx_ctx*, const void*, const int32_t*, int, int, int, int, const hmcx_mlp_params*,
                                const void*, double, hmcx_mlp_params*, double*);
template int mlp_loss_t<float>(hmcx_ctx*, const void*, const int32_t*, int, int, int, int, const hmcx_mlp_params*,
                               const void*, double*, void*);
template int mlp_loss_t<double>(hmcx_ctx*, const void*, const int32_t*, int, int, int, int, const hmcx_mlp_params*,
                                const void*, double*, void*);
template int mlp_sghmc_t<float>(hmcx_ctx*, const hmcx_mlp_sghmc_args*);
template int mlp_sghmc_t<double>(hmcx_ctx*, const hmcx_mlp_sghmc_args*);

}  // namespace hmcx
