// hmcx_rowspace.hip — single-chain SGHMC for the softmax model with the leapfrog in ROW SPACE:
// one exchange round per leapfrog iteration instead of three (hmcx_persist2.hip).
//
// Mathematics: cpu/sghmc.py:19-39 with the A1 completion and cpu/softmax.py:38-79, as in the other
// SGHMC paths.  Within a step the minibatch X (B × D) is fixed, and everything the softmax needs is
// linear in the state: with Z = X·W (logits without bias), Q = X·p, G = X·Xᵀ (B × B Gram matrix) and
// R_i = X·z_i (projection of iteration i's friction noise), one leapfrog iteration is
//     Z' = Z + ε·Q                                   (drift, sghmc.py:32)
//     d  = y − softmax(clip(Z' + b))                (rows, softmax.py:38-52)
//     Q' = (1 − ε)·Q + ε·(α·Z' − G·d) + 2ε·R_i        (X·(momentum update), sghmc.py:31,34)
// so the rows only need G·d — the diff rows of the WHOLE minibatch, one all-gather of B × K values —
// instead of the reduce-scatter / all-gather / all-reduce of the D-space formulation.  The weights
// and momenta themselves (D-space) are carried by their owners with exactly the reference's update
// order (w += ε·p; p = (1 − ε)·p + ε·(α·w − Xᵀd) + 2ε·z), fed by Xᵀ·d, which the same MFMA pass
// produces: its A operand stacks the workgroup's G rows and the X columns of its owned features.
//
//  * k_rs_noise / k_rs_gemm (before the chain, whole GPU): G_s for every step of the call and the
//    projections X_s·[p0 | z_1 … z_n] (state-independent: the minibatch rows and the Philox noise of
//    every step are known when the call starts).  G_s is built from its upper tiles and mirrored, so
//    it is exactly symmetric.
//  * k_sghmc_rs (RS_G workgroups, one per CU, co-resident): workgroup w owns rows [w·Ro, +Ro) and
//    weight elements [w·Eo, +Eo) of W (flat d·K + k).  Per step: an all-gather of the owners'
//    weights (step > 0), Z_0 = X·W of its rows, the log-likelihood at the start state; per iteration
//    one all-gather of diff rows + bias colsum partials; per step one accept round.  Transport:
//    tagged granules (hmcx_p2x.h), regions double-buffered, epochs unique per launch.
// Reductions run in fixed orders, so replicated values (bias, accept) are bit-identical in every
// workgroup and runs are deterministic.  Results match the reference within rounding (the logits
// are advanced, not recomputed, within a step); the parity tests hold this path to the oracle.
#include "hmcx_common.h"
#include "hmcx_internal.h"
#include "hmcx_persist.h"
#include "hmcx_p2x.h"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace hmcx {

constexpr int RS_G = 128;       // workgroups of the chain kernel
constexpr int RS_NMAX = 64;     // leapfrog iterations per step held in LDS (longer steps: other paths)
constexpr int RS_ROMAX = 8;     // rows per workgroup
constexpr int RTH = 512;        // threads per chain workgroup (8 waves: two per SIMD)
constexpr int RNW = RTH / 64;
constexpr int RS_KSW = 16;      // MFMA k-steps per wave (B ≤ 4·8·16 = 512)
constexpr int RS_GU = 13;       // granules per thread of the diff all-gather (np·nitems ≤ RS_GU·RTH)
constexpr int RS_GW = 8;        // ... of each half of the weights' all-gather
constexpr int RS_XU = 8;        // X-row elements per thread at step start (Ro·D ≤ RS_XU·RTH)
constexpr int RS_GT = 64;       // pre-kernel GEMM tile

struct RSPre {
  int B, D, K, P, DK, n_steps, ctiles;
  const double* X; const int64_t* row0; const int32_t* n_iter;
  uint64_t seed; uint32_t chain0, step_base;
  double* nz; const int64_t* nzo;           // noise of the weight elements: nz[nzo[s] + slot·P + e]
  const int64_t* poff;                      // projections of step s at proj + poff[s]: [n_s + 1][B][K]
  double* gram; double* proj;               // gram: [n_steps][B][B]
};

struct RSArgs {
  int B, D, K, P, DK, n_steps;
  int G, Ro, Eo, nks, nsl;                  // nsl: projection slots held in LDS (max n_iter + 1)
  int span;                                 // doubles from Dall to Zr (≥ DK: the step-start weights)
  double alpha, neg_inv_n, log_prior;
  const double* X; const double* Y;
  const double* eps; const double* u; const int64_t* row0; const int32_t* n_iter;
  int noise_mode; const double* noise; const int64_t* noff;
  uint64_t seed; uint32_t chain0, step_base;
  double* W; double* b;
  const double* gram; const double* proj; const int64_t* poff;
  char* arena; int arena_bytes; unsigned ep0;
  int oAG, oWG, oAC, nag, nwg;              // regions (granules) and per-producer block strides
  int* abort_flag; int force_abort;
  double* out_A; int32_t* out_acc; double* out_ll; double* out_E;
  double* out_trace; double* out_mom;
  unsigned long long* prof;                 // HMCX_RS_PROF=1: per-segment s_memtime totals (workgroup 0)
};

// Segment profiler (workgroup 0, thread 0; totals in LDS, flushed once)
struct RSProf {
  unsigned long long* out;
  unsigned long long* acc;
  unsigned long long last;
  int cur;
  __device__ inline void stamp(int next) {
    if (!out) return;
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    if (last) acc[cur] += t - last;
    last = t;
    cur = next;
  }
  __device__ inline void flush() {
    if (!out) return;
    for (int i = 0; i < 16; ++i) out[i] = acc[i];
  }
};

// ---------------------------------------------------------------- pre-kernels
// Philox normals of the weight elements for slots 0 … n_s of every step (slot 0: momentum,
// slot i + 1: friction noise of iteration i), one Box–Muller pair per thread — the same values as
// philox_normal_d(e) (hmcx_common.h) that the chain kernel's owners draw for their elements.
__global__ __launch_bounds__(256) void k_rs_noise(RSPre a) {
  const int s = blockIdx.y;
  const int nsl = max(a.n_iter[s], 0) + 1, npair = (a.DK + 1) / 2;
  double* base = a.nz + a.nzo[s];
  for (int q = blockIdx.x * 256 + threadIdx.x; q < nsl * npair; q += gridDim.x * 256) {
    const int slot = q / npair, pr = q - slot * npair;
    double z0, z1;
    philox_pair_d(a.seed, a.chain0, a.step_base + (uint32_t)s, (uint32_t)slot, (uint32_t)pr, z0, z1);
    double* dst = base + (int64_t)slot * a.P + 2 * pr;
    dst[0] = z0;
    if (2 * pr + 1 < a.DK) dst[1] = z1;
  }
}

// C_s = X_s · [X_sᵀ | Z_s] per step s: 64 × 64 tiles, 4 waves × (16 rows × 64 columns) of
// v_mfma_f64_16x16x4, the D loop staged through LDS in 16-deep chunks with the next chunk's loads in
// flight.  Columns [0, B): Gram (tiles below the diagonal skipped, the others mirrored); columns
// B + slot·K + k: projection of noise slot `slot`, class k.
__global__ __launch_bounds__(256) void k_rs_gemm(RSPre a) {
  using M = mfma16<double>;
  const int s = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int B = a.B, D = a.D, K = a.K;
  const int n = max(a.n_iter[s], 0), ncol = B + K * (n + 1);
  const int rt = (B + RS_GT - 1) / RS_GT;
  const int ti = blockIdx.x % rt, tc = blockIdx.x / rt;
  if (tc * RS_GT >= ncol) return;
  if (tc < ti) return;                               // below the diagonal: mirrored by tile (tc, ti)
  __shared__ double As[RS_GT][17];                   // [row][k]
  __shared__ double Bs[16][RS_GT + 1];               // [k][column]
  const double* Xs = a.X + (size_t)a.row0[s] * D;
  const double* nzs = a.nz + a.nzo[s];
  // staging maps: A element q = tid + 256u → row q / 16, k q % 16; B element → column q / 16, k q % 16
  double av[4], bv[4];
  auto load = [&](int d0) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = tid + 256 * u, r = q >> 4, k = q & 15, d = d0 + k;
      const int row = ti * RS_GT + r, col = tc * RS_GT + r;
      const bool okd = d < D;
      const double xa = Xs[(size_t)min(row, B - 1) * D + min(d, D - 1)];
      av[u] = (row < B && okd) ? xa : 0.0;
      // column col: Gram (X_s row col) or a noise column (slot, class)
      const int cn = max(col - B, 0), slot = cn / K, kk = cn - slot * K;
      const double xg = Xs[(size_t)min(col, B - 1) * D + min(d, D - 1)];
      const double zn = nzs[(int64_t)min(slot, n) * a.P + (int64_t)min(d, D - 1) * K + kk];
      bv[u] = !okd || col >= ncol ? 0.0 : (col < B ? xg : zn);
    }
  };
  typename M::acc_t acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = M::zero();
  load(0);
  for (int d0 = 0; d0 < D; d0 += 16) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = tid + 256 * u, r = q >> 4, k = q & 15;
      As[r][k] = av[u];
      Bs[k][r] = bv[u];
    }
    __syncthreads();
    if (d0 + 16 < D) load(d0 + 16);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const double af = As[wave * 16 + (lane & 15)][ks * 4 + (lane >> 4)];
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = M::fma(af, Bs[ks * 4 + (lane >> 4)][t * 16 + (lane & 15)], acc[t]);
    }
  }
  double* gs = a.gram + (size_t)s * B * B;
  double* ps = a.proj + a.poff[s];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = ti * RS_GT + wave * 16 + (lane >> 4) + 4 * q;
      const int col = tc * RS_GT + t * 16 + (lane & 15);
      if (row >= B || col >= ncol) continue;
      const double v = acc[t][q];
      if (col < B) {
        gs[(size_t)row * B + col] = v;
        if (tc != ti) gs[(size_t)col * B + row] = v;
      } else {
        const int cn = col - B, slot = cn / K, kk = cn - slot * K;
        ps[((size_t)slot * B + row) * K + kk] = v;
      }
    }
}

// ---------------------------------------------------------------- chain kernel helpers
__device__ inline double rs_noise(const RSArgs& a, int s, uint32_t slot, uint32_t e) {
  if (a.noise_mode == HMCX_NOISE_BUFFER) return a.noise[a.noff[s] + (int64_t)slot * a.P + e];
  return philox_normal_d(a.seed, a.chain0, a.step_base + (uint32_t)s, slot, e);
}

// All-gather of np producers × nitems granules (producer p's item i at base0 + p·pstride + i), U
// granules per thread in one batch of loads.  Item i < nsplit lands in dstA[p·nsplit + i] (pairs with
// p·nsplit + i ≥ limA are not polled), the others in dstB[p·(nitems − nsplit) + i − nsplit].
// With tK > 0 the A items are elements e = offA + p·nsplit + i (< limA) of a [.][tK] array stored
// transposed, at (e mod tK)·tD + e / tK.
template <int U>
__device__ inline bool rs_gather(__amdgpu_buffer_rsrc_t rs, int base0, int pstride, int np, int nitems, int nsplit,
                                 int limA, double* dstA, double* dstB, unsigned ep, int* abort_flag,
                                 int offA = 0, int tK = 0, int tD = 0) {
  static_assert(U <= 32, "pending mask");
  const int total = np * nitems, nb = nitems - nsplit;
  const int t = opaque((int)threadIdx.x);
  unsigned pend = 0;
  int o[U], dsto[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int q = t + u * RTH;
    const int p = q / nitems, i = q - p * nitems;
    const bool isA = i < nsplit;
    const int da = offA + p * nsplit + i;
    const bool w = q < total && (!isA || da < limA);
    pend |= w ? 1u << u : 0u;
    o[u] = (base0 + (w ? p * pstride + i : 0)) * 16;
    const int dt = tK > 0 ? (da % max(tK, 1)) * tD + da / max(tK, 1) : da;
    dsto[u] = isA ? dt : -1 - (p * nb + i - nsplit);
  }
  unsigned long long t0 = 0;
  for (int spins = 0; pend; ++spins) {
    gran_t v[U];
    // only the granules still missing are re-read (a received one would re-cross the fabric)
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = ((pend >> u) & 1u) ? __builtin_amdgcn_raw_buffer_load_b128(rs, o[u], 0, 16 /* sc1 */) : gran_t{0u, 0u, 0u, 0u};
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (((pend >> u) & 1u) && v[u].y == ep && v[u].w == ep) {
        const double x = decode(v[u]);
        if (dsto[u] >= 0) dstA[dsto[u]] = x;
        else dstB[-1 - dsto[u]] = x;
        pend &= ~(1u << u);
      }
    if (!pend) break;
    if (spins == 0) t0 = __builtin_amdgcn_s_memrealtime();
    if ((spins & 63) == 63 &&
        (__builtin_amdgcn_s_memrealtime() - t0 > QTIMEOUT ||
         __hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
      __hip_atomic_store(abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    if (HMCX_P2_SLEEP) __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

// Fixed-order sum of np partials src[p·stride] over a 32-lane group: lane j adds p ≡ j (mod 32) in
// increasing p, then a butterfly over the group — every lane of the group ends with the same bits.
__device__ inline double rs_gsum32(const double* src, int stride, int np, int j) {
  double v = 0.0;
  for (int p = j; p < np; p += 32) v += src[p * stride];
#pragma unroll
  for (int m = 16; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

// Deterministic workgroup sum over the RNW waves (fixed butterfly, fixed wave order).
__device__ inline double rs_wsum(double v, double* sh) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = sh[0];
#pragma unroll
  for (int w = 1; w < RNW; ++w) r += sh[w];
  __syncthreads();
  return r;
}

// ---------------------------------------------------------------- chain kernel
__global__ __launch_bounds__(RTH) void k_sghmc_rs(RSArgs a) {
  using M = mfma16<double>;
  extern __shared__ __align__(16) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int w = blockIdx.x, G = a.G, Ro = a.Ro, K = a.K, D = a.D, B = a.B, DK = a.DK;
  const int r0 = w * Ro, nr = max(0, min(Ro, B - r0));
  const int e0 = w * a.Eo, ne = max(0, min(a.Eo, DK - e0));
  const int fd0 = e0 / K;
  const bool own = tid < ne;
  const int e_own = e0 + (own ? tid : 0);
  const int d_own = e_own / K, k_own = e_own - d_own * K;
  const int m_own = Ro + d_own - fd0;                    // MFMA output row of the owned element
  const double hi = CLIP_HI, lo = CLIP_LO, alpha = a.alpha;
  const __amdgpu_buffer_rsrc_t rs = arena_rsrc(a.arena, a.arena_bytes);
  const int nag0 = Ro * K + K;                           // AG items per producer: diff rows, colsum

  // ---- LDS carve-up (mirrored by rs_lds)
  const int AP = 4 * RNW * a.nks;                        // A columns (minibatch rows, padded)
  double* Am = reinterpret_cast<double*>(smem);          // A [AP][16]: my G rows, then my X columns
  double* Rx = Am + 16 * AP;                             // [nsl][Ro][K]: Q0 = X·p0, R_i = X·z_i
  double* Dall = Rx + ((a.nsl * Ro * K + 1) & ~1);       // [B][K] diff rows of the whole minibatch
  double* Wst = Dall;                                    // [K][D] weights at step start (over Dall … csb)
  double* red = Dall + ((B * K + 1) & ~1);               // [RNW][256] per-wave MFMA tiles
  double* csb = red + RNW * 256;                         // [G][K] colsum partials | accept partials
  double* Zr = Dall + a.span;                            // [Ro][16]
  double* Qr = Zr + Ro * 16;
  double* Yr = Qr + Ro * 16;
  double* Cd = Yr + Ro * 16;                             // [Ro][16] diff at b' (bias sub-step)
  double* llr = Cd + Ro * 16;                            // [RS_ROMAX]
  double* bsh = llr + RS_ROMAX;                          // [16] b
  double* pbs = bsh + 16;                                // [16] pb
  double* b0s = pbs + 16;                                // [16] b at step start
  double* pb0s = b0s + 16;                               // [16] pb drawn at step start
  double* dsh = pb0s + 16;                               // [16] reductions
  int* ish = reinterpret_cast<int*>(dsh + 16);           // [4] flags
  unsigned long long* pacc = reinterpret_cast<unsigned long long*>(dsh + 18);   // [16] profiler
  double* zpart = dsh + 34;                              // [RNW][16] Z_0 partials (one per wave)

  if (__hip_atomic_load(a.abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  if (tid == 0) ish[0] = 0;
  if (tid < 16) pacc[tid] = 0ull;
  RSProf prof{(w == 0 && tid == 0) ? a.prof : nullptr, pacc, 0ull, 0};
  if (tid < 16) bsh[tid] = tid < K ? a.b[tid] : 0.0;
  double wv = own ? a.W[e_own] : 0.0;                    // owned weight
  double pw = 0.0;                                       // owned momentum
  unsigned ep = a.ep0 - 1;
  unsigned uAG = 0, uWG = 0, uAC = 0;

  // Operands of step sn that do not depend on the state: the MFMA A operand (my G rows, then the X
  // columns of my features; column j = minibatch row j; stored A[j][i] at j·16 + i), the labels and
  // projections of my rows (into LDS), and my rows of X for Z_0 (registers: thread t takes row t / (RTH/4),
  // features t mod (RTH/4) + (RTH/4)·u).  mid() runs while the loads travel (the previous step's accept
  // round); the LDS they replace must be dead by then.
  constexpr int XT = RTH / 4;                            // threads per X row (Ro ≤ 4)
  double xv0[RS_XU];
  auto prefetch = [&](int sn, auto mid) -> bool {
    const int tp = opaque(tid);
    const double* Xn = a.X + (size_t)a.row0[sn] * D;
    const double* Yn = a.Y + (size_t)a.row0[sn] * K;
    const double* gs = a.gram + (size_t)sn * B * B;
    const double* ps = a.proj + a.poff[sn];
    const int nsl = max(a.n_iter[sn], 0) + 1;
    double gv[16], xv[16], rv[4];
#pragma unroll
    for (int u = 0; u < 16; ++u) {                       // 32 loads in flight
      const int q = tp + u * RTH, j = q >> 4, i = q & 15;
      const int fi = fd0 + i - Ro, jc = min(j, B - 1);
      gv[u] = gs[(size_t)min(r0 + min(i, Ro - 1), B - 1) * B + jc];
      xv[u] = Xn[(size_t)jc * D + min(max(fi, 0), D - 1)];
    }
    {
      const int i = tp / XT, d0 = tp - (tp / XT) * XT;
#pragma unroll
      for (int u = 0; u < RS_XU; ++u) xv0[u] = Xn[(size_t)min(r0 + min(i, Ro - 1), B - 1) * D + min(d0 + XT * u, D - 1)];
    }
    const double yv = Yn[(size_t)min(r0 + min(tp >> 4, Ro - 1), B - 1) * K + min(tp & 15, K - 1)];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tp + u * RTH, sl = e / (Ro * K), rem = e - sl * Ro * K, i = rem / K, k = rem - i * K;
      rv[u] = ps[((size_t)min(sl, nsl - 1) * B + min(r0 + i, B - 1)) * K + k];
    }
    if (!mid()) return false;
#pragma unroll
    for (int u = 0; u < RS_XU; ++u) asm volatile("" : "+v"(xv0[u]));   // arrived here, not at first use
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int q = tp + u * RTH, j = q >> 4, i = q & 15;
      const int fi = fd0 + i - Ro;
      const bool isg = i < nr, isx = i >= Ro && ne > 0 && fi < D;
      if (q < 16 * AP) Am[q] = j >= B ? 0.0 : (isg ? gv[u] : (isx ? xv[u] : 0.0));
    }
    if (tp < Ro * 16) Yr[tp] = ((tp >> 4) < nr && (tp & 15) < K) ? yv : 0.0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tp + u * RTH, i = (e - (e / (Ro * K)) * Ro * K) / K;
      if (e < nsl * Ro * K) Rx[e] = i < nr ? rv[u] : 0.0;
    }
    return true;
  };
  prefetch(0, []() { return true; });
  __syncthreads();

  for (int s = 0; s < a.n_steps; ++s) {
    const double eps = a.eps[s], ome = 1.0 - eps, nsc = 2.0 * eps;
    const int n = a.n_iter[s];
    const int ts = opaque(tid), ls = ts & 63, ws = ts >> 6;   // step-local (not hoisted) thread ids
    const double* Xs = a.X + (size_t)a.row0[s] * D;
    const double* Ys = a.Y + (size_t)a.row0[s] * K;
    if (s == a.force_abort && w == G - 1) {              // test knob: a "timed-out" member
      if (ts == 0) __hip_atomic_store(a.abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    prof.stamp(0);
    // ---- step start (labels, projections, A operand and my X rows were prefetched): momentum
    pw = own ? rs_noise(a, s, 0u, (uint32_t)e_own) : 0.0;                 // hmc.py:82-87
    const double pw0 = pw, w0 = wv;
    if (ts < 16) {
      pbs[ts] = ts < K ? rs_noise(a, s, 0u, (uint32_t)(DK + ts)) : 0.0;
      pb0s[ts] = pbs[ts];
      b0s[ts] = bsh[ts];
    }
    prof.stamp(1);
    // weights of the whole model for Z_0 = X·W: step 0 from W, later from the owners (all-gather)
    if (s == 0) {
      for (int e = ts; e < DK; e += RTH) Wst[(e % K) * D + e / K] = a.W[e];   // stored [K][D]
      __syncthreads();
    } else {
      ++ep;
      const int base0 = a.oWG + (int)(uWG & 1) * G * a.nwg;
      ++uWG;
      // two halves of the producers, one batch of loads each (fewer registers than one wide batch)
      const int Gh = G / 2;
      bool ok = rs_gather<RS_GW>(rs, base0, a.nwg, Gh, a.Eo, a.Eo, DK, Wst, nullptr, ep, a.abort_flag, 0, K, D);
      ok = ok && rs_gather<RS_GW>(rs, base0 + Gh * a.nwg, a.nwg, G - Gh, a.Eo, a.Eo, DK, Wst, nullptr, ep,
                                  a.abort_flag, Gh * a.Eo, K, D);
      if (!all_ok(ok, ish)) return;
    }
    const double kin0 = rs_wsum(pw * pw, dsh);
    double kb0 = 0.0;
    for (int k = 0; k < K; ++k) kb0 += pb0s[k] * pb0s[k];
    prof.stamp(2);
    // Z_0 = X·W of my rows: XT threads per row (2 waves), features strided by XT, fixed-order sums
    {
      const int i = ts / XT, d0 = ts - (ts / XT) * XT;
      double acc[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[k] = 0.0;
#pragma unroll
      for (int u = 0; u < RS_XU; ++u) {
        const int d = d0 + XT * u;
        if (d < D) {
#pragma unroll
          for (int k = 0; k < 16; ++k)
            if (k < K) acc[k] += xv0[u] * Wst[k * D + d];
        }
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        if (k < K) {                                     // K is workgroup-uniform
          double v = acc[k];
#pragma unroll
          for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
          if (ls == 0) zpart[ws * 16 + k] = v;          // one partial per wave
        }
      }
    }
    __syncthreads();
    for (int e = ts; e < Ro * 16; e += RTH) {
      const int i = e >> 4, k = e & 15;
      const double z = zpart[(2 * i) * 16 + k] + zpart[(2 * i + 1) * 16 + k];   // the row's two waves
      Zr[e] = (k < K && i < nr) ? z : 0.0;
      Qr[e] = k < K ? Rx[i * K + k] : 0.0;             // Q_0 = X·p0 (slot 0)
    }
    prof.stamp(3);
    __syncthreads();
    // log-likelihood of my rows at the step-start state (E_current)
    double ll0 = 0.0, ll_last = 0.0;
    if (ts < Ro * 16) {
      const int i = ts >> 4, k = ts & 15;
      const bool kv = k < K && i < nr;
      const double z = kv ? clipz(Zr[i * 16 + k] + b0s[k], hi, lo) : -__builtin_inf();
      const double m = g16_max2(z);
      const double ex = kv ? exp(z - m) : 0.0;
      const double sm = g16_sum2(ex);
      const double lse = log(sm) + m;                                     // softmax.py:18
      const double t = kv ? Yr[i * 16 + k] * (z - lse) : 0.0;             // softmax.py:19-20
      const double rsum = g16_sum2(t);
      if (k == 0) llr[i] = i < nr ? rsum : 0.0;
    }
    __syncthreads();
    if (ts == 0) {
      double v = 0.0;
      for (int i = 0; i < nr; ++i) v += llr[i];
      dsh[4] = v;
    }
    __syncthreads();
    ll0 = dsh[4];

    // ---- leapfrog iterations in row space
    for (int it = 0; it < n; ++it) {
      const bool last = it == n - 1;
      const int ti = opaque(tid);                        // iteration-local thread id
      // drift, both softmaxes of my rows (at b for the weights, at b' = b + ε·pb for the bias)
      prof.stamp(4);
      ++ep;
      const int base0 = a.oAG + (int)(uAG & 1) * G * a.nag;
      ++uAG;
      if (ti < Ro * 16) {
        const int i = ti >> 4, k = ti & 15;
        const bool kv = k < K && i < nr;
        const double z = Zr[ti] + eps * Qr[ti];                         // X·(w + ε·p), sghmc.py:32
        Zr[ti] = z;
        const double y = Yr[ti];
        const double bp = bsh[k] + eps * pbs[k];
        const double zw = kv ? clipz(z + bsh[k], hi, lo) : -__builtin_inf();   // softmax.py:39-41
        const double mw = g16_max2(zw);
        const double ew = kv ? exp(zw - mw) : 0.0;                        // softmax.py:34
        const double sw = g16_sum2(ew);
        const double dw = kv ? y - ew / sw : 0.0;                         // softmax.py:52
        const double zb = kv ? clipz(z + bp, hi, lo) : -__builtin_inf();
        const double mb = g16_max2(zb);
        const double eb = kv ? exp(zb - mb) : 0.0;
        const double sb = g16_sum2(eb);
        Cd[ti] = kv ? y - eb / sb : 0.0;
        if (last) {
          const double lse = log(sb) + mb;
          const double t = kv ? y * (zb - lse) : 0.0;
          const double rsum = g16_sum2(t);
          if (k == 0) llr[i] = i < nr ? rsum : 0.0;
        }
        if (k < K) put(rs, base0 + w * a.nag + i * K + k, dw, ep);
      }
      __syncthreads();
      if (ti < K) {
        double c = 0.0;
        for (int i = 0; i < nr; ++i) c += Cd[i * 16 + ti];
        put(rs, base0 + w * a.nag + Ro * K + ti, c, ep);
      }
      if (last && ti == 0) {
        double v = 0.0;
        for (int i = 0; i < nr; ++i) v += llr[i];
        ll_last = v;
      }
      prof.stamp(5);
      // friction noise of this iteration while the round travels (sghmc.py:31)
      const double zn = own ? rs_noise(a, s, (uint32_t)(it + 1), (uint32_t)e_own) : 0.0;
      const double zbn = ((ti & 31) == 0 && (ti >> 5) < K)
                             ? rs_noise(a, s, (uint32_t)(it + 1), (uint32_t)(DK + (ti >> 5))) : 0.0;
      const bool ok = rs_gather<RS_GU>(rs, base0, a.nag, G, nag0, Ro * K, B * K, Dall, csb, ep, a.abort_flag);
      if (!all_ok(ok, ish)) return;
      prof.stamp(6);
      // [G rows | X columns]ᵀ·diff: G·d for my rows (rows < Ro), Xᵀ·d for my features (rows ≥ Ro)
      {
        typename M::acc_t c0 = M::zero(), c1 = M::zero();
        const int li = opaque(lane), col = li & 15;
        const int nks = a.nks;
        typename M::acc_t c2 = M::zero(), c3 = M::zero();
#pragma unroll
        for (int h = 0; h < RS_KSW; h += 8) {            // two batches of 8 k-steps: loads, then MFMAs
          double av[8], bv[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int j = 4 * (wave * nks + h + u) + (li >> 4);
            av[u] = Am[min(j, AP - 1) * 16 + col];
            bv[u] = Dall[min(j, B - 1) * K + min(col, K - 1)];
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int j = 4 * (wave * nks + h + u) + (li >> 4);
            const double bx = (h + u < nks && j < B && col < K) ? bv[u] : 0.0;
            if ((u & 3) == 0) c0 = M::fma(av[u], bx, c0);
            if ((u & 3) == 1) c1 = M::fma(av[u], bx, c1);
            if ((u & 3) == 2) c2 = M::fma(av[u], bx, c2);
            if ((u & 3) == 3) c3 = M::fma(av[u], bx, c3);
          }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) red[wave * 256 + ((lane >> 4) + 4 * q) * 16 + col] = (c0[q] + c1[q]) + (c2[q] + c3[q]);
      }
      __syncthreads();
      prof.stamp(7);
      const int gk = ti >> 5, gj = ti & 31;                                // 32-lane group per class
      const double cst = gk < K ? rs_gsum32(csb + gk, K, G, gj) : 0.0;         // Σ colsum partials
      if (!last && ti < Ro * 16) {
        const int m = ti >> 4, k = ti & 15;
        double gd = red[ti];
#pragma unroll
        for (int q = 1; q < RNW; ++q) gd += red[q * 256 + ti];
        const double rn = (k < K) ? Rx[((it + 1) * Ro + m) * K + min(k, K - 1)] : 0.0;
        Qr[ti] = k < K ? (ome * Qr[ti] + eps * (alpha * Zr[ti] - gd)) + nsc * rn : 0.0;
      }
      if (own) {                                                              // sghmc.py:31-34
        const int mi = m_own * 16 + k_own;
        double S = red[mi];
#pragma unroll
        for (int q = 1; q < RNW; ++q) S += red[q * 256 + mi];
        wv = wv + eps * pw;
        const double gz = -(S - alpha * wv);                                  // softmax.py:57-58
        pw = (ome * pw + eps * gz) + nsc * zn;
      }
      if (gk < K && gj == 0) {                                                // bias sub-step, replicated
        const double bp = bsh[gk] + eps * pbs[gk];
        const double gr = -(cst - alpha * bp);
        pbs[gk] = (ome * pbs[gk] + eps * gr) + nsc * zbn;
        bsh[gk] = bp;
      }
      __syncthreads();
    }

    prof.stamp(8);
    // ===== accept (hmc.py:67-71): kinetic / log-likelihood partials of every workgroup
    const double kin1 = rs_wsum(pw * pw, dsh);
    double kb1 = 0.0;
    for (int k = 0; k < K; ++k) kb1 += pbs[k] * pbs[k];
    ++ep;
    const int abase = a.oAC + (int)(uAC & 1) * G * 8;
    ++uAC;
    if (ts == 0) {
      put(rs, abase + w * 8 + 0, kin0, ep);
      put(rs, abase + w * 8 + 1, kin1, ep);
      put(rs, abase + w * 8 + 2, ll0, ep);
      put(rs, abase + w * 8 + 3, ll_last, ep);                               // ll(q_new) of my rows
    }
    {
      bool ok = true;
      const auto accept_round = [&]() {
        ok = rs_gather<4>(rs, abase, 8, G, 4, 4, 4 * G, csb, nullptr, ep, a.abort_flag);
        return ok;
      };
      // the next step's operands travel with the accept round (A, Rx, Yr have no reader left)
      if (s + 1 < a.n_steps) prefetch(s + 1, accept_round);
      else accept_round();
      if (!all_ok(ok, ish)) return;
    }
    if (ts < 128) {                                   // four 32-lane groups: K0, K1, ll0, ll(q_new)
      const double v = rs_gsum32(csb + (ts >> 5), 4, G, ts & 31);
      if ((ts & 31) == 0) dsh[8 + (ts >> 5)] = v;
    }
    __syncthreads();
    const double S0 = dsh[8], S1 = dsh[9], L0 = dsh[10], LL = dsh[11];
    __syncthreads();
    prof.stamp(9);
    const double K0 = (0.0 + 0.5 * S0) + 0.5 * kb0;
    const double Ecur = a.neg_inv_n * (L0 + a.log_prior) + K0;
    double A, Enew, llq;
    int acc;
    if (n <= 0) {
      A = 1.0; Enew = Ecur; llq = L0;
      acc = a.u[s] < A;
    } else {
      const double K1 = (0.0 + 0.5 * S1) + 0.5 * kb1;
      Enew = a.neg_inv_n * (LL + a.log_prior) + K1;
      const double x = exp(Ecur - Enew);
      A = (x < 1.0) ? x : 1.0;                                                // Python min(1, x)
      acc = a.u[s] < A;
      llq = acc ? LL : L0;
    }
    const bool keep_new = acc && n > 0;
    if (a.out_mom && s == a.n_steps - 1) {                                    // sghmc.py:36-39 returned p
      if (own) a.out_mom[e_own] = keep_new ? pw : pw0;
      if (w == 0 && ts < K) a.out_mom[DK + ts] = keep_new ? pbs[ts] : pb0s[ts];
    }
    if (!keep_new) {                                                          // keep q (sghmc.py:36-38)
      wv = w0;
      if (ts < 16) bsh[ts] = b0s[ts];
    }
    if (a.out_trace) {                                                        // sghmc_multicore.py:49-51 row
      double* tr = a.out_trace + (size_t)s * a.P;
      if (own) tr[e_own] = wv;
      if (w == 0 && ts < K) tr[DK + ts] = bsh[ts];
    }
    if (w == 0 && ts == 0) {
      a.out_A[s] = A;
      a.out_acc[s] = acc;
      a.out_ll[s] = llq;
      if (a.out_E) { a.out_E[2 * s] = Ecur; a.out_E[2 * s + 1] = Enew; }
    }
    // owned weights → every workgroup for the next step's Z_0
    if (s + 1 < a.n_steps) {
      const int reg = a.oWG + ((int)(uWG & 1) * G + w) * a.nwg;
      if (own) put(rs, reg + ts, wv, ep + 1);
    }
    __syncthreads();
  }
  prof.stamp(0);
  prof.flush();
  if (__hip_atomic_load(a.abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  if (own) a.W[e_own] = wv;
  if (w == 0 && tid < K) a.b[tid] = bsh[tid];
}

// ---------------------------------------------------------------- plan + launch
static int rs_span(int B, int D, int K, int G) {
  const int used = ((B * K + 1) & ~1) + RNW * 256 + std::max(G * K, 4 * G);
  return (std::max(used, D * K) + 1) & ~1;
}
static size_t rs_lds(int B, int D, int K, int Ro, int G, int nks, int nsl) {
  const int AP = 4 * RNW * nks;
  size_t t = (size_t)16 * AP + (size_t)((nsl * Ro * K + 1) & ~1) + rs_span(B, D, K, G) + 4 * (size_t)Ro * 16 +
             RS_ROMAX + 5 * 16 + 40 + RNW * 16;
  return t * sizeof(double) + 16;
}

struct RSPlan {
  bool ok;
  int G, Ro, Eo, nks, nsl;
  size_t lds;
};

static RSPlan plan_rs(const hmcx_ctx* ctx, const hmcx_sampler_args* s) {
  RSPlan p{};
  const int B = s->B, D = s->D, K = s->K, DK = D * K;
  if (s->dtype != HMCX_F64 || s->C != 1 || K < 2 || K > 16 || B < 1 || B > 4 * RNW * RS_KSW) return p;
  p.G = RS_G;
  if (ctx->num_cus < p.G) return p;
  p.Ro = (B + p.G - 1) / p.G;
  p.Eo = (DK + p.G - 1) / p.G;
  if (p.Ro > 4 || D > (RTH / 4) * RS_XU) return p;
  // features spanned by one workgroup's elements must fit the MFMA rows left after its G rows
  int fw = 0;
  for (int w = 0; w < p.G; ++w) {
    const int e0 = w * p.Eo, e1 = std::min(DK, e0 + p.Eo);
    if (e1 > e0) fw = std::max(fw, (e1 - 1) / K - e0 / K + 1);
  }
  if (p.Ro + fw > 16) return p;
  p.nks = ((B + 3) / 4 + RNW - 1) / RNW;
  if (p.nks > RS_KSW) return p;
  if (p.G * (p.Ro * K + K) > RS_GU * RTH || (p.G - p.G / 2) * p.Eo > RS_GW * RTH || p.Eo > RTH) return p;
  int nmax = 0;
  for (int i = 0; i < s->n_steps; ++i) nmax = std::max(nmax, (int)s->n_iter[i]);
  if (nmax > RS_NMAX) return p;
  p.nsl = nmax + 1;
  if (p.nsl * p.Ro * K > 4 * RTH) return p;              // projections: 4 per thread
  if (16 * 4 * RNW * p.nks > 16 * RTH) return p;          // the A operand is loaded 16 values per thread
  p.lds = rs_lds(B, D, K, p.Ro, p.G, p.nks, p.nsl);
  if (p.lds > ctx->lds_max) return p;
  p.ok = true;
  return p;
}

// Path 3 selects this kernel; under auto (path 0) it is used only with HMCX_RS=1 — measured at the
// speed of the 2-D kernel (12.8 vs 12.9 µs per leapfrog), which stays the default.
bool sghmc_rs_selected(hmcx_ctx* ctx, const hmcx_sampler_args* s) {
  static const bool on = getenv("HMCX_RS") && getenv("HMCX_RS")[0] == '1';
  if (ctx->sghmc_path != 3 && !(ctx->sghmc_path == 0 && on)) return false;
  return plan_rs(ctx, s).ok;
}

int sghmc_rs_t(hmcx_ctx* ctx, const hmcx_sampler_args* s) {
  const RSPlan pl = plan_rs(ctx, s);
  if (!pl.ok) return set_error(ctx, HMCX_EUNSUPPORTED, "row-space SGHMC: shape not supported");
  const int B = s->B, D = s->D, K = s->K, DK = D * K, P = DK + K, G = pl.G;
  const size_t n = (size_t)s->n_steps;
  int rc = abort_precheck(ctx);
  if (rc) return rc;
  // per-step offsets: noise (Philox mode: a scratch buffer of the weight slots; buffer mode: the
  // caller's noise with its own offsets) and projections
  const bool buf = s->noise_mode == HMCX_NOISE_BUFFER;
  std::vector<int64_t>& poff = ctx->rs_poff;
  std::vector<int64_t>& nzo = ctx->rs_nzo;
  poff.resize(n);
  nzo.resize(n);
  int64_t ptot = 0, ntot = 0;
  unsigned rounds = 0;
  for (size_t i = 0; i < n; ++i) {
    const int ni = std::max(s->n_iter[i], 0);
    poff[i] = ptot;
    ptot += (int64_t)(ni + 1) * B * K;
    nzo[i] = buf ? s->noise_off[i] : ntot;
    ntot += (int64_t)(ni + 1) * P;
    rounds += (unsigned)ni + 2;
  }
  // granule arena: AG [2][G][nag], WG [2][G][nwg], AC [2][G][8]
  const int nag = p2_pad(pl.Ro * K + K, 1), nwg = p2_pad(pl.Eo, 1);
  const long oAG = 0, oWG = 2L * G * nag, oAC = oWG + 2L * G * nwg, ngran = oAC + 2L * G * 8;
  if ((rc = gx_reserve(ctx, (size_t)ngran * 16))) return rc;
  unsigned ep0 = 1;
  if ((rc = gx_epochs(ctx, rounds, &ep0))) return rc;
  const void* hsrc[7] = {s->eps, s->u_accept, s->row0, s->n_iter, poff.data(), nzo.data(), nullptr};
  const size_t hbytes[7] = {n * sizeof(double), n * sizeof(double), n * sizeof(int64_t), n * sizeof(int32_t),
                            n * sizeof(int64_t), n * sizeof(int64_t), 0};
  for (int i = 0; i < 4; ++i)
    if (!hsrc[i]) return set_error(ctx, HMCX_EINVAL, "sghmc: null host schedule array");
  const size_t sched_bytes = packed_bytes(6, hbytes);
  Workspace ws(ctx);
  char* sched;
  double *gram, *proj, *nz = nullptr;
  do {
    ws.reset();
    sched = ws.take<char>(sched_bytes);
    gram = ws.take<double>(n * B * B);
    proj = ws.take<double>((size_t)ptot);
    if (!buf) nz = ws.take<double>((size_t)ntot);
  } while (ws.retry());
  if (ws.failed) return HMCX_ENOMEM;
  begin_call(ctx);
  char* dp[6];
  if ((rc = upload_packed(ctx, sched, 6, hsrc, hbytes, dp))) return rc;

  RSPre pre{};
  pre.B = B; pre.D = D; pre.K = K; pre.P = P; pre.DK = DK; pre.n_steps = (int)n;
  pre.X = reinterpret_cast<const double*>(s->X);
  pre.row0 = reinterpret_cast<const int64_t*>(dp[2]);
  pre.n_iter = reinterpret_cast<const int32_t*>(dp[3]);
  pre.seed = s->seed; pre.chain0 = s->chain0; pre.step_base = s->step_base;
  pre.nz = buf ? const_cast<double*>(s->noise) : nz;
  pre.nzo = reinterpret_cast<const int64_t*>(dp[5]);
  pre.poff = reinterpret_cast<const int64_t*>(dp[4]);
  pre.gram = gram; pre.proj = proj;
  int nmax = 0;
  for (size_t i = 0; i < n; ++i) nmax = std::max(nmax, (int)s->n_iter[i]);
  const int rt = (B + RS_GT - 1) / RS_GT, ct = (B + K * (nmax + 1) + RS_GT - 1) / RS_GT;
  pre.ctiles = ct;

  RSArgs a{};
  a.B = B; a.D = D; a.K = K; a.P = P; a.DK = DK; a.n_steps = (int)n;
  a.G = G; a.Ro = pl.Ro; a.Eo = pl.Eo; a.nks = pl.nks; a.nsl = pl.nsl;
  a.span = rs_span(B, D, K, G);
  a.alpha = s->alpha; a.neg_inv_n = -1.0 / (double)B; a.log_prior = s->log_prior;
  a.X = reinterpret_cast<const double*>(s->X); a.Y = reinterpret_cast<const double*>(s->Y);
  a.eps = reinterpret_cast<const double*>(dp[0]); a.u = reinterpret_cast<const double*>(dp[1]);
  a.row0 = pre.row0; a.n_iter = pre.n_iter;
  a.noise_mode = s->noise_mode; a.noise = s->noise; a.noff = pre.nzo;
  a.seed = s->seed; a.chain0 = s->chain0; a.step_base = s->step_base;
  a.W = reinterpret_cast<double*>(s->W); a.b = reinterpret_cast<double*>(s->b);
  a.gram = gram; a.proj = proj; a.poff = pre.poff;
  a.arena = ctx->gx_arena; a.arena_bytes = (int)(ngran * 16); a.ep0 = ep0;
  a.oAG = (int)oAG; a.oWG = (int)oWG; a.oAC = (int)oAC; a.nag = nag; a.nwg = nwg;
  a.abort_flag = ctx->abort_dev;
  a.force_abort = getenv("HMCX_P2_FORCE_ABORT") ? atoi(getenv("HMCX_P2_FORCE_ABORT")) : -1;
  a.out_A = s->out_A; a.out_acc = s->out_accepted; a.out_ll = s->out_ll; a.out_E = s->out_E;
  a.out_trace = reinterpret_cast<double*>(s->out_trace);
  a.out_mom = reinterpret_cast<double*>(s->out_mom);

  static const bool prof_on = getenv("HMCX_RS_PROF") && getenv("HMCX_RS_PROF")[0] == '1';
  if (prof_on) {
    HMCX_HIP(ctx, hipMalloc((void**)&a.prof, 16 * sizeof(unsigned long long)));
    HMCX_HIP(ctx, hipMemsetAsync(a.prof, 0, 16 * sizeof(unsigned long long), ctx->stream));
  }
  const void* kfn = (const void*)k_sghmc_rs;
  static bool lds_set = false;
  if (!lds_set) {
    HMCX_HIP(ctx, hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ctx->lds_max));
    lds_set = true;
  }
  int per_cu = 0;
  if ((rc = kernel_occupancy(ctx, kfn, RTH, (int)pl.lds, &per_cu))) return rc;
  if ((long)per_cu * ctx->num_cus < G)
    return set_error(ctx, HMCX_EUNSUPPORTED, "row-space SGHMC: workgroups cannot be co-resident");
  if ((rc = timing_begin(ctx, ctx->stream))) return rc;
  if (!buf) {
    const int npair = (DK + 1) / 2;
    const int gx = std::min(64, (npair * (nmax + 1) + 255) / 256);
    hipLaunchKernelGGL(k_rs_noise, dim3(std::max(gx, 1), (unsigned)n), dim3(256), 0, ctx->stream, pre);
  }
  hipLaunchKernelGGL(k_rs_gemm, dim3(rt * ct, (unsigned)n), dim3(256), 0, ctx->stream, pre);
  void* kargs[] = {&a};
  HMCX_HIP(ctx, hipLaunchKernel(kfn, dim3(G), dim3(RTH), kargs, (unsigned)pl.lds, ctx->stream));
  if ((rc = timing_end(ctx, ctx->stream))) return rc;
  if (a.prof) {
    unsigned long long h[16];
    HMCX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    HMCX_HIP(ctx, hipMemcpy(h, a.prof, sizeof(h), hipMemcpyDeviceToHost));
    (void)hipFree(a.prof);
    unsigned long long tot = 0;
    for (int i = 0; i < 10; ++i) tot += h[i];
    static const char* names[10] = {"step-start loads", "W gather", "Z_0", "proj+ll0", "softmax+publish",
                                    "AG wait", "MFMA", "update", "accept round", "post-accept"};
    fprintf(stderr, "[hmcx rs prof] %d steps, %llu ticks (100 MHz):", (int)n, tot);
    for (int i = 0; i < 10; ++i) fprintf(stderr, " %s %.1f%%", names[i], tot ? 100.0 * h[i] / tot : 0.0);
    fprintf(stderr, "\n");
  }
  if (s->out_abort) {
    HMCX_HIP(ctx, hipMemcpyAsync(s->out_abort, ctx->abort_dev, sizeof(int), hipMemcpyDeviceToDevice, ctx->stream));
    return HMCX_OK;
  }
  return abort_defer(ctx, a.abort_flag, ctx->stream);
}

}  // namespace hmcx
