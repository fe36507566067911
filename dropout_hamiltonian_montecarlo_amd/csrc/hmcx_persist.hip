// hmcx_persist.hip — persistent (one launch per call) SGHMC for the softmax model, C = 1.
//
// Same mathematics and op order as the kernel-per-phase path in hmcx_softmax.hip
// (reference: cpu/sghmc.py:19-39 with the A1 completion, cpu/softmax.py:38-79), re-laid out
// for the latency-bound single-chain case (BASELINE config 2: B=500, D=784, K=10):
//
//  * G = Gr x Gf workgroups, one per CU, co-resident (cooperative launch).  Block (r, f) keeps
//    the minibatch tile X[R_r, F_f] (rows R_r, features F_f) in LDS for a whole step, plus its
//    feature slice of the working weights W[F_f], momentum pW[F_f] and the step-start copy.
//  * Leapfrog iteration = two MFMA GEMM phases with TEAM-local exchanges (no grid-wide sync):
//      A: partial Z = X[R_r,F_f]·W[F_f] → row team r (Gf blocks) reduces in a fixed order →
//         every member holds Z[R_r]; softmax, diff, bias sub-step (b' = b + ε·pb) locally.
//      B: partial Xᵀ·diff over R_r → feature team f (Gr blocks) reduces → every member updates
//         W[F_f], pW[F_f] identically; the bias sub-step's Σ_rows uses the team's row partials.
//    Team barriers: monotone counters, producer stores → vmcnt(0) → release fence → atomic
//    arrive; consumer relaxed poll → acquire fence (cdna_hip_programming.md §6 G16).
//  * Accept (hmc.py:67-71): one grid-wide barrier per step exchanges the kinetic and
//    log-likelihood partials; every block evaluates the same A and decision.
// All reductions run in a fixed order, so every block holds bit-identical copies of the
// shared state, and runs are deterministic.
#include "hmcx_common.h"
#include "hmcx_internal.h"
#include "hmcx_persist.h"
#include <cstdio>
#include <cstdlib>

namespace hmcx {

constexpr int PTH = 512;         // threads per block (8 waves)
constexpr int PNW = PTH / 64;
constexpr long SPIN_LIMIT = 1L << 23;
constexpr int MAXJ = 4;          // per-thread elements of a compact [features][K] slice (= 1 Philox block)
constexpr int MAXT = 8;          // largest team (Gr, Gf <= MAXT, enforced by plan_persist)

// ---- write-through exchange (cdna_hip_programming.md §6 G16, "sc1" form): every store of
// handed-off bytes is a global_store … sc1 and every load of them a global_load … sc1, so the
// barrier needs no release/acquire fence (MI355X_MICROARCH.md, hand-off table row 1).
template <typename V> __device__ inline void st_wt(V* p, V v) {
  if constexpr (sizeof(V) == 8) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), __builtin_bit_cast(unsigned long long, v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    __hip_atomic_store(reinterpret_cast<unsigned*>(p), __builtin_bit_cast(unsigned, v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
}
template <typename V> __device__ inline V ld_wt(const V* p) {
  if constexpr (sizeof(V) == 8) {
    return __builtin_bit_cast(V, __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT));
  } else {
    return __builtin_bit_cast(V, __hip_atomic_load(reinterpret_cast<const unsigned*>(p), __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT));
  }
}

struct Bar {
  unsigned* ctr;
  unsigned gen;
  unsigned members;
};

// Team barrier for write-through exchanges: every wave drains its sc1 stores, then ONE lane
// arrives (agent atomic) and polls (sc1 load); the other waves wait at the workgroup barrier.
// Bounded spin: on timeout or abort it returns false and the kernel exits.
__device__ inline bool team_sync(Bar& b, int* abort_flag, int* sh_ok) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  b.gen += 1;
  if (threadIdx.x == 0) {
    int ok = 1;
    __hip_atomic_fetch_add(b.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned target = b.gen * b.members;
    long spins = 0;
    while (__hip_atomic_load(b.ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if ((++spins & 1023) == 0 &&
          (__hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) || spins > SPIN_LIMIT)) {
        __hip_atomic_store(abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
    }
    *sh_ok = ok;
  }
  __syncthreads();
  return *sh_ok != 0;
}

// out[j] = Σ_{t<n} p[t·stride + idx[j]] (fixed t order) for J elements: all J·MAXT write-through
// loads are issued before the first add (clamped indices, no predicated loads: guide §5 trap (c)).
template <typename V, int J>
__device__ inline void gather_sum(V* out, const V* p, size_t stride, int n, const int* idx) {
  V v[J][MAXT];
#pragma unroll
  for (int j = 0; j < J; ++j)
#pragma unroll
    for (int t = 0; t < MAXT; ++t) v[j][t] = ld_wt(p + (size_t)(t < n ? t : n - 1) * stride + idx[j]);
#pragma unroll
  for (int j = 0; j < J; ++j) {
    V acc = v[j][0];
#pragma unroll
    for (int t = 1; t < MAXT; ++t) acc = (t < n) ? acc + v[j][t] : acc;
    out[j] = acc;
  }
}

// Reductions over a 16-lane group (one softmax row); xor butterfly, identical in every block.
template <typename T> __device__ inline T g16_max(T v) {
#pragma unroll
  for (int m = 8; m >= 1; m >>= 1) v = max_nan(v, __shfl_xor(v, m, 16));
  return v;
}
template <typename T> __device__ inline T g16_sum(T v) {
#pragma unroll
  for (int m = 8; m >= 1; m >>= 1) v = v + __shfl_xor(v, m, 16);
  return v;
}

// Four consecutive noise values starting at element e0 (e0 % 4 == 0): one Philox block.
template <typename T>
__device__ inline void pnoise4(const PersistArgs<T>& a, int s, uint32_t slot, uint32_t e0, T z[4]) {
  if (a.noise_mode == HMCX_NOISE_BUFFER) {
    const double* src = a.noise + a.noff[s] + (int64_t)slot * a.P + e0;
#pragma unroll
    for (int q = 0; q < 4; ++q) z[q] = (e0 + q < (uint32_t)a.P) ? (T)src[q] : T(0);
  } else {
    float zf[4];
    philox_normal4(a.seed, a.chain0, a.step_base + (uint32_t)s, slot, e0 >> 2, zf);
#pragma unroll
    for (int q = 0; q < 4; ++q) z[q] = (T)zf[q];
  }
}

template <typename T>
__device__ inline double pnoise(const PersistArgs<T>& a, int s, uint32_t slot, uint32_t e) {
  if (a.noise_mode == HMCX_NOISE_BUFFER) return a.noise[a.noff[s] + (int64_t)slot * a.P + e];
  return (double)philox_normal(a.seed, a.chain0, a.step_base + (uint32_t)s, slot, e);
}

// In-kernel phase profiler (HMCX_PERSIST_PROF=1): block 0 accumulates s_memtime deltas.
struct Prof {
  unsigned long long* out;
  unsigned long long last = 0;
  int cur = 0;
  __device__ inline void stamp(int next) {
    if (!out) return;
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    if (last) out[cur] += t - last;     // global accumulator: no runtime-indexed register array
    last = t;
    cur = next;
  }
  __device__ inline void flush() {}
};

// Deterministic block sum of per-thread doubles (fixed tree).
__device__ inline double bsum(double v, double* sh) {
  const int t = threadIdx.x;
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);             // butterfly within a wave
  if ((t & 63) == 0) sh[t >> 6] = v;
  __syncthreads();
  double p[PNW];
#pragma unroll
  for (int w = 0; w < PNW; ++w) p[w] = sh[w];                               // all reads in flight
  double r = p[0];
#pragma unroll
  for (int w = 1; w < PNW; ++w) r += p[w];
  __syncthreads();
  return r;
}

// Σ_{t<n} s[t·stride] from LDS with all reads issued first (n <= NMAX, compile-time bound).
template <int NMAX, typename V>
__device__ inline V lds_sum(const V* s, int stride, int n) {
  V v[NMAX];
#pragma unroll
  for (int t = 0; t < NMAX; ++t) v[t] = s[(t < n ? t : 0) * stride];
  V acc = v[0];
#pragma unroll
  for (int t = 1; t < NMAX; ++t) acc = (t < n) ? acc + v[t] : acc;
  return acc;
}

// Minibatch tile X[row0:+nrow, feat0:+nfeat] → LDS [Br][BFP] (zero padded), 16-B loads, 8 in
// flight per thread before their LDS stores.
template <typename T>
__device__ inline void load_tile(T* Xs, const T* Xg, int Br, int Bf, int BFP, int nrow, int nfeat, int row0,
                                 int feat0, int D) {
  constexpr int V = 16 / sizeof(T);
  typedef T vec_t __attribute__((ext_vector_type(V)));
  const int nv = Bf / V;
  const int total = Br * nv;
  const bool vec_ok = (D % V) == 0;
  for (int base = threadIdx.x; base < total; base += 8 * PTH) {
    vec_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = base + u * PTH;
      const int i = e / nv, j = (e - (e / nv) * nv) * V;
      if (e < total && i < nrow && j < nfeat) {
        const T* src = Xg + (size_t)(row0 + i) * D + feat0 + j;
        if (vec_ok) {
          v[u] = *reinterpret_cast<const vec_t*>(src);
        } else {
#pragma unroll
          for (int q = 0; q < V; ++q) v[u][q] = (j + q < nfeat) ? src[q] : T(0);
        }
      } else {
#pragma unroll
        for (int q = 0; q < V; ++q) v[u][q] = T(0);
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = base + u * PTH;
      if (e < total) {
        const int i = e / nv, j = (e - (e / nv) * nv) * V;
#pragma unroll
        for (int q = 0; q < V; ++q) Xs[i * BFP + j + q] = v[u][q];
      }
    }
  }
}

template <typename T>
__global__ __launch_bounds__(PTH) void k_sghmc_persist(PersistArgs<T> a) {
  using M = mfma16<T>;
  extern __shared__ __align__(16) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int G = a.Gr * a.Gf;
  const int bid = blockIdx.x;
  const int r = bid / a.Gf, f = bid - (bid / a.Gf) * a.Gf;
  const int Br = a.Br, Bf = a.Bf, BFP = a.BFP, K = a.K, D = a.D, B = a.B;
  const int row0 = r * Br, feat0 = f * Bf;
  const int nrow = max(0, min(Br, B - row0));
  const int nfeat = max(0, min(Bf, D - feat0));
  const int NWE = Bf * 16;                                  // LDS weight slice (16 padded cols)
  const int NWC = nfeat * K;                                // compact weight-slice elements
  const int NRC = nrow * K;                                 // compact row-tile elements

  // ---- LDS carve-up (sizes mirrored by plan_persist)
  T* Xs = reinterpret_cast<T*>(smem);                       // [Br][BFP] minibatch tile
  T* Wf = Xs + (size_t)Br * BFP;                            // [Bf][16]  working weights (MFMA B operand)
  T* Zs = Wf + NWE;                                         // [Br][16]  XW / scratch
  T* Ds = Zs + Br * 16;                                     // [Br][16]  diff (phase-B operand)
  T* Ys = Ds + Br * 16;                                     // [Br][16]
  T* Es = Ys + Br * 16;                                     // [Br][16]  exponentials / scratch
  T* rs = Es + Br * 16;                                     // [4][Br]   row max / sum at b and b'
  T* bsh = rs + 4 * Br;                                     // [16] b
  T* pbsh = bsh + 16;                                       // [16] pb
  T* b0sh = pbsh + 16;                                      // [16] b at step start
  T* bpsh = b0sh + 16;                                      // [16] b'
  T* cssh = bpsh + 16;                                      // [16] colsum partial of this row team
  size_t off = ((size_t)(reinterpret_cast<char*>(cssh + 16) - smem) + 15) & ~(size_t)15;
  double* dsh = reinterpret_cast<double*>(smem + off);      // [PTH]
  int* ish = reinterpret_cast<int*>(dsh + PTH);             // [4]

  // this thread's compact weight-slice elements ec = 4·tid + j  (i = ec / K, k = ec % K): one
  // Philox block of noise per thread per draw
  int widx[MAXJ], wlds[MAXJ];
  bool wok[MAXJ];
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    const int ec = 4 * tid + j;
    wok[j] = ec < NWC;
    const int i = wok[j] ? ec / K : 0, k = wok[j] ? ec - i * K : 0;
    widx[j] = wok[j] ? ec : 0;
    wlds[j] = i * 16 + k;
  }
  T pw[MAXJ], w0[MAXJ], zn[MAXJ];                           // momentum, step-start W, noise (registers)
  // this thread's compact row-tile elements (phase-A reduce)
  int ridx[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) ridx[j] = min(tid + j * PTH, max(NRC - 1, 0));

  Prof prof;
  prof.out = (bid == 0 && tid == 0) ? a.prof : nullptr;
  Bar rowbar{a.rowc + r, 0u, (unsigned)a.Gf};
  Bar featbar{a.featc + f, 0u, (unsigned)a.Gr};
  Bar globbar{a.globc, 0u, (unsigned)G};
  unsigned useA = 0, useB = 0;

  // ---- initial state: feature slice of W, the bias (identical in every block)
  for (int e = tid; e < NWE; e += PTH) {
    const int i = e >> 4, k = e & 15;
    Wf[e] = (i < nfeat && k < K) ? a.W[(size_t)(feat0 + i) * K + k] : T(0);
  }
  for (int e = tid; e < Br * 16; e += PTH) { Ds[e] = T(0); Zs[e] = T(0); }
  if (tid < 16) bsh[tid] = tid < K ? a.b[tid] : T(0);
  __syncthreads();

  const T hi = (T)CLIP_HI, lo = (T)CLIP_LO;
  const T alpha = a.alpha;

  for (int s = 0; s < a.n_steps; ++s) {
    const double epsd = a.eps[s];
    const T eps = (T)epsd, ome = (T)(1.0 - epsd), nsc = (T)(2.0 * epsd);
    const int n = a.n_iter[s];
    const T* Xg = a.X + (size_t)a.row0[s] * D;
    const T* Yg = a.Y + (size_t)a.row0[s] * K;

    // ---- minibatch tile → LDS; momentum (hmc.py:82-87, drawn identically by all team members)
    prof.stamp(0);
    load_tile<T>(Xs, Xg, Br, Bf, BFP, nrow, nfeat, row0, feat0, D);
    for (int e = tid; e < Br * 16; e += PTH) {
      const int i = e >> 4, k = e & 15;
      Ys[e] = (i < nrow && k < K) ? Yg[(size_t)(row0 + i) * K + k] : T(0);
    }
    double kin = 0.0;
    {
      T z4[4];
      if (4 * tid < NWC) pnoise4(a, s, 0u, (uint32_t)(feat0 * K + 4 * tid), z4);
#pragma unroll
      for (int j = 0; j < MAXJ; ++j) {
        const T p = wok[j] ? z4[j] : T(0);
        kin += (double)p * (double)p;
        pw[j] = p;
        w0[j] = Wf[wlds[j]];
      }
    }
    if (tid < 16) {
      const T p = tid < K ? (T)pnoise(a, s, 0u, (uint32_t)(D * K + tid)) : T(0);
      pbsh[tid] = p;
      b0sh[tid] = bsh[tid];
    }
    const double kin0_f = bsum(kin, dsh);      // Σ p0² over this feature slice (ends with a barrier)
    double kb0 = 0.0;
    {
      const double pv = tid < K ? (double)pbsh[tid] : 0.0;
      kb0 = bsum(pv * pv, dsh);
    }

    double ll0_r = 0.0, ll_last = 0.0;
    // it = -1 evaluates the step-start logits (E_current); it >= 0 are the leapfrog iterations
    for (int it = -1; it < n; ++it) {
      T zb = T(0);
      if (it >= 0) {
        // this iteration's friction noise for the weight slice (sghmc.py:31), off the critical path
        if (4 * tid < NWC) pnoise4(a, s, (uint32_t)(it + 1), (uint32_t)(feat0 * K + 4 * tid), zn);
        if (tid < K) zb = (T)pnoise(a, s, (uint32_t)(it + 1), (uint32_t)(D * K + tid));
      }
      if (it == 0) {
#pragma unroll
        for (int j = 0; j < MAXJ; ++j)
          if (wok[j]) Wf[wlds[j]] = Wf[wlds[j]] + eps * pw[j];                 // sghmc.py:32
        __syncthreads();
      }
      // ================= phase A: partial logits over this feature slice
      prof.stamp(1);
      const int parA = useA & 1;
      ++useA;
      T* exA = a.exA + ((size_t)(parA * a.Gr + r) * a.Gf + f) * Br * K;
      {
        // wave w: tile mt = w % MT over k-part w / MT (split-K when the tiles are fewer than the waves;
        // the two halves meet in LDS: exactly two addends, so the sum is order independent)
        const int MT = Br / 16;
        const int WPT = (2 * MT <= PNW && Bf % 32 == 0) ? 2 : 1;          // halves meet in Zs / Es
        const int kspan = Bf / WPT;
        for (int item = wave; item < MT * WPT; item += PNW) {
          const int mt = item % MT, part = item / MT;
          typename M::acc_t c0 = M::zero(), c1 = M::zero();
          const T* xa = Xs + (mt * 16 + lr) * BFP + lg;
          const T* wb = Wf + lg * 16 + lr;
          const int kbeg = part * kspan, kend = kbeg + kspan;
#pragma unroll 2
          for (int k0 = kbeg; k0 < kend; k0 += 16) {                         // kspan % 16 == 0
            const T a0 = xa[k0], a1 = xa[k0 + 4], a2 = xa[k0 + 8], a3 = xa[k0 + 12];
            const T b0 = wb[k0 * 16], b1 = wb[(k0 + 4) * 16], b2 = wb[(k0 + 8) * 16], b3 = wb[(k0 + 12) * 16];
            c0 = M::fma(a0, b0, c0);
            c1 = M::fma(a1, b1, c1);
            c0 = M::fma(a2, b2, c0);
            c1 = M::fma(a3, b3, c1);
          }
          if (WPT == 1) {
            if (lr < K)
#pragma unroll
              for (int q = 0; q < 4; ++q) st_wt(exA + (mt * 16 + M::row(lane, q)) * K + lr, c0[q] + c1[q]);
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) (part ? Es : Zs)[mt * 256 + M::row(lane, q) * 16 + lr] = c0[q] + c1[q];
          }
        }
        if (WPT > 1) {
          __syncthreads();
          for (int e = tid; e < Br * 16; e += PTH) {
            const int i = e >> 4, k = e & 15;
            if (k >= K) continue;
            st_wt(exA + i * K + k, Zs[e] + Es[e]);
          }
        }
      }
      prof.stamp(2);
      if (!team_sync(rowbar, a.abort_flag, ish)) return;
      prof.stamp(3);   // A-gather
      {  // row team reduce (fixed f order) → XW for rows R_r
        const T* exAr = a.exA + (size_t)(parA * a.Gr + r) * a.Gf * Br * K;
        T z[2];
        gather_sum<T, 2>(z, exAr, (size_t)Br * K, a.Gf, ridx);
        if (prof.out) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
        prof.stamp(11);  // A-scatter
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int ec = tid + j * PTH;
          if (ec < NRC) {
            const int i = ec / K;
            Zs[i * 16 + (ec - i * K)] = z[j];
          }
        }
      }
      if (tid < 16 && it >= 0) bpsh[tid] = bsh[tid] + eps * pbsh[tid];         // b' (bias sub-step)
      __syncthreads();
      prof.stamp(8);   // softmax
      // ---- softmax rows: one 16-lane group per row (lane k = class), reductions by xor-shuffles
      const T* bz = (it < 0) ? b0sh : bsh;
      double llacc = 0.0;
      {
        const int k = lane & 15, grp = tid >> 4;
        const bool kv = k < K;
        const T ninf = -__builtin_inf();
        const T bk = kv ? bz[k] : T(0);
        const T bpk = (kv && it >= 0) ? bpsh[k] : T(0);
        T csacc = T(0);
        for (int i = grp; i < nrow; i += PTH / 16) {
          const T xw = Zs[i * 16 + k];
          const T y = Ys[i * 16 + k];
          const T z = kv ? clipz(xw + bk, hi, lo) : ninf;                     // softmax.py:39-41
          const T m = g16_max(z);                                             // np.max
          const T e = kv ? exp(z - m) : T(0);                                 // softmax.py:34
          const T sm = g16_sum(e);
          if (it < 0) {
            const T lse = log(sm) + m;                                        // logsumexp (softmax.py:18)
            if (kv) llacc += (double)(y * (z - lse));                         // softmax.py:19-20
          } else {
            Ds[i * 16 + k] = kv ? y - e / sm : T(0);                          // diff (softmax.py:52)
            const T z2 = kv ? clipz(xw + bpk, hi, lo) : ninf;                 // bias sub-step at b'
            const T m2 = g16_max(z2);
            const T e2 = kv ? exp(z2 - m2) : T(0);
            const T s2 = g16_sum(e2);
            if (kv) csacc += y - e2 / s2;                                     // Σ_rows (y − ŷ')
            if (it == n - 1) {                                                // ll(q_new): last iteration only
              const T lse2 = log(s2) + m2;
              if (kv) llacc += (double)(y * (z2 - lse2));
            }
          }
        }
        if (it < 0) {
          ll0_r = bsum(llacc, dsh);                                           // ends with a barrier
          continue;
        }
        if (it == n - 1) llacc = bsum(llacc, dsh);
        else __syncthreads();
        csacc += __shfl_xor(csacc, 16, 64);                                   // 4 row groups of a wave
        csacc += __shfl_xor(csacc, 32, 64);
        if (lane < 16) Zs[wave * 16 + k] = csacc;
        __syncthreads();
        if (tid < 16) cssh[tid] = lds_sum<PNW>(Zs + tid, 16, PNW);
        __syncthreads();
      }
      const double ll_r = llacc;

      // ================= phase B: partial Xᵀ·diff over this row slice
      prof.stamp(4);
      const int parB = useB & 1;
      ++useB;
      T* exB = a.exB + ((size_t)(parB * a.Gf + f) * a.Gr + r) * Bf * K;
      for (int mt = wave; mt < Bf / 16; mt += PNW) {
        typename M::acc_t c0 = M::zero(), c1 = M::zero();
        const T* xa = Xs + lg * BFP + mt * 16 + lr;
        const T* db = Ds + lg * 16 + lr;
#pragma unroll 2
        for (int k0 = 0; k0 < Br; k0 += 16) {                                // Br % 16 == 0
          const T a0 = xa[k0 * BFP], a1 = xa[(k0 + 4) * BFP], a2 = xa[(k0 + 8) * BFP], a3 = xa[(k0 + 12) * BFP];
          const T b0 = db[k0 * 16], b1 = db[(k0 + 4) * 16], b2 = db[(k0 + 8) * 16], b3 = db[(k0 + 12) * 16];
          c0 = M::fma(a0, b0, c0);
          c1 = M::fma(a1, b1, c1);
          c0 = M::fma(a2, b2, c0);
          c1 = M::fma(a3, b3, c1);
        }
        // D layout: row (feature) = M::row, col (class) = lr
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int kk = lr;
          if (kk < K) st_wt(exB + (mt * 16 + M::row(lane, q)) * K + kk, c0[q] + c1[q]);
        }
      }
      T* exBc = a.exBcs + ((size_t)(parB * a.Gf + f) * a.Gr + r) * 16;
      if (tid < 16) st_wt(exBc + tid, cssh[tid]);
      if (tid == 0) st_wt(a.exBll + (size_t)(parB * a.Gf + f) * a.Gr + r, ll_r);
      prof.stamp(5);
      if (!team_sync(featbar, a.abort_flag, ish)) return;
      prof.stamp(6);
      const T* exBf = a.exB + (size_t)(parB * a.Gf + f) * a.Gr * Bf * K;
      const bool last = it == n - 1;
      // issue the bias-colsum and log-likelihood partial loads first, then the weight partials:
      // one memory round trip for the whole update
      const T* csb = a.exBcs + (size_t)(parB * a.Gf + f) * a.Gr * 16;
      const double* llb = a.exBll + (size_t)(parB * a.Gf + f) * a.Gr;
      const T csone = ld_wt(csb + (tid < a.Gr * 16 ? tid : 0));
      const double llone = ld_wt(llb + (tid < a.Gr ? tid : 0));
      T dots[MAXJ];
      gather_sum<T, MAXJ>(dots, exBf, (size_t)Bf * K, a.Gr, widx);
      if (tid < a.Gr * 16) Es[tid] = csone;                                  // [r][16] partials → LDS
      if (tid < a.Gr) dsh[tid] = llone;
      if (prof.out) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
      prof.stamp(9);   // B-update
      double kin1 = 0.0;
#pragma unroll
      for (int j = 0; j < MAXJ; ++j) {
        if (!wok[j]) continue;
        const T w = Wf[wlds[j]];
        const T gr = -(dots[j] - alpha * w);                                  // softmax.py:57-58
        const T p = (ome * pw[j] + eps * gr) + nsc * zn[j];                   // sghmc.py:31,34
        pw[j] = p;
        if (!last) Wf[wlds[j]] = w + eps * p;                                 // next drift (:32)
        else kin1 += (double)p * (double)p;
      }
      __syncthreads();
      if (tid < K) {                                                          // bias sub-step (:32-34)
        const T c = lds_sum<MAXT>(Es + tid, 16, a.Gr);
        const T gr = -(c - alpha * bpsh[tid]);
        pbsh[tid] = (ome * pbsh[tid] + eps * gr) + nsc * zb;
        bsh[tid] = bpsh[tid];
      }
      if (last) {
        ll_last = lds_sum<MAXT>(dsh, 1, a.Gr);                                                          // ll(q_new) on this batch
        __syncthreads();                                                      // dsh is reused by bsum
        const double kin1_f = bsum(kin1, dsh);
        if (r == 0 && tid == 0) st_wt(a.exG + ((size_t)(s & 1) * a.Gf + f) * 2 + 1, kin1_f);
      }
      __syncthreads();
    }
    // ================= accept (hmc.py:67-71): one grid barrier for the global energies
    if (r == 0 && tid == 0) st_wt(a.exG + ((size_t)(s & 1) * a.Gf + f) * 2 + 0, kin0_f);
    if (f == 0 && tid == 0) st_wt(a.exL + (size_t)(s & 1) * a.Gr + r, ll0_r);
    prof.stamp(7);
    if (!team_sync(globbar, a.abort_flag, ish)) return;
    prof.stamp(10);  // accept
    double S0, S1 = 0.0, L0;
    {
      int gi[1] = {0};
      gather_sum<double, 1>(&S0, a.exG + (size_t)(s & 1) * a.Gf * 2, 2, a.Gf, gi);
      if (n > 0) gather_sum<double, 1>(&S1, a.exG + (size_t)(s & 1) * a.Gf * 2 + 1, 2, a.Gf, gi);
      gather_sum<double, 1>(&L0, a.exL + (size_t)(s & 1) * a.Gr, 1, a.Gr, gi);
    }
    double kb1 = 0.0;
    {
      const double pv = tid < K ? (double)pbsh[tid] : 0.0;
      kb1 = bsum(pv * pv, dsh);
    }
    const double K0 = (0.0 + 0.5 * S0) + 0.5 * kb0;
    const double Ecur = a.neg_inv_n * (L0 + a.log_prior) + K0;
    double A, Enew, llq;
    int acc;
    if (n <= 0) {
      A = 1.0; Enew = Ecur; llq = L0;
      acc = a.u[s] < A;
    } else {
      const double K1 = (0.0 + 0.5 * S1) + 0.5 * kb1;
      Enew = a.neg_inv_n * (ll_last + a.log_prior) + K1;
      const double x = exp(Ecur - Enew);
      A = (x < 1.0) ? x : 1.0;                                                // Python min(1, x)
      acc = a.u[s] < A;
      llq = acc ? ll_last : L0;
    }
    if (!acc || n <= 0) {                                                     // keep q (sghmc.py:36-38)
#pragma unroll
      for (int j = 0; j < MAXJ; ++j)
        if (wok[j]) Wf[wlds[j]] = w0[j];
      if (tid < 16) bsh[tid] = b0sh[tid];
    }
    if (bid == 0 && tid == 0) {
      a.out_A[s] = A;
      a.out_acc[s] = acc;
      a.out_ll[s] = llq;
      if (a.out_E) { a.out_E[2 * s] = Ecur; a.out_E[2 * s + 1] = Enew; }
    }
    __syncthreads();
  }
  prof.stamp(0);
  prof.flush();
  // ---- write back the committed state
  if (r == 0)
    for (int e = tid; e < nfeat * 16; e += PTH) {
      const int i = e >> 4, k = e & 15;
      if (k < K) a.W[(size_t)(feat0 + i) * K + k] = Wf[e];
    }
  if (bid == 0 && tid < K) a.b[tid] = bsh[tid];
}

// ------------------------------------------------------------------ host side
PersistPlan plan_persist(int B, int D, int K, size_t tsize, int num_cus, size_t lds_max) {
  PersistPlan p{};
  p.ok = false;
  if (K > 16) return p;
  for (int G = 1; G <= num_cus; ++G) {
    // prefer balanced teams: Gf ≈ 1.25 Gr (exchange volume B·Gf/Gr + D·Gr/Gf is minimal near √(D/B))
    for (int Gr = 1; Gr <= G; ++Gr) {
      if (G % Gr) continue;
      const int Gf = G / Gr;
      const int Br = ((B + Gr - 1) / Gr + 15) / 16 * 16;
      const int Bf = ((D + Gf - 1) / Gf + 15) / 16 * 16;
      if ((long)(Gr - 1) * Br >= B || (long)(Gf - 1) * Bf >= D) continue;   // no empty teams
      if (Br * 16 < PTH) continue;                                           // scratch reuse of Zs
      if (Gr > MAXT || Gf > MAXT) continue;                                  // gather_sum width
      if (Bf * K > MAXJ * PTH || Br * K > 2 * PTH) continue;                 // per-thread element slots
      const int BFP = Bf + (tsize == 8 ? 2 : 1);
      const size_t lds = ((tsize * ((size_t)Br * BFP + (size_t)Bf * 16 + 4 * (size_t)Br * 16 + 4 * (size_t)Br + 5 * 16) +
                           15) & ~(size_t)15) + 8 * PTH + 16;
      if (lds > lds_max) continue;
      const double cost = (double)B * Gf / Gr + (double)D * Gr / Gf;
      if (!p.ok || cost < p.cost || (cost == p.cost && G < p.Gr * p.Gf)) {
        p.ok = true; p.Gr = Gr; p.Gf = Gf; p.Br = Br; p.Bf = Bf; p.BFP = BFP; p.lds = lds; p.cost = cost;
      }
    }
    if (p.ok) break;   // smallest G whose tile fits LDS
  }
  return p;
}

template <typename T>
int sghmc_persist_t(hmcx_ctx* ctx, const hmcx_sampler_args* s, const PersistPlan& pl) {
  const int G = pl.Gr * pl.Gf;
  const size_t n = (size_t)s->n_steps;
  Workspace ws(ctx);
  T *exA, *exB, *exBcs;
  double *exBll, *exG, *exL, *d_eps, *d_u;
  int64_t *d_row0, *d_noff;
  int32_t* d_n;
  unsigned* ctrs;
  do {
    ws.reset();
    exA = ws.take<T>((size_t)2 * G * pl.Br * s->K);
    exB = ws.take<T>((size_t)2 * G * pl.Bf * s->K);
    exBcs = ws.take<T>((size_t)2 * G * 16);
    exBll = ws.take<double>((size_t)2 * G);
    exG = ws.take<double>((size_t)2 * pl.Gf * 2);
    exL = ws.take<double>((size_t)2 * pl.Gr);
    d_eps = ws.take<double>(n);
    d_u = ws.take<double>(n);
    d_row0 = ws.take<int64_t>(n);
    d_noff = ws.take<int64_t>(n);
    d_n = ws.take<int32_t>(n);
    ctrs = ws.take<unsigned>(pl.Gr + pl.Gf + 2);
  } while (ws.retry());
  if (ws.failed) return HMCX_ENOMEM;
  begin_call(ctx);
  int rc;
  if ((rc = upload(ctx, d_eps, s->eps, n * sizeof(double)))) return rc;
  if ((rc = upload(ctx, d_u, s->u_accept, n * sizeof(double)))) return rc;
  if ((rc = upload(ctx, d_row0, s->row0, n * sizeof(int64_t)))) return rc;
  if ((rc = upload(ctx, d_n, s->n_iter, n * sizeof(int32_t)))) return rc;
  if (s->noise_mode == HMCX_NOISE_BUFFER && (rc = upload(ctx, d_noff, s->noise_off, n * sizeof(int64_t)))) return rc;
  HMCX_HIP(ctx, hipMemsetAsync(ctrs, 0, (pl.Gr + pl.Gf + 2) * sizeof(unsigned), ctx->stream));

  PersistArgs<T> a{};
  a.X = (const T*)s->X; a.Y = (const T*)s->Y;
  a.B = s->B; a.D = s->D; a.K = s->K; a.P = s->D * s->K + s->K;
  a.n_steps = s->n_steps;
  a.Gr = pl.Gr; a.Gf = pl.Gf; a.Br = pl.Br; a.Bf = pl.Bf; a.BFP = pl.BFP;
  a.alpha = (T)s->alpha; a.neg_inv_n = -1.0 / (double)s->B; a.log_prior = s->log_prior;
  a.eps = d_eps; a.u = d_u; a.row0 = d_row0; a.n_iter = d_n;
  a.noise_mode = s->noise_mode; a.noise = s->noise; a.noff = d_noff;
  a.seed = s->seed; a.chain0 = s->chain0; a.step_base = s->step_base;
  a.W = (T*)s->W; a.b = (T*)s->b;
  a.exA = exA; a.exB = exB; a.exBcs = exBcs; a.exBll = exBll; a.exG = exG; a.exL = exL;
  a.rowc = ctrs; a.featc = ctrs + pl.Gr; a.globc = ctrs + pl.Gr + pl.Gf;
  a.abort_flag = reinterpret_cast<int*>(ctrs + pl.Gr + pl.Gf + 1);
  a.out_A = s->out_A; a.out_acc = s->out_accepted; a.out_ll = s->out_ll; a.out_E = s->out_E;
  static const bool prof_on = getenv("HMCX_PERSIST_PROF") && getenv("HMCX_PERSIST_PROF")[0] == '1';
  unsigned long long* dprof = nullptr;
  if (prof_on) {
    HMCX_HIP(ctx, hipMalloc((void**)&dprof, 16 * sizeof(unsigned long long)));
    HMCX_HIP(ctx, hipMemsetAsync(dprof, 0, 16 * sizeof(unsigned long long), ctx->stream));
  }
  a.prof = dprof;

  HMCX_HIP(ctx, hipFuncSetAttribute((const void*)k_sghmc_persist<T>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)pl.lds));
  void* kargs[] = {&a};
  if ((rc = timing_begin(ctx, ctx->stream))) return rc;
  int per_cu = 0;
  HMCX_HIP(ctx, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_sghmc_persist<T>, PTH, pl.lds));
  if ((long)per_cu * ctx->num_cus < G)
    return set_error(ctx, HMCX_EUNSUPPORTED, "persistent SGHMC: workgroups cannot be co-resident");
  HMCX_HIP(ctx, hipLaunchKernel((const void*)k_sghmc_persist<T>, dim3(G), dim3(PTH), kargs, (unsigned)pl.lds,
                                ctx->stream));
  if ((rc = timing_end(ctx, ctx->stream))) return rc;
  // the abort flag is checked synchronously: a timed-out barrier must not pass silently
  int flag = 0;
  HMCX_HIP(ctx, hipMemcpyAsync(&flag, a.abort_flag, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  HMCX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if ((rc = timing_collect(ctx))) return rc;
  if (dprof) {
    unsigned long long h[16];
    HMCX_HIP(ctx, hipMemcpy(h, dprof, sizeof(h), hipMemcpyDeviceToHost));
    (void)hipFree(dprof);
    unsigned long long tot = 0;
    for (int i = 0; i < 12; ++i) tot += h[i];
    static const char* names[12] = {"tile+momentum", "A-mfma+publish", "A-barrier", "A-gather", "B-mfma+publish",
                                    "B-barrier", "B-gather", "accept-barrier", "softmax+colsum", "B-update+noise",
                                    "accept", "A-scatter"};
    fprintf(stderr, "[hmcx persist prof] G=%dx%d Br=%d Bf=%d total %llu ticks:", pl.Gr, pl.Gf, pl.Br, pl.Bf, tot);
    for (int i = 0; i < 12; ++i) fprintf(stderr, " %s %.1f%%", names[i], tot ? 100.0 * h[i] / tot : 0.0);
    fprintf(stderr, "\n");
  }
  if (flag) return set_error(ctx, HMCX_EHIP, "persistent SGHMC: team barrier timed out (blocks not co-resident?)");
  return HMCX_OK;
}

template int sghmc_persist_t<float>(hmcx_ctx*, const hmcx_sampler_args*, const PersistPlan&);
template int sghmc_persist_t<double>(hmcx_ctx*, const hmcx_sampler_args*, const PersistPlan&);

}  // namespace hmcx
