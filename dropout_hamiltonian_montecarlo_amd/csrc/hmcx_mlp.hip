// hmcx_mlp.hip — the reference's dropout MLP (config 3) on gfx950: gradient, loss and fused SGHMC.
//
// Reference: hamiltonian/models/gpu/mlp.py:19-31 (MyNetwork: relu(dropout(l1 x)) → relu(dropout(l2 ·))
// → l3(dropout(·)), dropout ratio 0.1 in train mode) and :47-82 (grad = ∇ mean softmax-CE + ½αθ,
// log_likelihood returns the mean CE, nlp = loss + log_prior).  Chainer/CuPy are not available, so
// the arithmetic follows the NumPy restatement in oracle/models.py::mlp (parity with injected masks).
//
// Names: xw = X·W1ᵀ, a1 = xw + b1, h1 = max(a1·m0, 0), h2 = max((h1·W2ᵀ + b2)·m1, 0), d3 = h2·m2,
// z = d3·W3ᵀ + b3; m0, m1, m2 are the three dropout masks of one forward ([B][n_mid] each).
// xw is stored without the bias, so a move of b1 never re-runs the 784-deep layer-1 GEMM: every
// consumer forms a1 = xw + b1 on the fly (the same rounding as the reference's X·W1ᵀ + b1).
//
// Kernels:
//  * k_mm<T, EPI, AOP, BOP, ...>: C = op(A)·op(B) on v_mfma_*_16x16x4, 32x32 output tile per
//    workgroup, K split over its 8 waves (three k chunks in flight per wave, 16-byte vector loads
//    along k for k-contiguous operands, fixed-order LDS combine).  OP_H1 builds h1 from xw, b1 and
//    m0 on the fly (h1 is never stored).  Epilogues: layer 2 (bias, dropout, relu, next dropout →
//    h2, d3); layer 3 + softmax cross-entropy, which in the same workgroup also forms ga2 (the
//    layer-2 backward) and the row-block partials of the b2 / b3 / W3 gradients; the layer-1
//    backward ga1 (+ b1 partials); the weight gradients with the gradient + prior or the SGHMC
//    epilogue (sghmc.py:31-34), which also writes the NEXT iteration's drifted position into the
//    other half of a double buffer (no drift launch).
//  * Deferred updates: the gradient of a bias (or of W3) is a sum of per-row-block partials; its
//    gradient / SGHMC update runs in the prologue of whatever kernel is launched next (none of them
//    reads the momentum or the next-position buffer it writes) — no reduction launch.
//  * k_mlp_start (k_mlp_init + keep_flags) / k_sumsq12 / k_mlp_accept / k_mlp_commit: momentum draw,
//    first drift and energy partials together with the keep flags of every dropout mask of the step
//    (Philox), end-of-trajectory energy partials, MH accept (hmc.py:67-79), commit on accept.
//  * Batched iterations (mlp_sghmc_t): the six sub-steps of a leapfrog iteration only depend on the
//    previous iteration, so their kernels go out as multi-problem launches (k_mmb, blockIdx.z = sub-step)
//    and one dual launch (k_mm2: layer-1 backwards + W2 gradient); ≈1.0 GFLOP per iteration at
//    784-256-256-10, B = 500 (layer 1 runs once, after W1 moved), 5 launches per iteration (11 one
//    sub-step at a time).
#include "hmcx_common.h"
#include "hmcx_internal.h"
#include "hmcx_granule.h"
#include <type_traits>
#include <algorithm>
#include <vector>
#include <cstring>

namespace hmcx {

// Mask slots live above the noise slots (0 = momentum, it+1 = iteration it) of the same counter space.
constexpr uint32_t MASK_SLOT0 = 0x80000000u;
constexpr int NPART = 256;    // blocks per variable (grid.x) and energy partials per variable
constexpr int MM_NW = 8;      // waves per k_mm workgroup; the K range is split over them
constexpr int MM_NT = MM_NW * 64;

// Dropout masks of one forward: m0, m1, m2 at offsets 0, mn, 2·mn.
template <typename T> struct MaskSrc {
  const T* vals;          // explicit mask values (API / BUFFER mode), or
  const uint32_t* keep;   // keep flags, one bit per element (bit e % 32 of word e / 32): value = keep ? scale : 0;
                          // neither vals nor keep: no dropout or MK_PHILOX
  T scale;
  int mn;
  // MK_PHILOX: the keep flags are drawn where they are used — element e = which·mn + i is bit e % 64 of
  // keep_group(e / 64) under (seed, slot, step, chain), the values k_mlp_start and hmcx_mlp_masks give
  uint64_t seed; uint32_t chain, step, slot;
};

// Dropout keep flags (Chainer, mlp.py:30-31: keep iff u >= ratio 0.1, u a 24-bit float32 uniform — keep iff
// x >= 0x19999A for x uniform on [0, 2^24)), 64 elements per group G of one forward's flag space: element
// 64G + p is bit p of {lo, hi} (bit p % 32 of word p / 32: the keep-word layout).  Its x takes its top byte
// from byte p / 8 % 4 of word 8·(p / 32) + p % 8 of blocks 4G … 4G + 3 = Philox4x32-10({4G + k, slot, step,
// chain}, seed) (word k·4 + q of the group = word q of block k): a byte below 0x19 drops, above keeps;
// a byte equal to 0x19 (p = 1/256) takes x's low 16 bits from the fallback blocks Philox({0x80000000 |
// 8G + j, slot, step, chain}) — the a-th such element of the group (ascending p) reads 16-bit half a % 8
// (low half first) of block j = a / 8 — and keeps iff they are >= 0x999A.  Exactly the 24-bit law, at 16
// flags per Philox block plus about one fallback block per group (the round-5 form drew 4 per block).
// Host twin: tests/test_gpu_mlp.py::_keep_group_host.
__host__ __device__ inline uint32_t bytes_gt19(uint32_t w) {       // bit 8b + 7: byte b > 0x19
  return (((w & 0x7F7F7F7Fu) + 0x66666666u) | w) & 0x80808080u;
}
__host__ __device__ inline uint32_t bytes_eq19(uint32_t w) {       // bit 8b + 7: byte b == 0x19
  const uint32_t z = w ^ 0x19191919u;
  return ~(((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z) & 0x80808080u;
}
struct KeepGroup { uint32_t lo, hi; };
__host__ __device__ inline KeepGroup keep_group(uint64_t seed, uint32_t G, uint32_t slot, uint32_t step,
                                                uint32_t chain) {
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  uint32_t f0 = 0, f1 = 0, a0 = 0, a1 = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const u32x4 r = philox4x32_10(u32x4{{4u * G + (uint32_t)k, slot, step, chain}}, k0, k1);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = (k & 1) * 4 + q;                           // word of the half: bits 8b + j
      const uint32_t gt = bytes_gt19(r.v[q]) >> (7 - j), eq = bytes_eq19(r.v[q]) >> (7 - j);
      if (k < 2) { f0 |= gt; a0 |= eq; } else { f1 |= gt; a1 |= eq; }
    }
  }
  for (uint32_t j = 0; (a0 | a1) != 0u; ++j) {                 // at most 8 blocks (64 ambiguous bytes)
    const u32x4 r = philox4x32_10(u32x4{{0x80000000u | (G << 3) | j, slot, step, chain}}, k0, k1);
#pragma unroll
    for (int h = 0; h < 8; ++h) {
      const bool keep = ((r.v[h >> 1] >> (16 * (h & 1))) & 0xFFFFu) >= 0x999Au;
      if (a0) {
        const uint32_t low = a0 & (0u - a0);
        if (keep) f0 |= low;
        a0 ^= low;
      } else if (a1) {
        const uint32_t low = a1 & (0u - a1);
        if (keep) f1 |= low;
        a1 ^= low;
      }
    }
  }
  return KeepGroup{f0, f1};
}
// Keep flags of a step's forwards, one bit per element (bit e % 32 of word e / 32; forward f's words start
// at f·⌈n3/32⌉): work item gi = fl·⌈n3/64⌉ + G draws keep_group(G) of forward f (slot MASK_SLOT0 + f) and
// stores its two words (flags past n3 zero).  The nf forwards drawn: f = f0 + fl for fl < nlo, then
// fhi + (fl − nlo) — a contiguous range, or one range and the step's two energy forwards.
struct KeepRange { int nf, f0, nlo, fhi; };
__device__ inline void keep_flags(uint32_t* keep, int n3, KeepRange kr, uint64_t seed, uint32_t chain, uint32_t step,
                                  size_t gi) {
  const int W = (n3 + 31) / 32, ng = (n3 + 63) / 64;
  if (gi >= (size_t)kr.nf * ng) return;
  const int fl = (int)(gi / (size_t)ng), G = (int)(gi - (size_t)fl * ng);
  const int f = fl < kr.nlo ? kr.f0 + fl : kr.fhi + (fl - kr.nlo);
  const KeepGroup k = keep_group(seed, (uint32_t)G, MASK_SLOT0 + (uint32_t)f, step, chain);
  const int e0 = 64 * G;
  const uint32_t lo = n3 - e0 >= 32 ? k.lo : k.lo & ((1u << (n3 - e0)) - 1u);
  const uint32_t hi = n3 - e0 >= 64 ? k.hi : n3 - e0 > 32 ? k.hi & ((1u << (n3 - e0 - 32)) - 1u) : 0u;
  uint32_t* dst = keep + (size_t)f * W + 2 * G;
  dst[0] = lo;
  if (2 * G + 1 < W) dst[1] = hi;
}

// the keep word (32 flags) holding element e of a MK_PHILOX source: bit e % 32
template <typename T> __device__ inline uint32_t philox_keep_word(const MaskSrc<T>& s, size_t e) {
  const KeepGroup g = keep_group(s.seed, (uint32_t)(e >> 6), s.slot, s.step, s.chain);
  return (e & 32) ? g.hi : g.lo;
}

// Where the masks come from is a compile-time parameter (MK) of every kernel that reads them, so a
// mask read is one load of the one source (MK_KEEP / MK_VALS), a Philox draw (MK_PHILOX) or nothing.
// Loaded values are pinned by an empty asm after the batch they belong to, so hipcc cannot sink
// a load into a branch (which it then waits for on the spot).
enum MaskKind { MK_NONE = 0, MK_KEEP = 1, MK_VALS = 2, MK_PHILOX = 3 };
template <typename T> struct MRaw { T v; uint32_t k; };
template <typename T, int MK> __device__ inline MRaw<T> mraw(const MaskSrc<T>& s, int which, size_t i) {
  MRaw<T> r{T(1), 1u};
  const size_t e = (size_t)which * s.mn + i;
  if constexpr (MK == MK_KEEP) r.k = (s.keep[e >> 5] >> (e & 31)) & 1u;
  if constexpr (MK == MK_VALS) r.v = s.vals[e];
  if constexpr (MK == MK_PHILOX) r.k = (philox_keep_word(s, e) >> (e & 31)) & 1u;
  return r;
}
template <typename T, int MK> __device__ inline void mpin(MRaw<T>& r) {
  if constexpr (MK == MK_KEEP) asm volatile("" : "+v"(r.k));
  if constexpr (MK == MK_VALS) asm volatile("" : "+v"(r.v));
}
template <typename T, int MK> __device__ inline T mfin(const MaskSrc<T>& s, const MRaw<T>& r) {
  if constexpr (MK == MK_KEEP || MK == MK_PHILOX) return r.k ? s.scale : T(0);
  else if constexpr (MK == MK_VALS) return r.v;
  else return T(1);
}
template <typename T, int MK> __device__ inline T mval(const MaskSrc<T>& s, int which, size_t i) {
  MRaw<T> r = mraw<T, MK>(s, which, i);
  mpin<T, MK>(r);
  return mfin<T, MK>(s, r);
}
// V consecutive mask values from an element index that is a multiple of V (V = 16 / sizeof T)
template <typename T, int V, int MK> __device__ inline void mvals(const MaskSrc<T>& s, int which, size_t i, T (&m)[V]) {
  const size_t e = (size_t)which * s.mn + i;
  if constexpr (MK == MK_VALS) {
    T v[V];
#pragma unroll
    for (int q = 0; q < V; ++q) v[q] = s.vals[e + q];
#pragma unroll
    for (int q = 0; q < V; ++q) asm volatile("" : "+v"(v[q]));
#pragma unroll
    for (int q = 0; q < V; ++q) m[q] = v[q];
  } else if constexpr (MK == MK_KEEP) {
    uint32_t k = s.keep[e >> 5];                                 // e % V == 0: V bits of one word
    asm volatile("" : "+v"(k));
    k >>= (e & 31);
#pragma unroll
    for (int q = 0; q < V; ++q) m[q] = ((k >> q) & 1u) ? s.scale : T(0);
  } else if constexpr (MK == MK_PHILOX) {                        // e % V == 0: V bits of one keep word
    const uint32_t k = philox_keep_word(s, e) >> (e & 31);
#pragma unroll
    for (int q = 0; q < V; ++q) m[q] = ((k >> q) & 1u) ? s.scale : T(0);
  } else {
#pragma unroll
    for (int q = 0; q < V; ++q) m[q] = T(1);
  }
}

// Gradient + prior (mlp.py:63) or the SGHMC momentum update (sghmc.py:31,34) of one variable.
template <typename T> struct Upd {
  const T* W; T* P; T* Qn; T* G;     // θ, momentum, next drifted θ (or null), gradient output (GRAD)
  T half_alpha, eps, one_minus_eps, noise_scale;
  int noise_mode; const double* noise;
  uint64_t seed; uint32_t chain, step, slot, e0;
};
enum UpdMode { UPD_NONE = 0, UPD_GRAD = 1, UPD_SGHMC = 2 };

template <typename T>
__device__ inline void apply_upd(const Upd<T>& u, int mode, size_t i, T v) {
  if (mode == UPD_GRAD) {
    u.G[i] = v + u.half_alpha * u.W[i];
  } else {
    const T g = v + u.half_alpha * u.W[i];
    const T z = u.noise_mode == HMCX_NOISE_BUFFER ? (T)u.noise[i]
                                                  : philox_normal_t<T>(u.seed, u.chain, u.step, u.slot, u.e0 + (uint32_t)i);
    const T p = (u.one_minus_eps * u.P[i] + u.eps * g) + u.noise_scale * z;
    u.P[i] = p;
    if (u.Qn) u.Qn[i] = u.W[i] + u.eps * p;                   // sghmc.py:32 of the next iteration
  }
}

// A gradient given as nparts row-block partials [nparts][n], applied by the next kernel's prologue.
template <typename T> struct Pending {
  int mode, n, nparts;
  const T* part;
  Upd<T> u;
};
// the update of element i: the sum of its partials in fixed order (in-order sum of batches of 16 loads
// that all go out before it: one memory round trip per 16 partials instead of one per partial)
template <typename T>
__device__ inline void pending_elem(const Pending<T>& pd, int i) {
  constexpr int PB = 16;                                       // partials loaded per batch
  T s = T(0);
  if (pd.nparts == 4) {                                        // a split-K weight gradient (W2): 4 partials
    T v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = pd.part[(size_t)q * pd.n + i];
    s = ((v[0] + v[1]) + v[2]) + v[3];
    apply_upd(pd.u, pd.mode, i, s);
    return;
  }
  for (int b0 = 0; b0 < pd.nparts; b0 += PB) {
    T v[PB];
#pragma unroll
    for (int q = 0; q < PB; ++q) v[q] = pd.part[(size_t)min(b0 + q, pd.nparts - 1) * pd.n + i];   // clamped, unconditional
#pragma unroll
    for (int q = 0; q < PB; ++q)
      if (b0 + q < pd.nparts) s = (b0 + q == 0) ? v[q] : s + v[q];
  }
  apply_upd(pd.u, pd.mode, i, s);
}
// bid / nb: this workgroup's index among the nb workgroups that share the work (pending_elem's arithmetic,
// written out: routed through pending_elem, the sampler's pending planes measured 0.4 % slower)
template <typename T>
__device__ inline void run_pending(const Pending<T>& pd, int bid, int nb) {
  if (pd.mode == UPD_NONE) return;
  const int nthr = nb * blockDim.x;
  constexpr int PB = 16;                                       // partials loaded per batch
  for (int i = bid * blockDim.x + threadIdx.x; i < pd.n; i += nthr) {
    // all loads of a batch go out before the (in-order) sum: one memory round trip per 16
    // partials instead of one per partial
    T s = T(0);
    if (pd.nparts == 4) {                                      // a split-K weight gradient (W2): 4 partials
      T v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = pd.part[(size_t)q * pd.n + i];
      s = ((v[0] + v[1]) + v[2]) + v[3];
      apply_upd(pd.u, pd.mode, i, s);
      continue;
    }
    for (int b0 = 0; b0 < pd.nparts; b0 += PB) {
      T v[PB];
#pragma unroll
      for (int q = 0; q < PB; ++q) v[q] = pd.part[(size_t)min(b0 + q, pd.nparts - 1) * pd.n + i];   // clamped, unconditional
#pragma unroll
      for (int q = 0; q < PB; ++q)
        if (b0 + q < pd.nparts) s = (b0 + q == 0) ? v[q] : s + v[q];
    }
    apply_upd(pd.u, pd.mode, i, s);
  }
}
// The pending updates a launch applies first (up to four: the bias / W3 sub-steps of one batched
// iteration).  A batched launch (blockIdx.z = problem) runs them in an extra plane of workgroups of
// their own, z = number of problems, beside the problems.
constexpr int MAXPEND = 4;
template <typename T> struct PendSet {
  Pending<T> p[MAXPEND];
  int n;
};
// With at least one workgroup per update, update j gets its own share of the workgroups (they run side
// by side: each is a short chain of partial loads, a Philox draw and stores); otherwise every
// workgroup runs them in turn.
template <typename T>
__device__ inline void run_pendset(const PendSet<T>& ps, int bid, int nb) {
  if (ps.n == 0) return;
  const bool split = nb >= ps.n;
  const int per = split ? nb / ps.n : nb;
#pragma unroll
  for (int j = 0; j < MAXPEND; ++j)
    if (j < ps.n) {
      if (!split) {
        run_pending(ps.p[j], bid, nb);
      } else {
        const int lo = j * per, hi = j == ps.n - 1 ? nb : lo + per;
        if (bid >= lo && bid < hi) run_pending(ps.p[j], bid - lo, hi - lo);
      }
    }
}
template <typename T>
__global__ __launch_bounds__(256) void k_pending(PendSet<T> ps) {
  run_pendset(ps, (int)(blockIdx.y * gridDim.x + blockIdx.x), (int)(gridDim.x * gridDim.y));
}

enum MMEpi { MM_STORE = 0, MM_L2 = 1, MM_L3CE = 2, MM_GA1 = 3, MM_UPD = 4, MM_L23 = 5 };
enum MMOp { OP_PLAIN = 0, OP_H1 = 1 };

template <typename T> struct MMArgs {
  int M, N, K;
  const T* A; int lda, ta;           // A(m,k) = ta ? A[k·lda + m] : A[m·lda + k]
  const T* B; int ldb, tb;           // B(k,n) = tb ? B[n·ldb + k] : B[k·ldb + n]
  T* C; int ldc;                     // output [M][ldc]
  const T* bias;                     // L2: b2, L3CE: b3
  const T* b1;                       // OP_H1 / GA1: layer-1 bias
  MaskSrc<T> ms;
  const T* H;                        // GA1: xw (the relu gate is (xw + b1)·m0 > 0)
  T* C2;                             // L2: d3
  T* colpart;                        // GA1: b1 partials [gridDim.x][ldc]
  // L3CE extras (per 32-row block): loss, ga2 and the b2 / b3 / W3 gradient partials
  double* lpart; const int32_t* y;
  const T* W3; const T* h2; const T* d3; int n_mid;
  T* ga2; T* pb2; T* pb3; T* pw3;
  int upd_mode; Upd<T> u;            // MM_UPD
  PendSet<T> pend;                   // run first, by the whole grid
  // MM_L23 (layer 2 + layer 3 in one launch): the 32 × n_out logit partials of the column-slice
  // workgroups of one row block meet in a tagged-granule arena (see k_mm)
  char* gx; int gx_bytes; unsigned ep; int* abort_flag;
  int N3; const T* bias3; T* gz;     // n_out, b3 and the gz output of the fused layer 3
  T* h1out;                          // MM_L23: store the slice's columns of h1 = max((xw + b1)·m0, 0)
  const T* H1;                       // MM_GA1: the gate from a stored h1 (no mask reads)
  int force_abort;                   // test knob (HMCX_MLP_FORCE_ABORT): raise the abort word, skip the publish
  unsigned long long* prof;          // HMCX_MLP_PROF: per-workgroup s_memrealtime stamps of the MM_L23 phases
  int xmap, xbx, xby;                // GEMM plane placement over the XCDs (xcd_place): 0 dispatch order, 1 y-major
                                     // chunks, 2 xbx × xby tile blocks, one per XCD
};
constexpr int L23_NPH = 12;          // stamps per workgroup and launch (prof)

// Batched launches: several independent problems of one kernel in one grid, problem = blockIdx.z.
// The sub-steps of one leapfrog iteration are independent of each other (see mlp_sghmc_t), so their
// fused forwards (MM_L23) and layer-1 backwards (MM_GA1) go out as one launch each; a problem
// overrides the operands, masks and outputs of the shared MMArgs (dimensions, X, labels, xw shared).
constexpr int MAXPROB = 6;
template <typename T> struct MMProb {
  const T* A; const T* B; T* C;
  const T* b1; const T* bias; const T* W3; const T* bias3;
  MaskSrc<T> ms;
  T* ga2; T* pb2; T* pb3; T* pw3; T* gz; double* lpart; T* colpart;
  char* gx;                          // MM_L23: the problem's own region of the granule arena
  const T* H1;                       // MM_GA1: the gate from this problem's stored h1 (null: from xw, b1, m0)
};
template <typename T, int NP> struct MMProbsN {
  MMProb<T> p[NP];
  int n;                             // 0: a plain launch
};
template <typename T> using MMProbs = MMProbsN<T, MAXPROB>;
template <typename T> using MMProbs3 = MMProbsN<T, 4>;   // the sub-grids of a dual launch (up to 4 problems)

template <typename T, int OP>
__device__ inline T op_apply(T x, T mask, T bias) {
  if constexpr (OP == OP_H1) {
    const T t = (x + bias) * mask;                             // h1 = max((xw + b1)·m0, 0)
    return t > T(0) ? t : T(0);
  }
  return x;
}

// k offset, inside a 16-wide k chunk, of MFMA step u (0..3) for lane group lg: each lane's k values
// are contiguous (4 floats / 2+2 doubles), so a k-contiguous operand is one or two 16-byte loads.
template <typename T> __device__ inline int kmap(int u, int lg);
template <> __device__ inline int kmap<float>(int u, int lg) { return 4 * lg + u; }
template <> __device__ inline int kmap<double>(int u, int lg) { return ((u >> 1) << 3) + 2 * lg + (u & 1); }

// Operand values of one 16-k chunk for rows (A) / columns (B) r0 + 16·i + lr, i = 0, 1:
// x[u][i] = Op(r, k0 + kmap(u, lg)).  TR: element (r, k) at P[k·ld + r], else P[r·ld + k].
// VEC (requires !TR, ld % (16/sizeof T) == 0 and a 16-byte aligned P): 16-byte vector loads along k.
// OP_H1 masks index the stored matrix (element idx); its bias column is TR ? r : k.
template <typename T, int OP, int TR, int VEC, int MK>
__device__ inline void load_chunk(T (&x)[4][2], const T* P, int ld, int r0, int R, int k0, int ke, int lr, int lg,
                                  const MaskSrc<T>& ms, const T* b1) {
  if constexpr (!VEC) {
    // scalar path: all 8 operand loads (+ masks and b1 for OP_H1) of the chunk go out first
    T pv[2][4], bv[2][4];
    MRaw<T> mr[2][4];
    bool okv[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = r0 + 16 * i + lr;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = k0 + kmap<T>(u, lg);
        const bool ok = r < R && k < ke;
        const size_t idx = ok ? (TR ? (size_t)k * ld + r : (size_t)r * ld + k) : 0;
        okv[i][u] = ok;
        pv[i][u] = P[idx];
        if constexpr (OP == OP_H1) {
          mr[i][u] = mraw<T, MK>(ms, 0, idx);
          bv[i][u] = b1[ok ? (TR ? r : k) : 0];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if constexpr (OP == OP_H1) mpin<T, MK>(mr[i][u]);
        const T mv = OP == OP_H1 ? mfin<T, MK>(ms, mr[i][u]) : T(1);
        const T bb = OP == OP_H1 ? bv[i][u] : T(0);
        x[u][i] = okv[i][u] ? op_apply<T, OP>(pv[i][u], mv, bb) : T(0);
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = r0 + 16 * i + lr;
    const bool rok = r < R;
    if constexpr (VEC) {
      // VEC also requires K % V == 0 (host), so a vector lies entirely inside [k0, ke) or entirely
      // outside it.  Every load is unconditional (clamped address, zeroed afterwards): a load under
      // a branch makes hipcc wait for it before the next one, which serialises the k chunks.
      constexpr int V = 16 / sizeof(T);
#pragma unroll
      for (int h = 0; h < 4 / V; ++h) {                        // f32: one float4; f64: two double2
        const int kv = k0 + (sizeof(T) == 8 ? 8 * h + 2 * lg : 4 * lg);
        const bool ok = rok && kv < ke;
        const size_t base = ok ? (size_t)r * ld + kv : 0;
        T v[V], m[V], bb[V];
        if constexpr (V == 4) {
          const float4 w = *reinterpret_cast<const float4*>(P + base);
          v[0] = w.x; v[1] = w.y; v[2] = w.z; v[3] = w.w;
        } else {
          const double2 w = *reinterpret_cast<const double2*>(P + base);
          v[0] = w.x; v[1] = w.y;
        }
        if constexpr (OP == OP_H1) {
          mvals<T, V, MK>(ms, 0, base, m);
#pragma unroll
          for (int q = 0; q < V; ++q) bb[q] = b1[ok ? kv + q : q];
        }
#pragma unroll
        for (int q = 0; q < V; ++q) x[h * V + q][i] = ok ? op_apply<T, OP>(v[q], m[q], bb[q]) : T(0);
      }
    }
  }
}

// Softmax cross-entropy of the rows of one 32-row block held in LDS zt[32][zs] (F.softmax_cross_entropy,
// mean): gz = (softmax − onehot)/M replaces z in LDS and goes to gz[m][ldg]; lpart[blk] = Σ −log p[y].
template <typename T>
__device__ inline void ce_rows(T* zt, int zs, double* rowl, int m0, int M, int N, const int32_t* y, T* gz, int ldg,
                               double* lpart, int blk, bool writer = true) {
  const int t = threadIdx.x;
  if (t < 32) {
    T* zr = zt + t * zs;
    const int m = m0 + t;
    double l = 0.0;
    if (m < M) {
      T mx = zr[0];
      for (int k = 1; k < N; ++k) mx = zr[k] > mx ? zr[k] : mx;
      T s = T(0);
      for (int k = 0; k < N; ++k) s += exp(zr[k] - mx);
      const T ls = log(s);
      const int lab = y[m];
      l = -(double)((zr[lab] - mx) - ls);
      for (int k = 0; k < N; ++k) {
        T g = exp((zr[k] - mx) - ls);
        if (k == lab) g -= T(1);
        g = g / (T)M;
        zr[k] = g;
        if (writer) gz[(size_t)m * ldg + k] = g;
      }
    } else {
      for (int k = 0; k < N; ++k) zr[k] = T(0);
    }
    rowl[t] = l;
  }
  __syncthreads();
  if (t == 0 && writer) {
    double s = 0.0;
    for (int r = 0; r < 32; ++r) s += rowl[r];
    lpart[blk] = s;
  }
}

// ce_rows with the classes of a row spread over LPR lanes (LPR ≥ N; 16 or 32): max, Σexp and the
// label's log-probability by lane butterflies instead of serial loops over LDS, the row's label
// already in a register (yv[pass], loaded at kernel start).  Same formula as ce_rows (F.softmax_
// cross_entropy, mean): gz = (exp((z − max) − log Σ) − onehot)/M; lpart[blk] = Σ_rows −log p[y].
template <typename T, int LPR>
__device__ inline void ce_rows_lanes(T* zt, int zs, double* rowl, int m0, int M, int N, const int32_t (&yv)[2],
                                     T* gz, int ldg, double* lpart, int blk, bool writer) {
  constexpr int RPP = MM_NT / LPR;                               // rows per pass
  const int t = threadIdx.x, k = t % LPR;
#pragma unroll
  for (int pass = 0; pass < 32 / RPP; ++pass) {
    const int r = pass * RPP + t / LPR, m = m0 + r;
    const bool kin = k < N;
    const T z = kin ? zt[r * zs + k] : T(0);
    T mx = kin ? z : -INFINITY;
#pragma unroll
    for (int w = LPR / 2; w >= 1; w >>= 1) {                      // NaN propagates as in np.max
      const T o = __shfl_xor(mx, w, LPR);
      mx = (o > mx || o != o) ? o : mx;
    }
    T e = kin ? exp(z - mx) : T(0);
#pragma unroll
    for (int w = LPR / 2; w >= 1; w >>= 1) e += __shfl_xor(e, w, LPR);
    const T ls = log(e);
    const int lab = yv[pass];
    double l = (kin && k == lab && m < M) ? -(double)((z - mx) - ls) : 0.0;
    if (kin) {
      T g = T(0);
      if (m < M) {
        g = exp((z - mx) - ls);
        if (k == lab) g -= T(1);
        g = g / (T)M;
        if (writer) gz[(size_t)m * ldg + k] = g;
      }
      zt[r * zs + k] = g;
    }
#pragma unroll
    for (int w = LPR / 2; w >= 1; w >>= 1) l += __shfl_xor(l, w, LPR);
    if (k == 0) rowl[r] = l;
  }
  __syncthreads();
  if (t == 0 && writer) {
    double s = 0.0;
    for (int r = 0; r < 32; ++r) s += rowl[r];
    lpart[blk] = s;
  }
}

// Layer-3 backward of one 32-row block from gz in LDS (zt[32][zs], N = n_out columns; rows past M
// hold zeros):  ga2 = ((gz·W3)·m2)·[h2>0]·m1 and its column sums (b2 partial), column sums of gz
// (b3 partial), and gzᵀ·d3 over the block's rows (W3 partial).  Threads own a column j and a row
// group (rows ≡ g mod R, R = blockDim / n_mid); W3 is staged in LDS scratch `scr` when it fits.
// Columns [jlo, jhi) of n_mid only (the workgroup's slice: the layer-3 kernel runs one workgroup per
// (row block, column slice)); `first` marks the slice that also writes the b3 partial.
template <typename T, int MK>
__device__ inline void l3_backward(const MMArgs<T>& a, const T* zt, int zs, int m0, int blk, T* scr, int scr_n,
                                   int jlo, int jhi, bool first, int n_out = -1) {
  const int N = n_out >= 0 ? n_out : a.N, nm = a.n_mid, nj = jhi - jlo;
  const int rows = min(32, a.M - m0);
  const int tid = threadIdx.x, nt = blockDim.x;
  if (a.ga2 && nj > 0) {
    const bool wl = N * nm + nt <= scr_n;                      // W3 in LDS (+ nt values for the combine)
    T* w3 = scr + nt;
    if (wl) {                                                  // the slice's columns, 8 loads in flight
      const int nw = N * nj;
      for (int e0 = tid; e0 < nw; e0 += 8 * nt) {
        T v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int e = min(e0 + q * nt, nw - 1), o = e / nj;
          v[q] = a.W3[(size_t)o * nm + jlo + (e - o * nj)];
        }
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (e0 + q * nt < nw) {
            const int e = e0 + q * nt, o = e / nj;
            w3[o * nm + jlo + (e - o * nj)] = v[q];
          }
      }
      __syncthreads();
    }
    const int R = max(1, nt / nj), cols = nt / R;
#pragma unroll 1
    for (int jb = jlo; jb < jhi; jb += cols) {
      const int j = jb + tid % cols, g = tid / cols;
      const bool act = g < R && j < jhi;
      T cs = T(0);
      // RB rows per pass (rows g, g + R, …): their h2 / mask loads go out first, then RB independent
      // dot products; RB = 32 / R so that one pass covers the 32-row block
      auto rows_pass = [&](auto rbc) {
        constexpr int RB = decltype(rbc)::value;
#pragma unroll 1
        for (int r0 = g; r0 < rows; r0 += RB * R) {
          T hv[RB], m1v[RB], m2v[RB], acc8[RB];
#pragma unroll
          for (int c = 0; c < RB; ++c) {
            const int r = min(r0 + c * R, rows - 1);
            const size_t i = (size_t)(m0 + r) * nm + j;
            hv[c] = a.h2[i];
            m1v[c] = mval<T, MK>(a.ms, 1, i);
            m2v[c] = mval<T, MK>(a.ms, 2, i);
            acc8[c] = T(0);
          }
#pragma unroll 1
          for (int o = 0; o < N; ++o) {
            const T w = wl ? w3[o * nm + j] : a.W3[(size_t)o * nm + j];
#pragma unroll
            for (int c = 0; c < RB; ++c) acc8[c] += zt[min(r0 + c * R, 31) * zs + o] * w;
          }
#pragma unroll
          for (int c = 0; c < RB; ++c) {
            const int r = r0 + c * R;
            T t = acc8[c] * m2v[c];
            t = t * (hv[c] > T(0) ? T(1) : T(0));
            t = t * m1v[c];
            if (r < rows) {
              a.ga2[(size_t)(m0 + r) * nm + j] = t;
              cs += t;
            }
          }
        }
      };
      if (act) {
        if (R <= 2) rows_pass(std::integral_constant<int, 16>{});
        else if (R <= 4) rows_pass(std::integral_constant<int, 8>{});
        else if (R <= 8) rows_pass(std::integral_constant<int, 4>{});
        else rows_pass(std::integral_constant<int, 2>{});
      }
      if (a.pb2) {
        scr[tid] = cs;
        __syncthreads();
        if (act && g == 0) {
          T t = scr[tid];
          for (int q = 1; q < R; ++q) t += scr[q * cols + tid];
          a.pb2[(size_t)blk * nm + j] = t;
        }
        __syncthreads();
      }
    }
  }
  if (a.pb3 && first) {
    for (int j = tid; j < N; j += nt) {
      T cs = T(0);
      for (int r = 0; r < rows; ++r) cs += zt[r * zs + j];
      a.pb3[(size_t)blk * N + j] = cs;
    }
  }
  if (a.pw3) {
#pragma unroll 1
    for (int j = jlo + tid; j < jhi; j += nt) {                // one column of d3 per thread, all rows
      T dv[32];
#pragma unroll
      for (int r = 0; r < 32; ++r) dv[r] = a.d3[(size_t)(m0 + min(r, rows - 1)) * nm + j];
#pragma unroll 1
      for (int o = 0; o < N; ++o) {
        T sacc = T(0);
#pragma unroll
        for (int r = 0; r < 32; ++r) sacc += zt[r * zs + o] * dv[r];   // rows past M: gz = 0
        a.pw3[(size_t)blk * N * nm + (size_t)o * nm + j] = sacc;
      }
    }
  }
}

template <typename T, int EPI, int MK>
__device__ inline void mm_epilogue(const MMArgs<T>& a, int m, int n, T v) {
  const size_t i = (size_t)m * a.ldc + n;
  if constexpr (EPI == MM_STORE) {
    a.C[i] = v;
  } else if constexpr (EPI == MM_L2) {                          // mlp.py:30-31
    const T t = (v + a.bias[n]) * mval<T, MK>(a.ms, 1, i);
    const T h = t > T(0) ? t : T(0);
    a.C[i] = h;
    a.C2[i] = h * mval<T, MK>(a.ms, 2, i);
  } else if constexpr (EPI == MM_UPD) {
    apply_upd(a.u, a.upd_mode, i, v);
  }
}

// The workgroup's place in its (sub-)grid: a dual launch (k_mm2) runs two grids in one.
struct Blk { int x, y, z, gx, gy; };

template <typename T, int EPI, int AOP, int BOP, int TA, int TB, int AV, int BV, int MK, typename PR>
__device__ __forceinline__ void mm_body(const MMArgs<T>& a, const PR& pr, const Blk bk,
                                        T (&red)[MM_NW][32][33], double* rowl) {
  using M = mfma16<T>;
  const int pbid0 = bk.y * bk.gx + bk.x, nb0 = bk.gx * bk.gy;
  // The pending updates run in an extra plane of workgroups of their own (z = number of problems, 1
  // for a plain launch), beside the GEMM: nothing in this launch reads what they write (the momentum
  // and the NEXT iteration's position buffer of other variables), and no GEMM workgroup waits for them.
  if ((int)bk.z == (pr.n > 0 ? pr.n : 1)) {
    run_pendset(a.pend, pbid0, nb0);
    return;
  }
  // batched launch (pr.n > 0): the problem of this workgroup (bk.z) supplies the operands, masks
  // and outputs; the kernel argument block itself is never copied (a local MMArgs would live in scratch)
  const MMProb<T>* pp = pr.n > 0 ? &pr.p[bk.z] : nullptr;
  const T* const oA = pp ? pp->A : a.A;
  const T* const oB = pp ? pp->B : a.B;
  T* const oC = pp ? pp->C : a.C;
  const T* const ob1 = pp ? pp->b1 : a.b1;
  const T* const oH1 = pp ? pp->H1 : a.H1;
  const T* const obias = pp ? pp->bias : a.bias;
  const T* const oW3 = pp ? pp->W3 : a.W3;
  const T* const obias3 = pp ? pp->bias3 : a.bias3;
  const MaskSrc<T> oms = pp ? pp->ms : a.ms;
  T* const oga2 = pp ? pp->ga2 : a.ga2;
  T* const opb2 = pp ? pp->pb2 : a.pb2;
  T* const opb3 = pp ? pp->pb3 : a.pb3;
  T* const opw3 = pp ? pp->pw3 : a.pw3;
  T* const ogz = pp ? pp->gz : a.gz;
  double* const olpart = pp ? pp->lpart : a.lpart;
  T* const ocolpart = pp ? pp->colpart : a.colpart;
  char* const ogx = pp ? pp->gx : a.gx;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  // MM_L3CE: bk.y is the n_mid column slice of the layer-3 backward (N = n_out ≤ 32: one tile)
  const int m0 = bk.x * 32, n0 = EPI == MM_L3CE ? 0 : bk.y * 32;
  const int pbid = bk.y * bk.gx + bk.x;
  auto stamp = [&](int ph) {
    if constexpr (EPI == MM_L23)
      if (a.prof && tid == 0) a.prof[(size_t)pbid * L23_NPH + ph] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  // MM_L23: every operand of the epilogue and of layer 3 that does not depend on the GEMM (dropout
  // masks m1 / m2 and b2 of the two tile elements a thread finishes, the slice's W3 columns, b3) is
  // loaded before the GEMM's own operands, so the epilogue never waits on memory
  MRaw<T> pm1[2], pm2[2];
  T pb2v[2], pw3v[2], pb3v = T(0);
  int32_t yv[2] = {0, 0};
  if constexpr (EPI == MM_L23) {
    // labels of the rows this thread handles in the cross-entropy (ce_rows_lanes)
    const int lpr = a.N3 <= 16 ? 16 : 32, rpp = MM_NT / lpr;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) yv[pass] = a.y[min(m0 + pass * rpp + tid / lpr, a.M - 1)];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = tid + MM_NT * u, mm = e >> 5, nn = e & 31, m = m0 + mm, n = n0 + nn;
      const bool ok = m < a.M && n < a.N;
      const size_t i = ok ? (size_t)m * a.ldc + n : 0;
      pm1[u] = mraw<T, MK>(oms, 1, i);
      pm2[u] = mraw<T, MK>(oms, 2, i);
      pb2v[u] = obias[ok ? n : 0];
      const int o = e >> 5, c = e & 31;
      const bool okw = o < a.N3 && n0 + c < a.N;
      pw3v[u] = oW3[okw ? (size_t)o * a.n_mid + n0 + c : 0];
    }
    pb3v = obias3[tid < a.N3 ? tid : 0];
  }
  stamp(7);
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
    load_chunk<T, AOP, TA, AV, MK>(av[s], oA, a.lda, m0, a.M, k0, ke, lr, lg, oms, ob1);
    load_chunk<T, BOP, !TB, BV, MK>(bv[s], oB, a.ldb, n0, a.N, k0, ke, lr, lg, oms, ob1);
  };
  auto mfma = [&](int s, int k0) {
    if constexpr (EPI == MM_L23 && AOP == OP_H1) {
      // h1 of the k range of this WG's own column slice (one writer per element) for the kernels
      // that need h1 after this forward (layer-1 backward gate, W2 gradient)
      if (a.h1out) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int r = m0 + 16 * i + lr, k = k0 + kmap<T>(u, lg);
            if (r < a.M && k < ke && k >= n0 && k < n0 + 32) a.h1out[(size_t)r * a.lda + k] = av[s][u][i];
          }
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = M::fma(av[s][u][i], bv[s][u][j], acc[i][j]);
    if (s == 0) stamp(8);
  };
  if (kb < ke) load(0, kb);
  if (kb + 16 < ke) load(1, kb + 16);
  if (kb + 32 < ke) load(2, kb + 32);
  for (int k0 = kb; k0 < ke; k0 += 48) {
    mfma(0, k0);
    if (k0 + 48 < ke) load(0, k0 + 48);
    if (k0 + 16 < ke) {
      mfma(1, k0 + 16);
      if (k0 + 64 < ke) load(1, k0 + 64);
    }
    if (k0 + 32 < ke) {
      mfma(2, k0 + 32);
      if (k0 + 80 < ke) load(2, k0 + 80);
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) red[wave][16 * i + M::row(lane, q)][16 * j + lr] = acc[i][j][q];
  stamp(9);
  __syncthreads();
  stamp(10);
#pragma unroll
  for (int u = 0; u < 1024 / MM_NT; ++u) {
    const int e = tid + MM_NT * u, mm = e >> 5, nn = e & 31;
    const int m = m0 + mm, n = n0 + nn;
    T v = red[0][mm][nn];
#pragma unroll
    for (int w = 1; w < MM_NW; ++w) v += red[w][mm][nn];
    if constexpr (EPI == MM_L3CE) {
      red[0][mm][nn] = (n < a.N) ? v + obias[n] : T(0);     // logits of the block (one writer each)
    } else if constexpr (EPI == MM_GA1) {                      // (ga2·W2)·[(xw + b1)·m0 > 0]·m0
      T g = T(0);
      if (m < a.M && n < a.N) {
        const size_t i = (size_t)m * a.ldc + n;
        if (oH1) {
          // (xw + b1)·m0 > 0 ⟺ h1 > 0, and then m0 = scale; where h1 = 0 the product is ±0 either way
          // (the sign of v·0), so this is the reference's value without reading m0 again
          const bool pos = oH1[i] > T(0);
          g = (v * (pos ? T(1) : T(0))) * (pos ? oms.scale : T(0));
        } else {
          const T m0v = mval<T, MK>(oms, 0, i);
          g = (v * ((a.H[i] + ob1[n]) * m0v > T(0) ? T(1) : T(0))) * m0v;
        }
        oC[i] = g;
      }
      red[0][mm][nn] = g;
    } else if constexpr (EPI == MM_L23) {                      // mlp.py:30-31; the tile stays in LDS
      T d = T(0), h = T(0), m1 = T(0), m2 = T(0);
      mpin<T, MK>(pm1[u]);
      mpin<T, MK>(pm2[u]);
      if (m < a.M && n < a.N) {
        m1 = mfin<T, MK>(oms, pm1[u]);
        m2 = mfin<T, MK>(oms, pm2[u]);
        const T t = (v + pb2v[u]) * m1;
        h = t > T(0) ? t : T(0);
        d = h * m2;
        if (oC) {                                              // h2 / d3 are dead in the fused sampler
          const size_t i = (size_t)m * a.ldc + n;
          oC[i] = h;
          a.C2[i] = d;
        }
      }
      // planes of this element only (each (mm, nn) has one thread): d3, h2, m1, m2 of the tile
      red[0][mm][nn] = d;
      red[3][mm][nn] = h;
      red[4][mm][nn] = m1;
      red[5][mm][nn] = m2;
    } else if constexpr (EPI == MM_STORE) {
      if (m < a.M && n < a.N) oC[(size_t)m * a.ldc + n] = v;
    } else {
      if (m < a.M && n < a.N) mm_epilogue<T, EPI, MK>(a, m, n, v);
    }
  }
  if constexpr (EPI == MM_L3CE) {
    __syncthreads();
    const bool first = bk.y == 0;
    ce_rows<T>(&red[0][0][0], 33, rowl, m0, a.M, a.N, a.y, oC, a.ldc, olpart, bk.x, first);
    __syncthreads();
    const int cw = (a.n_mid + bk.gy - 1) / bk.gy;
    const int jlo = min(a.n_mid, (int)bk.y * cw), jhi = min(a.n_mid, jlo + cw);
    l3_backward<T, MK>(a, &red[0][0][0], 33, m0, bk.x, &red[1][0][0], (MM_NW - 1) * 32 * 33, jlo, jhi, first);
  }
  if constexpr (EPI == MM_L23) {
    // Layer 3 of this row block, in the same launch: z = d3·W3ᵀ + b3 (mlp.py:31) needs all n_mid
    // columns, which the S = bk.gy column-slice workgroups of the block hold.  Each publishes
    // its 32 × n_out partial (own 32 columns, k order within the slice) as 16-byte granules
    // {lo32, ep, hi32, ep} with write-through (sc1) stores; every member reads all S partials of
    // every (row, class) and sums them in slice order — the all-reduce by redundant reads of
    // hmcx_persist2.hip — then runs the cross-entropy of the block (slice 0 writes loss and gz) and
    // the layer-3 backward of its own columns.  The epoch is new per launch and the arena only ever
    // holds granules of earlier launches, so no stale value can match.
    const int No = a.N3, S = bk.gy, s = bk.y, rb = bk.x;
    T* d3t = &red[0][0][0];                                      // [32][33] d3 of the tile
    T* w3s = &red[1][0][0];                                      // [n_out][32] W3 columns of the slice
    T* zt = &red[2][0][0];                                       // [32][33] logits, then gz
    T* b3s = &red[7][0][0];                                      // [n_out] b3
    __syncthreads();                                             // the reduction has read every red[w]
    stamp(1);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = tid + MM_NT * u;
      if (e < No * 32) w3s[e] = n0 + (e & 31) < a.N ? pw3v[u] : T(0);  // prefetched; zero past n_mid
    }
    if (tid < No) b3s[tid] = pb3v;
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rs = gx_rsrc(ogx, a.gx_bytes);
    const int items = 32 * No;
    const int base_rb = rb * S * items;
    if (a.force_abort && pbid == 0 && tid == 0)                  // test knob: this launch never completes
      __hip_atomic_store(a.abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid < items && !(a.force_abort && pbid == 0)) {
      const int r = tid / No, o = tid - r * No;
      T zp = T(0);
#pragma unroll 8
      for (int c = 0; c < 32; ++c) zp += d3t[r * 33 + c] * w3s[o * 32 + c];
      gx_put(rs, base_rb + s * items + tid, (double)zp, a.ep);
    }
    stamp(2);
    stamp(3);
    if (tid < items) {
      const int r = tid / No, o = tid - r * No;
      double sum = 0.0;
      (void)gx_poll_sum(rs, base_rb + tid, items, S, a.ep, a.abort_flag, &sum);   // a timeout raises the
      zt[r * 33 + o] = (m0 + r < a.M) ? (T)sum + b3s[o] : T(0);                   // MLP abort word
    }
    __syncthreads();
    stamp(4);
    const bool first = s == 0;
    if (No <= 16) ce_rows_lanes<T, 16>(zt, 33, rowl, m0, a.M, No, yv, ogz, No, olpart, rb, first);
    else ce_rows_lanes<T, 32>(zt, 33, rowl, m0, a.M, No, yv, ogz, No, olpart, rb, first);
    __syncthreads();
    stamp(5);
    // layer-3 backward of the slice's columns, all operands in LDS (gz in zt, W3 slice in w3s, the
    // tile's h2 / d3 / masks): ga2 = ((gz·W3)·m2)·[h2 > 0]·m1 and its column sums (b2 partial),
    // gzᵀ·d3 (W3 partial), column sums of gz (b3 partial, slice 0)
    const int rows = min(32, a.M - m0), nm = a.n_mid;
    T* gat = &red[6][0][0];                                      // [32][33] ga2 of the tile
    for (int e = tid; e < 1024; e += MM_NT) {
      const int r = e >> 5, c = e & 31;
      T g = T(0);
      for (int o = 0; o < No; ++o) g += zt[r * 33 + o] * w3s[o * 32 + c];
      T t = g * red[5][r][c];
      t = t * (red[3][r][c] > T(0) ? T(1) : T(0));
      t = t * red[4][r][c];
      const bool ok2 = r < rows && n0 + c < nm;
      gat[r * 33 + c] = ok2 ? t : T(0);
      if (ok2 && oga2) oga2[(size_t)(m0 + r) * nm + n0 + c] = t;
    }
    __syncthreads();
    if (opb2 && tid < 32 && n0 + tid < nm) {
      T cs = T(0);
      for (int r = 0; r < rows; ++r) cs += gat[r * 33 + tid];
      opb2[(size_t)rb * nm + n0 + tid] = cs;
    }
    if (opw3)
      for (int e = tid; e < No * 32; e += MM_NT) {
        const int o = e >> 5, c = e & 31;
        if (n0 + c >= nm) continue;
        T acc = T(0);
        for (int r = 0; r < 32; ++r) acc += zt[r * 33 + o] * d3t[r * 33 + c];   // rows past M: gz = 0
        opw3[(size_t)rb * No * nm + (size_t)o * nm + n0 + c] = acc;
      }
    if (opb3 && first && tid < No) {
      T cs = T(0);
      for (int r = 0; r < rows; ++r) cs += zt[r * 33 + tid];
      opb3[(size_t)rb * No + tid] = cs;
    }
    stamp(6);
  }
  if constexpr (EPI == MM_GA1) {
    if (ocolpart) {
      __syncthreads();
      if (tid < 32 && n0 + tid < a.N) {
        T s = T(0);
        for (int r = 0; r < 32; ++r) s += red[0][r][tid];
        ocolpart[(size_t)bk.x * a.ldc + n0 + tid] = s;
      }
    }
  }
}

// amdgpu_waves_per_eu(4): two 8-wave workgroups per CU (≤ 128 registers): a batched fused launch
// (MM_L23) needs all its problems' workgroups co-resident, and at 136 registers only one fit per CU.
// Workgroups are dealt round-robin over the 8 XCDs in dispatch order (position lin of a launch plane
// whose size is a multiple of 8: XCD = lin % 8), and every XCD pulls its tiles' operands into its own
// L2.  xcd_place maps position (x, y) of a GX-wide plane to the tile it computes, or to none: xmap 1
// gives XCD k the tiles [k·P/8, (k+1)·P/8) of the gx × gy tiles in y-major order, xmap 2 the k-th
// xbx × xby block; both keep the tiles an XCD needs to few row tiles of A and few column slices of B
// (A and B tiles are both 32 × K).  xmap 0: the dispatch order itself.
template <typename T>
__device__ inline bool xcd_place(const MMArgs<T>& a, int GX, int gx, int gy, int& x, int& y) {
  if (!a.xmap) return x < gx && y < gy;
  const int lin = y * GX + x, k = lin & 7, s = lin >> 3;
  if (a.xmap == 1) {
    const int P = gx * gy, q = P >> 3, rem = P & 7;
    if (s >= q + (k < rem ? 1 : 0)) return false;
    const int t = k * q + min(k, rem) + s;
    x = t % gx;
    y = t / gx;
    return true;
  }
  if (s >= a.xbx * a.xby) return false;
  const int nbx = gx / a.xbx;
  x = (k % nbx) * a.xbx + s % a.xbx;
  y = (k / nbx) * a.xby + s / a.xbx;
  return true;
}

// A plain launch (k_mm) and a batched one (k_mmb, blockIdx.z = problem): the plain kernel keeps the
// small argument block (no problem table).
template <typename T, int EPI, int AOP, int BOP, int TA, int TB, int AV, int BV, int MK>
__global__ __launch_bounds__(MM_NT) __attribute__((amdgpu_waves_per_eu(4))) void k_mm(MMArgs<T> a) {
  __shared__ T red[MM_NW][32][33];
  __shared__ double rowl[32];
  MMProbsN<T, 1> none;
  none.n = 0;
  int x = blockIdx.x, y = blockIdx.y;
  if (a.xmap && blockIdx.z == 0 && !xcd_place(a, (int)gridDim.x, (int)gridDim.x, (int)gridDim.y, x, y)) return;
  mm_body<T, EPI, AOP, BOP, TA, TB, AV, BV, MK>(
      a, none, Blk{x, y, (int)blockIdx.z, (int)gridDim.x, (int)gridDim.y}, red, rowl);
}
template <typename T, int EPI, int AOP, int BOP, int TA, int TB, int AV, int BV, int MK>
__global__ __launch_bounds__(MM_NT) __attribute__((amdgpu_waves_per_eu(4))) void k_mmb(MMArgs<T> a, MMProbs<T> pr) {
  __shared__ T red[MM_NW][32][33];
  __shared__ double rowl[32];
  mm_body<T, EPI, AOP, BOP, TA, TB, AV, BV, MK>(
      a, pr, Blk{(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z, (int)gridDim.x, (int)gridDim.y}, red, rowl);
}

// Two independent launches as one: planes z < g1.z run grid 1 (g1.x × g1.y workgroups per plane, a
// batched launch with its problems), the planes after it grid 2 (a plain launch, g2.x × g2.y).  The
// launch grid is the larger of the two in x and y; workgroups outside their grid leave at once.
template <typename T, int E1, int A1, int B1, int TA1, int TB1, int AV1, int BV1,
          int E2, int A2, int B2, int TA2, int TB2, int AV2, int BV2, int MK>
__global__ __launch_bounds__(MM_NT) __attribute__((amdgpu_waves_per_eu(4)))
void k_mm2(MMArgs<T> a1, MMProbs3<T> p1, MMArgs<T> a2, int3 g1, int2 g2) {
  __shared__ T red[MM_NW][32][33];
  __shared__ double rowl[32];
  int x = blockIdx.x, y = blockIdx.y;
  const int z = blockIdx.z, GX = gridDim.x;
  if (z < g1.z) {
    // GEMM planes of grid 1 (not its pending plane) and grid 2's GEMM plane follow the XCD placement
    const bool gemm = z < (p1.n > 0 ? p1.n : 1);
    if (gemm ? xcd_place(a1, GX, g1.x, g1.y, x, y) : (x < g1.x && y < g1.y))
      mm_body<T, E1, A1, B1, TA1, TB1, AV1, BV1, MK>(a1, p1, Blk{x, y, z, g1.x, g1.y}, red, rowl);
  } else if (z == g1.z ? xcd_place(a2, GX, g2.x, g2.y, x, y) : (x < g2.x && y < g2.y)) {
    MMProbsN<T, 1> none;
    none.n = 0;
    mm_body<T, E2, A2, B2, TA2, TB2, AV2, BV2, MK>(a2, none, Blk{x, y, z - g1.z, g2.x, g2.y}, red, rowl);
  }
}

// Two batched launches as one: planes z < g1.z run batched grid 1, the next g2.z planes batched grid 2.
template <typename T, int E1, int A1, int B1, int TA1, int TB1, int AV1, int BV1,
          int E2, int A2, int B2, int TA2, int TB2, int AV2, int BV2, int MK>
__global__ __launch_bounds__(MM_NT) __attribute__((amdgpu_waves_per_eu(4)))
void k_mm2b(MMArgs<T> a1, MMProbs3<T> p1, MMArgs<T> a2, MMProbs3<T> p2, int3 g1, int3 g2) {
  __shared__ T red[MM_NW][32][33];
  __shared__ double rowl[32];
  const int x = blockIdx.x, y = blockIdx.y, z = blockIdx.z;
  if (z < g1.z) {
    if (x < g1.x && y < g1.y) mm_body<T, E1, A1, B1, TA1, TB1, AV1, BV1, MK>(a1, p1, Blk{x, y, z, g1.x, g1.y}, red, rowl);
  } else if (x < g2.x && y < g2.y) {
    mm_body<T, E2, A2, B2, TA2, TB2, AV2, BV2, MK>(a2, p2, Blk{x, y, z - g1.z, g2.x, g2.y}, red, rowl);
  }
}

// Layer 3 for n_out > 32: xw-free logits d3·W3ᵀ already stored in z; one 32-row block per
// workgroup, rows (+ b3) staged in dynamic LDS, then the same cross-entropy and layer-3 backward.
template <typename T, int MK>
__global__ __launch_bounds__(MM_NT) void k_l3_wide(MMArgs<T> a, const T* z) {
  extern __shared__ unsigned char dsm[];
  double* rowl = reinterpret_cast<double*>(dsm);
  T* scr = reinterpret_cast<T*>(dsm + 32 * sizeof(double));
  T* zt = scr + MM_NT;
  const int N = a.N, zs = N + 1, m0 = blockIdx.x * 32;
  run_pendset(a.pend, (int)blockIdx.x, (int)gridDim.x);
  for (int e = threadIdx.x; e < 32 * N; e += blockDim.x) {
    const int r = e / N, k = e - r * N;
    zt[r * zs + k] = (m0 + r < a.M) ? z[(size_t)(m0 + r) * N + k] + a.bias[k] : T(0);
  }
  __syncthreads();
  ce_rows<T>(zt, zs, rowl, m0, a.M, N, a.y, a.C, a.ldc, a.lpart, blockIdx.x);
  __syncthreads();
  l3_backward<T, MK>(a, zt, zs, m0, blockIdx.x, scr, MM_NT, 0, a.n_mid, true);
}

// ------------------------------------------------------------------ forwards by row block (k_fwdr)
// The forwards of a batched iteration (mlp.py:30-31 + the loss of :52 and its layer-3 backward), one
// workgroup per (16-row block, problem), holding ALL n_mid columns of its rows: layer 3 contracts over
// those columns, so the logits, the cross-entropy and the layer-3 backward of the block need no other
// workgroup — no cross-workgroup exchange, no co-residency requirement, and all six forwards of an
// iteration (plus the energy forwards that ride along) fit one launch.  Measured on the layer-2 GEMM
// alone (tools/microbench_fwdr.hip): 9.5 µs for six problems, flat in the problem count, against
// 8.3 µs for k_mm's 32 × 32 tiles before their exchange.
//   * h1 = max((xw + b1)·m0, 0) of the 16 rows is built once into LDS (A);
//   * wave w computes h2ᵀ for the columns n ∈ [32w, 32w + 32) over all of K = n_mid: A = W2 rows
//     (16-byte loads along k, three chunks in flight), B = h1ᵀ from LDS.  The accumulator layout (rows
//     n, columns r = lane & 15) is the B-operand layout of the layer-3 MFMA, so d3 never leaves the
//     registers: zᵀ[o][r] = Σ_n W3[o][n]·d3[r][n] is 8 more MFMAs per wave, then a fixed-order sum over
//     the waves in LDS;
//   * cross-entropy with 16 lanes per row (ce_rows_lanes' formula), then the layer-3 backward as MFMAs
//     in the same layout: ga2ᵀ = W3ᵀ·gzᵀ, the W3 partial (gzᵀ·d3)ᵀ from the d3 tile in LDS, the b2 / b3
//     partials as fixed-order sums over the block's rows.
// Partials are per 16-row block (nparts = ⌈B/16⌉).  Float32 results differ from the k_mm path by
// summation order only (K in one MFMA chain instead of split over the waves; slice partials of the
// logits summed in T instead of double).
constexpr int FR_ROWS = 16;
constexpr int FR_NW = 8;                 // waves per workgroup: n_mid ≤ 32·FR_NW
constexpr int FR_NMAX = 32 * FR_NW;
constexpr int FR_MAXP = 8;               // problems per launch: six sub-steps + E_new + E_current
template <typename T> struct RbFwdProb {
  const T* xw; const T* xw2;             // layer 1 as split-K planes: xw + xw2 (xw2 null: one plane)
  T* xwout;                              // the summed xw of the block's rows is stored here (null: not)
  T* h1out;                              // h1 of the block's rows is stored here (null: not)
  const T* b1; const T* W2; const T* b2; const T* W3; const T* b3;
  MaskSrc<T> ms;
  T* ga2; T* pb2; T* pb3; T* pw3;        // outputs, null when not wanted; partials [⌈B/16⌉][…]
  double* lpart;                         // loss partial of each 16-row block (null: none)
};
template <typename T> struct RbFwdArgs {
  int M, n_mid, n_out, np;
  const int32_t* y;
  RbFwdProb<T> p[FR_MAXP];
  PendSet<T> pend;                       // pending updates: run by the extra plane blockIdx.y == np
  unsigned long long* prof;              // HMCX_FWDR_PROF: FR_NPH s_memrealtime stamps per workgroup
  // the NEXT iteration's keep flags, drawn by the rows after the problems and the pending plane (kr.nf == 0:
  // none): they land on the CUs the problems leave free (192 + 32 workgroups on 256 CUs)
  uint32_t* keep; int n3; KeepRange kr; uint64_t seed; uint32_t chain, step;
};
constexpr int FR_NPH = 8;

template <typename T, int MK>
__global__ __launch_bounds__(FR_NW * 64) void k_fwdr(RbFwdArgs<T> a) {
  using Mf = mfma16<T>;
  constexpr int AP = FR_NMAX + 16 / (int)sizeof(T);               // pitch ≡ 4 dwords (mod 64): conflict-free
  __shared__ T At[FR_ROWS][AP];                                   // h1 tile, then the d3 tile
  __shared__ T w3s[16][FR_NMAX];                                  // W3 (rows ≥ n_out zero)
  __shared__ T zr[FR_NW][16][17];                                 // per-wave logit partials zᵀ[o][r]
  __shared__ T gzs[16][17];                                       // gz[r][o]
  __shared__ double rowl[FR_ROWS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  if ((int)blockIdx.y >= a.np + (a.pend.n > 0 ? 1 : 0)) {         // the next iteration's keep flags
    const int y0 = a.np + (a.pend.n > 0 ? 1 : 0);
    keep_flags(a.keep, a.n3, a.kr, a.seed, a.chain, a.step,
               ((size_t)((int)blockIdx.y - y0) * gridDim.x + blockIdx.x) * blockDim.x + tid);
    return;
  }
  if ((int)blockIdx.y == a.np) {                                  // the pending updates' plane
    run_pendset(a.pend, (int)blockIdx.x, (int)gridDim.x);
    return;
  }
  // this workgroup's problem, read through the kernel-argument segment pointer (address space 4) at a
  // uniform offset: scalar loads of ITS fields only (a.p[blockIdx.y] on the by-value argument made the
  // compiler load every problem's fields and select among them — 500+ spilled SGPRs)
  typedef __attribute__((address_space(4))) const RbFwdArgs<T> KArgs;
  KArgs* ka = (KArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  const int pb = (int)blockIdx.y;
  struct {
    const T *xw, *xw2; T *xwout, *h1out; const T *b1, *W2, *b2, *W3, *b3;
    const uint32_t* keep; const T* vals; T scale; int mn;
    T *ga2, *pb2, *pb3, *pw3; double* lpart;
  } P = {ka->p[pb].xw, ka->p[pb].xw2, ka->p[pb].xwout, ka->p[pb].h1out, ka->p[pb].b1, ka->p[pb].W2, ka->p[pb].b2,
         ka->p[pb].W3, ka->p[pb].b3, ka->p[pb].ms.keep, ka->p[pb].ms.vals, ka->p[pb].ms.scale, ka->p[pb].ms.mn,
         ka->p[pb].ga2, ka->p[pb].pb2, ka->p[pb].pb3, ka->p[pb].pw3, ka->p[pb].lpart};
  // MK_PHILOX: the masks are drawn here, as the sampler's keep flags would hold them (flag e of forward f =
  // bit e % 64 of keep_group(e / 64) under slot MASK_SLOT0 + f)
  MaskSrc<T> pms{};
  if constexpr (MK == MK_PHILOX) {
    pms.mn = P.mn; pms.seed = ka->p[pb].ms.seed; pms.chain = ka->p[pb].ms.chain; pms.step = ka->p[pb].ms.step;
    pms.slot = ka->p[pb].ms.slot;
  }
  auto pflags = [&](size_t e) {                               // flags e … e + 3 (e % 4 == 0) as 4 bits
    return (philox_keep_word(pms, e) >> (e & 31)) & 0xFu;
  };
  const MaskSrc<T> nomask{};
  const int rb = blockIdx.x, m0 = rb * FR_ROWS, nm = a.n_mid, No = a.n_out, M = a.M;
  auto stamp = [&](int ph) {
    if (a.prof && tid == 0) a.prof[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * FR_NPH + ph] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  static_assert(sizeof(T) == 4, "k_fwdr is the float32 kernel (fwdr_ok)");
  const int nwv = (nm + 31) / 32;                                  // waves with columns
  const int n0 = 32 * wave;
  const bool wact = wave < nwv;
  const int r = lr, m = m0 + r;
  const bool rok = m < M;
  const int mn = P.mn;
  // Every load of the prologue goes out before the first use (one memory round trip, not four):
  // 1. the first three 16-k chunks of this wave's W2 rows — the operand the launch waits on longest
  T bv[3][4][2];
  auto load = [&](int s, int k0) {
    load_chunk<T, OP_PLAIN, 0, 1, MK_NONE>(bv[s], P.W2, nm, n0, nm, k0, nm, lr, lg, nomask, nullptr);
  };
  load(0, 0);
  if (16 < nm) load(1, 16);
  if (32 < nm) load(2, 32);
  // 2. h1's inputs, two 4-element pieces per thread of the 16 × n_mid tile: xw, b1, the m0 mask
  constexpr int HP = FR_ROWS * FR_NMAX / 4 / (FR_NW * 64);
  float4 hx[HP], hx2[HP], hb[HP], hv4[HP];
  uint32_t hk[HP];
  size_t hbase[HP];
#pragma unroll
  for (int h = 0; h < HP; ++h) {
    const int e = tid + h * FR_NW * 64, rr = e / (nm / 4), c = (e % (nm / 4)) * 4, mm = m0 + rr;
    const bool ok = e < FR_ROWS * nm / 4 && mm < M;
    const size_t base = ok ? (size_t)mm * nm + c : 0;
    hbase[h] = base;
    hx[h] = *reinterpret_cast<const float4*>(P.xw + base);
    hx2[h] = *reinterpret_cast<const float4*>((P.xw2 ? P.xw2 : P.xw) + base);
    hb[h] = *reinterpret_cast<const float4*>(P.b1 + (ok ? c : 0));
    if constexpr (MK == MK_KEEP) hk[h] = P.keep[base >> 5];
    if constexpr (MK == MK_VALS) hv4[h] = *reinterpret_cast<const float4*>(P.vals + base);
  }
  // 3. W3, two 4-column pieces per thread (rows o ≥ n_out: zero)
  float4 w3v[HP];
#pragma unroll
  for (int h = 0; h < HP; ++h) {
    const int e = tid + h * FR_NW * 64, o = e / (FR_NMAX / 4), c = (e % (FR_NMAX / 4)) * 4;
    const bool ok = o < No && c < nm;
    w3v[h] = *reinterpret_cast<const float4*>(P.W3 + (ok ? (size_t)o * nm + c : 0));
  }
  // 4. the epilogue's operands for this lane's 8 elements (r = lr, n = n0 + 16j + 4·lg + q): b2, the
  //    m1 / m2 masks (one keep word or one 16-byte vector each); the labels and b3 of the cross-entropy
  float4 b2v[2], m1v4[2], m2v4[2];
  uint32_t k1[2], k2[2];
  size_t ebase[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + 16 * j + 4 * lg;
    const bool ok = rok && n < nm;
    const size_t e = ok ? (size_t)m * nm + n : 0;
    ebase[j] = e;
    b2v[j] = *reinterpret_cast<const float4*>(P.b2 + (ok ? n : 0));
    if constexpr (MK == MK_KEEP) {
      k1[j] = P.keep[((size_t)mn + e) >> 5];
      k2[j] = P.keep[((size_t)2 * mn + e) >> 5];
    }
    if constexpr (MK == MK_VALS) {
      m1v4[j] = *reinterpret_cast<const float4*>(P.vals + (size_t)mn + e);
      m2v4[j] = *reinterpret_cast<const float4*>(P.vals + (size_t)2 * mn + e);
    }
  }
  if constexpr (MK == MK_PHILOX) {                            // drawn while the loads above are in flight
#pragma unroll
    for (int h = 0; h < HP; ++h) hk[h] = pflags(hbase[h]);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      k1[j] = pflags((size_t)mn + ebase[j]);
      k2[j] = pflags((size_t)2 * mn + ebase[j]);
    }
    // pinned here, so the draws overlap the loads in flight instead of sinking into the epilogue
#pragma unroll
    for (int h = 0; h < HP; ++h) asm volatile("" : "+v"(hk[h]));
#pragma unroll
    for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(k1[j]), "+v"(k2[j]));
  }
  const int32_t yv = a.y[min(m0 + (tid >> 4), M - 1)];
  const T b3v = P.b3[min(tid & 15, No - 1)];
  // h1 = max((xw + b1)·m0, 0) (mlp.py:30) and W3 into LDS
  // the mask value of flag q of a 4-element piece at element e: one bit of a keep word (bit e % 32 + q), or
  // bit q of the drawn flags
  auto mbit = [&](uint32_t w, size_t e, int q) {
    const uint32_t sh = MK == MK_PHILOX ? (uint32_t)q : (uint32_t)((e & 31) + q);
    return ((w >> sh) & 1u) ? P.scale : T(0);
  };
#pragma unroll
  for (int h = 0; h < HP; ++h) {
    const int e = tid + h * FR_NW * 64, rr = e / (nm / 4), c = (e % (nm / 4)) * 4;
    if (e < FR_ROWS * nm / 4) {
      const bool ok = m0 + rr < M;
      if (P.xw2) {                                             // the two split-K planes, in plane order
        hx[h].x += hx2[h].x; hx[h].y += hx2[h].y; hx[h].z += hx2[h].z; hx[h].w += hx2[h].w;
        if (P.xwout && ok) *reinterpret_cast<float4*>(P.xwout + hbase[h]) = hx[h];
      }
      const T x[4] = {hx[h].x, hx[h].y, hx[h].z, hx[h].w}, bb[4] = {hb[h].x, hb[h].y, hb[h].z, hb[h].w};
      const T vv[4] = {hv4[h].x, hv4[h].y, hv4[h].z, hv4[h].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        T mk = T(1);
        if constexpr (MK == MK_KEEP || MK == MK_PHILOX) mk = mbit(hk[h], hbase[h], q);
        if constexpr (MK == MK_VALS) mk = vv[q];
        At[rr][c + q] = ok ? op_apply<T, OP_H1>(x[q], mk, bb[q]) : T(0);
      }
      if (P.h1out && ok)                                       // for the layer-1 backward's gate / the W2 gradient
        *reinterpret_cast<float4*>(P.h1out + hbase[h]) = *reinterpret_cast<const float4*>(&At[rr][c]);
    }
    const int o = e / (FR_NMAX / 4), c3 = (e % (FR_NMAX / 4)) * 4;
    const bool ok3 = o < No && c3 < nm;
    *reinterpret_cast<float4*>(&w3s[o][c3]) = ok3 ? w3v[h] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  stamp(1);
  __syncthreads();
  stamp(2);
  // layer 2, transposed: acc[j] = h2ᵀ[n0 + 16j + row][r] over all of K = n_mid; A = W2 rows (the ring),
  // B = h1ᵀ from LDS (16-byte reads)
  typename Mf::acc_t acc[2] = {Mf::zero(), Mf::zero()};
  if (wact) {
    auto mf = [&](int s, int k0) {
      const float4 w = *reinterpret_cast<const float4*>(&At[lr][k0 + 4 * lg]);
      const T hv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[j] = Mf::fma(bv[s][u][j], hv[u], acc[j]);
    };
    for (int k0 = 0; k0 < nm; k0 += 48) {
      mf(0, k0);
      if (k0 + 48 < nm) load(0, k0 + 48);
      if (k0 + 16 < nm) {
        mf(1, k0 + 16);
        if (k0 + 64 < nm) load(1, k0 + 64);
      }
      if (k0 + 32 < nm) {
        mf(2, k0 + 32);
        if (k0 + 80 < nm) load(2, k0 + 80);
      }
    }
  }
  stamp(3);
  // h2 = max((z2 + b2)·m1, 0), d3 = h2·m2 (mlp.py:30-31), kept in registers
  T dv[2][4], hp[2][4], m1v[2][4], m2v[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const T b2q[4] = {b2v[j].x, b2v[j].y, b2v[j].z, b2v[j].w};
    const T v1[4] = {m1v4[j].x, m1v4[j].y, m1v4[j].z, m1v4[j].w}, v2[4] = {m2v4[j].x, m2v4[j].y, m2v4[j].z, m2v4[j].w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = n0 + 16 * j + Mf::row(lane, q);
      const bool ok = rok && n < nm;
      m1v[j][q] = m2v[j][q] = T(1);
      if constexpr (MK == MK_KEEP || MK == MK_PHILOX) {
        m1v[j][q] = mbit(k1[j], (size_t)mn + ebase[j], q);
        m2v[j][q] = mbit(k2[j], (size_t)2 * mn + ebase[j], q);
      }
      if constexpr (MK == MK_VALS) {
        m1v[j][q] = v1[q];
        m2v[j][q] = v2[q];
      }
      const T t = (acc[j][q] + b2q[q]) * m1v[j][q];
      const T h = t > T(0) ? t : T(0);
      hp[j][q] = h > T(0) ? T(1) : T(0);
      dv[j][q] = ok ? h * m2v[j][q] : T(0);
    }
  }
  __syncthreads();                                                 // every wave is done with the h1 tile
  stamp(4);
  // layer 3: zᵀ[o][r] = Σ_n W3[o][n]·d3[r][n] over this wave's columns (k index n = n0 + 16j + row(u))
  {
    typename Mf::acc_t za = Mf::zero();
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int n = n0 + 16 * j + Mf::row(lane, u);
        za = Mf::fma(w3s[lr][min(n, FR_NMAX - 1)], dv[j][u], za);
        At[r][min(n, FR_NMAX - 1)] = dv[j][u];                     // the d3 tile, for the W3 partial
      }
#pragma unroll
    for (int q = 0; q < 4; ++q) zr[wave][Mf::row(lane, q)][lr] = za[q];
  }
  __syncthreads();
  stamp(5);
  // cross-entropy of the block's rows, 16 lanes per row (F.softmax_cross_entropy, mean over M)
  if (tid < 256) {
    const int rr = tid >> 4, k = tid & 15, mm = m0 + rr;
    const bool kin = k < No;
    T z = zr[0][k][rr];
    for (int w = 1; w < nwv; ++w) z += zr[w][k][rr];
    z = kin ? z + b3v : T(0);
    T mx = kin ? z : -INFINITY;
#pragma unroll
    for (int w = 8; w >= 1; w >>= 1) {                               // NaN propagates as in np.max
      const T o = __shfl_xor(mx, w, 16);
      mx = (o > mx || o != o) ? o : mx;
    }
    T e = kin ? exp(z - mx) : T(0);
#pragma unroll
    for (int w = 8; w >= 1; w >>= 1) e += __shfl_xor(e, w, 16);
    const T ls = log(e);
    double l = (kin && k == yv && mm < M) ? -(double)((z - mx) - ls) : 0.0;
    T g = T(0);
    if (kin && mm < M) {
      g = exp((z - mx) - ls);
      if (k == yv) g -= T(1);
      g = g / (T)M;
    }
    gzs[rr][k] = g;
#pragma unroll
    for (int w = 8; w >= 1; w >>= 1) l += __shfl_xor(l, w, 16);
    if (k == 0) rowl[rr] = l;
  }
  __syncthreads();
  stamp(6);
  if (tid == 0 && P.lpart) {
    double s = 0.0;
    for (int q = 0; q < FR_ROWS; ++q) s += rowl[q];
    P.lpart[rb] = s;
  }
  if (P.pb3 && tid < No) {                                           // b3 partial: Σ_rows gz
    T cs = T(0);
    for (int q = 0; q < FR_ROWS; ++q) cs += gzs[q][tid];
    P.pb3[(size_t)rb * No + tid] = cs;
  }
  if (!wact) return;
  // layer-3 backward (k index o = 4·lg + u < 16): ga2ᵀ[n][r] = Σ_o W3[o][n]·gz[r][o], then
  // ga2 = ((·)·m2)·[h2 > 0]·m1 in the layer-2 accumulator layout
  if (P.ga2 || P.pb2) {
    typename Mf::acc_t ga[2] = {Mf::zero(), Mf::zero()};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int o = 4 * lg + u;
      const T gzv = gzs[lr][o];
#pragma unroll
      for (int j = 0; j < 2; ++j) ga[j] = Mf::fma(w3s[o][min(n0 + 16 * j + lr, FR_NMAX - 1)], gzv, ga[j]);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      T gv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        T t = ga[j][q] * m2v[j][q];
        t = t * hp[j][q];
        t = t * m1v[j][q];
        const int n = n0 + 16 * j + Mf::row(lane, q);
        gv[q] = (rok && n < nm) ? t : T(0);
      }
      if (P.ga2 && rok) {
        if constexpr (sizeof(T) == 4) {                              // rows 4·lg … 4·lg + 3: one float4
          const int n = n0 + 16 * j + 4 * lg;
          if (n < nm) *reinterpret_cast<float4*>(P.ga2 + (size_t)m * nm + n) = make_float4(gv[0], gv[1], gv[2], gv[3]);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int n = n0 + 16 * j + Mf::row(lane, q);
            if (n < nm) P.ga2[(size_t)m * nm + n] = gv[q];
          }
        }
      }
      if (P.pb2) {                                                   // b2 partial: Σ over the block's rows
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          T s = gv[q];
#pragma unroll
          for (int w = 1; w < 16; w <<= 1) s += __shfl_xor(s, w, 16);
          const int n = n0 + 16 * j + Mf::row(lane, q);
          if (lr == 0 && n < nm) P.pb2[(size_t)rb * nm + n] = s;
        }
      }
    }
  }
  // W3 partial: pw3ᵀ[n][o] = Σ_r d3[r][n]·gz[r][o] over the block's rows (k index r = 4·lg + u)
  if (P.pw3) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      typename Mf::acc_t pw = Mf::zero();
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int rk = 4 * lg + u;
        pw = Mf::fma(At[rk][min(n0 + 16 * j + lr, FR_NMAX - 1)], gzs[rk][lr], pw);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = n0 + 16 * j + Mf::row(lane, q);
        if (lr < No && n < nm) P.pw3[(size_t)rb * No * nm + (size_t)lr * nm + n] = pw[q];
      }
    }
  }
  stamp(7);
}

// Mask values of one forward (the API twin of the sampler's keep flags: same groups, value = keep·(1/0.9)).
// Thread g: group g (64 elements), written as 16-byte vectors.
template <typename T>
__device__ inline void mlp_masks_group(T* masks, int n3, uint64_t seed, uint32_t chain, uint32_t step, uint32_t slot,
                                       int g) {
  if (64 * g >= n3) return;
  const KeepGroup k = keep_group(seed, (uint32_t)g, slot, step, chain);
  const T scale = (T)(1.0 / 0.9);
  constexpr int V = 16 / sizeof(T);
  typedef T tv __attribute__((ext_vector_type(V)));
  const int e0 = 64 * g, n = min(64, n3 - e0);
  for (int p = 0; p < 64; p += V) {
    tv v;
#pragma unroll
    for (int q = 0; q < V; ++q) v[q] = (((p + q < 32 ? k.lo >> (p + q) : k.hi >> (p + q - 32)) & 1u) ? scale : T(0));
    if (p + V <= n && (reinterpret_cast<uintptr_t>(masks + e0 + p) & 15) == 0) {
      *reinterpret_cast<tv*>(masks + e0 + p) = v;
    } else {
#pragma unroll
      for (int q = 0; q < V; ++q)
        if (p + q < n) masks[e0 + p + q] = v[q];
    }
  }
}
template <typename T>
__global__ void k_mlp_masks(T* masks, int n3, uint64_t seed, uint32_t chain, uint32_t step, uint32_t slot) {
  mlp_masks_group<T>(masks, n3, seed, chain, step, slot, (int)(blockIdx.x * blockDim.x + threadIdx.x));
}

// The kicks and the drift between two gradient calls of the full-batch trajectory in one launch
// (mlp_leapfrog_t; each row the per-element arithmetic of k_axpy, hmc.py:50-53): row 0 the previous
// sub-step's second kick p_u −= ε·g_u, row 1 the next sub-step's first kick and drift p_v −= (ε/2)·g_v,
// q_v += ε·p_v, row 2 the next gradient call's dropout masks (hmcx_mlp_masks).  u ≠ v always (consecutive
// variables of the order), so the rows touch disjoint memory.  A bias / W3 gradient the kick reads may still
// be pending (its row-block partials, UPD_GRAD): the row computes it element by element first (k_pending's
// arithmetic, the same thread reads back g[i]) — no k_pending launch of its own.
template <typename T> struct MlpKicks {
  T* pu; const T* gu; int64_t nu; T eu;
  T* pv; const T* gv; T* qv; int64_t nv; T hv, ev;
  T* masks; int n3; uint64_t seed; uint32_t chain, step, slot;   // masks null: no draw
  PendSet<T> ps;
};
template <typename T> __device__ inline int pend_of(const PendSet<T>& ps, const T* g) {
  int pj = -1;
#pragma unroll
  for (int j = 0; j < MAXPEND; ++j)
    if (j < ps.n && ps.p[j].mode == UPD_GRAD && ps.p[j].u.G == g) pj = j;
  return pj;
}
template <typename T>
__global__ __launch_bounds__(256) void k_mlp_kicks(MlpKicks<T> k) {
  const int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x, st = (int64_t)gridDim.x * 256;
  if (blockIdx.y == 0) {
    const int pj = pend_of(k.ps, k.gu);
    for (int64_t i = i0; i < k.nu; i += st) {
      if (pj >= 0) pending_elem(k.ps.p[pj], (int)i);
      const T ax = k.eu * k.gu[i];
      k.pu[i] = k.pu[i] - ax;
    }
  } else if (blockIdx.y == 1) {
    const int pj = pend_of(k.ps, k.gv);
    for (int64_t i = i0; i < k.nv; i += st) {
      if (pj >= 0) pending_elem(k.ps.p[pj], (int)i);
      const T ax = k.hv * k.gv[i];
      const T p = k.pv[i] - ax;
      k.pv[i] = p;
      const T aq = k.ev * p;
      k.qv[i] = k.qv[i] + aq;
    }
  } else if (k.masks) {
    for (int64_t g = i0; 64 * g < k.n3; g += st) mlp_masks_group<T>(k.masks, k.n3, k.seed, k.chain, k.step, k.slot, (int)g);
  }
}
// p = −p of the six variables (hmc.py:55-56, k_axpy's p − 2·p), one launch (row = variable)
template <typename T> struct Neg6 { T* p[6]; int64_t n[6]; };
template <typename T>
__global__ __launch_bounds__(256) void k_mlp_neg6(Neg6<T> a) {
  T* p = a.p[blockIdx.y];
  const T two = T(2);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < a.n[blockIdx.y]; i += (int64_t)gridDim.x * 256) {
    const T ax = two * p[i];
    p[i] = p[i] - ax;
  }
}

template <typename T>
__global__ void k_bias_into_z(T* z, const T* b, int n, int N) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) z[i] = z[i] + b[i % N];
}

// Six variables in the caller's order (position i of `order`).
struct VarTab {
  void* q[6]; void* qn[6]; void* p[6];
  void* qc[6];                 // step start: the previous step's proposal, committed here if accepted
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

// Blocks of grid.x that work on a variable of n elements (≈ 4 per thread): W1 (200,704 at config 3)
// gets 196 blocks instead of a fixed 32, so no thread walks a long serial chain of loads and Philox
// draws (k_mlp_init: 12.9 → 7.1 µs per step).  The other blocks only write zero partials.
__device__ inline int var_blocks(int n) { return min(NPART, max(1, (n + 1023) / 1024)); }

// Momentum draw (hmc.py:82-87) + first drift q' = q + ε·p + partials of Σp², Σq² (part [2][6][NPART]).
// With prev_acc set, the previous step's commit happens here first (state ← proposal where it was
// accepted, hmc.py:75-79): one launch less per step.
template <typename T>
__device__ inline void init_block(const VarTab& vt, T eps, int drift, int noise_mode, const double* noise,
                                  uint64_t seed, uint32_t chain, uint32_t step, double* part, int v, int bx,
                                  const int32_t* prev_acc) {
  const int n = vt.n[v];
  T* const qw = (T*)vt.q[v];
  const bool take = prev_acc != nullptr && vt.qc[v] != nullptr && *prev_acc != 0;   // uniform
  const T* q = take ? (const T*)vt.qc[v] : qw;
  T* qn = (T*)vt.qn[v];
  T* p = (T*)vt.p[v];
  const int nb = var_blocks(n);
  if (bx >= nb) {                                              // block-uniform
    if (threadIdx.x == 0) { part[v * NPART + bx] = 0.0; part[(6 + v) * NPART + bx] = 0.0; }
    return;
  }
  double sp = 0.0, sq = 0.0;
  for (int i = bx * 256 + threadIdx.x; i < n; i += nb * 256) {
    const uint32_t e = (uint32_t)(vt.e0[v] + i);
    const T z = noise_mode == HMCX_NOISE_BUFFER ? (T)noise[e] : philox_normal_t<T>(seed, chain, step, 0u, e);
    const T qv = q[i];
    if (take) qw[i] = qv;
    p[i] = z;
    if (drift) qn[i] = qv + eps * z;
    sp += (double)z * (double)z;
    sq += (double)qv * (double)qv;
  }
  block_sum2(sp, sq, part + v * NPART + bx, part + (6 + v) * NPART + bx);
}
template <typename T>
__global__ __launch_bounds__(256) void k_mlp_init(VarTab vt, T eps, int drift, int noise_mode, const double* noise,
                                                  uint64_t seed, uint32_t chain, uint32_t step, double* part,
                                                  const int32_t* prev_acc) {
  init_block<T>(vt, eps, drift, noise_mode, noise, seed, chain, step, part, (int)blockIdx.y, (int)blockIdx.x, prev_acc);
}
// Step start in one launch: rows y < 6 draw the momentum of variable y and the first drift (k_mlp_init),
// rows y ≥ 6 the keep flags of the step's nf forwards (keep_flags; work item (y − 6, x, thread) in
// row-major order) — independent work, one launch less per step.  grid.x = NPART.
template <typename T>
__global__ __launch_bounds__(256) void k_mlp_start(VarTab vt, T eps, int drift, int noise_mode, const double* noise,
                                                   uint64_t seed, uint32_t chain, uint32_t step, double* part,
                                                   const int32_t* prev_acc, uint32_t* keep, int n3, KeepRange kr) {
  if (blockIdx.y < 6) {
    init_block<T>(vt, eps, drift, noise_mode, noise, seed, chain, step, part, (int)blockIdx.y, (int)blockIdx.x,
                  prev_acc);
  } else {
    keep_flags(keep, n3, kr, seed, chain, step, ((size_t)(blockIdx.y - 6) * NPART + blockIdx.x) * 256 + threadIdx.x);
  }
}
// The keep flags alone (the forwards a k_fwdr step left undrawn when it falls back to the k_mm forwards).
static __global__ __launch_bounds__(256) void k_mlp_keep(uint32_t* keep, int n3, KeepRange kr, uint64_t seed, uint32_t chain,
                                                  uint32_t step) {
  keep_flags(keep, n3, kr, seed, chain, step, (size_t)blockIdx.x * 256 + threadIdx.x);
}

// End-of-trajectory partials: part[0][i] = Σp², part[1][i] = Σq² per variable (same layout as init).
template <typename T>
__global__ __launch_bounds__(256) void k_sumsq12(VarTab vt, double* part) {
  const int v = blockIdx.y, n = vt.n[v];
  const T* q = (const T*)vt.q[v];
  const T* p = (const T*)vt.p[v];
  const int nb = var_blocks(n);
  if ((int)blockIdx.x >= nb) {
    if (threadIdx.x == 0) { part[v * NPART + blockIdx.x] = 0.0; part[(6 + v) * NPART + blockIdx.x] = 0.0; }
    return;
  }
  double sp = 0.0, sq = 0.0;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += nb * 256) {
    const double pv = (double)p[i], qv = (double)q[i];
    sp += pv * pv;
    sq += qv * qv;
  }
  block_sum2(sp, sq, part + v * NPART + blockIdx.x, part + (6 + v) * NPART + blockIdx.x);
}

// MH accept (hmc.py:67-79): E = nlp + ½Σp², nlp = loss + log_prior, log_prior = −Σ_v ½α·Σθ²/dim.
struct MlpAccept {
  const double* part_cur; const double* part_new;   // [2][6][NPART]
  const double* lp_cur; const double* lp_new;       // loss partials [nlb_cur] / [nlb_new]
  int nlb_cur, nlb_new, B;
  int dim[6];
  double alpha, u;
  double* out_A; int32_t* out_acc; double* out_loss; double* out_nlp; double* out_E;
  int32_t* acc_flag;
};
// One workgroup of 26 × 32 threads: group g < 24 sums the NPART partials of (state g/12, kind, variable),
// groups 24/25 the loss partials of the current / proposed state — each lane a fixed-order strided
// sum, then a fixed-order tree.
static __global__ __launch_bounds__(1024) void k_mlp_accept(MlpAccept a) {
  __shared__ double sh[26][32];
  const int t = threadIdx.x, g = t >> 5, j = t & 31;
  double x = 0.0;
  if (g < 24) {
    const double* pp = (g < 12 ? a.part_cur : a.part_new) + (g % 12) * NPART;
    for (int q = 0; q < NPART / 32; ++q) x += pp[q * 32 + j];
  } else if (g < 26) {
    const double* lp = g == 24 ? a.lp_cur : a.lp_new;
    const int nb = g == 24 ? a.nlb_cur : a.nlb_new;
    for (int b = j; b < nb; b += 32) x += lp[b];
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

static __global__ void k_loss_final(const double* lpart, int nlb, int B, double* out) {
  double s = 0.0;
  for (int b = 0; b < nlb; ++b) s += lpart[b];
  *out = s / (double)B;
}

// ------------------------------------------------------------------ host side
namespace {

inline bool vec_ok(const void* p, int ld, int elt) {
  return ((uintptr_t)p % 16 == 0) && ((size_t)ld * elt) % 16 == 0;
}

template <typename T>
struct MlpNet {
  int B, n_in, n_mid, n_out, nlb;
  const T* X; const int32_t* y;
  T *xw, *h2, *d3, *z, *gz, *ga2, *ga1;
  T* h1 = nullptr; bool h1_valid = false;   // h1 of the last fused forward (when its sub-step needs it)
  T *pb1, *pb2, *pb3, *pw3;              // gradient partials of b1, b2, b3, W3 ([nlb][...])
  T *fpb2 = nullptr, *fpb3 = nullptr, *fpw3 = nullptr;   // the same partials per 16-row block (k_fwdr, [nrb][...])
  unsigned long long* fr_prof = nullptr;  // HMCX_FWDR_PROF: stamps of the call's k_fwdr launches
  int fr_prof_cap = 0, fr_prof_n = 0;
  std::vector<int> fr_prof_np;
  int nrb = 0;                           // 16-row blocks: ⌈B/16⌉
  hipStream_t st;
  bool xw_valid = false;
  bool vec_masks = true;                 // masks may be read as 4-/2-element vectors
  PendSet<T> pend{};                     // consumed by the next launch
  // fused layer 2 + layer 3 (MM_L23): granule arena and epoch counter of the context
  char* gx = nullptr; int gx_bytes = 0; hmcx_ctx* ctx = nullptr; int* abort_flag = nullptr; bool fuse = false;
  double* lpart_scr = nullptr;           // batched sampler: the sub-step's loss partials (unused output)
  int force_abort = -1, l23_count = 0;   // HMCX_MLP_FORCE_ABORT: the fused launch (0-based, per call) that aborts
  int l23_fit = 0;                       // fused grids that fit on the chip at once (occupancy × CUs / grid)
  unsigned long long* prof = nullptr;    // HMCX_MLP_PROF: stamps of every fused launch of the call
  int prof_cap = 0;
  int nvar(int v) const {
    switch (v) {
      case 0: return n_mid * n_in;  case 1: return n_mid;
      case 2: return n_mid * n_mid; case 3: return n_mid;
      case 4: return n_out * n_mid; default: return n_out;
    }
  }
};

template <typename T>
void net_init(MlpNet<T>& net, int B, int n_in, int n_mid, int n_out, hipStream_t st) {
  net.B = B; net.n_in = n_in; net.n_mid = n_mid; net.n_out = n_out; net.nlb = (B + 31) / 32; net.st = st;
  net.nrb = (B + FR_ROWS - 1) / FR_ROWS;
  net.vec_masks = n_mid % 4 == 0;
}

// Launch k_mm for a call site with compile-time operand layouts (TA: A stored [K][M], TB: B stored
// [N][K]); k-contiguous operands take the 16-byte vector path when aligned.  Takes the pending update.
// BAT: the call site passes a problem table (k_mmb); plain call sites instantiate k_mm only.
// XCD placement of one GEMM plane (xcd_place): the candidate that leaves each XCD the fewest distinct
// operand tiles (A row tiles + B column slices) — the dispatch order, y-major chunks, or one block of
// tiles per XCD.  f32 only: config 3's W1 gradient (8 × 25 tiles; chunks: 8 + 4 tiles per XCD instead
// of 1 + 25) went from 63 to 78 % L2 hits and 14.91 k to 15.04 k leapfrog/s, f64 measured 5.92 k → 5.90 k
// (DESIGN §5.3 Round 5).  HMCX_MLP_XMAP=0 keeps the dispatch order everywhere.
template <typename T>
void xcd_choose(MMArgs<T>& a, int GX, int GY, int gx, int gy) {
  static const bool off = getenv("HMCX_MLP_XMAP") && getenv("HMCX_MLP_XMAP")[0] == '0';
  a.xmap = 0;
  if (off || sizeof(T) != 4 || gx * gy < 16 || (GX * GY) % 8) return;
  const int per = GX * GY / 8;                                   // positions per XCD in the plane
  int best = GX % 8 == 0 ? (gx + 7) / 8 + gy : gx + gy;          // dispatch order
  const int P = gx * gy, q = P / 8 + (P % 8 ? 1 : 0);
  if (q <= per) {
    const int c = std::min(gx, q) + (q + gx - 1) / gx + 1;
    if (c < best) { best = c; a.xmap = 1; }
  }
  for (int bx = 1; bx <= gx; ++bx) {
    if (gx % bx) continue;
    for (int by = 1; by <= gy; ++by) {
      if (gy % by || (gx / bx) * (gy / by) != 8 || bx * by > per) continue;
      if (bx + by < best) { best = bx + by; a.xmap = 2; a.xbx = bx; a.xby = by; }
    }
  }
}

template <typename T, int EPI, int TA, int TB, int AOP = OP_PLAIN, int BOP = OP_PLAIN, bool BAT = false>
hipError_t mm(MlpNet<T>& net, MMArgs<T>& a, const MMProbs<T>* prp = nullptr) {
  if (a.ta != TA || a.tb != TB || (prp && !BAT)) return hipErrorInvalidValue;
  a.pend = net.pend;
  net.pend.n = 0;
  MMProbs<T> pr{};
  if (prp) pr = *prp;
  // a batched launch: one plane per problem, plus one for the pending updates
  dim3 grid((a.M + 31) / 32, (a.N + 31) / 32, (pr.n > 0 ? pr.n : 1) + (a.pend.n > 0 ? 1 : 0)), blk(MM_NT);
  if (EPI == MM_L3CE) grid.y = (unsigned)std::max(1, std::min(8, a.n_mid / 32));   // n_mid column slices
  if (pr.n == 0 && (EPI == MM_UPD || EPI == MM_STORE)) xcd_choose<T>(a, (int)grid.x, (int)grid.y, (int)grid.x, (int)grid.y);
  const bool h1ok = AOP != OP_H1 || net.vec_masks;
  const bool kvec = a.K % (int)(16 / sizeof(T)) == 0;       // vectors never straddle the K end
  bool aal = vec_ok(a.A, a.lda, sizeof(T)), bal = vec_ok(a.B, a.ldb, sizeof(T));
  for (int p = 0; p < pr.n; ++p) {                            // every problem's operands
    aal = aal && vec_ok(pr.p[p].A, a.lda, sizeof(T));
    bal = bal && vec_ok(pr.p[p].B, a.ldb, sizeof(T));
  }
  const bool av = !TA && h1ok && kvec && aal;
  const bool bv = TB && kvec && bal;
  hipStream_t st = net.st;
  auto go = [&](auto mkc) {
    constexpr int MK = decltype(mkc)::value;
    if constexpr (BAT) {
      if (pr.n > 0) {
        if (av && bv) hipLaunchKernelGGL((k_mmb<T, EPI, AOP, BOP, TA, TB, !TA, TB, MK>), grid, blk, 0, st, a, pr);
        else if (av) hipLaunchKernelGGL((k_mmb<T, EPI, AOP, BOP, TA, TB, !TA, 0, MK>), grid, blk, 0, st, a, pr);
        else if (bv) hipLaunchKernelGGL((k_mmb<T, EPI, AOP, BOP, TA, TB, 0, TB, MK>), grid, blk, 0, st, a, pr);
        else hipLaunchKernelGGL((k_mmb<T, EPI, AOP, BOP, TA, TB, 0, 0, MK>), grid, blk, 0, st, a, pr);
        return;
      }
    }
    if (av && bv) hipLaunchKernelGGL((k_mm<T, EPI, AOP, BOP, TA, TB, !TA, TB, MK>), grid, blk, 0, st, a);
    else if (av) hipLaunchKernelGGL((k_mm<T, EPI, AOP, BOP, TA, TB, !TA, 0, MK>), grid, blk, 0, st, a);
    else if (bv) hipLaunchKernelGGL((k_mm<T, EPI, AOP, BOP, TA, TB, 0, TB, MK>), grid, blk, 0, st, a);
    else hipLaunchKernelGGL((k_mm<T, EPI, AOP, BOP, TA, TB, 0, 0, MK>), grid, blk, 0, st, a);
  };
  constexpr bool masked = AOP == OP_H1 || BOP == OP_H1 || EPI == MM_L2 || EPI == MM_L3CE || EPI == MM_GA1 ||
                          EPI == MM_L23;
  if constexpr (!masked) go(std::integral_constant<int, MK_NONE>{});
  else if (a.ms.slot) go(std::integral_constant<int, MK_PHILOX>{});
  else if (a.ms.keep) go(std::integral_constant<int, MK_KEEP>{});
  else if (a.ms.vals) go(std::integral_constant<int, MK_VALS>{});
  else go(std::integral_constant<int, MK_NONE>{});
  return hipGetLastError();
}

template <typename T>
void mm_set(MMArgs<T>& a, int M, int N, int K, const T* A, int lda, int ta, const T* B, int ldb, int tb, T* C, int ldc) {
  a.M = M; a.N = N; a.K = K; a.A = A; a.lda = lda; a.ta = ta; a.B = B; a.ldb = ldb; a.tb = tb; a.C = C; a.ldc = ldc;
}

// What the layer-3 kernel produces besides the loss
struct L3Want { bool ga2, pb2, pb3, pw3, h1 = false; };

// Forward with masks `ms` at parameters q (+ the requested layer-3 backward pieces); loss partials
// into lpart (null: no loss); logits (optional) stored without b3.  Layer 1 only when xw is stale.
template <typename T>
hipError_t mlp_forward(MlpNet<T>& net, T* const* q, const MaskSrc<T>& ms, double* lpart, L3Want w,
                       T* logits = nullptr) {
  const int B = net.B, nm = net.n_mid;
  hipError_t e;
  net.h1_valid = false;
  if (!net.xw_valid) {                                        // xw = X·W1ᵀ
    MMArgs<T> a{};
    mm_set<T>(a, B, nm, net.n_in, net.X, net.n_in, 0, q[0], net.n_in, 1, net.xw, nm);
    if ((e = mm<T, MM_STORE, 0, 1>(net, a))) return e;
    net.xw_valid = true;
  }
  if (net.fuse && lpart && !logits && net.n_out <= 32) {
    // h2, d3 and layer 3 (cross-entropy, layer-3 backward) in one launch (MM_L23)
    MMArgs<T> a{};
    mm_set<T>(a, B, nm, nm, net.xw, nm, 0, q[2], nm, 1, net.h2, nm);
    a.bias = q[3]; a.b1 = q[1]; a.ms = ms; a.C2 = net.d3;
    a.N3 = net.n_out; a.bias3 = q[5]; a.gz = net.gz; a.y = net.y; a.lpart = lpart;
    a.W3 = q[4]; a.h2 = net.h2; a.d3 = net.d3; a.n_mid = nm;
    a.ga2 = w.ga2 ? net.ga2 : nullptr;
    a.pb2 = w.pb2 ? net.pb2 : nullptr;
    a.pb3 = w.pb3 ? net.pb3 : nullptr;
    a.pw3 = w.pw3 ? net.pw3 : nullptr;
    a.C = nullptr; a.C2 = nullptr;                             // h2 / d3 stay in LDS
    a.h1out = w.h1 ? net.h1 : nullptr;
    net.h1_valid = w.h1;
    a.gx = net.gx; a.gx_bytes = net.gx_bytes; a.ep = gx_next_epoch(net.ctx); a.abort_flag = net.abort_flag;
    a.force_abort = net.l23_count == net.force_abort;
    if (net.prof && net.l23_count < net.prof_cap)
      a.prof = net.prof + (size_t)net.l23_count * net.nlb * ((nm + 31) / 32) * L23_NPH;
    ++net.l23_count;
    return mm<T, MM_L23, 0, 1, OP_H1>(net, a);
  }
  {                                                           // h2, d3 from h1 = max((xw + b1)·m0, 0)
    MMArgs<T> a{};
    mm_set<T>(a, B, nm, nm, net.xw, nm, 0, q[2], nm, 1, net.h2, nm);
    a.bias = q[3]; a.b1 = q[1]; a.ms = ms; a.C2 = net.d3;
    if ((e = mm<T, MM_L2, 0, 1, OP_H1>(net, a))) return e;
  }
  if (logits) {
    MMArgs<T> a{};
    mm_set<T>(a, B, net.n_out, nm, net.d3, nm, 0, q[4], nm, 1, logits, net.n_out);
    if ((e = mm<T, MM_STORE, 0, 1>(net, a))) return e;
  }
  if (!lpart) return hipSuccess;
  MMArgs<T> a{};
  a.bias = q[5]; a.y = net.y; a.lpart = lpart; a.ms = ms;
  a.W3 = q[4]; a.h2 = net.h2; a.d3 = net.d3; a.n_mid = nm;
  a.ga2 = w.ga2 ? net.ga2 : nullptr;
  a.pb2 = w.pb2 ? net.pb2 : nullptr;
  a.pb3 = w.pb3 ? net.pb3 : nullptr;
  a.pw3 = w.pw3 ? net.pw3 : nullptr;
  if (net.n_out <= 32) {                                      // z, cross-entropy, layer-3 backward
    mm_set<T>(a, B, net.n_out, nm, net.d3, nm, 0, q[4], nm, 1, net.gz, net.n_out);
    return mm<T, MM_L3CE, 0, 1>(net, a);
  }
  {
    MMArgs<T> az{};
    mm_set<T>(az, B, net.n_out, nm, net.d3, nm, 0, q[4], nm, 1, net.z, net.n_out);
    if ((e = mm<T, MM_STORE, 0, 1>(net, az))) return e;       // d3·W3ᵀ; b3 is added in k_l3_wide
  }
  a.M = B; a.N = net.n_out; a.C = net.gz; a.ldc = net.n_out;
  a.pend = net.pend;
  net.pend.n = 0;
  const size_t lds = 32 * sizeof(double) + ((size_t)MM_NT + (size_t)32 * (net.n_out + 1)) * sizeof(T);
  if (a.ms.slot) hipLaunchKernelGGL((k_l3_wide<T, MK_PHILOX>), dim3(net.nlb), dim3(MM_NT), lds, net.st, a, (const T*)net.z);
  else if (a.ms.keep) hipLaunchKernelGGL((k_l3_wide<T, MK_KEEP>), dim3(net.nlb), dim3(MM_NT), lds, net.st, a, (const T*)net.z);
  else if (a.ms.vals) hipLaunchKernelGGL((k_l3_wide<T, MK_VALS>), dim3(net.nlb), dim3(MM_NT), lds, net.st, a, (const T*)net.z);
  else hipLaunchKernelGGL((k_l3_wide<T, MK_NONE>), dim3(net.nlb), dim3(MM_NT), lds, net.st, a, (const T*)net.z);
  return hipGetLastError();
}

template <typename T>
hipError_t mlp_ga1(MlpNet<T>& net, T* const* q, const MaskSrc<T>& ms, bool want_pb1) {
  MMArgs<T> a{};
  mm_set<T>(a, net.B, net.n_mid, net.n_mid, net.ga2, net.n_mid, 0, q[2], net.n_mid, 0, net.ga1, net.n_mid);
  a.ms = ms; a.H = net.xw; a.b1 = q[1];
  a.H1 = net.h1_valid ? net.h1 : nullptr;
  a.colpart = want_pb1 ? net.pb1 : nullptr;
  return mm<T, MM_GA1, 0, 0>(net, a);
}

// Weight gradient of W1 / W2 through the k_mm epilogue (biases and W3 come from partials).
template <typename T>
hipError_t mlp_wgrad(MlpNet<T>& net, T* const* q, const MaskSrc<T>& ms, int v, int mode, const Upd<T>& u) {
  const int B = net.B, nm = net.n_mid;
  MMArgs<T> a{};
  a.upd_mode = mode; a.u = u;
  if (v == 2) {                                               // ga2ᵀ·h1
    if (net.h1_valid) {                                       // h1 stored by the fused forward
      mm_set<T>(a, nm, nm, B, net.ga2, nm, 1, net.h1, nm, 0, nullptr, nm);
      return mm<T, MM_UPD, 1, 0>(net, a);
    }
    mm_set<T>(a, nm, nm, B, net.ga2, nm, 1, net.xw, nm, 0, nullptr, nm);
    a.ms = ms; a.b1 = q[1];
    return mm<T, MM_UPD, 1, 0, OP_PLAIN, OP_H1>(net, a);
  }
  mm_set<T>(a, nm, net.n_in, B, net.ga1, nm, 1, net.X, net.n_in, 0, nullptr, net.n_in);   // ga1ᵀ·X
  return mm<T, MM_UPD, 1, 0>(net, a);
}

// xw = X·W1ᵀ into net.xw
template <typename T>
hipError_t mlp_layer1(MlpNet<T>& net, const T* W1) {
  MMArgs<T> a{};
  mm_set<T>(a, net.B, net.n_mid, net.n_in, net.X, net.n_in, 0, W1, net.n_in, 1, net.xw, net.n_mid);
  net.xw_valid = true;
  return mm<T, MM_STORE, 0, 1>(net, a);
}

// xw = X·W1ᵀ for np (W1, out) pairs in one launch
template <typename T>
hipError_t mlp_layer1_batch(MlpNet<T>& net, const T* const* W1, T* const* out, int np) {
  MMArgs<T> a{};
  MMProbs<T> pr{};
  pr.n = np;
  for (int p = 0; p < np; ++p) {
    pr.p[p].A = net.X; pr.p[p].B = W1[p]; pr.p[p].C = out[p];
  }
  mm_set<T>(a, net.B, net.n_mid, net.n_in, net.X, net.n_in, 0, W1[0], net.n_in, 1, out[0], net.n_mid);
  return mm<T, MM_STORE, 0, 1, OP_PLAIN, OP_PLAIN, true>(net, a, &pr);
}

// One sub-step's share of a batched launch: its positions, masks, scratch net (ga2, ga1, gz and the
// gradient partials), loss partials and what its layer-3 backward must produce.
template <typename T> struct SubStep {
  const T* xw;                       // layer-1 output of its W1 (null: net's)
  const T* xw2 = nullptr;            // k_fwdr: the second split-K plane of layer 1 (xw = xw + xw2)
  T* xwout = nullptr;                // k_fwdr: store the summed xw here
  T* q[6];
  MaskSrc<T> ms;
  MlpNet<T>* scr;
  double* lpart;
  L3Want w;
  int v;
};

// Batched-launch argument builders: the shared MMArgs (problem 0's operands) and the problem table.
// Fused forwards (MM_L23) at net's xw (or the sub-step's own): problem p uses arena region p0 + p and
// writes into its own scratch.
template <typename T, typename PR>
void l23_build(MlpNet<T>& net, const SubStep<T>* const* ss, int np, int p0, MMArgs<T>& a, PR& pr) {
  const int nm = net.n_mid;
  a = MMArgs<T>{};
  pr.n = np;
  for (int p = 0; p < np; ++p) {
    const SubStep<T>& s = *ss[p];
    const MlpNet<T>& sc = *s.scr;
    MMProb<T>& q = pr.p[p];
    q = MMProb<T>{};
    q.A = s.xw ? s.xw : net.xw; q.B = s.q[2]; q.C = nullptr;
    q.b1 = s.q[1]; q.bias = s.q[3]; q.W3 = s.q[4]; q.bias3 = s.q[5];
    q.ms = s.ms;
    q.ga2 = s.w.ga2 ? sc.ga2 : nullptr;
    q.pb2 = s.w.pb2 ? sc.pb2 : nullptr;
    q.pb3 = s.w.pb3 ? sc.pb3 : nullptr;
    q.pw3 = s.w.pw3 ? sc.pw3 : nullptr;
    q.gz = sc.gz; q.lpart = s.lpart; q.colpart = nullptr;
    q.gx = net.gx + (size_t)(p0 + p) * net.gx_bytes;
  }
  const MMProb<T>& q0 = pr.p[0];
  mm_set<T>(a, net.B, nm, nm, q0.A, nm, 0, q0.B, nm, 1, nullptr, nm);
  a.bias = q0.bias; a.b1 = q0.b1; a.ms = q0.ms; a.C2 = nullptr;
  a.N3 = net.n_out; a.bias3 = q0.bias3; a.gz = q0.gz; a.y = net.y; a.lpart = q0.lpart;
  a.W3 = q0.W3; a.n_mid = nm;
  a.ga2 = q0.ga2; a.pb2 = q0.pb2; a.pb3 = q0.pb3; a.pw3 = q0.pw3;
  a.gx = q0.gx; a.gx_bytes = net.gx_bytes; a.ep = gx_next_epoch(net.ctx); a.abort_flag = net.abort_flag;
  a.force_abort = net.l23_count == net.force_abort;
  ++net.l23_count;
}

// Layer-1 backwards (MM_GA1: ga1 = (ga2·W2)·gate, + b1 partials for the b1 sub-step), each from its
// own ga2 into its own ga1.
template <typename T, typename PR>
void ga1_build(MlpNet<T>& net, const SubStep<T>* const* ss, int np, MMArgs<T>& a, PR& pr) {
  const int nm = net.n_mid;
  a = MMArgs<T>{};
  pr.n = np;
  for (int p = 0; p < np; ++p) {
    const SubStep<T>& s = *ss[p];
    MMProb<T>& q = pr.p[p];
    q = MMProb<T>{};
    q.A = s.scr->ga2; q.B = s.q[2]; q.C = s.scr->ga1;
    q.b1 = s.q[1]; q.ms = s.ms;
    q.H1 = s.w.h1 ? s.scr->h1 : nullptr;                        // k_fwdr stored h1: the gate reads it alone
    q.colpart = s.v == 1 ? s.scr->pb1 : nullptr;
  }
  const MMProb<T>& q0 = pr.p[0];
  mm_set<T>(a, net.B, nm, nm, q0.A, nm, 0, q0.B, nm, 0, q0.C, nm);
  a.ms = q0.ms; a.H = net.xw; a.b1 = q0.b1; a.H1 = nullptr; a.colpart = q0.colpart;
}

// Weight gradient of W1 (v = 0: ga1ᵀ·X) or W2 (v = 2: ga2ᵀ·h1) of sub-step net `sn` with the SGHMC
// epilogue, as mlp_wgrad.
template <typename T>
void wgrad_build(MlpNet<T>& sn, const SubStep<T>& s, int v, const Upd<T>& u, MMArgs<T>& a) {
  const int B = sn.B, nm = sn.n_mid;
  a = MMArgs<T>{};
  a.upd_mode = UPD_SGHMC; a.u = u;
  if (v == 2) {
    mm_set<T>(a, nm, nm, B, sn.ga2, nm, 1, sn.xw, nm, 0, nullptr, nm);
    a.ms = s.ms; a.b1 = s.q[1];
  } else {
    mm_set<T>(a, nm, sn.n_in, B, sn.ga1, nm, 1, sn.X, sn.n_in, 0, nullptr, sn.n_in);
  }
}

template <typename T>
hipError_t mlp_forward_batch(MlpNet<T>& net, const SubStep<T>* ss, int np) {
  const SubStep<T>* sp[MAXPROB];
  for (int p = 0; p < np; ++p) sp[p] = ss + p;
  MMArgs<T> a;
  MMProbs<T> pr{};
  l23_build(net, sp, np, 0, a, pr);
  return mm<T, MM_L23, 0, 1, OP_H1, OP_PLAIN, true>(net, a, &pr);
}

// mask kind of a launch (one per launch: every sub-grid reads the same kind)
template <typename T> inline int mask_kind(const MaskSrc<T>& ms) {
  return ms.slot ? MK_PHILOX : ms.keep ? MK_KEEP : ms.vals ? MK_VALS : MK_NONE;
}

// The layer-1 backwards of np sub-steps and the W2 gradient of sub-step net `w2n` in ONE launch
// (k_mm2): neither reads what the other writes.  net's pending updates run in the first grid's extra
// plane.
template <typename T>
hipError_t mlp_ga1_w2(MlpNet<T>& net, const SubStep<T>* const* ss, int np, MlpNet<T>& w2n, const SubStep<T>& s2,
                      const Upd<T>& u2) {
  const int nm = net.n_mid;
  MMArgs<T> a1, a2;
  MMProbs3<T> pr{};
  ga1_build(net, ss, np, a1, pr);
  a1.pend = net.pend;
  net.pend.n = 0;
  wgrad_build(w2n, s2, 2, u2, a2);
  a2.pend = w2n.pend;
  w2n.pend.n = 0;
  if (mask_kind(a1.ms) != mask_kind(a2.ms)) return hipErrorInvalidValue;
  const int3 g1 = make_int3((a1.M + 31) / 32, (a1.N + 31) / 32, np + (a1.pend.n > 0 ? 1 : 0));
  const int2 g2 = make_int2((a2.M + 31) / 32, (a2.N + 31) / 32);
  const dim3 grid((unsigned)std::max(g1.x, g2.x), (unsigned)std::max(g1.y, g2.y), (unsigned)(g1.z + 1));
  bool aal = nm % (int)(16 / sizeof(T)) == 0;
  for (int p = 0; p < np; ++p) aal = aal && vec_ok(pr.p[p].A, nm, sizeof(T));
  hipStream_t st = net.st;
  auto go = [&](auto mkc, auto avc) {
    constexpr int MK = decltype(mkc)::value, AV = decltype(avc)::value;
    hipLaunchKernelGGL((k_mm2<T, MM_GA1, OP_PLAIN, OP_PLAIN, 0, 0, AV, 0, MM_UPD, OP_PLAIN, OP_H1, 1, 0, 0, 0, MK>),
                       grid, dim3(MM_NT), 0, st, a1, pr, a2, g1, g2);
  };
  auto go_mk = [&](auto mkc) {
    if (aal) go(mkc, std::integral_constant<int, 1>{});
    else go(mkc, std::integral_constant<int, 0>{});
  };
  switch (mask_kind(a1.ms)) {
    case MK_PHILOX: go_mk(std::integral_constant<int, MK_PHILOX>{}); break;
    case MK_KEEP: go_mk(std::integral_constant<int, MK_KEEP>{}); break;
    case MK_VALS: go_mk(std::integral_constant<int, MK_VALS>{}); break;
    default: go_mk(std::integral_constant<int, MK_NONE>{}); break;
  }
  return hipGetLastError();
}

// Four launches per iteration (fit ≥ 4 fused grids co-resident, keep-flag or buffer masks, aligned
// operands): the fused forwards of 4 sub-steps (those of W1, b1, W2 and one more), then ONE launch of
// the other 2 fused forwards beside the layer-1 backwards of W1 / b1 (k_mm2b), then ONE launch of the
// W1 and W2 gradients (k_mm2, the pending bias / W3 updates in its extra plane), then layer 1.
template <typename T>
bool quad_ok(const MlpNet<T>& net, const SubStep<T>* ss) {
  if (sizeof(T) != 4) return false;                            // float64: two fused grids fit, not four
  const int mk = mask_kind(ss[0].ms);
  if (mk != MK_KEEP && mk != MK_VALS) return false;
  if (net.l23_fit < 4 || net.n_mid % (int)(16 / sizeof(T)) || net.n_in % (int)(16 / sizeof(T))) return false;
  if (!net.vec_masks || !vec_ok(net.xw, net.n_mid, sizeof(T))) return false;
  for (int i = 0; i < 6; ++i)
    if (!vec_ok(ss[i].q[2], net.n_mid, sizeof(T)) || !vec_ok(ss[i].scr->ga2, net.n_mid, sizeof(T))) return false;
  return true;
}

template <typename T>
hipError_t mlp_l23_ga1(MlpNet<T>& net, const SubStep<T>* const* fw, int nf, const SubStep<T>* const* ga, int nga) {
  MMArgs<T> a1, a2;
  MMProbs3<T> p1{}, p2{};
  l23_build(net, fw, nf, 0, a1, p1);
  ga1_build(net, ga, nga, a2, p2);
  a1.pend.n = 0;
  a2.pend.n = 0;
  const int3 g1 = make_int3((a1.M + 31) / 32, (a1.N + 31) / 32, nf);
  const int3 g2 = make_int3((a2.M + 31) / 32, (a2.N + 31) / 32, nga);
  const dim3 grid((unsigned)std::max(g1.x, g2.x), (unsigned)std::max(g1.y, g2.y), (unsigned)(g1.z + g2.z));
  hipStream_t st = net.st;
  if constexpr (sizeof(T) == 4) {                              // float32 only (quad_ok)
    auto go = [&](auto mkc) {
      constexpr int MK = decltype(mkc)::value;
      hipLaunchKernelGGL((k_mm2b<T, MM_L23, OP_H1, OP_PLAIN, 0, 1, 1, 1, MM_GA1, OP_PLAIN, OP_PLAIN, 0, 0, 1, 0, MK>),
                         grid, dim3(MM_NT), 0, st, a1, p1, a2, p2, g1, g2);
    };
    if (mask_kind(a1.ms) == MK_KEEP) go(std::integral_constant<int, MK_KEEP>{});
    else go(std::integral_constant<int, MK_VALS>{});
    return hipGetLastError();
  }
  return hipErrorInvalidValue;
}

// k_fwdr in the batched sampler: float32 (the bench's dtype; float64 keeps the k_mm forwards), n_mid a
// multiple of 32 up to 256, n_out ≤ 16, keep-flag or buffer masks, 16-byte aligned xw / W2 rows and
// masks.  HMCX_MLP_FWDR=0 (read per call) keeps the k_mm fused forwards (MM_L23) — whose results the
// one-sub-step-at-a-time order reproduces bit for bit.
template <typename T>
bool fwdr_ok(const MlpNet<T>& net, const SubStep<T>* ss, int n) {
  const char* env = getenv("HMCX_MLP_FWDR");
  if ((env && env[0] == '0') || sizeof(T) != 4) return false;
  if (net.n_mid % 32 || net.n_mid > FR_NMAX || net.n_out > 16 || !net.vec_masks || !net.fpb2) return false;
  // layer 1 in two 16-byte-aligned split-K halves; the W2 gradient in 4 row quarters whose m0 masks start
  // on a keep word
  if (net.n_in % 8 || net.B % 4 || ((size_t)(net.B / 4) * net.n_mid) % 32) return false;
  const int mk = mask_kind(ss[0].ms);
  if (mk != MK_KEEP && mk != MK_VALS && mk != MK_PHILOX) return false;
  for (int i = 0; i < n; ++i) {
    const T* xw = ss[i].xw ? ss[i].xw : net.xw;
    if (!vec_ok(xw, net.n_mid, sizeof(T)) || !vec_ok(ss[i].q[2], net.n_mid, sizeof(T)) || mask_kind(ss[i].ms) != mk)
      return false;
    if (!vec_ok(ss[i].q[1], 4, 4) || !vec_ok(ss[i].q[3], 4, 4) || !vec_ok(ss[i].q[4], net.n_mid, sizeof(T))) return false;
    if (mk == MK_VALS && !vec_ok(ss[i].ms.vals, 4, 4)) return false;
  }
  return true;
}

// The forwards of np problems (sub-steps and energy forwards) in one k_fwdr launch: sub-step v writes
// ga2 when a backward reads it (W1, b1: the layer-1 backward; W2: its gradient) and the 16-row-block
// partials of its own bias / W3 gradient into its net's fpb2 / fpw3 / fpb3; energy forwards (v < 0)
// only their loss partials.  net's pending updates run in the extra plane.
template <typename T>
hipError_t mlp_fwdr(MlpNet<T>& net, const SubStep<T>* const* ss, int np, const RbFwdArgs<T>* flags = nullptr) {
  if (np < 1 || np > FR_MAXP) return hipErrorInvalidValue;
  RbFwdArgs<T> a{};
  if (flags) {                                                   // keep-flag rows: keep, n3, kr, seed, chain, step
    a.keep = flags->keep; a.n3 = flags->n3; a.kr = flags->kr; a.seed = flags->seed; a.chain = flags->chain;
    a.step = flags->step;
  }
  if (net.fr_prof && net.fr_prof_n < net.fr_prof_cap) {          // HMCX_FWDR_PROF: this launch's stamps
    a.prof = net.fr_prof + (size_t)net.fr_prof_n * net.nrb * FR_MAXP * FR_NPH;
    net.fr_prof_np[net.fr_prof_n++] = np;
  }
  a.M = net.B; a.n_mid = net.n_mid; a.n_out = net.n_out; a.np = np; a.y = net.y;
  for (int p = 0; p < np; ++p) {
    const SubStep<T>& x = *ss[p];
    RbFwdProb<T>& q = a.p[p];
    q.xw = x.xw ? x.xw : net.xw;
    q.xw2 = x.xw2;
    q.xwout = x.xwout;
    q.h1out = x.w.h1 ? x.scr->h1 : nullptr;
    q.b1 = x.q[1]; q.W2 = x.q[2]; q.b2 = x.q[3]; q.W3 = x.q[4]; q.b3 = x.q[5];
    q.ms = x.ms;
    q.ga2 = (x.v >= 0 && x.v <= 2) ? x.scr->ga2 : nullptr;
    q.pb2 = x.w.pb2 ? x.scr->fpb2 : nullptr;
    q.pw3 = x.w.pw3 ? x.scr->fpw3 : nullptr;
    q.pb3 = x.w.pb3 ? x.scr->fpb3 : nullptr;
    q.lpart = x.v < 0 ? x.lpart : nullptr;
  }
  a.pend = net.pend;
  net.pend.n = 0;
  const size_t kitems = (size_t)a.kr.nf * ((a.n3 + 63) / 64), per_row = (size_t)net.nrb * FR_NW * 64;
  const unsigned krows = (unsigned)((kitems + per_row - 1) / per_row);
  const dim3 grid((unsigned)net.nrb, (unsigned)(np + (a.pend.n > 0 ? 1 : 0)) + krows);
  if constexpr (sizeof(T) == 4) {                              // float32 only (fwdr_ok)
    const int mk = mask_kind(a.p[0].ms);
    if (mk == MK_PHILOX) hipLaunchKernelGGL((k_fwdr<T, MK_PHILOX>), grid, dim3(FR_NW * 64), 0, net.st, a);
    else if (mk == MK_KEEP) hipLaunchKernelGGL((k_fwdr<T, MK_KEEP>), grid, dim3(FR_NW * 64), 0, net.st, a);
    else hipLaunchKernelGGL((k_fwdr<T, MK_VALS>), grid, dim3(FR_NW * 64), 0, net.st, a);
    return hipGetLastError();
  }
  return hipErrorInvalidValue;
}

// Layer 1 as two split-K planes (k_fwdr sums them, plane 0 + plane 1): out[w][h] = X[:, K_h]·W1_w[:, K_h]ᵀ
// over the h-th half of n_in, for nw W1s in one batched launch — twice the workgroups of the plain
// layer 1 (config 3: 256 instead of 128, each half the 784-deep dot products); net's pending updates run
// in the extra plane.  Needs n_in % 8 == 0 (16-byte vectors in both halves).
template <typename T>
hipError_t mlp_layer1_split(MlpNet<T>& net, const T* const* W1, T* const (*out)[2], int nw) {
  const int Kh = net.n_in / 2;
  MMArgs<T> a{};
  MMProbs<T> pr{};
  pr.n = 2 * nw;
  for (int w = 0; w < nw; ++w)
    for (int h = 0; h < 2; ++h) {
      MMProb<T>& q = pr.p[2 * w + h];
      q.A = net.X + (size_t)h * Kh; q.B = W1[w] + (size_t)h * Kh; q.C = out[w][h];
    }
  mm_set<T>(a, net.B, net.n_mid, Kh, pr.p[0].A, net.n_in, 0, pr.p[0].B, net.n_in, 1, pr.p[0].C, net.n_mid);
  return mm<T, MM_STORE, 0, 1, OP_PLAIN, OP_PLAIN, true>(net, a, &pr);
}

// The W1 gradient (SGHMC epilogue; pn's pending bias / W3 updates in its extra plane) and the W2 gradient
// of sub-step net `w2n` as 4 split-K partial planes wp[4][n_mid][n_mid] over the minibatch rows, in ONE
// launch (k_mm2b): the W2 update itself runs as a pending update (4 partials, summed in plane order) in
// the NEXT launch.  200 + 256 workgroups at config 3 instead of 200 and a separate 64-workgroup W2 launch.
template <typename T>
hipError_t mlp_w1_w2split(MlpNet<T>& pn0, const SubStep<T>& s1, const Upd<T>& u1, MlpNet<T>& w2n, const SubStep<T>& s2,
                          T* wp) {
  MMArgs<T> a1, a2;
  MMProbs3<T> p1{}, p2{};
  wgrad_build(pn0, s1, 0, u1, a1);
  a1.pend = pn0.pend;
  pn0.pend.n = 0;
  wgrad_build(w2n, s2, 2, Upd<T>{}, a2);
  a2.upd_mode = UPD_NONE;
  a2.pend.n = 0;
  const bool h1 = s2.w.h1;                                     // B = the stored h1 (no xw / b1 / mask reads)
  if (h1) a2.B = w2n.h1;
  const int nm = w2n.n_mid, Kq = w2n.B / 4;
  a2.K = Kq;
  p2.n = 4;
  for (int q = 0; q < 4; ++q) {
    MMProb<T>& x = p2.p[q];
    const size_t r0 = (size_t)q * Kq * nm;                       // rows q·Kq … of ga2 and xw (and the m0 mask)
    x.A = a2.A + r0; x.B = a2.B + r0; x.C = wp + (size_t)q * nm * nm; x.b1 = a2.b1;
    x.ms = a2.ms;
    if (x.ms.keep) x.ms.keep += r0 / 32;
    if (x.ms.vals) x.ms.vals += r0;
    if (h1) x.ms = MaskSrc<T>{};
  }
  a2.C = p2.p[0].C; a2.ldc = nm;
  const int3 g1 = make_int3((a1.M + 31) / 32, (a1.N + 31) / 32, 1 + (a1.pend.n > 0 ? 1 : 0));
  const int3 g2 = make_int3((nm + 31) / 32, (nm + 31) / 32, 4);
  const dim3 grid((unsigned)std::max(g1.x, g2.x), (unsigned)std::max(g1.y, g2.y), (unsigned)(g1.z + g2.z));
  if constexpr (sizeof(T) == 4) {                              // float32 only (the k_fwdr path)
    auto go = [&](auto mkc) {
      constexpr int MK = decltype(mkc)::value;                 // the W1 gradient reads no masks
      hipLaunchKernelGGL((k_mm2b<T, MM_UPD, OP_PLAIN, OP_PLAIN, 1, 0, 0, 0, MM_STORE, OP_PLAIN, OP_H1, 1, 0, 0, 0, MK>),
                         grid, dim3(MM_NT), 0, pn0.st, a1, p1, a2, p2, g1, g2);
    };
    if (h1) {
      hipLaunchKernelGGL((k_mm2b<T, MM_UPD, OP_PLAIN, OP_PLAIN, 1, 0, 0, 0, MM_STORE, OP_PLAIN, OP_PLAIN, 1, 0, 0, 0, MK_NONE>),
                         grid, dim3(MM_NT), 0, pn0.st, a1, p1, a2, p2, g1, g2);
      return hipGetLastError();
    }
    if (mask_kind(a2.ms) == MK_KEEP) go(std::integral_constant<int, MK_KEEP>{});
    else go(std::integral_constant<int, MK_VALS>{});
    return hipGetLastError();
  }
  return hipErrorInvalidValue;
}

// The layer-1 backwards of np sub-steps (W1, b1) in one batched launch.
template <typename T>
hipError_t mlp_ga1_batch(MlpNet<T>& net, const SubStep<T>* const* ss, int np) {
  MMArgs<T> a;
  MMProbs<T> pr{};
  ga1_build(net, ss, np, a, pr);
  return mm<T, MM_GA1, 0, 0, OP_PLAIN, OP_PLAIN, true>(net, a, &pr);
}

// Layer 1 of the next iteration (xw = X·W1ᵀ into `out`, net's X) and the W2 gradient of sub-step net
// `w2n` in one launch (k_mm2): the W2 gradient reads the CURRENT iteration's xw (another buffer) and
// writes only W2's momentum and next position; layer 1 reads only X and W1.  False: the operands are
// not all 16-byte aligned (the caller launches them one by one).
template <typename T>
hipError_t mlp_l1_w2(MlpNet<T>& net, const T* W1, T* out, MlpNet<T>& w2n, const SubStep<T>& s2, const Upd<T>& u2,
                     bool* done) {
  *done = false;
  MMArgs<T> a1{}, a2;
  MMProbs3<T> p1{};
  mm_set<T>(a1, net.B, net.n_mid, net.n_in, net.X, net.n_in, 0, W1, net.n_in, 1, out, net.n_mid);
  wgrad_build(w2n, s2, 2, u2, a2);
  a1.pend.n = 0;
  a2.pend.n = 0;
  const int mk = mask_kind(a2.ms);
  if (sizeof(T) != 4 || (mk != MK_KEEP && mk != MK_VALS) || net.n_in % 4 || !vec_ok(net.X, net.n_in, sizeof(T)) ||
      !vec_ok(W1, net.n_in, sizeof(T)))
    return hipSuccess;
  const int3 g1 = make_int3((a1.M + 31) / 32, (a1.N + 31) / 32, 1);
  const int2 g2 = make_int2((a2.M + 31) / 32, (a2.N + 31) / 32);
  const dim3 grid((unsigned)std::max(g1.x, g2.x), (unsigned)std::max(g1.y, g2.y), 2u);
  xcd_choose<T>(a1, (int)grid.x, (int)grid.y, g1.x, g1.y);     // layer 1: 4 × 4 tile blocks per XCD
  xcd_choose<T>(a2, (int)grid.x, (int)grid.y, g2.x, g2.y);     // W2 gradient: 2 × 4
  hipStream_t st = net.st;
  if constexpr (sizeof(T) == 4) {
    auto go = [&](auto mkc) {
      constexpr int MK = decltype(mkc)::value;   // layer 1 reads no masks: any kind is its plain code
      hipLaunchKernelGGL((k_mm2<T, MM_STORE, OP_PLAIN, OP_PLAIN, 0, 1, 1, 1, MM_UPD, OP_PLAIN, OP_H1, 1, 0, 0, 0, MK>),
                         grid, dim3(MM_NT), 0, st, a1, p1, a2, g1, g2);
    };
    if (mk == MK_KEEP) go(std::integral_constant<int, MK_KEEP>{});
    else go(std::integral_constant<int, MK_VALS>{});
    *done = true;
  }
  return hipGetLastError();
}

template <typename T>
hipError_t mlp_w1_w2(MlpNet<T>& net, MlpNet<T>& w1n, const SubStep<T>& s1, const Upd<T>& u1, MlpNet<T>& w2n,
                     const SubStep<T>& s2, const Upd<T>& u2) {
  MMArgs<T> a1, a2;
  MMProbs3<T> p1{};
  wgrad_build(w1n, s1, 0, u1, a1);
  wgrad_build(w2n, s2, 2, u2, a2);
  a1.pend = net.pend;
  net.pend.n = 0;
  a2.pend.n = 0;
  const int3 g1 = make_int3((a1.M + 31) / 32, (a1.N + 31) / 32, 1 + (a1.pend.n > 0 ? 1 : 0));
  const int2 g2 = make_int2((a2.M + 31) / 32, (a2.N + 31) / 32);
  const dim3 grid((unsigned)std::max(g1.x, g2.x), (unsigned)std::max(g1.y, g2.y), (unsigned)(g1.z + 1));
  xcd_choose<T>(a1, (int)grid.x, (int)grid.y, g1.x, g1.y);     // W1 gradient: y-major chunks
  xcd_choose<T>(a2, (int)grid.x, (int)grid.y, g2.x, g2.y);     // W2 gradient: 2 × 4 tile blocks
  hipStream_t st = net.st;
  if constexpr (sizeof(T) == 4) {                              // float32 only (quad_ok)
    auto go = [&](auto mkc) {
      constexpr int MK = decltype(mkc)::value;   // the W1 gradient reads no masks: any kind is its plain code
      hipLaunchKernelGGL((k_mm2<T, MM_UPD, OP_PLAIN, OP_PLAIN, 1, 0, 0, 0, MM_UPD, OP_PLAIN, OP_H1, 1, 0, 0, 0, MK>),
                         grid, dim3(MM_NT), 0, st, a1, p1, a2, g1, g2);
    };
    if (mask_kind(a2.ms) == MK_KEEP) go(std::integral_constant<int, MK_KEEP>{});
    else go(std::integral_constant<int, MK_VALS>{});
    return hipGetLastError();
  }
  return hipErrorInvalidValue;
}

// Queue the update of variable v from the partials of `src` (default: net's own) on net's next launch.
template <typename T>
void set_pending(MlpNet<T>& net, int v, int mode, const Upd<T>& u, const MlpNet<T>* src = nullptr) {
  if (!src) src = &net;
  Pending<T>& p = net.pend.p[net.pend.n++];
  p.mode = mode; p.u = u; p.nparts = net.nlb;
  switch (v) {
    case 1: p.part = src->pb1; p.n = net.n_mid; break;
    case 3: p.part = src->pb2; p.n = net.n_mid; break;
    case 4: p.part = src->pw3; p.n = net.n_out * net.n_mid; break;
    default: p.part = src->pb3; p.n = net.n_out; break;
  }
}

// The same from explicit partials [nparts][n] (k_fwdr's per-16-row-block partials).
template <typename T>
void set_pending_part(MlpNet<T>& net, int v, int mode, const Upd<T>& u, const T* part, int nparts) {
  Pending<T>& p = net.pend.p[net.pend.n++];
  p.mode = mode; p.u = u; p.nparts = nparts; p.part = part;
  p.n = net.nvar(v);
}

template <typename T>
hipError_t flush_pending(MlpNet<T>& net) {
  if (net.pend.n == 0) return hipSuccess;
  int n = 0;
  for (int j = 0; j < net.pend.n; ++j) n = std::max(n, net.pend.p[j].n);
  hipLaunchKernelGGL(k_pending<T>, dim3((n + 255) / 256), dim3(256), 0, net.st, net.pend);
  net.pend.n = 0;
  return hipGetLastError();
}

// Fused layer 2 + layer 3 (MM_L23) in the sampler when n_out ≤ 32, at most 16 column slices, and the
// whole grid fits on the chip at once (its slice workgroups wait for each other); HMCX_MLP_FUSE=0 or
// hmcx_set_mlp_fuse(ctx, 0) turns it off.  A timed-out exchange raises the MLP's own abort word
// (ctx->mlp_abort_dev, never the persistent SGHMC kernels' word) and the call reports it (out_abort).
// The arena holds `regions` equal parts: a batched fused launch gives problem p region p.
template <typename T>
int net_fuse(hmcx_ctx* ctx, MlpNet<T>& net, int regions = 1) {
  static const bool off = getenv("HMCX_MLP_FUSE") && getenv("HMCX_MLP_FUSE")[0] == '0';
  const int S = (net.n_mid + 31) / 32;
  if (off || ctx->mlp_nofuse || net.n_out > 32 || S > 16) return HMCX_OK;
  int per_cu = 0;
  const void* kfn = (const void*)k_mm<T, MM_L23, OP_H1, OP_PLAIN, 0, 1, 1, 1, MK_PHILOX>;
  HMCX_HIP(ctx, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, MM_NT, 0));
  if ((long)per_cu * ctx->num_cus < (long)net.nlb * S) return HMCX_OK;
  const size_t need = (size_t)net.nlb * S * 32 * net.n_out * 16;
  if (need > 0x7fffffff) return HMCX_OK;
  if (int rc = gx_reserve(ctx, need * regions)) return rc;
  // batched fused launches: the fewest workgroups per CU of the batched variants that can run
  int per_b = per_cu;
  for (const void* f : {(const void*)k_mmb<T, MM_L23, OP_H1, OP_PLAIN, 0, 1, 1, 1, MK_KEEP>,
                        (const void*)k_mmb<T, MM_L23, OP_H1, OP_PLAIN, 0, 1, 0, 0, MK_KEEP>,
                        (const void*)k_mmb<T, MM_L23, OP_H1, OP_PLAIN, 0, 1, 1, 1, MK_VALS>,
                        (const void*)k_mmb<T, MM_L23, OP_H1, OP_PLAIN, 0, 1, 0, 0, MK_VALS>,
                        (const void*)k_mmb<T, MM_L23, OP_H1, OP_PLAIN, 0, 1, 1, 1, MK_PHILOX>,
                        (const void*)k_mmb<T, MM_L23, OP_H1, OP_PLAIN, 0, 1, 0, 0, MK_PHILOX>}) {
    int pc = 0;
    if (int rc = kernel_occupancy(ctx, f, MM_NT, 0, &pc)) return rc;
    per_b = std::min(per_b, pc);
  }
  net.l23_fit = std::min(regions, (int)((long)per_b * ctx->num_cus / ((long)net.nlb * S)));
  if (!ctx->mlp_abort_dev) {
    HMCX_HIP(ctx, hipMalloc((void**)&ctx->mlp_abort_dev, sizeof(int)));
    HMCX_HIP(ctx, hipMemsetAsync(ctx->mlp_abort_dev, 0, sizeof(int), ctx->stream));
  }
  net.gx = ctx->gx_arena;
  net.gx_bytes = (int)need;
  net.ctx = ctx;
  net.abort_flag = ctx->mlp_abort_dev;
  net.fuse = true;
  const char* fa = getenv("HMCX_MLP_FORCE_ABORT");
  net.force_abort = fa ? atoi(fa) : -1;
  return HMCX_OK;
}

template <typename T>
void mlp_workspace(Workspace& ws, MlpNet<T>& net) {
  const size_t mn = (size_t)net.B * net.n_mid;
  net.xw = ws.take<T>(mn); net.h2 = ws.take<T>(mn); net.d3 = ws.take<T>(mn); net.h1 = ws.take<T>(mn);
  net.ga2 = ws.take<T>(mn); net.ga1 = ws.take<T>(mn);
  net.z = ws.take<T>((size_t)net.B * net.n_out); net.gz = ws.take<T>((size_t)net.B * net.n_out);
  net.pb1 = ws.take<T>((size_t)net.nlb * net.n_mid);
  net.pb2 = ws.take<T>((size_t)net.nlb * net.n_mid);
  net.pb3 = ws.take<T>((size_t)net.nlb * net.n_out);
  net.pw3 = ws.take<T>((size_t)net.nlb * net.n_out * net.n_mid);
}

}  // namespace

template <typename T>
int mlp_masks_t(hmcx_ctx* ctx, int B, int n_mid, uint64_t seed, uint32_t chain, uint32_t step, uint32_t slot,
                void* out) {
  const int n3 = 3 * B * n_mid;
  hipLaunchKernelGGL(k_mlp_masks<T>, dim3((unsigned)(((n3 + 63) / 64 + 255) / 256)), dim3(256), 0, ctx->stream,
                     (T*)out, n3, seed, chain, step, slot);
  HMCX_HIP(ctx, hipGetLastError());
  return HMCX_OK;
}

template <typename T>
int mlp_grad_t(hmcx_ctx* ctx, const void* X, const int32_t* y, int B, int n_in, int n_mid, int n_out,
               const hmcx_mlp_params* par, const void* masks, double alpha, hmcx_mlp_params* grads, double* loss) {
  MlpNet<T> net{};
  net_init(net, B, n_in, n_mid, n_out, ctx->stream);
  net.X = (const T*)X; net.y = y;          // one-off calls run unfused: no exchange that could time out
  Workspace ws(ctx);
  double* lpart;
  do { ws.reset(); mlp_workspace<T>(ws, net); lpart = ws.take<double>(net.nlb); } while (ws.retry());
  if (ws.failed) return HMCX_ENOMEM;
  const MaskSrc<T> ms{(const T*)masks, nullptr, T(1), B * n_mid, 0, 0, 0, 0};
  if (masks && (uintptr_t)masks % 16) net.vec_masks = false;
  T* q[6];
  for (int v = 0; v < 6; ++v) q[v] = (T*)par->p[v];
  HMCX_HIP(ctx, mlp_forward<T>(net, q, ms, lpart, L3Want{true, true, true, true}));
  HMCX_HIP(ctx, mlp_ga1<T>(net, q, ms, true));
  Upd<T> u{};
  u.half_alpha = (T)(0.5 * alpha);
  for (int v : {0, 2}) {
    u.W = q[v]; u.G = (T*)grads->p[v];
    HMCX_HIP(ctx, mlp_wgrad<T>(net, q, ms, v, UPD_GRAD, u));
  }
  for (int v : {1, 3, 4, 5}) {
    u.W = q[v]; u.G = (T*)grads->p[v];
    set_pending(net, v, UPD_GRAD, u);
    HMCX_HIP(ctx, flush_pending(net));
  }
  if (loss) {
    hipLaunchKernelGGL(k_loss_final, dim3(1), dim3(1), 0, ctx->stream, lpart, net.nlb, B, loss);
    HMCX_HIP(ctx, hipGetLastError());
  }
  return HMCX_OK;
}

// The full-batch HMC trajectory of hmcx_mlp_hmc_leapfrog (hmc.py:46-56): g = grad(q); per iteration and
// variable v = order[i]: p_v −= ε/2·g_v, q_v += ε·p_v, g = grad(q), p_v −= ε·g_v; then p = −p.  Of each
// gradient only two components are ever read — g_v (this sub-step's second kick) and g_v' of the next
// variable (its first kick) — so each call computes just those, with mlp_grad_t's kernels and flags
// for them (identical bits), and the layer-1 output xw is reused until W1 itself moves.
template <typename T>
int mlp_leapfrog_t(hmcx_ctx* ctx, const hmcx_mlp_leapfrog_args* s) {
  MlpNet<T> net{};
  net_init(net, s->B, s->n_in, s->n_mid, s->n_out, ctx->stream);
  net.X = (const T*)s->X; net.y = s->y;                       // unfused (see mlp_grad_t)
  Workspace ws(ctx);
  double* lpart;
  do { ws.reset(); mlp_workspace<T>(ws, net); lpart = ws.take<double>(net.nlb); } while (ws.retry());
  if (ws.failed) return HMCX_ENOMEM;
  const void* mptr = s->mask_mode == HMCX_MLP_MASKS_NONE ? nullptr : s->masks;
  const MaskSrc<T> ms{(const T*)mptr, nullptr, T(1), s->B * s->n_mid, 0, 0, 0, 0};
  if (mptr && (uintptr_t)mptr % 16) net.vec_masks = false;
  T *q[6], *p[6], *g[6];
  int64_t dim[6];
  for (int v = 0; v < 6; ++v) {
    q[v] = (T*)s->q.p[v]; p[v] = (T*)s->p.p[v]; g[v] = (T*)s->g.p[v];
    dim[v] = net.nvar(v);
  }
  uint32_t slot = s->slot0;
  const bool pmasks = s->mask_mode == HMCX_MLP_MASKS_PHILOX;
  // the gradient components `want` (bit v) at q, in mlp_grad_t's order: forward (+ the layer-3 backward
  // pieces the wanted components use), layer-1 backward, W1 / W2 gradients, then the bias / W3 updates (one
  // k_pending launch for all of them: independent element-wise updates).  The call's masks are drawn by the
  // kicks launch before it (draw = false), except for the first call.
  auto grad = [&](unsigned want, bool draw, bool defer) -> int {
    if (pmasks && draw)
      if (int rc = mlp_masks_t<T>(ctx, s->B, s->n_mid, s->seed, s->chain, s->step, slot++, s->masks)) return rc;
    const bool l1 = want & 3u;
    HMCX_HIP(ctx, mlp_forward<T>(net, q, ms, lpart,
                                 L3Want{(want & 15u) != 0, (want & 8u) != 0, (want & 32u) != 0, (want & 16u) != 0}));
    if (l1) HMCX_HIP(ctx, mlp_ga1<T>(net, q, ms, true));
    Upd<T> u{};
    u.half_alpha = (T)(0.5 * s->alpha);
    for (int v : {0, 2})
      if (want & (1u << v)) {
        u.W = q[v]; u.G = g[v];
        HMCX_HIP(ctx, mlp_wgrad<T>(net, q, ms, v, UPD_GRAD, u));
      }
    for (int v : {1, 3, 4, 5})
      if (want & (1u << v)) {
        u.W = q[v]; u.G = g[v];
        set_pending(net, v, UPD_GRAD, u);
      }
    if (!defer) HMCX_HIP(ctx, flush_pending(net));            // else: the next kicks launch applies them
    return HMCX_OK;
  };
  // one launch between two gradient calls: the second kick of variable pu (−1: none, hmc.py:53), the first
  // kick and the drift of variable nv (−1: none, :50-51), and the next call's masks
  auto kicks = [&](int pu, int nv, bool masks) -> int {
    MlpKicks<T> k{};
    int64_t n = 0;
    if (pu >= 0) { k.pu = p[pu]; k.gu = g[pu]; k.nu = dim[pu]; k.eu = (T)s->eps; n = std::max(n, k.nu); }
    if (nv >= 0) {
      k.pv = p[nv]; k.gv = g[nv]; k.qv = q[nv]; k.nv = dim[nv]; k.hv = (T)(0.5 * s->eps); k.ev = (T)s->eps;
      n = std::max(n, k.nv);
    }
    if (masks && pmasks) {
      k.masks = (T*)s->masks; k.n3 = 3 * s->B * s->n_mid; k.seed = s->seed; k.chain = s->chain; k.step = s->step;
      k.slot = slot++;
      n = std::max(n, (int64_t)(k.n3 + 63) / 64);
    }
    k.ps = net.pend;                                           // the previous call's deferred bias / W3 gradients
    net.pend.n = 0;
    if (n == 0) return HMCX_OK;
    const unsigned nb = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_mlp_kicks<T>, dim3(nb, 3), dim3(256), 0, ctx->stream, k);
    HMCX_HIP(ctx, hipGetLastError());
    return HMCX_OK;
  };
  const int* o = s->order;
  // the last gradient call computes all six components, so g is the full gradient at the final
  // position (as the header promises); every earlier call only the two the next kicks read
  if (int rc = grad(s->n_iter > 0 ? 1u << o[0] : 63u, true, s->n_iter > 0)) return rc;
  for (int it = 0; it < s->n_iter; ++it)
    for (int i = 0; i < 6; ++i) {
      const int v = o[i];
      const bool tail = it == s->n_iter - 1 && i == 5;        // no next kick follows
      // :53 of the previous sub-step (none before the first), :50-51 of this one, this call's masks
      int rc = kicks(it == 0 && i == 0 ? -1 : o[(i + 5) % 6], v, true);
      if (v == 0) net.xw_valid = false;
      if (!rc) rc = grad(tail ? 63u : (1u << v) | (1u << o[(i + 1) % 6]), false, !tail);   // :52
      if (rc) return rc;
    }
  if (s->n_iter > 0)
    if (int rc = kicks(o[5], -1, false)) return rc;                                   // :53 of the last sub-step
  Neg6<T> ng{};                                                                         // :55-56
  int64_t nmax = 0;
  for (int v = 0; v < 6; ++v) { ng.p[v] = p[v]; ng.n[v] = dim[v]; nmax = std::max(nmax, dim[v]); }
  hipLaunchKernelGGL(k_mlp_neg6<T>, dim3((unsigned)std::min<int64_t>((nmax + 255) / 256, 4096), 6), dim3(256), 0,
                     ctx->stream, ng);
  HMCX_HIP(ctx, hipGetLastError());
  return HMCX_OK;
}

template <typename T>
int mlp_loss_t(hmcx_ctx* ctx, const void* X, const int32_t* y, int B, int n_in, int n_mid, int n_out,
               const hmcx_mlp_params* par, const void* masks, double* loss, void* logits) {
  MlpNet<T> net{};
  net_init(net, B, n_in, n_mid, n_out, ctx->stream);
  net.X = (const T*)X; net.y = y;          // unfused (see mlp_grad_t)
  Workspace ws(ctx);
  double* lpart;
  do { ws.reset(); mlp_workspace<T>(ws, net); lpart = ws.take<double>(net.nlb); } while (ws.retry());
  if (ws.failed) return HMCX_ENOMEM;
  const MaskSrc<T> ms{(const T*)masks, nullptr, T(1), B * n_mid, 0, 0, 0, 0};
  if (masks && (uintptr_t)masks % 16) net.vec_masks = false;
  T* q[6];
  for (int v = 0; v < 6; ++v) q[v] = (T*)par->p[v];
  HMCX_HIP(ctx, mlp_forward<T>(net, q, ms, y ? lpart : nullptr, L3Want{false, false, false, false}, (T*)logits));
  if (logits) {
    const int n = B * n_out;
    hipLaunchKernelGGL(k_bias_into_z<T>, dim3((n + 255) / 256), dim3(256), 0, ctx->stream, (T*)logits, q[5], n, n_out);
    HMCX_HIP(ctx, hipGetLastError());
  }
  if (y && loss) {
    hipLaunchKernelGGL(k_loss_final, dim3(1), dim3(1), 0, ctx->stream, lpart, net.nlb, B, loss);
    HMCX_HIP(ctx, hipGetLastError());
  }
  return HMCX_OK;
}

template <typename T>
int mlp_sghmc_t(hmcx_ctx* ctx, const hmcx_mlp_sghmc_args* s) {
  MlpNet<T> net{};
  net_init(net, s->B, s->n_in, s->n_mid, s->n_out, ctx->stream);
  if (int rc0 = net_fuse<T>(ctx, net, MAXPROB)) return rc0;
  const int mn = s->B * s->n_mid, n3 = 3 * mn;
  int off_v[6], dim[6], P = 0;                                // element offset of each variable in `order`
  {
    int seen = 0;
    for (int i = 0; i < 6; ++i) {
      const int v = s->order[i];
      if (v < 0 || v > 5 || ((seen >> v) & 1))
        return set_error(ctx, HMCX_EINVAL, "mlp sghmc: order must be a permutation of 0..5");
      seen |= 1 << v;
      off_v[v] = P;
      dim[v] = net.nvar(v);
      P += dim[v];
    }
  }
  int maxF = 2;
  for (int si = 0; si < s->n_steps; ++si) {
    if (s->n_iter[si] < 0) return set_error(ctx, HMCX_EINVAL, "mlp sghmc: n_iter < 0");
    // the step-start launch has one grid row per forward of the step (gridDim.y = 6 + 6·n_iter + 2,
    // capped at 65535 by the hardware)
    if (s->n_iter[si] > (65535 - 8) / 6)
      return set_error(ctx, HMCX_EINVAL, "mlp sghmc: n_iter above 10921 leapfrog iterations per step");
    maxF = std::max(maxF, 6 * s->n_iter[si] + 2);
  }
  const bool philox_masks = s->mask_mode == HMCX_NOISE_PHILOX;
  // Philox masks: the flags of a whole step stored once by k_mlp_keep and loaded by the kernels
  // (default), or drawn inside the kernels where they are read (HMCX_MLP_MASKS=philox).  Measured on
  // one box at config 3 (tools/gpu_r03_mlp_env.sh): 7.22 k leapfrog/s stored vs 6.38 k drawn — the
  // draws sit on the layer-2 GEMM's critical path; stored h1 for the W1 / b1 / W2 backward
  // (HMCX_MLP_H1=1) recovers most of it when drawn (6.76 k) and changes nothing when stored (7.19 k).
  const char* mk_env = getenv("HMCX_MLP_MASKS");
  const bool keep_arr = philox_masks && !(mk_env && !strcmp(mk_env, "philox"));
  const char* ks_env = getenv("HMCX_MLP_KEEP_SPLIT");
  const bool keep_split_on = !(ks_env && ks_env[0] == '0');
  const char* h1_env = getenv("HMCX_MLP_H1");
  const bool store_h1 = philox_masks && h1_env && h1_env[0] == '1';    // m0 ∈ {0, scale} only for Philox masks
  // Batched iterations.  Sub-step i of leapfrog iteration it (variable v = order[i]) evaluates the
  // gradient at q_u(it) for the variables at order positions u ≤ i and q_u(it − 1) for the others
  // (sghmc.py:29-34: each variable is drifted just before its own gradient call) and moves only v's
  // momentum and v's NEXT position — so it needs iteration it − 1 complete and nothing of iteration it:
  // the six sub-steps of one iteration are independent.  With W1 first (one xw per iteration), an
  // iteration is: layer 1 (+ the previous iteration's bias / W3 updates in its prologue), the six fused
  // forwards in one launch (or in chunks of what fits co-resident), the W1 / b1 layer-1 backwards in
  // one launch, the W1 and W2 gradients with their SGHMC epilogues — 5 launches instead of 11.  Same
  // kernels, operands, masks and noise as the one-at-a-time order: identical results.
  // HMCX_MLP_BATCH=0 runs the sub-steps one at a time.
  const char* batch_env = getenv("HMCX_MLP_BATCH");             // read per call (tests switch it)
  const bool batch_off = batch_env && batch_env[0] == '0';
  const bool batch = !batch_off && net.fuse && s->order[0] == 0 && !store_h1 && net.l23_fit >= 1;
  MlpNet<T> pn[6]{};
  MlpNet<T> en[2]{};                                           // scratch (gz) of the E_new / E_current forwards
  if (philox_masks) {
    if (n3 % 4) net.vec_masks = false;
  } else {
    if ((uintptr_t)s->masks % 16 || ((size_t)n3 * sizeof(T)) % 16) net.vec_masks = false;
    for (int si = 0; si < s->n_steps; ++si)
      if ((s->mask_off[si] * sizeof(T)) % 16) net.vec_masks = false;
  }
  Workspace ws(ctx);
  T *pv[6], *qa[6], *qb[6], *qc[6], *xw_par = nullptr, *xw_b1 = nullptr;
  T *xwp[2] = {}, *xpar[2] = {}, *w2part = nullptr;           // k_fwdr path: layer-1 split-K planes, W2 partials
  double *part_cur, *part_new, *lp_cur, *lp_new, *lp_scr;
  uint32_t* keep = nullptr;                                  // keep flags of the step: one bit per element
  const int kw = (n3 + 31) / 32;                              // words per forward
  int32_t* accf;
  static const char* prof_path = getenv("HMCX_MLP_PROF");
  static const char* fr_prof_path = getenv("HMCX_FWDR_PROF");
  const int prof_cap = prof_path && net.fuse ? 8192 : 0;
  do {
    ws.reset();
    mlp_workspace<T>(ws, net);
    for (int i = 0; i < 6 && batch; ++i) {
      net_init(pn[i], s->B, s->n_in, s->n_mid, s->n_out, ctx->stream);
      mlp_workspace<T>(ws, pn[i]);
      pn[i].lpart_scr = ws.take<double>(net.nlb);
      pn[i].fpb2 = ws.take<T>((size_t)net.nrb * s->n_mid);       // k_fwdr's 16-row-block partials
      pn[i].fpw3 = ws.take<T>((size_t)net.nrb * s->n_out * s->n_mid);
      pn[i].fpb3 = ws.take<T>((size_t)net.nrb * s->n_out);
    }
    net.fpb2 = batch ? pn[0].fpb2 : nullptr;                       // marks the buffers as present (fwdr_ok)
    net.prof = prof_cap ? ws.take<unsigned long long>((size_t)prof_cap * net.nlb * ((net.n_mid + 31) / 32) * L23_NPH)
                        : nullptr;
    net.fr_prof_cap = fr_prof_path ? 512 : 0;
    net.fr_prof_np.assign(net.fr_prof_cap, 0);
    net.fr_prof = fr_prof_path ? ws.take<unsigned long long>((size_t)512 * net.nrb * FR_MAXP * FR_NPH) : nullptr;
    net.prof_cap = prof_cap;
    for (int v = 0; v < 6; ++v) {
      pv[v] = ws.take<T>(dim[v]); qa[v] = ws.take<T>(dim[v]); qb[v] = ws.take<T>(dim[v]);
      qc[v] = batch ? ws.take<T>(dim[v]) : nullptr;
    }
    if (batch) {
      xw_par = ws.take<T>((size_t)mn);
      xw_b1 = ws.take<T>((size_t)mn);
      for (int h = 0; h < 2; ++h) { xwp[h] = ws.take<T>((size_t)mn); xpar[h] = ws.take<T>((size_t)mn); }
      w2part = ws.take<T>((size_t)4 * s->n_mid * s->n_mid);
      for (auto& e : en) e.gz = ws.take<T>((size_t)s->B * s->n_out);
    }
    part_cur = ws.take<double>(12 * NPART);
    part_new = ws.take<double>(12 * NPART);
    lp_cur = ws.take<double>(std::max(net.nlb, net.nrb));        // 32-row (k_mm) or 16-row (k_fwdr) partials
    lp_new = ws.take<double>(std::max(net.nlb, net.nrb));
    lp_scr = ws.take<double>(net.nlb);
    if (keep_arr) keep = ws.take<uint32_t>((size_t)maxF * kw);
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
  bool commit_pending = false;                                // the previous step's proposal awaits its commit
  T* prev_prop[6] = {};

  for (int si = 0; si < s->n_steps; ++si) {
    net.X = Xall + (size_t)s->row0[si] * s->n_in;
    net.y = s->y + s->row0[si];
    net.xw_valid = false;
    const double eps = s->eps[si];
    const int n = s->n_iter[si], F = 6 * n + 2;
    const uint32_t step_id = s->step_base + (uint32_t)si;
    const double* nz = s->noise_mode == HMCX_NOISE_BUFFER ? s->noise + s->noise_off[si] : nullptr;
    // the k_fwdr path for this step's iterations (decided before the momentum launch: with Philox masks
    // k_fwdr draws every mask itself, so the step's keep flags are not drawn at all)
    bool fr_step = false;
    if (batch && n > 0) {
      SubStep<T> chk[6];
      for (int i = 0; i < 6; ++i) {
        for (int j = 0; j < 6; ++j) chk[i].q[s->order[j]] = j <= i ? qa[s->order[j]] : par[s->order[j]];
        chk[i].xw = xw_par;
        chk[i].ms = !philox_masks ? MaskSrc<T>{(const T*)s->masks + s->mask_off[si], nullptr, scale, mn, 0, 0, 0, 0}
                    : keep_arr ? MaskSrc<T>{nullptr, keep, scale, mn, 0, 0, 0, 0}
                               : MaskSrc<T>{nullptr, nullptr, scale, mn, s->seed, s->chain, step_id, MASK_SLOT0};
      }
      fr_step = fwdr_ok(net, chk, 6);
    }
    // keep flags of every forward of the step in the momentum launch (compute-bound Philox draws: drawn
    // instead beside each iteration's last launch, in an extra plane, they lengthened that launch by as
    // much as they took off this one — 21.46 k vs 22.2 k leapfrog/s at config 3)
    const bool fused_start = philox_masks && keep_arr;
    // On the k_fwdr path the step-start launch draws only iteration 0's flags and the two energy forwards';
    // each iteration's k_fwdr draws the next iteration's in rows of its own, on the CUs its problems leave free
    // (HMCX_MLP_KEEP_SPLIT=0: all at step start)
    const bool keep_split = fused_start && fr_step && n > 1 && keep_split_on;
    auto masks_for = [&](int f) -> MaskSrc<T> {
      // PHILOX: the kernels draw the flags they read (MK_PHILOX, slot MASK_SLOT0 + f); with
      // HMCX_MLP_MASKS=keep, k_mlp_keep stores the same flags once per step and the kernels load them
      if (philox_masks && !keep_arr)
        return MaskSrc<T>{nullptr, nullptr, scale, mn, s->seed, s->chain, step_id, MASK_SLOT0 + (uint32_t)f};
      if (philox_masks) return MaskSrc<T>{nullptr, keep + (size_t)f * kw, scale, mn, 0, 0, 0, 0};
      return MaskSrc<T>{(const T*)s->masks + s->mask_off[si] + (size_t)f * n3, nullptr, scale, mn, 0, 0, 0, 0};
    };
    // momentum (hmc.py:82-87), first drift into qa, Σp², Σθ² of the current state
    VarTab vt{};
    for (int i = 0; i < 6; ++i) {
      const int v = s->order[i];
      vt.q[i] = par[v]; vt.qn[i] = qa[v]; vt.p[i] = pv[v]; vt.n[i] = dim[v]; vt.e0[i] = off_v[v];
      vt.qc[i] = commit_pending ? prev_prop[v] : nullptr;
    }
    const int32_t* prev_acc = commit_pending ? accf : nullptr;   // the previous step's commit, folded in
    commit_pending = false;
    if (fused_start) {
      // forwards 0 … 5 and the energies 6n, 6n + 1 when split, else all F
      const KeepRange kr = keep_split ? KeepRange{8, 0, 6, 6 * n} : KeepRange{F, 0, F, 0};
      const size_t items = (size_t)kr.nf * ((n3 + 63) / 64);        // one keep group per thread
      const unsigned rows = (unsigned)((items + (size_t)NPART * 256 - 1) / ((size_t)NPART * 256));
      hipLaunchKernelGGL(k_mlp_start<T>, dim3(NPART, 6 + rows), dim3(256), 0, st, vt, (T)eps,
                         n > 0 ? 1 : 0, s->noise_mode, nz, s->seed, s->chain, step_id, part_cur, prev_acc, keep, n3, kr);
    } else {
      hipLaunchKernelGGL(k_mlp_init<T>, dim3(NPART, 6), dim3(256), 0, st, vt, (T)eps, n > 0 ? 1 : 0, s->noise_mode,
                         nz, s->seed, s->chain, step_id, part_cur, prev_acc);
    }
    T* cur[6];
    for (int v = 0; v < 6; ++v) cur[v] = par[v];
    int fwd = 0;
    bool e_fr[2] = {false, false};                            // E_new / E_current by k_fwdr (16-row partials)
    auto upd_for = [&](int it, int v, T* W, T* Qn) {
      Upd<T> u{};
      u.W = W; u.P = pv[v]; u.Qn = Qn;
      u.half_alpha = (T)(0.5 * s->alpha); u.eps = (T)eps; u.one_minus_eps = (T)(1.0 - eps);
      u.noise_scale = (T)(2.0 * eps);
      u.noise_mode = s->noise_mode;
      u.noise = nz ? nz + (size_t)P * (it + 1) + off_v[v] : nullptr;   // BUFFER: one block of P per iteration
      u.seed = s->seed; u.chain = s->chain; u.step = step_id; u.slot = (uint32_t)(it + 1);
      u.e0 = (uint32_t)off_v[v];
      return u;
    };
    if (batch && n > 0) {
      // positions of iteration it in q3[it % 3]: the sub-steps of iteration it read iterations it and
      // it − 1 and write it + 1, so three sets never alias within an iteration (the pending updates of
      // the bias / W3 sub-steps then run beside readers of it − 1)
      T* const* q3[3] = {qa, qb, qc};
      // as many fused forwards per launch as fit co-resident (f32 at config 3: 4 at two workgroups per
      // CU; three per CU with the registers spilled measured slower: one 6-problem launch 47.8 µs vs
      // 23.8 + 17.4 for 4 + 2)
      const int fit = std::min(MAXPROB, net.l23_fit);
      for (int i = 0; i < 6; ++i) {
        pn[i].X = net.X; pn[i].y = net.y; pn[i].xw = net.xw; pn[i].vec_masks = net.vec_masks;
      }
      // energies (hmc.py:67-71): E_new at the last iteration's positions with forward 6n's masks,
      // E_current at the start state with forward 6n + 1's.  Both only need what is known when the
      // last (first) iteration starts, so they ride in its second launch when there is room
      // xw of iteration it in xwb[it & 1]: the next iteration's layer 1 may run beside this
      // iteration's W2 gradient, which reads this iteration's xw
      T* const xwb[2] = {net.xw, xw_b1};
      SubStep<T> es[2];
      bool e_done[2] = {false, false};
      bool l1_done = false;
      T* const* Xlast = q3[(n - 1) % 3];
      for (int e = 0; e < 2; ++e) {
        SubStep<T>& x = es[e];
        x.xw = e == 0 ? xwb[(n - 1) & 1] : xw_par;
        for (int v = 0; v < 6; ++v) x.q[v] = e == 0 ? Xlast[v] : par[v];
        x.ms = masks_for(6 * n + e);
        x.scr = &en[e];
        x.lpart = e == 0 ? lp_new : lp_cur;
        x.w = L3Want{false, false, false, false, false};
        x.v = -1;
      }
      bool use_fr = false;                                     // the k_fwdr path (decided in iteration 0)
      for (int it = 0; it < n; ++it) {
        T* const* Xit = q3[it % 3];                              // positions of iteration it
        T* const* Xpr = it == 0 ? par : q3[(it + 2) % 3];        // of iteration it − 1
        T* const* Xnx = q3[(it + 1) % 3];                        // the next iteration's (written here)
        net.xw = xwb[it & 1];
        for (int i = 0; i < 6; ++i) pn[i].xw = net.xw;
        SubStep<T> ss[6];
        const SubStep<T>* ga[6];
        int nga = 0;
        for (int i = 0; i < 6; ++i) {
          const int v = s->order[i];
          SubStep<T>& x = ss[i];
          x.xw = nullptr;
          for (int j = 0; j < 6; ++j) x.q[s->order[j]] = j <= i ? Xit[s->order[j]] : Xpr[s->order[j]];
          x.ms = masks_for(6 * it + i);
          x.scr = &pn[i];
          x.lpart = pn[i].lpart_scr;
          x.w = L3Want{v <= 3, v == 3, v == 5, v == 4, false};
          x.v = v;
          if (v <= 1) ga[nga++] = &ss[i];
        }
        int i2 = 0;                                              // position of the W2 sub-step
        while (s->order[i2] != 2) ++i2;
        if (it == 0) {
          SubStep<T> chk[8];
          for (int i = 0; i < 6; ++i) chk[i] = ss[i];
          chk[6] = es[0];
          chk[7] = es[1];
          use_fr = fr_step && fwdr_ok(net, chk, 8);
          if (keep_split && !use_fr) {                          // the k_mm forwards: draw the rest now
            const KeepRange kr{6 * n - 6, 6, 6 * n - 6, 0};
            const size_t items = (size_t)kr.nf * ((n3 + 63) / 64);
            hipLaunchKernelGGL(k_mlp_keep, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, st, keep, n3, kr,
                               s->seed, s->chain, step_id);
          }
        }
        if (use_fr) {
          // 4 launches per iteration, the layer-1 GEMM and the W2 gradient as split-K partials:
          //  A  k_fwdr: every forward of the iteration (and the energy forwards due) — h1 from the two
          //     layer-1 planes, whose sum problem 0 stores as the iteration's xw;
          //  B  the W1 / b1 layer-1 backwards;
          //  C  the W1 gradient (SGHMC epilogue) + the W2 gradient as 4 row-quarter partials, the pending
          //     bias / W3 updates in the extra plane;
          //  D  the next iteration's layer 1 (two split-K planes) with the W2 update from its 4 partials in
          //     the extra plane (after the last iteration: flushed before the kinetic energies).
          if (it == 0) {                                          // layer 1 of iteration 0 and of the start state
            const T* w1[2] = {qa[0], par[0]};
            T* const out[2][2] = {{xwp[0], xwp[1]}, {xpar[0], xpar[1]}};
            HMCX_HIP(ctx, mlp_layer1_split<T>(net, w1, out, 2));
          }
          const SubStep<T>* fa[FR_MAXP];
          int na = 0;
          for (int i = 0; i < 6; ++i) {
            ss[i].xw = xwp[0];
            ss[i].xw2 = xwp[1];
            // masks drawn inside k_fwdr (HMCX_MLP_MASKS=philox) live only there: it stores h1 for the W1 / b1
            // gates and the W2 gradient
            ss[i].w.h1 = philox_masks && !keep_arr && ss[i].v <= 2;
            fa[na++] = &ss[i];
          }
          ss[0].xwout = net.xw;
          if (it == n - 1) {
            es[0].xw = xwp[0];
            es[0].xw2 = xwp[1];
            fa[na++] = &es[0];
            e_done[0] = e_fr[0] = true;
          }
          if (it == 0) {
            es[1].xw = xpar[0];
            es[1].xw2 = xpar[1];
            fa[na++] = &es[1];
            e_done[1] = e_fr[1] = true;
          }
          RbFwdArgs<T> kf{};                                    // the next iteration's flags, in k_fwdr's free rows
          if (keep_split && it + 1 < n) {
            kf.keep = keep; kf.n3 = n3; kf.kr = KeepRange{6, 6 * (it + 1), 6, 0};
            kf.seed = s->seed; kf.chain = s->chain; kf.step = step_id;
          }
          HMCX_HIP(ctx, mlp_fwdr<T>(net, fa, na, &kf));
          HMCX_HIP(ctx, mlp_ga1_batch<T>(net, ga, nga));
          for (int i = 0; i < 6; ++i) {
            const int v = s->order[i];
            if (v == 0 || v == 2) continue;
            const Upd<T> u = upd_for(it, v, Xit[v], it + 1 < n ? Xnx[v] : nullptr);
            if (v == 1) set_pending(pn[0], v, UPD_SGHMC, u, &pn[i]);   // b1: the layer-1 backward's 32-row partials
            else set_pending_part(pn[0], v, UPD_SGHMC, u, v == 3 ? pn[i].fpb2 : v == 4 ? pn[i].fpw3 : pn[i].fpb3,
                                  net.nrb);
          }
          HMCX_HIP(ctx, mlp_w1_w2split<T>(pn[0], ss[0], upd_for(it, 0, Xit[0], it + 1 < n ? Xnx[0] : nullptr),
                                          pn[i2], ss[i2], w2part));
          set_pending_part(net, 2, UPD_SGHMC, upd_for(it, 2, Xit[2], it + 1 < n ? Xnx[2] : nullptr), w2part, 4);
          if (it + 1 < n) {
            const T* w1[1] = {Xnx[0]};
            T* const out[1][2] = {{xwp[0], xwp[1]}};
            HMCX_HIP(ctx, mlp_layer1_split<T>(net, w1, out, 1));
          }
          fwd += 6;
          continue;
        }
        if (it == 0) {                                           // xw(0) and the start state's xw (E_current)
          const T* w1[2] = {qa[0], par[0]};
          T* out[2] = {net.xw, xw_par};
          HMCX_HIP(ctx, mlp_layer1_batch<T>(net, w1, out, 2));
        } else if (!l1_done) {
          HMCX_HIP(ctx, mlp_layer1<T>(net, Xit[0]));
        }
        l1_done = false;
        if (quad_ok(net, ss)) {
          // 4 launches: forwards of W1, b1, W2 (+ one more) | the other two forwards + the W1 / b1
          // layer-1 backwards | the W1 and W2 gradients + every pending update | layer 1
          const SubStep<T>* fa[6];
          const SubStep<T>* fb[6];
          int na = 0, nb = 0;
          for (int i = 0; i < 6; ++i)
            if (s->order[i] <= 2) fa[na++] = &ss[i];
          for (int i = 0; i < 6; ++i)
            if (s->order[i] > 2) {
              if (na < 4) fa[na++] = &ss[i];
              else fb[nb++] = &ss[i];
            }
          if (it == n - 1) { fb[nb++] = &es[0]; e_done[0] = true; }
          if (it == 0 && n > 1) { fb[nb++] = &es[1]; e_done[1] = true; }
          MMArgs<T> a;
          MMProbs<T> pr{};
          l23_build(net, fa, na, 0, a, pr);
          HMCX_HIP(ctx, (mm<T, MM_L23, 0, 1, OP_H1, OP_PLAIN, true>(net, a, &pr)));
          HMCX_HIP(ctx, mlp_l23_ga1<T>(net, fb, nb, ga, nga));
          // the W1 gradient with every pending bias / W3 update in its extra plane; then the next
          // iteration's layer 1 beside this iteration's W2 gradient (which needs neither)
          for (int i = 0; i < 6; ++i) {
            const int v = s->order[i];
            if (v != 0 && v != 2) set_pending(pn[0], v, UPD_SGHMC, upd_for(it, v, Xit[v], it + 1 < n ? Xnx[v] : nullptr), &pn[i]);
          }
          HMCX_HIP(ctx, mlp_wgrad<T>(pn[0], ss[0].q, ss[0].ms, 0, UPD_SGHMC,
                                     upd_for(it, 0, Xit[0], it + 1 < n ? Xnx[0] : nullptr)));
          const Upd<T> u2 = upd_for(it, 2, Xit[2], it + 1 < n ? Xnx[2] : nullptr);
          if (it + 1 < n) HMCX_HIP(ctx, mlp_l1_w2<T>(net, Xnx[0], xwb[(it + 1) & 1], pn[i2], ss[i2], u2, &l1_done));
          if (!l1_done) HMCX_HIP(ctx, mlp_wgrad<T>(pn[i2], ss[i2].q, ss[i2].ms, 2, UPD_SGHMC, u2));
          fwd += 6;
          continue;
        }
        for (int i0 = 0; i0 < 6; i0 += fit) HMCX_HIP(ctx, mlp_forward_batch<T>(net, ss + i0, std::min(fit, 6 - i0)));
        // bias / W3 updates from their partials: b2, W3, b3 (partials of the fused forwards) in the
        // layer-1 backward launch, b1 (whose partials that launch makes) in the W1 gradient launch
        for (int i = 0; i < 6; ++i) {
          const int v = s->order[i];
          if (v == 0 || v == 2) continue;
          set_pending(v == 1 ? pn[0] : net, v, UPD_SGHMC, upd_for(it, v, Xit[v], it + 1 < n ? Xnx[v] : nullptr), &pn[i]);
        }
        HMCX_HIP(ctx, mlp_ga1_w2<T>(net, ga, nga, pn[i2], ss[i2], upd_for(it, 2, Xit[2], it + 1 < n ? Xnx[2] : nullptr)));
        HMCX_HIP(ctx, mlp_wgrad<T>(pn[0], ss[0].q, ss[0].ms, 0, UPD_SGHMC,
                                   upd_for(it, 0, Xit[0], it + 1 < n ? Xnx[0] : nullptr)));
        fwd += 6;
      }
      for (int v = 0; v < 6; ++v) cur[v] = q3[(n - 1) % 3][v];
      // the energies that did not ride along (each names its xw), in one launch (xw holds the last iteration's xw)
      SubStep<T> rest[2];
      int nr = 0;
      for (int e = 0; e < 2; ++e)
        if (!e_done[e]) rest[nr++] = es[e];
      for (int e0 = 0; e0 < nr; e0 += fit) HMCX_HIP(ctx, mlp_forward_batch<T>(net, rest + e0, std::min(fit, nr - e0)));
      fwd += 2;
      net.xw = xwb[0];                                         // the net's own buffer again
    }
    for (int it = 0; it < n && !batch; ++it) {
      for (int i = 0; i < 6; ++i) {
        const int v = s->order[i];
        cur[v] = (it & 1) ? qb[v] : qa[v];                    // drifted position of this iteration
        if (v == 0) net.xw_valid = false;
        const MaskSrc<T> ms = masks_for(fwd++);
        const Upd<T> u = upd_for(it, v, cur[v], it + 1 < n ? ((it & 1) ? qa[v] : qb[v]) : nullptr);
        // h1 from the fused forward for the W1 / b1 / W2 sub-steps (HMCX_MLP_H1=0: recompute it)
        const L3Want w{v <= 3, v == 3, v == 5, v == 4, store_h1 && v <= 2};
        HMCX_HIP(ctx, mlp_forward<T>(net, cur, ms, lp_scr, w));
        if (v <= 1) HMCX_HIP(ctx, mlp_ga1<T>(net, cur, ms, v == 1));
        if (v == 0 || v == 2) HMCX_HIP(ctx, mlp_wgrad<T>(net, cur, ms, v, UPD_SGHMC, u));
        else set_pending(net, v, UPD_SGHMC, u);
      }
    }
    // energies (hmc.py:67-71: E_new first, then E_current), each with fresh masks
    if (!(batch && n > 0)) {
      HMCX_HIP(ctx, mlp_forward<T>(net, cur, masks_for(fwd++), lp_new, L3Want{false, false, false, false}));
      net.xw_valid = false;
      HMCX_HIP(ctx, mlp_forward<T>(net, par, masks_for(fwd++), lp_cur, L3Want{false, false, false, false}));
    }
    HMCX_HIP(ctx, flush_pending(net));
    VarTab ve{};
    for (int i = 0; i < 6; ++i) {
      const int v = s->order[i];
      ve.q[i] = cur[v]; ve.qn[i] = par[v]; ve.p[i] = pv[v]; ve.n[i] = dim[v];
    }
    hipLaunchKernelGGL(k_sumsq12<T>, dim3(NPART, 6), dim3(256), 0, st, ve, part_new);
    MlpAccept ac{};
    ac.part_cur = part_cur; ac.part_new = part_new; ac.lp_cur = lp_cur; ac.lp_new = lp_new;
    ac.nlb_new = e_fr[0] ? net.nrb : net.nlb;
    ac.nlb_cur = e_fr[1] ? net.nrb : net.nlb;
    ac.B = s->B;
    for (int i = 0; i < 6; ++i) ac.dim[i] = dim[s->order[i]];
    ac.alpha = s->alpha; ac.u = s->u_accept[si];
    ac.out_A = s->out_A + si; ac.out_acc = s->out_accepted + si; ac.out_loss = s->out_loss + si;
    ac.out_nlp = s->out_nlp ? s->out_nlp + si : nullptr;
    ac.out_E = s->out_E ? s->out_E + 2 * si : nullptr;
    ac.acc_flag = accf;
    hipLaunchKernelGGL(k_mlp_accept, dim3(1), dim3(26 * 32), 0, st, ac);
    if (n > 0) {                       // commit: in the next step's start launch, or here after the last step
      if (si + 1 < s->n_steps) {
        commit_pending = true;
        for (int v = 0; v < 6; ++v) prev_prop[v] = cur[v];
      } else {
        hipLaunchKernelGGL(k_mlp_commit<T>, dim3(NPART, 6), dim3(256), 0, st, ve, accf);
      }
    }
    HMCX_HIP(ctx, hipGetLastError());
  }
  if ((rc = gs.finish())) return rc;
  if ((rc = timing_end(ctx, ctx->stream))) return rc;
  if (net.fr_prof && net.fr_prof_n) {                        // HMCX_FWDR_PROF=<file>: append per launch
    HMCX_HIP(ctx, hipStreamSynchronize(st));                  // {np, nrb, FR_NPH} + stamps [np][nrb][FR_NPH]
    const size_t per = (size_t)net.nrb * FR_MAXP * FR_NPH;
    std::vector<unsigned long long> h(per * net.fr_prof_n);
    HMCX_HIP(ctx, hipMemcpy(h.data(), net.fr_prof, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    if (FILE* f = fopen(fr_prof_path, "ab")) {
      for (int l = 0; l < net.fr_prof_n; ++l) {
        const int hdr[3] = {net.fr_prof_np[l], net.nrb, FR_NPH};
        fwrite(hdr, sizeof(int), 3, f);
        fwrite(h.data() + l * per, sizeof(unsigned long long), (size_t)net.fr_prof_np[l] * net.nrb * FR_NPH, f);
      }
      fclose(f);
    }
  }
  if (net.prof) {                                            // HMCX_MLP_PROF=<file>: append the stamps
    HMCX_HIP(ctx, hipStreamSynchronize(st));
    const size_t n = (size_t)std::min(net.l23_count, net.prof_cap) * net.nlb * ((net.n_mid + 31) / 32) * L23_NPH;
    std::vector<unsigned long long> h(n);
    HMCX_HIP(ctx, hipMemcpy(h.data(), net.prof, n * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    if (FILE* f = fopen(getenv("HMCX_MLP_PROF"), "ab")) {
      const int hdr[4] = {std::min(net.l23_count, net.prof_cap), net.nlb, (net.n_mid + 31) / 32, L23_NPH};
      fwrite(hdr, sizeof(int), 4, f);
      fwrite(h.data(), sizeof(unsigned long long), n, f);
      fclose(f);
    }
  }
  if (!net.fuse) {
    if (s->out_abort) HMCX_HIP(ctx, hipMemsetAsync(s->out_abort, 0, sizeof(int32_t), st));
    return HMCX_OK;
  }
  // the call's verdict: the MLP abort word (raised by a timed-out exchange of any fused launch of this
  // call) goes to out_abort and is lowered for the next call — the call's outputs and state are then
  // invalid and the caller re-runs it unfused (sghmc._run_mlp); without out_abort, wait and report
  if (s->out_abort) {
    HMCX_HIP(ctx, hipMemcpyAsync(s->out_abort, ctx->mlp_abort_dev, sizeof(int32_t), hipMemcpyDeviceToDevice, st));
    HMCX_HIP(ctx, hipMemsetAsync(ctx->mlp_abort_dev, 0, sizeof(int), st));
    return HMCX_OK;
  }
  int flag = 0;
  HMCX_HIP(ctx, hipMemcpyAsync(&flag, ctx->mlp_abort_dev, sizeof(int), hipMemcpyDeviceToHost, st));
  HMCX_HIP(ctx, hipMemsetAsync(ctx->mlp_abort_dev, 0, sizeof(int), st));
  HMCX_HIP(ctx, hipStreamSynchronize(st));
  if (flag) return set_error(ctx, HMCX_EHIP, "mlp sghmc: fused layer-2/3 exchange timed out; state is invalid "
                                             "(re-run with hmcx_set_mlp_fuse(ctx, 0))");
  return HMCX_OK;
}

// HMCX_MLP_DTYPES (bit 0 float, bit 1 double; both by default): the build compiles this file once per
// dtype (__graft_entry__.UNITS), so the two halves of its template instantiations build in parallel.
#ifndef HMCX_MLP_DTYPES
#define HMCX_MLP_DTYPES 3
#endif
#if HMCX_MLP_DTYPES & 1
template int mlp_masks_t<float>(hmcx_ctx*, int, int, uint64_t, uint32_t, uint32_t, uint32_t, void*);
template int mlp_grad_t<float>(hmcx_ctx*, const void*, const int32_t*, int, int, int, int, const hmcx_mlp_params*,
                               const void*, double, hmcx_mlp_params*, double*);
template int mlp_loss_t<float>(hmcx_ctx*, const void*, const int32_t*, int, int, int, int, const hmcx_mlp_params*,
                               const void*, double*, void*);
template int mlp_sghmc_t<float>(hmcx_ctx*, const hmcx_mlp_sghmc_args*);
template int mlp_leapfrog_t<float>(hmcx_ctx*, const hmcx_mlp_leapfrog_args*);
#endif
#if HMCX_MLP_DTYPES & 2
template int mlp_masks_t<double>(hmcx_ctx*, int, int, uint64_t, uint32_t, uint32_t, uint32_t, void*);
template int mlp_grad_t<double>(hmcx_ctx*, const void*, const int32_t*, int, int, int, int, const hmcx_mlp_params*,
                                const void*, double, hmcx_mlp_params*, double*);
template int mlp_loss_t<double>(hmcx_ctx*, const void*, const int32_t*, int, int, int, int, const hmcx_mlp_params*,
                                const void*, double*, void*);
template int mlp_sghmc_t<double>(hmcx_ctx*, const hmcx_mlp_sghmc_args*);
template int mlp_leapfrog_t<double>(hmcx_ctx*, const hmcx_mlp_leapfrog_args*);
#endif

}  // namespace hmcx
