// hmcx_persist2.hip — single-chain SGHMC for the softmax model as ONE persistent launch per call,
// built around tagged-granule hand-offs (no counters, no fences, no grid barrier per leapfrog).
//
// Mathematics and op order: cpu/sghmc.py:19-39 with the A1 completion, cpu/softmax.py:38-79, as in
// the kernel-per-phase path (hmcx_softmax.hip).  Layout (BASELINE config 2: B=500, D=784, K=10):
//
//  * G = Gr x Gf workgroups (256 threads, one per CU, co-resident).  Workgroup (r, f) keeps the
//    minibatch tile X[R_r, F_f] in LDS for a whole step (rows R_r = Br rows, features F_f = Bf).
//  * Inside the row team r, workgroup f OWNS the row slice rho(r,f) (Ro rows); inside the feature
//    team f, workgroup r OWNS the feature slice phi(r,f) (Fo features x K weights and momenta).
//  * One leapfrog iteration = four team-local hand-off rounds, each a reduce-scatter or an
//    all-gather of a few KB:
//      A-RS  partial logits X[R_r,F_f]·W[F_f]          → owner of rho sums the Gf partials,
//            runs both softmaxes of its rows (at b and at b' = b + ε·pb), builds diff rows;
//      A-AG  diff rows + colsum/ll partials            → every member has diff[R_r];
//      B-RS  partial gradient X[R_r,F_f]ᵀ·diff         → owner of phi sums the Gr partials and
//            updates its weights/momenta (friction noise from Philox); the bias sub-step is
//            replicated from the all-row colsum that travels with the partials;
//      B-AG  drifted weights of phi                    → every member has W[F_f] for the next X·W.
//    Per step one more all-gather (kinetic and log-likelihood partials) decides the MH accept in
//    every workgroup identically.
//  * The two GEMMs run on MFMA (v_mfma_f64_16x16x4 / f32_16x16x4) with operands from the LDS tile;
//    the class dimension (KC = 10 compiled in, 16 generic) pads to the 16-wide tile.  A VALU
//    variant with the classes in registers measured 1.7x slower (LDS-latency bound).
//  * Transport: every value travels as one 16-byte granule {lo32, epoch, hi32, epoch} written by
//    ONE `buffer_store_dwordx4 … sc1` and read by `buffer_load_dwordx4 … sc1`; a consumer re-reads
//    a granule until both epoch words match (cdna_hip_programming.md §6 G16, recipe R2: the data
//    is the flag).  Epochs count rounds within the call; the arena is zeroed before each launch.
//    Measured on MI355X (tools/microbench_handoff.hip): one team round of 8 x 80-130 granules
//    ≈ 1.4-1.6 µs, against 3-3.4 µs for payload + counter barrier.
// All reductions run in a fixed order, so the replicated state is bit-identical in every
// workgroup and runs are deterministic.
#include "hmcx_common.h"
#include "hmcx_internal.h"
#include "hmcx_persist.h"
#include "hmcx_p2x.h"
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace hmcx {


struct Q2Args {
  int B, D, K, P, n_steps;
  int Gr, Gf, Br, Bf, BfP, BFP, Ro, Fo;
  double alpha, neg_inv_n, log_prior;
  const void* X; const void* Y;
  const double* eps; const double* u; const int64_t* row0; const int32_t* n_iter;
  int noise_mode; const double* noise; const int64_t* noff;
  uint64_t seed; uint32_t chain0, step_base;
  void* W; void* b;
  char* arena;                              // granule arena (zeroed per call)
  int oXA, oXD, oXB, oXW, oXS;              // region offsets in granules
  int oXC;                                  // commit round: one granule per workgroup
  int arena_bytes;
  int pad;                                  // line-aligned producer blocks (HMCX_P2_PAD, default on)
  unsigned ep0;                             // first round epoch of this launch (unique in the arena's life)
  int zoff;                                 // noise off the A-RS pollers (HMCX_P2_ZOFF, default on)
  int spread;                               // rounds with spread gathers, bits A-RS, A-AG, B-RS, B-AG
                                            // (HMCX_P2_SPREAD=<mask>; default A-AG, where it measured faster)
  int xmap;                                 // 1: logical id (b % 8)·(G/8) + b/8 — row teams on one XCD
  int fl2;                                  // feature teams share an XCD: B-round stores plain (kept in L2)
  int al2;                                  // row teams share an XCD (xmap): A-round stores plain
  int prefetch;                             // 1: next step's tile/labels loaded during the accept round
  int acc1;                                 // 1: accept partials polled in one batch (HMCX_P2_ACC1)
  int bar;                                  // 1: round B is an all-reduce by redundant reads (every feature-
                                            // team member sums all Gr partials of the WHOLE slice and updates
                                            // it identically) — no B-AG round (HMCX_P2_BAR, default on)
  int* abort_flag;                          // the context's sticky abort word (hmcx_clear_abort)
  int force_abort;                          // HMCX_P2_FORCE_ABORT=<step>: the last workgroup raises the
                                            // abort word at that step (tests the recovery path); −1 off
  double* out_A; int32_t* out_acc; double* out_ll; double* out_E;
  void* out_trace;                          // [n_steps][P] state after every step, or null
  void* out_mom;                            // [P] momentum returned by the last step, or null
  unsigned long long* prof;                 // HMCX_PERSIST_PROF=1: per-segment s_memtime totals (workgroup 0)
  unsigned long long* trace;                // HMCX_P2_TRACE=1: [G][P2TR_IT][8] s_memrealtime stamps (step 0)
  int* verdict;                             // this launch's abort verdict (hmcx_sampler_args::out_abort), or
                                            // null: 0 stored by workgroup 0 on completion, 1 by every
                                            // workgroup that leaves early (no device-to-device copy)
  int ninl;                                 // > 0: the schedule of the call's ninl steps rides in inl (no
                                            // host-to-device upload); 0: eps / u / row0 / n_iter above
  struct { double eps, u; int64_t row0; int32_t n_iter, pad_; } inl[32];
};
constexpr int P2_NINL = 32;                 // calls of up to this many steps pass their schedule inline
// One schedule value of step s: the kernel-argument copy (inline calls) and the global array are both
// loaded and the value selected.  A conditional `inl ? a.inl[s].x : a.x[s]` became one load through a
// pointer that may be the kernarg segment or global memory — a flat load, which every later
// `s_waitcnt lgkmcnt` (LDS traffic) then also waited for.  Inline calls point the arrays at zeros.
__device__ inline int sched_k(int s) { return s < P2_NINL ? s : P2_NINL - 1; }
template <typename V>
__device__ inline V sched_at(bool inl, int s, V kv, const V* g) {
  const V gv = g[inl ? 0 : s];
  return inl ? kv : gv;
}

// Writes the launch's abort verdict when a workgroup leaves the kernel without committing (a timed-out
// hand-off, a sticky abort word, or a decided abort): 1.  The host zeroes the verdict before the launch
// and nothing stores 0, so the verdict is sticky — an abort is never overwritten (the commit decision
// makes "no workgroup stored 1" and "every workgroup committed" the same event).
struct P2Verdict {
  int* out;
  bool done;
  __device__ ~P2Verdict() {
    if (out && !done) out[0] = 1;
  }
};
constexpr int P2TR_IT = 16;                 // traced leapfrog iterations

// Segment profiler (workgroup 0, thread 0): s_memtime deltas accumulate in LDS (a global
// read-modify-write per stamp would add a memory round trip to the critical path); flushed once.
struct P2Prof {
  unsigned long long* out;
  unsigned long long* acc;   // LDS [16]
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


// Noise value of flat element e for slot `slot` of step s: Philox block z4 (already generated for
// block e >> 2) or the host-drawn buffer (cpu/sghmc.py:21,31 draw order).
template <typename T>
__device__ inline T noise_at(const Q2Args& a, int s, uint32_t slot, uint32_t e, const T* z4) {
  if (a.noise_mode == HMCX_NOISE_BUFFER) return (T)a.noise[a.noff[s] + (int64_t)slot * a.P + e];
  return z4[e & 3];
}
template <typename T>
__device__ inline void philox4_if(const Q2Args& a, int s, uint32_t slot, uint32_t g, T z[4]) {
  if (a.noise_mode != HMCX_NOISE_BUFFER) philox_normal4(opaque_s64(a.seed), a.chain0, a.step_base + (uint32_t)s, slot, g, z);
}
// One element's noise (f32 chains: float Box–Muller; f64 chains: the double one, hmcx_common.h).
template <typename T>
__device__ inline T noise1(const Q2Args& a, int s, uint32_t slot, uint32_t e) {
  if (a.noise_mode == HMCX_NOISE_BUFFER) return (T)a.noise[a.noff[s] + (int64_t)slot * a.P + e];
  return philox_normal_t<T>(opaque_s64(a.seed), a.chain0, a.step_base + (uint32_t)s, slot, e);
}

// Minibatch tile X[row0:+nrow, feat0:+nfeat] → LDS [Br][BFP], zero padded to BfP columns;
// 16-byte loads, 8 in flight per thread when rows are 16-byte aligned.
template <typename T>
__device__ inline void load_tile(T* Xs, const T* Xg, int Br, int BfP, int BFP, int nrow, int nfeat, int row0,
                                 int feat0, int D) {
  constexpr int V = 16 / sizeof(T);
  typedef T vec_t __attribute__((ext_vector_type(V)));
  const int PR = BfP / V;                        // vectors per tile row
  const float inv = 1.0f / (float)PR;
  const int total = Br * PR;
  const bool vec_ok = (D % V) == 0 && (feat0 % V) == 0 &&
                      ((reinterpret_cast<uintptr_t>(Xg) & 15) == 0);
  for (int base = threadIdx.x; base < total; base += 8 * QTH) {
    vec_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = base + u * QTH;
      const int i = qdiv(e, inv), j = (e - i * PR) * V;
      const T* src = Xg + (size_t)(row0 + i) * D + feat0 + j;
      if (e < total && i < nrow && j + V <= nfeat && vec_ok) {
        v[u] = *reinterpret_cast<const vec_t*>(src);
      } else {
#pragma unroll
        for (int q = 0; q < V; ++q) v[u][q] = (e < total && i < nrow && j + q < nfeat) ? src[q] : T(0);
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = base + u * QTH;
      if (e < total) {
        const int i = qdiv(e, inv), j = (e - i * PR) * V;
#pragma unroll
        for (int q = 0; q < V; ++q) Xs[i * BFP + j + q] = v[u][q];
      }
    }
  }
}

// One step's minibatch rows: the X tile of this workgroup and the labels of its softmax rows
// (label loads issued first so they travel with the tile's).
template <typename T>
__device__ inline void load_step_rows(T* Xs, T* Yo, const T* Xg, const T* Yg, int Br, int BfP, int BFP, int nrow,
                                      int nfeat, int row0, int feat0, int D, int K, int Ro, int nro, int ro0) {
  const int tid = threadIdx.x;
  T y = T(0);
  if (tid < Ro * 16) {                       // Ro·16 ≤ QTH (plan_p2: Ro·KC + KC + 1 ≤ QTH, KC ≥ 10)
    const int ii = tid >> 4, k = tid & 15;
    if (ii < nro && k < K) y = Yg[(size_t)(row0 + ro0 + ii) * K + k];
  }
  for (int e = tid + QTH; e < Ro * 16; e += QTH) {
    const int ii = e >> 4, k = e & 15;
    Yo[e] = (ii < nro && k < K) ? Yg[(size_t)(row0 + ro0 + ii) * K + k] : T(0);
  }
  load_tile<T>(Xs, Xg, Br, BfP, BFP, nrow, nfeat, row0, feat0, D);
  if (tid < Ro * 16) Yo[tid] = y;
}

// C[16 x 16] += A[16 x 4·nk] · B[4·nk x 16] on one wave (v_mfma_*_16x16x4).  Lane group lg of k-step kk
// holds A(i, ·) = a[i·as_i + lg·a_lg + kk·a_kk] and B(·, j) = b[lg·b_lg + kk·b_kk + j]: (a_lg, a_kk) =
// (as_k, 4·as_k) walks k in order, (a_lg, a_kk) = (nk·as_k, as_k) lets the four lane groups of one
// k-step read k values nk apart (the same 4·nk terms, summed in another grouping).  Operands of 8
// k-steps are loaded before their MFMAs, two accumulators alternate.  Returns the D fragment (rows
// M::row(lane, q), column lane & 15).
template <typename T>
__device__ inline typename mfma16<T>::acc_t mfma_tile(const T* a, int as_i, int a_lg, int a_kk, const T* b, int b_lg,
                                                      int b_kk, int nk) {
  using M = mfma16<T>;
  const int lane = threadIdx.x & 63, lr = lane & 15, lg = lane >> 4;
  const T* pa = a + lr * as_i + lg * a_lg;
  const T* pb = b + lg * b_lg + lr;
  typename M::acc_t c0 = M::zero(), c1 = M::zero();
  int kk = 0;
  for (; kk + 8 <= nk; kk += 8) {
    T av[8], bv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      av[u] = pa[(kk + u) * a_kk];
      bv[u] = pb[(kk + u) * b_kk];
    }
#pragma unroll
    for (int u = 0; u < 8; u += 2) {
      c0 = M::fma(av[u], bv[u], c0);
      c1 = M::fma(av[u + 1], bv[u + 1], c1);
    }
  }
  // tail: the two accumulators still alternate (two dependent MFMA chains, not one)
  for (; kk + 2 <= nk; kk += 2) {
    c0 = M::fma(pa[kk * a_kk], pb[kk * b_kk], c0);
    c1 = M::fma(pa[(kk + 1) * a_kk], pb[(kk + 1) * b_kk], c1);
  }
  if (kk < nk) c0 = M::fma(pa[kk * a_kk], pb[kk * b_kk], c0);
  return c0 + c1;
}

template <typename T, int KC, int SPEC = 0>
__global__ __launch_bounds__(QTH) void k_sghmc_p2(Q2Args a) {
  using M = mfma16<T>;
  // SPEC = 1: the plan of BASELINE config 2 (f64, B=500, D=784, K=10: 8 x 16 teams, 64-row x 49-feature
  // tiles) with every knob at its default, folded into constants — fewer live scalars (the generic
  // kernel spills SGPRs into VGPR lanes) and no runtime branches on the knobs
  constexpr bool SP = SPEC != 0;
  const int spread = SP ? 2 : a.spread, pad = SP ? 1 : a.pad, xmap = SP ? 0 : a.xmap, fl2 = SP ? 1 : a.fl2,
            al2 = SP ? 0 : a.al2, prefetch = SP ? 1 : a.prefetch, acc1 = SP ? 1 : a.acc1,
            zoffa = SP ? 1 : a.zoff, bara = SP ? 1 : a.bar;
  extern __shared__ __align__(16) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15;
  const int Gr = SP ? 8 : a.Gr, Gf = SP ? 16 : a.Gf, G = Gr * Gf;
  // workgroups are dealt to the 8 XCDs round-robin by blockIdx: with the identity map feature team
  // f (blocks f, f+Gf, …) shares an XCD when Gf % 8 == 0; xmap = 1 puts each row team on one XCD
  const int pbid = blockIdx.x;
  const int bid = xmap ? (pbid & 7) * (G >> 3) + (pbid >> 3) : pbid;
  const int r = bid / Gf, f = bid - (bid / Gf) * Gf;
  const int Br = SP ? 64 : a.Br, Bf = SP ? 49 : a.Bf, BfP = SP ? 64 : a.BfP, BFP = SP ? 65 : a.BFP, Ro = SP ? 4 : a.Ro,
            Fo = SP ? 7 : a.Fo;
  const int K = SP ? 10 : a.K, D = SP ? 784 : a.D, B = SP ? 500 : a.B;
  const int row0 = r * Br, feat0 = f * Bf;
  const int nrow = max(0, min(Br, B - row0));
  const int nfeat = max(0, min(Bf, D - feat0));
  const int ro0 = f * Ro, nro = max(0, min(Ro, nrow - ro0));            // my softmax rows
  const int fo0 = r * Fo, nfo = max(0, min(Fo, nfeat - fo0));           // my owned features
  const T hi = (T)CLIP_HI, lo = (T)CLIP_LO;
  const T alpha = (T)a.alpha;
  const __amdgpu_buffer_rsrc_t rs = arena_rsrc(a.arena, a.arena_bytes);
  // MFMA work split: phase A m-tiles = Br/16 rows (k over BfP features), phase B m-tiles = BfP/16
  // features (k over Br rows); split-K parts when the tiles are fewer than the waves
  const int MTA = Br / 16, WPA = max(1, QNW / MTA);
  const int MTB = BfP / 16, WPB = max(1, QNW / MTB);
  const int HA = KC + 1;                              // payload header: colsum[KC], ll
  // payload blocks per producer, rounded to whole 128-byte lines (8 granules) when pad is set
  const int NXA0 = HA + Ro * KC;                      // A-AG payload per producer
  const int NXA = p2_pad(NXA0, pad);                // ... and its block stride
  const int NXB = p2_pad(HA + Bf * KC, pad);        // B-RS payload per producer
  const int NXS = pad ? 8 : 4;                      // accept partials per workgroup

  // ---- LDS carve-up (mirrored by p2_lds)
  T* Xs = reinterpret_cast<T*>(smem);                 // [Br][BFP]
  T* Wf = Xs + (size_t)Br * BFP;                      // [BfP][16] weights of F_f
  T* Wf0 = Wf + BfP * 16;                             // [BfP][16] step-start copy
  T* Ds = Wf0 + BfP * 16;                             // [Gf·Ro][16] diff of the row tile
  T* Zp = Ds + Gf * Ro * 16;                          // split-K partials: [WPA][Br][16] | [WPB][BfP][16]
  const int ZPN = max(WPA * Br, WPB * BfP) * 16;
  T* Zo = Zp + ZPN;                                   // [Ro][16] logits of my rows
  T* Yo = Zo + Ro * 16;                               // [Ro][16] labels of my rows
  T* Dme = Yo + Ro * 16;                              // [Ro][16] diff of my rows
  T* Csr = Dme + Ro * 16;                             // [Ro][16] y − ŷ' of my rows
  T* bsh = Csr + Ro * 16;                             // [16] b
  T* pbsh = bsh + 16;                                 // [16] pb
  T* b0sh = pbsh + 16;                                // [16] b at step start
  T* bpsh = b0sh + 16;                                // [16] b'
  T* pb0sh = bpsh + 16;                               // [16] pb drawn at step start
  size_t off = ((size_t)(reinterpret_cast<char*>(pb0sh + 16) - smem) + 15) & ~(size_t)15;
  double* rowll = reinterpret_cast<double*>(smem + off);  // [Ro] ll of my rows
  double* hdr = rowll + Ro;                               // [16] all-row colsum, ll
  double* dsh = hdr + 16;                                 // [16] reductions
  int* ish = reinterpret_cast<int*>(dsh + 16);            // [4] flags
  unsigned long long* profacc = reinterpret_cast<unsigned long long*>(ish + 4);   // [16]
  double* stg = reinterpret_cast<double*>(profacc + 16);                             // [QSTAGE] spread gathers
  T* zbuf = reinterpret_cast<T*>(stg + QSTAGE);                                      // [Fo·KC + 16] noise
  T* pWs = zbuf + Fo * 16 + 16;                       // [BfP][16] momentum of the whole slice (bar)
  // friction noise by the waves that do not poll A-RS (threads from NZ0 on), when they fit.  NZ0 comes
  // from the plan's Ro, not this member's nro: zoff decides `bar`, the protocol of round B, which every
  // workgroup must agree on — with a per-member nro, a member owning no rows (B = 40, D = 32: plan 2x2,
  // rows 32-39 in row team 1) chose the all-reduce while its team ran RS + AG, and the launch waited out
  // its 4 s timeout before the recovery re-ran it
  const int NZ0 = ((Ro * KC + 63) / 64) * 64;
  const bool zoff = zoffa && !(spread & 1) && NZ0 + Fo * KC + K <= QTH;
  // B all-reduce (bara) needs the owners' noise in LDS (zoff) to fold it into their partials
  const bool bar = bara && zoff;
  const auto all_items = [](int, int) { return true; };

  // owned weight of this thread: feature fo0 + od, class ok (thread t = od·KC + ok)
  const int od = tid / KC, okc = tid - (tid / KC) * KC;
  const bool own = od < nfo && okc < K;
  const int e_own = (feat0 + fo0 + od) * K + okc;     // flat index (W is [D][K])
  const int wl = (fo0 + od) * 16 + okc;               // index in Wf
  T pw = T(0), wv = T(0), w0 = T(0), zn = T(0);

  P2Verdict verdict{threadIdx.x == 0 ? a.verdict : nullptr, false};
  const bool inl = a.ninl > 0;
  // a launch behind a timed-out one (sticky abort word) leaves everything untouched
  if (__hip_atomic_load(a.abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  if (tid == 0) ish[0] = 0;
  if (tid < 16) profacc[tid] = 0ull;
  for (int e = tid; e < BfP * 16; e += QTH) {
    const int i = e >> 4, k = e & 15;
    Wf[e] = (i < nfeat && k < K) ? reinterpret_cast<const T*>(a.W)[(size_t)(feat0 + i) * K + k] : T(0);
  }
  for (int e = tid; e < Gf * Ro * 16; e += QTH) Ds[e] = T(0);
  for (int e = tid; e < Ro * 16; e += QTH) { Dme[e] = T(0); Csr[e] = T(0); }
  if (tid < 16) bsh[tid] = tid < K ? reinterpret_cast<const T*>(a.b)[tid] : T(0);
  __syncthreads();
  if (own) wv = Wf[wl];

  // segment profiler: compiled out of the config-2 instantiation (SPEC = 1); SPEC = 3 is that
  // instantiation with it (HMCX_PERSIST_PROF=1 at the config-2 shape)
  P2Prof prof{((!SP || SPEC == 3) && bid == 0 && tid == 0) ? a.prof : nullptr, profacc, 0ull, 0};
  // round trace: slot 2·round = payload published, 2·round + 1 = consumed (rounds A, D, B, W)
  unsigned long long* trb = (!SP && a.trace) ? a.trace + (size_t)bid * P2TR_IT * 8 : nullptr;
  auto tstamp = [&](int s_, int it_, int slot) {
    if (trb && tid == 0 && s_ == 0 && it_ >= 0 && it_ < P2TR_IT) trb[it_ * 8 + slot] = __builtin_amdgcn_s_memrealtime();
  };
  unsigned ep = a.ep0 - 1;                            // round epoch (same sequence in every workgroup)
  unsigned uA = 0, uD = 0, uB = 0, uW = 0, uS = 0;    // per-region use counters (buffer parity)

  // ---- phase A: partial logits X[R_r,F_f]·W[F_f] → XA(par, r, f) [nrow][KC], then A-RS consume:
  //      Zo[ii][k] = Σ_f' partials of my rows (f' order)
  // Two A rounds may be in flight (the step-start round of E_current and iteration 0's): each is
  // published into region parity `par` with its own epoch (epA[par]), and consumed from the same.
  unsigned epA[2] = {0u, 0u};
  auto roundA = [&](int par) -> bool {
    const int tid = opaque((int)threadIdx.x), lane = tid & 63, wave = tid >> 6, lr = lane & 15;   // not hoisted (registers)
    epA[par] = ++ep;
    const int reg = a.oXA + ((par * Gr + r) * Gf + f) * Br * KC;
    // zero-padded tail skipped; config 2: 49 features in every feature team → 13 k-steps (a constant:
    // the k loop unrolls completely)
    const int nkp = SP ? 13 : WPA == 1 ? (nfeat + 3) / 4 : (BfP / 4) / WPA;
    for (int item = wave; item < MTA * WPA; item += QNW) {
      const int mt = item % MTA, part = item / MTA;
      const typename M::acc_t c = mfma_tile<T>(Xs + mt * 16 * BFP + part * nkp * 4, BFP, 1, 4,
                                               Wf + part * nkp * 4 * 16, 16, 64, nkp);
      if (WPA == 1) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = mt * 16 + M::row(lane, q);
          if (row < nrow && lr < KC) put_t(al2, rs, reg + row * KC + lr, (double)c[q], epA[par]);
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) Zp[(part * Br + mt * 16 + M::row(lane, q)) * 16 + lr] = c[q];
      }
    }
    if (WPA > 1) {
      __syncthreads();
      for (int e = tid; e < nrow * KC; e += QTH) {
        const int i = e / KC, k = e - (e / KC) * KC;
        T v = Zp[i * 16 + k];
        for (int p = 1; p < WPA; ++p) v += Zp[(p * Br + i) * 16 + k];
        put_t(al2, rs, reg + e, (double)v, epA[par]);
      }
    }
    return true;
  };
  auto consumeA = [&](int par) -> bool {
    const int tid = opaque((int)threadIdx.x), lane = tid & 63, wave = tid >> 6, lr = lane & 15;   // not hoisted (registers)
    const int base0 = a.oXA + (par * Gr + r) * Gf * Br * KC;
    const unsigned ep = epA[par];
    ++uA;
    if (spread & 1) {
      const int ni = nro * KC;
      const bool ok = gather(rs, base0, Br * KC, Gf, ni, [&](int i) { return ro0 * KC + i; }, all_items, ep,
                             a.abort_flag, stg);
      if (!all_ok(ok, ish)) return false;
      if (tid < ni) {
        double z = stg[tid];
        for (int p = 1; p < Gf; ++p) z += stg[p * ni + tid];
        Zo[(tid / KC) * 16 + (tid % KC)] = (T)z;
      }
      __syncthreads();
      return true;
    }
    double z = 0.0;
    const bool ok = poll<true>(rs, base0, Br * KC, Gf, -1, ro0 * KC + tid, tid < nro * KC, ep, nullptr, 0, &z,
                               a.abort_flag);
    if (tid < nro * KC) Zo[(tid / KC) * 16 + (tid % KC)] = (T)z;
    return all_ok(ok, ish);
  };

  for (int s = 0; s < a.n_steps; ++s) {
    const int tid = opaque((int)threadIdx.x), lane = tid & 63, wave = tid >> 6, lr = lane & 15;   // not hoisted (registers)
    const double epsd = sched_at(inl, s, a.inl[sched_k(s)].eps, a.eps);
    const T eps = (T)epsd, ome = (T)(1.0 - epsd), nsc = (T)(2.0 * epsd);
    const int n = sched_at(inl, s, a.inl[sched_k(s)].n_iter, a.n_iter);
    const int64_t rw = sched_at(inl, s, a.inl[sched_k(s)].row0, a.row0);
    const T* Xg = reinterpret_cast<const T*>(a.X) + (size_t)rw * D;
    const T* Yg = reinterpret_cast<const T*>(a.Y) + (size_t)rw * K;
    prof.stamp(0);
    if (s == a.force_abort && bid == G - 1) {                             // test knob: a "timed-out" member
      if (tid == 0) __hip_atomic_store(a.abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }

    // ---- step start: tile, labels of my rows (step 0 only: later steps' were loaded while the
    //      previous accept round travelled), momentum (hmc.py:82-87), step-start copies
    if (s == 0 || !prefetch) load_step_rows<T>(Xs, Yo, Xg, Yg, Br, BfP, BFP, nrow, nfeat, row0, feat0, D, K, Ro, nro, ro0);
    for (int e = tid; e < BfP * 16; e += QTH) Wf0[e] = Wf[e];
    // momentum (hmc.py:82-87): the owned elements' by their threads, the bias's by the last 16 threads
    // (not the owners of elements 0..15: one Box–Muller latency per thread, not two)
    pw = own ? noise1<T>(a, s, 0u, (uint32_t)e_own) : T(0);
    const T pw0 = pw;
    w0 = wv;
    if (tid >= QTH - 16) {
      const int k = tid - (QTH - 16);
      pbsh[k] = k < K ? noise1<T>(a, s, 0u, (uint32_t)(D * K + k)) : T(0);
      pb0sh[k] = pbsh[k];
      b0sh[k] = bsh[k];
    }
    const double kin0 = wsum((double)pw * (double)pw, dsh);
    double kb0 = 0.0;
    for (int k = 0; k < K; ++k) kb0 += (double)pbsh[k] * (double)pbsh[k];

    // ---- it = -1: log-likelihood of my rows at the step-start state (E_current).  (Round 5 measured
    //      issuing iteration 0's A round before consuming this one, both rounds in flight: 1.724 vs
    //      1.701 ms per driver-shape launch, 3 A/B pairs — slower, not kept.)
    double ll0 = 0.0, ll_last = 0.0;
    prof.stamp(11);
    const int parm1 = (int)(uA & 1);
    roundA(parm1);
    if (n > 0) {
      // iteration 0's drift of the whole F_f slice by p0 (every member computes it identically;
      // sghmc.py:32), by the waves that do not poll this A-RS round, while the partials travel —
      // after a barrier: every wave's A-gemm has read Wf
      __syncthreads();
      const int nzp = (spread & 1) ? 0 : ((nro * KC + 63) / 64) * 64;   // the polling threads
      const int ge0 = (feat0 * K) >> 2, ge1 = ((feat0 + nfeat) * K + 3) >> 2;
      for (int g = ge0 + tid - nzp; tid >= nzp && g < ge1; g += QTH - nzp) {
        T z4[4];
        philox4_if(a, s, 0u, (uint32_t)g, z4);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int e = 4 * g + q;
          if (e < feat0 * K || e >= (feat0 + nfeat) * K) continue;
          const int i = e / K - feat0, k = e - (e / K) * K;
          const T p0 = noise_at<T>(a, s, 0u, (uint32_t)e, z4);
          Wf[i * 16 + k] = Wf[i * 16 + k] + eps * p0;
          if (bar) pWs[i * 16 + k] = p0;
        }
      }
    }
    if (!consumeA(parm1)) return;
    {
      const int k = lane & 15, grp = tid >> 4;
      const bool kv = k < K;
      for (int ii = grp; ii < nro; ii += QTH / 16) {
        const T z = kv ? clipz(Zo[ii * 16 + k] + b0sh[k], hi, lo) : (T)-__builtin_inf();
        const T m = g16_max2(z);
        const T e = kv ? exp(z - m) : T(0);
        const T sm = g16_sum2(e);
        const T lse = log(sm) + m;                                          // softmax.py:18
        const double t = kv ? (double)(Yo[ii * 16 + k] * (z - lse)) : 0.0;  // softmax.py:19-20
        const double rsum = g16_sum2(t);
        if (k == 0) rowll[ii] = rsum;
      }
      __syncthreads();
      if (tid == 0) {
        double v = 0.0;
        for (int ii = 0; ii < nro; ++ii) v += rowll[ii];
        dsh[4] = v;
      }
      __syncthreads();
      ll0 = dsh[4];
    }

    double kin1 = 0.0;
    T zb_prev = T(0);                                   // bias friction noise of the previous iteration
    for (int it = 0; it < n; ++it) {
      const int tid = opaque((int)threadIdx.x), lane = tid & 63, wave = tid >> 6, lr = lane & 15;   // not hoisted (registers)
      const bool last = it == n - 1;
      if (it == 0 && own) wv = wv + eps * pw;          // the slice drifted during the it = -1 round

      // ===== A-RS: partial logits → owners of the row slices
      prof.stamp(1);
      const int parA = (int)(uA & 1);
      roundA(parA);
      tstamp(s, it, 0);
      // B-AR: the previous iteration's bias sub-step runs here, after this workgroup's A partials went
      // out (it only has to be done before the softmax), then b' of this iteration
      if (bar && it > 0 && tid < K) {
        const T gr = -((T)hdr[tid] - alpha * bpsh[tid]);
        pbsh[tid] = (ome * pbsh[tid] + eps * gr) + nsc * zb_prev;
        bsh[tid] = bpsh[tid];
      }
      if (tid < 16) bpsh[tid] = bsh[tid] + eps * pbsh[tid];                // b' (bias sub-step)
      prof.stamp(2);
      // friction noise of this iteration (sghmc.py:31), generated while the partials travel
      T zb = T(0);
      if (zoff) {
        // by the waves that do not poll the A-RS round, into LDS; the owners pick it up below
        const int zi = tid - NZ0;
        if (zi >= 0 && zi < nfo * KC + K) {
          bool v = true;
          uint32_t e;
          if (zi < nfo * KC) {
            const int od_ = zi / KC, ok_ = zi - (zi / KC) * KC;
            v = ok_ < K;
            e = (uint32_t)((feat0 + fo0 + od_) * K + ok_);
          } else {
            e = (uint32_t)(D * K + zi - nfo * KC);
          }
          zbuf[zi] = v ? noise1<T>(a, s, (uint32_t)(it + 1), e) : T(0);
        }
      } else {
        zn = own ? noise1<T>(a, s, (uint32_t)(it + 1), (uint32_t)e_own) : T(0);
        if (tid < K) zb = noise1<T>(a, s, (uint32_t)(it + 1), (uint32_t)(D * K + tid));
      }
      prof.stamp(3);
      if (!consumeA(parA)) return;
      if (zoff) {                                       // consumeA ended in a barrier
        zn = own ? zbuf[tid] : T(0);
        zb = tid < K ? zbuf[nfo * KC + tid] : T(0);
      }
      tstamp(s, it, 1);
      prof.stamp(4);

      // ===== softmaxes of my rows: diff at b (weights sub-step), y − ŷ' at b' (bias sub-step)
      {
        const int k = lane & 15, grp = tid >> 4;
        const bool kv = k < K;
        for (int item = grp; item < 2 * nro; item += QTH / 16) {
          const bool v1 = item >= nro;
          const int ii = v1 ? item - nro : item;
          const T bias = kv ? (v1 ? bpsh[k] : bsh[k]) : T(0);
          const T y = Yo[ii * 16 + k];
          const T z = kv ? clipz(Zo[ii * 16 + k] + bias, hi, lo) : (T)-__builtin_inf();   // softmax.py:39-41
          const T m = g16_max2(z);
          const T e = kv ? exp(z - m) : T(0);                                                // softmax.py:34
          const T sm = g16_sum2(e);
          const T dd = kv ? y - e / sm : T(0);                                                // softmax.py:52
          if (!v1) {
            Dme[ii * 16 + k] = dd;
          } else {
            Csr[ii * 16 + k] = dd;
            if (last) {
              const T lse = log(sm) + m;
              const double t = kv ? (double)(y * (z - lse)) : 0.0;
              const double rsum = g16_sum2(t);
              if (k == 0) rowll[ii] = rsum;
            }
          }
        }
        __syncthreads();
      }
      // ===== A-AG: [colsum part (KC), ll part, diff rows (Ro·KC)] → every row-team member
      prof.stamp(5);
      double hv = 0.0;                                  // t < KC: team colsum; t == KC: team ll
      {
        ++ep;
        const int reg = a.oXD + (((int)(uD & 1) * Gr + r) * Gf + f) * NXA;
        for (int t = tid; t < NXA0; t += QTH) {
          double v;
          if (t < KC) {
            T c = T(0);
            for (int ii = 0; ii < nro; ++ii) c += Csr[ii * 16 + t];
            v = (double)c;
          } else if (t == KC) {
            v = 0.0;
            if (last) for (int ii = 0; ii < nro; ++ii) v += rowll[ii];
          } else {
            const int m = t - HA;
            v = (double)Dme[(m / KC) * 16 + (m % KC)];
          }
          put_t(al2, rs, reg + t, v, ep);
        }
        tstamp(s, it, 2);
        const int base0 = a.oXD + ((int)(uD & 1) * Gr + r) * Gf * NXA;
        ++uD;
        bool ok;
        if (spread & 2) {
          // diff rows straight into Ds, headers into stg (no staging copy, no second barrier)
          ok = gather_st(rs, base0, NXA, Gf, NXA0, [](int i) { return i; }, ep, a.abort_flag, [&](int q, double v) {
            const int p = q / NXA0, t = q - p * NXA0;
            if (t < HA) stg[q] = v;
            else Ds[(p * Ro + (t - HA) / KC) * 16 + (t - HA) % KC] = (T)v;
          });
          if (!all_ok(ok, ish)) return;
          if (tid < HA) {                           // producer order; the loads issued together
            double hvs[QNPM];
#pragma unroll
            for (int p = 0; p < QNPM; ++p) hvs[p] = stg[min(p, Gf - 1) * NXA0 + tid];
            hv = hvs[0];
#pragma unroll
            for (int p = 1; p < QNPM; ++p)
              if (p < Gf) hv += hvs[p];
          }
        } else if (tid < HA) {
          ok = poll<true>(rs, base0, NXA, Gf, -1, tid, true, ep, nullptr, 0, &hv, a.abort_flag);
        } else {
          const int m = tid - HA;
          ok = poll<false>(rs, base0, NXA, Gf, -1, tid, tid < NXA0, ep, nullptr, 0, nullptr, a.abort_flag,
                           Ds + (m / KC) * 16 + (m % KC), Ro * 16);
        }
        if (!(spread & 2) && !all_ok(ok, ish)) return;
        tstamp(s, it, 3);
      }

      // ===== B-RS: partial gradient X[R_r,F_f]ᵀ·diff → owners of the feature slices
      prof.stamp(6);
      {
        ++ep;
        const int reg = a.oXB + (((int)(uB & 1) * Gf + f) * Gr + r) * NXB;
        if (tid < HA) put_t(fl2, rs, reg + tid, hv, ep);
        // bar: the owner of an element folds its friction noise into its partial — Σ partials − 2z, so
        // ε·(−(Σ − 2z − αw)) = ε·g + 2ε·z (sghmc.py:31,34) arrives with the all-reduce and no other
        // member has to draw that noise
        const auto bpart = [&](int d, int k, double v) -> double {
          return (bar && d >= fo0 && d < fo0 + nfo && k < K) ? v - 2.0 * (double)zbuf[(d - fo0) * KC + k] : v;
        };
        const int nkp = (Br / 4) / WPB;
        for (int item = wave; item < MTB * WPB; item += QNW) {
          const int mt = item % MTB, part = item / MTB;
          const typename M::acc_t c = mfma_tile<T>(Xs + part * nkp * 4 * BFP + mt * 16, 1, nkp * BFP, BFP,
                                                   Ds + part * nkp * 4 * 16, nkp * 16, 16, nkp);
          if (WPB == 1) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int d = mt * 16 + M::row(lane, q);
              if (d < nfeat && lr < KC) put_t(fl2, rs, reg + HA + d * KC + lr, bpart(d, lr, (double)c[q]), ep);
            }
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) Zp[(part * BfP + mt * 16 + M::row(lane, q)) * 16 + lr] = c[q];
          }
        }
        if (WPB > 1) {
          __syncthreads();
          for (int e = tid; e < nfeat * KC; e += QTH) {
            const int i = e / KC, k = e - (e / KC) * KC;
            T v = Zp[i * 16 + k];
            for (int q = 1; q < WPB; ++q) v += Zp[(q * BfP + i) * 16 + k];
            put_t(fl2, rs, reg + HA + e, bpart(i, k, (double)v), ep);
          }
        }
        const int base0 = a.oXB + ((int)(uB & 1) * Gf + f) * Gr * NXB;
        ++uB;
        tstamp(s, it, 4);
        prof.stamp(7);
        if (bar) {
          // all-reduce by redundant reads: items [0, HA) header, [HA, HA + nfeat·KC) the slice's gradient
          // (noise folded in by the owners); every member sums the Gr partials of every item in producer
          // order and applies the same update to the whole slice (momentum pWs, position Wf), so no B-AG
          // round is needed
          const int ni = HA + nfeat * KC;
          bool ok = true;
          double kl = 0.0;
          for (int i0 = tid; i0 < ni; i0 += 2 * QTH) {
            int off[2] = {i0, i0 + QTH};
            const unsigned vm = 1u | (off[1] < ni ? 2u : 0u);
            double sm[2];
            ok = polln<2>(rs, base0, NXB, Gr, off, vm, ep, sm, a.abort_flag, []() {});
            if (!ok) break;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const int i = off[j];
              if (i >= ni) continue;
              if (i < HA) { hdr[i] = sm[j]; continue; }
              const int m = i - HA, d = m / KC, k = m - (m / KC) * KC;
              if (k >= K) continue;
              const int l = d * 16 + k;
              const T w = Wf[l];
              const T gz = -((T)sm[j] - alpha * w);                   // softmax.py:57-58 gradient + 2z
              const T p = ome * pWs[l] + eps * gz;                     // sghmc.py:31,34
              pWs[l] = p;
              if (!last) Wf[l] = w + eps * p;                          // sghmc.py:32
              else if (d >= fo0 && d < fo0 + nfo) kl += (double)p * (double)p;
            }
          }
          if (!all_ok(ok, ish)) return;
          tstamp(s, it, 5);
          prof.stamp(8);
          if (last) {
            if (tid < K) {                                                    // bias sub-step, replicated
              const T gr = -((T)hdr[tid] - alpha * bpsh[tid]);
              pbsh[tid] = (ome * pbsh[tid] + eps * gr) + nsc * zb;
              bsh[tid] = bpsh[tid];
            }
            ll_last = hdr[KC];                                                // ll(q_new) on this batch
            kin1 = kl;
            break;
          }
          zb_prev = zb;                               // its bias sub-step: after the next A publish
          continue;
        }
        // threads [0, nfo·KC): owned gradient element; threads [nfo·KC, nfo·KC + HA): header
        const int ng = nfo * KC;
        double sum = 0.0;
        const bool isg = tid < ng, ish_ = tid >= ng && tid < ng + HA;
        const int offB = isg ? HA + fo0 * KC + tid : tid - ng;
        if (spread & 4) {
          const int ni = ng + HA;
          const bool ok = gather(rs, base0, NXB, Gr, ni, [&](int i) { return i < ng ? HA + fo0 * KC + i : i - ng; },
                                 all_items, ep, a.abort_flag, stg);
          if (!all_ok(ok, ish)) return;
          if (tid < ni) {
            sum = stg[tid];
            for (int p = 1; p < Gr; ++p) sum += stg[p * ni + tid];
          }
          if (ish_) hdr[tid - ng] = sum;
          __syncthreads();
        } else {
          const bool ok = fl2 ? poll<true, double, 16>(rs, base0, NXB, Gr, -1, offB, isg || ish_, ep, nullptr, 0, &sum,
                                                        a.abort_flag)
                                : poll<true>(rs, base0, NXB, Gr, -1, offB, isg || ish_, ep, nullptr, 0, &sum, a.abort_flag);
          if (ish_) hdr[tid - ng] = sum;
          if (!all_ok(ok, ish)) return;
        }
        tstamp(s, it, 5);
        prof.stamp(8);
        // owned weight: gradient (softmax.py:57-58), momentum (sghmc.py:31,34), drift (:32)
        if (own) {
          const T gr = -((T)sum - alpha * wv);
          const T p = (ome * pw + eps * gr) + nsc * zn;
          pw = p;
          if (!last) wv = wv + eps * p;
          else kin1 = (double)p * (double)p;
        }
        if (tid < K) {                                                      // bias sub-step, replicated
          const T gr = -((T)hdr[tid] - alpha * bpsh[tid]);
          pbsh[tid] = (ome * pbsh[tid] + eps * gr) + nsc * zb;
          bsh[tid] = bpsh[tid];
        }
        if (last) ll_last = hdr[KC];                                        // ll(q_new) on this batch
      }
      if (last) break;
      // ===== B-AG: drifted owned weights → every member of the feature team
      prof.stamp(9);
      {
        ++ep;
        const int per = p2_pad(Fo * KC, pad);
        const int reg = a.oXW + (((int)(uW & 1) * Gf + f) * Gr + r) * per;
        if (tid < nfo * KC) put_t(fl2, rs, reg + tid, own ? (double)wv : 0.0, ep);
        tstamp(s, it, 6);
        if (own) Wf[wl] = wv;
        const int base0 = a.oXW + ((int)(uW & 1) * Gf + f) * Gr * per;
        ++uW;
        if (spread & 8) {
          const int ni = Fo * KC;
          const auto want = [&](int p, int i) { return p != r && p < min(Gr, (nfeat - i / KC + Fo - 1) / Fo); };
          const bool ok = gather(rs, base0, per, Gr, ni, [](int i) { return i; }, want, ep, a.abort_flag, stg);
          if (!all_ok(ok, ish)) return;
          for (int q = tid; q < Gr * ni; q += QTH) {
            const int p = q / ni, i = q - p * ni;
            if (want(p, i)) Wf[(p * Fo + i / KC) * 16 + i % KC] = (T)stg[q];
          }
          __syncthreads();
          tstamp(s, it, 7);
          continue;
        }
        const int dloc = tid / KC, kk = tid - (tid / KC) * KC;
        const int npd = tid < Fo * KC ? min(Gr, (nfeat - dloc + Fo - 1) / Fo) : 0;   // producers owning feature dloc
        const bool ok = fl2 ? poll<false, T, 16>(rs, base0, per, npd, r, tid, tid < Fo * KC, ep, nullptr, 0, nullptr,
                                                  a.abort_flag, Wf + dloc * 16 + kk, Fo * 16)
                              : poll<false>(rs, base0, per, npd, r, tid, tid < Fo * KC, ep, nullptr, 0, nullptr,
                                            a.abort_flag, Wf + dloc * 16 + kk, Fo * 16);
        if (!all_ok(ok, ish)) return;
        tstamp(s, it, 7);
      }
    }

    if (bar && n > 0 && own) wv = Wf[wl];            // the slice lives in LDS (last write: barrier-ed)
    // ===== accept (hmc.py:67-71): all-gather of the kinetic / log-likelihood partials
    prof.stamp(10);
    const double kin1w = wsum(kin1, dsh);
    double kb1 = 0.0;
    for (int k = 0; k < K; ++k) kb1 += (double)pbsh[k] * (double)pbsh[k];
    ++ep;
    {
      const int reg = a.oXS + ((int)(uS & 1) * G + bid) * NXS;
      if (tid == 0) put(rs, reg + 0, kin0, ep);
      if (tid == 1) put(rs, reg + 1, kin1w, ep);
      if (tid == 2) put(rs, reg + 2, ll0, ep);
    }
    // next step's tile and labels while the partials travel: Xs and Yo have no reader left in this
    // step (the last B-gemm and softmax ended before a barrier)
    // (measured: loading it with only the half of the workgroup that does not poll the accept round
    // is slower — 9.68 vs 9.44 µs per leapfrog: two load batches instead of one)
    if (prefetch && s + 1 < a.n_steps) {
      const int64_t rn = sched_at(inl, s + 1, a.inl[sched_k(s + 1)].row0, a.row0);
      const T* Xn = reinterpret_cast<const T*>(a.X) + (size_t)rn * D;
      const T* Yn = reinterpret_cast<const T*>(a.Y) + (size_t)rn * K;
      load_step_rows<T>(Xs, Yo, Xn, Yn, Br, BfP, BFP, nrow, nfeat, row0, feat0, D, K, Ro, nro, ro0);
    }
    const int sbase = a.oXS + (int)(uS & 1) * G * NXS;
    ++uS;
    double v3[3] = {0.0, 0.0, 0.0};
    if (acc1) {
      // the three partials of workgroup tid in one batch of loads (one round trip, not three)
      const bool ok = poll_nb<1, false, double>(rs, sbase + tid * NXS, 1, 3, -1, 0, tid < G, ep, nullptr,
                                                a.abort_flag, stg + 3 * tid, 1);
      if (!all_ok(ok, ish)) return;
      if (tid < G) { v3[0] = stg[3 * tid]; v3[1] = stg[3 * tid + 1]; v3[2] = stg[3 * tid + 2]; }
    } else {
      bool ok = true;
#pragma unroll
      for (int j = 0; j < 3; ++j)
        ok = ok && poll<true>(rs, sbase + j, NXS, 1, -1, tid * NXS, tid < G, ep, nullptr, 0, &v3[j], a.abort_flag);
      if (!all_ok(ok, ish)) return;
    }
    const double S0 = wsum(v3[0], dsh), S1 = wsum(v3[1], dsh), L0 = wsum(v3[2], dsh);
    const double K0 = (0.0 + 0.5 * S0) + 0.5 * kb0;
    const double Ecur = a.neg_inv_n * (L0 + a.log_prior) + K0;
    double A, Enew, llq;
    int acc;
    if (n <= 0) {
      A = 1.0; Enew = Ecur; llq = L0;
      acc = sched_at(inl, s, a.inl[sched_k(s)].u, a.u) < A;
    } else {
      const double K1 = (0.0 + 0.5 * S1) + 0.5 * kb1;
      Enew = a.neg_inv_n * (ll_last + a.log_prior) + K1;
      const double x = exp(Ecur - Enew);
      A = (x < 1.0) ? x : 1.0;                                             // Python min(1, x)
      acc = sched_at(inl, s, a.inl[sched_k(s)].u, a.u) < A;
      llq = acc ? ll_last : L0;
    }
    if (!acc || n <= 0) {                                                  // keep q (sghmc.py:36-38)
      for (int e = tid; e < BfP * 16; e += QTH) Wf[e] = Wf0[e];
      wv = w0;
      if (tid < 16) bsh[tid] = b0sh[tid];
    }
    if (a.out_mom && s == a.n_steps - 1) {                                 // sghmc.py:36-39 returned p
      T* mo = reinterpret_cast<T*>(a.out_mom);
      const bool keep_new = acc && n > 0;
      if (own) mo[e_own] = keep_new ? (bar ? pWs[wl] : pw) : pw0;
      if (bid == 0 && tid < K) mo[D * K + tid] = keep_new ? pbsh[tid] : pb0sh[tid];
    }
    if (a.out_trace) {                                                     // sghmc_multicore.py:49-51 row
      T* tr = reinterpret_cast<T*>(a.out_trace) + (size_t)s * (D * K + K);
      if (own) tr[e_own] = wv;
      if (bid == 0 && tid < K) tr[D * K + tid] = bsh[tid];
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
  // ---- commit round: every workgroup publishes a 'done' granule; workgroup 0 gathers all G and
  //      proposes commit (or abort, when its gather times out or sees the abort word) on the launch's
  //      decision word; the others wait for the decision (bounded: on timeout they propose abort).
  //      The first compare-and-swap decides and everyone follows it, so either every workgroup
  //      writes its slice of W/b or none does — independent timeouts (each measured from its own
  //      publish) cannot split the launch, and a decided abort leaves W/b untouched for the re-run.
  //      A member that timed out anywhere earlier never publishes, so workgroup 0 cannot commit.
  ++ep;
  if (tid == 0) put(rs, a.oXC + bid, 1.0, ep);
  {
    unsigned long long* dword = reinterpret_cast<unsigned long long*>(a.arena + (size_t)(a.oXC + G) * 16);
    if (bid == 0) {
      const bool ok = gather_st(rs, a.oXC, 1, G, 1, [](int) { return 0; }, ep, a.abort_flag, [](int, double) {});
      const bool all = all_ok(ok, ish);
      if (tid == 0) ish[1] = p2_decide(dword, ep, all ? P2_COMMIT : P2_ABORT);
    } else if (tid == 0) {
      ish[1] = p2_wait_decision(dword, ep, a.abort_flag);
    }
    __syncthreads();
    if (ish[1] != P2_COMMIT) return;
  }
  // ---- committed state: owners write their weights, workgroup 0 the bias
  verdict.done = true;
  if (own) reinterpret_cast<T*>(a.W)[e_own] = wv;
  if (bid == 0 && tid < K) reinterpret_cast<T*>(a.b)[tid] = bsh[tid];
}

// ---------------------------------------------------------------- plan + launch
static int kc_of(int K) { return K == 10 ? 10 : 16; }

static size_t p2_lds(const PersistPlan2& p, int K, size_t ts) {
  const int WPA = std::max(1, QNW / (p.Br / 16)), WPB = std::max(1, QNW / (p.BfP / 16));
  const int ZPN = std::max(WPA * p.Br, WPB * p.BfP) * 16;
  size_t t = ts * ((size_t)p.Br * p.BFP + 2 * (size_t)p.BfP * 16 + (size_t)p.Gf * p.Ro * 16 + ZPN +
                   4 * (size_t)p.Ro * 16 + 64);
  t += ts * 16;                                                              // pb0sh
  t = (t + 15) & ~(size_t)15;
  t += 8 * ((size_t)p.Ro + 32) + 16 + 16 * 8 + 8 * (size_t)QSTAGE + ts * ((size_t)p.Fo * 16 + 16);
  t += ts * ((size_t)p.BfP * 16);                                            // pWs (bar)
  (void)K;
  return t;
}

PersistPlan2 plan_p2(int B, int D, int K, size_t ts, int num_cus, size_t lds_max) {
  PersistPlan2 best{};
  best.ok = false;
  if (K > 16 || K < 1 || B < 1 || D < 1) return best;
  const int KC = kc_of(K);
  int fGr = 0, fGf = 0;
  if (const char* env = getenv("HMCX_P2_GRID")) sscanf(env, "%dx%d", &fGr, &fGf);
  const int cand[] = {1, 2, 4, 8, 16};
  for (int Gr : cand)
    for (int Gf : cand) {
      if (fGr && (Gr != fGr || Gf != fGf)) continue;
      const int G = Gr * Gf;
      if (G > num_cus) continue;
      PersistPlan2 p{};
      p.Gr = Gr; p.Gf = Gf;
      const int rows = (B + Gr - 1) / Gr;
      p.Br = 16;
      while (p.Br < rows) p.Br <<= 1;                                         // power of two (GEMM split)
      if (p.Br > QTH) continue;
      p.Bf = (D + Gf - 1) / Gf;
      p.BfP = (p.Bf + 15) / 16 * 16;
      // odd row pitch: the A-gemm's column reads (16 rows per ds_read2_b64 group) hit 16 distinct bank
      // pairs; the B-gemm reads its k values Br/4 rows apart per lane group (mfma_tile), 2·BFP·16 ≡ 32
      // dwords mod 64, so the two half-waves of its ds_read_b64 land on disjoint banks
      p.BFP = p.BfP + 1;
      p.Ro = (p.Br + Gf - 1) / Gf;
      p.Fo = (p.Bf + Gr - 1) / Gr;
      if ((long)(Gr - 1) * rows >= B || (long)(Gf - 1) * p.Bf >= D) continue;  // no empty teams
      // thread ↔ element mappings of the rounds (one granule per producer per thread)
      if (KC + 1 + p.Ro * KC > QTH || p.Fo * KC + KC + 1 > QTH || G > QTH) continue;
      p.lds = p2_lds(p, K, ts);
      if (p.lds > lds_max) continue;
      // cost model (calibrated on MI355X at B=500, D=784, K=10: 8x16 15.6, 16x8 16.3, 8x8 16.7,
      // 16x16 16.8, 4x16 27 µs per leapfrog): f64 MFMAs per wave of the two GEMMs, plus a price per
      // member of the row teams (A rounds, softmax skew) and of the feature teams
      const int WPA = std::max(1, QNW / (p.Br / 16)), WPB = std::max(1, QNW / (p.BfP / 16));
      const double mfma = (double)(p.Br / 16) * (p.BfP / 4) / QNW + (double)(p.BfP / 16) * (p.Br / 4) / QNW;
      const double cost = 300.0 * mfma + 700.0 * Gr + 400.0 * Gf + 0.0 * (WPA + WPB);
      p.cost = cost;
      p.ok = true;
      if (!best.ok || cost < best.cost) best = p;
    }
  return best;
}

template <typename T>
int sghmc_p2_t(hmcx_ctx* ctx, const hmcx_sampler_args* s, const PersistPlan2& pl) {
  const int G = pl.Gr * pl.Gf, K = s->K, KC = kc_of(K);
  const size_t n = (size_t)s->n_steps;
  // granule arena: XA, XD, XB, XW, XS (double-buffered), then the abort word
  static const int pad = !(getenv("HMCX_P2_PAD") && getenv("HMCX_P2_PAD")[0] == '0');
  const long nXA = 2L * G * pl.Br * KC, nXD = 2L * G * p2_pad(KC + 1 + pl.Ro * KC, pad),
             nXB = 2L * G * p2_pad(KC + 1 + pl.Bf * KC, pad), nXW = 2L * G * p2_pad(pl.Fo * KC, pad),
             nXS = 2L * G * (pad ? 8 : 4);
  const long nXC = G + 1;                        // 'done' granules + the launch's decision word
  const long ngran = nXA + nXD + nXB + nXW + nXS + nXC + 1;
  if (ngran * 16 > 0x7fffffffL) return set_error(ctx, HMCX_EUNSUPPORTED, "persistent SGHMC: arena too large");
  int rc = abort_precheck(ctx);                  // an earlier launch's timeout, before enqueueing more
  if (rc) return rc;
  // the call's schedule travels in one packed host-to-device copy
  const bool buf = s->noise_mode == HMCX_NOISE_BUFFER;
  const void* hsrc[5] = {s->eps, s->u_accept, s->row0, s->n_iter, buf ? (const void*)s->noise_off : nullptr};
  const size_t hbytes[5] = {n * sizeof(double), n * sizeof(double), n * sizeof(int64_t), n * sizeof(int32_t),
                            buf ? n * sizeof(int64_t) : 0};
  for (int i = 0; i < 5; ++i)
    if (hbytes[i] && !hsrc[i]) return set_error(ctx, HMCX_EINVAL, "sghmc: null host schedule array");
  const size_t sched_bytes = packed_bytes(5, hbytes);
  // the exchange arena is the context's granule arena: every launch polls for epochs of its own,
  // never written before, so it is not cleared per call
  if ((rc = gx_reserve(ctx, (size_t)ngran * 16))) return rc;
  char* arena = ctx->gx_arena;
  unsigned rounds = 0;                           // ≤ 5 epochs per leapfrog iteration (it = -1 … L-1, accept)
  for (size_t i = 0; i < n; ++i) rounds += 5u * (unsigned)(std::max(s->n_iter[i], 0) + 2);
  rounds += 1;                                   // the commit round
  unsigned ep0 = 1;
  if ((rc = gx_epochs(ctx, rounds, &ep0))) return rc;
  Q2Args a{};
  // a short call's schedule (the driver's 20-step call) rides in the kernel arguments: no staging
  // copy, no upload, no staging event ahead of the launch
  char* dp[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  if (!buf && n <= (size_t)P2_NINL) {
    a.ninl = (int)n;
    for (size_t i = 0; i < n; ++i) {
      a.inl[i].eps = s->eps[i];
      a.inl[i].u = s->u_accept[i];
      a.inl[i].row0 = s->row0[i];
      a.inl[i].n_iter = s->n_iter[i];
    }
  } else {
    Workspace ws(ctx);
    char* sched;
    do {
      ws.reset();
      sched = ws.take<char>(sched_bytes);
    } while (ws.retry());
    if (ws.failed) return HMCX_ENOMEM;
    begin_call(ctx);
    if ((rc = upload_packed(ctx, sched, 5, hsrc, hbytes, dp))) return rc;
  }
  double* d_eps = reinterpret_cast<double*>(dp[0]);
  double* d_u = reinterpret_cast<double*>(dp[1]);
  int64_t* d_row0 = reinterpret_cast<int64_t*>(dp[2]);
  int32_t* d_n = reinterpret_cast<int32_t*>(dp[3]);
  int64_t* d_noff = reinterpret_cast<int64_t*>(dp[4]);

  a.B = s->B; a.D = s->D; a.K = K; a.P = s->D * K + K; a.n_steps = s->n_steps;
  a.Gr = pl.Gr; a.Gf = pl.Gf; a.Br = pl.Br; a.Bf = pl.Bf; a.BfP = pl.BfP; a.BFP = pl.BFP; a.Ro = pl.Ro; a.Fo = pl.Fo;
  a.alpha = s->alpha; a.neg_inv_n = -1.0 / (double)s->B; a.log_prior = s->log_prior;
  a.X = s->X; a.Y = s->Y;
  a.eps = d_eps; a.u = d_u; a.row0 = d_row0; a.n_iter = d_n;
  if (a.ninl > 0) {              // the kernel loads both sources and selects the value (sched_at)
    a.eps = a.u = reinterpret_cast<double*>(ctx->zeros_dev);
    a.row0 = reinterpret_cast<int64_t*>(ctx->zeros_dev);
    a.n_iter = reinterpret_cast<int32_t*>(ctx->zeros_dev);
  }
  a.noise_mode = s->noise_mode; a.noise = s->noise; a.noff = d_noff;
  a.seed = s->seed; a.chain0 = s->chain0; a.step_base = s->step_base;
  a.W = s->W; a.b = s->b;
  a.arena = arena;
  a.oXA = 0; a.oXD = (int)nXA; a.oXB = (int)(nXA + nXD); a.oXW = (int)(nXA + nXD + nXB);
  a.oXS = (int)(nXA + nXD + nXB + nXW);
  a.oXC = (int)(nXA + nXD + nXB + nXW + nXS);
  a.arena_bytes = (int)(ngran * 16);
  a.ep0 = ep0;
  a.pad = pad;
  static const bool dbg = getenv("HMCX_P2_DEBUG") && getenv("HMCX_P2_DEBUG")[0] == '1';
  if (dbg)
    fprintf(stderr, "[hmcx p2] B=%d D=%d K=%d plan %dx%d Br=%d Bf=%d BfP=%d Ro=%d Fo=%d; granule bases XA %d XD %d XB %d "
            "XW %d XS %d XC %d; epochs %u..%u\n", s->B, s->D, K, pl.Gr, pl.Gf, pl.Br, pl.Bf, pl.BfP, pl.Ro, pl.Fo,
            a.oXA, a.oXD, a.oXB, a.oXW, a.oXS, a.oXC, ep0, ep0 + rounds - 1);
  {
    const int HA = KC + 1;
    const bool fits = pl.Gf * pl.Ro * KC <= QSTAGE && pl.Gf * (HA + pl.Ro * KC) <= QSTAGE &&
                      pl.Gr * (pl.Fo * KC + HA) <= QSTAGE && pl.Gr * pl.Fo * KC <= QSTAGE;
    static const int spread_env = getenv("HMCX_P2_SPREAD") ? atoi(getenv("HMCX_P2_SPREAD")) : 2;
    a.spread = fits ? spread_env : 0;
    a.zoff = !(getenv("HMCX_P2_ZOFF") && getenv("HMCX_P2_ZOFF")[0] == '0');
    static const int bar_env = getenv("HMCX_P2_BAR") ? atoi(getenv("HMCX_P2_BAR")) : 1;
    a.bar = bar_env == 1 ? 1 : 0;
    // HMCX_P2_XMAP: which team shares an XCD (workgroups are dealt to the XCDs round-robin).  0 = identity
    // map: each FEATURE team on one XCD, its B rounds kept in that XCD's L2 (default with the B all-
    // reduce: its redundant reads, 8x the bytes of the other rounds, then stay off the fabric — same
    // speed, 11.1 -> 4.5 MB of fabric traffic per leapfrog); 1 = each ROW team on one XCD (default
    // without it); 2 = deliberately MISPLACED (test knob, read per call): identity map with the row-team
    // rounds published into one XCD's L2, so members on other XCDs never see them — the launch times
    // out (4 s) and aborts
    const int xmap_env = getenv("HMCX_P2_XMAP") ? atoi(getenv("HMCX_P2_XMAP")) : (a.bar ? 0 : 1);
    a.xmap = (xmap_env == 1 && (pl.Gr * pl.Gf) % 8 == 0) ? 1 : 0;
    static const int fl2_env = getenv("HMCX_P2_FL2") ? atoi(getenv("HMCX_P2_FL2")) : 1;
    a.fl2 = (fl2_env == 1 && !a.xmap && pl.Gf % 8 == 0 && xmap_env != 2) ? 1 : 0;
    a.al2 = (fl2_env == 1 && a.xmap && ((pl.Gr * pl.Gf) / 8) % pl.Gf == 0) ? 1 : 0;
    if (xmap_env == 2) a.al2 = 1;
    static const int pf_env = getenv("HMCX_P2_PREFETCH") ? atoi(getenv("HMCX_P2_PREFETCH")) : 1;
    a.prefetch = pf_env == 1 ? 1 : 0;
    static const int acc1_env = getenv("HMCX_P2_ACC1") ? atoi(getenv("HMCX_P2_ACC1")) : 1;
    a.acc1 = acc1_env == 1 ? 1 : 0;
  }
  a.abort_flag = ctx->abort_dev;
  a.force_abort = getenv("HMCX_P2_FORCE_ABORT") ? atoi(getenv("HMCX_P2_FORCE_ABORT")) : -1;
  a.out_A = s->out_A; a.out_acc = s->out_accepted; a.out_ll = s->out_ll; a.out_E = s->out_E;
  a.out_trace = s->out_trace;
  a.out_mom = s->out_mom;
  a.verdict = s->out_abort;
  // out_host in the packed layout (include/hmcx.h): the kernel stores the per-step outputs and its
  // verdict straight into the pinned host block (a handful of values per step) — no copy behind the
  // launch, so the host's wait ends when the kernel does
  const bool direct_host = s->out_host && s->out_E && s->out_abort && s->out_ll == s->out_A + n &&
                           s->out_E == s->out_A + 2 * n &&
                           reinterpret_cast<char*>(s->out_accepted) == reinterpret_cast<char*>(s->out_A) + 32 * n &&
                           reinterpret_cast<char*>(s->out_abort) == reinterpret_cast<char*>(s->out_A) + 36 * n;
  if (direct_host) {
    char* h = reinterpret_cast<char*>(s->out_host);
    a.out_A = reinterpret_cast<double*>(h);
    a.out_ll = a.out_A + n;
    a.out_E = a.out_A + 2 * n;
    a.out_acc = reinterpret_cast<int32_t*>(h + 32 * n);
    a.verdict = reinterpret_cast<int*>(h + 36 * n);
  }
  static const bool prof_on = getenv("HMCX_PERSIST_PROF") && getenv("HMCX_PERSIST_PROF")[0] == '1';
  unsigned long long* dprof = nullptr;
  if (prof_on) {
    HMCX_HIP(ctx, hipMalloc((void**)&dprof, 16 * sizeof(unsigned long long)));
    HMCX_HIP(ctx, hipMemsetAsync(dprof, 0, 16 * sizeof(unsigned long long), ctx->stream));
  }
  a.prof = dprof;
  static const bool trace_on = getenv("HMCX_P2_TRACE") && getenv("HMCX_P2_TRACE")[0] == '1';
  unsigned long long* dtrace = nullptr;
  const size_t ntr = (size_t)G * P2TR_IT * 8;
  if (trace_on) {
    HMCX_HIP(ctx, hipMalloc((void**)&dtrace, ntr * sizeof(unsigned long long)));
    HMCX_HIP(ctx, hipMemsetAsync(dtrace, 0, ntr * sizeof(unsigned long long), ctx->stream));
  }
  a.trace = dtrace;
  // the folded instantiation when the call is exactly BASELINE config 2's plan with default knobs
  const bool spec = sizeof(T) == 8 && KC == 10 && s->B == 500 && s->D == 784 && K == 10 && pl.Gr == 8 && pl.Gf == 16 &&
                    pl.Br == 64 && pl.Bf == 49 && pl.BfP == 64 && pl.BFP == 65 && pl.Ro == 4 && pl.Fo == 7 &&
                    a.spread == 2 && a.pad == 1 && a.xmap == 0 && a.fl2 == 1 && a.al2 == 0 && a.prefetch == 1 &&
                    a.acc1 == 1 && a.zoff == 1 && a.bar == 1 && !a.trace;
  static const bool no_spec = getenv("HMCX_P2_SPEC") && getenv("HMCX_P2_SPEC")[0] == '0';
  const void* kfn = (spec && !no_spec) ? (a.prof ? (const void*)k_sghmc_p2<T, 10, 3> : (const void*)k_sghmc_p2<T, 10, 1>)
                    : KC == 10 ? (const void*)k_sghmc_p2<T, 10> : (const void*)k_sghmc_p2<T, 16>;
  void* kargs[] = {&a};
  // co-residency of all G workgroups is checked here (occupancy query × CUs, cached per kernel); a
  // plain launch then has the same residency as a cooperative one without its per-launch host cost
  int per_cu = 0;
  if ((rc = kernel_occupancy(ctx, kfn, QTH, (int)pl.lds, &per_cu))) return rc;
  if ((long)per_cu * ctx->num_cus < G)
    return set_error(ctx, HMCX_EUNSUPPORTED, "persistent SGHMC: workgroups cannot be co-resident");
  // the verdict is sticky (P2Verdict): zeroed here, only a workgroup that leaves without committing
  // stores 1.  The call's output slot is idle at enqueue time (the caller collected its previous use).
  if (direct_host)
    *reinterpret_cast<volatile int*>(a.verdict) = 0;
  else if (a.verdict)
    HMCX_HIP(ctx, hipMemsetAsync(a.verdict, 0, sizeof(int), ctx->stream));
  if ((rc = timing_begin(ctx, ctx->stream))) return rc;
  HMCX_HIP(ctx, hipLaunchKernel(kfn, dim3(G), dim3(QTH), kargs, (unsigned)pl.lds, ctx->stream));
  if ((rc = timing_end(ctx, ctx->stream))) return rc;
  if (s->out_host && direct_host) {
    if (!dprof && !dtrace) return HMCX_OK;
  } else if (s->out_host) {                      // outputs and this launch's verdict
    char* h = reinterpret_cast<char*>(s->out_host);
    const bool packed = s->out_abort == reinterpret_cast<int32_t*>(reinterpret_cast<char*>(s->out_A) + 36 * n);
    HMCX_HIP(ctx, hipMemcpyAsync(h, s->out_A, 36 * n + (packed ? sizeof(int) : 0), hipMemcpyDeviceToHost,
                                 ctx->stream));
    if (!packed)
      HMCX_HIP(ctx, hipMemcpyAsync(h + 36 * n, s->out_abort ? (const void*)s->out_abort : ctx->abort_dev,
                                   sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    if (!dprof && !dtrace) return HMCX_OK;
  }
  if (s->out_abort) {                            // the kernel stored this launch's verdict there itself
    if (!dprof && !dtrace) return HMCX_OK;
  } else if (!dprof && !dtrace) {                // no per-call sync: checked once the launch is done
    return abort_defer(ctx, a.abort_flag, ctx->stream);
  }
  int flag = 0;
  HMCX_HIP(ctx, hipMemcpyAsync(&flag, a.abort_flag, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  HMCX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (dprof) {
    unsigned long long h[16];
    HMCX_HIP(ctx, hipMemcpy(h, dprof, sizeof(h), hipMemcpyDeviceToHost));
    (void)hipFree(dprof);
    unsigned long long tot = 0;
    for (int i = 0; i < 12; ++i) tot += h[i];
    static const char* names[12] = {"step-start", "A-gemm+publish", "noise", "A-RS wait", "softmax", "A-AG",
                                    "B-gemm+publish", "B-RS wait", "update", "B-AG", "accept", "it=-1"};
    fprintf(stderr, "[hmcx p2 prof] G=%dx%d Br=%d Bf=%d Ro=%d Fo=%d total %llu ticks:", pl.Gr, pl.Gf, pl.Br, pl.Bf,
            pl.Ro, pl.Fo, tot);
    for (int i = 0; i < 12; ++i) fprintf(stderr, " %s %.1f%%", names[i], tot ? 100.0 * h[i] / tot : 0.0);
    fprintf(stderr, "\n");
  }
  if (dtrace) {
    std::vector<unsigned long long> h(ntr);
    HMCX_HIP(ctx, hipMemcpy(h.data(), dtrace, ntr * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    (void)hipFree(dtrace);
    // per round: latency = consumed(b) − last publish of b's team; skew = last team publish − publish(b)
    static const char* rn[4] = {"A-RS", "A-AG", "B-RS", "B-AG"};
    for (int rd = 0; rd < 4; ++rd) {
      double lat = 0, skew = 0, lmax = 0;
      long cnt = 0;
      for (int it = 1; it < P2TR_IT; ++it)
        for (int b = 0; b < G; ++b) {
          const int r = b / pl.Gf, f = b % pl.Gf;
          const unsigned long long pub = h[((size_t)b * P2TR_IT + it) * 8 + 2 * rd];
          const unsigned long long done = h[((size_t)b * P2TR_IT + it) * 8 + 2 * rd + 1];
          if (!pub || !done) continue;
          unsigned long long mx = 0;
          const bool rowteam = rd < 2;
          const int nm = rowteam ? pl.Gf : pl.Gr;
          bool okm = true;
          for (int m = 0; m < nm; ++m) {
            const int pb = rowteam ? r * pl.Gf + m : m * pl.Gf + f;
            const unsigned long long v = h[((size_t)pb * P2TR_IT + it) * 8 + 2 * rd];
            if (!v) okm = false;
            mx = v > mx ? v : mx;
          }
          if (!okm) continue;
          const double l = (double)(long long)(done - mx) * 10.0 / 1000.0;   // µs (100 MHz ticks)
          lat += l; lmax = l > lmax ? l : lmax;
          skew += (double)(long long)(mx - pub) * 10.0 / 1000.0;
          ++cnt;
        }
      if (cnt) fprintf(stderr, "[hmcx p2 trace] %s: latency after last team publish %.2f us (max %.2f), own wait for "
                       "slowest member %.2f us (n=%ld)\n", rn[rd], lat / cnt, lmax, skew / cnt, cnt);
    }
    // iteration period from block 0
    const unsigned long long t1 = h[1 * 8 + 0], t2 = h[(P2TR_IT - 1) * 8 + 0];
    if (t1 && t2) fprintf(stderr, "[hmcx p2 trace] leapfrog period %.2f us\n", (double)(t2 - t1) * 10.0 / 1000.0 / (P2TR_IT - 2));
  }
  if (flag) return set_error(ctx, HMCX_EHIP, "persistent SGHMC: hand-off timed out (workgroups not co-resident?)");
  return HMCX_OK;
}

template int sghmc_p2_t<float>(hmcx_ctx*, const hmcx_sampler_args*, const PersistPlan2&);
template int sghmc_p2_t<double>(hmcx_ctx*, const hmcx_sampler_args*, const PersistPlan2&);

}  // namespace hmcx
