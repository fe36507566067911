// hmcx_sgld_p.hip — single-chain SGLD for wide feature / class counts (BASELINE config 5: PlantVillage-
// like conv features, D = 2048, K = 38, batch 500) as ONE persistent launch per sampler call.
//
// Mathematics and op order: cpu/sgld.py:31-46 (p = N(0,(2ε)²) drawn per variable, p += −½ε·g,
// q += p) with the gradient of cpu/softmax.py:38-61 (z = XW + b, clip, softmax, diff = y − ŷ,
// gW = −(Xᵀ·diff − αW), gb = −(Σ_rows diff − αb)), exactly as the three-launch path of
// hmcx_wide.hip; only the schedule differs.  The per-10-minibatch log-likelihood of sgmcmc.py:60-62,
// 74-76 (the state after the step, on the step's minibatch) rides in the same launch.
//
// Geometry.  G = Gr × Gf workgroups (config 5: 8 × 32 = 256, one per CU).  Workgroup (r, f) holds
// the minibatch tile X[R_r, F_f] (Br ≤ 64 rows × Bf ≤ 64 features) in LDS — double-buffered, the
// next step's tile is loaded while this step's exchanges travel — and the weight slice W[F_f, :]
// (every member of feature team f holds the same bits).  Per step, four team rounds over tagged
// granules (hmcx_p2x.h: one 16-byte {lo, epoch, hi, epoch} store per value, re-read until both
// epoch words match; bounded spins):
//   A   MFMA partial logits X[R_r,F_f]·W[F_f] → row team r; reduce-scatter: owner f of rows
//       [f·Ro, (f+1)·Ro) sums the Gf partials in producer order, adds b, runs the softmax;
//   AG  the owners' diff rows → every member of the row team (the whole row block in LDS);
//   B   MFMA partial gradient X[R_r,F_f]ᵀ·diff[R_r] (+ the row block's diff column sums, for the
//       bias) → feature team f; reduce-scatter: owner r of slice elements [r·Eo, (r+1)·Eo) sums the
//       Gr partials in producer order and applies the SGLD update;
//   BAG the owners' new weights → every member of the feature team.
// The bias is updated by every workgroup identically (its Gr column sums arrive with round B).
// Logging steps add one forward of the new state (A + reduce-scatter) and a sum of the owners'
// log-likelihood partials by workgroup 0.
//
// Every round has its own epoch (unique over the arena's life) and its region is double-buffered by
// step parity.  A producer cannot overwrite a region before its consumers have read it: writing
// round A of step s+1 needs round AG of step s, which needs every row-team member to have finished
// its A reads of step s (and likewise for the other rounds).  A timed-out spin raises the call's
// abort word; the workgroups then leave, no weight reaches global memory (W / b are written once,
// at the end of the call) and the host re-runs the call on the three-launch path.
#include "hmcx_common.h"
#include "hmcx_internal.h"
#include "hmcx_p2x.h"
#include <algorithm>
#include <vector>
#include <cstdio>

namespace hmcx {

constexpr int SPT = 256;          // threads per workgroup (4 waves)
constexpr int SPB = 64;           // largest row block / feature slice (one 16-row MFMA tile per wave)

struct SgldSched { double eps; int64_t row0; int64_t noff; int32_t want_ll; int32_t pad_; };

template <typename T> struct SgldPArgs {
  int B, D, K, KP, Gr, Gf, Br, Bf, Ro, Eo, n_steps;
  T alpha, clip_hi, clip_lo;
  const T* X; const T* Y; T* W; T* b;
  const SgldSched* sched;
  int noise_mode; const double* noise; uint64_t seed; uint32_t chain, step_base;
  char* arena; int arena_bytes;
  int oXA, oXD, oXB, oXW, oXL;      // region offsets (granules); each region is [2][...] by step parity
  unsigned ep0;
  int* abort_flag;
  int force_abort;                  // HMCX_SGLD_FORCE_ABORT=1: the last workgroup leaves at step 0 (tests)
  unsigned long long* prof;         // HMCX_SGLD_PROF=<file>: per-workgroup phase totals (s_memrealtime)
  double* out_ll;
  // LDS pitches (elements)
  int xp, wp, dp;
};

template <typename T> __device__ inline T sgld_noise(const SgldPArgs<T>& a, int64_t noff, uint32_t step, uint32_t e) {
  // sgld.py:41-46 draw_momentum: N(0, 1) per element in start.keys() order (weights, then bias),
  // scaled by 2ε at the use
  if (a.noise_mode == HMCX_NOISE_BUFFER) return (T)a.noise[noff + e];
  return philox_normal_t<T>(a.seed, a.chain, step, 0u, e);
}

// Gather `np` producers × `ni` items: item i of producer p is granule base + p·pstride + i; every
// (p, i) pair with want(p, i) is dealt over the workgroup, ≤ 16 pairs per thread per pass (larger
// rounds in chunks), and handed to store(p, i, value).  false on timeout / abort.
struct IdOff { __device__ int operator()(int i) const { return i; } };
template <typename Want, typename Store, typename Off = IdOff>
__device__ inline bool sgld_gather(__amdgpu_buffer_rsrc_t rs, int base, int pstride, int np, int ni, unsigned ep,
                                   int* abort_flag, Want want, Store store, Off ioff = Off()) {
  constexpr int U = 16;
  const int npairs = np * ni;
  for (int q0 = 0; q0 < npairs; q0 += U * SPT) {
    unsigned pend = 0;
    int o[U], pp[U], ii[U];
    const int t0 = opaque((int)threadIdx.x);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = q0 + t0 + u * SPT;
      const int p = q / ni, i = q - p * ni;
      const bool w = q < npairs && want(p, i);
      pend |= w ? 1u << u : 0u;
      o[u] = (base + (w ? p * pstride + ioff(i) : 0)) * 16;
      pp[u] = p;
      ii[u] = i;
    }
    unsigned long long ts = 0;
    for (int spins = 0; pend; ++spins) {
      gran_t v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, o[u], 0, 16 /* sc1 */);
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (((pend >> u) & 1u) && v[u].y == ep && v[u].w == ep) {
          store(pp[u], ii[u], decode(v[u]));
          pend &= ~(1u << u);
        }
      if (!pend) break;
      if (spins == 0) ts = __builtin_amdgcn_s_memrealtime();
      if ((spins & 63) == 63 &&
          (__builtin_amdgcn_s_memrealtime() - ts > QTIMEOUT ||
           __hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
        __hip_atomic_store(abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  return true;
}

template <typename T> __device__ inline T wave_max_t(T v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = max_nan(v, __shfl_xor(v, m, 64));
  return v;
}
template <typename T> __device__ inline T wave_sum_t(T v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

// A: partial logits of the tile, published to the row team.  Wave w: rows [16w, 16w + 16) × all
// KP/16 class tiles over the slice's features (Bf / 4 k-steps, KP/16 independent MFMA chains).
template <typename T>
__device__ inline void sgld_phase_a(const SgldPArgs<T>& a, const T* Xs, const T* Ws, __amdgpu_buffer_rsrc_t rs,
                                    int reg, int nrow, int nfeat, unsigned ep) {
  using M = mfma16<T>;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  const int KT = a.KP / 16, nks = (nfeat + 3) / 4;
  typename M::acc_t acc[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) acc[nt] = M::zero();
  if (16 * wave < nrow) {
    for (int ks = 0; ks < nks; ++ks) {
      const int kk = 4 * ks + lg;
      const T av = Xs[(16 * wave + lr) * a.xp + kk];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        if (nt < KT) acc[nt] = M::fma(av, Ws[kk * a.wp + 16 * nt + lr], acc[nt]);
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 16 * wave + M::row(lane, q), k = 16 * nt + lr;
        if (nt < KT && row < nrow && k < a.K) put(rs, reg + row * a.K + k, (double)acc[nt][q], ep);
      }
  }
}

template <typename T>
__global__ __launch_bounds__(SPT) void k_sgld_p(SgldPArgs<T> a) {
  using M = mfma16<T>;
  extern __shared__ __align__(16) unsigned char sm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  const int bid = blockIdx.x, r = bid / a.Gf, f = bid - (bid / a.Gf) * a.Gf;
  const int K = a.K, Gr = a.Gr, Gf = a.Gf, G = Gr * Gf;
  const int rlo = r * a.Br, nrow = max(0, min(a.B - rlo, a.Br));
  const int dlo = f * a.Bf, nfeat = max(0, min(a.D - dlo, a.Bf));
  const int ro0 = f * a.Ro, nro = max(0, min(nrow - ro0, a.Ro));          // rows this member owns
  const int nE = nfeat * K, eo0 = r * a.Eo, neo = max(0, min(nE - eo0, a.Eo));   // slice elements owned
  // LDS: Xs[2][SPB][xp] | Ws[SPB][wp] | Ds[SPB][dp] | stage (reduce-scatter sums) | bias, colsums
  T* Xs0 = reinterpret_cast<T*>(sm);
  T* Ws = Xs0 + 2 * SPB * a.xp;
  T* Ds = Ws + SPB * a.wp;
  double* stage = reinterpret_cast<double*>(Ds + SPB * a.dp);
  const int nstage = max(Gf * a.Ro * K, Gr * (a.Eo + K));
  T* bs = reinterpret_cast<T*>(stage + nstage);                            // [KP] bias
  T* csr = bs + 64;                                                        // [KP] row-block diff column sums
  double* llw = reinterpret_cast<double*>(csr + 64);                       // [4] per-wave ll
  __shared__ int sh_fail;
  if (tid == 0) sh_fail = 0;
  const __amdgpu_buffer_rsrc_t rs = arena_rsrc(a.arena, a.arena_bytes);
  const int XA_n = G * a.Br * K, XD_n = G * a.Ro * K, XB_n = G * (a.Bf * K + K), XW_n = G * a.Eo;

  // ---- prologue: weight slice, bias, step 0's tile (zero padded)
  for (int e = tid; e < SPB * a.KP; e += SPT) {
    const int i = e / a.KP, k = e - (e / a.KP) * a.KP;
    const bool ok = i < nfeat && k < K;
    const T v = a.W[ok ? (size_t)(dlo + i) * K + k : 0];
    Ws[i * a.wp + k] = ok ? v : T(0);
  }
  if (tid < 64) bs[tid] = tid < K ? a.b[min(tid, K - 1)] : T(0);
  auto load_tile = [&](int s, T* dst) {
    const T* xsrc = a.X + ((size_t)a.sched[s].row0 + rlo) * a.D + dlo;
    for (int e0 = 0; e0 < SPB * SPB; e0 += 8 * SPT) {
      T v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + tid + u * SPT, i = e >> 6, j = e & 63;
        const bool ok = i < nrow && j < nfeat;
        v[u] = xsrc[ok ? (size_t)i * a.D + j : 0];
        if (!ok) v[u] = T(0);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + tid + u * SPT;
        dst[(e >> 6) * a.xp + (e & 63)] = v[u];
      }
    }
  };
  load_tile(0, Xs0);
  __syncthreads();

  constexpr int NPF = SPB * SPB / SPT;                                     // next-tile values per thread
  bool failed = false;
  unsigned long long pacc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pt = __builtin_amdgcn_s_memrealtime();
  auto ph = [&](int i) {
    if (a.prof) {
      const unsigned long long t = __builtin_amdgcn_s_memrealtime();
      pacc[i] += t - pt;
      pt = t;
    }
  };
  for (int s = 0; s < a.n_steps && !failed; ++s) {
    const int par = s & 1;
    const T* Xs = Xs0 + par * SPB * a.xp;
    T* Xn = Xs0 + (par ^ 1) * SPB * a.xp;
    const SgldSched sc = a.sched[s];
    const uint32_t step_id = a.step_base + (uint32_t)s;
    const T noise_scale = (T)(2.0 * sc.eps), m_half_eps = (T)(-0.5 * sc.eps);   // sgld.py:43, 37
    const unsigned epA = a.ep0 + 8u * (unsigned)s;
    if (a.force_abort && s == 0 && bid == G - 1) {                        // test knob: a member that never publishes
      if (tid == 0) __hip_atomic_store(a.abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }

    // next step's tile: loads now, LDS stores once this step's B GEMM is done with the other buffer
    T xn[NPF];
    const bool pf = s + 1 < a.n_steps;
    {
      const T* xsrc = a.X + ((size_t)a.sched[pf ? s + 1 : s].row0 + rlo) * a.D + dlo;
#pragma unroll
      for (int u = 0; u < NPF; ++u) {
        const int e = tid + u * SPT, i = e >> 6, j = e & 63;
        const bool ok = pf && i < nrow && j < nfeat;
        xn[u] = xsrc[ok ? (size_t)i * a.D + j : 0];
        if (!ok) xn[u] = T(0);
      }
    }

    // ===== A: partial logits → row team; reduce-scatter to the row owners
    const int regA = a.oXA + par * XA_n + (r * Gf) * a.Br * K;            // producer f' at + f'·Br·K
    ph(0);
    sgld_phase_a<T>(a, Xs, Ws, rs, regA + f * a.Br * K, nrow, nfeat, epA);
    ph(1);
    const int niA = nro * K;
    auto all = [](int, int) { return true; };
    bool ok = sgld_gather(rs, regA + ro0 * K, a.Br * K, Gf, niA, epA, a.abort_flag, all,
                          [&](int p, int i, double v) { stage[p * niA + i] = v; });
    if (!all_ok(ok, &sh_fail)) { failed = true; break; }
    ph(2);
    // softmax of the owned rows (one wave per row, lane = class), diff → own Ds rows + round AG
    const int regD = a.oXD + par * XD_n + (r * Gf) * a.Ro * K;
    const unsigned epD = epA + 1;
    for (int rr = wave; rr < nro; rr += 4) {
      const int k = lane, kc = min(k, K - 1);
      const bool kv = k < K;
      double zs = stage[rr * K + kc];
      for (int p = 1; p < Gf; ++p) zs += stage[p * niA + rr * K + kc];
      const int row = ro0 + rr;
      const T yk = a.Y[((size_t)sc.row0 + rlo + row) * K + kc];
      const T zz = kv ? clipz((T)zs + bs[kc], a.clip_hi, a.clip_lo) : (T)-__builtin_inf();   // softmax.py:39-41
      const T mx = wave_max_t(zz);
      const T ex = kv ? exp(zz - mx) : T(0);                                              // softmax.py:34
      const T sm_ = wave_sum_t(ex);
      const T d = kv ? (kv ? yk : T(0)) - ex / sm_ : T(0);                                // softmax.py:52
      if (kv) {
        Ds[row * a.dp + k] = d;
        put(rs, regD + f * a.Ro * K + rr * K + k, (double)d, epD);
      }
    }
    ph(3);
    // ===== AG: every owner's diff rows → the whole row block in Ds
    // (producer p published the rows it owns: p·Ro + i/K < nrow; its own rows are in Ds already)
    ok = sgld_gather(rs, regD, a.Ro * K, Gf, a.Ro * K, epD, a.abort_flag,
                     [&](int p, int i) { return p != f && p * a.Ro + i / K < nrow; },
                     [&](int p, int i, double v) { Ds[(p * a.Ro + i / K) * a.dp + (i - (i / K) * K)] = (T)v; });
    if (!all_ok(ok, &sh_fail)) { failed = true; break; }
    ph(4);
    // rows past the block and classes past K are zero (for the B GEMM's padding)
    for (int e = tid; e < SPB * a.KP; e += SPT) {
      const int i = e / a.KP, k = e - (e / a.KP) * a.KP;
      if (i >= nrow || k >= K) Ds[i * a.dp + k] = T(0);
    }
    __syncthreads();
    if (tid < K) {                                                        // softmax.py:55 column sums
      T c = Ds[tid];
      for (int i = 1; i < nrow; ++i) c += Ds[i * a.dp + tid];
      csr[tid] = c;
    }

    // ===== B: partial gradient Xᵀ·diff of the slice → feature team (+ the row block's column sums)
    const int regB = a.oXB + par * XB_n + (f * Gr) * (a.Bf * K + K);      // producer r' at + r'·(Bf·K + K)
    const unsigned epB = epA + 2;
    {
      const int KT = a.KP / 16, nks = (nrow + 3) / 4;
      typename M::acc_t acc[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[nt] = M::zero();
      if (16 * wave < nfeat) {
        for (int ks = 0; ks < nks; ++ks) {
          const int kk = 4 * ks + lg;                                     // minibatch row
          const T av = Xs[kk * a.xp + 16 * wave + lr];                    // Xᵀ[feature][row]
#pragma unroll
          for (int nt = 0; nt < 4; ++nt)
            if (nt < KT) acc[nt] = M::fma(av, Ds[kk * a.dp + 16 * nt + lr], acc[nt]);
        }
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int fe = 16 * wave + M::row(lane, q), k = 16 * nt + lr;
            if (nt < KT && fe < nfeat && k < K) put(rs, regB + r * (a.Bf * K + K) + fe * K + k, (double)acc[nt][q], epB);
          }
      }
      __syncthreads();                                                    // csr written
      if (tid < K) put(rs, regB + r * (a.Bf * K + K) + a.Bf * K + tid, (double)csr[tid], epB);
    }
    // the next tile goes into the other buffer now (its last reader, the previous step's B GEMM, is done)
    if (pf) {
#pragma unroll
      for (int u = 0; u < NPF; ++u) {
        const int e = tid + u * SPT;
        Xn[(e >> 6) * a.xp + (e & 63)] = xn[u];
      }
    }
    ph(5);
    // ===== B reduce-scatter: owned elements' gradients and all column sums, producer order
    const int niB = neo + K;          // items: the owned elements (at eo0), then the K column sums
    // (producer r' publishes its gradient partial at element offsets and the sums at Bf·K: the
    // owned elements are granules eo0 .. eo0 + neo − 1 of every producer block, the sums Bf·K + k)
    ok = sgld_gather(rs, regB, a.Bf * K + K, Gr, niB, epB, a.abort_flag, all,
                     [&](int p, int i, double v) { stage[p * niB + i] = v; },
                     [&](int i) { return i < neo ? eo0 + i : a.Bf * K + (i - neo); });
    if (!all_ok(ok, &sh_fail)) { failed = true; break; }
    ph(6);
    // ... the SGLD update of the owned weights (sgld.py:37-38 with softmax.py:57-58), published
    const int regW = a.oXW + par * XW_n + (f * Gr) * a.Eo;
    const unsigned epW = epA + 3;
    for (int i = tid; i < neo; i += SPT) {
      const int e = eo0 + i, fe = e / K, k = e - (e / K) * K;
      double g = stage[i];
      for (int p = 1; p < Gr; ++p) g += stage[p * niB + i];
      const T w = Ws[fe * a.wp + k];
      const T gr = -((T)g - a.alpha * w);
      const T z = sgld_noise(a, sc.noff, step_id, (uint32_t)((dlo + fe) * K + k));
      T pm = noise_scale * z;
      pm = pm + m_half_eps * gr;
      const T wn = w + pm;
      put(rs, regW + r * a.Eo + i, (double)wn, epW);
      stage[i] = (double)wn;                                              // own values, for Ws below
    }
    // bias: identical in every workgroup (softmax.py:55,59-60; noise element D·K + k)
    T bnew = T(0);
    if (tid < K) {
      double c = stage[neo + tid];
      for (int p = 1; p < Gr; ++p) c += stage[p * niB + neo + tid];
      const T bb = bs[tid];
      const T gr = -((T)c - a.alpha * bb);
      const T z = sgld_noise(a, sc.noff, step_id, (uint32_t)(a.D * K + tid));
      T pm = noise_scale * z;
      pm = pm + m_half_eps * gr;
      bnew = bb + pm;
    }
    __syncthreads();                                                      // stage reads done
    // ===== BAG: every owner's new weights → the whole slice in Ws
    for (int i = tid; i < neo; i += SPT) {
      const int e = eo0 + i, fe = e / K, k = e - (e / K) * K;
      Ws[fe * a.wp + k] = (T)stage[i];
    }
    if (tid < K) bs[tid] = bnew;
    ok = sgld_gather(rs, regW, a.Eo, Gr, a.Eo, epW, a.abort_flag,
                     [&](int p, int i) { return p != r && p * a.Eo + i < nE; },
                     [&](int p, int i, double v) {
                       const int e = p * a.Eo + i;
                       Ws[(e / K) * a.wp + (e - (e / K) * K)] = (T)v;
                     });
    if (!all_ok(ok, &sh_fail)) { failed = true; break; }
    ph(7);

    // ===== logging (sgmcmc.py:60-62): log-likelihood of the new state on this step's minibatch
    if (sc.want_ll) {
      const unsigned epL = epA + 4;
      const int regL = a.oXA + par * XA_n + (r * Gf) * a.Br * K;       // round A's region, new epoch
      sgld_phase_a<T>(a, Xs, Ws, rs, regL + f * a.Br * K, nrow, nfeat, epL);
      ok = sgld_gather(rs, regL + ro0 * K, a.Br * K, Gf, niA, epL, a.abort_flag, all,
                       [&](int p, int i, double v) { stage[p * niA + i] = v; });
      if (!all_ok(ok, &sh_fail)) { failed = true; break; }
      double llsum = 0.0;
      for (int rr = wave; rr < nro; rr += 4) {
        const int k = lane, kc = min(k, K - 1);
        const bool kv = k < K;
        double zs = stage[rr * K + kc];
        for (int p = 1; p < Gf; ++p) zs += stage[p * niA + rr * K + kc];
        const T yk = a.Y[((size_t)sc.row0 + rlo + ro0 + rr) * K + kc];
        const T zz = kv ? clipz((T)zs + bs[kc], a.clip_hi, a.clip_lo) : (T)-__builtin_inf();
        const T mx = wave_max_t(zz);
        const T ex = kv ? exp(zz - mx) : T(0);
        const T lse = log(wave_sum_t(ex)) + mx;                                           // softmax.py:18-20
        double t = kv ? (double)(yk * (zz - lse)) : 0.0;
        llsum += wave_sum_t(t);
      }
      if (lane == 0) llw[wave] = llsum;
      __syncthreads();
      const int regLL = a.oXL + par * G;
      if (tid == 0) put(rs, regLL + bid, ((llw[0] + llw[1]) + llw[2]) + llw[3], epA + 5);
      if (bid == 0) {                                                     // Σ over the workgroups, in order
        ok = sgld_gather(rs, regLL, 1, G, 1, epA + 5, a.abort_flag, all, [&](int p, int, double v) { stage[p] = v; });
        if (!all_ok(ok, &sh_fail)) { failed = true; break; }
        if (tid == 0) {
          double t = stage[0];
          for (int p = 1; p < G; ++p) t += stage[p];
          a.out_ll[s] = t;
        }
      }
      __syncthreads();
    }
  }
  if (a.prof && tid == 0)
    for (int i = 0; i < 8; ++i) a.prof[bid * 8 + i] = pacc[i];
  if (failed) return;
  // ---- the call's final state (untouched if any workgroup timed out: the abort word is raised
  // before a member leaves, and no member can pass the last round without every member's data)
  __syncthreads();
  if (__hip_atomic_load(a.abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  for (int i = tid; i < neo; i += SPT) {
    const int e = eo0 + i, fe = e / K, k = e - (e / K) * K;
    a.W[(size_t)(dlo + fe) * K + k] = Ws[fe * a.wp + k];
  }
  if (bid == 0 && tid < K) a.b[tid] = bs[tid];
}

// ---------------------------------------------------------------- host
struct SgldPPlan { int Gr, Gf, Br, Bf, Ro, Eo, KP, lds; };

static bool sgld_p_plan(int B, int D, int K, int elt, SgldPPlan* p) {
  if (K < 1 || K > 64 || B < 1 || D < 1) return false;
  p->KP = (K + 15) / 16 * 16;
  p->Gr = (B + SPB - 1) / SPB;
  p->Gf = (D + SPB - 1) / SPB;
  if (p->Gr * p->Gf > 256) return false;
  p->Br = (B + p->Gr - 1) / p->Gr;
  p->Bf = (D + p->Gf - 1) / p->Gf;
  p->Ro = (p->Br + p->Gf - 1) / p->Gf;
  p->Eo = (p->Bf * K + p->Gr - 1) / p->Gr;
  const int xp = SPB + (elt == 8 ? 2 : 1), wp = p->KP + (elt == 8 ? 2 : 1), dp = wp;
  const int nstage = std::max(p->Gf * p->Ro * K, p->Gr * (p->Eo + K));
  p->lds = (2 * SPB * xp + SPB * wp + SPB * dp) * elt + nstage * 8 + 128 * elt + 4 * 8 + 64;
  return p->lds <= 160 * 1024;
}

bool sgld_p_eligible(hmcx_ctx* ctx, const hmcx_sampler_args* s) {
  const char* env = getenv("HMCX_SGLD_WIDE");
  if (env && env[0] != '2' && env[0] != 'p') return false;     // 0: kernel-per-phase, 1: three launches
  if (s->C != 1 || s->pW || s->pb) return false;                // CPU semantics, one chain
  SgldPPlan pl;
  if (!sgld_p_plan(s->B, s->D, s->K, s->dtype == HMCX_F64 ? 8 : 4, &pl)) return false;
  // opt-in only (HMCX_SGLD_WIDE=2): at config 5 it measured 34.4 µs per step against 28.7 for the
  // three-launch path (tools/gpu_r03_sgld.sh) — its granule traffic (≈ 230 KB per workgroup per step in
  // the four rounds, HMCX_SGLD_PROF) is bandwidth-bound at these partial sizes
  if (!(env && (env[0] == '2' || env[0] == 'p'))) return false;
  int per_cu = 0;
  const void* kfn = s->dtype == HMCX_F64 ? (const void*)k_sgld_p<double> : (const void*)k_sgld_p<float>;
  if (kernel_occupancy(ctx, kfn, SPT, pl.lds, &per_cu)) return false;
  return (long)per_cu * ctx->num_cus >= (long)pl.Gr * pl.Gf;
}

template <typename T>
int sgld_p_t(hmcx_ctx* ctx, const hmcx_sampler_args* s, bool* aborted) {
  *aborted = false;
  SgldPPlan pl;
  if (!sgld_p_plan(s->B, s->D, s->K, sizeof(T), &pl)) return set_error(ctx, HMCX_EUNSUPPORTED, "sgld_p: shape");
  const int K = s->K, G = pl.Gr * pl.Gf, n = s->n_steps;
  // arena regions (granules), each [2] by step parity
  const int XA_n = G * pl.Br * K, XD_n = G * pl.Ro * K, XB_n = G * (pl.Bf * K + K), XW_n = G * pl.Eo, XL_n = G;
  SgldPArgs<T> a{};
  a.oXA = 0; a.oXD = a.oXA + 2 * XA_n; a.oXB = a.oXD + 2 * XD_n; a.oXW = a.oXB + 2 * XB_n; a.oXL = a.oXW + 2 * XW_n;
  const size_t gran = (size_t)a.oXL + 2 * XL_n;
  if (gran * 16 > 0x7fffffffull) return set_error(ctx, HMCX_EUNSUPPORTED, "sgld_p: arena");
  if (int rc = gx_reserve(ctx, gran * 16)) return rc;
  if (!ctx->sgld_abort_dev) {
    HMCX_HIP(ctx, hipMalloc((void**)&ctx->sgld_abort_dev, sizeof(int)));
    HMCX_HIP(ctx, hipMemsetAsync(ctx->sgld_abort_dev, 0, sizeof(int), ctx->stream));
  }
  unsigned ep0 = 1;
  if (int rc = gx_epochs(ctx, 8u * (unsigned)n + 8u, &ep0)) return rc;
  Workspace ws(ctx);
  SgldSched* sched;
  double* ll_scratch;
  do {
    ws.reset();
    sched = ws.take<SgldSched>(n);
    ll_scratch = ws.take<double>(n);
  } while (ws.retry());
  if (ws.failed) return HMCX_ENOMEM;
  std::vector<SgldSched> h(n);
  for (int i = 0; i < n; ++i) {
    h[i].eps = s->eps[i];
    h[i].row0 = s->row0[i];
    h[i].noff = s->noise_mode == HMCX_NOISE_BUFFER ? s->noise_off[i] : 0;
    h[i].want_ll = (s->want_ll && s->want_ll[i] && s->out_ll) ? 1 : 0;
    h[i].pad_ = 0;
  }
  begin_call(ctx);
  if (int rc = upload(ctx, sched, h.data(), sizeof(SgldSched) * n)) return rc;
  a.B = s->B; a.D = s->D; a.K = K; a.KP = pl.KP; a.Gr = pl.Gr; a.Gf = pl.Gf; a.Br = pl.Br; a.Bf = pl.Bf;
  a.Ro = pl.Ro; a.Eo = pl.Eo; a.n_steps = n;
  a.alpha = (T)s->alpha; a.clip_hi = (T)CLIP_HI; a.clip_lo = (T)CLIP_LO;
  a.X = (const T*)s->X; a.Y = (const T*)s->Y; a.W = (T*)s->W; a.b = (T*)s->b;
  a.sched = sched;
  a.noise_mode = s->noise_mode; a.noise = s->noise; a.seed = s->seed; a.chain = s->chain0; a.step_base = s->step_base;
  a.arena = ctx->gx_arena; a.arena_bytes = (int)ctx->gx_bytes;
  a.ep0 = ep0;
  a.abort_flag = ctx->sgld_abort_dev;
  a.force_abort = getenv("HMCX_SGLD_FORCE_ABORT") && getenv("HMCX_SGLD_FORCE_ABORT")[0] == '1';
  static const char* prof_path = getenv("HMCX_SGLD_PROF");
  unsigned long long* prof_dev = nullptr;
  if (prof_path) {
    HMCX_HIP(ctx, hipMalloc((void**)&prof_dev, (size_t)G * 8 * sizeof(unsigned long long)));
    HMCX_HIP(ctx, hipMemsetAsync(prof_dev, 0, (size_t)G * 8 * sizeof(unsigned long long), ctx->stream));
  }
  a.prof = prof_dev;
  a.out_ll = s->out_ll ? s->out_ll : ll_scratch;
  a.xp = SPB + (sizeof(T) == 8 ? 2 : 1); a.wp = pl.KP + (sizeof(T) == 8 ? 2 : 1); a.dp = a.wp;
  int per_cu = 0;
  if (int rc = kernel_occupancy(ctx, (const void*)k_sgld_p<T>, SPT, pl.lds, &per_cu)) return rc;
  if ((long)per_cu * ctx->num_cus < G) return set_error(ctx, HMCX_EUNSUPPORTED, "sgld_p: grid not co-resident");
  if (int rc = timing_begin(ctx, ctx->stream)) return rc;
  hipLaunchKernelGGL(k_sgld_p<T>, dim3(G), dim3(SPT), pl.lds, ctx->stream, a);
  HMCX_HIP(ctx, hipGetLastError());
  if (int rc = timing_end(ctx, ctx->stream)) return rc;
  // verdict of the call: a timed-out hand-off leaves W / b untouched; the caller re-runs the call
  int flag = 0;
  HMCX_HIP(ctx, hipMemcpyAsync(&flag, ctx->sgld_abort_dev, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  HMCX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (flag) {
    HMCX_HIP(ctx, hipMemsetAsync(ctx->sgld_abort_dev, 0, sizeof(int), ctx->stream));
    *aborted = true;
  }
  if (prof_dev) {                                  // per step: median / max over workgroups, per phase
    std::vector<unsigned long long> hp((size_t)G * 8);
    HMCX_HIP(ctx, hipMemcpy(hp.data(), prof_dev, hp.size() * 8, hipMemcpyDeviceToHost));
    (void)hipFree(prof_dev);
    if (FILE* fo = fopen(prof_path, "a")) {
      static const char* nm[8] = {"step-start", "A gemm+publish", "A-RS", "softmax", "AG", "B gemm+publish", "B-RS",
                                  "update+BAG"};
      fprintf(fo, "sgld_p G=%d steps=%d (us per step)\n", G, n);
      for (int i = 0; i < 8; ++i) {
        std::vector<double> v(G);
        for (int g = 0; g < G; ++g) v[g] = hp[(size_t)g * 8 + i] / 100.0 / n;
        std::sort(v.begin(), v.end());
        fprintf(fo, "  %-16s median %.2f max %.2f\n", nm[i], v[G / 2], v[G - 1]);
      }
      fclose(fo);
    }
  }
  return HMCX_OK;
}

template int sgld_p_t<float>(hmcx_ctx*, const hmcx_sampler_args*, bool*);
template int sgld_p_t<double>(hmcx_ctx*, const hmcx_sampler_args*, bool*);

}  // namespace hmcx
