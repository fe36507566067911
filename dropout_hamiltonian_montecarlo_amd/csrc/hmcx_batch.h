// hmcx_batch.h — chain-batched SGHMC leapfrog GEMMs: C chains sharing one minibatch (C >= 16, K = 10).
//
// Same arithmetic as k_fwd / k_grad (hmcx_softmax.hip; reference cpu/sghmc.py:28-34 and
// cpu/softmax.py:38-61), re-tiled for the chain-batched gradient GEMMs of SURVEY §8d,
// [B×D]·[D×10C] and [D×B]·[B×10C]:
//
//  * k_bfwd: tile = 32 minibatch rows × 16 chains (160 columns); the D loop is staged through LDS in
//    32-deep chunks (register prefetch of the next chunk), 4 waves × (16 rows × 80 columns) of
//    v_mfma_*_16x16x4.  Epilogue per (row, chain): both softmaxes (at b and b' = b + ε·pb), diff,
//    bias colsum partial, log-likelihood partial.
//  * k_bgrad: tile = 32 features × 16 chains; the minibatch loop staged the same way; the friction
//    noise of the tile is generated into LDS before the loop (one Philox block per 4 elements), the
//    SGHMC update (gradient, momentum, drift, kinetic partial) runs on the accumulators in registers;
//    workgroups of feature tile 0 finish the bias sub-step.
//  * Active-chain compaction: per step the host orders chains by path length (descending); at
//    leapfrog iteration `it` only ranks < c_act(it) are launched, so the work is proportional to the
//    leapfrog count, not to max_c L_c.
#pragma once
#include "hmcx_common.h"
#include "hmcx_internal.h"

namespace hmcx {

constexpr int BCT = 16;           // chains per tile
constexpr int BKC = 10;           // classes (compiled for K = 10)
constexpr int BNT = BCT * BKC;    // 160 columns per tile
constexpr int BRW = 32;           // rows (k_bfwd) / features (k_bgrad) per tile
constexpr int BCH = 32;           // depth of one staged k-chunk
// LDS pitches chosen for conflict-free operand reads (bank = dword address mod 64 for ds_read_b64,
// mod 32 for ds_read_b32; lanes 0-15 and 16-31 of a half-wave must hit disjoint banks):
//  * k_bfwd X chunk [row][k], read down a column (16 rows × 2 k): pitch ≡ 2 (mod 32) elements;
//  * row-contiguous reads (W / diff chunk, k_bgrad X chunks; 16 elements × 2 rows): pitch ≡ 16 (mod 32).
constexpr int BXP = BCH + 2;      // 34: k_bfwd X chunk
constexpr int BXPG = 48;          // k_bgrad X chunk [row][32 features]
constexpr int BWP = BNT + 16;     // 176: W / diff chunk [k][160 columns]
// k_bfwd's epilogue tile Zt (in the W chunk's LDS): thread (row il, chain cs) reads its chain's 10
// classes as five ds_read_b128 at 20·cs dwords into row il.  A ds_read_b128 lane group mixes rows il and
// il + 1 ({0-3, 12-15} of one row with {20-27} of the next, and so on), and the 16-byte starts 20·cs of one
// row and 20·cs' + pitch of the next never share banks when the pitch is ≡ 0 (mod 64) dwords: 160
// doubles.  (The chunk pitch 176, ≡ 32 dwords, put every chunk of the next row on a busy bank.)
constexpr int ZTP = BNT;          // 160
// Row pitch of the p² partials [row][BNP] (doubles, written by 16-lane rows: any pitch is conflict-free).
constexpr int BNP = BNT + 4;      // 164
// Row pitch of the friction-noise tile Nz, read in the MFMA fragment layout (hmcx_common.h): the lane
// groups lg = 0 / 1 of a half-wave read rows 4 apart in f32 (row = 4·lg + q; ds_read_b32, banks mod 32:
// pitch ≡ 4 (mod 8) puts them 16 banks apart) but ADJACENT rows in f64 (row = lg + 4·q; ds_read_b64,
// banks mod 64: pitch ≡ 16 (mod 32) puts them 32 banks apart — the round-4 pitch 164 overlapped 24 of the
// 32 banks, the k_bgradw bank conflicts of profiles/pmc_r04_batched_sq.json)
template <typename T> constexpr int bnz() { return sizeof(T) == 8 ? BNT + 16 : BNT + 4; }

// XCD-grouped tile order: the 1-D grid holds 8·nX·ceil(nCT/8) blocks; blocks b, b+8, b+16, ... share
// one XCD (round-robin dispatch), so every x tile of chain tile ct lands on XCD ct mod 8 and the
// chain tile's operand slice (W columns / diff columns) is fetched into that XCD's L2 once.
// Placement is a speed assumption only; any placement gives the same results.
__device__ inline bool xcd_tile(int nX, int nCT, int& bx, int& by) {
  const int L = blockIdx.x, x = L & 7, s = L >> 3;
  by = x + 8 * (s / nX);
  bx = s - (s / nX) * nX;
  return by < nCT;
}
inline unsigned xcd_grid(int nX, int nCT) { return 8u * (unsigned)nX * (unsigned)((nCT + 7) / 8); }
// Same grid and XCD grouping, with every tile of the last x tile (a partial feature tile, cheap once
// its empty m-tiles skip the MFMA loop) dispatched after all full tiles: the full tiles fill whole
// rounds of the chip's workgroup slots and the partial ones run as a short final round, instead of
// being spread through the rounds and leaving the last round a quarter full of full-cost tiles.
__device__ inline bool xcd_tile_tail_last(int nX, int nCT, int& bx, int& by) {
  const int L = blockIdx.x, x = L & 7, s = L >> 3, ng = (nCT + 7) / 8, nXm = nX - 1;
  if (s < nXm * ng) {
    by = x + 8 * (s / nXm);
    bx = s - (s / nXm) * nXm;
  } else {
    by = x + 8 * (s - nXm * ng);
    bx = nXm;
  }
  return by < nCT;
}

template <typename T> struct BFwdArgs {
  const T* X; const T* Y;           // minibatch rows (offset to the step's first row)
  const T* W; const T* b; const T* pb;
  int B, D, C, N, mode, iter, c_act;
  T eps;
  const int32_t* n_iter;            // [C] of this step
  const int32_t* perm;              // [C] chain of each rank (path length descending)
  T* diff;                          // [B][N]
  int nX, nCT;                      // row tiles × chain tiles (XCD-grouped 1-D grid, xcd_tile)
  T* colsum_part;                   // [nRB][N]
  double* ll_part;                  // [nRB][C]
  int nRB_all;                      // partial blocks of the call: the last row tile zero-fills those past its own
};

template <typename T> struct BGradArgs {
  const T* X; const T* diff; const T* colsum_part;
  int B, D, C, N, nRB, iter, c_act, P;
  T alpha, eps, one_minus_eps, noise_scale;
  const int32_t* n_iter; const int32_t* perm;
  T* W; T* b; T* pW; T* pb;
  double* kin_part;                 // [nDB][C]
  int nDB_all;                      // k_bgrad2: kin_part rows past its grid are zero-filled up to here
  int nX, nCT;                      // feature tiles × chain tiles (XCD-grouped 1-D grid, xcd_tile)
  int tail_last;                    // k_bgradw: partial last feature tile dispatched last (xcd_tile_tail_last)
  double* kinb;                     // [C]
  int noise_mode; const double* noise; const int64_t* noff;
  uint64_t seed; uint32_t chain0, step, slot;
};

// Staging map of one 32-deep chunk: X part [32][32] as 512 two-element vectors (thread: 2), W/diff
// part [32][16 chains × 10] as 2560 vectors (thread: 10); vector j of the W part covers row
// j / 80, chain slot (j % 80) / 5, classes 2·(j % 5) .. +1, so 5 consecutive lanes read one chain's
// contiguous 10-value row segment.
template <typename T, int XM = 1> struct StageMap {
  typedef T v2 __attribute__((ext_vector_type(2)));
  int xr[2 * XM], xc[2 * XM];
  int wr[10], wcol[10], wls[10];
  bool wok[10];
  __device__ StageMap(int tid, const int* chs) {
#pragma unroll
    for (int u = 0; u < 2 * XM; ++u) {
      const int j = tid + 256 * u;
      xr[u] = j >> 4;
      xc[u] = (j & 15) * 2;
    }
#pragma unroll
    for (int u = 0; u < 10; ++u) {
      const int j = tid + 256 * u;
      const int row = j / 80, rem = j - row * 80, cs = rem / 5, pp = rem - cs * 5;
      const int ch = chs[cs];
      wr[u] = row;
      wok[u] = ch >= 0;
      wcol[u] = (ch >= 0 ? ch : 0) * BKC + 2 * pp;
      wls[u] = cs * BKC + 2 * pp;
    }
  }
};
// two consecutive elements (zero when !ok; only the first when avail == 1)
template <typename T>
__device__ inline typename StageMap<T>::v2 ld2(const T* p, bool ok, int avail) {
  typename StageMap<T>::v2 v = {T(0), T(0)};
  if (ok && avail >= 2) {
    v = *reinterpret_cast<const typename StageMap<T>::v2*>(p);
  } else if (ok && avail == 1) {
    v[0] = p[0];
  }
  return v;
}
template <typename T> __device__ inline void st2(T* p, typename StageMap<T>::v2 v) { p[0] = v[0]; p[1] = v[1]; }

// Staging map of a chain-major [chain][row][10] operand chunk (32 rows × 16 chain slots × 10 classes =
// 2560 two-element vectors, 10 per thread): vector j covers row j / 80, chain slot (j % 80) / 5,
// classes 2·(j % 5) .. +1, so 5 lanes read one chain's 80-B row and consecutive lanes write
// consecutive LDS addresses of one row (a lane order walking one chain's rows instead would put
// 3-4 rows on the same banks of every ds_write: the LDS row pitch is ≡ 0 (mod 32) dwords for the
// conflict-free MFMA operand reads).  Source element: base + wsrc + (r0 + wr)·10; LDS
// destination: row wr, column wls (slot·10 + class).
struct StageCM {
  int wr[10], wls[10];
  size_t wsrc[10];
  bool wok[10];
  __device__ StageCM(int tid, const int* chs, size_t stride) {
#pragma unroll
    for (int u = 0; u < 10; ++u) {
      const int j = tid + 256 * u;
      const int row = j / 80, rem = j - row * 80, cs = rem / 5, k2 = (rem - cs * 5) * 2, ch = chs[cs];
      wr[u] = row;
      wok[u] = ch >= 0;
      wsrc[u] = (size_t)(ch >= 0 ? ch : 0) * stride + k2;
      wls[u] = cs * BKC + k2;
    }
  }
};

// MT = m-tiles per wave: the tile is 32·MT minibatch rows × 16 chains (MT = 2 halves the W
// staging per MFMA; used when enough chains are active to fill the chip).
// CM: W is the chain-major working copy [C][D][10] (else the caller's [D][C·10]); diff is written
// chain-major [C][B][10].
// NWV = 8 (MT = 2 only): the same 64-row tile and partial layout with 8 waves, one m-tile each — for
// launches too small to give every CU two workgroups (the compaction tail), where one 4-wave
// workgroup per CU leaves the MFMA latency exposed.  Waves 0-3 stage the chunks.
template <typename T, int MT, int CM, int NWV = 4>
__global__ __launch_bounds__(64 * NWV) void k_bfwd(BFwdArgs<T> a) {
  using M = mfma16<T>;
  constexpr int ROWS = 32 * MT;
  constexpr int NTH = 64 * NWV;
  constexpr int MW = NWV == 8 ? MT / 2 : MT;          // m-tiles per wave
  // partials are laid out per 32-row block whatever the tile height (every launch of a call may pick
  // its own): a 64-row tile writes its sums into block 2·bx and zeros into 2·bx + 1
  constexpr int PREP = MT;
  static_assert(NWV == 4 || (NWV == 8 && MT == 2), "k_bfwd: 8 waves need 64-row tiles");
  __shared__ T Xs[ROWS * BXP];
  __shared__ T Ws[BCH * BWP];          // also the epilogue tile, 32 rows at a time
  __shared__ double Lt[ROWS][BCT];
  __shared__ int chs[BCT];
  // epilogue operands loaded with the first chunk (their latency hidden by the main loop, not paid
  // per row pair in the epilogue): the tile's labels, the chains' b / pb, the path-end flags
  __shared__ T Ysh[ROWS * BKC];
  __shared__ T bsh[BNT], pbsh[BNT];
  __shared__ int lastsh[BCT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  int bx, by;
  if (!xcd_tile(a.nX, a.nCT, bx, by)) return;
  const int m0 = bx * ROWS, rank0 = by * BCT;
  const int nrow = min(ROWS, a.B - m0);
  const int D = a.D, N = a.N;
  if (tid < BCT) chs[tid] = rank0 + tid < a.c_act ? a.perm[rank0 + tid] : -1;
  __syncthreads();

  // staging: 2-element vectors; X chunk [ROWS][32 d] (2·MT per thread), W chunk
  // [32 d][16 chains × 10] = 2560 vectors (10 per thread, consecutive lanes walk one chain's row)
  StageMap<T, MT> sm(tid, chs);
  const StageCM scm(tid, chs, (size_t)a.D * BKC);
  const T* xsrc[2 * MT];
#pragma unroll
  for (int u = 0; u < 2 * MT; ++u) xsrc[u] = a.X + (size_t)(m0 + min(sm.xr[u], nrow - 1)) * D + sm.xc[u];
  typename StageMap<T>::v2 xv[2 * MT], wv[10];
  const bool stager = NWV == 4 || tid < 256;         // wave-uniform
  auto fetch = [&](int k0) {
    if (!stager) return;
#pragma unroll
    for (int u = 0; u < 2 * MT; ++u) xv[u] = ld2<T>(xsrc[u] + k0, sm.xr[u] < nrow, D - k0 - sm.xc[u]);
#pragma unroll
    for (int u = 0; u < 10; ++u) {
      if constexpr (CM) {
        const int d = k0 + scm.wr[u];
        wv[u] = ld2<T>(a.W + scm.wsrc[u] + (size_t)min(d, D - 1) * BKC, scm.wok[u] && d < D, 2);
      } else {
        const int d = k0 + sm.wr[u];
        wv[u] = ld2<T>(a.W + (size_t)min(d, D - 1) * N + sm.wcol[u], sm.wok[u] && d < D, 2);
      }
    }
  };
  auto stash = [&]() {
    if (!stager) return;
#pragma unroll
    for (int u = 0; u < 2 * MT; ++u) st2<T>(Xs + sm.xr[u] * BXP + sm.xc[u], xv[u]);
#pragma unroll
    for (int u = 0; u < 10; ++u) {
      if constexpr (CM) st2<T>(Ws + scm.wr[u] * BWP + scm.wls[u], wv[u]);
      else st2<T>(Ws + sm.wr[u] * BWP + sm.wls[u], wv[u]);
    }
  };

  // rows [16·(wm·MW + i)], 5 n-tiles per wave
  const int wm = NWV == 8 ? (wave & 3) : (wave & 1), nh = NWV == 8 ? (wave >> 2) : (wave >> 1);
  typename M::acc_t acc[MW][5];
#pragma unroll
  for (int i = 0; i < MW; ++i)
#pragma unroll
    for (int j = 0; j < 5; ++j) acc[i][j] = M::zero();
  fetch(0);
  if (stager) {
    const bool sg = a.mode == FWD_SGHMC;
    constexpr int NYV = (ROWS * BKC + 255) / 256;
    T yv[NYV];
#pragma unroll
    for (int u = 0; u < NYV; ++u) {
      const int t = min(tid + 256 * u, ROWS * BKC - 1), r = t / BKC;
      yv[u] = a.Y[(size_t)(m0 + min(r, nrow - 1)) * BKC + (t - r * BKC)];
    }
    const int tb = min(tid, BNT - 1), cs = tb / BKC, ch = chs[cs];
    const size_t bi = (size_t)(ch >= 0 ? ch : 0) * BKC + (tb - cs * BKC);
    const T bv0 = a.b[bi], pbv0 = sg ? a.pb[bi] : T(0);
    const int cl = chs[tid & (BCT - 1)];
    const int nt = a.n_iter[cl >= 0 ? cl : 0];
#pragma unroll
    for (int u = 0; u < NYV; ++u)
      if (tid + 256 * u < ROWS * BKC) Ysh[tid + 256 * u] = yv[u];
    if (tid < BNT) { bsh[tid] = bv0; pbsh[tid] = pbv0; }
    if (tid < BCT) lastsh[tid] = sg && cl >= 0 && a.iter == nt - 1;
  }
  for (int k0 = 0; k0 < D; k0 += BCH) {
    __syncthreads();
    stash();
    __syncthreads();
    if (k0 + BCH < D) fetch(k0 + BCH);                 // next chunk in flight during the MFMAs
    const int nks = min(BCH, D - k0 + 3) / 4;
#pragma unroll 2
    for (int ks = 0; ks < nks; ++ks) {
      T av[MW], bv[5];
#pragma unroll
      for (int i = 0; i < MW; ++i) av[i] = Xs[((wm * MW + i) * 16 + lr) * BXP + ks * 4 + lg];
#pragma unroll
      for (int j = 0; j < 5; ++j) bv[j] = Ws[(ks * 4 + lg) * BWP + (nh * 5 + j) * 16 + lr];
#pragma unroll
      for (int i = 0; i < MW; ++i)
#pragma unroll
        for (int j = 0; j < 5; ++j) acc[i][j] = M::fma(av[i], bv[j], acc[i][j]);
    }
  }

  // ---- epilogue, 32 rows at a time through Zt: softmax.py:32-36 (clip, max, exp, normalise), :52
  const T hi = (T)CLIP_HI, lo = (T)CLIP_LO;
  const bool sghmc = a.mode == FWD_SGHMC;
  static_assert(32 * ZTP <= BCH * BWP, "k_bfwd: the epilogue tile must fit the W chunk's LDS");
  T* Zt = Ws;                                          // [32][ZTP] logits, then y − ŷ'
  T cs_acc = T(0);                                     // thread t < 160: Σ_rows (y − ŷ') of column t
  for (int half = 0; half < MT; ++half) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MW; ++i) {
      // wave rows of m-tile (wm·MW + i) fall in half (wm·MW + i) / 2
      const int mtile = wm * MW + i;
      if ((mtile >> 1) != half) continue;
#pragma unroll
      for (int j = 0; j < 5; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          Zt[((mtile & 1) * 16 + M::row(lane, q)) * ZTP + (nh * 5 + j) * 16 + lr] = acc[i][j][q];
    }
    __syncthreads();
    for (int pr = tid; pr < 32 * BCT; pr += NTH) {
      const int il = pr >> 4, cs = pr & 15, ch = chs[cs];
      const int i = half * 32 + il;
      if (ch < 0 || i >= nrow) { Lt[i][cs] = 0.0; continue; }
      const bool last = lastsh[cs];
      T z[BKC], y[BKC];
#pragma unroll
      for (int k = 0; k < BKC; ++k) {
        z[k] = Zt[il * ZTP + cs * BKC + k];
        y[k] = Ysh[i * BKC + k];
      }
      // variant 1: bias b (weights sub-step diff / LL mode)
      T zc[BKC], m = T(0), s = T(0);
#pragma unroll
      for (int k = 0; k < BKC; ++k) {
        zc[k] = clipz(z[k] + bsh[cs * BKC + k], hi, lo);
        m = k == 0 ? zc[0] : max_nan(m, zc[k]);
      }
      T e[BKC];
#pragma unroll
      for (int k = 0; k < BKC; ++k) { e[k] = exp(zc[k] - m); s += e[k]; }
      if (!sghmc) {
        const T lse = log(s) + m;
        double ll = 0.0;
#pragma unroll
        for (int k = 0; k < BKC; ++k) ll += (double)(y[k] * (zc[k] - lse));
        Lt[i][cs] = ll;
        continue;
      }
      T* drow = a.diff + ((size_t)ch * a.B + (m0 + i)) * BKC;
#pragma unroll
      for (int k = 0; k < BKC; ++k) drow[k] = y[k] - e[k] / s;
      // variant 2: bias b' = b + ε·pb (bias sub-step, sghmc.py:32 on the bias)
      T m2 = T(0), s2 = T(0);
#pragma unroll
      for (int k = 0; k < BKC; ++k) {
        const T bp = bsh[cs * BKC + k] + a.eps * pbsh[cs * BKC + k];
        zc[k] = clipz(z[k] + bp, hi, lo);
        m2 = k == 0 ? zc[0] : max_nan(m2, zc[k]);
      }
#pragma unroll
      for (int k = 0; k < BKC; ++k) { e[k] = exp(zc[k] - m2); s2 += e[k]; }
#pragma unroll
      for (int k = 0; k < BKC; ++k) Zt[il * ZTP + cs * BKC + k] = y[k] - e[k] / s2;
      double ll = 0.0;
      if (last) {
        const T lse = log(s2) + m2;
#pragma unroll
        for (int k = 0; k < BKC; ++k) ll += (double)(y[k] * (zc[k] - lse));
      }
      Lt[i][cs] = ll;
    }
    __syncthreads();
    if (sghmc && tid < BNT) {
      const int nr = min(32, nrow - half * 32);
      for (int il = 0; il < nr; ++il) cs_acc += Zt[il * ZTP + tid];
    }
  }
  if (sghmc && tid < BNT) {                            // Σ_rows (y − ŷ') of this tile
    const int cs = tid / BKC, ch = chs[cs];
    if (ch >= 0) {
      a.colsum_part[(size_t)bx * PREP * N + ch * BKC + (tid - cs * BKC)] = cs_acc;
      const int r1 = bx == a.nX - 1 ? max(a.nRB_all, (bx + 1) * PREP) : (bx + 1) * PREP;
      for (int r = bx * PREP + 1; r < r1; ++r) a.colsum_part[(size_t)r * N + ch * BKC + (tid - cs * BKC)] = T(0);
    }
  }
  if (tid < BCT) {
    const int ch = chs[tid];
    if (ch >= 0 && (!sghmc || a.iter == a.n_iter[ch] - 1)) {
      double v = 0.0;
      for (int i = 0; i < nrow; ++i) v += Lt[i][tid];
      a.ll_part[(size_t)bx * PREP * a.C + ch] = v;
      const int r1 = bx == a.nX - 1 ? max(a.nRB_all, (bx + 1) * PREP) : (bx + 1) * PREP;
      for (int r = bx * PREP + 1; r < r1; ++r) a.ll_part[(size_t)r * a.C + ch] = 0.0;
    }
  }
}

template <typename T>
__device__ inline T bnoise(const BGradArgs<T>& a, int ch, uint32_t e) {
  if (a.noise_mode == HMCX_NOISE_BUFFER) return (T)a.noise[a.noff[ch] + (int64_t)a.slot * a.P + e];
  return philox_normal_t<T>(a.seed, a.chain0 + ch, a.step, a.slot, e);
}

// Friction noise of a feature tile into LDS: Nz[fl][cs·K + k] for the local features fl < nfl (tile
// feature fi = fmap(fl)), chain slots cs.  f64 chains: one Philox block per element pair (k, k+1)
// of one feature (K = 10 is even), double Box–Muller; f32 chains: blocks of four elements of the
// flat index e = d·K + k (they may straddle two features), float Box–Muller (hmcx_common.h).
template <typename T, typename FMap>
__device__ inline void gen_tile_noise(const BGradArgs<T>& a, const int* chs, int d0, int nfeat, T* Nz, int nfl,
                                      FMap fmap) {
  const int tid = threadIdx.x;
  if constexpr (sizeof(T) == 8) {
    // one Philox block per element pair (k, k+1); lane order: chain slot and pair fastest, so the
    // lanes of a wave write consecutive 16-byte pairs of one feature row of Nz
    constexpr int NP = BKC / 2;
    for (int t = tid; t < BCT * nfl * NP; t += blockDim.x) {
      const int fl = t / (BCT * NP), r = t - fl * (BCT * NP), cs = r / NP, kk = r - cs * NP;
      const int ch = chs[cs], fi = fmap(fl);
      if (ch < 0 || fi >= nfeat) continue;
      double z0, z1;
      philox_pair_d(a.seed, a.chain0 + ch, a.step, a.slot, (uint32_t)((d0 + fi) * NP + kk), z0, z1);
      Nz[fl * bnz<T>() + cs * BKC + 2 * kk] = z0;
      Nz[fl * bnz<T>() + cs * BKC + 2 * kk + 1] = z1;
    }
  } else {                                        // nfl == tile width, fmap = identity
    const int e0 = d0 * BKC, ne = min(nfl, nfeat) * BKC;
    const int g0 = e0 >> 2, ng = ((e0 + ne + 3) >> 2) - g0;
    for (int t = tid; t < BCT * ng; t += blockDim.x) {
      const int cs = t / ng, g = g0 + (t - cs * ng), ch = chs[cs];
      if (ch < 0) continue;
      float z4[4];
      philox_normal4(a.seed, a.chain0 + ch, a.step, a.slot, (uint32_t)g, z4);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int e = 4 * g + q - e0;
        if (e >= 0 && e < ne) Nz[(e / BKC) * bnz<T>() + cs * BKC + (e % BKC)] = z4[q];
      }
    }
  }
}

// Bias sub-step of one 16-chain tile (sghmc.py:32-34 on the bias), run by the feature-tile-0
// workgroup of k_bgrad / k_bgrad2: gradient from the colsum partials, momentum, drift, p² at the end.
template <typename T>
__device__ inline void bias_substep(const BGradArgs<T>& a, const int* chs, T* pbs) {
  const int tid = threadIdx.x, D = a.D, N = a.N;
  if (tid < BNT) {
    const int cs = tid / BKC, k = tid - cs * BKC, ch = chs[cs];
    T pb_new = T(0);
    if (ch >= 0) {
      const int col = ch * BKC + k;
      T c = T(0);
      for (int rb = 0; rb < a.nRB; ++rb) c += a.colsum_part[(size_t)rb * N + col];
      const T bb = a.b[col];
      T p = a.pb[col];
      const T bp = bb + a.eps * p;
      const T gr = -(c - a.alpha * bp);
      const T z = bnoise(a, ch, (uint32_t)(D * BKC + k));
      p = (a.one_minus_eps * p + a.eps * gr) + a.noise_scale * z;
      a.pb[col] = p;
      a.b[col] = bp;
      pb_new = p;
    }
    pbs[tid] = pb_new;
  }
  {
    __syncthreads();
    if (tid < BCT) {
      const int ch = chs[tid];
      if (ch >= 0 && a.iter == a.n_iter[ch] - 1) {
        double v = 0.0;
        for (int k = 0; k < BKC; ++k) {
          const double p = (double)pbs[tid * BKC + k];
          v += p * p;
        }
        a.kinb[ch] = v;
      }
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_bgrad(BGradArgs<T> a) {
  using M = mfma16<T>;
  constexpr int XSN = BCH * BXPG > 8 * BNP * 8 / (int)sizeof(T) ? BCH * BXPG : 8 * BNP * 8 / (int)sizeof(T);
  __shared__ __attribute__((aligned(16))) T Xs[XSN];   // [row][feature]; later the per-lane-group p² sums
  __shared__ __attribute__((aligned(16))) T Ds[BCH * BWP];   // [row][column]; later the friction noise
  __shared__ int chs[BCT];
  __shared__ T pbs[BNT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  int bx, by;
  if (!xcd_tile(a.nX, a.nCT, bx, by)) return;
  const int d0 = bx * BRW, rank0 = by * BCT;
  const int nfeat = min(BRW, a.D - d0);
  const int D = a.D, N = a.N, B = a.B;
  if (tid < BCT) chs[tid] = rank0 + tid < a.c_act ? a.perm[rank0 + tid] : -1;
  __syncthreads();

  StageMap<T> sm(tid, chs);                          // X chunk [32 rows][32 features]
  const StageCM scm(tid, chs, (size_t)B * BKC);      // diff chunk [32 rows][16 chains × 10]
  typename StageMap<T>::v2 xv[2], dv[10];
  auto fetch = [&](int r0) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = r0 + sm.xr[u];
      xv[u] = ld2<T>(a.X + (size_t)min(r, B - 1) * D + d0 + sm.xc[u], r < B, nfeat - sm.xc[u]);
    }
#pragma unroll
    for (int u = 0; u < 10; ++u) {
      const int r = r0 + scm.wr[u];
      dv[u] = ld2<T>(a.diff + scm.wsrc[u] + (size_t)min(r, B - 1) * BKC, scm.wok[u] && r < B, 2);
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int u = 0; u < 2; ++u) st2<T>(Xs + sm.xr[u] * BXPG + sm.xc[u], xv[u]);
#pragma unroll
    for (int u = 0; u < 10; ++u) st2<T>(Ds + scm.wr[u] * BWP + scm.wls[u], dv[u]);
  };

  const int mt = wave & 1, nh = wave >> 1;
  typename M::acc_t acc[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) acc[j] = M::zero();
  fetch(0);
  for (int r0 = 0; r0 < B; r0 += BCH) {
    __syncthreads();
    stash();
    __syncthreads();
    if (r0 + BCH < B) fetch(r0 + BCH);
    const int nks = min(BCH, B - r0 + 3) / 4;
#pragma unroll 2
    for (int ks = 0; ks < nks; ++ks) {
      const T av = Xs[(ks * 4 + lg) * BXPG + mt * 16 + lr];         // A(feature, row) = X[row][feature]
      T bv[5];
#pragma unroll
      for (int j = 0; j < 5; ++j) bv[j] = Ds[(ks * 4 + lg) * BWP + (nh * 5 + j) * 16 + lr];
#pragma unroll
      for (int j = 0; j < 5; ++j) acc[j] = M::fma(av, bv[j], acc[j]);
    }
  }
  __syncthreads();
  // friction noise of the tile into the diff chunk's space ([32 features][bnz], T)
  static_assert(BRW * bnz<T>() <= BCH * BWP, "k_bgrad: the noise tile must fit the diff chunk's LDS");
  T* Nz = Ds;
  if (a.noise_mode != HMCX_NOISE_BUFFER) {
    gen_tile_noise(a, chs, d0, nfeat, Nz, BRW, [](int fl) { return fl; });
    __syncthreads();
  }

  // ---- epilogue on the accumulators: softmax.py:57-58 gradient, sghmc.py:31,34 momentum, :32 drift
  double* kp = reinterpret_cast<double*>(Xs);        // [mt·4 + lg][160] Σ p² over the lane's rows
  T* __restrict__ Wg = a.W;                          // all 20 W / pW loads first (no aliasing), then
  T* __restrict__ Pg = a.pW;                         // the updates: one HBM round trip per thread
  // every load unconditional (clamped address, value selected afterwards) and the noise source chosen
  // per launch outside the element loops (see k_bgradw)
  const bool buf = a.noise_mode == HMCX_NOISE_BUFFER;
  T wv[5][4], pv[5][4];
  int lastm = 0;
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const int col = (nh * 5 + j) * 16 + lr;
    const int cs = col / BKC, k = col - cs * BKC, ch = chs[cs];
    const int n = a.n_iter[ch >= 0 ? ch : 0];
    lastm |= (ch >= 0 && a.iter >= n - 1) << j;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int fi = mt * 16 + M::row(lane, q);
      const bool ok = ch >= 0 && fi < nfeat;
      const size_t idx = ok ? ((size_t)ch * D + (d0 + fi)) * BKC + k : 0;
      const T w = Wg[idx], pw = Pg[idx];
      wv[j][q] = ok ? w : T(0);
      pv[j][q] = ok ? pw : T(0);
    }
  }
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const int col = (nh * 5 + j) * 16 + lr;
    const int cs = col / BKC, k = col - cs * BKC, ch = chs[cs];
    const bool last = (lastm >> j) & 1;
    T zv[4];
    if (buf) {
      const int64_t nb = (ch >= 0 ? a.noff[ch] : 0) + (int64_t)a.slot * a.P;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int fi = mt * 16 + M::row(lane, q);
        const bool ok = ch >= 0 && fi < nfeat;
        const double z = a.noise[ok ? nb + (uint32_t)((d0 + fi) * BKC + k) : 0];
        zv[q] = ok ? (T)z : T(0);
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) zv[q] = Nz[(mt * 16 + M::row(lane, q)) * bnz<T>() + col];
    }
    double p2s = 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int fi = mt * 16 + M::row(lane, q);
      if (ch >= 0 && fi < nfeat) {
        const int d = d0 + fi;
        const size_t idx = ((size_t)ch * D + d) * BKC + k;
        const T w = wv[j][q];
        const T gr = -(acc[j][q] - a.alpha * w);
        const T p = (a.one_minus_eps * pv[j][q] + a.eps * gr) + a.noise_scale * zv[q];
        Pg[idx] = p;
        if (!last) Wg[idx] = w + a.eps * p;
        else p2s += (double)(p * p);
      }
    }
    kp[(mt * 4 + lg) * BNP + col] = p2s;
  }
  __syncthreads();
  if (tid < BCT) {                                   // Σ pW² per chain ending at this iteration
    const int ch = chs[tid];
    if (ch >= 0 && a.iter == a.n_iter[ch] - 1) {
      double v = 0.0;
      for (int k = 0; k < BKC; ++k)
        for (int g = 0; g < 8; ++g) v += kp[g * BNP + tid * BKC + k];
      a.kin_part[(size_t)bx * a.C + ch] = v;
    }
  }
  if (bx == 0) bias_substep(a, chs, pbs);
}

// k_bgrad with wide feature tiles: NW waves, FT = 16·NW features × 16 chains (two m-tiles per wave:
// 10 MFMAs per 7 LDS operand reads instead of 5 per 6), used when many chains are active.  Built with
// NW = 4: 64 features, 66 KB of LDS, two workgroups per CU.  (NW = 8 — 128 features, 122 KB, one
// 8-wave workgroup per CU, 7 feature tiles instead of 13 re-reading each diff slice — measured
// slower: 247 vs 231 ms per 24-step call at 2048 chains)
// LDS (dynamic): X chunk [32 rows][FT features] (later the per-lane-group p² sums) and the diff chunk
// [32 rows][160] (later the friction noise of one pass: f64 chains in two passes of FT/2 features —
// m-tile i = pass, local feature fl = mt·16 + row — f32 chains in one).
template <typename T, int NW> struct BGW {
  static constexpr int NT = 64 * NW, FT = 16 * NW, XP = FT + 16;     // XP ≡ 16 (mod 32)
  static constexpr int NXV = BCH * FT / 2 / NT;                        // X 2-vectors per thread (4)
  static constexpr int NDV = BCH * BNT / 2 / NT;                       // diff 2-vectors per thread
  static constexpr int NMT = NW / 2;                                   // feature groups of 32
  static constexpr int NPASS = sizeof(T) == 8 ? 2 : 1;
  static constexpr int NZR = FT / NPASS;                               // noise rows per pass
  static constexpr int XSN = BCH * XP > 2 * NW * BNP * 8 / (int)sizeof(T) ? BCH * XP : 2 * NW * BNP * 8 / (int)sizeof(T);
  static constexpr int DSN = BCH * BWP > NZR * bnz<T>() ? BCH * BWP : NZR * bnz<T>();
  static constexpr size_t lds() { return (size_t)(XSN + DSN + BNT) * sizeof(T) + BCT * sizeof(int); }
};
constexpr int BRW2 = 64;          // k_bgradw<T, 4> feature tile

// amdgpu_waves_per_eu(2): two 4-wave workgroups per CU (the LDS allows two) need <= 256 registers.
template <typename T, int NW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(2))) void k_bgradw(BGradArgs<T> a) {
  using M = mfma16<T>;
  using G = BGW<T, NW>;
  typedef typename StageMap<T>::v2 v2;
  extern __shared__ __attribute__((aligned(16))) unsigned char bgw_smem[];
  T* Xs = reinterpret_cast<T*>(bgw_smem);                // [row][feature]; later the p² sums
  T* Ds = Xs + G::XSN;                                   // [row][column]; later the friction noise
  T* pbs = Ds + G::DSN;
  int* chs = reinterpret_cast<int*>(pbs + BNT);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  int bx, by;
  if (!(a.tail_last ? xcd_tile_tail_last(a.nX, a.nCT, bx, by) : xcd_tile(a.nX, a.nCT, bx, by))) return;
  const int d0 = bx * G::FT, rank0 = by * BCT;
  const int nfeat = min(G::FT, a.D - d0);
  const int D = a.D, N = a.N, B = a.B;
  if (tid < BCT) chs[tid] = rank0 + tid < a.c_act ? a.perm[rank0 + tid] : -1;
  __syncthreads();

  // diff chunk [32 rows][16 chains × 10]: 2560 vectors, NDV per thread (StageCM's map, stride NT)
  int wr[G::NDV], wls[G::NDV];
  size_t wsrc[G::NDV];
  bool wok[G::NDV];
#pragma unroll
  for (int u = 0; u < G::NDV; ++u) {
    const int j = tid + G::NT * u;
    const int row = j / 80, rem = j - row * 80, cs = rem / 5, k2 = (rem - cs * 5) * 2, ch = chs[cs];
    wr[u] = row;
    wok[u] = ch >= 0;
    wsrc[u] = (size_t)(ch >= 0 ? ch : 0) * ((size_t)B * BKC) + k2;
    wls[u] = cs * BKC + k2;
  }
  int xr[G::NXV], xc[G::NXV];                            // X chunk [32 rows][FT features]
#pragma unroll
  for (int u = 0; u < G::NXV; ++u) {
    const int j = tid + G::NT * u;
    xr[u] = j / (G::FT / 2);
    xc[u] = (j - xr[u] * (G::FT / 2)) * 2;
  }
  v2 xv[G::NXV], dv[G::NDV];
  auto fetch = [&](int r0) {
#pragma unroll
    for (int u = 0; u < G::NXV; ++u) {
      const int r = r0 + xr[u];
      xv[u] = ld2<T>(a.X + (size_t)min(r, B - 1) * D + d0 + xc[u], r < B, nfeat - xc[u]);
    }
#pragma unroll
    for (int u = 0; u < G::NDV; ++u) {
      const int r = r0 + wr[u];
      dv[u] = ld2<T>(a.diff + wsrc[u] + (size_t)min(r, B - 1) * BKC, wok[u] && r < B, 2);
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int u = 0; u < G::NXV; ++u) st2<T>(Xs + xr[u] * G::XP + xc[u], xv[u]);
#pragma unroll
    for (int u = 0; u < G::NDV; ++u) st2<T>(Ds + wr[u] * BWP + wls[u], dv[u]);
  };

  const int mt = wave % G::NMT, nh = wave / G::NMT;     // wave: features mt·32 .. +32, columns nh·80 .. +80
  // bit j: column j of this lane belongs to a chain whose path ends at this iteration (read once here,
  // its latency hidden by the main loop, instead of a waited load per column in the epilogue)
  int lastm = 0;
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const int ch = chs[((nh * 5 + j) * 16 + lr) / BKC];
    const int n = a.n_iter[ch >= 0 ? ch : 0];
    lastm |= (ch >= 0 && a.iter >= n - 1) << j;
  }
  // m-tiles of this wave holding features (wave-uniform): a partial last tile (D = 784: 16 of 64
  // features) skips the MFMAs of its empty m-tiles; their accumulators stay zero and are never stored
  const int nmw = min(2, max(0, (nfeat - mt * 32 + 15) / 16));
  typename M::acc_t acc[2][5];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 5; ++j) acc[i][j] = M::zero();
  fetch(0);
  for (int r0 = 0; r0 < B; r0 += BCH) {
    __syncthreads();
    stash();
    __syncthreads();
    if (r0 + BCH < B) fetch(r0 + BCH);
    const int nks = min(BCH, B - r0 + 3) / 4;
    if (nmw == 2) {
#pragma unroll 2
      for (int ks = 0; ks < nks; ++ks) {
        T av[2], bv[5];
#pragma unroll
        for (int i = 0; i < 2; ++i) av[i] = Xs[(ks * 4 + lg) * G::XP + mt * 32 + i * 16 + lr];
#pragma unroll
        for (int j = 0; j < 5; ++j) bv[j] = Ds[(ks * 4 + lg) * BWP + (nh * 5 + j) * 16 + lr];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 5; ++j) acc[i][j] = M::fma(av[i], bv[j], acc[i][j]);
      }
    } else if (nmw == 1) {
#pragma unroll 2
      for (int ks = 0; ks < nks; ++ks) {
        T bv[5];
        const T av = Xs[(ks * 4 + lg) * G::XP + mt * 32 + lr];
#pragma unroll
        for (int j = 0; j < 5; ++j) bv[j] = Ds[(ks * 4 + lg) * BWP + (nh * 5 + j) * 16 + lr];
#pragma unroll
        for (int j = 0; j < 5; ++j) acc[0][j] = M::fma(av, bv[j], acc[0][j]);
      }
    }
  }
  __syncthreads();
  // ---- epilogue on the accumulators: softmax.py:57-58 gradient, sghmc.py:31,34 momentum, :32 drift
  T* Nz = Ds;
  double* kp = reinterpret_cast<double*>(Xs);        // [mt·4 + lg][BNP] Σ p² over the lane's rows
  // The elements of one column (the pass's m-tiles × 4 rows) are loaded together (W and pW never
  // alias); every load is unconditional (clamped address, value selected afterwards) and the noise source is
  // chosen per launch outside the element loops: a load under a branch — or one through a pointer
  // that may be LDS or global, i.e. a flat load — made hipcc wait for each element's load (and the
  // previous element's stores) before the next.
  T* __restrict__ Wg = a.W;
  T* __restrict__ Pg = a.pW;
  const bool buf = a.noise_mode == HMCX_NOISE_BUFFER;
  double p2s[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  constexpr int NI = 2 / G::NPASS;                   // m-tiles of one pass
#pragma unroll
  for (int h = 0; h < G::NPASS; ++h) {
    const int i0 = G::NPASS == 2 ? h : 0;
    if (!buf) {
      if (h) __syncthreads();                      // pass 0's noise has been read
      if constexpr (G::NPASS == 2)
        gen_tile_noise(a, chs, d0, nfeat, Nz, G::NZR, [h](int fl) { return (fl >> 4) * 32 + h * 16 + (fl & 15); });
      else
        gen_tile_noise(a, chs, d0, nfeat, Nz, G::FT, [](int fl) { return fl; });
      __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int col = (nh * 5 + j) * 16 + lr;
      const int cs = col / BKC, k = col - cs * BKC, ch = chs[cs];
      const bool last = (lastm >> j) & 1;
      T wv[NI * 4], pv[NI * 4], zv[NI * 4];
#pragma unroll
      for (int ii = 0; ii < NI; ++ii)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int fi = mt * 32 + (i0 + ii) * 16 + M::row(lane, q);
          const bool ok = ch >= 0 && fi < nfeat;
          const size_t idx = ok ? ((size_t)ch * D + (d0 + fi)) * BKC + k : 0;
          const T w = Wg[idx], pw = Pg[idx];
          wv[ii * 4 + q] = ok ? w : T(0);
          pv[ii * 4 + q] = ok ? pw : T(0);
        }
      if (buf) {
        const int64_t nb = (ch >= 0 ? a.noff[ch] : 0) + (int64_t)a.slot * a.P;
#pragma unroll
        for (int ii = 0; ii < NI; ++ii)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int fi = mt * 32 + (i0 + ii) * 16 + M::row(lane, q);
            const bool ok = ch >= 0 && fi < nfeat;
            const double z = a.noise[ok ? nb + (uint32_t)((d0 + fi) * BKC + k) : 0];
            zv[ii * 4 + q] = ok ? (T)z : T(0);
          }
      } else {
#pragma unroll
        for (int ii = 0; ii < NI; ++ii)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int fi = mt * 32 + (i0 + ii) * 16 + M::row(lane, q);
            const int nzr = G::NPASS == 2 ? mt * 16 + M::row(lane, q) : fi;
            zv[ii * 4 + q] = Nz[nzr * bnz<T>() + col];
          }
      }
#pragma unroll
      for (int ii = 0; ii < NI; ++ii)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = i0 + ii;
          const int fi = mt * 32 + i * 16 + M::row(lane, q);
          if (ch >= 0 && fi < nfeat) {
            const int d = d0 + fi;
            const size_t idx = ((size_t)ch * D + d) * BKC + k;
            const T w = wv[ii * 4 + q];
            const T gr = -(acc[i][j][q] - a.alpha * w);
            const T p = (a.one_minus_eps * pv[ii * 4 + q] + a.eps * gr) + a.noise_scale * zv[ii * 4 + q];
            Pg[idx] = p;
            if (!last) Wg[idx] = w + a.eps * p;
            else p2s[j] += (double)(p * p);
          }
        }
    }
  }
#pragma unroll
  for (int j = 0; j < 5; ++j) kp[(mt * 4 + lg) * BNP + (nh * 5 + j) * 16 + lr] = p2s[j];
  __syncthreads();
  if (tid < BCT) {                                   // Σ pW² per chain ending at this iteration
    const int ch = chs[tid];
    if (ch >= 0 && a.iter == a.n_iter[ch] - 1) {
      double v = 0.0;
      for (int k = 0; k < BKC; ++k)
        for (int g = 0; g < 4 * G::NMT; ++g) v += kp[g * BNP + tid * BKC + k];
      a.kin_part[(size_t)bx * a.C + ch] = v;
      if (bx == 0)
        for (int b2 = a.nX; b2 < a.nDB_all; ++b2) a.kin_part[(size_t)b2 * a.C + ch] = 0.0;
    }
  }
  if (bx == 0) bias_substep(a, chs, pbs);
}

}  // namespace hmcx
