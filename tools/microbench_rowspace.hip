// Per-iteration cost of a row-space SGHMC leapfrog on ONE XCD (design probe, round 5).
//
// W workers = the workgroups with blockIdx % 8 < NX (so NX = 1 puts all of them on XCD 0 and its L2).
// Worker w owns R = ceil(B / W) minibatch rows.  One iteration:
//   1. a softmax-like pass over its R × K logits → diff rows (+ a K-wide colsum partial);
//   2. publish R·K + K values as tagged 16-B granules {lo, ep, hi, ep} (L2-local plain stores when
//      NX = 1, sc1 write-through otherwise);
//   3. gather ALL W·(R·K + K) granules into LDS (sc0 loads hit the XCD's L2; sc1 otherwise);
//   4. (G rows) · diff_all on v_mfma_f64_16x16x4 — G rows (R × B) resident in LDS, K-split over the waves,
//      combined through LDS in wave order;
//   5. the row updates (Zp, Zw) from the product.
// Reports µs per iteration (max over workers) for a few (W, NX, threads) shapes at B = 500, K = 10.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("ERR %s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
typedef unsigned int g4 __attribute__((ext_vector_type(4)));
typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int B = 500, K = 10, BP = 512;

struct Args {
  int W, NX, R, rounds, local;
  char* arena; int arena_bytes;
  unsigned long long* out;
  double* sink;
  const double* G;      // [B][BP] (row-major, padded), any values
};

template <int NT>
__global__ __launch_bounds__(NT) void k_rs(Args a) {
  const int tid = threadIdx.x, b = blockIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NW = NT / 64;
  if ((b & 7) >= a.NX) return;
  const int w = (b >> 3) * a.NX + (b & 7);
  if (w >= a.W) return;
  const int R = a.R, r0 = w * R, nown = min(R, B - r0);
  const int P = R * K + K;                        // granules per producer (fixed stride)
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.arena, 0, a.arena_bytes, 0x00020000);
  extern __shared__ double lds[];
  double* Gs = lds;                               // [16][BP + 2]  (R ≤ 16 rows; rest zero)
  double* Ds = Gs + 16 * (BP + 2);                // [BP][K + 2]   diff of every row
  double* Red = Ds + BP * (K + 2);                // [NW][16][16]
  double* Zw = Red + NW * 256;                    // [16][K]
  double* Zp = Zw + 16 * K;                       // [16][K]
  double* Cs = Zp + 16 * K;                       // [W][K] colsum partials
  for (int i = tid; i < 16 * (BP + 2); i += NT) {
    const int r = i / (BP + 2), c = i % (BP + 2);
    Gs[i] = (r < nown && c < B) ? a.G[(size_t)(r0 + r) * BP + c] : 0.0;
  }
  for (int i = tid; i < BP * (K + 2); i += NT) Ds[i] = 0.0;
  for (int i = tid; i < 16 * K; i += NT) { Zw[i] = 0.01 * i; Zp[i] = 0.0; }
  __syncthreads();
  const int n_all = a.W * P;
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < a.rounds; ++it) {
    const unsigned ep = it + 1;
    const int base = (it & 1) * a.W * P;
    // 1 + 2: "softmax" of the owned rows and publish (one thread per (row, class) value)
    if (tid < P) {
      double v;
      if (tid < R * K) {
        const int r = tid / K, k = tid % K;
        v = r < nown ? 1.0 / (1.0 + exp(-Zw[r * K + k])) - 0.1 : 0.0;
        Zw[r * K + k] += 1e-3 * Zp[r * K + k];
      } else {
        v = 0.5 + tid;
      }
      const unsigned long long x = __builtin_bit_cast(unsigned long long, v);
      g4 q = {(unsigned)x, ep, (unsigned)(x >> 32), ep};
      if (a.local) __builtin_amdgcn_raw_buffer_store_b128(q, rs, (base + w * P + tid) * 16, 0, 0);
      else __builtin_amdgcn_raw_buffer_store_b128(q, rs, (base + w * P + tid) * 16, 0, 16);
    }
    // 3: gather every producer's granules into LDS (batches of 16 loads per thread)
    for (int b0 = 0; b0 < n_all; b0 += NT * 16) {
      g4 v[16];
      int o[16];
      unsigned pend = 0;
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int j = b0 + tid + u * NT;
        o[u] = j < n_all ? j : 0;
        pend |= j < n_all ? 1u << u : 0u;
      }
      unsigned long long tb = __builtin_amdgcn_s_memrealtime();
      while (pend) {
        if (__builtin_amdgcn_s_memrealtime() - tb > 200000000ull) { a.sink[0] = -1.0; return; }   // 2 s bound
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (pend & (1u << u))
            v[u] = a.local ? __builtin_amdgcn_raw_buffer_load_b128(rs, (base + o[u]) * 16, 0, 1)
                           : __builtin_amdgcn_raw_buffer_load_b128(rs, (base + o[u]) * 16, 0, 16);
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if ((pend & (1u << u)) && v[u].y == ep && v[u].w == ep) {
            const double d = __builtin_bit_cast(double, (unsigned long long)v[u].x | ((unsigned long long)v[u].z << 32));
            const int j = o[u], p = j / P, e = j - p * P;
            if (e < R * K) {
              const int row = p * R + e / K;
              Ds[row * (K + 2) + e % K] = d;
            } else {
              Cs[p * K + (e - R * K)] = d;
            }
            pend &= ~(1u << u);
          }
      }
    }
    __syncthreads();
    // 4: (G rows) · Ds over k in [0, BP): wave wv takes k-steps wv, wv + NW, ... (4 rows of k per step)
    d4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
    const int lr = lane & 15, lk = lane >> 4;
    for (int ks = wave; ks < BP / 4; ks += 2 * NW) {
      const int k0 = 4 * ks + lk, k1 = 4 * (ks + NW) + lk;
      const double a0 = Gs[lr * (BP + 2) + k0], b0v = lr < K ? Ds[k0 * (K + 2) + lr] : 0.0;
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0v, acc0, 0, 0, 0);
      if (ks + NW < BP / 4) {
        const double a1 = Gs[lr * (BP + 2) + k1], b1v = lr < K ? Ds[k1 * (K + 2) + lr] : 0.0;
        acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1v, acc1, 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) Red[wave * 256 + ((lane >> 4) + 4 * i) * 16 + lr] = acc0[i] + acc1[i];
    __syncthreads();
    // 5: row updates
    if (tid < 16 * K) {
      const int r = tid / K, k = tid % K;
      double s = 0.0;
      for (int wv = 0; wv < NW; ++wv) s += Red[wv * 256 + r * 16 + k];
      Zp[r * K + k] = 0.999 * Zp[r * K + k] - 1e-3 * (s + 0.01 * Zw[r * K + k]) + 1e-6 * Cs[k];
    }
    __syncthreads();
  }
  unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) a.out[w] = t1 - t0;
  if (tid < 16 * K) a.sink[w * 256 + tid] = Zp[tid];
}

template <int NT>
int run(const char* name, int W, int NX, int local, char* arena, int arena_bytes, unsigned long long* out,
        double* sink, const double* G) {
  const int rounds = 2000;
  const int R = (B + W - 1) / W;
  if (R > 16) return 0;
  Args a{W, NX, R, rounds, local, arena, arena_bytes, out, sink, G};
  const size_t lds = (16 * (BP + 2) + BP * (K + 2) + (NT / 64) * 256 + 32 * K + 64 * K) * sizeof(double);
  CK(hipFuncSetAttribute((const void*)k_rs<NT>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CK(hipMemset(arena, 0, arena_bytes));
  CK(hipMemset(out, 0, 256 * 8));
  const int grid = 8 * ((W + NX - 1) / NX);
  hipLaunchKernelGGL(k_rs<NT>, dim3(grid), dim3(NT), lds, 0, a);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  unsigned long long h[256];
  double s0;
  CK(hipMemcpy(h, out, 256 * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&s0, sink, 8, hipMemcpyDeviceToHost));
  unsigned long long mx = 0, mn = ~0ull;
  for (int i = 0; i < W; ++i) { mx = h[i] > mx ? h[i] : mx; mn = h[i] < mn ? h[i] : mn; }
  printf("%-10s workers %3d on %d XCD(s) %s rows %2d threads %d: %.3f us/iteration (min worker %.3f)%s\n", name, W, NX,
         local ? "L2-local" : "sc1     ", R, NT, mx / 100.0 / rounds, mn / 100.0 / rounds, s0 == -1.0 ? "  TIMEOUT" : "");
  return 0;
}

int main() {
  const int arena_bytes = 2 * 64 * 200 * 16;
  char* arena;
  CK(hipMalloc(&arena, arena_bytes));
  unsigned long long* out;
  CK(hipMalloc(&out, 256 * 8));
  double* sink;
  CK(hipMalloc(&sink, 256 * 256 * 8));
  double* G;
  CK(hipMalloc(&G, (size_t)B * BP * 8));
  CK(hipMemset(G, 0, (size_t)B * BP * 8));
  // 32 workers on one XCD (L2-local), the design point; then 32 spread over 8 XCDs; 64 on 2 XCDs
  if (run<256>("1xcd", 32, 1, 1, arena, arena_bytes, out, sink, G)) return 1;
  if (run<512>("1xcd", 32, 1, 1, arena, arena_bytes, out, sink, G)) return 1;
  if (run<256>("1xcd-sc1", 32, 1, 0, arena, arena_bytes, out, sink, G)) return 1;
  if (run<256>("8xcd", 32, 8, 0, arena, arena_bytes, out, sink, G)) return 1;
  if (run<256>("2xcd", 64, 2, 0, arena, arena_bytes, out, sink, G)) return 1;
  if (run<512>("8xcd", 64, 8, 0, arena, arena_bytes, out, sink, G)) return 1;
  return 0;
}
