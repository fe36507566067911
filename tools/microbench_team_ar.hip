// Round A of the persistent single-chain kernel (csrc/hmcx_persist2.hip) in its real team geometry:
// 128 workgroups of 256 threads, row teams of 16 consecutive blocks (identity map: a team's members
// sit on all 8 XCDs, two per XCD), 8 teams exchanging at once.  Each member publishes P = 640 partial
// logits (64 rows x 10 classes) per leapfrog.  Two ways to give every member the team's summed rows:
//   RS+AG (the kernel's): reduce-scatter — member f sums the 16 partials of its 4 rows (40 items x 16
//     producers), then publishes 56 granules (header + diff rows) and gathers all 16 x 56 of them;
//   AR: all-reduce by redundant reads — every member reads all 16 x 640 partials (no second round).
// Transport as in the kernel: sc1 stores, sc1 loads, 16-byte granules {lo, ep, hi, ep}, bounded spins.
// Also with the team on ONE XCD (plain stores kept in that XCD's L2, sc1 loads: the kernel's HMCX_P2_XMAP=1 placement
// for row teams), and round B's all-reduce (8 members x 504 granules: the kernel's B-AR) both ways.
// Reports µs per leapfrog-round (max over members), 2000 rounds per variant.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("ERR %s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
typedef unsigned int g4 __attribute__((ext_vector_type(4)));
constexpr int TH = 256, GF = 16, G = 128, P = 640, RO = 40, NXA = 56;

struct Args {
  int mode, rounds, T, PP, local;
  char* arena; int arena_bytes;
  unsigned long long* out;
  double* sink;
  int* abortf;                                           // raised by a timed-out spin: every member stops
};

__device__ inline void put(__amdgpu_buffer_rsrc_t rs, int g, double v, unsigned ep, bool local) {
  const unsigned long long x = __builtin_bit_cast(unsigned long long, v);
  g4 q = {(unsigned)x, ep, (unsigned)(x >> 32), ep};
  if (local) __builtin_amdgcn_raw_buffer_store_b128(q, rs, g * 16, 0, 0);
  else __builtin_amdgcn_raw_buffer_store_b128(q, rs, g * 16, 0, 16);
}

// every thread waits for its pairs q = tid + u·TH (< n) of granule offset off(q); returns Σ values
template <int U, typename Off>
__device__ inline double gather(__amdgpu_buffer_rsrc_t rs, int n, Off off, unsigned ep, int* abortf, bool local) {
  double sum = 0.0;
  for (int b0 = 0; b0 < n; b0 += U * TH) {
    g4 v[U];
    int o[U];
    unsigned pend = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = b0 + threadIdx.x + u * TH;
      o[u] = (q < n ? off(q) : 0) * 16;
      pend |= q < n ? 1u << u : 0u;
    }
    const unsigned long long tb = __builtin_amdgcn_s_memrealtime();
    for (int spins = 0; pend; ++spins) {
      if ((spins & 63) == 63 && (__builtin_amdgcn_s_memrealtime() - tb > 100000000ull ||      // 1 s bound
                                 __hip_atomic_load(abortf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
        __hip_atomic_store(abortf, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return sum;
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (pend & (1u << u))
          v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, o[u], 0, 16);   // sc1, as the kernel polls
#pragma unroll
      for (int u = 0; u < U; ++u)
        if ((pend & (1u << u)) && v[u].y == ep && v[u].w == ep) {
          sum += __builtin_bit_cast(double, (unsigned long long)v[u].x | ((unsigned long long)v[u].z << 32));
          pend &= ~(1u << u);
        }
    }
  }
  return sum;
}

__global__ __launch_bounds__(TH) void k_round(Args a) {
  const int tid = threadIdx.x, b = blockIdx.x, T = a.T, PP = a.PP;
  // team / member: consecutive blocks (a team spans the XCDs), or blocks of one XCD (b % 8 equal)
  const int r = a.local ? (b & 7) * (G / 8 / T) + (b >> 3) / T : b / T;
  const int f = a.local ? (b >> 3) % T : b % T;
  const bool lc = a.local;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.arena, 0, a.arena_bytes, 0x00020000);
  __shared__ double acc[TH];
  double sum = 0.0;
  unsigned ep = 0;
  const int RS = PP / T;                                // items per owner in the reduce-scatter
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < a.rounds; ++it) {
    const int par = it & 1;
    // region A: [par][team][member][PP]; region D: [par][team][member][NXA] after it
    const int regA = (par * (G / T) + r) * T * PP, regD = 2 * G * PP + (par * (G / T) + r) * T * NXA;
    ++ep;
    for (int e = tid; e < PP; e += TH) put(rs, regA + f * PP + e, (double)(b + e + it), ep, lc);
    if (a.mode == 0) {            // RS: my PP/T items of all T producers, then AG of T x 56
      sum += gather<4>(rs, T * RS, [&](int q) { return regA + (q / RS) * PP + f * RS + q % RS; }, ep, a.abortf, lc);
      __syncthreads();
      ++ep;
      for (int e = tid; e < NXA; e += TH) put(rs, regD + f * NXA + e, sum + e, ep, lc);
      sum += gather<4>(rs, T * NXA, [&](int q) { return regD + q; }, ep, a.abortf, lc);
    } else {                      // AR: all T x PP partials, 16 granules in flight per thread
      sum += gather<16>(rs, T * PP, [&](int q) { return regA + q; }, ep, a.abortf, lc);
    }
    acc[tid] = sum;
    __syncthreads();
    if (__hip_atomic_load(a.abortf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) a.out[b] = t1 - t0;
  a.sink[b * TH + tid] = sum + acc[(tid + 1) % TH];
}

int main() {
  const int rounds = 2000;
  const int arena_bytes = (2 * G * P + 2 * G * NXA) * 16;
  char* arena;
  CK(hipMalloc(&arena, arena_bytes));
  unsigned long long* out;
  CK(hipMalloc(&out, G * 8));
  double* sink;
  CK(hipMalloc(&sink, G * TH * 8));
  int* abortf;
  CK(hipMalloc(&abortf, sizeof(int)));
  // {mode, team size, granules per member, local}
  const int cfg[][4] = {{0, GF, P, 0}, {1, GF, P, 0}, {0, GF, P, 1}, {1, GF, P, 1}, {1, 8, 504, 0}, {1, 8, 504, 1}};
  const char* names[] = {"A: RS+AG, team across 8 XCDs (kernel default)", "A: AR,    team across 8 XCDs",
                         "A: RS+AG, team on one XCD", "A: AR,    team on one XCD",
                         "B: AR (8 x 504), team across 8 XCDs", "B: AR (8 x 504), team on one XCD (default)"};
  for (int rep = 0; rep < 3; ++rep)
    for (int c = 0; c < 6; ++c) {
      Args a{cfg[c][0], rounds, cfg[c][1], cfg[c][2], cfg[c][3], arena, arena_bytes, out, sink, abortf};
      CK(hipMemset(arena, 0, arena_bytes));
      CK(hipMemset(abortf, 0, sizeof(int)));
      void* args[] = {&a};
      CK(hipLaunchKernel((const void*)k_round, dim3(G), dim3(TH), args, 0, 0));
      CK(hipDeviceSynchronize());
      unsigned long long h[G];
      CK(hipMemcpy(h, out, G * 8, hipMemcpyDeviceToHost));
      unsigned long long mx = 0;
      for (int i = 0; i < G; ++i) mx = h[i] > mx ? h[i] : mx;
      int ab = 0;
      CK(hipMemcpy(&ab, abortf, sizeof(int), hipMemcpyDeviceToHost));
      printf("%-46s %.3f us per round%s\n", names[c], mx / 100.0 / rounds, ab ? "  [TIMED OUT]" : "");
      fflush(stdout);
    }
  return 0;
}
