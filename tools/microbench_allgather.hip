// All-gather round cost on MI355X: W worker workgroups (512 threads) each publish P values per round
// as tagged 16-B granules and gather all W·P values (every worker reads everything), for the
// row-space SGHMC design (csrc/hmcx_rowspace.hip: one all-gather of diff rows per leapfrog).
// Placement: the grid holds 8·W/NX workgroups and the workers are those with blockIdx % 8 < NX
// (NX XCDs; the others exit at once).  Transport: sc1 stores + sc1 loads, or (NX = 1 only) plain
// stores + sc0 loads kept in the one XCD's L2.  Reports µs per round (max over workers).
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("ERR %s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
typedef unsigned int g4 __attribute__((ext_vector_type(4)));

struct Args {
  int W, P, NX, rounds, local;
  char* arena; int arena_bytes;
  unsigned long long* out;
  double* sink;
};

__global__ __launch_bounds__(512) void k_ag(Args a) {
  const int tid = threadIdx.x, b = blockIdx.x;
  if ((b & 7) >= a.NX) return;
  const int w = (b >> 3) * a.NX + (b & 7);            // worker id
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.arena, 0, a.arena_bytes, 0x00020000);
  __shared__ double acc[512];
  double sum = 0.0;
  const int n = a.W * a.P;
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < a.rounds; ++it) {
    const unsigned ep = it + 1;
    const int base = (it & 1) * a.W * a.P;
    for (int e = tid; e < a.P; e += 512) {
      const double v = (double)(w * 1000 + e + it);
      const unsigned long long x = __builtin_bit_cast(unsigned long long, v);
      g4 q = {(unsigned)x, ep, (unsigned)(x >> 32), ep};
      if (a.local) __builtin_amdgcn_raw_buffer_store_b128(q, rs, (base + w * a.P + e) * 16, 0, 0);
      else __builtin_amdgcn_raw_buffer_store_b128(q, rs, (base + w * a.P + e) * 16, 0, 16);
    }
    for (int b0 = 0; b0 < n; b0 += 512 * 16) {
      g4 v[16];
      int o[16];
      unsigned pend = 0;
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int j = b0 + tid + u * 512;
        o[u] = (base + (j < n ? j : 0)) * 16;
        pend |= j < n ? 1u << u : 0u;
      }
      unsigned long long tb = __builtin_amdgcn_s_memrealtime();
      while (pend) {
        if (__builtin_amdgcn_s_memrealtime() - tb > 200000000ull) { a.sink[0] = -1.0; return; }   // 2 s bound
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (pend & (1u << u))
            v[u] = a.local ? __builtin_amdgcn_raw_buffer_load_b128(rs, o[u], 0, 1)
                           : __builtin_amdgcn_raw_buffer_load_b128(rs, o[u], 0, 16);
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if ((pend & (1u << u)) && v[u].y == ep && v[u].w == ep) {
            sum += __builtin_bit_cast(double, (unsigned long long)v[u].x | ((unsigned long long)v[u].z << 32));
            pend &= ~(1u << u);
          }
        if (pend) __builtin_amdgcn_s_sleep(1);
      }
    }
    acc[tid] = sum;
    __syncthreads();
  }
  unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) a.out[w] = t1 - t0;
  a.sink[w * 512 + tid] = sum + acc[(tid + 1) & 511];
}

int main() {
  const int rounds = 1000;
  const int arena_bytes = 2 * 128 * 400 * 16;
  char* arena;
  CK(hipMalloc(&arena, arena_bytes));
  unsigned long long* out;
  CK(hipMalloc(&out, 256 * 8));
  double* sink;
  CK(hipMalloc(&sink, 256 * 512 * 8));
  const int cfg[][3] = {{16, 1, 1}, {16, 1, 0}, {16, 2, 0}, {16, 8, 0}, {32, 2, 0}, {32, 4, 0}, {32, 8, 0},
                        {64, 4, 0}, {64, 8, 0}, {128, 8, 0}};
  const int Ps[] = {50, 100, 170, 330};
  for (auto& c : cfg)
    for (int P : Ps) {
      const int W = c[0], NX = c[1], local = c[2];
      if (W * P > 16 * 512 * 4) continue;
      Args a{W, P, NX, rounds, local, arena, arena_bytes, out, sink};
      CK(hipMemset(arena, 0, arena_bytes));
      void* args[] = {&a};
      const int grid = 8 * W / NX;
      CK(hipLaunchKernel((const void*)k_ag, dim3(grid), dim3(512), args, 0, 0));
      CK(hipDeviceSynchronize());
      unsigned long long h[256];
      CK(hipMemcpy(h, out, 256 * 8, hipMemcpyDeviceToHost));
      unsigned long long mx = 0;
      for (int i = 0; i < W; ++i) mx = h[i] > mx ? h[i] : mx;
      printf("workers %3d on %d XCD(s) %s P=%3d (%5d granules per reader): %.3f us/round\n", W, NX,
             local ? "L2-local" : "sc1     ", P, W * P, mx / 100.0 / rounds);
    }
  return 0;
}
