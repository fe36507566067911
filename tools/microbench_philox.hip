// Philox-4x32-10 throughput on gfx950: the 32×32 products as v_mul_hi_u32 + v_mul_lo_u32 (what the
// compiler emits for hmcx_common.h) against one v_mad_u64_u32 per product.  Same outputs checked.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

struct u4 { uint32_t v[4]; };

__device__ inline void mulhilo_split(uint32_t m, uint32_t a, uint32_t& hi, uint32_t& lo) {
  hi = (uint32_t)(((uint64_t)m * a) >> 32);
  lo = m * a;
}
__device__ inline void mulhilo_mad(uint32_t m, uint32_t a, uint32_t& hi, uint32_t& lo) {
  uint64_t p;
  asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(p) : "v"(a), "s"(m) : "vcc");
  hi = (uint32_t)(p >> 32);
  lo = (uint32_t)p;
}

template <int V>
__device__ inline u4 philox(u4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, lo0, hi1, lo1;
    if (V == 0) { mulhilo_split(0xD2511F53u, c.v[0], hi0, lo0); mulhilo_split(0xCD9E8D57u, c.v[2], hi1, lo1); }
    else { mulhilo_mad(0xD2511F53u, c.v[0], hi0, lo0); mulhilo_mad(0xCD9E8D57u, c.v[2], hi1, lo1); }
    u4 n;
    n.v[0] = hi1 ^ c.v[1] ^ k0; n.v[1] = lo1; n.v[2] = hi0 ^ c.v[3] ^ k1; n.v[3] = lo0;
    c = n;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return c;
}

template <int V>
__global__ __launch_bounds__(256) void k(uint32_t* out, int n, uint32_t k0, uint32_t k1) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  u4 c = {{(uint32_t)g, 7u, 3u, 1u}};
  const u4 r = philox<V>(c, k0, k1);
  out[g] = r.v[0] ^ (r.v[1] * 3u) ^ (r.v[2] * 5u) ^ (r.v[3] * 7u);
}

int main() {
  const int n = 1 << 25;
  uint32_t *a, *b;
  hipMalloc(&a, n * 4); hipMalloc(&b, n * 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    for (int V = 0; V < 2; ++V) {
      hipEventRecord(e0);
      for (int i = 0; i < 20; ++i) {
        if (V == 0) hipLaunchKernelGGL(k<0>, dim3(n / 256), dim3(256), 0, 0, a, n, 0x1234u, 0x5678u);
        else hipLaunchKernelGGL(k<1>, dim3(n / 256), dim3(256), 0, 0, b, n, 0x1234u, 0x5678u);
      }
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      printf("variant %s: %.2f us per launch, %.1f G philox/s\n", V ? "mad_u64" : "mulhi+lo", ms * 1e3 / 20, n / (ms / 20 * 1e-3) / 1e9);
    }
  }
  std::vector<uint32_t> ha(n), hb(n);
  hipMemcpy(ha.data(), a, n * 4, hipMemcpyDeviceToHost); hipMemcpy(hb.data(), b, n * 4, hipMemcpyDeviceToHost);
  size_t diff = 0;
  for (int i = 0; i < n; ++i) diff += ha[i] != hb[i];
  printf("outputs differ at %zu of %d\n", diff, n);
  return diff != 0;
}
