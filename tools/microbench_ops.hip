// Per-operation cycle costs inside one 512-thread workgroup (MI355X): barrier, LDS chain, f64 exp,
// write-through store drain, write-through load, agent atomic round trip. Clock = s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("ERR %s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ __launch_bounds__(512) void k_ops(double* buf, unsigned* ctr, unsigned long long* out, int reps) {
  __shared__ double lds[4096];
  const int t = threadIdx.x;
  for (int i = t; i < 4096; i += 512) lds[i] = (double)((i * 7) % 4096);
  __syncthreads();
  unsigned long long t0, t1;
  // (0) barrier
  t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) __syncthreads();
  t1 = __builtin_amdgcn_s_memtime();
  if (t == 0) out[0] = (t1 - t0) / reps;
  // (1) dependent LDS read chain
  int idx = t;
  t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) idx = (int)lds[idx & 4095];
  t1 = __builtin_amdgcn_s_memtime();
  if (t == 0) out[1] = (t1 - t0) / reps + (idx == -1);
  // (2) f64 exp chain
  double x = 0.001 * t;
  t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) x = exp(x) * 1e-3;
  t1 = __builtin_amdgcn_s_memtime();
  if (t == 0) out[2] = (t1 - t0) / reps + (x == -1.0);
  // (3) write-through store + drain
  t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(buf + t), (unsigned long long)r, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (t == 0) out[3] = (t1 - t0) / reps;
  // (4) dependent write-through loads
  unsigned long long v = 0;
  t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r)
    v += __hip_atomic_load(reinterpret_cast<unsigned long long*>(buf + ((t + v) & 511)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
  t1 = __builtin_amdgcn_s_memtime();
  if (t == 0) out[4] = (t1 - t0) / reps + (v == 12345);
  // (5) plain dependent global loads
  double w = 0;
  t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) w += buf[((int)w + t) & 511];
  t1 = __builtin_amdgcn_s_memtime();
  if (t == 0) out[5] = (t1 - t0) / reps + (w == -1.0);
  // (6) lane-0 atomic add + sc1 poll (single block: immediate)
  __syncthreads();
  t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
    if (t == 0) {
      __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)(r + 1)) {}
    }
    __syncthreads();
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (t == 0) out[6] = (t1 - t0) / reps;
  // (7) s_memrealtime vs s_memtime over a busy loop
  unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();
  t0 = __builtin_amdgcn_s_memtime();
  double y = 1.0;
  for (int r = 0; r < 200000; ++r) y = y * 1.0000001 + 1e-9;
  t1 = __builtin_amdgcn_s_memtime();
  unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
  if (t == 0) { out[7] = t1 - t0; out[8] = rt1 - rt0; out[9] = (y == 0.0); }
}

int main() {
  double* buf;
  unsigned* ctr;
  unsigned long long* out;
  CK(hipMalloc(&buf, 8192 * 8));
  CK(hipMalloc(&ctr, 4));
  CK(hipMalloc(&out, 16 * 8));
  CK(hipMemset(buf, 0, 8192 * 8));
  for (int pass = 0; pass < 3; ++pass) {
    CK(hipMemset(ctr, 0, 4));
    hipLaunchKernelGGL(k_ops, dim3(1), dim3(512), 0, 0, buf, ctr, out, 200);
    CK(hipDeviceSynchronize());
    unsigned long long h[16];
    CK(hipMemcpy(h, out, 16 * 8, hipMemcpyDeviceToHost));
    printf("pass %d: barrier %llu | lds-chain %llu | exp-f64 %llu | sc1-store+drain %llu | sc1-load-chain %llu | "
           "plain-load-chain %llu | atomic+poll+barrier %llu | memtime/realtime %.2f (x100MHz)\n",
           pass, h[0], h[1], h[2], h[3], h[4], h[5], h[6], (double)h[7] / (double)h[8]);
  }
  return 0;
}
