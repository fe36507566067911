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

typedef double d4v __attribute__((ext_vector_type(4)));
typedef float f4v __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_mfma64(double* out, int reps) {
  d4v c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  double a = 1e-3 * threadIdx.x, b = 2e-3;
  for (int r = 0; r < reps; ++r) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
  }
  out[blockIdx.x * 256 + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
}
__global__ __launch_bounds__(256) void k_mfma32(double* out, int reps) {
  f4v c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  float a = 1e-3f * threadIdx.x, b = 2e-3f;
  for (int r = 0; r < reps; ++r) {
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
  }
  out[blockIdx.x * 256 + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
}

int main() {
  {
    double* o;
    CK(hipMalloc(&o, 256 * 1024 * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 20000, blocks = 1024;
    for (int pass = 0; pass < 2; ++pass) {
      float ms64 = 0, ms32 = 0;
      CK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(k_mfma64, dim3(blocks), dim3(256), 0, 0, o, reps);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms64, e0, e1));
      CK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(k_mfma32, dim3(blocks), dim3(256), 0, 0, o, reps);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms32, e0, e1));
      const double flop = (double)blocks * 4 /*waves*/ * reps * 4 /*mfma*/ * 2048.0;
      if (pass) printf("MFMA f64 16x16x4: %.1f TFLOP/s | f32 16x16x4: %.1f TFLOP/s\n", flop / ms64 / 1e9, flop / ms32 / 1e9);
    }
  }
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
