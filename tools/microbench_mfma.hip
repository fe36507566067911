// f64 / f32 16x16x4 MFMA issue cost for ONE wave per SIMD (256-thread workgroups, one per CU):
// cycles per MFMA (s_memtime) with 1, 2, 4 and 8 independent accumulator chains; "x2" rows run
// 512-thread workgroups (two waves per SIMD) and report cycles per instruction per wave.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <int NA>
__global__ __launch_bounds__(512) void k64(double* out, unsigned long long* cyc, int reps) {
  d4 c[NA];
  for (int i = 0; i < NA; ++i) c[i] = d4{0, 0, 0, 0};
  double a = 1e-3 * threadIdx.x, b = 2e-3;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r)
#pragma unroll
    for (int i = 0; i < NA; ++i) c[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[i], 0, 0, 0);
  double s = 0;
  for (int i = 0; i < NA; ++i) s += c[i][0];
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 512 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int NA>
__global__ __launch_bounds__(256) void k32(double* out, unsigned long long* cyc, int reps) {
  f4 c[NA];
  for (int i = 0; i < NA; ++i) c[i] = f4{0, 0, 0, 0};
  float a = 1e-3f * threadIdx.x, b = 2e-3f;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r)
#pragma unroll
    for (int i = 0; i < NA; ++i) c[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[i], 0, 0, 0);
  float s = 0;
  for (int i = 0; i < NA; ++i) s += c[i][0];
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
// VALU f64 FMA chain throughput for comparison: NA independent chains
template <int NA>
__global__ __launch_bounds__(256) void kv64(double* out, unsigned long long* cyc, int reps) {
  double c[NA];
  for (int i = 0; i < NA; ++i) c[i] = i;
  double a = 1.0000001, b = 1e-9 * threadIdx.x;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r)
#pragma unroll
    for (int i = 0; i < NA; ++i) c[i] = __builtin_fma(c[i], a, b);
  double s = 0;
  for (int i = 0; i < NA; ++i) s += c[i];
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <typename F>
void run(const char* name, F kern, int na, double* o, unsigned long long* c, int reps, int nt = 256) {
  hipLaunchKernelGGL(kern, dim3(256), dim3(nt), 0, 0, o, c, reps);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(kern, dim3(256), dim3(nt), 0, 0, o, c, reps);
  hipDeviceSynchronize();
  unsigned long long h[256];
  hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < 256; ++i) m += h[i];
  m /= 256;
  printf("%s acc=%d: %.1f cycles per instruction per wave\n", name, na, m / ((double)reps * na));
}
int main() {
  double* o;
  unsigned long long* c;
  hipMalloc(&o, 256 * 512 * 8);
  hipMalloc(&c, 256 * 8);
  const int reps = 4096;
  run("mfma_f64_16x16x4", k64<1>, 1, o, c, reps);
  run("mfma_f64_16x16x4", k64<2>, 2, o, c, reps);
  run("mfma_f64_16x16x4", k64<4>, 4, o, c, reps);
  run("mfma_f64_16x16x4", k64<8>, 8, o, c, reps);
  run("mfma_f64_16x16x4 x2", k64<1>, 1, o, c, reps, 512);
  run("mfma_f64_16x16x4 x2", k64<2>, 2, o, c, reps, 512);
  run("mfma_f64_16x16x4 x2", k64<4>, 4, o, c, reps, 512);
  run("mfma_f32_16x16x4", k32<1>, 1, o, c, reps);
  run("mfma_f32_16x16x4", k32<2>, 2, o, c, reps);
  run("mfma_f32_16x16x4", k32<4>, 4, o, c, reps);
  run("v_fma_f64", kv64<1>, 1, o, c, reps);
  run("v_fma_f64", kv64<4>, 4, o, c, reps);
  run("v_fma_f64", kv64<8>, 8, o, c, reps);
  return 0;
}
