// Microbenchmark: cost of straight-line code on MI355X.  k_fat<N> runs N FMAs fully unrolled (code
// ≈ 8 B per FMA), k_thin the same FMAs in a rolled loop of 8.  Every launch is 256 workgroups x 256
// threads; the time per launch (HIP events over 200 back-to-back launches) against N gives the cost
// per KB of code executed once per wave.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int N>
__global__ __launch_bounds__(256) void k_fat(float* out, float a, float c) {
  float x[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) x[q] = threadIdx.x * (q + 1);
#pragma unroll
  for (int i = 0; i < N; ++i) x[i & 7] = x[i & 7] * a + c;
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < 8; ++q) s += x[q];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_thin(float* out, float a, float c, int n) {
  float x[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) x[q] = threadIdx.x * (q + 1);
#pragma unroll 1
  for (int i = 0; i < n; i += 8) {
#pragma unroll
    for (int q = 0; q < 8; ++q) x[q] = x[q] * a + c;
  }
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < 8; ++q) s += x[q];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

float* d;
hipEvent_t e0, e1;
template <typename F> void run(const char* name, F launch) {
  const int R = 200;
  for (int i = 0; i < 20; ++i) launch();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int i = 0; i < R; ++i) launch();
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  printf("%-28s %9.2f us per launch\n", name, ms * 1e3 / R);
}

int main() {
  (void)hipMalloc(&d, 256 * 256 * sizeof(float));
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  dim3 g(256), b(256);
  run("empty-ish thin n=8", [&] { hipLaunchKernelGGL(k_thin, g, b, 0, 0, d, 0.999f, 1.f, 8); });
  run("thin n=3000", [&] { hipLaunchKernelGGL(k_thin, g, b, 0, 0, d, 0.999f, 1.f, 3000); });
  run("fat N=256", [&] { hipLaunchKernelGGL(k_fat<256>, g, b, 0, 0, d, 0.999f, 1.f); });
  run("fat N=512", [&] { hipLaunchKernelGGL(k_fat<512>, g, b, 0, 0, d, 0.999f, 1.f); });
  run("fat N=1024", [&] { hipLaunchKernelGGL(k_fat<1024>, g, b, 0, 0, d, 0.999f, 1.f); });
  run("fat N=2048", [&] { hipLaunchKernelGGL(k_fat<2048>, g, b, 0, 0, d, 0.999f, 1.f); });
  run("fat N=2304", [&] { hipLaunchKernelGGL(k_fat<2304>, g, b, 0, 0, d, 0.999f, 1.f); });
  run("fat N=2560", [&] { hipLaunchKernelGGL(k_fat<2560>, g, b, 0, 0, d, 0.999f, 1.f); });
  run("fat N=2816", [&] { hipLaunchKernelGGL(k_fat<2816>, g, b, 0, 0, d, 0.999f, 1.f); });
  run("fat N=3000", [&] { hipLaunchKernelGGL(k_fat<3000>, g, b, 0, 0, d, 0.999f, 1.f); });
  run("fat N=4096", [&] { hipLaunchKernelGGL(k_fat<4096>, g, b, 0, 0, d, 0.999f, 1.f); });
  run("fat N=3000, 1 workgroup", [&] { hipLaunchKernelGGL(k_fat<3000>, dim3(1), b, 0, 0, d, 0.999f, 1.f); });
  run("fat N=3000, 256 wg x 64", [&] { hipLaunchKernelGGL(k_fat<3000>, g, dim3(64), 0, 0, d, 0.999f, 1.f); });
  dim3 g1(1);
  run("fat N=2048, 1 workgroup", [&] { hipLaunchKernelGGL(k_fat<2048>, g1, b, 0, 0, d, 0.999f, 1.f); });
  run("thin n=2048, 1 workgroup", [&] { hipLaunchKernelGGL(k_thin, g1, b, 0, 0, d, 0.999f, 1.f, 2048); });
  return 0;
}
