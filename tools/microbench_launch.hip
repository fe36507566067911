// Microbenchmark: dependent-kernel launch floor vs in-kernel grid barrier cost on MI355X.
// Decides whether the SGHMC leapfrog should be kernel-per-phase or a persistent kernel.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("ERR %s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_empty(int* p) { if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345) p[1] = 1; }

__global__ void k_big_args(int* p, double a0, double a1, double a2, double a3, double a4, double a5, double a6,
                           double a7, double a8, double a9, double a10, double a11, double a12, double a13) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345) p[1] = (int)(a0 + a13);
}

// grid barrier: monotone counter, lane-0 release/acquire (agent), bounded spin
__device__ inline bool grid_sync(unsigned* ctr, unsigned target) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    long spins = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > 20000000) return false;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
  return true;
}

__global__ void k_persist(unsigned* ctr, int rounds, int* fail) {
  for (int r = 1; r <= rounds; ++r) {
    if (!grid_sync(ctr, (unsigned)r * gridDim.x)) { if (threadIdx.x == 0) atomicAdd(fail, 1); return; }
  }
}

int main() {
  int* d;
  CK(hipMalloc(&d, 64));
  CK(hipMemset(d, 0, 64));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int N = 4000;
  for (int blocks : {1, 64, 256}) {
    for (int pass = 0; pass < 2; ++pass) {
      CK(hipStreamSynchronize(s));
      auto t0 = std::chrono::high_resolution_clock::now();
      for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(256), 0, s, d);
      auto t1 = std::chrono::high_resolution_clock::now();
      CK(hipStreamSynchronize(s));
      auto t2 = std::chrono::high_resolution_clock::now();
      if (pass) printf("eager own-stream  blocks=%3d: enqueue %.2f us/launch, wall %.2f us/launch\n", blocks,
                       std::chrono::duration<double, std::micro>(t1 - t0).count() / N,
                       std::chrono::duration<double, std::micro>(t2 - t0).count() / N);
    }
  }
  for (int pass = 0; pass < 2; ++pass) {
    CK(hipDeviceSynchronize());
    auto t0 = std::chrono::high_resolution_clock::now();
    for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_empty, dim3(64), dim3(256), 0, 0, d);
    CK(hipDeviceSynchronize());
    auto t2 = std::chrono::high_resolution_clock::now();
    if (pass) printf("eager null-stream blocks= 64: wall %.2f us/launch\n",
                     std::chrono::duration<double, std::micro>(t2 - t0).count() / N);
  }
  for (int pass = 0; pass < 2; ++pass) {
    CK(hipStreamSynchronize(s));
    auto t0 = std::chrono::high_resolution_clock::now();
    for (int i = 0; i < N; ++i)
      hipLaunchKernelGGL(k_big_args, dim3(64), dim3(256), 0, s, d, 1., 2., 3., 4., 5., 6., 7., 8., 9., 10., 11., 12.,
                         13., 14.);
    CK(hipStreamSynchronize(s));
    auto t2 = std::chrono::high_resolution_clock::now();
    if (pass) printf("eager own-stream 120B args:   wall %.2f us/launch\n",
                     std::chrono::duration<double, std::micro>(t2 - t0).count() / N);
  }
  // graph of N dependent launches
  {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < 1000; ++i) hipLaunchKernelGGL(k_empty, dim3(64), dim3(256), 0, s, d);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int pass = 0; pass < 3; ++pass) {
      CK(hipStreamSynchronize(s));
      auto t0 = std::chrono::high_resolution_clock::now();
      CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      auto t2 = std::chrono::high_resolution_clock::now();
      if (pass) printf("graph 1000 nodes  blocks= 64: wall %.2f us/node\n",
                       std::chrono::duration<double, std::micro>(t2 - t0).count() / 1000);
    }
  }
  // persistent kernel barrier
  unsigned* ctr;
  int* fail;
  CK(hipMalloc(&ctr, 4));
  CK(hipMalloc(&fail, 4));
  for (int G : {8, 16, 32, 64, 128, 256}) {
    for (int pass = 0; pass < 2; ++pass) {
      CK(hipMemset(ctr, 0, 4));
      CK(hipMemset(fail, 0, 4));
      CK(hipDeviceSynchronize());
      const int R = 2000;
      auto t0 = std::chrono::high_resolution_clock::now();
      hipLaunchKernelGGL(k_persist, dim3(G), dim3(256), 0, s, ctr, R, fail);
      CK(hipStreamSynchronize(s));
      auto t2 = std::chrono::high_resolution_clock::now();
      int f = 0;
      CK(hipMemcpy(&f, fail, 4, hipMemcpyDeviceToHost));
      if (pass) printf("persistent barrier G=%3d: %.2f us/barrier (fail=%d)\n", G,
                       std::chrono::duration<double, std::micro>(t2 - t0).count() / R, f);
    }
  }
  return 0;
}
