// Operand layout and rate of v_mfma_f64_4x4x4_4b_f64 on gfx950 (for the row-space kernel's G·d,
// csrc/hmcx_rowspace.hip): for every lane la, A = one-hot at la (B = 1) shows which output lanes the
// A value of lane la feeds; B = one-hot at la (A = 1) likewise.  Then the cycles per instruction for a
// dependent chain and for 4 independent chains, and the same for v_mfma_f64_16x16x4.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("ERR %s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void k_layout(double* outA, double* outB) {
  const int l = threadIdx.x;
  for (int la = 0; la < 64; ++la) {
    double d = __builtin_amdgcn_mfma_f64_4x4x4f64(l == la ? 1.0 : 0.0, 1.0, 0.0, 0, 0, 0);
    outA[la * 64 + l] = d;
    d = __builtin_amdgcn_mfma_f64_4x4x4f64(1.0, l == la ? 1.0 : 0.0, 0.0, 0, 0, 0);
    outB[la * 64 + l] = d;
  }
}

__global__ void k_rate(unsigned long long* t, double* sink, int n) {
  const int l = threadIdx.x;
  double a = 1.0 + l * 1e-9, b = 1.0 - l * 1e-9;
  double c0 = 0, c1 = 0, c2 = 0, c3 = 0;
  d4 e0 = {0, 0, 0, 0}, e1 = {0, 0, 0, 0};
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) c0 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c0, 0, 0, 0);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c3, 0, 0, 0);
  }
  unsigned long long t2 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
    e0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, e0, 0, 0, 0);
    e1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, e1, 0, 0, 0);
  }
  unsigned long long t3 = __builtin_amdgcn_s_memtime();
  if (l == 0) { t[0] = t1 - t0; t[1] = t2 - t1; t[2] = t3 - t2; }
  sink[l] = c0 + c1 + c2 + c3 + e0[0] + e1[1];
}

int main() {
  double *dA, *dB, *sink;
  unsigned long long* dt;
  CK(hipMalloc(&dA, 64 * 64 * 8));
  CK(hipMalloc(&dB, 64 * 64 * 8));
  CK(hipMalloc(&sink, 64 * 8));
  CK(hipMalloc(&dt, 3 * 8));
  hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, 0, dA, dB);
  CK(hipDeviceSynchronize());
  static double hA[64 * 64], hB[64 * 64];
  CK(hipMemcpy(hA, dA, sizeof(hA), hipMemcpyDeviceToHost));
  CK(hipMemcpy(hB, dB, sizeof(hB), hipMemcpyDeviceToHost));
  for (int la = 0; la < 64; ++la) {
    printf("A lane %2d feeds:", la);
    for (int l = 0; l < 64; ++l) if (hA[la * 64 + l] != 0.0) printf(" %d", l);
    printf("   | B lane %2d feeds:", la);
    for (int l = 0; l < 64; ++l) if (hB[la * 64 + l] != 0.0) printf(" %d", l);
    printf("\n");
  }
  const int n = 4096;
  hipLaunchKernelGGL(k_rate, dim3(1), dim3(64), 0, 0, dt, sink, n);
  CK(hipDeviceSynchronize());
  unsigned long long h[3];
  CK(hipMemcpy(h, dt, sizeof(h), hipMemcpyDeviceToHost));
  printf("s_memtime ticks per instruction: 4x4x4 dependent %.2f, 4x4x4 four chains %.2f, 16x16x4 two chains %.2f\n",
         (double)h[0] / n, (double)h[1] / (4.0 * n), (double)h[2] / (2.0 * n));
  return 0;
}
