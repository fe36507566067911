// Layer-2 GEMM of the MLP's forwards (config 3: h2 = h1·W2ᵀ, B = 500, n_mid = 256, f32), by tiling.
// Question: can one workgroup own 16 whole rows (all 256 columns, so layer 3 needs no cross-workgroup
// exchange) and still finish the six forwards of a leapfrog iteration in one short launch?
//
//   rowblock : grid (32 row blocks of 16) × P problems; the 16 × 256 h1 tile in LDS (A), wave w computes
//              columns 32w … 32w+31 over K = 256 with W2 rows read straight from global (B, float4 along k)
//   tile32   : k_mm's tiling for comparison: 32 × 32 output tile per workgroup, K split over the 8 waves
//              (direct float4 loads of both operands, LDS reduction), grid 16 × 8 × P
// Problems alternate between two W2 matrices (as the old / new W2 of a batched iteration).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>

typedef float f4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
__device__ inline f4 mfma(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

constexpr int NM = 256, AP = NM + 4;                   // n_mid, LDS pitch of the A tile (floats)

template <int RING, int STAG>
__global__ __launch_bounds__(512) void k_rowblock(const float* H, const float* W2a, const float* W2b, float* C, int M) {
  __shared__ float At[16][AP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  const int m0 = blockIdx.x * 16, p = blockIdx.y;
  const float* W2 = (p & 1) ? W2b : W2a;
  // A tile: 16 rows × 256 (two float4 per thread)
  for (int e = tid; e < 16 * NM / 4; e += 512) {
    const int r = e / (NM / 4), c4 = e % (NM / 4);
    const bool ok = m0 + r < M;
    const f4 v = *reinterpret_cast<const f4*>(H + (size_t)p * M * NM + (ok ? (size_t)(m0 + r) * NM : 0) + 4 * c4);
    *reinterpret_cast<f4*>(&At[r][4 * c4]) = ok ? v : f4{0, 0, 0, 0};
  }
  const int n0 = 32 * wave;
  f4 acc[2] = {f4{0, 0, 0, 0}, f4{0, 0, 0, 0}};
  f4 bv[RING][2];
  // STAG: every workgroup walks the k chunks from its own starting chunk (blockIdx-dependent), so the 24
  // workgroups of an XCD do not all request the same W2 lines together
  const int c0 = STAG ? (int)(blockIdx.x * 5 + blockIdx.y * 3) % (NM / 16) : 0;
  auto load = [&](int s, int k0) {
    k0 = (k0 + 16 * c0) % NM;
    for (int j = 0; j < 2; ++j) bv[s][j] = *reinterpret_cast<const f4*>(W2 + (size_t)(n0 + 16 * j + lr) * NM + k0 + 4 * lg);
  };
  for (int s = 0; s < RING; ++s) load(s, 16 * s);
  __syncthreads();
  for (int c = 0; c < NM / 16; c += RING) {
#pragma unroll
    for (int s = 0; s < RING; ++s) {
      const int k0 = (16 * (c + s + c0)) % NM;
      const f4 a = *reinterpret_cast<const f4*>(&At[lr][k0 + 4 * lg]);
      f4 b0 = bv[s][0], b1 = bv[s][1];
      if (c + s + RING < NM / 16) load(s, 16 * (c + s + RING));
      for (int u = 0; u < 4; ++u) {
        acc[0] = mfma(a[u], b0[u], acc[0]);
        acc[1] = mfma(a[u], b1[u], acc[1]);
      }
    }
  }
  for (int j = 0; j < 2; ++j)
    for (int q = 0; q < 4; ++q) {
      const int r = m0 + lg * 4 + q;
      if (r < M) C[(size_t)p * M * NM + (size_t)r * NM + n0 + 16 * j + lr] = acc[j][q];
    }
}

// 16 waves (1024 threads), wave w computes columns 16w … 16w+15: four waves per SIMD hide each other's loads
template <int RING>
__global__ __launch_bounds__(1024) void k_rowblock16(const float* H, const float* W2a, const float* W2b, float* C, int M) {
  __shared__ float At[16][AP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  const int m0 = blockIdx.x * 16, p = blockIdx.y;
  const float* W2 = (p & 1) ? W2b : W2a;
  {
    const int e = tid, r = e / (NM / 4), c4 = e % (NM / 4);
    const bool ok = m0 + r < M;
    const f4 v = *reinterpret_cast<const f4*>(H + (size_t)p * M * NM + (ok ? (size_t)(m0 + r) * NM : 0) + 4 * c4);
    *reinterpret_cast<f4*>(&At[r][4 * c4]) = ok ? v : f4{0, 0, 0, 0};
  }
  const int n0 = 16 * wave;
  f4 acc = f4{0, 0, 0, 0};
  f4 bv[RING];
  auto load = [&](int s, int k0) { bv[s] = *reinterpret_cast<const f4*>(W2 + (size_t)(n0 + lr) * NM + k0 + 4 * lg); };
  for (int s = 0; s < RING; ++s) load(s, 16 * s);
  __syncthreads();
  for (int c = 0; c < NM / 16; c += RING) {
#pragma unroll
    for (int s = 0; s < RING; ++s) {
      const int k0 = 16 * (c + s);
      const f4 a = *reinterpret_cast<const f4*>(&At[lr][k0 + 4 * lg]);
      f4 b = bv[s];
      if (c + s + RING < NM / 16) load(s, 16 * (c + s + RING));
      for (int u = 0; u < 4; ++u) acc = mfma(a[u], b[u], acc);
    }
  }
  for (int q = 0; q < 4; ++q) {
    const int r = m0 + lg * 4 + q;
    if (r < M) C[(size_t)p * M * NM + (size_t)r * NM + n0 + lr] = acc[q];
  }
}

__global__ __launch_bounds__(512) void k_tile32(const float* H, const float* W2a, const float* W2b, float* C, int M) {
  __shared__ float red[8][32][33];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  const int m0 = blockIdx.x * 32, n0 = blockIdx.y * 32, p = blockIdx.z;
  const float* W2 = (p & 1) ? W2b : W2a;
  const float* A = H + (size_t)p * M * NM;
  const int kb = wave * 32;
  f4 acc[2][2];
  for (int i = 0; i < 2; ++i) for (int j = 0; j < 2; ++j) acc[i][j] = f4{0, 0, 0, 0};
  f4 av[2][2], bv[2][2];
  for (int c = 0; c < 2; ++c)
    for (int i = 0; i < 2; ++i) {
      const int r = m0 + 16 * i + lr;
      av[c][i] = *reinterpret_cast<const f4*>(A + (size_t)(r < M ? r : 0) * NM + kb + 16 * c + 4 * lg);
      bv[c][i] = *reinterpret_cast<const f4*>(W2 + (size_t)(n0 + 16 * i + lr) * NM + kb + 16 * c + 4 * lg);
    }
  for (int c = 0; c < 2; ++c)
    for (int u = 0; u < 4; ++u)
      for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma(av[c][i][u], bv[c][j][u], acc[i][j]);
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j)
      for (int q = 0; q < 4; ++q) red[wave][16 * i + lg * 4 + q][16 * j + lr] = acc[i][j][q];
  __syncthreads();
  for (int e = tid; e < 1024; e += 512) {
    const int mm = e >> 5, nn = e & 31;
    float v = red[0][mm][nn];
    for (int w = 1; w < 8; ++w) v += red[w][mm][nn];
    if (m0 + mm < M) C[(size_t)p * M * NM + (size_t)(m0 + mm) * NM + n0 + nn] = v;
  }
}

int main(int argc, char** argv) {
  const int M = 500, reps = argc > 1 ? atoi(argv[1]) : 400, PMAX = 8;
  std::vector<float> hH((size_t)PMAX * M * NM), hW((size_t)2 * NM * NM);
  srand(3);
  for (auto& x : hH) x = (float)rand() / (float)RAND_MAX - 0.5f;
  for (auto& x : hW) x = (float)rand() / (float)RAND_MAX - 0.5f;
  float *H, *W, *C;
  CHECK(hipMalloc(&H, hH.size() * 4));
  CHECK(hipMalloc(&W, hW.size() * 4));
  CHECK(hipMalloc(&C, hH.size() * 4));
  CHECK(hipMemcpy(H, hH.data(), hH.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(W, hW.data(), hW.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto check = [&](int P) {
    std::vector<float> hC((size_t)P * M * NM);
    CHECK(hipMemcpy(hC.data(), C, hC.size() * 4, hipMemcpyDeviceToHost));
    double err = 0;
    for (int p = 0; p < P; ++p)
      for (int m = p; m < M; m += 41)
        for (int n = 3 * p; n < NM; n += 29) {
          double s = 0;
          for (int k = 0; k < NM; ++k) s += (double)hH[((size_t)p * M + m) * NM + k] * hW[((size_t)(p & 1) * NM + n) * NM + k];
          err = fmax(err, fabs(s - hC[((size_t)p * M + m) * NM + n]));
        }
    return err;
  };
  auto time = [&](const char* name, int P, auto launch) {
    for (int w = 0; w < 20; ++w) launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    printf("P=%d  %-34s %7.2f us/launch (incl. boundary)  max|err| %.2e\n", P, name, 1e3 * ms / reps, check(P));
  };
  for (int P : {1, 4, 6, 8}) {
    time("rowblock 16x256, ring 2", P, [&] {
      hipLaunchKernelGGL((k_rowblock<2, 0>), dim3((M + 15) / 16, P), dim3(512), 0, 0, H, W, W + NM * NM, C, M); });
    time("rowblock 16x256, ring 4", P, [&] {
      hipLaunchKernelGGL((k_rowblock<4, 0>), dim3((M + 15) / 16, P), dim3(512), 0, 0, H, W, W + NM * NM, C, M); });
    time("rowblock 16x256, ring 2, staggered", P, [&] {
      hipLaunchKernelGGL((k_rowblock<2, 1>), dim3((M + 15) / 16, P), dim3(512), 0, 0, H, W, W + NM * NM, C, M); });
    time("rowblock 16x256, ring 4, staggered", P, [&] {
      hipLaunchKernelGGL((k_rowblock<4, 1>), dim3((M + 15) / 16, P), dim3(512), 0, 0, H, W, W + NM * NM, C, M); });
    time("rowblock 16 waves, ring 4", P, [&] {
      hipLaunchKernelGGL((k_rowblock16<4>), dim3((M + 15) / 16, P), dim3(1024), 0, 0, H, W, W + NM * NM, C, M); });
    time("rowblock 16 waves, ring 8", P, [&] {
      hipLaunchKernelGGL((k_rowblock16<8>), dim3((M + 15) / 16, P), dim3(1024), 0, 0, H, W, W + NM * NM, C, M); });
    time("tile32 (k_mm tiling)", P, [&] {
      hipLaunchKernelGGL(k_tile32, dim3((M + 31) / 32, NM / 32, P), dim3(512), 0, 0, H, W, W + NM * NM, C, M); });
  }
  return 0;
}
