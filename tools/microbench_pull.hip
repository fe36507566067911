// Operand pull rate of the MLP's GEMM tiles (layer-1 shape: C[M][N] = A[M][K]·B[N][K]ᵀ, f32,
// M = 500, K = 784), by fetch pattern.  Question: is a CU's pull rate set by the number of L2
// requests it keeps outstanding, so that a wave-instruction covering whole 128-B lines (8 rows ×
// 128 B) pulls faster than k_mm's 16 rows × 64 B?
//
//   d3 : k_mm's fetch — per wave its own k range, 16-k chunks, lane (lr, lg) loads row lr's
//        k0 + 4lg .. +3 (float4) straight into the MFMA operand registers, 3 chunks in flight
//   l2 / l3 : full-line fetch — 32-k chunks, lane (lane>>3, lane&7) loads row 8j + lane>>3,
//        k0 + 4·(lane&7) (8 rows × 128 B per instruction), staged through a wave-private LDS tile
//        (pitch 36 floats: conflict-free ds_write_b128 / ds_read_b128), 2 or 3 chunks in flight
//   p-d / p-l : the same two fetch patterns with no LDS and no MFMA (sum of the loaded values)
// Each kernel: 32×32 output tile per 8-wave workgroup, K split over the waves, LDS reduction.
// Grid = (M/32) × (N/32) workgroups; N = 256 (128 WGs), 512 (256), 1024 (512: two per CU).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>

typedef float f4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ inline f4 mfma(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

__device__ inline void reduce_store(f4 (&acc)[2][2], float (*red)[32][33], float* C, int M, int N, int m0, int n0) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15;
  __syncthreads();
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j)
      for (int q = 0; q < 4; ++q) red[wave][16 * i + (lane >> 4) * 4 + q][16 * j + lr] = acc[i][j][q];
  __syncthreads();
  for (int e = tid; e < 1024; e += 512) {
    const int mm = e >> 5, nn = e & 31;
    float v = red[0][mm][nn];
    for (int w = 1; w < 8; ++w) v += red[w][mm][nn];
    if (m0 + mm < M && n0 + nn < N) C[(size_t)(m0 + mm) * N + n0 + nn] = v;
  }
}

// k_mm's pattern: 16-k chunks, direct to registers, 3 in flight
__global__ __launch_bounds__(512) void k_d3(const float* A, const float* B, float* C, int M, int N, int K) {
  __shared__ float red[8][32][33];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  const int m0 = blockIdx.x * 32, n0 = blockIdx.y * 32;
  const int Kq = ((K + 127) / 128) * 16, kb = wave * Kq, ke = min(K, kb + Kq);
  f4 acc[2][2];
  for (int i = 0; i < 2; ++i) for (int j = 0; j < 2; ++j) acc[i][j] = f4{0, 0, 0, 0};
  f4 av[3][2], bv[3][2];
  auto load = [&](int s, int k0) {
    for (int i = 0; i < 2; ++i) {
      const int r = m0 + 16 * i + lr, c = n0 + 16 * i + lr, k = k0 + 4 * lg;
      const bool oka = r < M && k < ke, okb = c < N && k < ke;
      const f4 a = *reinterpret_cast<const f4*>(A + (oka ? (size_t)r * K + k : 0));
      const f4 b = *reinterpret_cast<const f4*>(B + (okb ? (size_t)c * K + k : 0));
      av[s][i] = oka ? a : f4{0, 0, 0, 0};
      bv[s][i] = okb ? b : f4{0, 0, 0, 0};
    }
  };
  auto mf = [&](int s) {
    for (int u = 0; u < 4; ++u)
      for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma(av[s][i][u], bv[s][j][u], acc[i][j]);
  };
  if (kb < ke) load(0, kb);
  if (kb + 16 < ke) load(1, kb + 16);
  if (kb + 32 < ke) load(2, kb + 32);
  for (int k0 = kb; k0 < ke; k0 += 48) {
    mf(0);
    if (k0 + 48 < ke) load(0, k0 + 48);
    if (k0 + 16 < ke) { mf(1); if (k0 + 64 < ke) load(1, k0 + 64); }
    if (k0 + 32 < ke) { mf(2); if (k0 + 80 < ke) load(2, k0 + 80); }
  }
  reduce_store(acc, red, C, M, N, m0, n0);
}

// full-line pattern: 32-k chunks (8 rows × 128 B per load instruction), wave-private LDS tile, D in flight
constexpr int SP = 36;                                  // LDS pitch (floats)
template <int D>
__global__ __launch_bounds__(512) void k_l(const float* A, const float* B, float* C, int M, int N, int K) {
  __shared__ float st[8][2][32][SP];                   // per wave: A and B tiles of one 32-k chunk (73.7 KB)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  const int rr = lane >> 3, kc = lane & 7;
  const int m0 = blockIdx.x * 32, n0 = blockIdx.y * 32;
  const int Kq = ((K + 255) / 256) * 32, kb = wave * Kq, ke = min(K, kb + Kq);
  f4 acc[2][2];
  for (int i = 0; i < 2; ++i) for (int j = 0; j < 2; ++j) acc[i][j] = f4{0, 0, 0, 0};
  f4 ra[D][4], rb[D][4];
  auto load = [&](int s, int k0) {
    const int k = k0 + 4 * kc;
    for (int j = 0; j < 4; ++j) {
      const int r = m0 + 8 * j + rr, c = n0 + 8 * j + rr;
      const bool oka = r < M && k < ke, okb = c < N && k < ke;
      const f4 a = *reinterpret_cast<const f4*>(A + (oka ? (size_t)r * K + k : 0));
      const f4 b = *reinterpret_cast<const f4*>(B + (okb ? (size_t)c * K + k : 0));
      ra[s][j] = oka ? a : f4{0, 0, 0, 0};
      rb[s][j] = okb ? b : f4{0, 0, 0, 0};
    }
  };
  float(*sa)[SP] = st[wave][0];
  float(*sb)[SP] = st[wave][1];
  auto compute = [&](int s) {
    for (int j = 0; j < 4; ++j) {
      *reinterpret_cast<f4*>(&sa[8 * j + rr][4 * kc]) = ra[s][j];
      *reinterpret_cast<f4*>(&sb[8 * j + rr][4 * kc]) = rb[s][j];
    }
    for (int h = 0; h < 2; ++h) {
      f4 a[2], b[2];
      for (int i = 0; i < 2; ++i) {
        a[i] = *reinterpret_cast<const f4*>(&sa[16 * i + lr][16 * h + 4 * lg]);
        b[i] = *reinterpret_cast<const f4*>(&sb[16 * i + lr][16 * h + 4 * lg]);
      }
      for (int u = 0; u < 4; ++u)
        for (int i = 0; i < 2; ++i)
          for (int j = 0; j < 2; ++j) acc[i][j] = mfma(a[i][u], b[j][u], acc[i][j]);
    }
  };
  for (int s = 0; s < D; ++s) if (kb + 32 * s < ke) load(s, kb + 32 * s);
  for (int k0 = kb; k0 < ke; k0 += 32 * D) {
#pragma unroll
    for (int s = 0; s < D; ++s) {
      if (k0 + 32 * s < ke) {
        compute(s);
        if (k0 + 32 * (s + D) < ke) load(s, k0 + 32 * (s + D));
      }
    }
  }
  __syncthreads();                                     // the reduction reuses the staging LDS
  reduce_store(acc, reinterpret_cast<float(*)[32][33]>(&st[0][0][0][0]), C, M, N, m0, n0);
}

// pull only: the same two patterns, every loaded value summed (no LDS, no MFMA)
template <int FULL>
__global__ __launch_bounds__(512) void k_pull(const float* A, const float* B, float* C, int M, int N, int K) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  const int rr = lane >> 3, kc = lane & 7;
  const int m0 = blockIdx.x * 32, n0 = blockIdx.y * 32;
  const int CH = FULL ? 32 : 16;
  const int Kq = ((K + 8 * CH - 1) / (8 * CH)) * CH, kb = wave * Kq, ke = min(K, kb + Kq);
  f4 s = f4{0, 0, 0, 0};
  for (int k0 = kb; k0 < ke; k0 += 3 * CH) {
    f4 v[3][8];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int j = 0; j < (FULL ? 4 : 2); ++j) {
        const int k = FULL ? k0 + c * CH + 4 * kc : k0 + c * CH + 4 * lg;
        const int r = FULL ? m0 + 8 * j + rr : m0 + 16 * j + lr;
        const int cc = FULL ? n0 + 8 * j + rr : n0 + 16 * j + lr;
        const bool oka = r < M && k < ke, okb = cc < N && k < ke;
        v[c][2 * j] = *reinterpret_cast<const f4*>(A + (oka ? (size_t)r * K + k : 0));
        v[c][2 * j + 1] = *reinterpret_cast<const f4*>(B + (okb ? (size_t)cc * K + k : 0));
      }
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int j = 0; j < (FULL ? 8 : 4); ++j) s += v[c][j];
  }
  if (s[0] + s[1] + s[2] + s[3] == 12345.f) C[tid] = s[0];
}

typedef void (*Kern)(const float*, const float*, float*, int, int, int);

static double cpu_check(const std::vector<float>& A, const std::vector<float>& B, const std::vector<float>& C,
                        int M, int N, int K) {
  double err = 0;
  for (int m = 0; m < M; m += 37)
    for (int n = 0; n < N; n += 13) {
      double s = 0;
      for (int k = 0; k < K; ++k) s += (double)A[(size_t)m * K + k] * B[(size_t)n * K + k];
      err = fmax(err, fabs(s - C[(size_t)m * N + n]));
    }
  return err;
}

int main(int argc, char** argv) {
  const int M = 500, K = 784, reps = argc > 1 ? atoi(argv[1]) : 400;
  const int Ns[3] = {256, 512, 1024};
  struct V { const char* name; Kern k; bool check; };
  V vs[] = {{"d3 (k_mm fetch)", k_d3, true}, {"l2 (full lines, LDS, 2 in flight)", k_l<2>, true},
            {"l3 (full lines, LDS, 3 in flight)", k_l<3>, true},
            {"p-d (pull only, k_mm pattern)", k_pull<0>, false}, {"p-l (pull only, full lines)", k_pull<1>, false}};
  std::vector<float> hA((size_t)M * K), hB((size_t)1024 * K);
  srand(1);
  for (auto& x : hA) x = (float)rand() / RAND_MAX - 0.5f;
  for (auto& x : hB) x = (float)rand() / RAND_MAX - 0.5f;
  float *A, *B, *C;
  CHECK(hipMalloc(&A, hA.size() * 4));
  CHECK(hipMalloc(&B, hB.size() * 4));
  CHECK(hipMalloc(&C, (size_t)M * 1024 * 4));
  CHECK(hipMemcpy(A, hA.data(), hA.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(B, hB.data(), hB.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int ni = 0; ni < 3; ++ni) {
    const int N = Ns[ni];
    dim3 grid((M + 31) / 32, N / 32);
    const double bytes_wg = 64.0 * K * 4;              // 32 rows of A + 32 rows of B over the whole K
    for (const V& v : vs) {
      for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(v.k, grid, dim3(512), 0, 0, A, B, C, M, N, K);
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(e0));
      for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(v.k, grid, dim3(512), 0, 0, A, B, C, M, N, K);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double us = 1e3 * ms / reps;
      double err = -1;
      if (v.check) {
        std::vector<float> hC((size_t)M * N);
        CHECK(hipMemcpy(hC.data(), C, hC.size() * 4, hipMemcpyDeviceToHost));
        err = cpu_check(hA, hB, hC, M, N, K);
      }
      printf("N=%4d WGs=%3d  %-36s %7.2f us/launch (incl. boundary)  %.1f KB/WG  max|err| %.2e\n", N,
             grid.x * grid.y, v.name, us, bytes_wg / 1024, err);
    }
  }
  return 0;
}
