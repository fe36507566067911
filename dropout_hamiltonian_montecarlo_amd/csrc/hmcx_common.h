// hmcx_common.h — shared device/host helpers for the MI355X (gfx950) SG-HMC engine.
//
//  * Philox4x32-10 counter-based RNG (host + device; uniforms bit-identical), used in
//    HMCX_NOISE_PHILOX mode for momenta / SGHMC friction noise / SGLD noise and, on the
//    host, for path lengths and accept uniforms.  The reference draws these from
//    NumPy streams (cpu/sghmc.py:21,25,31,36; cpu/sgld.py:45); HMCX_NOISE_BUFFER mode
//    replays host-drawn NumPy normals instead, bit for bit.
//  * MFMA wrappers for the two dense GEMMs of the softmax gradient (softmax.py:39,54):
//    v_mfma_f64_16x16x4_f64 (parity dtype) and v_mfma_f32_16x16x4_f32 (fast dtype).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

namespace hmcx {

// ---------------------------------------------------------------- Philox4x32-10
struct u32x4 { uint32_t v[4]; };

__host__ __device__ inline u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one 32 × 32 → 64-bit product per multiplier: a single v_mad_u64_u32 on gfx950 instead of
    // v_mul_hi_u32 + v_mul_lo_u32 (tools/microbench_philox.hip: same words, 12–18 % more blocks/s)
    const uint64_t p0 = (uint64_t)M0 * c.v[0], p1 = (uint64_t)M1 * c.v[2];
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    u32x4 n;
    n.v[0] = hi1 ^ c.v[1] ^ k0;
    n.v[1] = lo1;
    n.v[2] = hi0 ^ c.v[3] ^ k1;
    n.v[3] = lo0;
    c = n;
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// 53-bit uniform in [0,1) from two 32-bit words.
__host__ __device__ inline double u53(uint32_t a, uint32_t b) {
  return (double)(((uint64_t)a << 21) ^ (uint64_t)(b >> 11)) * (1.0 / 9007199254740992.0);
}

// Counter layout: {element pair, slot, step, chain}; key = seed.
// slot 0 = momentum / SGLD noise, slot i+1 = leapfrog iteration i noise,
// SLOT_PATH / SLOT_ACCEPT = per-step uniforms.
constexpr uint32_t SLOT_PATH = 0xFFFFFFFEu;
constexpr uint32_t SLOT_ACCEPT = 0xFFFFFFFDu;

__host__ __device__ inline double philox_uniform(uint64_t seed, uint32_t chain, uint32_t step,
                                                 uint32_t slot, uint32_t idx) {
  u32x4 c = {{idx, slot, step, chain}};
  u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  return u53(r.v[0], r.v[1]);
}

// Standard normals, four per Philox block: element e uses block e>>2; words (0,1) feed the
// Box–Muller pair of elements 4b, 4b+1 (cos, sin) and words (2,3) that of 4b+2, 4b+3.
// The same formula runs on the host (hmcx_philox_normals) up to transcendental rounding (the
// device uses the hardware v_log/v_sin/v_cos approximations); device values are what the
// samplers use.
__host__ __device__ inline void box_muller(uint32_t w0, uint32_t w1, float& z0, float& z1) {
  const float u1 = ((float)(w0 >> 8) + 1.0f) * 5.9604644775390625e-08f;  // (0,1]
  const float u2 = (float)(w1 >> 8) * 5.9604644775390625e-08f;           // [0,1)
  const float th = 6.28318530717958647692f * u2;
#if defined(__HIP_DEVICE_COMPILE__)
  const float rad = __fsqrt_rn(-2.0f * __logf(u1));
  z0 = rad * __cosf(th);
  z1 = rad * __sinf(th);
#else
  const float rad = sqrtf(-2.0f * logf(u1));
  z0 = rad * cosf(th);
  z1 = rad * sinf(th);
#endif
}

__host__ __device__ inline void philox_normal4(uint64_t seed, uint32_t chain, uint32_t step, uint32_t slot,
                                               uint32_t blk, float z[4]) {
  u32x4 c = {{blk, slot, step, chain}};
  u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  box_muller(r.v[0], r.v[1], z[0], z[1]);
  box_muller(r.v[2], r.v[3], z[2], z[3]);
}

__host__ __device__ inline float philox_normal(uint64_t seed, uint32_t chain, uint32_t step,
                                               uint32_t slot, uint32_t e) {
  u32x4 c = {{e >> 2, slot, step, chain}};
  u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  float z0, z1;
  if (e & 2u) box_muller(r.v[2], r.v[3], z0, z1);
  else box_muller(r.v[0], r.v[1], z0, z1);
  return (e & 1u) ? z1 : z0;
}

// Float64 standard normals for the f64 chains (the reference draws f64 normals, cpu/sghmc.py:21,31,
// cpu/sgld.py:45): one Philox block = two 53-bit uniforms = one Box–Muller pair in double precision
// (u1 = (k+1)·2⁻⁵³ ∈ (0,1], so |z| reaches sqrt(2·53·ln 2) ≈ 8.57σ; θ = 2π·u2 via sincospi, no
// range reduction).  Element e uses the block with counter e >> 1 (e & 1 picks cos / sin), so four
// elements 4b..4b+3 are blocks 2b and 2b+1.
__host__ __device__ inline void box_muller_d(const u32x4& r, double& z0, double& z1) {
  const uint64_t k1 = ((uint64_t)r.v[0] << 21) ^ (uint64_t)(r.v[1] >> 11);
  const double u1 = (double)(k1 + 1) * (1.0 / 9007199254740992.0);       // (0,1]
  const double u2 = u53(r.v[2], r.v[3]);                                 // [0,1)
  const double rad = sqrt(-2.0 * log(u1));
  double s, c;
#if defined(__HIP_DEVICE_COMPILE__)
  sincospi(2.0 * u2, &s, &c);
#else
  const double th = 6.283185307179586476925 * u2;
  s = sin(th);
  c = cos(th);
#endif
  z0 = rad * c;
  z1 = rad * s;
}

__host__ __device__ inline void philox_normal4(uint64_t seed, uint32_t chain, uint32_t step, uint32_t slot,
                                               uint32_t blk, double z[4]) {
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  u32x4 c0 = {{2u * blk, slot, step, chain}}, c1 = {{2u * blk + 1u, slot, step, chain}};
  box_muller_d(philox4x32_10(c0, k0, k1), z[0], z[1]);
  box_muller_d(philox4x32_10(c1, k0, k1), z[2], z[3]);
}

// Elements 2·pair and 2·pair + 1 of the f64 stream.
__host__ __device__ inline void philox_pair_d(uint64_t seed, uint32_t chain, uint32_t step, uint32_t slot,
                                              uint32_t pair, double& z0, double& z1) {
  u32x4 c = {{pair, slot, step, chain}};
  box_muller_d(philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32)), z0, z1);
}

__host__ __device__ inline double philox_normal_d(uint64_t seed, uint32_t chain, uint32_t step,
                                                  uint32_t slot, uint32_t e) {
  u32x4 c = {{e >> 1, slot, step, chain}};
  double z0, z1;
  box_muller_d(philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32)), z0, z1);
  return (e & 1u) ? z1 : z0;
}

// Noise of a chain computing in T: f32 chains take the float Box–Muller above (24-bit uniforms,
// |z| ≤ 5.77σ, fast transcendentals), f64 chains the double one.
template <typename T> struct NormalT;
template <> struct NormalT<float> {
  __host__ __device__ static inline float one(uint64_t s, uint32_t c, uint32_t st, uint32_t sl, uint32_t e) {
    return philox_normal(s, c, st, sl, e);
  }
};
template <> struct NormalT<double> {
  __host__ __device__ static inline double one(uint64_t s, uint32_t c, uint32_t st, uint32_t sl, uint32_t e) {
    return philox_normal_d(s, c, st, sl, e);
  }
};
template <typename T>
__host__ __device__ inline T philox_normal_t(uint64_t seed, uint32_t chain, uint32_t step, uint32_t slot,
                                             uint32_t e) {
  return NormalT<T>::one(seed, chain, step, slot, e);
}

// ---------------------------------------------------------------- MFMA 16x16x4
// A[i][k]: lane l holds i = l&15, k = l>>4; B[k][j]: k = l>>4, j = l&15 (both dtypes).
// C/D: f32: row = (l>>4)*4 + r, col = l&15;  f64: row = (l>>4) + 4*r, col = l&15.
typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <typename T> struct mfma16;
template <> struct mfma16<double> {
  typedef d4 acc_t;
  __device__ static inline acc_t zero() { return acc_t{0.0, 0.0, 0.0, 0.0}; }
  __device__ static inline acc_t fma(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  __device__ static inline int row(int lane, int r) { return (lane >> 4) + 4 * r; }
};
template <> struct mfma16<float> {
  typedef f4 acc_t;
  __device__ static inline acc_t zero() { return acc_t{0.f, 0.f, 0.f, 0.f}; }
  __device__ static inline acc_t fma(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  __device__ static inline int row(int lane, int r) { return (lane >> 4) * 4 + r; }
};

// NaN-propagating min/max with NumPy semantics (np.minimum / np.maximum / np.max).
template <typename T> __device__ inline T np_min(T a, T b) { return (a != a) ? a : ((b < a) ? b : a); }
template <typename T> __device__ inline T np_max(T a, T b) { return (a != a) ? a : ((b > a) ? b : a); }
template <typename T> __device__ inline T max_nan(T m, T z) { return (z > m || z != z) ? z : m; }
// softmax.py:40-41: np.maximum(np.minimum(z, hi), lo)
template <typename T> __device__ inline T clipz(T z, T hi, T lo) { return np_max(np_min(z, hi), lo); }

}  // namespace hmcx
