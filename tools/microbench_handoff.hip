// Team hand-off round cost on MI355X: G = Gr x Gf workgroups (256 threads), rounds alternate
// between row teams (Gf members) and feature teams (Gr members); every member publishes P values
// and gathers the P values of every team member.  Reports µs per round for three transports:
//   0: tagged 16-B granules, every thread polls its own granules (sc1 loads, s_sleep between passes)
//   1: tagged 16-B granules, lane 0 of each producer slice polls ONE granule per producer first,
//      then all threads load once and re-poll only misses
//   2: sc1 payload + vmcnt(0) + workgroup barrier + one agent atomic per producer on the team
//      counter; lane 0 polls the counter, then every thread loads the payload (sc1)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("ERR %s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
typedef unsigned int g4 __attribute__((ext_vector_type(4)));

struct Args {
  int Gr, Gf, P, rounds, mode;
  char* arena; int arena_bytes;
  unsigned* ctr;
  unsigned long long* out;
  double* sink;
};

__device__ inline __amdgpu_buffer_rsrc_t mk(char* p, int n) { return __builtin_amdgcn_make_buffer_rsrc(p, 0, n, 0x00020000); }

__global__ __launch_bounds__(256) void k_handoff(Args a) {
  const int tid = threadIdx.x, bid = blockIdx.x;
  const int r = bid / a.Gf, f = bid % a.Gf, G = a.Gr * a.Gf;
  const __amdgpu_buffer_rsrc_t rs = mk(a.arena, a.arena_bytes);
  __shared__ double acc[1024];
  __shared__ int okflag;
  double sum = 0.0;
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < a.rounds; ++it) {
    const unsigned ep = it + 1;
    const bool rowround = (it & 1) == 0;
    const int team = rowround ? r : f;
    const int me = rowround ? f : r;
    const int np = rowround ? a.Gf : a.Gr;
    const int par = it & 1;
    // region of (par, team kind, team, member): P granules
    const int tbase = ((par * 2 + (rowround ? 0 : 1)) * 16 + team) * 16;   // member index added below
    // publish
    for (int e = tid; e < a.P; e += 256) {
      const double v = (double)(bid * 1000 + e + it);
      const unsigned long long x = __builtin_bit_cast(unsigned long long, v);
      g4 w = {(unsigned)x, ep, (unsigned)(x >> 32), ep};
      __builtin_amdgcn_raw_buffer_store_b128(w, rs, ((tbase + me) * a.P + e) * 16, 0, 16);
    }
    if (a.mode == 2) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      unsigned* c = a.ctr + (rowround ? 0 : 32) + team;
      if (tid == 0) {
        __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned target = (unsigned)(it / 2 + 1) * np;
        while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) __builtin_amdgcn_s_sleep(1);
      }
      __syncthreads();
      const int n = np * a.P;
      for (int j = tid; j < n; j += 256) {
        const int p = j / a.P, e = j - p * a.P;
        g4 w = __builtin_amdgcn_raw_buffer_load_b128(rs, ((tbase + p) * a.P + e) * 16, 0, 16);
        sum += __builtin_bit_cast(double, (unsigned long long)w.x | ((unsigned long long)w.z << 32));
      }
    } else {
      if (a.mode == 1) {
        // one lane per producer polls that producer's last granule
        if (tid < np) {
          const int off = ((tbase + tid) * a.P + a.P - 1) * 16;
          for (;;) {
            g4 w = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16);
            if (w.y == ep && w.w == ep) break;
            __builtin_amdgcn_s_sleep(1);
          }
        }
        __syncthreads();
      }
      const int n = np * a.P;
      for (int base = 0; base < n; base += 256 * 8) {
        g4 v[8];
        int o[8];
        unsigned pend = 0;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int j = base + tid + u * 256;
          o[u] = 0;
          if (j < n) {
            const int p = j / a.P, e = j - p * a.P;
            o[u] = ((tbase + p) * a.P + e) * 16;
            pend |= 1u << u;
          }
        }
        while (pend) {
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if (pend & (1u << u)) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, o[u], 0, 16);
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if ((pend & (1u << u)) && v[u].y == ep && v[u].w == ep) {
              sum += __builtin_bit_cast(double, (unsigned long long)v[u].x | ((unsigned long long)v[u].z << 32));
              pend &= ~(1u << u);
            }
          if (pend) __builtin_amdgcn_s_sleep(1);
        }
      }
    }
    acc[tid] = sum;
    __syncthreads();
  }
  unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) a.out[bid] = t1 - t0;
  a.sink[bid * 256 + tid] = sum + acc[(tid + 1) & 255];
}

int main(int argc, char** argv) {
  const int rounds = 2000;
  char* arena;
  const int arena_bytes = 2 * 2 * 16 * 16 * 1200 * 16;
  CK(hipMalloc(&arena, arena_bytes));
  unsigned* ctr;
  CK(hipMalloc(&ctr, 64 * 4));
  unsigned long long* out;
  CK(hipMalloc(&out, 256 * 8));
  double* sink;
  CK(hipMalloc(&sink, 256 * 256 * 8));
  const int grids[][2] = {{4, 4}, {8, 8}, {16, 8}, {8, 16}};
  const int Ps[] = {8, 80, 130, 640};
  for (auto& g : grids)
    for (int P : Ps)
      for (int mode = 0; mode < 3; ++mode) {
        Args a{g[0], g[1], P, rounds, mode, arena, arena_bytes, ctr, out, sink};
        CK(hipMemset(arena, 0, arena_bytes));
        CK(hipMemset(ctr, 0, 64 * 4));
        void* args[] = {&a};
        CK(hipLaunchCooperativeKernel((const void*)k_handoff, dim3(g[0] * g[1]), dim3(256), args, 0, 0));
        CK(hipDeviceSynchronize());
        unsigned long long h[256];
        CK(hipMemcpy(h, out, 256 * 8, hipMemcpyDeviceToHost));
        unsigned long long mx = 0;
        for (int i = 0; i < g[0] * g[1]; ++i) mx = h[i] > mx ? h[i] : mx;
        printf("grid %2dx%-2d P=%4d mode %d: %.3f us/round\n", g[0], g[1], P, mode, mx / 100.0 / rounds);
      }
  return 0;
}
