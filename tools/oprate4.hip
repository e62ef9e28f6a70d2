// Issue cost vs live lanes per wave and waves per SIMD (the step kernel's occupancy question).
// B = 65,536 envs on 1,024 SIMDs is 64 envs per SIMD: one full wave, or two waves of 32 live lanes,
// or four of 16.  For each split, time a fixed amount of per-env work (every live lane runs the
// same instruction stream) and report ns per 64-env instruction per SIMD.
//   indep : 8 independent xor chains (issue-bound)
//   dep   : 1 dependent xor chain (latency-bound)
//   lds   : dependent ds_read_b32 -> v_xor -> next address (LDS-latency-bound)
//   mix   : 6 independent xors + 1 dependent ds_read per group (roughly the step kernel's mix)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#define ITERS 2048

#define X(a) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"(b));

__global__ __launch_bounds__(256) void k_indep(uint32_t* out, uint32_t s, int live) {
  if ((int)(threadIdx.x & 63) >= live) return;
  uint32_t a0 = threadIdx.x ^ s, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 + 11u, a5 = a0 + 13u,
           a6 = a0 ^ 0x55u, a7 = a0 ^ 0xAAu, b = s | 1u;
  for (int i = 0; i < ITERS; ++i) { X(a0) X(a1) X(a2) X(a3) X(a4) X(a5) X(a6) X(a7) }
  out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ __launch_bounds__(256) void k_dep(uint32_t* out, uint32_t s, int live) {
  if ((int)(threadIdx.x & 63) >= live) return;
  uint32_t a0 = threadIdx.x ^ s, b = s | 1u;
  for (int i = 0; i < ITERS; ++i) { X(a0) X(a0) X(a0) X(a0) X(a0) X(a0) X(a0) X(a0) }
  out[blockIdx.x * 256 + threadIdx.x] = a0;
}

__global__ __launch_bounds__(256) void k_lds(uint32_t* out, uint32_t s, int live) {
  __shared__ uint32_t L[1024];
  for (int i = threadIdx.x; i < 1024; i += 256) L[i] = (uint32_t)(i * 4) ^ (s & 0);
  __syncthreads();
  if ((int)(threadIdx.x & 63) >= live) return;
  uint32_t a = 4u * threadIdx.x, b = 0;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      asm volatile("ds_read_b32 %0, %0\n s_waitcnt lgkmcnt(0)" : "+v"(a));
      X(a)
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = a;
}

__global__ __launch_bounds__(256) void k_mix(uint32_t* out, uint32_t s, int live) {
  __shared__ uint32_t L[1024];
  for (int i = threadIdx.x; i < 1024; i += 256) L[i] = (uint32_t)(i * 4);
  __syncthreads();
  if ((int)(threadIdx.x & 63) >= live) return;
  uint32_t a = 4u * threadIdx.x, b = s | 1u;
  uint32_t a0 = threadIdx.x ^ s, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 + 11u, a5 = a0 + 13u;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("ds_read_b32 %0, %0" : "+v"(a));
    X(a0) X(a1) X(a2) X(a3) X(a4) X(a5)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    X(a)
  }
  out[blockIdx.x * 256 + threadIdx.x] = a ^ a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5;
}

typedef void (*KF)(uint32_t*, uint32_t, int);
int main() {
  struct { const char* n; KF f; int insts; } ks[] = {
      {"indep", k_indep, 8}, {"dep", k_dep, 8}, {"lds", k_lds, 16}, {"mix", k_mix, 8}};
  struct { int wps, live; } splits[] = {{1, 64}, {2, 32}, {4, 16}, {8, 8}, {2, 64}, {4, 32}};
  uint32_t* out;
  (void)hipMalloc(&out, 8 * 1024 * 256 * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  setvbuf(stdout, NULL, _IONBF, 0);
  printf("ns per 64-env instruction per SIMD (1,024 SIMDs; waves/SIMD x live lanes)\n%-6s", "");
  for (auto& sp : splits) printf("  %dx%-5d", sp.wps, sp.live);
  printf("\n");
  for (auto& k : ks) {
    printf("%-6s", k.n);
    for (auto& sp : splits) {
      const int blocks = 256 * sp.wps;
      k.f<<<blocks, 256>>>(out, 7, sp.live);
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0);
      for (int r = 0; r < 5; ++r) k.f<<<blocks, 256>>>(out, 7, sp.live);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      ms /= 5;
      // 64-env instructions per SIMD = waves * live / 64 * ITERS * insts
      const double n64 = (double)sp.wps * sp.live / 64.0 * ITERS * k.insts;
      printf("  %7.3f", ms * 1e6 / n64);
    }
    printf("\n");
  }
  return 0;
}
