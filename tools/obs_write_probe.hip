// Write-phase probe for a fused sampler kernel (round 4): how fast can a workgroup of THREADS lanes
// stream the f32 observation rows of ENVS envs (Medium-8: 8 rows x 82 floats per env) gathered from
// per-env byte images in LDS, as k_observe's write loop does?  Shapes: k_observe's own (256 lanes,
// 16 envs) against the shapes a fused step + rows kernel would have (512 / 1024 lanes, 256 envs,
// one workgroup per CU).  MODE 0: gather from LDS (k_observe's loop); MODE 1: the same with the LDS
// reads of U iterations issued before their stores; MODE 2: stores of a constant (no gathers).
//   hipcc --offload-arch=gfx950 -O3 tools/obs_write_probe.hip -o tools/obs_write_probe_bin
//   hipcc --offload-arch=gfx950 -O3 -DPROBE_LARGE tools/obs_write_probe.hip -o tools/obs_write_probe_large   (Large-16 rows)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

#ifdef PROBE_LARGE   // Large-16 rows: 16 x 145 floats per env (round 6: what bounds k_observe<Large>?)
constexpr int NA = 16, L = 145, IMG = 148, PER_ENV = NA * L, QE = PER_ENV / 4;   // 580 float4 per env
#else
constexpr int NA = 8, L = 82, IMG = 84, PER_ENV = NA * L, QE = PER_ENV / 4;   // 164 float4 per env
#endif
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ void st(f32x4* p, f32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <int THREADS, int ENVS, int MODE, int U, bool NT>
__global__ __launch_bounds__(THREADS) void k_probe(float* __restrict__ obs, int64_t B) {
  __shared__ uint8_t img[ENVS][IMG];
  __shared__ uint32_t lim[ENVS];
  __shared__ uint32_t src[QE];
  const int tid = threadIdx.x;
  for (int k = tid; k < ENVS * IMG; k += THREADS) (&img[0][0])[k] = (uint8_t)((k * 7) & 31);
  for (int k = tid; k < ENVS; k += THREADS) lim[k] = PER_ENV - 4 * (k & 3);
  for (int k = tid; k < QE; k += THREADS) {
    uint32_t w = 0;
    for (int b = 0; b < 4; ++b) w |= (uint32_t)((4 * k + b) % L) << (8 * b);
    src[k] = w;
  }
  __syncthreads();
  const int64_t e0 = (int64_t)blockIdx.x * ENVS;
  const uint32_t nenv = (uint32_t)((B - e0) < ENVS ? (B - e0) : ENVS);
  const uint32_t total = nenv * QE;
  const uint32_t magic = 0xFFFFFFFFu / QE + 1u;
  f32x4* out4 = reinterpret_cast<f32x4*>(obs + e0 * PER_ENV);
  if (MODE == 2) {
    for (uint32_t q = tid; q < total; q += THREADS) st<NT>(&out4[q], (f32x4){1.0f, 2.0f, 3.0f, 4.0f});
    return;
  }
  auto value = [&](uint32_t q) -> f32x4 {
    const uint32_t el4 = __umulhi(q, magic);
    const uint32_t k4 = q - el4 * QE;
    const uint32_t lm = lim[el4];
    const uint32_t sw = src[k4];
    const int live = (int)lm - 4 * (int)k4;
    const uint8_t* im = img[el4];
    f32x4 v;
    v.x = live > 0 ? (float)im[sw & 0xFFu] : 0.0f;
    v.y = live > 1 ? (float)im[(sw >> 8) & 0xFFu] : 0.0f;
    v.z = live > 2 ? (float)im[(sw >> 16) & 0xFFu] : 0.0f;
    v.w = live > 3 ? (float)im[sw >> 24] : 0.0f;
    return v;
  };
  if (MODE == 0) {
    for (uint32_t q = tid; q < total; q += THREADS) st<NT>(&out4[q], value(q));
  } else {
    uint32_t q = tid;
    for (; q + (U - 1) * THREADS < total; q += U * THREADS) {
      f32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = value(q + u * THREADS);
#pragma unroll
      for (int u = 0; u < U; ++u) st<NT>(&out4[q + u * THREADS], v[u]);
    }
    for (; q < total; q += THREADS) st<NT>(&out4[q], value(q));
  }
}

// Persistent form (round 6, Large rows): GRID workgroups; CONTIG: workgroup w writes the groups of
// envs [w * B / GRID, (w + 1) * B / GRID) in order (one long sequential stream per workgroup), else
// groups w, w + GRID, ... (interleaved).  Constant stores: the write shape alone.
template <int THREADS, int ENVS, bool CONTIG, bool NT>
__global__ __launch_bounds__(THREADS) void k_probe_p(float* __restrict__ obs, int64_t B) {
  const int tid = threadIdx.x;
  const int64_t ng = (B + ENVS - 1) / ENVS;
  const int64_t per = (ng + gridDim.x - 1) / gridDim.x;
  const int64_t g0 = CONTIG ? blockIdx.x * per : blockIdx.x;
  const int64_t g1 = CONTIG ? (g0 + per < ng ? g0 + per : ng) : ng;
  const int64_t gs = CONTIG ? 1 : gridDim.x;
  for (int64_t g = g0; g < g1; g += gs) {
    f32x4* out4 = reinterpret_cast<f32x4*>(obs + g * ENVS * PER_ENV);
    for (uint32_t q = tid; q < (uint32_t)(ENVS * QE); q += THREADS) st<NT>(&out4[q], (f32x4){1.0f, 2.0f, 3.0f, 4.0f});
  }
}

// Grid-stride sweep over the whole buffer (the fill_ / memset pattern): U stores per iteration.
template <int THREADS, int U, bool NT>
__global__ __launch_bounds__(THREADS) void k_sweep(float* __restrict__ obs, int64_t n4) {
  f32x4* out4 = reinterpret_cast<f32x4*>(obs);
  const int64_t stride = (int64_t)gridDim.x * THREADS;
  for (int64_t q = (int64_t)blockIdx.x * THREADS + threadIdx.x; q < n4; q += U * stride) {
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (q + u * stride < n4) st<NT>(&out4[q + u * stride], (f32x4){1.0f, 2.0f, 3.0f, 4.0f});
  }
}

template <int THREADS, int U, bool NT>
void run_s(float* obs, int64_t B, unsigned grid, const char* name) {
  const int64_t n4 = B * (int64_t)QE;
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_sweep<THREADS, U, NT>), dim3(grid), dim3(THREADS), 0, 0, obs, n4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    hipEventRecord(a, 0);
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL((k_sweep<THREADS, U, NT>), dim3(grid), dim3(THREADS), 0, 0, obs, n4);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    best = ms / 20 < best ? ms / 20 : best;
  }
  const double bytes = (double)B * PER_ENV * 4;
  printf("%-44s threads=%4d unroll=%d grid=%6u: %7.2f us  %6.2f TB/s\n", name, THREADS, U, grid, best * 1e3,
         bytes / (best * 1e-3) / 1e12);
}

// No loop: workgroup w writes the U * THREADS float4s [w * U * THREADS, (w + 1) * U * THREADS), U
// stores per lane issued back to back, workgroups in dispatch order (the stores in flight form one
// moving window of about resident-workgroups x U x 4 KB).
template <int THREADS, int U, bool NT>
__global__ __launch_bounds__(THREADS) void k_chunk(float* __restrict__ obs, int64_t n4) {
  f32x4* out4 = reinterpret_cast<f32x4*>(obs);
  const int64_t q0 = (int64_t)blockIdx.x * (U * THREADS) + threadIdx.x;
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (q0 + u * THREADS < n4) st<NT>(&out4[q0 + u * THREADS], (f32x4){1.0f, 2.0f, 3.0f, 4.0f});
}

template <int THREADS, int U, bool NT>
void run_c(float* obs, int64_t B, const char* name) {
  const int64_t n4 = B * (int64_t)QE;
  const unsigned grid = (unsigned)((n4 + U * THREADS - 1) / (U * THREADS));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_chunk<THREADS, U, NT>), dim3(grid), dim3(THREADS), 0, 0, obs, n4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    hipEventRecord(a, 0);
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL((k_chunk<THREADS, U, NT>), dim3(grid), dim3(THREADS), 0, 0, obs, n4);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    best = ms / 20 < best ? ms / 20 : best;
  }
  const double bytes = (double)B * PER_ENV * 4;
  printf("%-44s threads=%4d stores/lane=%d grid=%6u: %7.2f us  %6.2f TB/s\n", name, THREADS, U, grid, best * 1e3,
         bytes / (best * 1e-3) / 1e12);
}

template <int THREADS, int ENVS, bool CONTIG, bool NT>
void run_p(float* obs, int64_t B, unsigned grid, const char* name) {
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_probe_p<THREADS, ENVS, CONTIG, NT>), dim3(grid), dim3(THREADS), 0, 0, obs, B);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    hipEventRecord(a, 0);
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL((k_probe_p<THREADS, ENVS, CONTIG, NT>), dim3(grid), dim3(THREADS), 0, 0, obs, B);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    best = ms / 20 < best ? ms / 20 : best;
  }
  const double bytes = (double)B * PER_ENV * 4;
  printf("%-44s threads=%4d envs/WG=%3d grid=%6u: %7.2f us  %6.2f TB/s\n", name, THREADS, ENVS, grid, best * 1e3,
         bytes / (best * 1e-3) / 1e12);
}

template <int THREADS, int ENVS, int MODE, int U = 1, bool NT = false>
void run(float* obs, int64_t B, const char* name) {
  const unsigned grid = (unsigned)((B + ENVS - 1) / ENVS);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_probe<THREADS, ENVS, MODE, U, NT>), dim3(grid), dim3(THREADS), 0, 0, obs, B);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    hipEventRecord(a, 0);
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL((k_probe<THREADS, ENVS, MODE, U, NT>), dim3(grid), dim3(THREADS), 0, 0, obs, B);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    best = ms / 20 < best ? ms / 20 : best;
  }
  const double bytes = (double)B * PER_ENV * 4;
  printf("%-44s threads=%4d envs/WG=%3d grid=%6u: %7.2f us  %6.2f TB/s\n", name, THREADS, ENVS, grid, best * 1e3,
         bytes / (best * 1e-3) / 1e12);
}

int main() {
  const int64_t B = 65536;
  float* obs;
  hipMalloc(&obs, (size_t)B * PER_ENV * 4);
#ifdef PROBE_LARGE
  if (getenv("PROBE_CHUNKS")) {
    run_c<256, 1, true>(obs, B, "chunk 4 KB per WG, nt");
    run_c<256, 1, false>(obs, B, "chunk 4 KB per WG, plain");
    run_c<256, 2, true>(obs, B, "chunk 8 KB per WG, nt");
    run_c<256, 4, true>(obs, B, "chunk 16 KB per WG, nt");
    run_c<256, 4, false>(obs, B, "chunk 16 KB per WG, plain");
    run_c<256, 8, true>(obs, B, "chunk 32 KB per WG, nt");
    run_c<256, 9, true>(obs, B, "chunk 36 KB per WG, nt");
    run_c<512, 4, true>(obs, B, "chunk 32 KB per 512-lane WG, nt");
    run_c<1024, 2, true>(obs, B, "chunk 32 KB per 1024-lane WG, nt");
    return 0;
  }
  run<256, 4, 0, 1, true>(obs, B, "Large k_observe shape (4 envs), gather, nt");
  run<256, 4, 1, 2, true>(obs, B, "Large 4 envs, gather unroll 2, nt");
  run<256, 4, 2, 1, true>(obs, B, "Large 4 envs, constant stores, nt");
  run<256, 4, 0, 1, false>(obs, B, "Large 4 envs, gather, plain");
  run<256, 4, 2, 1, false>(obs, B, "Large 4 envs, constant stores, plain");
  run<256, 8, 0, 1, true>(obs, B, "Large 8 envs, gather, nt");
  run<256, 8, 2, 1, true>(obs, B, "Large 8 envs, constant stores, nt");
  run<512, 8, 1, 2, true>(obs, B, "Large 512 lanes 8 envs, gather unroll 2, nt");
  run<512, 8, 2, 1, true>(obs, B, "Large 512 lanes 8 envs, constant stores, nt");
  run<1024, 16, 2, 1, true>(obs, B, "Large 1024 lanes 16 envs, constant stores, nt");
  run_p<256, 4, true, true>(obs, B, 256 * 8, "persistent contiguous 8/CU, const, nt");
  run_p<256, 4, false, true>(obs, B, 256 * 8, "persistent interleaved 8/CU, const, nt");
  run_p<1024, 4, true, true>(obs, B, 256, "persistent contiguous 1x1024/CU, const, nt");
  run_p<1024, 4, true, true>(obs, B, 512, "persistent contiguous 2x1024/CU, const, nt");
  run_p<256, 4, true, true>(obs, B, 256 * 4, "persistent contiguous 4/CU, const, nt");
  run_p<256, 4, true, false>(obs, B, 256 * 8, "persistent contiguous 8/CU, const, plain");
  run_p<256, 1, false, true>(obs, B, 65536, "1 env per WG (65536 WGs), const, nt");
  run_p<256, 16, false, true>(obs, B, 4096, "16 envs per WG (4096 WGs), const, nt");
  run_s<256, 1, true>(obs, B, 2048, "sweep 256 lanes x 2048 WGs, nt");
  run_s<256, 1, false>(obs, B, 2048, "sweep 256 lanes x 2048 WGs, plain");
  run_s<256, 4, true>(obs, B, 2048, "sweep 256 lanes x 2048 WGs unroll 4, nt");
  run_s<256, 4, false>(obs, B, 2048, "sweep 256 lanes x 2048 WGs unroll 4, plain");
  run_s<256, 1, true>(obs, B, 16384, "sweep 256 lanes x 16384 WGs, nt");
  run_s<256, 1, true>(obs, B, 148480, "sweep one float4 per lane (no loop), nt");
  run_s<256, 1, false>(obs, B, 148480, "sweep one float4 per lane (no loop), plain");
  run_s<1024, 4, false>(obs, B, 512, "sweep 1024 lanes x 512 WGs unroll 4, plain");
  hipMemset(obs, 0, (size_t)B * PER_ENV * 4);
  {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(a, 0);
      for (int i = 0; i < 20; ++i) hipMemsetAsync(obs, i, (size_t)B * PER_ENV * 4, 0);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      best = ms / 20 < best ? ms / 20 : best;
    }
    printf("%-44s %7.2f us  %6.2f TB/s\n", "hipMemsetAsync of the same buffer", best * 1e3,
           (double)B * PER_ENV * 4 / (best * 1e-3) / 1e12);
  }
  return 0;
#endif
  if (getenv("PROBE_CHUNKS")) {   // Medium-8 rows (172 MB): chunked regions vs the fused launch's 672 KB ones
    for (int pass = 0; pass < 2; ++pass) {
      run<512, 256, 2>(obs, B, "fused 512 lanes 256 envs (672 KB/WG), constant");
      run<256, 16, 2>(obs, B, "k_observe shape 16 envs (42 KB/WG), constant");
      run_c<256, 1, false>(obs, B, "chunk 4 KB per WG, plain");
      run_c<256, 4, false>(obs, B, "chunk 16 KB per WG, plain");
      run_c<256, 8, false>(obs, B, "chunk 32 KB per WG, plain");
    }
    return 0;
  }
  run<256, 16, 0>(obs, B, "k_observe shape, gather");
  run<256, 16, 2>(obs, B, "k_observe shape, constant stores");
  run<256, 64, 0>(obs, B, "256 lanes 64 envs, gather");
  run<512, 256, 0>(obs, B, "fused 512 lanes, gather");
  run<512, 256, 1, 2>(obs, B, "fused 512 lanes, gather unroll 2");
  run<512, 256, 1, 4>(obs, B, "fused 512 lanes, gather unroll 4");
  run<512, 256, 2>(obs, B, "fused 512 lanes, constant stores");
  run<1024, 256, 0>(obs, B, "fused 1024 lanes, gather");
  run<1024, 256, 1, 2>(obs, B, "fused 1024 lanes, gather unroll 2");
  run<1024, 256, 2>(obs, B, "fused 1024 lanes, constant stores");
  run<256, 256, 0>(obs, B, "fused 256 lanes, gather");
  run<256, 256, 1, 4>(obs, B, "fused 256 lanes, gather unroll 4");
  run<256, 256, 2>(obs, B, "fused 256 lanes, constant stores");
  run<512, 128, 0>(obs, B, "512 lanes 128 envs, gather");
  return 0;
}
