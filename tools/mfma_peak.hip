#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
__global__ __launch_bounds__(256) void k(float* out, int iters, float seed) {
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (__bf16)(seed * (threadIdx.x + j)); b[j] = (__bf16)(seed - j); }
  f32x16 acc[8] = {};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[t], 0, 0, 0);
  }
  float s = 0;
  for (int t = 0; t < 8; ++t) for (int g = 0; g < 16; ++g) s += acc[t][g];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
  float* out; hipMalloc(&out, 256 * 256 * 4 * 16);
  int iters = 4096;
  for (int grid : {256, 512, 1024}) {
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, iters, 0.001f);
    hipDeviceSynchronize();
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, iters, 0.001f);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    double flop = (double)grid * 4 * iters * 8 * 32 * 32 * 16 * 2;
    printf("grid %d: %.3f ms  %.1f TFLOP/s\n", grid, ms, flop / ms / 1e9);
  }
  return 0;
}
