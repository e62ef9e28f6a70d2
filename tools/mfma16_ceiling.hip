// What a bare v_mfma_f32_16x16x32_bf16 loop holds on this chip, on random data, in k_mlp16's shape:
// 8 waves per workgroup (two per SIMD), one workgroup per CU, every A operand re-read from LDS with
// one ds_read_b128 per lane and fed to two MFMAs (two 16-sample tiles), B operands in registers --
// the policy kernel's inner loop without its weight staging, barriers, bias/ReLU and logits.  The
// bf16 peak the bench prices against (2.5 PF) is a spec clock; MI355X_MICROARCH.md 'DVFS give-back'
// says random-data bf16 loops hold well under it, so this is the ceiling the kernel can approach.
//   hipcc --offload-arch=gfx950 -O3 -o build/mfma16_ceiling tools/mfma16_ceiling.hip && ./build/mfma16_ceiling
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int OPS = 64;   // staged A operands of 1 KiB (64 KiB of LDS, as one k_mlp16 stage)

// WAVES waves per workgroup (8: two per SIMD, 4: one), NT 16-sample tiles per A operand read
template <bool LDS_A, int WAVES = 8, int NT = 2>
__global__ __launch_bounds__(64 * WAVES) void k(float* out, const uint4* __restrict__ src, int iters) {
  __shared__ uint4 lds[OPS * 64];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < OPS * 64; i += 64 * WAVES) lds[i] = src[i];
  __syncthreads();
  bf16x8 bt[NT];
  for (int t = 0; t < NT; ++t) bt[t] = __builtin_bit_cast(bf16x8, src[(blockIdx.x * 512 + tid + 7 * t) % (OPS * 64)]);
  bf16x8 areg[4];
  for (int j = 0; j < 4; ++j) areg[j] = __builtin_bit_cast(bf16x8, src[(tid * 4 + j) % (OPS * 64)]);
  f32x4 acc[4 * NT] = {};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int g = 0; g < OPS; g += 4) {
      bf16x8 a[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        a[j] = LDS_A ? __builtin_bit_cast(bf16x8, lds[(g + j) * 64 + lane]) : areg[j];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int t = 0; t < NT; ++t)
          acc[NT * j + t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[j], bt[t], acc[NT * j + t], 0, 0, 0);
    }
  }
  float s = 0.0f;
  for (int t = 0; t < 4 * NT; ++t)
    for (int q = 0; q < 4; ++q) s += acc[t][q];
  out[blockIdx.x * 512 + tid] = s;
}

// k_mlp16's own operand pipeline: stream_ops (fragments read DEPTH = 2 groups of 4 ahead of their
// MFMAs, sched_barriers around each group), PRIO: s_setprio 1 over each group's MFMAs
template <int WAVES, bool PRIO>
__global__ __launch_bounds__(64 * WAVES) void kp(float* out, const uint4* __restrict__ src, int iters) {
  __shared__ uint4 lds[OPS * 64];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < OPS * 64; i += 64 * WAVES) lds[i] = src[i];
  __syncthreads();
  const bf16x8 b0 = __builtin_bit_cast(bf16x8, src[(blockIdx.x * 512 + tid) % (OPS * 64)]);
  const bf16x8 b1 = __builtin_bit_cast(bf16x8, src[(blockIdx.x * 512 + tid + 7) % (OPS * 64)]);
  f32x4 acc[8] = {};
  constexpr int GS = 4, NG = OPS / GS, DEPTH = 2;
  for (int it = 0; it < iters; ++it) {
    bf16x8 buf[DEPTH + 1][GS];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
#pragma unroll
      for (int i = 0; i < GS; ++i) buf[d][i] = __builtin_bit_cast(bf16x8, lds[(d * GS + i) * 64 + lane]);
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
      if (gi + DEPTH < NG) {
#pragma unroll
        for (int i = 0; i < GS; ++i)
          buf[(gi + DEPTH) % (DEPTH + 1)][i] = __builtin_bit_cast(bf16x8, lds[((gi + DEPTH) * GS + i) * 64 + lane]);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < GS; ++i) {
        acc[2 * i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(buf[gi % (DEPTH + 1)][i], b0, acc[2 * i], 0, 0, 0);
        acc[2 * i + 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(buf[gi % (DEPTH + 1)][i], b1, acc[2 * i + 1], 0, 0, 0);
      }
      if (PRIO) __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  float s = 0.0f;
  for (int t = 0; t < 8; ++t)
    for (int q = 0; q < 4; ++q) s += acc[t][q];
  out[blockIdx.x * 512 + tid] = s;
}

template <int WAVES, bool PRIO>
void runp(const char* name, float* out, const uint4* src, int grid, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  int warm = 0;
  float ms = 0.0f;
  do {
    hipLaunchKernelGGL((kp<WAVES, PRIO>), dim3(grid), dim3(64 * WAVES), 0, 0, out, src, iters);
    ++warm;
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
  } while (ms < 2000.0f);
  const int reps = 20;
  hipEventRecord(a);
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((kp<WAVES, PRIO>), dim3(grid), dim3(64 * WAVES), 0, 0, out, src, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  hipEventElapsedTime(&ms, a, b);
  const double flop = (double)grid * WAVES * iters * OPS * 2 * (16.0 * 16 * 32 * 2) * reps;
  printf("%-44s grid %d x %d: %.3f ms per launch, %.1f TFLOP/s = %.3f of 2.5 PF (after %d warm-up launches)\n", name,
         grid, 64 * WAVES, ms / reps, flop / (ms * 1e-3) / 1e12, flop / (ms * 1e-3) / 2.5e15, warm);
}

template <bool LDS_A, int WAVES = 8, int NT = 2>
void run(const char* name, float* out, const uint4* src, int grid, int iters) {
  // >= 2 s of back-to-back launches first, so the clock has settled (MI355X_MICROARCH.md item 6)
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  int warm = 0;
  float ms = 0.0f;
  do {
    hipLaunchKernelGGL((k<LDS_A, WAVES, NT>), dim3(grid), dim3(64 * WAVES), 0, 0, out, src, iters);
    ++warm;
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
  } while (ms < 2000.0f);
  const int reps = 20;
  hipEventRecord(a);
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((k<LDS_A, WAVES, NT>), dim3(grid), dim3(64 * WAVES), 0, 0, out, src, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  hipEventElapsedTime(&ms, a, b);
  const double flop = (double)grid * WAVES * iters * OPS * NT * (16.0 * 16 * 32 * 2) * reps;
  printf("%-44s grid %d x %d: %.3f ms per launch, %.1f TFLOP/s = %.3f of 2.5 PF (after %d warm-up launches)\n", name,
         grid, 64 * WAVES, ms / reps, flop / (ms * 1e-3) / 1e12, flop / (ms * 1e-3) / 2.5e15, warm);
}

int main() {
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  std::vector<uint16_t> h(OPS * 64 * 8);
  srand(7);
  for (auto& v : h) {
    const float f = (float)rand() / RAND_MAX * 2.0f - 1.0f;   // random bf16 in [-1, 1]
    uint32_t u;
    memcpy(&u, &f, 4);
    v = (uint16_t)(u >> 16);
  }
  uint4* src;
  float* out;
  hipMalloc(&src, h.size() * 2);
  hipMalloc(&out, (size_t)cus * 512 * 4);
  hipMemcpy(src, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  const int iters = 1024;
  run<true, 8, 2>("A from LDS, 2 waves/SIMD, 2 tiles (k_mlp16)", out, src, cus, iters);
  run<false, 8, 2>("registers, 2 waves/SIMD, 2 tiles", out, src, cus, iters);
  run<true, 4, 4>("A from LDS, 1 wave/SIMD, 4 tiles", out, src, cus, iters / 2);
  run<true, 4, 2>("A from LDS, 1 wave/SIMD, 2 tiles", out, src, cus, iters);
  run<true, 8, 4>("A from LDS, 2 waves/SIMD, 4 tiles", out, src, cus, iters / 2);
  runp<8, false>("stream_ops pipeline, 2 waves/SIMD", out, src, cus, iters);
  runp<8, true>("stream_ops pipeline + setprio, 2 waves/SIMD", out, src, cus, iters);
  runp<4, false>("stream_ops pipeline, 1 wave/SIMD", out, src, cus, iters);
  hipFree(src);
  hipFree(out);
  return 0;
}
