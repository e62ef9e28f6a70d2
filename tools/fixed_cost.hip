// Floor of a fused-rollout launch's fixed cost at B = 65,536 (256 workgroups x 256 lanes, one wave
// per SIMD): what a launch costs that only moves the packed Medium-8 state (28 word planes) in and
// out, with and without the per-workgroup table load into LDS and one step's reward/done stores.
// Compared with a 1-step k_step launch (tools/anatomy.py), the difference is the step kernel's own
// prologue/epilogue work.  hipcc --offload-arch=gfx950 -O3 tools/fixed_cost.hip -o tools/fixed_cost_bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

constexpr int BT = 256, WORDS = 28, TBLW = 2360;   // Medium-8: 28 state words, 9.4 KB of tables
constexpr int64_t B = 65536;

__global__ __launch_bounds__(BT) void k_empty(uint32_t* st) {
  if (threadIdx.x == 1000) st[0] = 0;
}

__global__ __launch_bounds__(BT) void k_state(uint32_t* st) {
  const int64_t e = (int64_t)blockIdx.x * BT + threadIdx.x;
  uint32_t v[WORDS];
#pragma unroll
  for (int w = 0; w < WORDS; ++w) v[w] = st[w * B + e];
#pragma unroll
  for (int w = 0; w < WORDS; ++w) st[w * B + e] = v[w] + 1u;
}

template <int LDS_BYTES>
__global__ __launch_bounds__(BT) void k_state_tables(uint32_t* st, const uint32_t* tables, float* rew, uint8_t* dn,
                                                     int steps) {
  __shared__ alignas(16) uint32_t lds[LDS_BYTES / 4];
  const int64_t e = (int64_t)blockIdx.x * BT + threadIdx.x;
  uint32_t v[WORDS];
#pragma unroll
  for (int w = 0; w < WORDS; ++w) v[w] = st[w * B + e];
  constexpr int TBL4 = (TBLW + 3) / 4, IT = (TBL4 + BT - 1) / BT;
  uint4 t[IT];
  const uint4* src = reinterpret_cast<const uint4*>(tables);
#pragma unroll
  for (int i = 0; i < IT; ++i)
    if (i + 1 < IT || (int)threadIdx.x + i * BT < TBL4) t[i] = src[threadIdx.x + i * BT];
#pragma unroll
  for (int i = 0; i < IT; ++i)
    if (i + 1 < IT || (int)threadIdx.x + i * BT < TBL4) reinterpret_cast<uint4*>(lds)[threadIdx.x + i * BT] = t[i];
  __syncthreads();
  uint32_t acc = lds[(threadIdx.x * 7) % TBLW];
  for (int s = 0; s < steps; ++s) {
    float4* row = reinterpret_cast<float4*>(rew + ((int64_t)s * B + e) * 8);
    row[0] = make_float4((float)(acc & 1), 0.f, 0.f, 0.f);
    row[1] = make_float4(0.f, 0.f, 0.f, (float)(v[3] & 1));
    dn[(int64_t)s * B + e] = (uint8_t)(v[0] & 1);
    acc = acc * 1664525u + 1013904223u;
  }
#pragma unroll
  for (int w = 0; w < WORDS; ++w) st[w * B + e] = v[w] + acc;
}

#define CK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(err_), __LINE__); return 1; } } while (0)

int main() {
  uint32_t *st, *tab;
  float* rew;
  uint8_t* dn;
  CK(hipMalloc(&st, WORDS * B * 4));
  CK(hipMalloc(&tab, TBLW * 4 + 64));
  CK(hipMalloc(&rew, 20 * B * 8 * 4));
  CK(hipMalloc(&dn, 20 * B));
  CK(hipMemset(st, 0, WORDS * B * 4));
  CK(hipMemset(tab, 0, TBLW * 4 + 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const dim3 g(B / BT), b(BT);
  struct Case { const char* name; int kind; int steps; };
  const Case cases[] = {{"empty", 0, 0},           {"state in+out", 1, 0},
                        {"state+tables 12KB LDS", 2, 0}, {"state+tables 52KB LDS", 3, 0},
                        {"state+tables+1 step stores", 3, 1}, {"state+tables+20 step stores", 3, 20}};
  for (const Case& c : cases) {
    for (int warm = 0; warm < 2; ++warm) {
      std::vector<float> ts;
      for (int r = 0; r < 25; ++r) {
        if (warm) {   // queued right behind a busy launch
          hipLaunchKernelGGL(k_state_tables<53248>, g, b, 0, 0, st, tab, rew, dn, 20);
        }
        CK(hipEventRecord(e0, 0));
        switch (c.kind) {
          case 0: hipLaunchKernelGGL(k_empty, g, b, 0, 0, st); break;
          case 1: hipLaunchKernelGGL(k_state, g, b, 0, 0, st); break;
          case 2: hipLaunchKernelGGL(k_state_tables<12288>, g, b, 0, 0, st, tab, rew, dn, c.steps); break;
          default: hipLaunchKernelGGL(k_state_tables<53248>, g, b, 0, 0, st, tab, rew, dn, c.steps); break;
        }
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ts.push_back(ms * 1000.f);
      }
      std::sort(ts.begin(), ts.end());
      printf("%-30s %-5s median %7.2f us  min %7.2f us\n", c.name, warm ? "warm" : "cold", ts[ts.size() / 2], ts[0]);
    }
  }
  return 0;
}
