// philox.h -- Philox4x32-10 (Salmon et al., SC'11), shared by the simulator and policy kernels.
// Modelled bit-exactly on the host by oracle/philox.py (Random123 known-answer vectors).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ __forceinline__ uint4 philox10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;   // one v_mad_u64_u32 each
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    // three-input xors as single v_bitop3 ops
    c = make_uint4(__builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c.y, k0, 0x96), (uint32_t)p1,
                   __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c.w, k1, 0x96), (uint32_t)p0);
  }
  return c;
}
