// Control-flow and special-op costs at 1 wave per SIMD (1,024 waves), the step kernel's regime:
// taken branches (instruction-fetch bubbles), VALU->VCC->s_cbranch round trips, and a few VALU
// opcodes the step loop uses.  Reports ns per group of 8 independent v_xor plus the extra op.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#define ITERS 1024

#define XORS "v_xor_b32 %0, %0, %8\n v_xor_b32 %1, %1, %8\n v_xor_b32 %2, %2, %8\n v_xor_b32 %3, %3, %8\n" \
             "v_xor_b32 %4, %4, %8\n v_xor_b32 %5, %5, %8\n v_xor_b32 %6, %6, %8\n v_xor_b32 %7, %7, %8\n"
#define OUTS "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)

#define KERN(name, extra, clob)                                                                      \
  __global__ __launch_bounds__(256) void k_##name(uint32_t* out, uint32_t s) {                        \
    uint32_t a0 = threadIdx.x ^ s, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 + 11u,           \
             a5 = a0 + 13u, a6 = a0 ^ 0x55u, a7 = a0 ^ 0xAAu, b = s | 1u;                             \
    for (int i = 0; i < ITERS; ++i) asm volatile(XORS extra : OUTS : "v"(b) clob);                   \
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                      \
  }

KERN(base, "", )
KERN(br, "s_branch 1f\n 1:\n", )
KERN(brfar, "s_branch 1f\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n "
            "s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n 1:\n", )
KERN(vcmpbr_nt, "v_cmp_gt_u32 vcc, %0, -1\n s_cbranch_vccnz 1f\n 1:\n", : "vcc")
KERN(vcmpbr_t, "v_cmp_le_u32 vcc, %0, -1\n s_cbranch_vccnz 1f\n s_nop 0\n 1:\n", : "vcc")
KERN(scmp_br, "s_cmp_eq_u32 s0, s0\n s_cbranch_scc0 1f\n 1:\n", : "scc")
KERN(ffbl, "v_ffbl_b32 %0, %1\n", )
KERN(sad, "v_sad_hi_u8 %0, %1, %2, %3\n", )
KERN(dot2, "v_dot2c_i32_i16 %0, %1, %2\n", )
KERN(nop, "s_nop 0\n", )
KERN(readlane, "v_readlane_b32 s2, %0, 0\n", : "s2")
KERN(pkmin, "v_pk_min_i16 %0, %1, %2\n", )
KERN(bfei, "v_bfe_i32 %0, %1, %2, 1\n", )
KERN(mulhi, "v_mul_hi_u32 %0, %1, %2\n", )
KERN(mullo, "v_mul_lo_u32 %0, %1, %2\n", )
KERN(mul24, "v_mul_u32_u24 %0, %1, %2\n", )
#define CL_MAD : "v2", "v3", "s2", "s3"
KERN(madu64, "v_mad_u64_u32 v[2:3], s[2:3], %1, %2, 0\n", CL_MAD)

typedef void (*KF)(uint32_t*, uint32_t);
int main() {
  struct { const char* n; KF f; } ks[] = {
      {"base (8 xor)", k_base}, {"+ s_branch next", k_br}, {"+ s_branch over 16 nops", k_brfar},
      {"+ v_cmp vcc; cbranch not taken", k_vcmpbr_nt}, {"+ v_cmp vcc; cbranch taken", k_vcmpbr_t},
      {"+ s_cmp; cbranch_scc0 nt", k_scmp_br}, {"+ v_ffbl", k_ffbl}, {"+ v_sad_hi_u8", k_sad},
      {"+ v_dot2c_i32_i16", k_dot2}, {"+ s_nop 0", k_nop},
      {"+ v_readlane", k_readlane}, {"+ v_pk_min_i16", k_pkmin}, {"+ v_bfe_i32", k_bfei},
      {"+ v_mul_hi_u32", k_mulhi}, {"+ v_mul_lo_u32", k_mullo}, {"+ v_mul_u32_u24", k_mul24},
      {"+ v_mad_u64_u32", k_madu64}};
  uint32_t* out;
  (void)hipMalloc(&out, 1024 * 256 * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  setvbuf(stdout, NULL, _IONBF, 0);
  printf("ns per group per SIMD at 1 wave per SIMD (1,024 waves); base = 8 independent v_xor\n");
  float base = 0;
  for (auto& k : ks) {
    k.f<<<256, 256>>>(out, 7);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) k.f<<<256, 256>>>(out, 7);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const float ns = ms / 5 * 1e6f / ITERS;
    if (k.f == k_base) base = ns;
    printf("%-34s %7.2f ns/group  extra %6.2f ns\n", k.n, ns, ns - base);
  }
  return 0;
}
