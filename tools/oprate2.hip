// Which VALU ops issue at the 2-cycle rate with 2+ waves per SIMD, and do half-exec waves (32 live lanes) cost less?
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define ITERS 2048
#define OPK(name, body) \
template <int HALF> __global__ __launch_bounds__(256) void k_##name(uint32_t* out, uint32_t s) { \
  uint32_t a0 = threadIdx.x ^ s, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 + 11u, a5 = a0 + 13u, a6 = a0 ^ 0x55u, a7 = a0 ^ 0xAAu; \
  uint32_t b = s | 1u, c = s >> 3; \
  if (HALF && (threadIdx.x & 63) >= 32) return; \
  for (int i = 0; i < ITERS; ++i) { body(a0) body(a1) body(a2) body(a3) body(a4) body(a5) body(a6) body(a7) } \
  out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; }
#define I2(op) asm volatile(op " %0, %0, %1" : "+v"(x) : "v"(b));
#define B_XOR(x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(b));
#define B_AND(x) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(b));
#define B_ADD(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b));
#define B_SUB(x) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x) : "v"(b));
#define B_SHL(x) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(x) : "v"(b));
#define B_LSHLOR(x) asm volatile("v_lshl_or_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define B_ANDOR(x) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define B_OR3(x) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define B_ADD3(x) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define B_BFE(x) asm volatile("v_bfe_u32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define B_MIN(x) asm volatile("v_min_u32 %0, %0, %1" : "+v"(x) : "v"(b));
#define B_MIN3(x) asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define B_MOV(x) asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(x));
#define B_CNDS(x) asm volatile("v_cndmask_b32 %0, %0, %1, s[2:3]" : "+v"(x) : "v"(b) : "s2", "s3");
#define B_CMP(x) asm volatile("v_cmp_gt_u32 s[2:3], %0, %1" :: "v"(x), "v"(b) : "s2", "s3");
#define B_SAD(x) asm volatile("v_sad_hi_u8 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define B_PKADD(x) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x) : "v"(b));
#define B_PKMAX(x) asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(x) : "v"(b));
#define B_BITOP3(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(b), "v"(c));
#define B_MULLO(x) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(b));
#define B_BCNT(x) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(x) : "v"(b));
#define B_MIX(x) asm volatile("v_xor_b32 %0, %0, %1\n v_min3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
OPK(xor, B_XOR) OPK(and, B_AND) OPK(add, B_ADD) OPK(sub, B_SUB) OPK(shl, B_SHL) OPK(lshlor, B_LSHLOR) OPK(andor, B_ANDOR)
OPK(or3, B_OR3) OPK(add3, B_ADD3) OPK(bfe, B_BFE) OPK(min, B_MIN) OPK(min3, B_MIN3) OPK(mov, B_MOV) OPK(cnds, B_CNDS) OPK(cmp, B_CMP)
OPK(sad, B_SAD) OPK(pkadd, B_PKADD) OPK(pkmax, B_PKMAX) OPK(bitop3, B_BITOP3) OPK(mullo, B_MULLO) OPK(bcnt, B_BCNT) OPK(mix, B_MIX)
typedef void (*KF)(uint32_t*, uint32_t);
#define E(n, cnt) {#n, k_##n<0>, k_##n<1>, cnt}
int main() {
  struct { const char* n; KF f, h; int insts; } ks[] = {
    E(xor,1), E(and,1), E(add,1), E(sub,1), E(shl,1), E(lshlor,1), E(andor,1), E(or3,1), E(add3,1), E(bfe,1), E(min,1), E(min3,1),
    E(mov,1), E(cnds,1), E(cmp,1), E(sad,1), E(pkadd,1), E(pkmax,1), E(bitop3,1), E(mullo,1), E(bcnt,1), E(mix,2)};
  uint32_t* out; (void)hipMalloc(&out, 1024 * 256 * 4 * 8);
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  printf("ns per wave-instruction per SIMD; columns: waves/SIMD = 1, 2, 4 (full exec) | 2, 4 (half exec: lanes 0-31)\n");
  for (auto& k : ks) {
    printf("%-8s", k.n);
    for (int half = 0; half < 2; ++half)
      for (int wps : {1, 2, 4}) {
        if (half && wps == 1) continue;
        KF f = half ? k.h : k.f;
        int blocks = 256 * wps;
        f<<<blocks, 256>>>(out, 7); (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0); for (int r = 0; r < 5; ++r) f<<<blocks, 256>>>(out, 7); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1); ms /= 5;
        double ns_per = ms * 1e6 / ((double)wps * ITERS * 8 * k.insts);
        printf("  %6.3f", ns_per);
      }
    printf("\n");
  }
  return 0;
}
