// Operand-type costs at 1 wave per SIMD (B = 65,536 envs -> 1,024 waves): SGPR / literal operands,
// cndmask and compare forms, VALU->SALU->VALU mask round trips.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define ITERS 2048
#define OPK(name, body, pre) \
__global__ __launch_bounds__(256) void k_##name(uint32_t* out, uint32_t s) { \
  uint32_t a0 = threadIdx.x ^ s, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 + 11u, a5 = a0 + 13u, a6 = a0 ^ 0x55u, a7 = a0 ^ 0xAAu; \
  uint32_t b = s | 1u, c = s >> 3; \
  pre \
  for (int i = 0; i < ITERS; ++i) { body(a0) body(a1) body(a2) body(a3) body(a4) body(a5) body(a6) body(a7) } \
  out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; }
#define NOPRE
#define PRE_VCC asm volatile("v_cmp_gt_u32 vcc, %0, %1" :: "v"(a0), "v"(b) : "vcc");
#define PRE_S23 asm volatile("v_cmp_gt_u32 s[2:3], %0, %1" :: "v"(a0), "v"(b) : "s2", "s3");
#define B_XOR(x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(b));
#define B_XORS(x) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(x) : "s"(s));
#define B_XORL(x) asm volatile("v_xor_b32 %0, 0x12345, %0" : "+v"(x));
#define B_XORI(x) asm volatile("v_xor_b32 %0, 15, %0" : "+v"(x));
#define B_ANDL3(x) asm volatile("v_and_or_b32 %0, %0, %2, %1" : "+v"(x) : "v"(b), "s"(s));
#define B_CNDVCC(x) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(b) : "vcc");
#define B_CNDS(x) asm volatile("v_cndmask_b32 %0, %0, %1, s[2:3]" : "+v"(x) : "v"(b) : "s2", "s3");
#define B_CNDK(x) asm volatile("v_cndmask_b32 %0, 0, %0, s[2:3]" : "+v"(x) :: "s2", "s3");
#define B_BSEL(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca" : "+v"(x) : "v"(b), "v"(c));
#define B_BFI(x) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define B_CMPV(x) asm volatile("v_cmp_gt_u32 vcc, %0, %1" :: "v"(x), "v"(b) : "vcc");
#define B_CMPROT(x) asm volatile("v_cmp_gt_u32 s[2:3], %0, %1\n v_cmp_gt_u32 s[4:5], %0, %2\n v_cmp_gt_u32 s[6:7], %0, %1\n v_cmp_gt_u32 s[8:9], %0, %2" :: "v"(x), "v"(b), "v"(c) : "s2","s3","s4","s5","s6","s7","s8","s9");
#define B_RT(x) asm volatile("v_cmp_gt_u32 s[2:3], %0, %1\n s_and_b64 s[2:3], s[2:3], exec\n v_cndmask_b32 %0, %0, %1, s[2:3]" : "+v"(x) : "v"(b) : "s2", "s3");
#define B_CMPCND(x) asm volatile("v_cmp_gt_u32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(b) : "vcc");
#define B_MASKSEL(x) asm volatile("v_sub_u32 %0, %0, %1\n v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca" : "+v"(x) : "v"(b), "v"(c));
#define B_DPP(x) asm volatile("v_xor_b32_dpp %0, %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x) : "v"(b));
#define B_SALU(x) asm volatile("s_add_u32 s2, s2, s3" ::: "s2", "s3", "scc");
#define B_SALUMIX(x) asm volatile("v_xor_b32 %0, %0, %1\n s_add_u32 s2, s2, s3" : "+v"(x) : "v"(b) : "s2", "s3", "scc");
#define B_LDSW(q) asm volatile("ds_write_b32 %0, %1" :: "v"(4u * (threadIdx.x & 255)), "v"(q));
#define B_LDSOR(q) asm volatile("ds_or_b32 %0, %1" :: "v"(4u * (threadIdx.x & 255)), "v"(q));
#define B_LDSR(q) asm volatile("ds_read_b32 %0, %1" : "=v"(q) : "v"(4u * (threadIdx.x & 255)));
#define B_LDSR_U8(q) asm volatile("ds_read_u8 %0, %1" : "=v"(q) : "v"(threadIdx.x & 1023));
OPK(xor, B_XOR, NOPRE) OPK(xors, B_XORS, NOPRE) OPK(xorl, B_XORL, NOPRE) OPK(xori, B_XORI, NOPRE) OPK(andorl, B_ANDL3, NOPRE)
OPK(cndvcc, B_CNDVCC, PRE_VCC) OPK(cnds, B_CNDS, PRE_S23) OPK(cndk, B_CNDK, PRE_S23) OPK(bsel, B_BSEL, NOPRE) OPK(bfi, B_BFI, NOPRE)
OPK(cmpv, B_CMPV, NOPRE) OPK(cmprot, B_CMPROT, NOPRE) OPK(rt, B_RT, NOPRE) OPK(cmpcnd, B_CMPCND, NOPRE) OPK(masksel, B_MASKSEL, NOPRE)
OPK(dpp, B_DPP, NOPRE) OPK(salu, B_SALU, NOPRE) OPK(salumix, B_SALUMIX, NOPRE)
__global__ __launch_bounds__(256) void k_ldsw(uint32_t* out, uint32_t s) { __shared__ uint32_t L[1024]; uint32_t a0 = s, a1 = s+1, a2=s+2,a3=s+3,a4=s+4,a5=s+5,a6=s+6,a7=s+7;
  for (int i = 0; i < ITERS; ++i) { B_LDSW(a0) B_LDSW(a1) B_LDSW(a2) B_LDSW(a3) B_LDSW(a4) B_LDSW(a5) B_LDSW(a6) B_LDSW(a7) } asm volatile("s_waitcnt lgkmcnt(0)"); __syncthreads(); out[blockIdx.x * 256 + threadIdx.x] = L[threadIdx.x]; }
__global__ __launch_bounds__(256) void k_ldsor(uint32_t* out, uint32_t s) { __shared__ uint32_t L[1024]; L[threadIdx.x] = 0; __syncthreads(); uint32_t a0 = s, a1 = s+1, a2=s+2,a3=s+3,a4=s+4,a5=s+5,a6=s+6,a7=s+7;
  for (int i = 0; i < ITERS; ++i) { B_LDSOR(a0) B_LDSOR(a1) B_LDSOR(a2) B_LDSOR(a3) B_LDSOR(a4) B_LDSOR(a5) B_LDSOR(a6) B_LDSOR(a7) } asm volatile("s_waitcnt lgkmcnt(0)"); __syncthreads(); out[blockIdx.x * 256 + threadIdx.x] = L[threadIdx.x]; }
__global__ __launch_bounds__(256) void k_ldsr(uint32_t* out, uint32_t s) { __shared__ uint32_t L[1024]; L[threadIdx.x] = s; __syncthreads(); uint32_t a0, a1, a2,a3,a4,a5,a6,a7, acc = 0;
  for (int i = 0; i < ITERS; ++i) { B_LDSR(a0) B_LDSR(a1) B_LDSR(a2) B_LDSR(a3) B_LDSR(a4) B_LDSR(a5) B_LDSR(a6) B_LDSR(a7) asm volatile("s_waitcnt lgkmcnt(0)"); acc ^= a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; } out[blockIdx.x * 256 + threadIdx.x] = acc; }
__global__ __launch_bounds__(256) void k_ldsru8(uint32_t* out, uint32_t s) { __shared__ uint32_t L[1024]; L[threadIdx.x] = s; __syncthreads(); uint32_t a0, a1, a2,a3,a4,a5,a6,a7, acc = 0;
  for (int i = 0; i < ITERS; ++i) { B_LDSR_U8(a0) B_LDSR_U8(a1) B_LDSR_U8(a2) B_LDSR_U8(a3) B_LDSR_U8(a4) B_LDSR_U8(a5) B_LDSR_U8(a6) B_LDSR_U8(a7) asm volatile("s_waitcnt lgkmcnt(0)"); acc ^= a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; } out[blockIdx.x * 256 + threadIdx.x] = acc; }
typedef void (*KF)(uint32_t*, uint32_t);
#define E(n, cnt, note) {#n, k_##n, cnt, note}
int main() {
  struct { const char* n; KF f; int insts; const char* note; } ks[] = {
    E(xor,1,"v,v"), E(xors,1,"SGPR operand"), E(xorl,1,"literal"), E(xori,1,"inline const"), E(andorl,1,"VOP3 + SGPR operand"),
    E(cndvcc,1,"cndmask vcc (vcc set once)"), E(cnds,1,"cndmask e64 s[2:3]"), E(cndk,1,"cndmask e64 const,v,s"), E(bsel,1,"bitop3 0xca select"), E(bfi,1,"bfi select"),
    E(cmpv,1,"v_cmp -> vcc"), E(cmprot,4,"v_cmp -> 4 rotating sgpr pairs"), E(rt,3,"cmp->s_and->cndmask chain"), E(cmpcnd,2,"cmp vcc + cndmask vcc"),
    E(masksel,2,"sub + bitop3 select"), E(dpp,1,"xor with DPP quad_perm"), E(salu,1,"s_add only"), E(salumix,2,"xor + s_add interleaved"),
    E(ldsw,1,"ds_write_b32 (issue)"), E(ldsor,1,"ds_or_b32 (issue)"), E(ldsr,1,"8 ds_read_b32 then wait"), E(ldsru8,1,"8 ds_read_u8 then wait")};
  uint32_t* out; (void)hipMalloc(&out, 1024 * 256 * 4 * 8);
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  setvbuf(stdout, NULL, _IONBF, 0);
  printf("ns per instruction per SIMD at 1 wave per SIMD (1,024 waves), and at 2 waves per SIMD\n");
  for (auto& k : ks) {
    printf("%-9s %-34s", k.n, k.note); fflush(stdout);
    for (int wps : {1, 2}) {
      int blocks = 256 * wps;
      k.f<<<blocks, 256>>>(out, 7); (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0); for (int r = 0; r < 5; ++r) k.f<<<blocks, 256>>>(out, 7); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
      float ms; (void)hipEventElapsedTime(&ms, e0, e1); ms /= 5;
      printf("  %6.3f", ms * 1e6 / ((double)wps * ITERS * 8 * k.insts));
    }
    printf("\n");
  }
  return 0;
}
