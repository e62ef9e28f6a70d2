// Throughput of single VALU ops: 8 independent chains per lane, 1 wave per SIMD (1024 waves) and 4 per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define ITERS 2048
#define OPK(name, body) \
__global__ __launch_bounds__(256) void k_##name(uint32_t* out, uint32_t s) { \
  uint32_t a0 = threadIdx.x ^ s, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 + 11u, a5 = a0 + 13u, a6 = a0 ^ 0x55u, a7 = a0 ^ 0xAAu; \
  uint32_t b = s | 1u, c = s >> 3; \
  for (int i = 0; i < ITERS; ++i) { body(a0) body(a1) body(a2) body(a3) body(a4) body(a5) body(a6) body(a7) } \
  out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; }
#define B_XOR(x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(b));
#define B_MULLO(x) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(b));
#define B_MULHI(x) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(b));
#define B_MUL24(x) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(b));
#define B_SAD(x) asm volatile("v_sad_hi_u8 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define B_BITOP3(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(b), "v"(c));
#define B_MIN3(x) asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define B_PKMAX(x) asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(x) : "v"(b));
#define B_BCNT(x) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(x) : "v"(b));
#define B_FFBL(x) asm volatile("v_ffbl_b32 %0, %0" : "+v"(x));
#define B_CNDM(x) asm volatile("v_cmp_gt_u32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(b) : "vcc");
#define B_CNDONLY(x) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(b) : "vcc");
#define B_MAD64(x) { uint64_t r; asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, 0" : "=v"(r) : "v"(x), "v"(b) : "s0","s1"); x = (uint32_t)r ^ (uint32_t)(r >> 32); }
#define B_SHL64(x) { uint64_t r = ((uint64_t)x << 32) | c; asm volatile("v_lshlrev_b64 %0, %1, %0" : "+v"(r) : "v"(b)); x = (uint32_t)(r >> 32); }
#define B_LDS(x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(b));
OPK(xor, B_XOR)
__global__ __launch_bounds__(256) void k_xor1(uint32_t* out, uint32_t s) {
  uint32_t a0 = threadIdx.x ^ s, b = s | 1u;
  for (int i = 0; i < ITERS; ++i) { B_XOR(a0) B_XOR(a0) B_XOR(a0) B_XOR(a0) B_XOR(a0) B_XOR(a0) B_XOR(a0) B_XOR(a0) }
  out[blockIdx.x * 256 + threadIdx.x] = a0; }
__global__ __launch_bounds__(256) void k_sad1(uint32_t* out, uint32_t s) {
  uint32_t a0 = threadIdx.x ^ s, b = s | 1u, c = s >> 3;
  for (int i = 0; i < ITERS; ++i) { B_SAD(a0) B_SAD(a0) B_SAD(a0) B_SAD(a0) B_SAD(a0) B_SAD(a0) B_SAD(a0) B_SAD(a0) }
  out[blockIdx.x * 256 + threadIdx.x] = a0; }
__global__ __launch_bounds__(256) void k_lds1(uint32_t* out, uint32_t s) {
  __shared__ uint32_t L[256 * 8];
  for (int i = 0; i < 8; ++i) L[i * 256 + threadIdx.x] = 4 * (i * 256 + threadIdx.x);   // identity: a chain of reads
  __syncthreads();
  uint32_t a0 = 4 * threadIdx.x;
  for (int i = 0; i < ITERS; ++i) { for (int k = 0; k < 8; ++k) { asm volatile("ds_read_b32 %0, %0\n s_waitcnt lgkmcnt(0)" : "+v"(a0)); } }
  out[blockIdx.x * 256 + threadIdx.x] = a0; }
 OPK(mullo, B_MULLO) OPK(mulhi, B_MULHI) OPK(mul24, B_MUL24) OPK(sad, B_SAD) OPK(bitop3, B_BITOP3)
OPK(min3, B_MIN3) OPK(pkmax, B_PKMAX) OPK(bcnt, B_BCNT) OPK(ffbl, B_FFBL) OPK(cndm, B_CNDM) OPK(cndonly, B_CNDONLY) OPK(mad64, B_MAD64) OPK(shl64, B_SHL64)
typedef void (*KF)(uint32_t*, uint32_t);
int main() {
  struct { const char* n; KF f; int insts; } ks[] = {
    {"xor", k_xor, 1}, {"xor 1 chain", k_xor1, 1}, {"sad 1 chain", k_sad1, 1}, {"ds_read chain(+shl)", k_lds1, 1}, {"mul_lo_u32", k_mullo, 1}, {"mul_hi_u32", k_mulhi, 1}, {"mul_u32_u24", k_mul24, 1},
    {"sad_hi_u8", k_sad, 1}, {"bitop3", k_bitop3, 1}, {"min3_u32", k_min3, 1}, {"pk_max_i16", k_pkmax, 1},
    {"bcnt", k_bcnt, 1}, {"ffbl", k_ffbl, 1}, {"cmp+cndmask", k_cndm, 2}, {"cndmask(vcc)", k_cndonly, 1}, {"mad_u64_u32(+2 xor/mov)", k_mad64, 2}, {"lshlrev_b64(+movs)", k_shl64, 1}};
  uint32_t* out; hipMalloc(&out, 1024 * 256 * 4 * 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int wps : {1, 2, 4}) {
    int blocks = 256 * wps;
    for (auto& k : ks) {
      k.f<<<blocks, 256>>>(out, 7); hipDeviceSynchronize();
      hipEventRecord(e0); for (int r = 0; r < 5; ++r) k.f<<<blocks, 256>>>(out, 7); hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 5;
      double ops_per_simd = (double)wps * ITERS * 8;     // wave-instructions per SIMD (per op)
      double ns_per = ms * 1e6 / ops_per_simd;
      printf("waves/SIMD=%d %-26s %.3f ns per wave-op per SIMD (%.2f cyc @2.4GHz)\n", wps, k.n, ns_per, ns_per * 2.4);
    }
  }
  return 0;
}
