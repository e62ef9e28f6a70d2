// policy_mlp.hip -- the SAC policy network forward on observation rows (bf16 MFMA, gfx950).
//
// What it replaces: `trainer.compute_action(obs)` of scripts/rollout.py:84-86 for the policy
// model of scripts/experiments/warehouse-*-sac/*.yaml (policy_model: relu MLP, hidden_layer_sizes
// [256,256] Small / [512,512] Medium / [1024,256] Large, 9 action logits), evaluated for every
// agent row of a batch: explore = 0 -> argmax (compute_action(explore=False)), explore = 1 ->
// a sample of Categorical(logits) by Gumbel-max with philox noise.
//
// Design (policy kernel):
//  * Column-major activations.  Every layer is H^T = W . X^T: the 32 samples of a wave are the
//    COLUMNS of a v_mfma_f32_32x32x16_bf16 tile, hidden units are its rows.  A 32x32 f32
//    accumulator keeps its column on the lane and its rows in the 16 registers, so after bias +
//    ReLU + v_cvt_pk_bf16_f32, registers 8s..8s+7 ARE the B operand of k-step s of the next layer
//    (cdna_hip_programming.md §3, "accumulator tile as the next MFMA's operand"): activations
//    never leave registers.  The permuted k order this implies is folded into the packed weights.
//  * Layer 0 is streamed in chunks of CH hidden tiles straight into layer 1's accumulators, so
//    only layer 1's [H1 x 32] accumulators (+ one chunk) are live: <= 512 registers per lane at
//    one wave per SIMD for all three variants.
//  * Weights are packed once (wh_mlp_pack) in fragment order: one MFMA A operand = 64 lanes x 16
//    contiguous bytes, one dwordx4 load per lane.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <string.h>
#include <vector>

#include "philox.h"
#include "warehouse_amd.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int MT = 256;                 // threads per workgroup: 4 waves x 32 samples
constexpr uint32_t PUR_MLP = 5;         // philox purpose (1-4 are the simulator's, philox.h)

template <int IN_, int H0_, int H1_, int CH_>
struct Net {
  static constexpr int IN = IN_, INP = (IN_ + 15) / 16 * 16, H0 = H0_, H1 = H1_, CH = CH_;
  static constexpr int KQ0 = INP / 16;        // layer-0 k-steps
  static constexpr int T0 = H0 / 32, T1 = H1 / 32;
  static constexpr int OUT = 9;
  // packed blob, in 16-byte fragments: W0 [T0][KQ0][64], W1 [T1][T0][2][64], W2 [T1][2][64],
  // then f32 biases b0[H0], b1[H1], b2[32]
  static constexpr int64_t W0F = (int64_t)T0 * KQ0 * 64;
  static constexpr int64_t W1F = (int64_t)T1 * T0 * 2 * 64;
  static constexpr int64_t W2F = (int64_t)T1 * 2 * 64;
  static constexpr int64_t BYTES = (W0F + W1F + W2F) * 16 + 4 * (H0 + H1 + 32);
  static_assert(H0 % 32 == 0 && H1 % 32 == 0 && T0 % CH == 0, "tile shapes");
};

struct MlpArgs {
  const void* packed;
  int64_t rows;
  const float* obs;
  float* logits;
  int32_t* actions;
  int32_t explore;
  uint32_t k0, k1, step;
};

__device__ __forceinline__ bf16x8 frag(const u32x4* p) { return __builtin_bit_cast(bf16x8, *p); }

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// bias + ReLU on a 32x32 accumulator tile whose rows start at hidden unit `base`, then the two
// bf16 B-operand fragments (k-steps s = 0, 1) of the next layer.  Accumulator register g of lane
// half h holds row (g&3) + 8(g>>2) + 4h.
__device__ __forceinline__ void relu_to_frags(f32x16 t, const float* __restrict__ bias, int base, int h,
                                              bf16x8& f0, bf16x8& f1) {
#pragma unroll
  for (int G = 0; G < 4; ++G) {
    const f32x4 bv = *reinterpret_cast<const f32x4*>(bias + base + 8 * G + 4 * h);
#pragma unroll
    for (int e = 0; e < 4; ++e) t[4 * G + e] = fmaxf(t[4 * G + e] + bv[e], 0.0f);
  }
  f32x8 lo, hi;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    lo[j] = t[j];
    hi[j] = t[8 + j];
  }
  f0 = __builtin_convertvector(lo, bf16x8);
  f1 = __builtin_convertvector(hi, bf16x8);
}

template <class N>
__global__ __launch_bounds__(MT) void k_mlp(MlpArgs a) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int64_t s0 = ((int64_t)blockIdx.x * (MT / 64) + w) * 32;
  if (s0 >= a.rows) return;                       // whole wave past the end
  const int64_t row = s0 + r;
  const bool live = row < a.rows;
  const u32x4* W0 = static_cast<const u32x4*>(a.packed);
  const u32x4* W1 = W0 + N::W0F;
  const u32x4* W2 = W1 + N::W1F;
  const float* b0 = reinterpret_cast<const float*>(W2 + N::W2F);
  const float* b1 = b0 + N::H0;
  const float* b2 = b1 + N::H1;

  // X^T as layer-0 B fragments: lane (r, h) holds obs[row][16q + 8h + j]
  bf16x8 xb[N::KQ0];
  const float* x = a.obs + (live ? row : 0) * N::IN;
#pragma unroll
  for (int q = 0; q < N::KQ0; ++q) {
    f32x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 16 * q + 8 * h + j;
      v[j] = (live && k < N::IN) ? x[k] : 0.0f;
    }
    xb[q] = __builtin_convertvector(v, bf16x8);
  }

  f32x16 t1[N::T1];
#pragma unroll
  for (int n = 0; n < N::T1; ++n) t1[n] = f32x16{};
  for (int c = 0; c < N::T0; c += N::CH) {
    bf16x8 hb[N::CH][2];
#pragma unroll
    for (int m = 0; m < N::CH; ++m) {
      f32x16 t0{};
#pragma unroll
      for (int q = 0; q < N::KQ0; ++q) t0 = mfma(frag(W0 + ((int64_t)(c + m) * N::KQ0 + q) * 64 + lane), xb[q], t0);
      relu_to_frags(t0, b0, 32 * (c + m), h, hb[m][0], hb[m][1]);
    }
#pragma unroll
    for (int n = 0; n < N::T1; ++n)
#pragma unroll
      for (int m = 0; m < N::CH; ++m)
#pragma unroll
        for (int s = 0; s < 2; ++s)
          t1[n] = mfma(frag(W1 + (((int64_t)n * N::T0 + c + m) * 2 + s) * 64 + lane), hb[m][s], t1[n]);
  }

  f32x16 lg{};
#pragma unroll
  for (int n = 0; n < N::T1; ++n) {
    bf16x8 f0, f1;
    relu_to_frags(t1[n], b1, 32 * n, h, f0, f1);
    lg = mfma(frag(W2 + ((int64_t)n * 2 + 0) * 64 + lane), f0, lg);
    lg = mfma(frag(W2 + ((int64_t)n * 2 + 1) * 64 + lane), f1, lg);
  }

  // logit o of sample r: o 0-3 in lane r regs 0-3, o 4-7 in lane r+32 regs 0-3, o 8 in lane r reg 4
  float up[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) up[e] = __shfl_xor(lg[e], 32);
  if (h != 0 || !live) return;
  float z[N::OUT];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    z[e] = lg[e] + b2[e];
    z[4 + e] = up[e] + b2[4 + e];
  }
  z[8] = lg[4] + b2[8];
  if (a.logits) {
#pragma unroll
    for (int o = 0; o < N::OUT; ++o) a.logits[row * N::OUT + o] = z[o];
  }
  if (!a.actions) return;
  float best = -INFINITY;
  int arg = 0;
  if (a.explore) {
    // Gumbel-max: argmax(z + g), g = -log(-log u), u in (0,1) from philox(row, step)
    const uint4 b0w = philox10(make_uint4((uint32_t)row, (uint32_t)(row >> 32), a.step, PUR_MLP << 24), a.k0, a.k1);
    const uint4 b1w = philox10(make_uint4((uint32_t)row, (uint32_t)(row >> 32), a.step, (PUR_MLP << 24) | 1u), a.k0, a.k1);
    const uint4 b2w = philox10(make_uint4((uint32_t)row, (uint32_t)(row >> 32), a.step, (PUR_MLP << 24) | 2u), a.k0, a.k1);
    const uint32_t u32[12] = {b0w.x, b0w.y, b0w.z, b0w.w, b1w.x, b1w.y, b1w.z, b1w.w, b2w.x, b2w.y, b2w.z, b2w.w};
#pragma unroll
    for (int o = 0; o < N::OUT; ++o) {
      const float u = ((float)(u32[o] >> 8) + 0.5f) * (1.0f / 16777216.0f);
      const float v = z[o] - __logf(-__logf(u));
      if (v > best) { best = v; arg = o; }
    }
  } else {
#pragma unroll
    for (int o = 0; o < N::OUT; ++o)
      if (z[o] > best) { best = z[o]; arg = o; }   // first maximum wins (numpy/torch argmax)
  }
  a.actions[row] = arg;
}

// ------------------------------------------------------------------------------------- host
uint16_t to_bf16(float f) {   // round to nearest even (NaN not expected in weights)
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

template <class N>
std::vector<uint8_t> pack(const float* w0, const float* b0, const float* w1, const float* b1,
                          const float* w2, const float* b2) {
  std::vector<uint8_t> blob(N::BYTES, 0);
  uint16_t* f = reinterpret_cast<uint16_t*>(blob.data());
  // operand `op` = one MFMA A operand = 64 lanes x 8 bf16; the kernel reads lane l's 16 bytes
  auto put = [&](int64_t op, int lane, int j, float v) { f[(op * 64 + lane) * 8 + j] = to_bf16(v); };
  // W0 [H0][IN]: natural k order (X^T fragments come from memory)
  for (int m = 0; m < N::T0; ++m)
    for (int q = 0; q < N::KQ0; ++q)
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 8; ++j) {
          const int k = 16 * q + 8 * (l >> 5) + j;
          put((int64_t)m * N::KQ0 + q, l, j, k < N::IN ? w0[(int64_t)(32 * m + (l & 31)) * N::IN + k] : 0.0f);
        }
  // W1 [H1][H0], W2 [9][H1]: k order of an accumulator-as-operand fragment
  auto kperm = [](int i, int s, int l, int j) { return 32 * i + 16 * s + 8 * (j >> 2) + 4 * (l >> 5) + (j & 3); };
  int64_t o1 = N::W0F / 64;                // operand (64-lane fragment) index of W1
  for (int n = 0; n < N::T1; ++n)
    for (int i = 0; i < N::T0; ++i)
      for (int s = 0; s < 2; ++s)
        for (int l = 0; l < 64; ++l)
          for (int j = 0; j < 8; ++j)
            put(o1 + ((int64_t)n * N::T0 + i) * 2 + s, l, j, w1[(int64_t)(32 * n + (l & 31)) * N::H0 + kperm(i, s, l, j)]);
  int64_t o2 = (N::W0F + N::W1F) / 64;
  for (int i = 0; i < N::T1; ++i)
    for (int s = 0; s < 2; ++s)
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 8; ++j) {
          const int o = l & 31;
          put(o2 + (int64_t)i * 2 + s, l, j, o < N::OUT ? w2[(int64_t)o * N::H1 + kperm(i, s, l, j)] : 0.0f);
        }
  float* bias = reinterpret_cast<float*>(blob.data() + (N::W0F + N::W1F + N::W2F) * 16);
  memcpy(bias, b0, 4 * N::H0);
  memcpy(bias + N::H0, b1, 4 * N::H1);
  memcpy(bias + N::H0 + N::H1, b2, 4 * N::OUT);
  return blob;
}

struct MlpKernel {
  int in, h0, h1;
  int64_t bytes;
  void (*fwd)(MlpArgs);
  std::vector<uint8_t> (*pack)(const float*, const float*, const float*, const float*, const float*, const float*);
};

template <int IN, int H0, int H1, int CH>
MlpKernel make_mlp() {
  using N = Net<IN, H0, H1, CH>;
  return MlpKernel{IN, H0, H1, N::BYTES, k_mlp<N>, pack<N>};
}

const MlpKernel* find_mlp(const wh_mlp_desc* d) {
  // the policy_model shapes of scripts/experiments/warehouse-{small,medium,large}-sac/*.yaml
  static const MlpKernel reg[] = {
      make_mlp<37, 256, 256, 4>(),     // Small:  obs 9*4+1,  [256, 256]
      make_mlp<82, 512, 512, 2>(),     // Medium: obs 9*9+1,  [512, 512]
      make_mlp<145, 1024, 256, 8>(),   // Large:  obs 9*16+1, [1024, 256]
  };
  if (!d || d->out_dim != 9) return nullptr;
  for (const auto& k : reg)
    if (k.in == d->in_dim && k.h0 == d->hidden0 && k.h1 == d->hidden1) return &k;
  return nullptr;
}

int hip_rc(hipError_t e) { return e == hipSuccess ? WH_OK : WH_EHIP + (int)e; }

}  // namespace

extern "C" {

int wh_mlp_query(const wh_mlp_desc* d, int64_t* packed_bytes) {
  const MlpKernel* k = find_mlp(d);
  if (!k) return d ? WH_ENOTSUP : WH_EINVAL;
  if (packed_bytes) *packed_bytes = k->bytes;
  return WH_OK;
}

int wh_mlp_pack(const wh_mlp_desc* d, const float* w0, const float* b0, const float* w1,
                const float* b1, const float* w2, const float* b2, void* packed) {
  const MlpKernel* k = find_mlp(d);
  if (!k) return d ? WH_ENOTSUP : WH_EINVAL;
  if (!w0 || !b0 || !w1 || !b1 || !w2 || !b2 || !packed) return WH_EINVAL;
  std::vector<uint8_t> blob = k->pack(w0, b0, w1, b1, w2, b2);
  return hip_rc(hipMemcpy(packed, blob.data(), blob.size(), hipMemcpyHostToDevice));
}

int wh_mlp_forward(const wh_mlp_desc* d, const void* packed, int64_t rows, const float* obs,
                   float* logits, int32_t* actions, int32_t explore, uint64_t seed, uint32_t step,
                   void* stream) {
  const MlpKernel* k = find_mlp(d);
  if (!k) return d ? WH_ENOTSUP : WH_EINVAL;
  if (rows < 0) return WH_EINVAL;
  if (rows == 0) return WH_OK;
  if (!packed || !obs || (!logits && !actions)) return WH_EINVAL;
  MlpArgs a{packed, rows, obs, logits, actions, explore ? 1 : 0, (uint32_t)(seed & 0xFFFFFFFFu),
            (uint32_t)(seed >> 32), step};
  const int64_t rows_per_wg = 32 * (MT / 64);
  hipLaunchKernelGGL(k->fwd, dim3((unsigned)((rows + rows_per_wg - 1) / rows_per_wg)), dim3(MT), 0,
                     (hipStream_t)stream, a);
  return hip_rc(hipGetLastError());
}

}  // extern "C"
