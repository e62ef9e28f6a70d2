// policy_mlp.hip -- the SAC policy network forward on observation rows (bf16 MFMA, gfx950).
//
// What it replaces: `trainer.compute_action(obs)` of scripts/rollout.py:72 for the policy
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
//  * Every layer runs once per sample (struct Net: MODE 0 keeps all layer-0 activations, MODE 1
//    all layer-1 accumulators, whichever fits 256 registers at two waves per SIMD).
//  * Layer 0's bias rides in the MFMA (two input columns fixed at 1.0 carry b0 as bf16 hi + lo);
//    ReLU runs on the packed bf16 bits (v_pk_max_i16 with 0).
//  * Weights are packed once (wh_mlp_pack) in consumption order, one MFMA A operand = 64 lanes x
//    16 contiguous bytes, and streamed chunk by chunk into two LDS stages by LDS-DMA
//    (global_load_lds_dwordx4, lane-linear); all 8 waves read every staged operand.
//  * Persistent workgroups (one per CU) walk 256-row tasks, so the weight pipeline and the
//    biases carry over from task to task.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>
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

constexpr uint32_t PUR_MLP = 5;         // philox purpose (1-4 are the simulator's, philox.h)

// One launch shape per network; every layer runs exactly once per sample.  A wave computes 32
// samples (the MFMA tile's columns); WAVES waves per workgroup share every staged weight operand,
// which streams through two LDS stages in consumption order.  Two dataflows, by which layer's
// activations fit the registers:
//  MODE 0 (H0 <= 512): layer 0 first, all H0 hidden units kept as bf16 B-operand fragments (T0 x 8
//    VGPRs); then layer 1 row tile by row tile with K = H0 at hand, each tile's bias + ReLU
//    feeding its two layer-2 MFMAs at once.  Stream: L0C chunks of L0T layer-0 tiles, then L1C
//    chunks of L1T layer-1 row tiles, each followed by its two W2 operands.
//  MODE 1 (H1 <= 256, Large): all T1 layer-1 accumulators live (T1 x 16 registers); layer-0 tiles
//    are produced one at a time and consumed at once by every layer-1 tile.  Stream: chunks of L0T
//    units {W0 tile t [KQ0], W1 k-steps of t for every row tile [T1][2]}, then W2 [T1][2].
template <int IN_, int H0_, int H1_, int WAVES_, int MODE_, int L0T_, int L1T_, bool XPF_ = false>
struct Net {
  // inputs padded to whole k-steps, with two spare columns IN, IN+1 = 1.0 carrying b0 as a
  // bf16 hi + lo pair, so layer 0's bias is added inside the MFMA at ~f32 precision
  static constexpr int IN = IN_, INP = (IN_ + 2 + 15) / 16 * 16, H0 = H0_, H1 = H1_, OUT = 9;
  static constexpr int KQ0 = INP / 16;        // layer-0 k-steps
  static constexpr int T0 = H0 / 32, T1 = H1 / 32;
  static constexpr int WAVES = WAVES_, MT = 64 * WAVES_, ROWS = 32 * WAVES_;   // samples per task
  static constexpr int MODE = MODE_, L0T = L0T_, L1T = L1T_;
  // MODE 0: load the next task's X during layer 1 (registers permitting: measured a gain where
  // T0 x 8 leaves room -- Small -- and a loss at Medium, whose 256 registers then spill)
  static constexpr bool XPF = XPF_ && MODE == 0;
  // operands (1 KiB MFMA A fragments) per unit and chunk
  static constexpr int U0 = MODE == 0 ? KQ0 : KQ0 + 2 * T1;   // per layer-0 tile
  static constexpr int U1 = 2 * T0 + 2;                       // MODE 0: per layer-1 row tile (+ its W2)
  static constexpr int L0C = T0 / L0T, L0OPS = L0T * U0;
  static constexpr int L1C = MODE == 0 ? T1 / L1T : 1, L1OPS = MODE == 0 ? L1T * U1 : 2 * T1;
  static constexpr int NCH = L0C + L1C;
  static constexpr int SOPS = L0OPS > L1OPS ? L0OPS : L1OPS;   // one LDS stage
  static constexpr int64_t STREAM_OPS = (int64_t)L0C * L0OPS + (int64_t)L1C * L1OPS;
  static constexpr int64_t BIAS_OFF = STREAM_OPS * 1024;
  static constexpr int64_t BYTES = BIAS_OFF + 4 * (H0 + H1 + 32);
  static constexpr int STAGES = 2;            // chunk g in use, chunk g+1 landing
  static constexpr int LDS_BYTES = STAGES * SOPS * 1024 + 4 * H1;
  static_assert(H0 % 32 == 0 && H1 % 32 == 0 && T0 % L0T == 0 && (MODE == 1 || T1 % L1T == 0), "tile shapes");
  static_assert(LDS_BYTES <= 160 * 1024, "two weight stages + b1 must fit the 160 KiB LDS");
  __host__ __device__ static constexpr int64_t chunk_off(int c) {
    return c < L0C ? (int64_t)c * L0OPS : (int64_t)L0C * L0OPS + (int64_t)(c - L0C) * L1OPS;
  }
  __host__ __device__ static constexpr int chunk_ops(int c) { return c < L0C ? L0OPS : L1OPS; }
};

struct MlpArgs {
  const void* packed;
  int64_t rows;
  const float* obs;
  float* logits;
  int32_t* actions;
  int32_t explore;
  uint32_t k0, k1, step;
  int32_t ablate;   // timing experiments only (env WH_MLP_ABLATE): 1 = no staging in the loop
  const u32x4* xfrag;   // non-null: X already in fragment order (wh_observe_x), obs unused
};

__device__ __forceinline__ bf16x8 frag(const u32x4* p) { return __builtin_bit_cast(bf16x8, *p); }

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

typedef short s16x8 __attribute__((ext_vector_type(8)));

// ReLU after the bf16 rounding, on the packed bits: a bf16 with the sign bit set is a negative
// int16, so v_pk_max_i16(x, 0) is max(x, +0) for two values per op (round(max(v,0)) ==
// max(round(v),0) since rounding keeps the sign).
__device__ __forceinline__ bf16x8 relu_bf16(bf16x8 v) {
  return __builtin_bit_cast(bf16x8, __builtin_elementwise_max(__builtin_bit_cast(s16x8, v), (s16x8){}));
}

// bias + ReLU on a 32x32 accumulator tile whose rows start at hidden unit `base`, then the two
// bf16 B-operand fragments (k-steps s = 0, 1) of the next layer.  Accumulator register g of lane
// half h holds row (g&3) + 8(g>>2) + 4h.
__device__ __forceinline__ void relu_to_frags(f32x16 t, const float* bias, int base, int h,
                                              bf16x8& f0, bf16x8& f1) {
#pragma unroll
  for (int G = 0; G < 4; ++G) {
    const f32x4 bv = *reinterpret_cast<const f32x4*>(bias + base + 8 * G + 4 * h);
#pragma unroll
    for (int e = 0; e < 4; ++e) t[4 * G + e] += bv[e];
  }
  f32x8 lo, hi;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    lo[j] = t[j];
    hi[j] = t[8 + j];
  }
  f0 = relu_bf16(__builtin_convertvector(lo, bf16x8));
  f1 = relu_bf16(__builtin_convertvector(hi, bf16x8));
}

// Layer-0 tile (bias already inside the MFMA) -> the two bf16 B-operand fragments.
__device__ __forceinline__ void relu_to_frags_nb(f32x16 t, bf16x8& f0, bf16x8& f1) {
  f32x8 lo, hi;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    lo[j] = t[j];
    hi[j] = t[8 + j];
  }
  f0 = relu_bf16(__builtin_convertvector(lo, bf16x8));
  f1 = relu_bf16(__builtin_convertvector(hi, bf16x8));
}

// Timing-only ablations (builds with -DWH_MLP_ABLATION, env WH_MLP_ABLATE; results are wrong):
// 2 = no bias/ReLU/bf16 conversion (accumulator bits reused as fragments), 4 = no chunk barriers,
// 8 = no observation loads, 16 = no wait for the next chunk's LDS-DMA before the barrier.
#ifdef WH_MLP_ABLATION
#define MLP_ABL(a, bit) (((a).ablate & (bit)) != 0)
#else
#define MLP_ABL(a, bit) false
#endif
__device__ __forceinline__ void raw_frags(const f32x16& t, bf16x8& f0, bf16x8& f1) {
  f0 = __builtin_bit_cast(bf16x8, (f32x4){t[0], t[1], t[2], t[3]});
  f1 = __builtin_bit_cast(bf16x8, (f32x4){t[8], t[9], t[10], t[11]});
}

// Chunk c of the packed stream, global -> LDS stage by LDS-DMA: wave w copies every WAVES-th
// operand, one global_load_lds_dwordx4 (1 KiB, lane-linear) per operand.
template <class N>
__device__ __forceinline__ void stage_chunk(const u32x4* __restrict__ src, u32x4* dst, int nops, int w, int lane) {
  for (int o = w; o < nops; o += N::WAVES)
    __builtin_amdgcn_global_load_lds(src + o * 64 + lane, dst + o * 64, 16, 0, 0);
}

// NOPS consecutive staged operands, each fed to MFMA f(i, A fragment): fragments are read from LDS
// DEPTH groups of GS ahead of their MFMAs; the sched_barriers keep the reads ahead of the MFMAs and
// stop the compiler from hoisting a whole chunk's reads (NOPS x 4 VGPRs would spill).
struct NoPre {
  __device__ __forceinline__ void operator()(int, int) const {}
};
template <int NOPS, int GS_ = 4, int DEPTH = 2, class F, class P = NoPre>
__device__ __forceinline__ void stream_ops(const u32x4* S, int lane, F&& f, P&& pre = P{}) {
  constexpr int GS = NOPS % GS_ == 0 ? GS_ : 2, NG = NOPS / GS;
  static_assert(NOPS % GS == 0 && NG >= DEPTH, "operand groups");
  bf16x8 buf[DEPTH + 1][GS];
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
#pragma unroll
    for (int i = 0; i < GS; ++i) buf[d][i] = frag(S + (d * GS + i) * 64 + lane);
#pragma unroll
  for (int gi = 0; gi < NG; ++gi) {
    if (gi + DEPTH < NG) {
#pragma unroll
      for (int i = 0; i < GS; ++i) buf[(gi + DEPTH) % (DEPTH + 1)][i] = frag(S + ((gi + DEPTH) * GS + i) * 64 + lane);
    }
    pre(gi, NG);                                   // (k_mlp16: this group's share of the next chunk's DMA)
    __builtin_amdgcn_sched_barrier(0);             // later groups' reads issue BEFORE this group's MFMAs
#pragma unroll
    for (int i = 0; i < GS; ++i) f(gi * GS + i, buf[gi % (DEPTH + 1)][i]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Logit o of sample r sits in the output tile as: o 0-3 in lane r regs 0-3, o 4-7 in lane r+32
// regs 0-3, o 8 in lane r reg 4 (C/D map row = (reg&3) + 8(reg>>2) + 4(lane>>5)).  Adds b2, then
// writes logits and/or the argmax (first maximum) or a Gumbel-max sample.
__device__ __forceinline__ void emit_logits(const f32x16& lg, const float* b2, int64_t row, bool live, int h,
                                            const MlpArgs& a) {
  float up[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) up[e] = __shfl_xor(lg[e], 32);
  if (h == 0 && live) {
    constexpr int OUT = 9;
    float z[OUT];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      z[e] = lg[e] + b2[e];
      z[4 + e] = up[e] + b2[4 + e];
    }
    z[8] = lg[4] + b2[8];
    if (a.logits) {
#pragma unroll
      for (int o = 0; o < OUT; ++o) a.logits[row * OUT + o] = z[o];
    }
    if (a.actions) {
      float best = -INFINITY;
      int arg = 0;
      if (a.explore) {
        // Gumbel-max: argmax(z + g), g = -log(-log u), u in (0,1) from philox(row, step)
        uint32_t u32[12];
#pragma unroll
        for (int b = 0; b < 3; ++b) {
          const uint4 v = philox10(make_uint4((uint32_t)row, (uint32_t)(row >> 32), a.step, (PUR_MLP << 24) | (uint32_t)b),
                                   a.k0, a.k1);
          u32[4 * b] = v.x;
          u32[4 * b + 1] = v.y;
          u32[4 * b + 2] = v.z;
          u32[4 * b + 3] = v.w;
        }
#pragma unroll
        for (int o = 0; o < OUT; ++o) {
          const float u = ((float)(u32[o] >> 8) + 0.5f) * (1.0f / 16777216.0f);
          const float v = z[o] - __logf(-__logf(u));
          if (v > best) { best = v; arg = o; }
        }
      } else {
#pragma unroll
        for (int o = 0; o < OUT; ++o)
          if (z[o] > best) { best = z[o]; arg = o; }   // first maximum wins (numpy/torch argmax)
      }
      a.actions[row] = arg;
    }
  }
}

template <class N>
__global__ __launch_bounds__(N::MT) void k_mlp(MlpArgs a) {
  // two weight stages + b1; A fragments are ds_read_b128 at operand*1 KiB + lane*16: conflict-free,
  // and each 1 KiB operand is read by all WAVES waves.
  // ONE __shared__ object: with a second one beside the LDS-DMA target, hipcc (ROCm 7.2) emits
  // vmcnt(0) before ds_reads and the staging stops overlapping (cdna_hip_programming.md §5, trap (a))
  __shared__ __attribute__((aligned(16))) u32x4 lds[N::STAGES * N::SOPS * 64 + N::H1 / 4];
  float* b1s = reinterpret_cast<float*>(lds + N::STAGES * N::SOPS * 64);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (LDS-DMA base in m0)
  const int r = lane & 31, h = lane >> 5;
  const u32x4* chunks = static_cast<const u32x4*>(a.packed);
  const float* gb = reinterpret_cast<const float*>(static_cast<const uint8_t*>(a.packed) + N::BIAS_OFF);
  const float* b2 = gb + N::H0 + N::H1;
  // Persistent: one workgroup per CU walks the ROWS-sample tasks, so the weight pipeline (and b1)
  // carry over from task to task instead of restarting behind every workgroup's prologue.
  const int64_t ntask = (a.rows + N::ROWS - 1) / N::ROWS;
  const int my_tasks = (int)((ntask - blockIdx.x + gridDim.x - 1) / gridDim.x);

  for (int i = tid; i < N::H1; i += N::MT) b1s[i] = gb[N::H0 + i];
  auto stage_of = [&](int gg) { return lds + (gg & 1) * (N::SOPS * 64); };
  // running chunk counter gg = task_iter * NCH + c; chunk gg is stream chunk gg % NCH
  auto fetch = [&](int gg) {
    if (gg < my_tasks * N::NCH && !(a.ablate & 1)) {
      const int c = gg % N::NCH;
      stage_chunk<N>(chunks + N::chunk_off(c) * 64, stage_of(gg), N::chunk_ops(c), w, lane);
    }
  };
  fetch(0);
  __builtin_amdgcn_s_waitcnt(0x0F70);             // vmcnt(0): chunk 0 landed
  __syncthreads();

  // X^T fragments: lane (r,h) holds obs[row][16q+8h+j] (bias columns IN, IN+1 = 1.0)
  // (raw values of k-steps [q0, q1) at xr[(q - q0) * 8 + j])
  auto load_x = [&](int64_t xrow, float* xr, int q0 = 0, int q1 = N::KQ0) {
    const float* x = a.obs + (xrow < a.rows ? xrow : 0) * N::IN;
#pragma unroll
    for (int q = q0; q < q1; ++q)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 16 * q + 8 * h + j;
        xr[(q - q0) * 8 + j] = MLP_ABL(a, 8) ? 0.5f : x[k < N::IN ? k : N::IN - 1];   // clamp, then select
      }
  };
  auto cvt_x = [&](const float* xr, bool lv, bf16x8 (&xb)[N::KQ0], int q0 = 0, int q1 = N::KQ0) {
#pragma unroll
    for (int q = q0; q < q1; ++q) {
      f32x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 16 * q + 8 * h + j;
        v[j] = k < N::IN ? (lv ? xr[(q - q0) * 8 + j] : 0.0f) : (k < N::IN + 2 ? 1.0f : 0.0f);
      }
      xb[q] = __builtin_convertvector(v, bf16x8);
    }
  };
  // fragment-order X (wh_observe_x): the wave's 32 rows are tile task * WAVES + w, one coalesced
  // 16-byte load per k-step (tiles past the last row read tile 0: those rows are never emitted)
  const bool xf = a.xfrag != nullptr;
  auto load_xf = [&](int64_t task_i, bf16x8 (&xb)[N::KQ0]) {
    int64_t tile = task_i * N::WAVES + w;
    tile = tile * 32 < a.rows ? tile : 0;
    const u32x4* src = a.xfrag + tile * (N::KQ0 * 64) + lane;
#pragma unroll
    for (int q = 0; q < N::KQ0; ++q) xb[q] = frag(src + q * 64);
  };
  bf16x8 xb[N::KQ0];
  if (my_tasks > 0) {
    if (xf) {
      load_xf(blockIdx.x, xb);
    } else {
      const int64_t row0 = (int64_t)blockIdx.x * N::ROWS + w * 32 + r;
      float xr[N::KQ0 * 8];
      load_x(row0, xr);
      cvt_x(xr, row0 < a.rows, xb);
    }
  }

  for (int it = 0; it < my_tasks; ++it) {
    const int64_t task = blockIdx.x + (int64_t)it * gridDim.x;
    const int64_t row = task * N::ROWS + w * 32 + r;
    const bool live = row < a.rows;               // (a wave past the end still joins the barriers)
    const int base = it * N::NCH;
    if (!xf && !N::XPF && it > 0) {               // X of this task, loaded now
      float xr[N::KQ0 * 8];
      load_x(row, xr);
      cvt_x(xr, live, xb);
    }
    // MODE 0: the NEXT task's rows are loaded during layer-1 chunks and converted after their
    // barriers (X is dead once layer 0 is done), so no task starts behind an HBM round trip; in NS
    // parts of QP k-steps, part p during chunk PF + p, to keep the raw f32 values within the
    // register budget
    constexpr int NS = N::L1C >= 3 ? 2 : 1;      // parts, one per chunk
    constexpr int QP = (N::KQ0 + NS - 1) / NS, PF = N::L1C - 1 - NS;  // k-steps per part, first chunk
    static_assert(N::MODE == 1 || PF >= 0, "layer-1 chunks to prefetch in");
    const int64_t row_next = row + (int64_t)gridDim.x * N::ROWS;
    const bool has_next = it + 1 < my_tasks;

    f32x16 lg{};
    if constexpr (N::MODE == 0) {
      // layer 0, once: every hidden unit of the wave's 32 samples as bf16 fragments in registers
      bf16x8 hb[N::T0][2];
#pragma unroll
      for (int c = 0; c < N::L0C; ++c) {
        const int g = base + c;
        fetch(g + 1);
        f32x16 acc{};
        stream_ops<N::L0OPS>(stage_of(g), lane, [&](int i, bf16x8 af) {
          const int m = i / N::KQ0, q = i % N::KQ0;
          acc = mfma(af, xb[q], q == 0 ? f32x16{} : acc);
          if (q == N::KQ0 - 1) {
            if (MLP_ABL(a, 2)) raw_frags(acc, hb[c * N::L0T + m][0], hb[c * N::L0T + m][1]);
            else relu_to_frags_nb(acc, hb[c * N::L0T + m][0], hb[c * N::L0T + m][1]);
          }
        });
        if (!MLP_ABL(a, 4)) {
          if (!MLP_ABL(a, 16)) __builtin_amdgcn_s_waitcnt(0x0F70);     // chunk g+1 landed
          __syncthreads();                        // ... and stage g is free for chunk g+2
        }
      }
      // layer 1 row tile by row tile (K = H0 from the registers), each tile's bias + ReLU feeding
      // its two layer-2 MFMAs at once
      for (int d = 0; d < N::L1C; ++d) {
        const int g = base + N::L0C + d;
        fetch(g + 1);
        // fragment-order X: the next task's operand straight into xb during the last chunk
        if (xf && d == N::L1C - 1 && has_next) load_xf(task + gridDim.x, xb);
        float xr[QP * 8];                         // one part at a time
        if (!xf && N::XPF && d == PF && has_next) load_x(row_next, xr, 0, QP);
        if (!xf && N::XPF && NS == 2 && d == PF + 1 && has_next) load_x(row_next, xr, QP, N::KQ0);
        f32x16 acc{};
        bf16x8 f0, f1;
        // with the X prefetch: 4-op groups one group ahead (fewer fragments in flight)
        stream_ops<N::L1OPS, 4, N::XPF ? 1 : 2>(stage_of(g), lane, [&](int i, bf16x8 af) {
          const int nn = i / N::U1, k = i % N::U1;
          if (k < 2 * N::T0) {
            // (one chain per tile: splitting it into two accumulators, even / odd k-steps, measured
            // 2-6 % slower -- the dependent MFMAs are not what binds)
            acc = mfma(af, hb[k >> 1][k & 1], k == 0 ? f32x16{} : acc);
            if (k == 2 * N::T0 - 1) {
              if (MLP_ABL(a, 2)) raw_frags(acc, f0, f1);
              else relu_to_frags(acc, b1s, 32 * (d * N::L1T + nn), h, f0, f1);
            }
          } else {
            lg = mfma(af, k == 2 * N::T0 ? f0 : f1, lg);
          }
        });
        if (!MLP_ABL(a, 4)) {
          if (!MLP_ABL(a, 16)) __builtin_amdgcn_s_waitcnt(0x0F70);
          __syncthreads();
        }
        if (!xf && N::XPF && d == PF && has_next) cvt_x(xr, row_next < a.rows, xb, 0, QP);
        if (!xf && N::XPF && NS == 2 && d == PF + 1 && has_next) cvt_x(xr, row_next < a.rows, xb, QP, N::KQ0);
      }
    } else {
      // every layer-1 accumulator live; layer-0 tiles streamed through them
      f32x16 acc1[N::T1];
#pragma unroll
      for (int n = 0; n < N::T1; ++n) acc1[n] = f32x16{};
      for (int c = 0; c < N::L0C; ++c) {
        const int g = base + c;
        fetch(g + 1);
        f32x16 acc0{};
        bf16x8 hb0, hb1;
        stream_ops<N::L0OPS>(stage_of(g), lane, [&](int i, bf16x8 af) {
          const int k = i % N::U0;
          if (k < N::KQ0) {
            acc0 = mfma(af, xb[k], k == 0 ? f32x16{} : acc0);
            if (k == N::KQ0 - 1) {
              if (MLP_ABL(a, 2)) raw_frags(acc0, hb0, hb1);
              else relu_to_frags_nb(acc0, hb0, hb1);
            }
          } else {
            const int j = k - N::KQ0;
            acc1[j >> 1] = mfma(af, (j & 1) ? hb1 : hb0, acc1[j >> 1]);
          }
        });
        if (!MLP_ABL(a, 4)) {
          if (!MLP_ABL(a, 16)) __builtin_amdgcn_s_waitcnt(0x0F70);
          __syncthreads();
        }
      }
      {
        const int g = base + N::L0C;
        fetch(g + 1);
        if (xf && has_next) load_xf(task + gridDim.x, xb);   // X is dead once layer 0 is done
        bf16x8 f0, f1;
        stream_ops<N::L1OPS>(stage_of(g), lane, [&](int i, bf16x8 af) {
          if ((i & 1) == 0) {
            if (MLP_ABL(a, 2)) raw_frags(acc1[i >> 1], f0, f1);
            else relu_to_frags(acc1[i >> 1], b1s, 32 * (i >> 1), h, f0, f1);
          }
          lg = mfma(af, (i & 1) ? f1 : f0, lg);
        });
        if (!MLP_ABL(a, 4)) {
          if (!MLP_ABL(a, 16)) __builtin_amdgcn_s_waitcnt(0x0F70);
          __syncthreads();
        }
      }
    }

    emit_logits(lg, b2, row, live, h, a);
  }
}

// ------------------------------------------------------------------------ bf16 on 16x16x32 tiles
// The same network and dataflows on v_mfma_f32_16x16x32_bf16 (k_mlp16, the default).  On gfx950 a
// loop of this shape holds a higher clock under load than the 32x32x16 loop at equal cycles per FLOP
// (MI355X_MICROARCH.md, 'DVFS give-back' item 7: 1.12-1.14x FLOP/s with the operands re-read from
// LDS), and its accumulator is 4 registers instead of 16.  Layouts (cdna_hip_programming.md §3):
// A lane l = row l&15, k 8(l>>4)+j; B lane l = column l&15, same k; C lane l = column l&15, rows
// 4(l>>4)+i.  A wave still computes 32 samples: two sample tiles s of 16 columns, each staged A
// fragment (16 hidden rows x 32 k, 1 KiB) feeding one MFMA per sample tile.  Hidden units come in
// groups of 32 = two 16-row tiles whose accumulators, bias + ReLU + bf16, are register for register
// the B fragment of one 32-k step of the next layer: element j of lane l is unit
// 32m + (j < 4 ? 4g + j : 16 + 4g + j - 4), g = l>>4 (kperm16, folded into the packed weights).
//  MODE 0: layer 0 group by group (all H0 units kept as B fragments, 2 x 4 VGPRs per group), then
//    layer 1 group by group with K = H0 at hand, each group's two tiles feeding one W2 k-step.
//  MODE 1 (Large): all layer-1 tiles live (2 x 4 VGPRs each); layer-0 groups streamed through them.
//  NS (2 or 4): 16-sample tiles per wave, each staged A fragment feeding NS MFMAs.  NS = 2 at 8 waves
//    (two per SIMD, 256 registers each); NS = 4 at 4 waves (one per SIMD, 512 registers): the same
//    256 samples per task, half the fragment reads per MFMA, and the bare loop of that shape holds
//    1,998 against 1,472 TFLOP/s on random data (tools/mfma16_ceiling.hip, profiles/r05_mfma16_ceiling.txt).
template <int IN_, int H0_, int H1_, int WAVES_, int MODE_, int L0T_, int L1T_, int NS_ = 2>
struct Net16 {
  static constexpr int IN = IN_, INP = (IN_ + 2 + 31) / 32 * 32, H0 = H0_, H1 = H1_, OUT = 9;
  static constexpr int NS = NS_;
  static constexpr int KQ0 = INP / 32;              // layer-0 k-steps of 32
  static constexpr int KQX = (IN_ + 2 + 15) / 16;   // k-steps of 16 in wh_observe_x's operand
  static constexpr int G0 = H0 / 32, G1 = H1 / 32;  // groups of 32 hidden units
  static constexpr int WAVES = WAVES_, MT = 64 * WAVES_, ROWS = 16 * NS_ * WAVES_;
  static constexpr int MODE = MODE_, L0T = L0T_, L1T = L1T_;
  static_assert(NS_ == 2 || NS_ == 4, "16-sample tiles per wave: two per 32-row operand tile");
  static constexpr int U0 = MODE == 0 ? 2 * KQ0 : 2 * KQ0 + 2 * G1;   // operands per layer-0 group
  static constexpr int U1 = 2 * G0 + 1;                               // MODE 0: per layer-1 group (+ W2)
  static constexpr int L0C = G0 / L0T, L0OPS = L0T * U0;
  static constexpr int L1C = MODE == 0 ? G1 / L1T : 1, L1OPS = MODE == 0 ? L1T * U1 : G1;
  static constexpr int NCH = L0C + L1C;
  static constexpr int SOPS = L0OPS > L1OPS ? L0OPS : L1OPS;
  static constexpr int64_t STREAM_OPS = (int64_t)L0C * L0OPS + (int64_t)L1C * L1OPS;
  static constexpr int64_t BIAS_OFF = STREAM_OPS * 1024;
  static constexpr int64_t BYTES = BIAS_OFF + 4 * (H0 + H1 + 32);
  static constexpr int STAGES = 2;
  static constexpr int LDS_BYTES = STAGES * SOPS * 1024 + 4 * H1;
  static_assert(H0 % 32 == 0 && H1 % 32 == 0 && G0 % L0T == 0 && (MODE == 1 || G1 % L1T == 0), "tile shapes");
  static_assert(LDS_BYTES <= 160 * 1024, "two weight stages + b1 must fit the 160 KiB LDS");
  __host__ __device__ static constexpr int64_t chunk_off(int c) {
    return c < L0C ? (int64_t)c * L0OPS : (int64_t)L0C * L0OPS + (int64_t)(c - L0C) * L1OPS;
  }
  __host__ __device__ static constexpr int chunk_ops(int c) { return c < L0C ? L0OPS : L1OPS; }
};

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// two 16-row accumulator tiles of a group (+ bias) -> ReLU'd bf16 B fragment of the next layer
__device__ __forceinline__ bf16x8 group_frag(const f32x4& t0, const f32x4& t1) {
  const f32x8 v = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
  return relu_bf16(__builtin_convertvector(v, bf16x8));
}
__device__ __forceinline__ bf16x8 group_frag_bias(f32x4 t0, f32x4 t1, const float* bias, int base, int g) {
  const f32x4 b0 = *reinterpret_cast<const f32x4*>(bias + base + 4 * g);
  const f32x4 b1 = *reinterpret_cast<const f32x4*>(bias + base + 16 + 4 * g);
  return group_frag(t0 + b0, t1 + b1);
}

// Logits of sample tile s: output o of sample n sits in lane n + 16 (o >> 2), register o & 3.  Lanes
// 16s .. 16s + 15 gather their sample's nine and emit it (16 NS samples per wave).
template <int NS>
__device__ __forceinline__ void emit_logits16(const f32x4 (&lg)[NS], const float* b2, int64_t row0, int64_t rows,
                                              int lane, const MlpArgs& a) {
  const int n = lane & 15, part = lane >> 4;
  f32x16 z16{};
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    float v[9];
#pragma unroll
    for (int o = 0; o < 9; ++o) v[o] = __shfl(lg[s][o & 3], n + 16 * (o >> 2));
    if (part == s) {
#pragma unroll
      for (int o = 0; o < 9; ++o) z16[o] = v[o];
    }
  }
  const int64_t row = row0 + 16 * part + n;
  if (part < NS && row < rows) {
    constexpr int OUT = 9;
    float z[OUT];
#pragma unroll
    for (int o = 0; o < OUT; ++o) z[o] = z16[o] + b2[o];
    if (a.logits) {
#pragma unroll
      for (int o = 0; o < OUT; ++o) a.logits[row * OUT + o] = z[o];
    }
    if (a.actions) {
      float best = -INFINITY;
      int arg = 0;
      if (a.explore) {
        uint32_t u32[12];
#pragma unroll
        for (int b = 0; b < 3; ++b) {
          const uint4 v = philox10(make_uint4((uint32_t)row, (uint32_t)(row >> 32), a.step, (PUR_MLP << 24) | (uint32_t)b),
                                   a.k0, a.k1);
          u32[4 * b] = v.x;
          u32[4 * b + 1] = v.y;
          u32[4 * b + 2] = v.z;
          u32[4 * b + 3] = v.w;
        }
#pragma unroll
        for (int o = 0; o < OUT; ++o) {
          const float u = ((float)(u32[o] >> 8) + 0.5f) * (1.0f / 16777216.0f);
          const float v = z[o] - __logf(-__logf(u));
          if (v > best) { best = v; arg = o; }
        }
      } else {
#pragma unroll
        for (int o = 0; o < OUT; ++o)
          if (z[o] > best) { best = z[o]; arg = o; }   // first maximum wins (numpy/torch argmax)
      }
      a.actions[row] = arg;
    }
  }
}

// The next chunk's LDS-DMA pieces, spread over the current chunk's operand groups (group gi of NG
// issues this wave's pieces j in [gi NPW / NG, (gi + 1) NPW / NG)) instead of all at the chunk's
// start, where each piece's issue competes with the chunk's first fragment reads (100-185 cycles a
// piece there against ~60 among MFMAs, MI355X_MICROARCH.md).  -DWH_MLP_NO_SPREAD: at the start (A/B).
#ifndef WH_MLP_NO_SPREAD
constexpr bool kSpreadDma = true;
#else
constexpr bool kSpreadDma = false;
#endif
#ifdef WH_MLP_SPREAD_L0   // (A/B) also in MODE 0's layer-0 chunks: Medium +13 % (spills), profiles/r05_tune_ab.txt
constexpr bool kSpreadL0 = kSpreadDma;
#else
constexpr bool kSpreadL0 = false;
#endif
struct NextChunk {
  int op0;    // the chunk's first operand in the packed stream
  int dst;    // LDS stage, in 16-byte units from the kernel's LDS object
  int nops;   // 0: no next chunk
};
// One staged operand (1 KiB) by buffer-to-LDS DMA: the packed stream as a buffer resource, the
// operand's byte offset in an SGPR (soffset), the lane's 16 bytes by the one lane-offset VGPR every
// piece shares -- no 64-bit address per piece (with global_load_lds each piece's address pair was
// live across the operand stream and spread-out pieces spilled, profiles/r05_tune_ab.txt).
__device__ __forceinline__ void dma_piece(__amdgpu_buffer_rsrc_t wr, u32x4* dst, int op, int lane) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (__attribute__((address_space(3))) void*)dst, 16, lane * 16,
                                           op * 1024, 0, 0);
}
// The last kSpreadTail % of a chunk's groups issue no pieces, so the last ones have landed when the
// chunk ends (its vmcnt(0) before the barrier): 25 % -2.6 % (Medium) / -1.0 % (Large) against 0,
// 50 % no better (profiles/r05_mlptail_ab.txt).
#ifndef WH_MLP_SPREAD_TAIL
#define WH_MLP_SPREAD_TAIL 25
#endif
constexpr int kSpreadTail = WH_MLP_SPREAD_TAIL;
template <class N>
__device__ __forceinline__ void stage_slice(__amdgpu_buffer_rsrc_t wr, u32x4* lds, const NextChunk& nc, int gi,
                                            int ng_all, int w, int lane) {
  constexpr int NPW = (N::SOPS + N::WAVES - 1) / N::WAVES;   // pieces per wave, at most
  const int ng = ng_all - ng_all * kSpreadTail / 100 > 0 ? ng_all - ng_all * kSpreadTail / 100 : 1;
  if (gi >= ng) return;
  const int j0 = (gi * NPW + ng - 1) / ng, j1 = ((gi + 1) * NPW + ng - 1) / ng;
  for (int j = j0; j < j1; ++j) {
    const int o = w + N::WAVES * j;   // wave-uniform: SGPR bases, one lane offset VGPR
    if (o < nc.nops) dma_piece(wr, lds + nc.dst + o * 64, nc.op0 + o, lane);
  }
}
// (the LDS destination stays an offset from the __shared__ object: a generic pointer rebuilt from
// its low 32 bits is NULL for offset 0, and its cast to the LDS address space then yields the LDS
// null value, not offset 0)
__device__ __forceinline__ NextChunk uniform_chunk(int op0, int dst, int nops) {
  return NextChunk{__builtin_amdgcn_readfirstlane(op0), __builtin_amdgcn_readfirstlane(dst),
                   __builtin_amdgcn_readfirstlane(nops)};
}

template <class N>
__global__ __launch_bounds__(N::MT) void k_mlp16(MlpArgs a) {
  // ONE __shared__ object (see k_mlp)
  __shared__ __attribute__((aligned(16))) u32x4 lds[N::STAGES * N::SOPS * 64 + N::H1 / 4];
  float* b1s = reinterpret_cast<float*>(lds + N::STAGES * N::SOPS * 64);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = lane & 15, g = lane >> 4;
  const float* gb = reinterpret_cast<const float*>(static_cast<const uint8_t*>(a.packed) + N::BIAS_OFF);
  const float* b2 = gb + N::H0 + N::H1;
  const int64_t ntask = (a.rows + N::ROWS - 1) / N::ROWS;
  const int my_tasks = (int)((ntask - blockIdx.x + gridDim.x - 1) / gridDim.x);

  for (int i = tid; i < N::H1; i += N::MT) b1s[i] = gb[N::H0 + i];
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.packed), (short)0, (int)N::BIAS_OFF, 0x00020000);
  auto stage_of = [&](int gg) { return lds + (gg & 1) * (N::SOPS * 64); };
  auto fetch = [&](int gg) {
    if (gg < my_tasks * N::NCH) {
      const int c = gg % N::NCH, op0 = (int)N::chunk_off(c);
      u32x4* dst = stage_of(gg);
      for (int o = w; o < N::chunk_ops(c); o += N::WAVES) dma_piece(wr, dst + o * 64, op0 + o, lane);
    }
  };
  auto next_of = [&](int gg) -> NextChunk {
    if (gg >= my_tasks * N::NCH) return NextChunk{0, 0, 0};
    const int c = gg % N::NCH;
    return uniform_chunk((int)N::chunk_off(c), (gg & 1) * (N::SOPS * 64), N::chunk_ops(c));
  };
  fetch(0);
  __builtin_amdgcn_s_waitcnt(0x0F70);
  __syncthreads();

  // X^T fragments xb[q][s]: lane (n, g) holds features 32q + 8g + j of sample 16s + n of the wave
  constexpr int NS = N::NS;
  bf16x8 xb[N::KQ0][NS];
  const bool xf = a.xfrag != nullptr;
  auto load_x = [&](int64_t task_i) {
    const int64_t r0 = task_i * N::ROWS + w * (16 * NS);
    if (xf) {
      // wh_observe_x's 32x32x16 fragment order: 16-byte chunk ((tile * KQX + q16) * 64 + h * 32 + r)
      // holds features 16 q16 + 8 h + j of row r of the 32-row tile; sample tile s of the wave is
      // rows 16 (s & 1) .. + 15 of the wave's 32-row tile s >> 1
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        int64_t tile = (task_i * N::WAVES + w) * (NS / 2) + (s >> 1);
        tile = tile * 32 < a.rows ? tile : 0;
        const u32x4* src = a.xfrag + tile * (N::KQX * 64);
#pragma unroll
        for (int q = 0; q < N::KQ0; ++q) {
          const int q16 = 2 * q + (g >> 1);
          xb[q][s] = q16 < N::KQX ? frag(src + q16 * 64 + (g & 1) * 32 + 16 * (s & 1) + n) : bf16x8{};
        }
      }
    } else {
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const int64_t row = r0 + 16 * s + n;
        const bool lv = row < a.rows;
        const float* x = a.obs + (lv ? row : 0) * N::IN;
#pragma unroll
        for (int q = 0; q < N::KQ0; ++q) {
          f32x8 v;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int k = 32 * q + 8 * g + j;
            const float xv = x[k < N::IN ? k : N::IN - 1];
            v[j] = k < N::IN ? (lv ? xv : 0.0f) : (k < N::IN + 2 ? 1.0f : 0.0f);
          }
          xb[q][s] = __builtin_convertvector(v, bf16x8);
        }
      }
    }
  };
  if (my_tasks > 0) load_x(blockIdx.x);

  for (int it = 0; it < my_tasks; ++it) {
    const int64_t task = blockIdx.x + (int64_t)it * gridDim.x;
    const int base = it * N::NCH;
    const bool has_next = it + 1 < my_tasks;
    f32x4 lg[NS];
#pragma unroll
    for (int s2 = 0; s2 < NS; ++s2) lg[s2] = f32x4{};
    if constexpr (N::MODE == 0) {
      bf16x8 hb[N::G0][NS];
#pragma unroll
      for (int c = 0; c < N::L0C; ++c) {
        const int gg = base + c;
        if (!kSpreadL0) fetch(gg + 1);   // (spread: 46 more registers spilled -- layer 0's fragments are all live)
        const NextChunk nc = kSpreadL0 ? next_of(gg + 1) : NextChunk{0, 0, 0};
        f32x4 acc[2][NS];
        stream_ops<N::L0OPS>(stage_of(gg), lane, [&](int i, bf16x8 af) {
          const int m = i / N::U0, k = i % N::U0, rt = k / N::KQ0, q = k % N::KQ0;
#pragma unroll
          for (int s2 = 0; s2 < NS; ++s2) acc[rt][s2] = mfma16(af, xb[q][s2], q == 0 ? f32x4{} : acc[rt][s2]);
          if (k == N::U0 - 1) {
#pragma unroll
            for (int s2 = 0; s2 < NS; ++s2) hb[c * N::L0T + m][s2] = group_frag(acc[0][s2], acc[1][s2]);
          }
        }, [&](int gi, int ng) { stage_slice<N>(wr, lds, nc, gi, ng, w, lane); });
        __builtin_amdgcn_s_waitcnt(0x0F70);
        __syncthreads();
      }
      for (int d = 0; d < N::L1C; ++d) {
        const int gg = base + N::L0C + d;
        if (!kSpreadDma) fetch(gg + 1);
        const NextChunk nc = kSpreadDma ? next_of(gg + 1) : NextChunk{0, 0, 0};
        // the next task's X during the last chunk (X is dead once layer 0 is done; loading it for
        // the whole of layer 1 would keep its registers live beside all of layer 0's fragments)
        if (d == N::L1C - 1 && has_next) load_x(task + gridDim.x);
        f32x4 acc[2][NS];
        stream_ops<N::L1OPS>(stage_of(gg), lane, [&](int i, bf16x8 af) {
          const int uu = i / N::U1, k = i % N::U1;
          if (k < 2 * N::G0) {
            const int rt = k / N::G0, m = k % N::G0;
#pragma unroll
            for (int s2 = 0; s2 < NS; ++s2) acc[rt][s2] = mfma16(af, hb[m][s2], m == 0 ? f32x4{} : acc[rt][s2]);
          } else {
            const int u = d * N::L1T + uu;
#pragma unroll
            for (int s2 = 0; s2 < NS; ++s2)
              lg[s2] = mfma16(af, group_frag_bias(acc[0][s2], acc[1][s2], b1s, 32 * u, g), lg[s2]);
          }
        }, [&](int gi, int ng) { stage_slice<N>(wr, lds, nc, gi, ng, w, lane); });
        __builtin_amdgcn_s_waitcnt(0x0F70);
        __syncthreads();
      }
    } else {
      f32x4 acc1[2 * N::G1][NS];
#pragma unroll
      for (int v = 0; v < 2 * N::G1; ++v)
#pragma unroll
        for (int s2 = 0; s2 < NS; ++s2) acc1[v][s2] = f32x4{};
      for (int c = 0; c < N::L0C; ++c) {
        const int gg = base + c;
        if (!kSpreadDma) fetch(gg + 1);
        const NextChunk nc = kSpreadDma ? next_of(gg + 1) : NextChunk{0, 0, 0};
        f32x4 acc0[2][NS];
        bf16x8 hb0[NS];
        stream_ops<N::L0OPS, 4, 1>(stage_of(gg), lane, [&](int i, bf16x8 af) {
          const int k = i % N::U0;
          if (k < 2 * N::KQ0) {
            const int rt = k / N::KQ0, q = k % N::KQ0;
#pragma unroll
            for (int s2 = 0; s2 < NS; ++s2) acc0[rt][s2] = mfma16(af, xb[q][s2], q == 0 ? f32x4{} : acc0[rt][s2]);
            if (k == 2 * N::KQ0 - 1) {
#pragma unroll
              for (int s2 = 0; s2 < NS; ++s2) hb0[s2] = group_frag(acc0[0][s2], acc0[1][s2]);
            }
          } else {
            const int v = k - 2 * N::KQ0;
#pragma unroll
            for (int s2 = 0; s2 < NS; ++s2) acc1[v][s2] = mfma16(af, hb0[s2], acc1[v][s2]);
          }
        }, [&](int gi, int ng) { stage_slice<N>(wr, lds, nc, gi, ng, w, lane); });
        __builtin_amdgcn_s_waitcnt(0x0F70);
        __syncthreads();
      }
      {
        const int gg = base + N::L0C;
        if (!kSpreadDma) fetch(gg + 1);
        const NextChunk nc = kSpreadDma ? next_of(gg + 1) : NextChunk{0, 0, 0};
        if (has_next) load_x(task + gridDim.x);
        stream_ops<N::L1OPS, 4, 1>(stage_of(gg), lane, [&](int u, bf16x8 af) {
#pragma unroll
          for (int s2 = 0; s2 < NS; ++s2)
            lg[s2] = mfma16(af, group_frag_bias(acc1[2 * u][s2], acc1[2 * u + 1][s2], b1s, 32 * u, g), lg[s2]);
        }, [&](int gi, int ng) { stage_slice<N>(wr, lds, nc, gi, ng, w, lane); });
        __builtin_amdgcn_s_waitcnt(0x0F70);
        __syncthreads();
      }
    }
    emit_logits16<NS>(lg, b2, task * N::ROWS + w * (16 * NS), a.rows, lane, a);
  }
}

// ------------------------------------------------------------------------------------- f32 mode
// The same network in exact f32 (the reference policy is TF fp32): every layer on
// v_mfma_f32_32x32x2_f32, whose result is bit-for-bit a k-ordered f32 fmaf chain, so logits differ
// from a float32 reference only by summation order (~1e-7 relative).  Same orientation as the
// bf16 kernel: a wave's 32 samples are the tile COLUMNS, so a 32x32 f32 accumulator register g
// (rows (g&3) + 8(g>>2) + 4h on lane half h) is, after bias + ReLU, directly the B operand of one
// K = 2 step of the next layer -- the k pair (r_g, r_g + 4) is folded into the packed weights.
// Weights stream from L2 as one 256-byte A operand per MFMA, in exactly the order the MFMAs
// consume them, through a 16-deep register ring (a load issued 16 MFMAs = ~1,000 cycles ahead).
template <int IN_, int H0_, int H1_, int PASSES_>
struct NetF {
  static constexpr int IN = IN_, H0 = H0_, H1 = H1_, PASSES = PASSES_, OUT = 9;
  static constexpr int KS0 = (IN + 1) / 2;                 // layer-0 K = 2 steps
  static constexpr int KS0P = (KS0 + 15) / 16 * 16;        // padded so every segment is 16 ops long
  static constexpr int T0 = H0 / 32, T1 = H1 / 32, T1P = T1 / PASSES;
  static constexpr int RING = 16;
  // operand stream (64 f32 per op, lane-linear): per pass { per layer-0 tile t: W0 [KS0P],
  // W1 [16 g][T1P u] }, then W2 [T1P u][16 g]; RING zero ops of read-ahead padding; then f32
  // biases b0[H0], b1[H1], b2[32]
  static constexpr int64_t OPS = (int64_t)PASSES * (T0 * (KS0P + 16 * T1P) + 16 * T1P);
  static constexpr int64_t BIAS_OFF = (OPS + RING) * 256;
  static constexpr int64_t BYTES = BIAS_OFF + 4 * (H0 + H1 + 32);
  static_assert(H0 % 32 == 0 && H1 % 32 == 0 && T1 % PASSES == 0, "tile shapes");
};

__device__ __forceinline__ f32x16 mfma_f32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

template <class N>
__global__ __launch_bounds__(256) void k_mlp_f32(MlpArgs a) {
  __shared__ float bias[N::H0 + N::H1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int n = lane & 31, h = lane >> 5;
  const float* ops = static_cast<const float*>(a.packed);
  const float* gb = reinterpret_cast<const float*>(static_cast<const uint8_t*>(a.packed) + N::BIAS_OFF);
  for (int i = tid; i < N::H0 + N::H1; i += 256) bias[i] = gb[i];
  __syncthreads();
  const int64_t task = (int64_t)blockIdx.x * 4 + w;
  const int64_t row0 = task * 32;
  if (row0 >= a.rows) return;
  const int64_t row = row0 + n;
  const bool live = row < a.rows;
  // X^T operands: lane (n, h) holds obs[row n][2s + h]
  float xop[N::KS0P];
  {
    const float* x = a.obs + (live ? row : row0) * N::IN;
#pragma unroll
    for (int q = 0; q < N::KS0P; ++q) {
      const int k = 2 * q + h;
      xop[q] = (k < N::IN && live) ? x[k < N::IN ? k : 0] : 0.0f;
    }
  }
  const float* sp = ops + lane;           // op i of this lane: sp[i * 64]
  float ring[N::RING];
#pragma unroll
  for (int q = 0; q < N::RING; ++q) ring[q] = sp[q * 64];
  sp += N::RING * 64;                      // sp = the op RING ahead of the next consumed one
  f32x16 lg{};
  for (int p = 0; p < N::PASSES; ++p) {
    f32x16 acc1[N::T1P];
#pragma unroll
    for (int u = 0; u < N::T1P; ++u) acc1[u] = f32x16{};
    for (int t = 0; t < N::T0; ++t) {
      f32x16 acc0{};
#pragma unroll
      for (int q = 0; q < N::KS0P; ++q) {
        acc0 = mfma_f32(ring[q % N::RING], xop[q], acc0);
        ring[q % N::RING] = sp[q * 64];
      }
      sp += N::KS0P * 64;
      float hv[16];
#pragma unroll
      for (int g = 0; g < 16; ++g)
        hv[g] = fmaxf(acc0[g] + bias[32 * t + (g & 3) + 8 * (g >> 2) + 4 * h], 0.0f);
#pragma unroll
      for (int g = 0; g < 16; ++g)
#pragma unroll
        for (int u = 0; u < N::T1P; ++u) {
          const int j = g * N::T1P + u;
          acc1[u] = mfma_f32(ring[j % N::RING], hv[g], acc1[u]);
          ring[j % N::RING] = sp[j * 64];
        }
      sp += 16 * N::T1P * 64;
    }
#pragma unroll
    for (int u = 0; u < N::T1P; ++u) {
      const int tile = p * N::T1P + u;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const float v = fmaxf(acc1[u][g] + bias[N::H0 + 32 * tile + (g & 3) + 8 * (g >> 2) + 4 * h], 0.0f);
        const int j = u * 16 + g;
        lg = mfma_f32(ring[j % N::RING], v, lg);
        ring[j % N::RING] = sp[j * 64];
      }
    }
    sp += 16 * N::T1P * 64;
  }
  emit_logits(lg, gb + N::H0 + N::H1, row, live, h, a);
}

// ------------------------------------------------------------------------------------- host
uint16_t to_bf16(float f) {   // round to nearest even (NaN not expected in weights)
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

float from_bf16(uint16_t b) {
  const uint32_t u = (uint32_t)b << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

template <class N>
std::vector<uint8_t> pack(const float* w0, const float* b0, const float* w1, const float* b1,
                          const float* w2, const float* b2) {
  std::vector<uint8_t> blob(N::BYTES, 0);
  uint16_t* f = reinterpret_cast<uint16_t*>(blob.data());
  // operand `op` = one MFMA A operand = 64 lanes x 8 bf16; the kernel reads lane l's 16 bytes
  auto put = [&](int64_t op, int lane, int j, float v) { f[(op * 64 + lane) * 8 + j] = to_bf16(v); };
  // k order of an accumulator-as-operand fragment (layers 1, 2)
  auto kperm = [](int i, int s, int l, int j) { return 32 * i + 16 * s + 8 * (j >> 2) + 4 * (l >> 5) + (j & 3); };
  auto w1op = [&](int64_t op, int n, int t, int s) {   // W1 [H1][H0]: row tile n, k-step (t, s)
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 8; ++j) put(op, l, j, w1[(int64_t)(32 * n + (l & 31)) * N::H0 + kperm(t, s, l, j)]);
  };
  auto w2op = [&](int64_t op, int n, int s) {          // W2 [9][H1]: k-step (n, s), rows padded to 32
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 8; ++j) {
        const int o = l & 31;
        put(op, l, j, o < N::OUT ? w2[(int64_t)o * N::H1 + kperm(n, s, l, j)] : 0.0f);
      }
  };
  for (int c = 0; c < N::L0C; ++c)
    for (int m = 0; m < N::L0T; ++m) {
      const int t = c * N::L0T + m;                // layer-0 row tile
      const int64_t base = N::chunk_off(c) + (int64_t)m * N::U0;
      for (int q = 0; q < N::KQ0; ++q)             // W0 [H0][IN], natural k order (X^T from memory)
        for (int l = 0; l < 64; ++l)
          for (int j = 0; j < 8; ++j) {
            const int k = 16 * q + 8 * (l >> 5) + j, o = 32 * t + (l & 31);
            const float bh = from_bf16(to_bf16(b0[o]));        // b0 = hi + lo, both bf16
            const float v = k < N::IN ? w0[(int64_t)o * N::IN + k] : k == N::IN ? bh : k == N::IN + 1 ? b0[o] - bh : 0.0f;
            put(base + q, l, j, v);
          }
      if (N::MODE == 1)                             // this tile's k-steps of every layer-1 row tile
        for (int n = 0; n < N::T1; ++n)
          for (int s = 0; s < 2; ++s) w1op(base + N::KQ0 + 2 * n + s, n, t, s);
    }
  if (N::MODE == 0) {
    for (int d = 0; d < N::L1C; ++d)
      for (int nn = 0; nn < N::L1T; ++nn) {
        const int n = d * N::L1T + nn;             // layer-1 row tile
        const int64_t base = N::chunk_off(N::L0C + d) + (int64_t)nn * N::U1;
        for (int t = 0; t < N::T0; ++t)
          for (int s = 0; s < 2; ++s) w1op(base + 2 * t + s, n, t, s);
        for (int s = 0; s < 2; ++s) w2op(base + 2 * N::T0 + s, n, s);
      }
  } else {
    for (int n = 0; n < N::T1; ++n)
      for (int s = 0; s < 2; ++s) w2op(N::chunk_off(N::L0C) + 2 * n + s, n, s);
  }
  float* bias = reinterpret_cast<float*>(blob.data() + N::BIAS_OFF);
  memcpy(bias, b0, 4 * N::H0);
  memcpy(bias + N::H0, b1, 4 * N::H1);
  memcpy(bias + N::H0 + N::H1, b2, 4 * N::OUT);
  return blob;
}

// Net16 blob: operands of 16 rows x 32 k, lane l = row l&15, k 8(l>>4)+j; layer-0 k order natural
// (X^T from memory), layers 1-2 in kperm16 order (the accumulator-as-operand fragments).
template <class N>
std::vector<uint8_t> pack16(const float* w0, const float* b0, const float* w1, const float* b1,
                            const float* w2, const float* b2) {
  std::vector<uint8_t> blob(N::BYTES, 0);
  uint16_t* f = reinterpret_cast<uint16_t*>(blob.data());
  auto put = [&](int64_t op, int lane, int j, float v) { f[(op * 64 + lane) * 8 + j] = to_bf16(v); };
  auto kperm16 = [](int m, int l, int j) { const int g = l >> 4; return 32 * m + (j < 4 ? 4 * g + j : 16 + 4 * g + j - 4); };
  auto w0op = [&](int64_t op, int rt, int q) {          // W0 [H0][IN] row tile rt, k-step q (+ b0 hi/lo columns)
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 8; ++j) {
        const int k = 32 * q + 8 * (l >> 4) + j, o = 16 * rt + (l & 15);
        const float bh = from_bf16(to_bf16(b0[o]));
        const float v = k < N::IN ? w0[(int64_t)o * N::IN + k] : k == N::IN ? bh : k == N::IN + 1 ? b0[o] - bh : 0.0f;
        put(op, l, j, v);
      }
  };
  auto w1op = [&](int64_t op, int rt, int m) {          // W1 [H1][H0] row tile rt, k-step m (layer-0 group)
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 8; ++j) put(op, l, j, w1[(int64_t)(16 * rt + (l & 15)) * N::H0 + kperm16(m, l, j)]);
  };
  auto w2op = [&](int64_t op, int u) {                  // W2 [9][H1], rows padded to 16, k-step u
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 8; ++j) {
        const int o = l & 15;
        put(op, l, j, o < N::OUT ? w2[(int64_t)o * N::H1 + kperm16(u, l, j)] : 0.0f);
      }
  };
  for (int c = 0; c < N::L0C; ++c)
    for (int mm = 0; mm < N::L0T; ++mm) {
      const int t = c * N::L0T + mm;                     // layer-0 group
      const int64_t base = N::chunk_off(c) + (int64_t)mm * N::U0;
      for (int rt = 0; rt < 2; ++rt)
        for (int q = 0; q < N::KQ0; ++q) w0op(base + rt * N::KQ0 + q, 2 * t + rt, q);
      if (N::MODE == 1)
        for (int v = 0; v < 2 * N::G1; ++v) w1op(base + 2 * N::KQ0 + v, v, t);
    }
  if (N::MODE == 0) {
    for (int d = 0; d < N::L1C; ++d)
      for (int uu = 0; uu < N::L1T; ++uu) {
        const int u = d * N::L1T + uu;                   // layer-1 group
        const int64_t base = N::chunk_off(N::L0C + d) + (int64_t)uu * N::U1;
        for (int rt = 0; rt < 2; ++rt)
          for (int m = 0; m < N::G0; ++m) w1op(base + rt * N::G0 + m, 2 * u + rt, m);
        w2op(base + 2 * N::G0, u);
      }
  } else {
    for (int u = 0; u < N::G1; ++u) w2op(N::chunk_off(N::L0C) + u, u);
  }
  float* bias = reinterpret_cast<float*>(blob.data() + N::BIAS_OFF);
  memcpy(bias, b0, 4 * N::H0);
  memcpy(bias + N::H0, b1, 4 * N::H1);
  memcpy(bias + N::H0 + N::H1, b2, 4 * N::OUT);
  return blob;
}

template <class N>
std::vector<uint8_t> pack_f32(const float* w0, const float* b0, const float* w1, const float* b1,
                              const float* w2, const float* b2) {
  std::vector<uint8_t> blob(N::BYTES, 0);
  float* f = reinterpret_cast<float*>(blob.data());
  int64_t op = 0;
  auto rg = [](int g) { return (g & 3) + 8 * (g >> 2); };   // accumulator register g -> row (half 0)
  for (int p = 0; p < N::PASSES; ++p) {
    for (int t = 0; t < N::T0; ++t) {
      for (int q = 0; q < N::KS0P; ++q, ++op)        // W0 [H0][IN]: lane (i, h) = W0[32t + i][2q + h]
        for (int l = 0; l < 64; ++l) {
          const int i = l & 31, k = 2 * q + (l >> 5);
          f[op * 64 + l] = k < N::IN ? w0[(int64_t)(32 * t + i) * N::IN + k] : 0.0f;
        }
      for (int g = 0; g < 16; ++g)                   // W1 [H1][H0]: k pair (r_g, r_g + 4) of tile t
        for (int u = 0; u < N::T1P; ++u, ++op)
          for (int l = 0; l < 64; ++l) {
            const int i = l & 31, k = 32 * t + rg(g) + 4 * (l >> 5);
            f[op * 64 + l] = w1[(int64_t)(32 * (p * N::T1P + u) + i) * N::H0 + k];
          }
    }
    for (int u = 0; u < N::T1P; ++u)                 // W2 [9][H1], rows padded to 32 with zeros
      for (int g = 0; g < 16; ++g, ++op)
        for (int l = 0; l < 64; ++l) {
          const int i = l & 31, k = 32 * (p * N::T1P + u) + rg(g) + 4 * (l >> 5);
          f[op * 64 + l] = i < N::OUT ? w2[(int64_t)i * N::H1 + k] : 0.0f;
        }
  }
  float* bias = reinterpret_cast<float*>(blob.data() + N::BIAS_OFF);
  memcpy(bias, b0, 4 * N::H0);
  memcpy(bias + N::H0, b1, 4 * N::H1);
  memcpy(bias + N::H0 + N::H1, b2, 4 * N::OUT);
  return blob;
}

struct MlpKernel {
  int in, h0, h1, precision;
  int threads, rows_per_task;
  int64_t bytes;
  void (*fwd)(MlpArgs);
  std::vector<uint8_t> (*pack)(const float*, const float*, const float*, const float*, const float*, const float*);
};

template <int IN, int H0, int H1, int WAVES, int MODE, int L0T, int L1T, bool XPF>
MlpKernel make_mlp() {
  using N = Net<IN, H0, H1, WAVES, MODE, L0T, L1T, XPF>;
  return MlpKernel{IN, H0, H1, WH_MLP_BF16, N::MT, N::ROWS, N::BYTES, k_mlp<N>, pack<N>};
}

template <int IN, int H0, int H1, int WAVES, int MODE, int L0T, int L1T, int NS = 2>
MlpKernel make_mlp16() {
  using N = Net16<IN, H0, H1, WAVES, MODE, L0T, L1T, NS>;
  return MlpKernel{IN, H0, H1, WH_MLP_BF16, N::MT, N::ROWS, N::BYTES, k_mlp16<N>, pack16<N>};
}

template <int IN, int H0, int H1, int PASSES>
MlpKernel make_mlp_f32() {
  using N = NetF<IN, H0, H1, PASSES>;
  return MlpKernel{IN, H0, H1, WH_MLP_F32, 256, 128, N::BYTES, k_mlp_f32<N>, pack_f32<N>};
}

const MlpKernel* find_mlp(const wh_mlp_desc* d) {
  // the policy_model shapes of scripts/experiments/warehouse-{small,medium,large}-sac/*.yaml:
  // bf16 on 16x16x32 tiles (k_mlp16) for Medium and Large, +4-7 % over the 32x32x16 kernel on the
  // same box; Small keeps the 32x32x16 kernel, whose next-task X prefetch fits its registers there
  // (16x16x32 without it: -3 to -8 %, profiles/r04_mlp16_ab.txt).  WH_MLP_LEGACY=1 selects the
  // 32x32x16 kernel everywhere (A/B runs; a blob is packed for the kernel of its process).
  static const bool legacy = getenv("WH_MLP_LEGACY") != nullptr;
  // (One wave per SIMD -- 4 waves, 128 samples per task, 512 registers -- ran 25-28 % slower: the
  // weight stream per sample doubles, profiles/r05_mlpw4_ab.txt; four sample tiles per wave to keep
  // 256 samples per task do not fit 512 registers at Medium.)
  static const MlpKernel reg16[] = {
      make_mlp16<82, 512, 512, 8, 0, 8, 2>(),      // Medium
      make_mlp16<145, 1024, 256, 8, 1, 2, 1>(),    // Large
  };
  if (d && d->out_dim == 9 && d->precision == WH_MLP_BF16 && !legacy)
    for (const auto& k : reg16)
      if (k.in == d->in_dim && k.h0 == d->hidden0 && k.h1 == d->hidden1) return &k;
  static const MlpKernel reg[] = {
      // (waves per workgroup, dataflow MODE, layer-0 tiles per chunk, layer-1 tiles per chunk,
      // next-task X prefetch): 8 waves = two per SIMD (256 registers each)
      make_mlp<37, 256, 256, 8, 0, 8, 4, true>(),     // Small:  obs 9*4+1,  [256, 256]
      make_mlp<82, 512, 512, 8, 0, 8, 2, false>(),    // Medium: obs 9*9+1,  [512, 512]
      make_mlp<145, 1024, 256, 8, 1, 2, 1, false>(),  // Large:  obs 9*16+1, [1024, 256]
      make_mlp_f32<37, 256, 256, 1>(),    // the same shapes in exact f32
      make_mlp_f32<82, 512, 512, 2>(),
      make_mlp_f32<145, 1024, 256, 1>(),
  };
  if (!d || d->out_dim != 9) return nullptr;
  for (const auto& k : reg)
    if (k.in == d->in_dim && k.h0 == d->hidden0 && k.h1 == d->hidden1 && k.precision == d->precision) return &k;
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

static int mlp_forward(const wh_mlp_desc* d, const void* packed, int64_t rows, const float* obs,
                       const void* xfrag, float* logits, int32_t* actions, int32_t explore, uint64_t seed,
                       uint32_t step, void* stream) {
  const MlpKernel* k = find_mlp(d);
  if (!k) return d ? WH_ENOTSUP : WH_EINVAL;
  if (rows < 0) return WH_EINVAL;
  if (rows == 0) return WH_OK;
  if (!packed || (!obs && !xfrag) || (!logits && !actions)) return WH_EINVAL;
  if (xfrag && (k->precision != WH_MLP_BF16 || (uintptr_t)xfrag % 16 != 0)) return WH_ENOTSUP;
  const char* abl = getenv("WH_MLP_ABLATE");
  MlpArgs a{packed, rows, obs, logits, actions, explore ? 1 : 0, (uint32_t)(seed & 0xFFFFFFFFu),
            (uint32_t)(seed >> 32), step, abl ? atoi(abl) : 0, static_cast<const u32x4*>(xfrag)};
  static int cus = 0;                         // one persistent workgroup per CU
  if (!cus) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return WH_EHIP;
    cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  }
  if (k->precision == WH_MLP_F32) {         // 32 rows per wave, 4 waves per workgroup
    const int64_t ntask = (rows + 31) / 32;
    hipLaunchKernelGGL(k->fwd, dim3((unsigned)((ntask + 3) / 4)), dim3(256), 0, (hipStream_t)stream, a);
    return hip_rc(hipGetLastError());
  }
  const int64_t ntask = (rows + k->rows_per_task - 1) / k->rows_per_task;
  const unsigned grid = (unsigned)(ntask < cus ? ntask : cus);
  hipLaunchKernelGGL(k->fwd, dim3(grid), dim3(k->threads), 0, (hipStream_t)stream, a);
  return hip_rc(hipGetLastError());
}

int wh_mlp_forward(const wh_mlp_desc* d, const void* packed, int64_t rows, const float* obs,
                   float* logits, int32_t* actions, int32_t explore, uint64_t seed, uint32_t step,
                   void* stream) {
  return mlp_forward(d, packed, rows, obs, nullptr, logits, actions, explore, seed, step, stream);
}

int wh_mlp_forward_x(const wh_mlp_desc* d, const void* packed, int64_t rows, const void* xfrag,
                     float* logits, int32_t* actions, int32_t explore, uint64_t seed, uint32_t step,
                     void* stream) {
  if (!xfrag) return WH_EINVAL;
  return mlp_forward(d, packed, rows, nullptr, xfrag, logits, actions, explore, seed, step, stream);
}

}  // extern "C"
