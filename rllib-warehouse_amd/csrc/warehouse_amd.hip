// warehouse_amd.hip -- gfx950 kernels + C ABI for the batched warehouse hot path.
//
// Design (DESIGN.md has the rationale and the measurements behind each choice):
//  * ONE LANE PER ENV.  The per-env work of core.py:262-442 is a short, mostly serial integer
//    program (sequential collision resolution, core.py:279-300).  One env per lane with the batch
//    across lanes makes every HBM access a coalesced word plane (state[w * B + e]) and shares each
//    issued instruction among 64 envs.  With B = 65,536 that is one wave per SIMD, so the kernel
//    is VALU-issue bound and every instruction per env-step counts.
//  * 16-bit coordinate pairs.  An agent word is x | dx<<8 | y<<16 | dy<<24 (dx,dy = delivery
//    target cell, 0xFF = idle): a move is 3 packed-i16 ops (the reference's "keep the old
//    coordinate off the grid" rule equals a clamp for +-1 moves, core.py:282-287), a delivery test
//    is one compare (core.py:354-362) and Manhattan distance is one v_sad_hi_u8, which also
//    carries the pickup index and cell as a 16-bit tag so a v_min gives argmin-first-wins
//    (solvers.py:53-58).
//  * SWAR on packed bytes.  Pickup tables are 1 byte per point, 4 per register: expiry
//    (core.py:303-306) and clearing/opening (core.py:330-351) run 4 points per VALU op; the set of
//    open requests is a 64-bit mask kept in registers across fused steps.
//  * Per-lane LDS scratch for the data-dependent lookups (occupancy rows core.py:275-291, pickup
//    target bytes core.py:327-329), laid out [word][lane] so every lane hits its own bank, and no
//    data-dependent branches: LDS side effects are predicated through neutral operands.
//  * Counter-based Philox streams (no RNG state in HBM) or injected draws (parity mode).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <mutex>
#include <type_traits>
#include <unordered_set>
#include <new>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "philox.h"
#include "warehouse_amd.h"

namespace {

constexpr int BT = 256;  // lanes (= envs) per workgroup
// Pickup-plane cell width: 16-bit cells put lanes 2k and 2k+1 in one LDS bank (b32-and-narrower
// accesses bank by dword mod 32 over 32-lane groups), a 2-way conflict on every access whose rows
// differ between the two lanes -- the move loop's target-byte lookups, the pickup clears and the
// regeneration stores.  32-bit cells (the upper half unused) give every lane of a group its own
// bank for twice the LDS, and measured slower anyway (Medium-8 +0.3 %, Large-16 +0.4 % per
// 200-step launch, profiles/r05_occ_ab.txt; round 4 the same), so the cells stay 16-bit;
// -DWH_PKP32 selects 32-bit cells (A/B).
#if defined(WH_PKP32)
constexpr bool kPkWide = true;
#else
constexpr bool kPkWide = false;
#endif
using PkCell = std::conditional_t<kPkWide, uint32_t, uint16_t>;
constexpr uint32_t PKW = sizeof(PkCell);
constexpr uint32_t ROWB = PKW * BT;   // bytes per pickup-point row of the LDS pickup plane

enum Policy { POL_EXTERNAL = 0, POL_GREEDY = 1, POL_RANDOM = 2 };
enum Purpose : uint32_t { PUR_RESET = 1, PUR_REGEN = 2, PUR_POLICY = 3, PUR_RANDOM = 4 };
constexpr int PH_ALL = 0, PH_PRE = 1, PH_REGEN = 2, PH_POLICY = 3;
#ifdef WH_ABLATION
constexpr bool kAblationBuild = true;    // ablation moves are arbitrary: keep the off-grid clamp
#else
constexpr bool kAblationBuild = false;
#endif

// A/B switches of the fused fast path (tools/anat_ab.sh): -DWH_NO_BIAS keeps plain occupancy-row
// addressing, -DWH_NO_REGEN_HOIST computes the regeneration's Philox block inside the regeneration.
#ifndef WH_NO_BIAS
constexpr bool kBiasAddr = true;
#else
constexpr bool kBiasAddr = false;
#endif
// -DWH_OBS_EB0=<n>: envs per workgroup of the observation kernel for the widest f32 rows (Large)
#ifndef WH_OBS_EB0
#define WH_OBS_EB0 4
#endif
constexpr int kObsEB[4] = {WH_OBS_EB0, 8, 16, 64};   // the observation kernel's instances
// The widest f32 rows (kObsEB[0]'s: Large) are written in chunks of WH_OBS_CHUNK float4s per workgroup
// (k_observe's CHUNK form; 0 = each workgroup writes its own envs' rows).  Large-16 sampler step
// 127 -> 109-112 us, wh_observe 110 -> 100-104 us (profiles/r06_obschunk_ab.txt, r06_obschunk2_ab.txt:
// 512 / 768 / 1280 / 1536 float4s, plain stores and 2 vs 4 float4s in flight compared).
#ifndef WH_OBS_CHUNK
#define WH_OBS_CHUNK 1024
#endif
constexpr int kObsChunk = WH_OBS_CHUNK;
#ifndef WH_FUSE_ROWS_MAX   // rows per env (bytes) up to which the sampler routes fuse step + rows (fuse_rows)
#define WH_FUSE_ROWS_MAX 4096
#endif
// Observation stores (same-box A/Bs, tools/obs_bench.py, sampler_probe.py and policy_probe.py;
// profiles/r05_l16rows_ab.txt, r05_ntm8_ab.txt, r05_ntsel_ab.txt): f32 rows nontemporal for rows of
// <= 1 KB or > 4 KB per env (Small / Large: observe -5 % / -2 %, Large-16's sampler route -3 %,
// Small-4's 1-step sampler -3 %), except in multi-step sampler fragments (Small-4 +11 %); plain for
// Medium's rows (nontemporal: observe +10 %, sampler step +24 %).  The fragment operand plain: stored
// nontemporal it is written 5-11 % faster but the policy network then reads it from HBM instead of
// the last-level cache, and the policy route is 1 % slower at Medium-8 (no gain at Large-16).
// -DWH_OBS_NT / -DWH_OBS_NO_NT: every single-step row store nontemporal / none (A/B switches).
template <class C>
constexpr bool rows_nt() {
#if defined(WH_OBS_NT)
  return true;
#elif defined(WH_OBS_NO_NT)
  return false;
#else
  return C::NAM * C::L * 4 <= 1024 || C::NAM * C::L * 4 > 4096;
#endif
}
constexpr bool kFragNT = false;

#ifndef WH_REV_SPLIT_MAX_NAM   // agent counts up to which the move loop has the no-reverse-key variant
#define WH_REV_SPLIT_MAX_NAM 9
#endif
#ifndef WH_UKEY_MIN_NAM        // agent counts from which the ascending move loop uses one key per move
#define WH_UKEY_MIN_NAM 0      // (A/B builds: 99 = the two-key form with its reverse-key split)
#endif
constexpr int kUKeyMinNam = WH_UKEY_MIN_NAM;
#ifndef WH_BIAS_MAX_NAM
#define WH_BIAS_MAX_NAM 64
#endif
constexpr int kRevSplitMaxNam = WH_REV_SPLIT_MAX_NAM, kBiasMaxNam = WH_BIAS_MAX_NAM;
#ifndef WH_NO_REGEN_HOIST
constexpr bool kRegenHoist = true;
#else
constexpr bool kRegenHoist = false;
#endif
// Regeneration targets of items 1 and 2 by skipping the earlier items' targets (a compare-add each)
// instead of a rank selection on a used-target mask; the mask is built only from item 3 on.  Same
// values.  -DWH_NO_REGEN_SKIP: the mask for every item (A/B).
// The regeneration's first Philox block is computed in the fused step's policy block (its ten rounds
// fill that block's issue gaps) rather than inside the move loop's: -0.5 % per step at Medium-8 and
// Large-16 (profiles/r05_step3_ab.txt).  -DWH_NO_HOIST_POLICY: inside the move loop (A/B).
// The ascending move loop reads agent s's occupancy word kOccAhead turns early and corrects it in
// registers for the agents that moved in between (4 VALU per corrected agent), so the LDS latency
// -- which queues behind the turn's own lookups, lgkmcnt being in order -- is covered by that many
// turns of work.  Two turns measured slower than one (Medium-8 +2.4 %, Large-16 +3.1 % per 200-step
// launch, profiles/r05_occ_ab.txt: the second correction's VALU cost more than the wait it hid), so
// the default is one; -DWH_OCC_AHEAD=2 (A/B).
#ifndef WH_OCC_AHEAD
#define WH_OCC_AHEAD 1
#endif
constexpr int kOccAhead = WH_OCC_AHEAD;
// Turns between the move loop's dependent pickup lookups (cell -> point row, point -> target byte,
// target -> delivery cell, then the decision): each lookup is issued kPickDist turns after the one
// it depends on, so its LDS latency is covered by that many turns of the serial chain.  Two turns:
// Medium-8 -1.0 %, Large-16 -1.0 % per 200-step launch against one (profiles/r05_pick_ab.txt); three
// turns +1.3 % / +0.9 % against two (profiles/r05_tune_ab.txt).  -DWH_PICK_DIST=1 / 3 (A/B).
#ifndef WH_PICK_DIST
#define WH_PICK_DIST 2
#endif
constexpr int kPickDist = WH_PICK_DIST;
static_assert(kOccAhead == 1 || kOccAhead == 2, "occupancy read distance");
#ifndef WH_NO_HOIST_POLICY
constexpr bool kHoistPolicy = true;
#else
constexpr bool kHoistPolicy = false;
#endif
#ifndef WH_NO_REGEN_SKIP
constexpr bool kRegenSkip = true;
#else
constexpr bool kRegenSkip = false;
#endif

constexpr uint32_t IDLE = 0xFF00FF00u;    // delivery-target bytes of an idle agent
constexpr uint32_t XY16 = 0x00FF00FFu;    // position bytes of an agent word

// Cell -> pickup table (u8 per cell).  Byte x | y << 8 (one v_perm of the packed position): its dword
// -- the LDS bank -- is x >> 2, so every lane of a wave reads one of D/4 banks (~8- to 13-way
// conflicts).  Skewed: byte 4x + 132y (one v_dot4_u32_u8 of the agent word), bank (x + y) mod 32.
// Same-box A/B (profiles/r05_step3_ab.txt): Large-16 -1.6 % per step (-2.9 % with the policy-block
// Philox hoist), Medium-8 +3 % -- so the skewed table is used from D = 20 (Large) on.
// -DWH_CELL_SKEW / -DWH_NO_CELL_SKEW force it on / off for every geometry (A/B).
#if defined(WH_CELL_SKEW)
__host__ __device__ constexpr bool cell_skew(int) { return true; }
#elif defined(WH_NO_CELL_SKEW)
__host__ __device__ constexpr bool cell_skew(int) { return false; }
#else
__host__ __device__ constexpr bool cell_skew(int D) { return D >= 20; }
#endif
__host__ __device__ constexpr int cell_bytes(int D) { return cell_skew(D) ? 132 * D : 256 * D; }
__host__ __device__ constexpr int cell_index(int x, int y, int D) { return cell_skew(D) ? 4 * x + 132 * y : (x | (y << 8)); }

// Shared (per-workgroup) table layout in bytes; built identically by build_tables() on the host.
struct TableLayout {
  int cell, rp, tag, dst, mv, valid, bytes;
  __host__ __device__ constexpr TableLayout(int D, int P, int DP, int NV)
      : cell(0), rp(cell_bytes(D)), tag(cell_bytes(D) + 4), dst(cell_bytes(D) + 8 * (P + 1)),   // rp/tag interleaved
        mv(cell_bytes(D) + 8 * (P + 1) + 4 * DP), valid(cell_bytes(D) + 8 * (P + 1) + 4 * DP + 48),
        bytes(cell_bytes(D) + 8 * (P + 1) + 4 * DP + 48 + 4 * NV) {}
};

template <int D_, int R_, int NR_, int NAM_>
struct Cfg {
  static constexpr int D = D_, R = R_, NR = NR_, NAM = NAM_;
  static constexpr int P = 4 * NR * NR;
  static constexpr int DP = 4 * (D - 4);
  static constexpr int PW = P / 4;
  static constexpr int NV = (D - 2) * (D - 2) - P;      // interior cells that are not pickups
  static constexpr TableLayout T = TableLayout(D, P, DP, NV);
  static constexpr int TBLW = T.bytes / 4;
  static constexpr int TBL4 = (TBLW + 3) / 4;           // 16-byte chunks (device copy padded to them)
  static constexpr int L = 9 * R + 1;                    // observation row length
  static_assert(D <= 32, "positions are 5-bit fields (occupancy rows are 32-bit words)");
  static_assert(P <= 64 && DP <= 64, "bitmask sets hold at most 64 points");
  static_assert(NAM <= R, "agents <= requests (core.py:89)");
};

typedef short short2v __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ short2v as_s2(uint32_t v) { return __builtin_bit_cast(short2v, v); }
__device__ __forceinline__ uint32_t as_u(short2v v) { return __builtin_bit_cast(uint32_t, v); }

// ----------------------------------------------------------------------------- small helpers
__device__ __forceinline__ uint32_t comp(const uint4& v, int i) {
  return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}

struct Keys {
  uint32_t k0, k1;
};

// Block b of stream (env, episode, t, purpose).
__device__ __forceinline__ uint4 stream_block(const Keys& k, uint32_t env, uint32_t ep, uint32_t t,
                                              uint32_t purpose, uint32_t b) {
  return philox10(make_uint4(env, ep, t, (purpose << 24) | b), k.k0, k.k1);
}

// Sequential reader for streams whose word indices are only known at run time (reset).
struct Reader {
  Keys k;
  uint32_t env, ep, t, purpose;
  int cur;
  uint4 blk;
  __device__ Reader(Keys k_, uint32_t env_, uint32_t ep_, uint32_t t_, uint32_t p_)
      : k(k_), env(env_), ep(ep_), t(t_), purpose(p_), cur(-1), blk(make_uint4(0, 0, 0, 0)) {}
  __device__ __forceinline__ uint32_t word(int j) {
    const int b = j >> 2;
    if (b != cur) {
      blk = stream_block(k, env, ep, t, purpose, (uint32_t)b);
      cur = b;
    }
    return comp(blk, j & 3);
  }
};

// Branch-free selects without VCC: a one-wave-per-SIMD kernel pays for every v_cmp -> SGPR mask ->
// v_cndmask round trip (measured: tools/oprate3.hip), while v_bitop3 is a plain full-rate VALU op.
// Masks are 0 / 0xFFFFFFFF in VGPRs; every consumer goes through the bitop3 builtin so LLVM cannot
// fold the mask arithmetic back into compare + select.
constexpr uint32_t TA = 0xF0, TB = 0xCC, TC = 0xAA;   // truth-table columns of operands 0, 1, 2
template <uint32_t TT>
__device__ __forceinline__ uint32_t bop3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, (unsigned char)(TT & 0xFFu));
}
// Sign bit -> 0 / all-ones.  As inline asm: LLVM turns ashr(a - b, 31) into a carry-out compare
// plus v_cndmask (the round trip this file avoids).
__device__ __forceinline__ uint32_t sgn(uint32_t x) {
  uint32_t r;
  asm("v_ashrrev_i32 %0, 31, %1" : "=v"(r) : "v"(x));
  return r;
}
// The same sign mask as v_bfe_i32 x, 31, 1 through the builtin: no inline asm, so the hazard
// recognizer does not pad the next VALU with an s_nop (select_bit64 chains five of them per call);
// where LLVM would rewrite it into a compare (a difference of two values) the asm form stays.
__device__ __forceinline__ uint32_t sgn_bfe(uint32_t x) { return (uint32_t)__builtin_amdgcn_sbfe((int)x, 31u, 1u); }
__device__ __forceinline__ uint32_t mask_z(uint32_t x) { return sgn(x - 1u); }   // x == 0 (x < 2^31)
__device__ __forceinline__ uint32_t msel(uint32_t m, uint32_t a, uint32_t b) { return bop3<(TA & TB) | (~TA & TC)>(m, a, b); }

// Index of the r-th (0-based) set bit of m (r < popcount(m)).  Binary search over popcounts with
// the rank kept as sr = -1 - r: popcount(x) + sr is negative exactly when r >= popcount(x), and is
// then the rank left for the upper part.  Selects are v_bitop3 on sign masks (no VCC).
__device__ __forceinline__ uint32_t select_bit64(uint64_t m, uint32_t r) {
  uint32_t sr = ~r;
  uint32_t u = (uint32_t)__popc((uint32_t)m) + sr;
  uint32_t g = sgn_bfe(u);
  uint32_t w = msel(g, (uint32_t)(m >> 32), (uint32_t)m);
  sr = msel(g, u, sr);
  const uint32_t half = bop3<TA & TB>(g, 32u, 0u);
  // binary search inside w: the field of width k at offset base (v_bfe) instead of shifting w
  uint32_t base = 0;
#pragma unroll
  for (int k = 16; k >= 1; k >>= 1) {
    u = (uint32_t)__popc(__builtin_amdgcn_ubfe(w, base, (uint32_t)k)) + sr;
    g = sgn_bfe(u);
    if (k > 1) sr = msel(g, u, sr);
    base = bop3<(TA & TB) | TC>(g, (uint32_t)k, base);
  }
  return base | half;
}

// high bit of every nonzero byte
__device__ __forceinline__ uint32_t nz_hi(uint32_t x) {
  return (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
}
// 4 byte-flags (bit 7 of each byte) -> 4-bit nibble
__device__ __forceinline__ uint32_t nib_of(uint32_t hi) { return ((hi >> 7) * 0x00204081u) >> 21 & 0xFu; }
// 4-bit nibble -> 0xFF byte mask (full-rate 24-bit multiply)
__device__ __forceinline__ uint32_t expand_nib(uint32_t nib) {
  const uint32_t ones = __umul24(nib, 0x00204081u) & 0x01010101u;
  return (ones << 8) - ones;
}

// packed i16 max/min, pinned: hipcc rewrites clamp(x, -1, 1) on i16 pairs into per-half
// compare/select cascades (it recognises sign(x)); one v_pk_* op per bound is what we want.
__device__ __forceinline__ uint32_t pk_max_i16(uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_pk_max_i16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ uint32_t pk_min_i16(uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_pk_min_i16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ uint32_t pk_min_u16(uint32_t a, uint32_t b) {
  typedef unsigned short ushort2v __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(ushort2v, a),
                                                                __builtin_bit_cast(ushort2v, b)));
}
__device__ __forceinline__ uint32_t pk_sub_i16(uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_pk_sub_i16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// dx * dy of a packed (dx, dy) i16 pair in ONE op, in both halves: v_pk_mul_lo_u16 of the pair with
// itself, the second operand's halves swapped by op_sel (a builtin dot2 costs a v_alignbit and a
// zeroed accumulator on top).
__device__ __forceinline__ uint32_t mul_swap(uint32_t d) {
  uint32_t r;
  asm("v_pk_mul_lo_u16 %0, %1, %1 op_sel:[0,1] op_sel_hi:[1,0]" : "=v"(r) : "v"(d));
  return r;
}

// clamp(p + d) per 16-bit lane: the reference keeps the old coordinate when a +-1 move leaves
// [0, D) (core.py:284-287), which for unit moves is exactly a clamp to [0, D-1].
template <int D>
__device__ __forceinline__ uint32_t step16(uint32_t p, uint32_t d) {
  short2v v = as_s2(p) + as_s2(d);
  v = __builtin_elementwise_max(v, (short2v){0, 0});
  v = __builtin_elementwise_min(v, (short2v){(short)(D - 1), (short)(D - 1)});
  return as_u(v);
}

// action index of a unit step packed as (dx, dy) i16 pair: MOVES[a] = (a//3-1, a%3-1), core.py:38
__device__ __forceinline__ uint32_t action_of(uint32_t d) {
  const short2v v = as_s2(d);
  return (uint32_t)(3 * ((int)v.x + 1) + ((int)v.y + 1));
}

// Rare wave-uniform branches of the step loop (expiry pass, grid rebuild, resets, random moves): marked
// cold so that block placement keeps their code out of the hot path's instruction stream.
// -DWH_NO_COLD: no annotation (A/B).
#ifndef WH_NO_COLD
#define WH_RARE(x) __builtin_expect(!!(x), 0)
#else
#define WH_RARE(x) (x)
#endif

// Phase labels in the device assembly for instruction-count analysis (`make asm` defines
// WH_PHASE_MARKS).  Not in the library: each label is an asm volatile with a memory clobber, a
// scheduling barrier for memory operations -- without them Large-16 runs 0.9 % and Medium-8 0.3 %
// faster per 200-step launch (profiles/r06_nomarks_ab.txt).
#ifdef WH_PHASE_MARKS
#define WH_PHASE_MARK(name) asm volatile("; PHASE " #name ::: "memory")
#else
#define WH_PHASE_MARK(name) ((void)0)
#endif

template <class C>
struct Regs {
  uint32_t hdr, epi;
  uint32_t ag[C::NAM];
  uint64_t am;   // open requests (bit j = pickup point j has one; kept in registers across steps)
  // Wave-uniform first step of the expiry phase: W, since a request opened at t0 >= 0 lives W
  // steps, or 0 if some lane was loaded holding one that expires sooner (no episode reaches that).
  uint32_t wskip;
};

template <class C>
struct Lds {
  alignas(16) uint32_t tbl[4 * C::TBL4];
  uint32_t occ[C::D][BT];        // occupancy row y: bit x
  // Pickup point j of lane tid: low byte = request target + 1 (0 = none), high byte = expiry step
  // (low 8 bits).  Row P is scratch: predicated stores of lanes with nothing to write go there.
  // One cell per (point, lane) (PkCell: 32-bit, the upper half unused, so that no two lanes of a
  // 32-lane group share a bank) makes every per-point access a single ds op whose address is
  // j * BT + tid, and keeps the pickup table out of the VGPRs.
  PkCell pkp[C::P + 1][BT];
  // Agent words when processing in action-dict order; afterwards the reward-row staging area.
  // Wave w only ever touches its own 64 columns [64w, 64w + 64) of every row.
  alignas(16) uint32_t agl[C::NAM][BT];
  // Cell (x | y << 16) -> pickup index + 1, 0 for other cells: one v_perm (the byte index
  // x | y << 8) + one ds_read_u8; the point's row in pkp is then one v_lshl_add away (row_byte).
  __device__ __forceinline__ uint32_t cell_row(uint32_t xy16) const {
    if constexpr (cell_skew(C::D)) {
      // one v_dot4_u32_u8 of the agent word's bytes [x, dx, y, dy] with [4, 0, 132, 0]
      const uint32_t i = __builtin_amdgcn_udot4(xy16, 0x00840004u, 0u, false);
      return reinterpret_cast<const uint8_t*>(tbl)[i];
    } else {
      return reinterpret_cast<const uint8_t*>(tbl)[__builtin_amdgcn_perm(xy16, xy16, 0x0C0C0200u)];
    }
  }

  // (pickup cell, greedy tag) of point j: one 8-byte LDS read
  __device__ __forceinline__ uint2 rtag(uint32_t j) const {
    return reinterpret_cast<const uint2*>(&tbl[C::T.rp / 4])[j];
  }
  __device__ __forceinline__ uint32_t mv(uint32_t a) const { return tbl[C::T.mv / 4 + a]; }
  __device__ __forceinline__ uint32_t valid_cell(uint32_t v) const { return tbl[C::T.valid / 4 + v]; }
  __device__ __forceinline__ uint32_t target_byte(uint32_t j, int tid) const {
    return *reinterpret_cast<const uint8_t*>(&pkp[j][tid]);
  }
  __device__ __forceinline__ void clear_target(uint32_t j, int tid) {
    *reinterpret_cast<uint8_t*>(&pkp[j][tid]) = 0;
  }
  // Target byte of the point whose cell_row() value is cv (0: the row before pkp -- garbage,
  // never used).
  __device__ __forceinline__ uint32_t pkp_offset() const {
    return (uint32_t)(reinterpret_cast<const char*>(&pkp[0][0]) - reinterpret_cast<const char*>(this));
  }
  __device__ __forceinline__ const uint8_t* row_byte(uint32_t cv, int tid) const {
    return reinterpret_cast<const uint8_t*>(this) + (pkp_offset() - ROWB) + cv * ROWB + PKW * tid;
  }
  __device__ __forceinline__ uint8_t* row_byte(uint32_t cv, int tid) {
    return reinterpret_cast<uint8_t*>(this) + (pkp_offset() - ROWB) + cv * ROWB + PKW * tid;
  }
  // Delivery cell of a target byte (target + 1; 0 reads the word before the table: never used) in
  // agent-word form: x << 8 | y << 24 in the target bytes, ones in the position bytes, so a pickup
  // is one AND of the (idle: 0xFF target bytes) agent word.
  __device__ __forceinline__ uint32_t dst_tb(uint32_t tb) const { return tbl[C::T.dst / 4 - 1 + tb]; }
};

// Reset slots (fused rollout only: their own __shared__ object in that k_step instance, so the
// other step instances and k_reset do not carry them): lane tid's NEXT episode's reset state,
// precomputed for the whole wave at once (reset_philox<..., TO_SLOT>) and consumed when the lane ends
// its episode (reset_from_slot): agent words, R requests (point | (target + 1) << 8), open mask,
// header, and the episode the slot was computed for (valid iff rs_ep == epi + 1).
template <class C>
struct Slots {
  uint32_t rs_ag[C::NAM][BT];
  uint16_t rs_req[C::R][BT];
  uint32_t rs_am[2][BT], rs_hdr[BT], rs_ep[BT];
};
struct NoSlots {};

// Every 16-byte load of a lane is issued before its first LDS write, so the prologue pays one
// memory round trip.  (A strided `for` loop over words compiled to load -> vmcnt(0) -> ds_write per
// iteration: ~10 serial round trips per launch at Medium-8, most of a short launch's fixed cost.)
// Split in two: issue_tables() puts the loads in flight first (the table is L2-resident: it comes back
// well before the state planes from HBM), commit_tables() writes them to LDS -- the waitcnt pass then
// waits for the table loads only (vmcnt counts in order), with the state loads still in flight.
// Chunk i (16 bytes per lane) of the table, as plain values: a struct or array of them crossing
// the state loads was kept in memory by LLVM (promoted to LDS, 32 bytes per lane, or put in scratch).
template <class C>
constexpr int kTableChunks = (C::TBL4 + BT - 1) / BT;
template <class C>
__device__ __forceinline__ bool table_lane(int i) {
  return i < kTableChunks<C> && (C::TBL4 % BT == 0 || i + 1 < kTableChunks<C> || (int)threadIdx.x + i * BT < C::TBL4);
}
template <class C>
__device__ __forceinline__ uint4 issue_table_chunk(const uint32_t* __restrict__ tables, int i) {
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  if (table_lane<C>(i)) v = reinterpret_cast<const uint4*>(tables)[threadIdx.x + i * BT];
  return v;
}
template <class C>
__device__ __forceinline__ void commit_table_chunk(uint32_t* dst, int i, uint4 v) {
  if (table_lane<C>(i)) reinterpret_cast<uint4*>(dst)[threadIdx.x + i * BT] = v;
}
template <class C>
__device__ __forceinline__ void load_tables(uint32_t* dst, const uint32_t* __restrict__ tables) {
  static_assert(kTableChunks<C> <= 2, "tables of at most 2 x 4 KB");
  const uint4 v0 = issue_table_chunk<C>(tables, 0), v1 = issue_table_chunk<C>(tables, 1);
  commit_table_chunk<C>(dst, 0, v0);
  commit_table_chunk<C>(dst, 1, v1);
}

template <class C>
__device__ __forceinline__ uint64_t active_mask(const uint32_t (&pt)[C::PW]) {
  uint64_t am = 0;
#pragma unroll
  for (int w = 0; w < C::PW; ++w) am |= (uint64_t)nib_of(nz_hi(pt[w])) << (4 * w);
  return am;
}

template <int N>
__device__ __forceinline__ uint64_t low_mask() {
  return N >= 64 ? ~0ull : ((1ull << N) - 1ull);
}

// The packed words of one env, loaded to registers.  Word plane w of the workgroup's envs is
// st + w * B + e0 (e0 = the workgroup's first env): a wave-uniform pointer, advanced by B with two
// scalar adds per plane, and the lane's offset tid * 4 -- global loads in SGPR-base form, so no
// per-lane 64-bit address arithmetic (it was ~100 VALU, a third of them v_mad_u64_u32, in front of
// the first load).  Issue order = use order: the header and the pickup planes (target, expiry
// pairs: the pickup plane is built from them while the rest arrive), then the episode counter and
// the agent words (first used in the step loop).
template <class C>
struct RawEnv {
  uint32_t hdr, epi, ag[C::NAM], pt[C::PW], pm[C::PW];
};

template <class C>
__device__ __forceinline__ void load_env_issue(RawEnv<C>& r, const uint32_t* __restrict__ st, int64_t B,
                                               int64_t e0, int tid, int na) {
  const uint32_t* pl = st + e0;
  r.hdr = pl[tid];
  const uint32_t* pt = pl + (int64_t)(2 + na) * B;
  const uint32_t* pm = pt + (int64_t)C::PW * B;
#pragma unroll
  for (int w = 0; w < C::PW; ++w) {
    r.pt[w] = pt[tid];
    r.pm[w] = pm[tid];
    pt += B;
    pm += B;
  }
  pl += B;
  r.epi = pl[tid];
#pragma unroll
  for (int i = 0; i < C::NAM; ++i) {
    pl += B;
    r.ag[i] = (i < na) ? pl[tid] : IDLE;
  }
}

// SWAR byte ops on 4 packed unsigned bytes (H = the bytes' high bits)
constexpr uint32_t SWAR_H = 0x80808080u;
__device__ __forceinline__ uint32_t swar_sub(uint32_t x, uint32_t y) {   // (x_b - y_b) mod 256 per byte
  return ((x | SWAR_H) - (y & ~SWAR_H)) ^ ((x ^ ~y) & SWAR_H);
}
__device__ __forceinline__ uint32_t swar_lt(uint32_t x, uint32_t y) {    // bit 7 of byte b: x_b < y_b
  return (((~x & y) | (~(x ^ y) & swar_sub(x, y))) & SWAR_H);
}

template <class C>
__device__ __forceinline__ void load_env_finish(Regs<C>& s, Lds<C>& L, const RawEnv<C>& r, uint32_t W, int tid) {
  s.hdr = r.hdr;
  s.epi = r.epi;
#pragma unroll
  for (int i = 0; i < C::NAM; ++i) s.ag[i] = r.ag[i];
  // pickup cell j = target byte | expiry byte << 8: two cells per v_perm, stored as 16-bit halves
#pragma unroll
  for (int w = 0; w < C::PW; ++w) {
    const uint32_t lo = __builtin_amdgcn_perm(r.pm[w], r.pt[w], 0x05010400u);   // cells 4w, 4w+1
    const uint32_t hi = __builtin_amdgcn_perm(r.pm[w], r.pt[w], 0x07030602u);   // cells 4w+2, 4w+3
    L.pkp[4 * w][tid] = (uint16_t)lo;
    L.pkp[4 * w + 1][tid] = (uint16_t)(lo >> 16);
    L.pkp[4 * w + 2][tid] = (uint16_t)hi;
    L.pkp[4 * w + 3][tid] = (uint16_t)(hi >> 16);
  }
  s.am = active_mask<C>(r.pt);
  // An open request expires at step t0 + ((expiry byte - t0) mod 256), as the expiry phase counts;
  // it is "early" if that is before W, i.e. its steps left < W - t0 (never when t0 >= W).  Four
  // points per SWAR test.
  const uint32_t t0 = s.hdr & 0xFFFFu;
  const uint32_t thr = t0 < W ? W - t0 : 0u;          // <= 255
  uint32_t early = 0;
#pragma unroll
  for (int w = 0; w < C::PW; ++w)
    early |= nz_hi(r.pt[w]) & swar_lt(swar_sub(r.pm[w], (t0 & 0xFFu) * 0x01010101u), thr * 0x01010101u);
  s.wskip = __any(early != 0u) ? 0u : W;
}

template <class C>
__device__ __forceinline__ void store_env(const Regs<C>& s, const Lds<C>& L, uint32_t* __restrict__ st,
                                          int64_t B, int64_t e0, int na, int tid) {
  uint32_t* pl = st + e0;   // word planes as in load_env_issue: wave-uniform base + lane offset
  pl[tid] = s.hdr;
  pl += B;
  pl[tid] = s.epi;
#pragma unroll
  for (int i = 0; i < C::NAM; ++i)
    if (i < na) {
      pl += B;
      pl[tid] = s.ag[i];
    }
  uint32_t* pt = pl + B;
  uint32_t* pm = pt + (int64_t)C::PW * B;
#pragma unroll
  for (int w = 0; w < C::PW; ++w) {
    // four 16-bit cells -> target bytes and expiry bytes: two shift-ors and two v_perm
    const uint32_t lo = (uint32_t)L.pkp[4 * w][tid] | ((uint32_t)L.pkp[4 * w + 1][tid] << 16);
    const uint32_t hi = (uint32_t)L.pkp[4 * w + 2][tid] | ((uint32_t)L.pkp[4 * w + 3][tid] << 16);
    pt[tid] = __builtin_amdgcn_perm(hi, lo, 0x06040200u);
    pm[tid] = __builtin_amdgcn_perm(hi, lo, 0x07050301u);
    pt += B;
    pm += B;
  }
}

// ----------------------------------------------------------------------------- reset
// core.py:167-221 (philox draws): spawn on interior non-pickup cells, open R requests.
// Law (the same as the reference's np.random.choice(P, R) paired with choice(Dp, R)): a uniform
// R-subset of the pickup points, each given a distinct uniformly random delivery target.  The
// subset comes from Floyd's algorithm (item j: r = uniform over [0, m] with m = P - R + j, take r
// unless already taken, else m), one test and two ors per item; the targets are a uniform ordered
// R-tuple without replacement (the r-th unused delivery point, r uniform over Dp - j), so pairing
// them with the points in Floyd's order is a uniform injection.  NAC >= 0 is the agent count at
// compile time (the fused rollout): every stream word then has a fixed place in the precomputed
// Philox blocks, and the whole reset is straight-line code.
// TO_SLOT: the same draws and results for every lane, written to the lane's reset slot (Lds::rs_*)
// instead of its registers and pickup plane, for episode epi + 1.
// The pickup-plane rows (and, with occ, the occupancy rows) of the wave's 64 columns cleared with
// 16-byte stores, for a reset of every lane of a full wave (synchronised episodes end together): 5
// stores instead of 36 (Medium) per lane, 4 instead of 16 for the grid.
template <class C>
__device__ __forceinline__ void clear_wave_columns(Lds<C>& L, int tid, bool occ) {
  const int wb = tid & ~63, lane = tid & 63;
  constexpr int CPL = 16 / PKW, LPR = 64 / CPL, RPS = 64 / LPR;   // cells per lane, lanes per row, rows
#pragma unroll
  for (int j0 = 0; j0 < C::P; j0 += RPS) {
    const int j = j0 + lane / LPR;
    if (C::P % RPS == 0 || j < C::P)
      *reinterpret_cast<uint4*>(&L.pkp[j][wb + CPL * (lane % LPR)]) = make_uint4(0u, 0u, 0u, 0u);
  }
  if (occ) {
#pragma unroll
    for (int y0 = 0; y0 < C::D; y0 += 4) {
      const int y = y0 + (lane >> 4);
      if (C::D % 4 == 0 || y < C::D)
        *reinterpret_cast<uint4*>(&L.occ[y][wb + 4 * (lane & 15)]) = make_uint4(0u, 0u, 0u, 0u);
    }
  }
}

// WAVE: every lane of a full wave resets (the caller checked): the pickup plane is cleared
// wave-wide with clear_wave_columns.
template <class C, int NAC = -1, bool TO_SLOT = false, bool WAVE = false>
__device__ __forceinline__ void reset_philox(Regs<C>& s, Lds<C>& L, const Keys& k, uint32_t gid,
                                             int na_rt, int variable_n, uint32_t W, int tid,
                                             Slots<C>* RS = nullptr) {
  WH_PHASE_MARK(reset);
  const uint32_t ep = s.epi + 1u;
  const int na = NAC >= 0 ? NAC : na_rt;
  constexpr int NB = NAC >= 0 ? (1 + NAC + 2 * C::R + 3) / 4 : 1;
  uint4 blk[NB];
  if constexpr (NAC >= 0) {
#pragma unroll
    for (int b = 0; b < NB; ++b) blk[b] = stream_block(k, gid, ep, 0u, PUR_RESET, (uint32_t)b);
  }
  Reader rd(k, gid, ep, 0u, PUR_RESET);
  auto word = [&](int j) -> uint32_t {
    if constexpr (NAC >= 0) return comp(blk[j >> 2], j & 3);
    else return rd.word(j);
  };
  const uint32_t n = variable_n ? 1u + __umulhi(word(0), (uint32_t)na) : (uint32_t)na;
#pragma unroll
  for (int i = 0; i < C::NAM; ++i) {
    uint32_t a = IDLE;
    if (i < na) {
      const uint32_t v = __umulhi(word(1 + i), (uint32_t)C::NV);
      const uint32_t cell = L.valid_cell(v);
      a = (i < (int)n) ? (cell | IDLE) : IDLE;
    }
    if (TO_SLOT) RS->rs_ag[i][tid] = a;
    else s.ag[i] = a;
  }
  if (!TO_SLOT) {
    if constexpr (WAVE) {
      clear_wave_columns<C>(L, tid, true);
    } else {
#pragma unroll
      for (int j = 0; j < C::P; ++j) L.pkp[j][tid] = 0;
    }
  }
  const uint32_t wexp = (W & 0xFFu) << 8;   // opened at t = 0: expires at step W
  uint32_t plo = 0, phi = 0;                // Floyd's subset so far
  uint32_t sel[C::R], tg[C::R];
#pragma unroll
  for (int j = 0; j < C::R; ++j) {
    constexpr int M0 = C::P - C::R;
    const uint32_t m = (uint32_t)(M0 + j);
    const uint32_t r = __umulhi(word(1 + na + 2 * j), m + 1u);
    sel[j] = r;
    if (j > 0) {   // taken already: bit r of the subset, moved to bit 63 by one 64-bit shift
      const uint64_t sh = (((uint64_t)phi << 32) | plo) << (63u - r);
      sel[j] = msel(sgn((uint32_t)(sh >> 32)), m, r);
    }
    const uint64_t sb = 1ull << sel[j];
    plo |= (uint32_t)sb;
    phi |= (uint32_t)(sb >> 32);
    tg[j] = __umulhi(word(2 + na + 2 * j), (uint32_t)(C::DP - j));   // rank among unused targets
  }
  // ranks -> targets (item j: the tg[j]-th delivery point not taken by items < j), decoded from
  // the last item back: every later item at or above item j's value moves up one.  The same
  // values as a rank selection per item, as independent compare-adds instead of a serial chain.
#pragma unroll
  for (int j = C::R - 2; j >= 0; --j)
#pragma unroll
    for (int i = j + 1; i < C::R; ++i) tg[i] += 1u - ((tg[i] - tg[j]) >> 31);   // + (tg[i] >= tg[j])
  if (TO_SLOT) {
#pragma unroll
    for (int j = 0; j < C::R; ++j) RS->rs_req[j][tid] = (uint16_t)(sel[j] | ((tg[j] + 1u) << 8));
    RS->rs_am[0][tid] = plo;
    RS->rs_am[1][tid] = phi;
    RS->rs_hdr[tid] = (n << 16) | (1u << 24);
    RS->rs_ep[tid] = ep;
  } else {
#pragma unroll
    for (int j = 0; j < C::R; ++j) L.pkp[sel[j]][tid] = (uint16_t)((tg[j] + 1u) | wexp);
    s.am = ((uint64_t)phi << 32) | plo;
    s.hdr = (n << 16) | (1u << 24);
    s.epi = ep;
  }
  WH_PHASE_MARK(reset_end);
}

// The reset of the env of lane l of this wave from its reset slot (valid: rs_ep == epi + 1), by
// the whole wave: agent words and request cells read across lanes (lane i reads field i of lane
// l's column), the pickup-plane and occupancy columns cleared and written one cell per lane.
// Bit-identical to reset_philox<C, NA> (plus the occupancy clear) for that env, for ~40 issue slots
// instead of a Philox block per lane, a Floyd chain on wave-uniform values and the rank decode.
template <class C, int NA>
__device__ __forceinline__ void reset_from_slot(Regs<C>& s, Lds<C>& L, const Slots<C>& RS, uint32_t W, int tid, int l) {
  WH_PHASE_MARK(slot_reset);
  const int lane = tid & 63;
  const int col = (tid & ~63) + l;
  const uint32_t me = mask_z((uint32_t)(lane ^ l));
  const uint32_t av = RS.rs_ag[lane < NA ? lane : 0][col];
  const uint32_t rq = RS.rs_req[lane < C::R ? lane : 0][col];
  const uint32_t alo = RS.rs_am[0][col], ahi = RS.rs_am[1][col], hdr = RS.rs_hdr[col];
#pragma unroll
  for (int i = 0; i < C::NAM; ++i)
    s.ag[i] = msel(me, i < NA ? (uint32_t)__builtin_amdgcn_readlane(av, i) : IDLE, s.ag[i]);
  if (lane < C::P) L.pkp[lane][col] = 0;
  if (lane < C::D) L.occ[lane][col] = 0u;
  if (lane < C::R) L.pkp[rq & 0xFFu][col] = (uint16_t)((rq >> 8) | ((W & 0xFFu) << 8));   // after the clear
  s.am = ((uint64_t)msel(me, ahi, (uint32_t)(s.am >> 32)) << 32) | msel(me, alo, (uint32_t)s.am);
  s.hdr = msel(me, hdr, s.hdr);
  s.epi = msel(me, s.epi + 1u, s.epi);
}

// The same philox reset for ONE env -- the env of lane l of this wave -- computed by the whole
// wave: a Philox block per lane (lane b holds block b), words read across lanes, the subset and
// target arithmetic on wave-uniform values (target ranks by v_mbcnt + ballot), and lane l's LDS
// column (pickup cells, occupancy rows) written one cell per lane.  Bit-identical to
// reset_philox<C, NA> (plus the occupancy clear) for that env, at a fraction of its issue cost:
// the fused rollout uses it when a single lane of the wave ends its episode, which is what
// desynchronised episodes produce (env ends are spread over the steps, B/T per step).
template <class C, int NA>
__device__ __forceinline__ void reset_lane(Regs<C>& s, Lds<C>& L, const Keys& k, uint32_t gid,
                                           int variable_n, uint32_t W, int tid, int l) {
  WH_PHASE_MARK(lane_reset);
  const int lane = tid & 63;
  const int col = (tid & ~63) + l;                      // lane l's LDS column
  const uint32_t me = mask_z((uint32_t)(lane ^ l));      // all-ones on lane l
  const uint32_t gid_l = __builtin_amdgcn_readlane(gid, l);
  const uint32_t ep = __builtin_amdgcn_readlane(s.epi, l) + 1u;
  constexpr int NB = (1 + NA + 2 * C::R + 3) / 4;
  static_assert(NB <= 64, "one Philox block per lane");
  const uint4 mine = stream_block(k, gid_l, ep, 0u, PUR_RESET, (uint32_t)(lane < NB ? lane : 0));
  auto word = [&](int j) -> uint32_t { return __builtin_amdgcn_readlane(comp(mine, j & 3), j >> 2); };
  const uint32_t n = variable_n ? 1u + __umulhi(word(0), (uint32_t)NA) : (uint32_t)NA;
  // every spawn cell is read (all reads in flight together) and slots >= n are then masked: with
  // `i < n` as the condition of the read, n being wave-uniform, each read sat in its own scalar
  // branch behind a waitcnt -- NA serial LDS round trips per reset
  uint32_t cell[C::NAM];
#pragma unroll
  for (int i = 0; i < C::NAM; ++i)
    cell[i] = i < NA ? L.valid_cell(__umulhi(word(1 + i), (uint32_t)C::NV)) : 0u;
#pragma unroll
  for (int i = 0; i < C::NAM; ++i) {
    const uint32_t live = sgn((uint32_t)i - n);   // all-ones: i < n
    s.ag[i] = msel(me, bop3<(TA & TB) | TC>(live, cell[i], IDLE), s.ag[i]);
  }
  if (lane < C::P) L.pkp[lane][col] = 0;
  if (lane < C::D) L.occ[lane][col] = 0u;
  const uint32_t wexp = (W & 0xFFu) << 8;
  // points: Floyd's subset on wave-uniform values (a short scalar chain); lane j < R keeps item j
  uint64_t S = 0;
  uint32_t selv = (uint32_t)C::P, tgv = 0;
#pragma unroll
  for (int j = 0; j < C::R; ++j) {
    const uint32_t m = (uint32_t)(C::P - C::R + j);
    const uint32_t r = __umulhi(word(1 + NA + 2 * j), m + 1u);
    const uint32_t sel = (j > 0 && ((S >> r) & 1ull)) ? m : r;
    S |= 1ull << sel;
    // (computed on every lane, then selected: as `lane == j ? rank : tgv` each item was an
    // exec-masked branch, ~8 issue slots of branching per item)
    const uint32_t rank = __umulhi(word(2 + NA + 2 * j), (uint32_t)(C::DP - j));   // r2_j
    const uint32_t mj = mask_z((uint32_t)(lane ^ j));
    selv = msel(mj, sel, selv);
    tgv = msel(mj, rank, tgv);
  }
  // targets: item j is the r2_j-th delivery point not taken by items < j.  Decoded in parallel
  // (lane j holds item j): from the last item back, every later item at or above item j's value
  // moves up one -- the same values as the per-lane rank selection, without its serial chain.
#pragma unroll
  for (int j = C::R - 2; j >= 0; --j) {
    const uint32_t xj = __builtin_amdgcn_readlane(tgv, j);
    tgv += (lane > j && lane < C::R && tgv >= xj) ? 1u : 0u;
  }
  const uint32_t valv = (tgv + 1u) | wexp;
  if (lane < C::R) L.pkp[selv][col] = (uint16_t)valv;     // after the clear (LDS ops in order)
  s.am = ((uint64_t)msel(me, (uint32_t)(S >> 32), (uint32_t)(s.am >> 32)) << 32) | msel(me, (uint32_t)S, (uint32_t)s.am);
  s.hdr = msel(me, (n << 16) | (1u << 24), s.hdr);
  s.epi = msel(me, ep, s.epi);
}

template <class C>
__device__ __forceinline__ void reset_injected(Regs<C>& s, Lds<C>& L, int64_t e, int na,
                                               const int32_t* spawn, const int32_t* pickups,
                                               const int32_t* targets, const int32_t* nn,
                                               uint32_t W, int tid) {
  const uint32_t n = nn ? min((uint32_t)nn[e], (uint32_t)na) : (uint32_t)na;
#pragma unroll
  for (int i = 0; i < C::NAM; ++i) {
    uint32_t a = IDLE;
    if (i < na && i < (int)n) {
      const uint32_t x = min((uint32_t)spawn[(e * na + i) * 2], (uint32_t)(C::D - 1));
      const uint32_t y = min((uint32_t)spawn[(e * na + i) * 2 + 1], (uint32_t)(C::D - 1));
      a = x | (y << 16) | IDLE;
    }
    s.ag[i] = a;
  }
#pragma unroll
  for (int j = 0; j < C::P; ++j) L.pkp[j][tid] = 0;
  const uint32_t wexp = (W & 0xFFu) << 8;   // opened at t = 0: expires at step W
  uint64_t opened = 0;
  for (int j = 0; j < C::R; ++j) {
    const uint32_t sel = (uint32_t)pickups[e * C::R + j];
    const uint32_t tg = (uint32_t)targets[e * C::R + j];
    if (sel >= (uint32_t)C::P || tg >= (uint32_t)C::DP) continue;   // invalid injected draw: ignored
    opened |= 1ull << sel;
    L.pkp[sel][tid] = (uint16_t)((tg + 1u) | wexp);
  }
  s.am = opened;
  s.hdr = (n << 16) | (1u << 24);
  s.epi = s.epi + 1u;
}

// ----------------------------------------------------------------------------- policy
// baseline/solvers.py:27-58 evaluated on the state, producing unit steps d (packed i16 pairs):
// availability 0 (fresh reset, or carrying) -> head for the own delivery target (the null cell
// after reset), else for the nearest open request by Manhattan distance, first (lowest pickup
// index) minimum wins; step = clip(goal - pos, -1, 1).  Random actions come from the
// POLICY/RANDOM streams.  Slots >= n get arbitrary steps: step_env never moves them.
// EFF: random moves are returned as the step they take (off-grid coordinates kept, core.py:282-287),
// so a step loop can add them without the clamp (step_env<CLAMP = false>); wh_policy reports the
// drawn action itself (EFF = false), as solvers.py:44-45 returns action_space.sample().
template <class C, int POLICY, bool EFF = false>
__device__ __forceinline__ void policy_steps(const Regs<C>& s, const Lds<C>& L, const Keys& k,
                                             uint32_t gid, float p, uint32_t (&d)[C::NAM]) {
  const uint32_t t = s.hdr & 0xFFFFu;
  if (POLICY == POL_RANDOM) {
#pragma unroll
    for (int b = 0; b < (C::NAM + 3) / 4; ++b) {
      const uint4 blk = stream_block(k, gid, s.epi, t, PUR_RANDOM, (uint32_t)b);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int i = 4 * b + c;
        if (i < C::NAM) d[i] = L.mv(__umulhi(comp(blk, c), 9u));
      }
    }
  } else {
    WH_PHASE_MARK(policy_rtag);
    // Open requests in ascending pickup order (core.py:409-418).  Index P of the tables is a
    // sentinel (far-away cell, null-cell tag) that fills missing slots; after a reset every slot is
    // the sentinel, so every agent's "nearest request" is the null cell, which is where the
    // reference's reset observation sends the greedy solver (availability 0, core.py:233-236).
    const uint32_t mf = 0u - ((s.hdr >> 24) & 1u);
    uint32_t mlo = bop3<~TA & TB>(mf, (uint32_t)s.am, 0u);
    uint32_t mhi = bop3<~TA & TB>(mf, (uint32_t)(s.am >> 32), 0u);
    uint32_t rp[C::R], tg[C::R];
#pragma unroll
    for (int r = 0; r < C::R; ++r) {
      uint32_t flo, fhi;
      asm("v_ffbl_b32 %0, %1" : "=v"(flo) : "v"(mlo));   // 0xFFFFFFFF when empty
      asm("v_ffbl_b32 %0, %1" : "=v"(fhi) : "v"(mhi));
      const uint32_t j = __builtin_elementwise_min(
          __builtin_elementwise_min(flo, __builtin_elementwise_add_sat(fhi, 32u)), (uint32_t)C::P);
      const uint2 v = L.rtag(j);
      rp[r] = v.x;
      tg[r] = v.y;
      uint64_t m = ((uint64_t)mhi << 32) | mlo;
      m &= m - 1ull;
      mlo = (uint32_t)m;
      mhi = (uint32_t)(m >> 32);
    }
    WH_PHASE_MARK(policy_agents);
#pragma unroll
    for (int i = 0; i < C::NAM; ++i) {
      const uint32_t a = s.ag[i];
      const uint32_t pos = a & XY16;
      uint32_t best = 0xFFFFFFFFu;
#pragma unroll
      for (int r = 0; r < C::R; ++r)   // key = dist << 16 | pickup << 10 | y << 5 | x
        best = min(best, __builtin_amdgcn_sad_hi_u8(pos, rp[r], tg[r]));
      const uint32_t near = (__builtin_amdgcn_ubfe(best, 5u, 5u) << 16) | (best & 31u);   // y << 16 | x
      const uint32_t dst = __builtin_amdgcn_perm(a, a, 0x0C030C01u);   // target bytes 1, 3 -> x | y << 16
      const uint32_t idle = (uint32_t)__builtin_amdgcn_sbfe((int)a, 15, 1);   // target byte 0xFF
      const uint32_t goal = msel(idle, near, dst);
      // goal is a grid cell, so pos + d stays on the grid: step_env<CLAMP = false> adds it as is
      d[i] = pk_min_i16(pk_max_i16(pk_sub_i16(goal, pos), 0xFFFFFFFFu), 0x00010001u);
    }
    if (WH_RARE(p > 0.0f)) {
#pragma unroll
      for (int b = 0; b < (C::NAM + 1) / 2; ++b) {
        const uint4 blk = stream_block(k, gid, s.epi, t, PUR_POLICY, (uint32_t)b);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int i = 2 * b + h;
          if (i < C::NAM) {
            const float u = (float)(comp(blk, 2 * h) >> 8) * (1.0f / 16777216.0f);
            uint32_t rnd = L.mv(__umulhi(comp(blk, 2 * h + 1), 9u));
            if (EFF) {
              const uint32_t pos = s.ag[i] & XY16;
              rnd = pk_sub_i16(step16<C::D>(pos, rnd), pos);
            }
            d[i] = (u < p) ? rnd : d[i];
          }
        }
      }
    }
  }
  // (slots >= n: whatever d says, step_env never moves them)
}

// ----------------------------------------------------------------------------- step
// core.py:267-368 on one env held in registers.  Returns done.  No data-dependent branches:
// LDS side effects are predicated through neutral operands (and ~0 / or 0 / the scratch word),
// so each phase is one basic block and its LDS reads issue back to back.
// INJ = false compiles the injected-draw regeneration out (the fused rollout and the sampler step
// always draw from philox): less code in the step loop and no per-step test of `regen`.
// CLAMP = false: the steps come from the greedy policy, whose goals are grid cells, so pos + d
// never leaves the grid and the off-grid rule (a clamp) is the identity.
struct LazyGrid {
  bool rebuild;   // the occupancy grid may lack an agent's cell: rebuild it before the next move
  uint32_t cm;    // slots sharing a cell (found by the last rebuild or reset): rebuild once one moves
};

#ifdef WH_COUNT_REV
__device__ unsigned long long g_wh_revcount[2];   // [0] reverse-key loops, [1] crossing-only loops
#endif

// The action-dict order of the ORDERED path: entry rows [B, ol] (ol = 1 .. 4 * NA: a dict may name an
// agent under each of its key forms) and the per-lane LDS key list of the entries' moves (16 bits
// each, [entry][lane]: OKeys, only in the ORDERED instances).
struct OrderIn {
  const int32_t* __restrict__ order;
  int ol;
  uint16_t* keys;
};
template <class C>
struct OKeys {
  uint16_t k[4 * C::NAM][BT];
};

template <class C, bool ORDERED, bool INJ = true, bool CLAMP = true, bool LAZY = false>
__device__ __forceinline__ bool step_env(Regs<C>& s, Lds<C>& L, const uint32_t (&dstep)[C::NAM],
                                         const OrderIn& oi,
                                         const int32_t* __restrict__ actions_g,
                                         const int32_t* __restrict__ regen, const Keys& k,
                                         uint32_t gid, int64_t e, int na, int phase, uint32_t T,
                                         uint32_t W, float (&rew)[C::NAM], int32_t* n_inactive,
                                         int tid, int ablate, LazyGrid* lg = nullptr,
                                         const uint4* pre_rblk = nullptr) {
  const uint32_t n = (s.hdr >> 16) & 0xFFu;
  uint32_t t = s.hdr & 0xFFFFu;
  uint32_t rewm[C::NAM];   // reward masks: all-ones = 1.0f
  constexpr bool HOIST = LAZY && !INJ && kRegenHoist && !kHoistPolicy;   // (see the move phase)
  uint4 rblk0 = make_uint4(0u, 0u, 0u, 0u);
  bool hoisted = false;
  if (pre_rblk) {   // computed by the caller ahead of the policy (kHoistPolicy)
    rblk0 = *pre_rblk;
    hoisted = true;
  }

  if (phase != PH_REGEN) {
    t = (t + 1u) & 0xFFFFu;                                 // core.py:267
#pragma unroll
    for (int i = 0; i < C::NAM; ++i) rewm[i] = 0u;

    // ---- request expiry (core.py:303-306), 4 pickup points per op.  Timer bytes hold the low 8
    //      bits of the step at which the request expires (opened at t0 with wait W: t0 + W, the
    //      step whose decrement would reach 0), so nothing is decremented.  A request opened at
    //      t0 >= 0 cannot expire before step W, so waves with every t < W skip the phase (with
    //      T = W, 199 of 200 steps) unless they were loaded from a state outside that invariant
    //      (s.wskip).  Run before the move: expiry reads no positions and the move reads no
    //      requests, so the two commute, and the pickup table is final before the move loop --
    //      which lets its lookups be issued inside it.
    WH_PHASE_MARK(expire);
    const uint64_t em = (ablate & 4) ? 0ull : __ballot(t >= s.wskip);
    if (WH_RARE(em != 0) && __popcll(em) == 1 && __ballot(true) == ~0ull) {
      // one lane of a full wave due (desynchronised episodes): its P pickup cells checked one per
      // lane of the wave, instead of the whole wave walking every lane's requests
      const int l = __builtin_ctzll(em), lane = tid & 63, col = (tid & ~63) + l;
      const uint32_t t8 = (uint32_t)__builtin_amdgcn_readlane(t, l) & 0xFFu;
      const uint32_t v = lane < C::P ? (uint32_t)L.pkp[lane][col] : 0u;
      const bool ex = (v & 0xFFu) != 0u && (v >> 8) == t8;
      if (ex) L.clear_target(lane, col);
      const uint64_t exm = __ballot(ex);
      s.am = lane == l ? (s.am & ~exm) : s.am;
    } else if (WH_RARE(em != 0)) {
      if (__any(__popcll(s.am) > C::R)) {   // a hand-built state with more than R requests: scan all
        uint64_t expired = 0;
#pragma unroll
        for (int j = 0; j < C::P; ++j) {
          const uint32_t v = L.pkp[j][tid];
          const bool ex = (v & 0xFFu) != 0u && (v >> 8) == (t & 0xFFu);
          if (ex) L.clear_target(j, tid);
          expired |= (uint64_t)ex << j;
        }
        s.am &= ~expired;
      } else {
        // walk the (at most R) open requests in the mask, as the policy does; index P (missing
        // slots) is the scratch row, and its "expiry" is discarded by the j < P test
        uint32_t mlo = (uint32_t)s.am, mhi = (uint32_t)(s.am >> 32), elo = 0, ehi = 0;
        const uint32_t t8 = t & 0xFFu;
#pragma unroll
        for (int r = 0; r < C::R; ++r) {
          uint32_t flo, fhi;
          asm("v_ffbl_b32 %0, %1" : "=v"(flo) : "v"(mlo));   // 0xFFFFFFFF when empty
          asm("v_ffbl_b32 %0, %1" : "=v"(fhi) : "v"(mhi));
          const uint32_t j = __builtin_elementwise_min(
              __builtin_elementwise_min(flo, __builtin_elementwise_add_sat(fhi, 32u)), (uint32_t)C::P);
          const uint32_t v = L.pkp[j][tid];
          const uint32_t ex = bop3<TA & TB>(mask_z((v >> 8) ^ t8), sgn(j - (uint32_t)C::P), 0xFFFFFFFFu);
          *reinterpret_cast<uint8_t*>(&L.pkp[msel(ex, j, (uint32_t)C::P)][tid]) = 0;
          const uint64_t b = 1ull << (j & 63u);
          elo |= bop3<TA & TB>(ex, (uint32_t)b, 0u);
          ehi |= bop3<TA & TB>(ex, (uint32_t)(b >> 32), 0u);
          uint64_t m = ((uint64_t)mhi << 32) | mlo;
          m &= m - 1ull;
          mlo = (uint32_t)m;
          mhi = (uint32_t)(m >> 32);
        }
        s.am &= ~(((uint64_t)ehi << 32) | elo);
      }
    }

    // ---- move + collision, sequential in action-dict order (core.py:275-300)
    WH_PHASE_MARK(move);
    // The fused rollout's regeneration almost always draws (some lane of the wave reopens a point
    // on nearly every step), so its first Philox block -- a chain of ten dependent rounds -- is
    // computed inside the move loop's basic block, where the scheduler fills the serial chain's
    // issue gaps with it, instead of on its own after the pickups.
    uint32_t cp[C::NAM], tb[C::NAM], dst[C::NAM];   // pickup lookups (core.py:309-329): cell_row,
                                                    // target byte, delivery cell
    bool looked = false;
    // pickups (core.py:309-335): agent i takes iff it stands on a pickup point (cp != 0) with an
    // open request (tb != 0) and is idle -- slots >= n sit idle on the corner cell (0, 0), which is
    // no pickup point; min3 of the three 0/1-ish terms is 1 exactly when all hold.  Every agent
    // decides against the pre-pickup table (two agents on one point both take it), so the
    // points are cleared only after every agent's target byte has been read (clr[i]: the byte to
    // zero, row P = scratch).  The ascending move loop issues an agent's three dependent lookups
    // kPickDist turns apart and decides its pickup 3 * kPickDist turns after its move, when the
    // last lookup has landed, so only a few agents' lookups are live at a time.
    uint32_t prlo = 0, prhi = 0;   // points picked up, rotated left by one (see pick)
    uint32_t clr[C::NAM];
    auto pick = [&](int i, uint32_t cpv, uint32_t tbv, uint32_t dstv) {
      const uint32_t a = s.ag[i];
      const uint32_t idle01 = (a >> 15) & 1u;   // delivery-target byte 0xFF
      const uint32_t m = 0u - __builtin_elementwise_min(__builtin_elementwise_min(cpv, tbv), idle01);
      s.ag[i] = bop3<(TA & TB & TC) | (~TA & TB)>(m, a, dstv);   // idle target bytes are 0xFF
      // bit (j + 1) mod 64 for point j (cpv = j + 1): rotated back once after the loop
      const uint64_t bit = 1ull << (cpv & 63u);
      prlo = bop3<(TA & TB) | TC>(m, (uint32_t)bit, prlo);
      prhi = bop3<(TA & TB) | TC>(m, (uint32_t)(bit >> 32), prhi);
      clr[i] = msel(m, cpv, (uint32_t)(C::P + 1));
      rewm[i] = m;
    };
#ifndef WH_NO_PICK_IN_LOOP   // (A/B builds: -DWH_NO_PICK_IN_LOOP decides after the move loop)
    constexpr bool PICK_IN_LOOP = true;
#else
    constexpr bool PICK_IN_LOOP = false;
#endif
    if (!(ablate & 2)) {
      // The grid is rebuilt as {live agents' cells} (core.py:275-276) by OR-ing the cells into
      // what the previous step left, which is always a subset of them (a set bit is an arrival
      // or an agent that stayed; leaving clears), so no per-step clear is needed.  k_step clears
      // it at launch and after an auto-reset; the ordered (drop-in) path clears it every step.
      // LAZY (fused rollout): once rebuilt, the grid a lane carries stays exactly its agents' cells
      // (a move is accepted only into a free cell) until an agent leaves a cell it shares -- the
      // reference clears the cell under the agent that stays (core.py:290), and only its per-step
      // rebuild sets it again.  Shared cells come from resets, whose spawns are drawn independently
      // (core.py:191-201), and persist only while the agents sharing them stay put.  So a lane asks
      // for the rebuild (lg->rebuild) after a grid clear, and after a step in which an agent that
      // shares a cell (lg->cm) moved; the wave skips it when no lane asks.
      if (ORDERED) {
#pragma unroll
        for (int y = 0; y < C::D; ++y) L.occ[y][tid] = 0u;
      }
      if (!LAZY) {
#pragma unroll
        for (int i = 0; i < C::NAM; ++i) {
          const uint32_t p = s.ag[i] & XY16;
          const uint32_t mlive = sgn((uint32_t)i - n);
          atomicOr(&L.occ[p >> 16][tid], bop3<TA & TB>(mlive, 1u << (p & 31u), 0u));
        }
      } else if (WH_RARE(__any(lg->rebuild))) {
        // (the terms are written so that none is shared with the move loop below: a shared one
        // would be hoisted above the branch, and the skip path would pay a register copy per term)
        const uint32_t livebits = (2u << (n - 1u)) - 1u;   // n >= 1
        uint32_t q[C::NAM];   // live cells; slots >= n get distinct off-grid stand-ins
#pragma unroll
        for (int i = 0; i < C::NAM; ++i) {
          const uint32_t a = s.ag[i];
          const uint32_t mlive = (uint32_t)__builtin_amdgcn_sbfe((int)livebits, (uint32_t)i, 1u);
          uint32_t bit;
          asm volatile("v_lshlrev_b32 %0, %1, 1" : "=v"(bit) : "v"(a));   // 1 << (x & 31)
          atomicOr(&L.occ[__builtin_amdgcn_ubfe(a, 16u, 8u)][tid], bop3<TA & TB>(mlive, bit, 0u));
          q[i] = msel(mlive, a, 0x80u + (uint32_t)i);   // position bytes compared below
        }
        uint32_t m[C::NAM];   // m[i] == 0: slot i shares its cell
#pragma unroll
        for (int i = 0; i < C::NAM; ++i) m[i] = 0xFFFFFFFFu;
#pragma unroll
        for (int i = 1; i < C::NAM; ++i)
#pragma unroll
          for (int j = 0; j < i; ++j) {
            const uint32_t x = bop3<(TA ^ TB) & TC>(q[i], q[j], XY16);
            m[i] = min(m[i], x);
            m[j] = min(m[j], x);
          }
        uint32_t cm = 0;
#pragma unroll
        for (int i = 0; i < C::NAM; ++i) cm |= (m[i] == 0u ? 1u : 0u) << i;
        lg->cm = cm;
        lg->rebuild = false;
      }
      uint32_t rk[C::NAM], xk[C::NAM];   // ascending path: reverse key, crossing pair
      if (ORDERED) {   // drop-in single env / BaseEnv: entries in action-dict order, records in LDS
        // Forbidden moves (core.py:293-297) by the one-key-per-move form of the ascending loop (UKEY,
        // below): a move p -> c is keyed by its direction and its undirected edge / square / cell
        // (u = p + c per coordinate), and an accepted move forbids exactly the moves with its u and
        // another direction (an accepted stay: every later stay on its cell, via a flipped low bit).
        // 16 bits per key: (dx + 1) | (dy + 1) << 2 | xsum << 4 | ysum << 10, so entry k is blocked iff
        // 1 <= (K_k ^ S_j) <= 15 for an earlier entry j; a rejected entry stores 0xFFFF (xsum 63:
        // never a real sum, D <= 32).  The keys live in LDS ([entry][lane]), so a dict of any length
        // up to 4 * NA entries runs in one pass: the first NAM entries unrolled (their order words
        // and key reads issued together), the rest -- only a dict naming agents under several keys
        // has them -- in a rolled loop.
#pragma unroll
        for (int i = 0; i < C::NAM; ++i) L.agl[i][tid] = s.ag[i];
        auto entry = [&](int sidx, int32_t raw, bool unrolled) {
          // entry: agent id in bits 0-7, optionally the entry's own action + 1 in bits 8-15 (a dict
          // naming one agent under several keys moves it once per key, with that key's action)
          int who = raw < 0 ? -1 : (raw & 0xFF);
          const uint32_t sact = raw < 0 ? 0u : ((uint32_t)raw >> 8) & 0xFFu;
          const bool live = who >= 0 && who < (int)n && who < C::NAM;
          who = live ? who : 0;
          const uint32_t a = L.agl[who][tid];
          const uint32_t mv = live ? (sact ? sact - 1u : (uint32_t)actions_g[e * na + who]) : 4u;
          const uint32_t p = a & XY16;
          const uint32_t c = step16<C::D>(p, L.mv(mv > 8u ? 4u : mv));
          const bool occupied = (L.occ[c >> 16][tid] >> (c & 31u)) & 1u;
          const uint32_t sum = as_u(as_s2(p) + as_s2(c)), dd = pk_sub_i16(c, p);
          const uint32_t key = (((dd + 1u) & 3u) | ((((dd >> 16) + 1u) & 3u) << 2) | ((sum & 63u) << 4) |
                                (((sum >> 16) & 63u) << 10));
          uint32_t f = 15u;
          if (unrolled) {
#pragma unroll
            for (int j = 0; j < C::NAM; ++j)
              if (j < sidx) f = min(f, (key ^ (uint32_t)oi.keys[j * BT + tid]) - 1u);
          } else {
            for (int j = 0; j < sidx; ++j) f = min(f, (key ^ (uint32_t)oi.keys[j * BT + tid]) - 1u);
          }
          const bool ok = live && !occupied && f >= 15u;
          atomicAnd(&L.occ[p >> 16][tid], ok ? ~(1u << (p & 31u)) : 0xFFFFFFFFu);
          atomicOr(&L.occ[c >> 16][tid], ok ? (1u << (c & 31u)) : 0u);
          oi.keys[sidx * BT + tid] = (uint16_t)(ok ? (dd == 0u ? key ^ 1u : key) : 0xFFFFu);
          L.agl[who][tid] = ok ? ((a & ~XY16) | c) : a;
        };
        const int32_t* orow = oi.order + e * oi.ol;
        int32_t raws[C::NAM];
#pragma unroll
        for (int sidx = 0; sidx < C::NAM; ++sidx) raws[sidx] = sidx < oi.ol ? orow[sidx] : -1;
#pragma unroll
        for (int sidx = 0; sidx < C::NAM; ++sidx) entry(sidx, raws[sidx], true);
        for (int sidx = C::NAM; sidx < oi.ol; ++sidx) entry(sidx, orow[sidx], false);
#pragma unroll
        for (int i = 0; i < C::NAM; ++i) s.ag[i] = L.agl[i][tid];
      } else {
        // Ascending agent order.  Every agent moves only on its own turn, so all candidate cells
        // are known up front.  The occupancy word for agent s+1 is read one turn early (before
        // agent s updates the grid) and corrected in registers for agent s's clear/set, so no
        // LDS round trip sits on the serial chain; agent s's pickup lookups (cell -> point, point
        // -> target byte, target -> cell) are issued on turns s, s+1, s+2.
        // BIAS (greedy steps, never off the grid): positions carry the lane id in bits 8-15
        // (x | lane << 8 | y << 16), so `q >> 6` is the byte offset of the occupancy word
        // occ[y][lane] (y * 1024 + lane * 4; x < 32) -- one shift per LDS address instead of a
        // field extract and a shift-or.  Equality tests, x-bit selects and the square key's
        // packed minimum are unaffected (every position of a lane carries the same lane bits).
        constexpr bool BIAS = !CLAMP && kBiasAddr && C::NAM <= kBiasMaxNam;
        static_assert(BT * 4 == 1024 && C::D <= 32, "occ[y][lane] = byte y << 10 | lane << 2");
        const uint32_t lbias = BIAS ? ((uint32_t)tid & 255u) << 8 : 0u;
        auto occ_at = [&](uint32_t q) -> uint32_t* {
          if constexpr (BIAS)
            return reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(&L.occ[0][0]) + (q >> 6));
          else
            return &L.occ[q >> 16][tid];
        };
        uint32_t pp[C::NAM], cc[C::NAM];
#pragma unroll
        for (int i = 0; i < C::NAM; ++i) {
          pp[i] = (s.ag[i] & XY16) | lbias;
          cc[i] = CLAMP ? step16<C::D>(pp[i], dstep[i]) : as_u(as_s2(pp[i]) + as_s2(dstep[i]));
        }
        // Predicates are kept in bit 31 of VGPRs (x31 names) and selects are v_bitop3 with
        // 0 / all-ones masks (m names): no VCC round trips on the serial chain.
        //
        // Forbidden moves (core.py:293-297): the reverse of every accepted move, matched as an
        // ordered (from, to) key, and for accepted diagonals the two crossing moves.  A move's
        // square key is the low corner of the 2x2 square it spans plus dx*dy in the top byte
        // (0x01 one diagonal, 0xFF the other, 0 straight or stay); "either crossing move of i" is
        // exactly "same square, opposite diagonal", i.e. square key == i's with the top byte
        // flipped (^ 0xFE000000: 0x01 <-> 0xFF), which no straight move's key (0) ever equals.
        // REV = false drops the reverse keys: a later agent can stand on the cell an accepted move
        // went to only if that cell had been freed by a co-located agent leaving it (the grid was
        // rebuilt from every position, and a move is accepted only into a free cell), so without
        // co-located agents in the lane no reverse key can ever match.  The lazy grid knows the
        // lanes with shared cells (lg->cm, from the last rebuild; new sharing needs an existing
        // one), so a wave with none of them tests the crossing keys only -- one xor per earlier
        // agent, reduced three at a time, instead of two xors and a min3.
        //
        // UKEY: one key per move and ONE test per earlier agent, exact in every lane, so there is a
        // single loop variant.  A unit move p -> c is keyed by its undirected edge or
        // square, u = p + c per coordinate (x and y sums; a stay has both even, an axis move one odd,
        // a diagonal both odd -- and both diagonals of a square share it), and by its direction
        // (dx, dy) bytes: K = dx | dy << 8 | xsum << 16 | ysum << 24.  The moves an accepted move
        // forbids (core.py:293-297) are exactly those with its u and another direction -- its
        // reverse, and for a diagonal the two directions of the other diagonal -- so agent i is
        // blocked iff some stored key S_j has 1 <= (K_i ^ S_j) <= 0xFFFF: one v_xad ((K ^ S) - 1)
        // and half a v_min3 per pair against a cap of 0xFFFF.  An accepted stay adds its own key
        // (p, p) to the reference's set (it can be accepted where a co-located agent left the cell):
        // its stored key has the low bit flipped, so a later stay on that cell lands on 1.  A
        // rejected move stores ~0 (its high bytes never match: sums <= 62).  Same-box A/B against
        // the two-key form below (reverse-key split): 200-step launches Large-16 -10 %, Medium-8
        // -5 % (at Large the split variant made the step loop spill in its common path).
        constexpr bool UKEY = C::NAM >= kUKeyMinNam;
        uint32_t sk[C::NAM];
        auto move_loop = [&](auto rev_tag) {
          constexpr bool REV = decltype(rev_tag)::value;
          if constexpr (HOIST) {   // (an opaque zero keeps LLVM from hoisting it above the branch)
            uint32_t z;
            asm volatile("v_mov_b32 %0, 0" : "=v"(z));
            rblk0 = stream_block(k, gid ^ z, s.epi, t, PUR_REGEN, 0u);
            hoisted = true;
          }
          // raws[s % kOccAhead]: agent s's row word, read kOccAhead turns early (before the
          // updates of agents s - kOccAhead .. s - 1, which the turn applies in registers)
          uint32_t raws[kOccAhead];
#pragma unroll
          for (int j = 0; j < kOccAhead; ++j) raws[j] = j < C::NAM ? *occ_at(cc[j < C::NAM ? j : 0]) : 0u;
          uint32_t mokh[C::NAM];   // accept masks of the agents already moved
#pragma unroll
          for (int sidx = 0; sidx < C::NAM; ++sidx) {
            const uint32_t p = pp[sidx], c = cc[sidx], a = s.ag[sidx];
            // occupied: bit c of the row word, corrected for the clear-then-set of each agent that
            // moved after the word was read, in order
            uint32_t occ31 = (uint32_t)__builtin_amdgcn_sbfe((int)raws[sidx % kOccAhead], c, 1);
#pragma unroll
            for (int j = sidx - kOccAhead; j < sidx; ++j) {
              if (j < 0) continue;
              const uint32_t set31 = (c ^ cc[j]) - 1u;   // bit 31: c == agent j's new cell
              const uint32_t clr31 = (c ^ pp[j]) - 1u;   // bit 31: c == agent j's old cell
              occ31 = bop3<(TA & TB) | (TC & ~(TA & TB))>(mokh[j], set31, bop3<TC & ~(TA & TB)>(mokh[j], clr31, occ31));
            }
            // agent sidx + kOccAhead's word, before this turn's update
            if (sidx + kOccAhead < C::NAM) raws[sidx % kOccAhead] = *occ_at(cc[sidx + kOccAhead < C::NAM ? sidx + kOccAhead : 0]);
            const uint32_t dd = CLAMP ? pk_sub_i16(c, p) : dstep[sidx];
            uint32_t ukey, kpr = 0;
            uint32_t f = 0x7FFFFFFFu;   // unused key slots hold ~0: their xor is never 0
            if constexpr (UKEY) {
              kpr = __builtin_amdgcn_perm(as_u(as_s2(p) + as_s2(c)), dd, 0x06040200u);
              f = 0xFFFFu;
#pragma unroll
              for (int j = 0; j < sidx; ++j) f = min(f, (kpr ^ sk[j]) - 1u);
              f -= 0xFFFEu;   // bit 31 of f - 1 below: blocked (f was < 0xFFFF)
            } else {
              ukey = pk_min_u16(p, c) + (mul_swap(dd) << 24);   // top byte dx*dy: 1, 0xFF, 0
              if constexpr (REV) {
                const uint32_t key = (p & XY16) | ((c & XY16) << 8);
#pragma unroll
                for (int j = 0; j < sidx; ++j) f = min(f, min(rk[j] ^ key, xk[j] ^ ukey));
              } else {
#pragma unroll
                for (int j = 0; j < sidx; ++j) f = min(f, xk[j] ^ ukey);
              }
            }
            const uint32_t live31 = (uint32_t)sidx - n;                 // bit 31: sidx < n
            const uint32_t mok = sgn(bop3<TA & ~TB & ~TC>(live31, occ31, f - 1u));
            atomicAnd(occ_at(p), bop3<~(TA & TB)>(mok, 1u << (p & 31u), 0u));
            atomicOr(occ_at(c), bop3<TA & TB>(mok, 1u << (c & 31u), 0u));
            const uint32_t dxy = c ^ p;
            if constexpr (UKEY) {
              if constexpr (REV) {
                uint32_t z;   // 1 for a stay: v_ffbl of 0 is ~0
                asm("v_ffbl_b32 %0, %1" : "=v"(z) : "v"(dd));
                sk[sidx] = bop3<~TA | (TB ^ TC)>(mok, kpr, z >> 31);
              } else {
                // No lane of the wave has co-located agents: a later agent can then never make the
                // same move p -> c as an accepted one (it would have to stand on p too), so every
                // stored key may carry the flipped low bit a stay's needs -- one op instead of three
                sk[sidx] = bop3<~TA | (TB ^ TC)>(mok, kpr, 1u);
              }
            } else {
              if constexpr (REV) rk[sidx] = bop3<~TA | TB>(mok, (c & XY16) | ((p & XY16) << 8), 0u);
              xk[sidx] = bop3<~TA | (TB ^ TC)>(mok, ukey, 0xFE000000u);
            }
            const uint32_t moved = bop3<TA ^ (TB & TC)>(a, mok, dxy);
            s.ag[sidx] = moved;
            mokh[sidx] = mok;
            constexpr int PD = kPickDist;
            cp[sidx] = L.cell_row(moved);
            if (sidx >= PD) tb[sidx - PD] = *L.row_byte(cp[sidx >= PD ? sidx - PD : 0], tid);
            if (sidx >= 2 * PD) dst[sidx - 2 * PD] = L.dst_tb(tb[sidx >= 2 * PD ? sidx - 2 * PD : 0]);
            if (PICK_IN_LOOP && !(ablate & 8) && sidx >= 3 * PD) {
              const int j = sidx >= 3 * PD ? sidx - 3 * PD : 0;
              pick(j, cp[j], tb[j], dst[j]);
            }
          }
          // pin the hoisted block to this basic block (LLVM would sink it back to its only use)
          if constexpr (HOIST) asm volatile("" : "+v"(rblk0.x), "+v"(rblk0.y), "+v"(rblk0.z), "+v"(rblk0.w));
        };
        // REV: the exact loop for waves with co-located agents (reverse keys in the two-key form; in
        // the one-key form every stay's key flipped), else the loop for waves without any (no reverse
        // keys / every key flipped).  From kRevSplitMaxNam agents on a single (exact) loop.
#ifdef WH_FORCE_NOREV   // timing-only A/B builds: never the reverse-key loop (wrong with co-located agents)
        if (!LAZY)
#else
        if (!LAZY || C::NAM > kRevSplitMaxNam || WH_RARE(__any(lg->cm != 0u)))
#endif
        {
#ifdef WH_COUNT_REV   // A/B builds: count the wave-steps that take the reverse-key loop (wh_check_read)
          if (LAZY && __lane_id() == 0) atomicAdd(&g_wh_revcount[0], 1ull);
#endif
          move_loop(std::true_type{});
        } else {
#ifdef WH_COUNT_REV
          if (__lane_id() == 0) atomicAdd(&g_wh_revcount[1], 1ull);
#endif
          move_loop(std::false_type{});
        }
        // the lookups and decisions the loop's last turns did not reach, in dependency order
        constexpr int PD = kPickDist;
#pragma unroll
        for (int i = (C::NAM > PD ? C::NAM - PD : 0); i < C::NAM; ++i) tb[i] = *L.row_byte(cp[i], tid);
#pragma unroll
        for (int i = (C::NAM > 2 * PD ? C::NAM - 2 * PD : 0); i < C::NAM; ++i) dst[i] = L.dst_tb(tb[i]);
        if (PICK_IN_LOOP && !(ablate & 8)) {
#pragma unroll
          for (int i = (C::NAM > 3 * PD ? C::NAM - 3 * PD : 0); i < C::NAM; ++i) pick(i, cp[i], tb[i], dst[i]);
        }
        looked = true;
        if (LAZY && WH_RARE(__any(lg->cm != 0u))) {   // did an agent that shares a cell move?
          uint32_t acc = 0;
#pragma unroll
          for (int i = 0; i < C::NAM; ++i)
            acc |= (s.ag[i] ^ pp[i]) & (XY16 & (uint32_t)__builtin_amdgcn_sbfe((int)lg->cm, (uint32_t)i, 1u));
          lg->rebuild = lg->rebuild || acc != 0u;
        }
      }
    }

    // ---- pickups: every agent decided against the pre-pickup table, then the table is cleared
    //      (core.py:309-335; two agents on one point both pick it up)
    WH_PHASE_MARK(pickup);
    if (!(ablate & 8)) {
      if (!looked) {
#pragma unroll
        for (int i = 0; i < C::NAM; ++i) cp[i] = L.cell_row(s.ag[i]);
#pragma unroll
        for (int i = 0; i < C::NAM; ++i) tb[i] = *L.row_byte(cp[i], tid);
#pragma unroll
        for (int i = 0; i < C::NAM; ++i) dst[i] = L.dst_tb(tb[i]);
      }
      if (!looked || !PICK_IN_LOOP) {
#pragma unroll
        for (int i = 0; i < C::NAM; ++i) pick(i, cp[i], tb[i], dst[i]);
      }
#pragma unroll
      for (int i = 0; i < C::NAM; ++i) *L.row_byte(clr[i], tid) = 0;
      const uint64_t pr = ((uint64_t)prhi << 32) | prlo;
      s.am &= ~((pr >> 1) | (pr << 63));
    }
  }

  // ---- regeneration: reopen k = R - P + |inactive| points (core.py:338-351)
  WH_PHASE_MARK(regen);
  if (!(ablate & 16)) {
    const uint64_t inactive = ~s.am & low_mask<C::P>();
    const uint32_t nin = (uint32_t)__popcll(inactive);
    // The fused rollout (INJ = false) always auto-resets a finished episode, and a regeneration
    // at its last step (t = T) lands in state the reset replaces: skipped.  (With desynchronised
    // episodes that step's expiry makes it the deepest regeneration of the episode, and the whole
    // wave would walk it for one lane.)
    const int kreq = (!INJ && t >= T) ? 0 : C::R - C::P + (int)nin;
    if (phase == PH_PRE) {
      if (n_inactive) n_inactive[e] = (int32_t)nin;
    } else {
      // 64-bit sets as (lo, hi) halves so that every mask consumer is a v_bitop3
      uint32_t rlo = (uint32_t)inactive, rhi = (uint32_t)(inactive >> 32);   // still selectable
      uint32_t ulo = 0, uhi = 0;                                               // targets used
      uint32_t olo = 0, ohi = 0;                                               // points opened
      uint32_t tj[3] = {0u, 0u, 0u};   // targets of items 0-2 (kRegenSkip)
      uint32_t first_t = 0;
      const uint32_t wexp = ((t + W) & 0xFFu) << 8;   // expires at step t + W
      uint4 blk = make_uint4(0u, 0u, 0u, 0u);   // words 2j (pickup) and 2j+1 (target) share a block
#pragma unroll
      for (int j = 0; j < C::R; ++j) {
        // wave-uniform: once no env needs item j, none needs a later one -- leave the loop (one
        // branch test per executed item + 1, instead of one per item)
        if (!__any(j < kreq)) break;
        {
          uint32_t ma = sgn((uint32_t)j - (uint32_t)kreq);   // j < kreq
          uint32_t sel, tgi;
          if (INJ && regen) {
            const uint32_t rpos = (uint32_t)regen[e * 2 * C::R + j];
            tgi = (uint32_t)regen[e * 2 * C::R + C::R + j];
            const bool valid = rpos < nin && tgi < (uint32_t)C::DP;   // invalid draws are ignored
            ma = bop3<TA & TB>(ma, 0u - (uint32_t)valid, 0u);
            sel = select_bit64(inactive, rpos);   // positions into the inactive list, host-drawn
          } else {
            if ((j & 1) == 0) blk = ((HOIST || kHoistPolicy) && j == 0 && hoisted) ? rblk0 : stream_block(k, gid, s.epi, t, PUR_REGEN, (uint32_t)(j >> 1));
            const uint32_t w1 = comp(blk, (2 * j) & 3), w2 = comp(blk, (2 * j + 1) & 3);
            sel = select_bit64(((uint64_t)rhi << 32) | rlo, __umulhi(w1, nin - (uint32_t)j));
            const uint32_t r2 = __umulhi(w2, (uint32_t)(C::DP - j));
            if (j == 0) tgi = r2;                                               // nothing used yet
            else if (j == 1) tgi = r2 + ((first_t - 1u - r2) >> 31);   // + (r2 >= first): skip it
            else if (kRegenSkip && j == 2) {
              // the r2-th target not used by items 0 and 1: skip each of them at or below it, in
              // ascending order (the same value as the rank selection on the used mask)
              const uint32_t lo = min(tj[0], tj[1]), hi = max(tj[0], tj[1]);
              tgi = r2 + ((lo - 1u - r2) >> 31);
              tgi += (hi - 1u - tgi) >> 31;
            } else {
              if (kRegenSkip && j == 3) {   // from item 3 on: the used mask, built from items 0-2
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                  const uint64_t b = 1ull << (tj[q] & 63u);
                  ulo |= (uint32_t)b;
                  uhi |= (uint32_t)(b >> 32);
                }
              }
              tgi = select_bit64(~(((uint64_t)uhi << 32) | ulo) & low_mask<C::DP>(), r2);
            }
            if (j == 0) first_t = r2;
            if (j < 3) tj[j] = tgi;
          }
          const uint64_t sb = 1ull << (sel & 63u), tb64 = 1ull << (tgi & 63u);
          const uint32_t slo = bop3<TA & TB>(ma, (uint32_t)sb, 0u), shi = bop3<TA & TB>(ma, (uint32_t)(sb >> 32), 0u);
          rlo &= ~slo;
          rhi &= ~shi;
          olo |= slo;
          ohi |= shi;
          if (!kRegenSkip || j >= 3) {   // (kRegenSkip: items 0-2 skip their targets arithmetically)
            ulo = bop3<(TA & TB) | TC>(ma, (uint32_t)tb64, ulo);
            uhi = bop3<(TA & TB) | TC>(ma, (uint32_t)(tb64 >> 32), uhi);
          }
          // predicated store: lanes with nothing to open write the scratch row
          L.pkp[msel(ma, sel, (uint32_t)C::P)][tid] = (uint16_t)((tgi + 1u) | wexp);
        }
      }
      const uint64_t opened = ((uint64_t)ohi << 32) | olo;
      s.am |= opened;
    }
  }

  bool done = false;
  if (phase != PH_REGEN) {
    // ---- deliveries (core.py:354-368): target cell == position (idle agents never match)
    WH_PHASE_MARK(deliver);
    // Manhattan distance position -> target cell minus 1 is ONE v_sad_u8 of the agent word against
    // its target bytes doubled ([x, dx, y, dy] vs [dx, dx, dy, dy], accumulator -1): negative exactly
    // when the agent stands on its target (an idle agent's 0xFF bytes never match).  The reward of
    // the pickup or the delivery is folded into the same bitop3 that makes the 1.0f.
    uint32_t delm[C::NAM];
#pragma unroll
    for (int i = 0; i < C::NAM; ++i) delm[i] = 0u;
    if (!(ablate & 32)) {
#pragma unroll
      for (int i = 0; i < C::NAM; ++i) {
        const uint32_t a = s.ag[i];
        const uint32_t m = sgn(__builtin_amdgcn_sad_u8(a, __builtin_amdgcn_perm(a, a, 0x03030101u), 0xFFFFFFFFu));
        s.ag[i] = bop3<(TA & TB) | TC>(m, IDLE, a);
        delm[i] = m;   // a pickup (interior cell) and a delivery (border cell) never share a step
      }
    }
#pragma unroll
    for (int i = 0; i < C::NAM; ++i) rew[i] = __uint_as_float(bop3<(TA | TB) & TC>(rewm[i], delm[i], 0x3F800000u));
    WH_PHASE_MARK(tail);
    done = t >= T;                                            // core.py:438
    s.hdr = t | (n << 16);                                    // clears `fresh`
  }
  return done;
}

// Image offset of output value f of agent row i (sorted-key order, see wh_observe).
// Image layout: [0] n, [A0 + r] availability of agent r, [G0 + 2r] its delivery target (x, y),
// [P0 + 2r] its position (x, y), [Q0 + 4q] request q (pickup x, y, delivery x, y); k_observe's
// byte image packs the sections back to back (the defaults).
template <int R, int A0 = 1, int G0 = 1 + R, int P0 = 1 + 3 * R, int Q0 = 1 + 5 * R>
__host__ __device__ constexpr uint32_t obs_src(int i, int f, bool fresh) {
  if (f == 0) return 0;                                                    // num_agents
  if (f < R) {                                                             // other_availabilities
    const int j = f - 1;
    return A0 + (j < i ? j : j + 1);
  }
  if (f < 3 * R - 2) {                                                     // other_delivery_targets
    const int k = f - R, j = k >> 1, drop = fresh ? i : 1;
    return G0 + 2 * (j < drop ? j : j + 1) + (k & 1);
  }
  if (f < 5 * R - 4) {                                                     // other_positions
    const int k = f - (3 * R - 2), j = k >> 1;
    return P0 + 2 * (j < i ? j : j + 1) + (k & 1);
  }
  if (f < 9 * R - 4) return Q0 + (f - (5 * R - 4));                        // requests
  if (f == 9 * R - 4) return A0 + i;                                       // self_availability
  if (f < 9 * R - 1) return G0 + 2 * i + (f - (9 * R - 3));                // self_delivery_target
  return P0 + 2 * i + (f - (9 * R - 1));                                   // self_position
}

// ----------------------------------------------------------------------------- kernels
// rewards[B, na]: a wave's 64 envs own one contiguous block of 64*na floats.  Even agent counts
// store each lane's row with 16/8-byte stores; otherwise lanes write their rows into LDS (the agl
// scratch, free after the move phase) and read the block back so every global store instruction
// writes contiguous 16-byte lanes instead of one strided row per lane.
template <class C>
__device__ __forceinline__ void store_rewards(Lds<C>& L, const float (&rew)[C::NAM], float* out,
                                              int64_t B, int64_t e, int na, int tid, bool direct) {
  if ((C::NAM & 1) == 0 && na == C::NAM && (reinterpret_cast<uintptr_t>(out) & 15u) == 0) {
    // One row of 16-byte (8-byte) stores per lane: the two wave-instructions of a Medium-8 step
    // cover the wave's contiguous 2 KiB block between them (A/B: 5 % faster than the LDS transpose
    // below, whose row writes are 8-way bank conflicts).
    if ((C::NAM & 3) == 0) {
      float4* row = reinterpret_cast<float4*>(out + e * na);
#pragma unroll
      for (int q = 0; q < C::NAM / 4; ++q)
        row[q] = make_float4(rew[4 * q], rew[4 * q + 1], rew[4 * q + 2], rew[4 * q + 3]);
    } else {
      float2* row = reinterpret_cast<float2*>(out + e * na);
#pragma unroll
      for (int q = 0; q < C::NAM / 2; ++q) row[q] = make_float2(rew[2 * q], rew[2 * q + 1]);
    }
    return;
  }
  const int lane = tid & 63;
  const int64_t e0 = e - lane;
  // tail wave (lanes past B have exited) or masked step (unstepped lanes have exited): no
  // transpose -- one row per lane
  if (direct || B - e0 < 64) {
    float* row = out + e * na;
#pragma unroll
    for (int i = 0; i < C::NAM; ++i)
      if (i < na) row[i] = rew[i];
    return;
  }
  // Staging element k of this wave's 64*na floats lives at agl[k / 64][wave base + k % 64]: inside
  // the wave's own columns, so no other wave's agent words (ordered path) are overwritten.
  const int wbase = tid & ~63;
  auto stg = [&](int k) -> float* { return reinterpret_cast<float*>(&L.agl[k >> 6][wbase + (k & 63)]); };
#pragma unroll
  for (int i = 0; i < C::NAM; ++i)
    if (i < na) *stg(lane * na + i) = rew[i];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int nvalid = 64 * na;
  float* wout = out + e0 * na;
  if ((reinterpret_cast<uintptr_t>(wout) & 15u) == 0 && (na & 3) == 0) {
#pragma unroll
    for (int q = 0; q < C::NAM / 4; ++q)
      if (4 * q < na)   // 4 consecutive k (k % 4 == 0) sit in one row, 16-byte aligned
        reinterpret_cast<float4*>(wout)[lane + 64 * q] = *reinterpret_cast<const float4*>(stg(4 * (lane + 64 * q)));
  } else {
#pragma unroll
    for (int q = 0; q < C::NAM; ++q)
      if (lane + 64 * q < nvalid) wout[lane + 64 * q] = *stg(lane + 64 * q);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// ----------------------------------------------------------------------------- assert mode
// -DWH_CHECK builds verify SURVEY §5's invariants in the kernel after the state load and after
// every step (and auto-reset): exactly R open requests (core.py:210-221 opens R, core.py:338-351
// refills to R), every live agent inside the grid, every carried target a delivery cell
// (core.py:177-188), every request byte a valid delivery index, the open-request mask equal to the
// table, n <= agent slots.  Violations are counted in g_wh_check (read by wh_check_read): [0]
// violations, [1] first failing env id, [2] its bit mask of failed checks, [3] env-states checked.
#ifdef WH_CHECK
__device__ unsigned long long g_wh_check[4];

template <class C>
__device__ __forceinline__ void check_env(const Regs<C>& s, const Lds<C>& L, int64_t e, int tid) {
  const uint32_t n = (s.hdr >> 16) & 0xFFu;
  uint32_t code = 0;
  if (n > (uint32_t)C::NAM) code |= 1u;
  if (__popcll(s.am) != C::R) code |= 2u;
#pragma unroll
  for (int i = 0; i < C::NAM; ++i) {
    if ((uint32_t)i >= n) continue;
    const uint32_t a = s.ag[i];
    const uint32_t x = a & 0xFFu, y = (a >> 16) & 0xFFu, dx = (a >> 8) & 0xFFu, dy = a >> 24;
    if (x >= (uint32_t)C::D || y >= (uint32_t)C::D) code |= 4u;
    if ((dx == 0xFFu) != (dy == 0xFFu)) code |= 8u;
    if (dx != 0xFFu) {
      const bool xb = dx == 0u || dx == (uint32_t)(C::D - 1), yb = dy == 0u || dy == (uint32_t)(C::D - 1);
      const bool ok = (xb && !yb && dy >= 2u && dy <= (uint32_t)(C::D - 3)) ||
                      (yb && !xb && dx >= 2u && dx <= (uint32_t)(C::D - 3));
      if (!ok) code |= 8u;
    }
  }
#pragma unroll
  for (int j = 0; j < C::P; ++j) {
    const uint32_t tb = L.pkp[j][tid] & 0xFFu;
    if ((tb != 0u) != (((s.am >> j) & 1ull) != 0ull)) code |= 16u;
    if (tb > (uint32_t)C::DP) code |= 32u;
  }
  if (code) {
    if (atomicAdd(&g_wh_check[0], 1ull) == 0ull) {
      g_wh_check[1] = (unsigned long long)e;
      g_wh_check[2] = code;
    }
  }
}
#define WH_CHECK_ENV(s, L, e, tid) check_env<C>(s, L, e, tid)
#else
#define WH_CHECK_ENV(s, L, e, tid) ((void)0)
#endif

struct StepParams {
  uint32_t* state;
  int64_t B;
  int32_t na, T, W;
  const uint32_t* tables;
  const int32_t* actions;
  const int32_t* order;
  int32_t ol;               // order row length (1 .. 4 * NA; resolve_step turns 0 into NA)
  float* rewards;
  uint8_t* dones;
  float* returns;
  const int32_t* regen;
  int32_t* n_inactive;
  int32_t* actions_out;
  float p;
  uint32_t k0, k1;
  int64_t env_offset;
  int32_t steps, phase, autoreset, variable_n;
  int32_t ablate;  // timing-only phase skips (env WH_ABLATE), never set in normal use
  wh_episode_stats stats;   // all-NULL = off
  const uint8_t* mask;      // [B] or NULL: envs to step (wh_vector_step)
  uint32_t* state_out;      // NULL: in place; else the state is read from `state`, written here
                            // (wh_sampler_step_to: double-buffered, no mask)
};

// Folds the episodes this wave finished into the per-n bins of wh_episode_stats (the
// on_episode_end metrics of scripts/train.py:18-23): one set of global atomics per distinct n in
// the wave.  Sums, minima and maxima are built from ballots over bit slices, so only active lanes
// contribute and the integer results do not depend on lane or wave order.
__device__ __forceinline__ void flush_episodes(bool fin, uint32_t n, uint32_t ret, const wh_episode_stats& st) {
  uint64_t pend = __ballot(fin);
  while (pend) {
    const int leader = __ffsll((unsigned long long)pend) - 1;
    const uint32_t nb = (uint32_t)__shfl((int)n, leader);
    const bool g = fin && n == nb;
    const uint64_t gm = __ballot(g);
    pend &= ~gm;
    uint64_t sum = 0;
    uint32_t mn = 0, mx = 0;
    bool cmin = g, cmax = g;
    for (int b = 31; b >= 0; --b) {
      const bool bit = (ret >> b) & 1u;
      sum += (uint64_t)__popcll(__ballot(g && bit)) << b;
      if (__ballot(cmax && bit)) { mx |= 1u << b; cmax = cmax && bit; }
      if (__ballot(cmin && !bit)) cmin = cmin && !bit;
      else mn |= 1u << b;
    }
    if ((int)__lane_id() == leader) {
      if (st.return_sum) atomicAdd(&st.return_sum[nb], (unsigned long long)sum);
      if (st.episodes) atomicAdd(&st.episodes[nb], (unsigned long long)__popcll(gm));
      if (st.return_min) atomicMin(&st.return_min[nb], mn);
      if (st.return_max) atomicMax(&st.return_max[nb], mx);
    }
  }
}

// The step loop of k_step.  PHASE >= 0 fixes the phase at compile time (the fused rollout and the
// sampler path run PH_ALL), so the phase tests fold away and each step is a few large basic blocks
// the scheduler can interleave; -1 reads it from the launch (the drop-in's split step).  Phase
// ablation (tools/ablate.py) exists only in builds with -DWH_ABLATION.
template <class C, int POLICY, bool ORDERED, int PHASE>
__device__ __forceinline__ void run_steps(const StepParams& a, Regs<C>& s, Lds<C>& L, const Keys& k,
                                          uint32_t gid, int64_t e, int tid, uint16_t* okeys = nullptr) {
  const int phase = PHASE >= 0 ? PHASE : a.phase;
  const OrderIn oi{a.order, a.ol, okeys};
#ifdef WH_ABLATION
  const int ablate = a.ablate;
#else
  constexpr int ablate = 0;
#endif
  float ret = 0.0f;
  const bool stats = a.stats.episode_return != nullptr;
  uint32_t epr = stats ? a.stats.episode_return[e] : 0u;
  for (int stp = 0; stp < a.steps; ++stp) {
    uint32_t d[C::NAM];
    if (POLICY == POL_EXTERNAL) {
      const bool have = phase != PH_REGEN && !ORDERED;   // REGEN reads no actions
#pragma unroll
      for (int i = 0; i < C::NAM; ++i) {
        uint32_t mv = (have && i < a.na) ? (uint32_t)a.actions[e * a.na + i] : 4u;
        d[i] = L.mv(mv > 8u ? 4u : mv);
      }
    } else if (ablate & 1) {
#pragma unroll
      for (int i = 0; i < C::NAM; ++i) d[i] = L.mv((uint32_t)((i + stp) % 9));
    } else {
      policy_steps<C, POLICY, POLICY == POL_GREEDY && !kAblationBuild>(s, L, k, gid, a.p, d);
    }
    float rew[C::NAM];
    const bool done = step_env<C, ORDERED, true, POLICY != POL_GREEDY || kAblationBuild>(s, L, d, oi, a.actions, a.regen, k, gid, e, a.na, phase,
                                  (uint32_t)a.T, (uint32_t)a.W, rew, a.n_inactive, tid, ablate);
    if (phase != PH_REGEN) {
      if (a.rewards && !(ablate & 64))
        store_rewards<C>(L, rew, a.rewards + (int64_t)stp * a.B * a.na, a.B, e, a.na, tid, a.mask != nullptr);
      if (a.dones && !(ablate & 64)) a.dones[(int64_t)stp * a.B + e] = done ? 1 : 0;
      if (a.returns) {
#pragma unroll
        for (int i = 0; i < C::NAM; ++i) ret += rew[i];
      }
      if (stats) {
        float r = 0.0f;
#pragma unroll
        for (int i = 0; i < C::NAM; ++i) r += rew[i];   // whole numbers: exact
        epr += (uint32_t)r;
        if (__any(done)) flush_episodes(done, (s.hdr >> 16) & 0xFFu, epr, a.stats);
        if (done) epr = 0;
      }
      if (done && a.autoreset && !(ablate & 128)) {
        reset_philox<C>(s, L, k, gid, a.na, a.variable_n, (uint32_t)a.W, tid);
#pragma unroll
        for (int y = 0; y < C::D; ++y) L.occ[y][tid] = 0u;
      }
    }
    if (phase != PH_PRE) WH_CHECK_ENV(s, L, e, tid);
  }
  if (a.returns) a.returns[e] += ret;
  if (stats) a.stats.episode_return[e] = epr;
}

// The fused rollout's common case as its own instance: wh_rollout with rewards + dones written,
// auto-reset on, no returns / episode stats / env mask, na == NAM with NAM even (16/8-byte reward
// rows).  No per-step tests of launch options, and the injected-draw path is compiled out, so a
// step executes few branch instructions -- each costs several issue slots at one wave per SIMD
// (tools/oprate5.hip: ~8 ns per s_cbranch/s_branch against ~2.6 ns per VALU op).
#ifndef WH_EAGER_GRID   // (A/B builds: -DWH_EAGER_GRID rebuilds the grid every step)
constexpr bool kLazyGrid = true;
#else
constexpr bool kLazyGrid = false;
#endif

// Lanes of a wave ending their episodes in the same step that are reset one at a time from their
// reset slots (~40 issue slots each); more than this take the all-lane reset_philox (~700 VALU).
constexpr int kSlotResetMax = 8;
// A fill costs about two single-lane resets and a launch of K desynchronised steps ends ~K/3 episodes
// per wave (Medium-8), so launches shorter than this reset single lanes from scratch (reset_lane).
constexpr int kSlotMinSteps = 8;

template <class C>
__device__ __forceinline__ void store_row(float* row, const float (&rew)[C::NAM]) {
  if constexpr ((C::NAM & 3) == 0) {
#pragma unroll
    for (int q = 0; q < C::NAM / 4; ++q)
      reinterpret_cast<float4*>(row)[q] = make_float4(rew[4 * q], rew[4 * q + 1], rew[4 * q + 2], rew[4 * q + 3]);
  } else {
#pragma unroll
    for (int q = 0; q < C::NAM / 2; ++q) reinterpret_cast<float2*>(row)[q] = make_float2(rew[2 * q], rew[2 * q + 1]);
  }
}

// One step of the fused rollout's common case at a time (run_steps_fast loops over it; k_sampler
// interleaves it with writing observation rows).  Carries the lazy grid and the output rows.
// SLOTS = false: no reset slots -- a lone ending lane is reset by reset_lane, as launches shorter
// than kSlotMinSteps do.
template <class C, int POLICY, bool SLOTS = true>
struct FastRun {
  float* rrow;
  uint8_t* drow;
  int64_t rstride;
  LazyGrid lg;
  uint32_t act[POLICY == POL_EXTERNAL ? C::NAM : 1];   // external actions of the (single) step
  __device__ __forceinline__ FastRun(const StepParams& a, int64_t e)
      : rrow(a.rewards + e * C::NAM), drow(a.dones + e), rstride(a.B * C::NAM), lg{true, 0u} {}   // the grid starts empty (k_step)
  // POL_EXTERNAL: the step's actions, loaded with the state in the prologue (their HBM latency then
  // overlaps the table loads instead of sitting on the first step)
  __device__ __forceinline__ void load_actions(const StepParams& a, int64_t e) {
    if constexpr (POLICY == POL_EXTERNAL) {
      if constexpr (C::NAM % 4 == 0) {
        const uint4* src = reinterpret_cast<const uint4*>(a.actions + e * C::NAM);
#pragma unroll
        for (int q = 0; q < C::NAM / 4; ++q) {
          const uint4 v = src[q];
          act[4 * q] = v.x; act[4 * q + 1] = v.y; act[4 * q + 2] = v.z; act[4 * q + 3] = v.w;
        }
      } else {
        const uint2* src = reinterpret_cast<const uint2*>(a.actions + e * C::NAM);
#pragma unroll
        for (int q = 0; q < C::NAM / 2; ++q) {
          const uint2 v = src[q];
          act[2 * q] = v.x; act[2 * q + 1] = v.y;
        }
      }
    }
  }

  __device__ __forceinline__ void step(const StepParams& a, Regs<C>& s, Lds<C>& L, Slots<C>* RS, const Keys& k,
                                       uint32_t gid, int64_t e, int tid, int stp) {
#ifdef WH_ABLATION
    const int ablate = a.ablate;
#else
    constexpr int ablate = 0;
#endif
    uint32_t d[C::NAM];
    if constexpr (POLICY == POL_EXTERNAL) {
#pragma unroll
      for (int i = 0; i < C::NAM; ++i) d[i] = L.mv(act[i] > 8u ? 4u : act[i]);   // MOVES[a]; others stay
    } else if (ablate & 1) {
#pragma unroll
      for (int i = 0; i < C::NAM; ++i) d[i] = L.mv((uint32_t)((i + stp) % 9));
    } else {
      policy_steps<C, POLICY, POLICY == POL_GREEDY && !kAblationBuild>(s, L, k, gid, a.p, d);
    }
    float rew[C::NAM];
    const bool done = step_env<C, false, false, POLICY != POL_GREEDY || kAblationBuild, kLazyGrid>(s, L, d, OrderIn{nullptr, 0, nullptr}, nullptr, nullptr, k, gid, e, C::NAM, PH_ALL,
                                                (uint32_t)a.T, (uint32_t)a.W, rew, nullptr, tid, ablate, &lg);
    if (!(ablate & 64)) {
      store_row<C>(rrow, rew);
      *drow = done ? 1 : 0;
    }
    rrow += rstride;
    drow += a.B;
    if (!(ablate & 128) && WH_RARE(__any(done))) {   // wave-uniform test first: one branch on the common path
      const uint64_t dm = __ballot(done);
      // a few envs of a full wave end (desynchronised episodes): wave-wide resets of them, one env
      // at a time (every lane takes part, so not in a tail wave whose lanes past B have exited)
      const bool full = __ballot(true) == ~0ull;
#ifndef WH_NO_RESET_SLOTS   // (A/B builds: -DWH_NO_RESET_SLOTS resets one lane from scratch)
      if (SLOTS && a.steps >= kSlotMinSteps && __popcll(dm) <= kSlotResetMax && full) {
        // their precomputed next-episode states, after (re)filling the wave's slots if one of
        // theirs is stale: one wave-wide fill (every lane's next episode) serves the resets of
        // the lanes that end later in this launch
        if constexpr (SLOTS) {
          if (__any(done && RS->rs_ep[tid] != s.epi + 1u))
            reset_philox<C, C::NAM, true>(s, L, k, gid, C::NAM, a.variable_n, (uint32_t)a.W, tid, RS);
          for (uint64_t m = dm; m; m &= m - 1ull) reset_from_slot<C, C::NAM>(s, L, *RS, (uint32_t)a.W, tid, __builtin_ctzll(m));
          lg.rebuild = lg.rebuild || done;   // their grid columns were cleared
        }
      } else
#endif
      if (__popcll(dm) == 1 && full) {
        // short launches (the sampler's 1-step ones): a fill would serve few later resets
        reset_lane<C, C::NAM>(s, L, k, gid, a.variable_n, (uint32_t)a.W, tid, __builtin_ctzll(dm));
        lg.rebuild = lg.rebuild || done;   // its grid column was cleared
      } else if (dm == ~0ull) {
        // every lane of the wave (synchronised episodes): the grid and pickup plane cleared wave-wide
        reset_philox<C, C::NAM, false, true>(s, L, k, gid, C::NAM, a.variable_n, (uint32_t)a.W, tid);
        lg.rebuild = true;
      } else if (done) {
        reset_philox<C, C::NAM>(s, L, k, gid, C::NAM, a.variable_n, (uint32_t)a.W, tid);
#pragma unroll
        for (int y = 0; y < C::D; ++y) L.occ[y][tid] = 0u;
        lg.rebuild = true;
      }
    }
    WH_CHECK_ENV(s, L, e, tid);
  }
};

// k_step's fused rollout loop: FastRun's step, written out as one loop (the same body as a member
// call measured 2 % slower per step at Medium-8: profiles/r04_fastrun_ab.txt).
template <class C, int POLICY, bool SLOTS = true>
__device__ __forceinline__ void run_steps_fast(const StepParams& a, Regs<C>& s, Lds<C>& L, Slots<C>* RS,
                                               const Keys& k, uint32_t gid, int64_t e, int tid) {
#ifdef WH_ABLATION
  const int ablate = a.ablate;
#else
  constexpr int ablate = 0;
#endif
  // output rows of step stp: wave-uniform bases (scalar adds per step) + the lane's offset
  float* rrow = a.rewards + (e - tid) * C::NAM;
  uint8_t* drow = a.dones + (e - tid);
  const int64_t rstride = a.B * C::NAM;
  LazyGrid lg{true, 0u};   // the grid starts empty (k_step)
  for (int stp = 0; stp < a.steps; ++stp) {
    uint32_t d[C::NAM];
    if constexpr (POLICY == POL_EXTERNAL) {   // (wh_vector_step's fast case: one step)
#pragma unroll
      for (int i = 0; i < C::NAM; ++i) {
        const uint32_t mv = (uint32_t)a.actions[e * C::NAM + i];
        d[i] = L.mv(mv > 8u ? 4u : mv);
      }
    } else if (ablate & 1) {
#pragma unroll
      for (int i = 0; i < C::NAM; ++i) d[i] = L.mv((uint32_t)((i + stp) % 9));
    } else {
      policy_steps<C, POLICY, POLICY == POL_GREEDY && !kAblationBuild>(s, L, k, gid, a.p, d);
    }
    uint4 rb = make_uint4(0u, 0u, 0u, 0u);
    if constexpr (kHoistPolicy) {   // pinned to the policy's block (LLVM would sink it to its use)
      rb = stream_block(k, gid, s.epi, (s.hdr + 1u) & 0xFFFFu, PUR_REGEN, 0u);
      asm volatile("" : "+v"(rb.x), "+v"(rb.y), "+v"(rb.z), "+v"(rb.w));
    }
    float rew[C::NAM];
    const bool done = step_env<C, false, false, POLICY != POL_GREEDY || kAblationBuild, kLazyGrid>(s, L, d, OrderIn{nullptr, 0, nullptr}, nullptr, nullptr, k, gid, e, C::NAM, PH_ALL,
                                                (uint32_t)a.T, (uint32_t)a.W, rew, nullptr, tid, ablate, &lg,
                                                kHoistPolicy ? &rb : nullptr);
    if (!(ablate & 64)) {
      store_row<C>(rrow + tid * C::NAM, rew);
      drow[tid] = done ? 1 : 0;
    }
    rrow += rstride;
    drow += a.B;
    if (!(ablate & 128) && WH_RARE(__any(done))) {   // wave-uniform test first: one branch on the common path
      const uint64_t dm = __ballot(done);
      // a few envs of a full wave end (desynchronised episodes): wave-wide resets of them, one env
      // at a time (every lane takes part, so not in a tail wave whose lanes past B have exited)
      const bool full = __ballot(true) == ~0ull;
#ifndef WH_NO_RESET_SLOTS   // (A/B builds: -DWH_NO_RESET_SLOTS resets one lane from scratch)
      if (SLOTS && a.steps >= kSlotMinSteps && __popcll(dm) <= kSlotResetMax && full) {
        // their precomputed next-episode states, after (re)filling the wave's slots if one of
        // theirs is stale: one wave-wide fill (every lane's next episode) serves the resets of
        // the lanes that end later in this launch
        if constexpr (SLOTS) {
          if (__any(done && RS->rs_ep[tid] != s.epi + 1u))
            reset_philox<C, C::NAM, true>(s, L, k, gid, C::NAM, a.variable_n, (uint32_t)a.W, tid, RS);
          for (uint64_t m = dm; m; m &= m - 1ull) reset_from_slot<C, C::NAM>(s, L, *RS, (uint32_t)a.W, tid, __builtin_ctzll(m));
          lg.rebuild = lg.rebuild || done;   // their grid columns were cleared
        }
      } else
#endif
      if (__popcll(dm) == 1 && full) {
        // short launches (the sampler's 1-step ones): a fill would serve few later resets
        reset_lane<C, C::NAM>(s, L, k, gid, a.variable_n, (uint32_t)a.W, tid, __builtin_ctzll(dm));
        lg.rebuild = lg.rebuild || done;   // its grid column was cleared
      } else if (dm == ~0ull) {
        // every lane of the wave (synchronised episodes): the grid and pickup plane cleared wave-wide
        reset_philox<C, C::NAM, false, true>(s, L, k, gid, C::NAM, a.variable_n, (uint32_t)a.W, tid);
        lg.rebuild = true;
      } else if (done) {
        reset_philox<C, C::NAM>(s, L, k, gid, C::NAM, a.variable_n, (uint32_t)a.W, tid);
#pragma unroll
        for (int y = 0; y < C::D; ++y) L.occ[y][tid] = 0u;
        lg.rebuild = true;
      }
    }
    WH_CHECK_ENV(s, L, e, tid);
  }
}


// -DWH_TIMING builds (tools/launch_timeline.py): per-wave s_memrealtime stamps (100 MHz) of the fused
// rollout's phases -- entry, tables in LDS, state loaded, step loop done, state stored -- read back
// with wh_debug_times.  Written by lane 0 of each wave with vector stores.
#ifdef WH_TIMING
constexpr int kTimeSlots = 6, kTimeWaves = 4096;
__device__ unsigned long long g_wh_times[kTimeWaves * kTimeSlots];
#define WH_T(i)                                                                                   \
  do {                                                                                            \
    const unsigned long long now_ = __builtin_amdgcn_s_memrealtime();                             \
    const int w_ = (int)blockIdx.x * (BT / 64) + (int)(threadIdx.x >> 6);                        \
    if ((threadIdx.x & 63) == 0 && w_ < kTimeWaves) g_wh_times[w_ * kTimeSlots + (i)] = now_;     \
  } while (0)
#else
#define WH_T(i) ((void)0)
#endif

template <class C, int POLICY, bool ORDERED, bool FAST>
__global__ __launch_bounds__(BT) void k_step(StepParams a) {
  __shared__ Lds<C> L;
  __shared__ std::conditional_t<FAST, Slots<C>, NoSlots> RS;   // reset slots: fused rollout only
  __shared__ std::conditional_t<ORDERED, OKeys<C>, NoSlots> OK;   // dict-order move keys: ORDERED only
  const int tid = threadIdx.x;
  if (FAST) WH_T(0);
  const int64_t e = (int64_t)blockIdx.x * BT + tid;
  const bool live = e < a.B && (FAST || !a.mask || a.mask[e]);
  const int na = FAST ? C::NAM : a.na;   // the fast instance runs na == NAM only (resolve_step)
  const int64_t e0 = (int64_t)blockIdx.x * BT;
  // Prologue: the table loads (L2) first, then the state planes (HBM); the table is written to LDS
  // and the occupancy grid cleared while the state is still in flight, and the pickup plane is
  // built as the state words land (the waitcnt pass counts each use against the in-order vmcnt).
  const uint4 tv0 = issue_table_chunk<C>(a.tables, 0), tv1 = issue_table_chunk<C>(a.tables, 1);
  __builtin_amdgcn_sched_barrier(0);   // keep the table loads ahead of the state loads
  // every lane loads (a lane past B or masked out re-reads env e0, which exists): a load under an exec
  // branch would make the waitcnt pass drain the state loads before the table's LDS writes
  RawEnv<C> raw;
  load_env_issue<C>(raw, a.state, a.B, e0, live ? tid : 0, na);
  commit_table_chunk<C>(L.tbl, 0, tv0);
  commit_table_chunk<C>(L.tbl, 1, tv1);
#pragma unroll
  for (int y = 0; y < C::D; ++y) L.occ[y][tid] = 0u;   // occupancy grid starts empty (step_env)
  __syncthreads();
  if (FAST) WH_T(1);
  if (!live) return;
  const Keys k{a.k0, a.k1};
  const uint32_t gid = (uint32_t)(a.env_offset + e);
  Regs<C> s;
  load_env_finish<C>(s, L, raw, (uint32_t)a.W, tid);
#ifdef WH_CHECK
  if (a.phase != PH_REGEN) WH_CHECK_ENV(s, L, e, tid);   // (a REGEN launch continues a PRE one)
  atomicAdd(&g_wh_check[3], (unsigned long long)a.steps + 1ull);
#endif
  // Drain the state loads here.  Their first uses are inside the step loop, so otherwise the
  // waitcnt pass places vmcnt waits in the loop body, where on every later iteration they also
  // wait for the previous step's reward/done stores to retire (a full memory round trip per step).
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0), expcnt/lgkmcnt untouched (gfx9 encoding)
  if constexpr (FAST) RS.rs_ep[tid] = s.epi;            // reset slots start stale (!= epi + 1)
  if (FAST) WH_T(2);

  if (!FAST && a.phase == PH_POLICY) {
    uint32_t d[C::NAM];
    policy_steps<C, POLICY>(s, L, k, gid, a.p, d);
    const uint32_t n = (s.hdr >> 16) & 0xFFu;
#pragma unroll
    for (int i = 0; i < C::NAM; ++i)
      if (i < a.na) a.actions_out[e * a.na + i] = (i < (int)n) ? (int32_t)action_of(d[i]) : 4;
    return;
  }

  if constexpr (FAST)
    run_steps_fast<C, POLICY>(a, s, L, &RS, k, gid, e, tid);
  else if (!ORDERED && a.phase == PH_ALL)
    run_steps<C, POLICY, ORDERED, PH_ALL>(a, s, L, k, gid, e, tid);
  else if constexpr (ORDERED)
    run_steps<C, POLICY, ORDERED, -1>(a, s, L, k, gid, e, tid, &OK.k[0][0]);
  else
    run_steps<C, POLICY, ORDERED, -1>(a, s, L, k, gid, e, tid);
  if (FAST) WH_T(3);
  store_env<C>(s, L, a.state_out ? a.state_out : a.state, a.B, e0, na, tid);
#ifdef WH_TIMING
  if (FAST) {
    __builtin_amdgcn_s_waitcnt(0);   // the state stores have left the wave
    WH_T(4);
  }
#endif
}

struct ResetParams {
  uint32_t* state;
  int64_t B;
  int32_t na, W;
  const uint32_t* tables;
  const uint8_t* mask;
  const int32_t *spawn, *pickups, *targets, *n;
  int32_t injected, variable_n;
  uint32_t k0, k1;
  int64_t env_offset;
};

template <class C>
__global__ __launch_bounds__(BT) void k_reset(ResetParams a) {
  __shared__ Lds<C> L;
  load_tables<C>(L.tbl, a.tables);
  __syncthreads();
  const int tid = threadIdx.x;
  const int64_t e = (int64_t)blockIdx.x * BT + tid;
  if (e >= a.B) return;
  if (a.mask && !a.mask[e]) return;
  Regs<C> s;
  s.epi = a.state[a.B + e];
  if (a.injected)
    reset_injected<C>(s, L, e, a.na, a.spawn, a.pickups, a.targets, a.n, (uint32_t)a.W, tid);
  else
    reset_philox<C>(s, L, Keys{a.k0, a.k1}, (uint32_t)(a.env_offset + e), a.na, a.variable_n,
                    (uint32_t)a.W, tid);
  if (!a.injected) WH_CHECK_ENV(s, L, e, tid);   // injected draws may legitimately be partial
  store_env<C>(s, L, a.state, a.B, (int64_t)blockIdx.x * BT, a.na, tid);
}

// Observation rows (core.py:371-432, reset rows core.py:224-260), HBM-write bound.
// Each env's values live in a small byte image whose layout is one row's value pool:
//   [0] n, [1..R] availability, R x (x,y) delivery targets, R x (x,y) positions,
//   R x (px,py,dx,dy) requests (active slots, ascending pickup index).
// Output float k of an env (k = i*L + f for agent row i, feature f) is img[src[fresh][k]] when
// i < n, else 0.  src is a compile-time byte table per (R, NAM): every row's "other agents"
// gather (skip row i; other_delivery_targets skips row 1 unless the episode is fresh, core.py:428
// vs :256) is folded into it, so the write loop is branch-free.  A workgroup images 16 envs with
// 16 lanes per env, then writes the group's contiguous [16 env x na x L] float region as float4s.
// Small workgroups keep many groups in flight per CU, so one group's image build overlaps the
// others' streaming stores.

template <int R, int NAM>
struct ObsSrc {
  static constexpr int L = 9 * R + 1, W = (NAM * L + 3) / 4;
  uint32_t w[2][W];
};
template <int R, int NAM, int A0 = 1, int G0 = 1 + R, int P0 = 1 + 3 * R, int Q0 = 1 + 5 * R>
constexpr ObsSrc<R, NAM> make_obs_src() {
  ObsSrc<R, NAM> t{};
  constexpr int L = 9 * R + 1;
  for (int fr = 0; fr < 2; ++fr)
    for (int k = 0; k < NAM * L; ++k)
      t.w[fr][k >> 2] |= obs_src<R, A0, G0, P0, Q0>(k / L, k % L, fr != 0) << (8 * (k & 3));
  return t;
}
template <int R, int NAM>
__constant__ ObsSrc<R, NAM> kObsSrc = make_obs_src<R, NAM>();

// The rows [nenv x na x L] f32 of a group's envs from their LDS byte images, float4 q per lane of
// NT lanes (per env: qe float4s, lim = live floats | fresh << 31, gather bytes from src0 / src1 by
// freshness).  Every LDS read is unconditional -- a dead value reads a byte of the image (or past the
// LDS object, which returns 0 without a fault) and is selected away: the conditional form compiled
// to a branch and an lgkmcnt(0) round trip per float, four serial LDS latencies per store.  Both
// gather words are read beside lim, so a float4 takes two LDS round trips, and RU float4s per lane
// are in flight together.
#ifndef WH_ROWS_RU
#define WH_ROWS_RU 2
#endif
template <int NT, int IMG, bool NTS, int RU = WH_ROWS_RU>
__device__ __forceinline__ void stream_rows(const uint32_t* lims, const uint32_t* src0, const uint32_t* src1,
                                            const uint8_t* img, f32x4* __restrict__ out4, uint32_t nenv,
                                            uint32_t qe, int tid, uint32_t q0 = 0, uint32_t q1 = ~0u) {
  const uint32_t magic = 0xFFFFFFFFu / qe + 1u;   // q / qe == umulhi(q, magic) while q * qe < 2^32
  const uint32_t total = nenv * qe < q1 ? nenv * qe : q1;   // float4s [q0, total) of the group
  for (uint32_t q = q0 + tid; q < total; q += RU * NT) {
    f32x4 v[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const uint32_t qu = q + (uint32_t)u * NT < total ? q + (uint32_t)u * NT : q;
      const uint32_t el4 = __umulhi(qu, magic);
      const uint32_t k4 = qu - el4 * qe;
      const uint32_t lim = lims[el4];
      const uint32_t s0 = src0[k4], s1 = src1[k4];
      const uint32_t sw = (int32_t)lim < 0 ? s1 : s0;
      const int lv = (int)(lim & 0x7FFFFFFFu) - 4 * (int)k4;   // > j  <=>  value j is live
      const uint8_t* im = img + el4 * IMG;
      const uint32_t b0 = im[sw & 0xFFu], b1 = im[(sw >> 8) & 0xFFu], b2 = im[(sw >> 16) & 0xFFu],
                     b3 = im[sw >> 24];
      v[u].x = lv > 0 ? (float)b0 : 0.0f;
      v[u].y = lv > 1 ? (float)b1 : 0.0f;
      v[u].z = lv > 2 ? (float)b2 : 0.0f;
      v[u].w = lv > 3 ? (float)b3 : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const uint32_t qu = q + (uint32_t)u * NT;
      if (u == 0 || qu < total) {
        if constexpr (NTS) __builtin_nontemporal_store(v[u], &out4[qu]);
        else out4[qu] = v[u];
      }
    }
  }
}

// The same rows as the policy network's layer-0 B operand (wh_observe_x's layout, below) for the
// group's envs [e0, e0 + nenv), from the images: NT lanes, 16 bytes of whole 32-row tiles each
// (the group's rows nenv * na are whole tiles except in a tail group).  src0 / src1: the gather
// tables (fresh / not fresh: lim's top bit), img: IMG bytes per env.
template <int NT, int L, int IMG>
__device__ __forceinline__ void stream_frags(const uint32_t* lims, const uint32_t* src0, const uint32_t* src1,
                                             const uint8_t* img, uint4* __restrict__ xfrag, int64_t e0,
                                             uint32_t nenv, int na, int tid) {
  constexpr int KQ = (L + 2 + 15) / 16;
  const uint32_t rows = nenv * (uint32_t)na, tiles = (rows + 31u) / 32u;   // (a tail group: fewer)
  // row / na == umulhi(row, magic) while row * na < 2^32, for na >= 2; for na == 1 the constant
  // 2^32 wraps to 0, so that case takes the row itself (every env but the first of a
  // group read env 0's image)
  const bool one = na == 1;
  const uint32_t magic = one ? 0u : 0xFFFFFFFFu / (uint32_t)na + 1u;
  uint4* out = xfrag + ((e0 * na) / 32) * (int64_t)(KQ * 64);
  for (uint32_t c = tid; c < tiles * KQ * 64; c += NT) {
    const uint32_t lane = c & 63u, tq = c >> 6, q = tq % KQ, t = tq / KQ;
    const uint32_t row = t * 32u + (lane & 31u);   // counted from the group's first env
    const uint32_t el1 = one ? row : __umulhi(row, magic), i = row - el1 * (uint32_t)na;
    const bool rl = row < rows;
    const uint32_t lim = lims[rl ? el1 : 0];
    const bool live_row = rl && i < ((lim & 0x7FFFFFFFu) / L);
    const uint8_t* sb = reinterpret_cast<const uint8_t*>((int32_t)lim < 0 ? src1 : src0);
    const uint8_t* im = img + (rl ? el1 : 0) * IMG;
    // unconditional gathers (see stream_rows): the index of a padding feature (k >= L) reads a
    // gather byte past the row, or past the table, and is selected away
    const uint32_t k0 = 16u * q + 8u * (lane >> 5);
    uint32_t gb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) gb[j] = sb[i * L + k0 + j];
    uint32_t w[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      uint32_t hv[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const uint32_t k = k0 + 2u * jj + u;
        const float x = (float)im[gb[2 * jj + u]];
        const float v = k < (uint32_t)L ? (live_row ? x : 0.0f) : (k < (uint32_t)L + 2u ? 1.0f : 0.0f);
        hv[u] = __float_as_uint(v) >> 16;   // byte values and 1.0: exact in bf16
      }
      w[jj] = hv[0] | (hv[1] << 16);
    }
    typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
    const u32x4v v = {w[0], w[1], w[2], w[3]};
    if constexpr (kFragNT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4v*>(&out[c]));
    else *reinterpret_cast<u32x4v*>(&out[c]) = v;
  }
}

template <class C, int OBS_EB>
struct ObsLds {
  static constexpr int IMG = (C::L + 3) & ~3;
  static constexpr int SRCW = ObsSrc<C::R, C::NAM>::W;
  uint8_t img[OBS_EB][IMG];
  uint32_t lim[OBS_EB];          // n * L (floats of live rows) | fresh << 31
  uint32_t ptw[OBS_EB][C::PW];   // pickup target words (nonzero byte = active slot)
  uint32_t src[2][SRCW];
  uint32_t rp[C::P];             // pickup cell, x | y << 16
  uint32_t dst[C::DP];           // delivery cell, x << 8 | y << 24 | 0x00FF00FF
};

// xfrag (optional): the same rows as the policy network's layer-0 B operand (policy_mlp.hip),
// bf16, in MFMA fragment order: 16-byte chunk ((tile * KQ + q) * 64 + lane) of agent-row tile
// `tile` (32 rows) holds features 16q + 8h + j (j < 8) of row tile*32 + (lane & 31), h = lane >> 5;
// features L, L+1 are 1.0 (the MLP's bias columns), the rest of the padding 0.  One coalesced
// 16-byte load per k-step for the MLP instead of scattered f32 rows (and half the bytes).
// CHUNK > 0 (f32 rows as whole float4s only): workgroup c writes the CHUNK float4s [c * CHUNK,
// (c + 1) * CHUNK) of the flat rows instead of its own envs' rows, imaging the (at most OBS_EB) envs
// they belong to -- smaller regions per workgroup, which the write path takes faster (constant
// stores: 16 KB per workgroup 100 us against 37 KB 113 us for Large-16's 608 MB,
// profiles/r06_obs_write_probe_chunks.txt).
template <class C, int OBS_EB, int CHUNK = 0>
__global__ __launch_bounds__(BT) void k_observe(const uint32_t* __restrict__ state, int64_t B, int na,
                                                const uint32_t* __restrict__ tables,
                                                float* __restrict__ obs, int quads,
                                                uint4* __restrict__ xfrag) {
  __shared__ ObsLds<C, OBS_EB> O;
  constexpr int OBS_PARTS = BT / OBS_EB;
  constexpr int R = C::R, D = C::D, L = C::L, SRCW = ObsLds<C, OBS_EB>::SRCW;
  constexpr int A0 = 1, G0 = 1 + R, P0 = 1 + 3 * R, Q0 = 1 + 5 * R;
  const int tid = threadIdx.x;
  int64_t e0;
  uint32_t nenv, qlo = 0, qhi = ~0u;
  if constexpr (CHUNK > 0) {
    const int64_t qe = (int64_t)na * L / 4;
    const int64_t qa = (int64_t)blockIdx.x * CHUNK, qb = min(qa + CHUNK, B * qe);
    e0 = qa / qe;
    nenv = (uint32_t)((qb - 1) / qe - e0 + 1);   // <= OBS_EB (observe_impl: CHUNK <= (OBS_EB - 1) * qe + 1)
    qlo = (uint32_t)(qa - e0 * qe);
    qhi = (uint32_t)(qb - e0 * qe);
  } else {
    e0 = (int64_t)blockIdx.x * OBS_EB;
    nenv = (uint32_t)((B - e0) < OBS_EB ? (B - e0) : OBS_EB);
  }
  const int el = tid / OBS_PARTS, part = tid % OBS_PARTS;
  const bool mine = (uint32_t)el < nenv;
  const int64_t e = e0 + el;
  // Every global load of the prologue is issued before its first use: as strided loops, each
  // iteration compiled to a load -> vmcnt(0) -> LDS write round trip, and the agent rows waited on
  // the header (their guard was r < n) -- about eight serial memory latencies per workgroup for
  // Large-16 (five for its 4.6 KB gather table alone), now one.  An agent row past n is loaded and
  // replaced by IDLE below (rows r < na exist in the state).
  constexpr int NSRC = (2 * SRCW + BT - 1) / BT, NRP = (C::P + BT - 1) / BT, NDP = (C::DP + BT - 1) / BT;
  constexpr int NAR = (R + OBS_PARTS - 1) / OBS_PARTS, NPW = (C::PW + OBS_PARTS - 1) / OBS_PARTS;
  const uint32_t* srcg = &kObsSrc<C::R, C::NAM>.w[0][0];
  uint32_t sv[NSRC], rv[NRP], dv[NDP], av[NAR], pv[NPW], hdr = 0;
#pragma unroll
  for (int i = 0; i < NSRC; ++i) sv[i] = tid + i * BT < 2 * SRCW ? srcg[tid + i * BT] : 0u;
#pragma unroll
  for (int i = 0; i < NRP; ++i) rv[i] = tid + i * BT < C::P ? tables[C::T.rp / 4 + 2 * (tid + i * BT)] : 0u;
#pragma unroll
  for (int i = 0; i < NDP; ++i) dv[i] = tid + i * BT < C::DP ? tables[C::T.dst / 4 + tid + i * BT] : 0u;
  if (mine) {
    hdr = state[e];
#pragma unroll
    for (int i = 0; i < NAR; ++i) {
      const int r = part + i * OBS_PARTS;
      av[i] = (r < R && r < na) ? state[(2 + r) * B + e] : IDLE;
    }
#pragma unroll
    for (int i = 0; i < NPW; ++i) {
      const int w = part + i * OBS_PARTS;
      pv[i] = w < C::PW ? state[(2 + na + w) * B + e] : 0u;
    }
  }
#pragma unroll
  for (int i = 0; i < NSRC; ++i)
    if (tid + i * BT < 2 * SRCW) (&O.src[0][0])[tid + i * BT] = sv[i];
#pragma unroll
  for (int i = 0; i < NRP; ++i)
    if (tid + i * BT < C::P) O.rp[tid + i * BT] = rv[i];
#pragma unroll
  for (int i = 0; i < NDP; ++i)
    if (tid + i * BT < C::DP) O.dst[tid + i * BT] = dv[i];

  const uint8_t nul = (uint8_t)(D / 2);
  if (mine) {
    uint32_t n = (hdr >> 16) & 0xFFu;
    n = n < (uint32_t)na ? n : (uint32_t)na;
    const bool fresh = (hdr >> 24) & 1u;
    uint8_t* im = O.img[el];
    if (part == 0) {
      im[0] = (uint8_t)n;
      O.lim[el] = n * L | (fresh ? 0x80000000u : 0u);
    }
#pragma unroll
    for (int i = 0; i < NAR; ++i) {                       // agent rows
      const int r = part + i * OBS_PARTS;
      if (r < R) {
        const bool live = r < (int)n;
        const uint32_t a = live ? av[i] : IDLE;
        const bool carry = (a & 0xFF00u) != 0xFF00u;
        im[A0 + r] = (uint8_t)((live && !fresh && !carry) ? 1 : 0);
        const bool show = live && !fresh && carry;
        im[G0 + 2 * r] = show ? (uint8_t)((a >> 8) & 0xFFu) : nul;
        im[G0 + 2 * r + 1] = show ? (uint8_t)(a >> 24) : nul;
        im[P0 + 2 * r] = live ? (uint8_t)(a & 0xFFu) : nul;
        im[P0 + 2 * r + 1] = live ? (uint8_t)((a >> 16) & 0xFFu) : nul;
      }
    }
#pragma unroll
    for (int i = 0; i < NPW; ++i) {
      const int w = part + i * OBS_PARTS;
      if (w < C::PW) O.ptw[el][w] = pv[i];
    }
  }
  __syncthreads();
  if (mine) {                                             // requests: ascending pickup index
    uint8_t* im = O.img[el];
    for (int w = part; w < C::PW; w += OBS_PARTS) {
      uint32_t r = 0;
      for (int v = 0; v < w; ++v) r += __popc(nz_hi(O.ptw[el][v]));
      const uint32_t pt = O.ptw[el][w];
      for (int b = 0; b < 4; ++b) {
        const uint32_t tg = (pt >> (8 * b)) & 0xFFu;
        if (tg && r < (uint32_t)R) {
          const uint32_t pxy = O.rp[4 * w + b];
          const uint32_t dxy = O.dst[(tg - 1u) % C::DP];   // x << 8 | y << 24 (| 0x00FF00FF)
          im[Q0 + 4 * r] = (uint8_t)(pxy & 0xFFu);
          im[Q0 + 4 * r + 1] = (uint8_t)(pxy >> 16);
          im[Q0 + 4 * r + 2] = (uint8_t)(dxy >> 8);
          im[Q0 + 4 * r + 3] = (uint8_t)(dxy >> 24);
          ++r;
        }
      }
      if (w == C::PW - 1)      // fewer than R active slots never occurs after reset/step; keep rows defined
        for (; r < (uint32_t)R; ++r)
          im[Q0 + 4 * r] = im[Q0 + 4 * r + 1] = im[Q0 + 4 * r + 2] = im[Q0 + 4 * r + 3] = 0;
    }
  }
  __syncthreads();
  const uint32_t per_env = (uint32_t)na * L;
  if (xfrag)   // the group's rows are whole 32-row tiles (OBS_EB * na % 32 == 0, checked on the host)
    stream_frags<BT, L, ObsLds<C, OBS_EB>::IMG>(O.lim, O.src[0], O.src[1], &O.img[0][0], xfrag, e0, nenv, na, tid);
  if (!obs) return;
  float* out = obs + e0 * per_env;
  if (quads) {
    // per_env % 4 == 0 and obs 16-byte aligned (checked on the host)
    // (the chunk form: all of a lane's float4s in flight together)
    constexpr int RU = CHUNK > 0 ? (CHUNK / BT < 1 ? 1 : (CHUNK / BT > 4 ? 4 : CHUNK / BT)) : WH_ROWS_RU;
    stream_rows<BT, ObsLds<C, OBS_EB>::IMG, rows_nt<C>(), RU>(O.lim, O.src[0], O.src[1], &O.img[0][0],
                                                              reinterpret_cast<f32x4*>(out), nenv, per_env >> 2, tid,
                                                              qlo, qhi);
  } else {
    const uint32_t total = nenv * per_env;
    const uint32_t magic = 0xFFFFFFFFu / per_env + 1u;
    for (uint32_t o = tid; o < total; o += BT) {
      const uint32_t el1 = __umulhi(o, magic);
      const uint32_t k = o - el1 * per_env;
      const uint32_t lim = O.lim[el1];
      const uint8_t* sb = reinterpret_cast<const uint8_t*>(O.src[lim >> 31]);
      out[o] = k < (lim & 0x7FFFFFFFu) ? (float)O.img[el1][sb[k]] : 0.0f;
    }
  }
}

// ----------------------------------------------------------------------------- fused sampler step
// The sampler route (wh_sampler_step: device policy + step + auto-reset, then the observation rows)
// as ONE launch.  A workgroup of 2 x BT lanes owns BT envs: lanes [0, BT) run the fused rollout's
// step for one env each (exactly k_step's fast instance, one step, lane = env), and write their
// env's byte image straight from the registers and the pickup plane; then all 2 x BT lanes stream the
// group's contiguous rows [BT x NA x L] f32 from the images, as k_observe's write loop does.
// Against k_step + k_observe: no second launch, no re-read of the state, no per-env image pass.
// Measured write phase of this shape (tools/obs_write_probe.hip, Medium-8): 512 lanes and 256 envs
// per workgroup stream at the constant-store ceiling (6.45 TB/s); 256 lanes alone (the step
// launch's own shape) reach half of it, so the second half of the workgroup is what makes the rows
// fast.  Two waves per SIMD cap the step code at 256 registers per lane.
//
// Image layout (FImg): word/half-word aligned sections so the step lanes write them with b16/b32
// stores; the compile-time gather table kObsSrcF uses the same offsets.
template <int R>
struct FImg {
  static constexpr int A0 = 1, G0 = (R + 2) & ~1, P0 = G0 + 2 * R, Q0 = (P0 + 2 * R + 3) & ~3,
                       IMG = Q0 + 4 * R;
  static_assert(IMG <= 256, "image byte offsets are 8-bit gather indices");
};
template <int R, int NAM>
__constant__ ObsSrc<R, NAM> kObsSrcF =
    make_obs_src<R, NAM, FImg<R>::A0, FImg<R>::G0, FImg<R>::P0, FImg<R>::Q0>();

template <class C, int NBUF = 1>
struct SampLds {
  static constexpr int IMG = FImg<C::R>::IMG, SRCW = ObsSrc<C::R, C::NAM>::W;
  // multi-step launches: two image buffers, step k's images written while step k-1's rows stream
  // from the other
  alignas(16) uint8_t img[NBUF][BT][IMG];
  uint32_t lim[NBUF][BT];  // n * L (floats of live rows) | fresh << 31
  uint32_t src[2][SRCW];
};

// core.py:224-260 / 371-432 for the env of this lane, from its registers after the step: the image
// k_observe builds from the packed state (n, availability, delivery targets, positions, the open
// requests in ascending pickup order with their pickup and delivery cells).
template <class C, int NBUF>
__device__ __forceinline__ void write_image(const Regs<C>& s, const Lds<C>& L, SampLds<C, NBUF>& O, int tid, int na,
                                            int buf) {
  using F = FImg<C::R>;
  uint8_t* im = O.img[buf][tid];
  uint32_t n = (s.hdr >> 16) & 0xFFu;
  n = n < (uint32_t)na ? n : (uint32_t)na;
  const bool fresh = (s.hdr >> 24) & 1u;
  constexpr uint32_t nul = (uint32_t)(C::D / 2), nul2 = nul | (nul << 8);
  im[0] = (uint8_t)n;
#pragma unroll
  for (int r = 0; r < C::R; ++r) {
    const uint32_t a = r < C::NAM ? s.ag[r] : IDLE;
    const bool live = (uint32_t)r < n;
    const bool carry = (a & 0xFF00u) != 0xFF00u;
    im[F::A0 + r] = (uint8_t)((live && !fresh && !carry) ? 1 : 0);
    const uint32_t dtg = __builtin_amdgcn_perm(a, a, 0x0C0C0301u);   // dx | dy << 8
    const uint32_t pos = __builtin_amdgcn_perm(a, a, 0x0C0C0200u);   // x | y << 8
    *reinterpret_cast<uint16_t*>(im + F::G0 + 2 * r) = (uint16_t)((live && !fresh && carry) ? dtg : nul2);
    *reinterpret_cast<uint16_t*>(im + F::P0 + 2 * r) = (uint16_t)(live ? pos : nul2);
  }
  // open requests, ascending pickup index (core.py:409-418); fewer than R open (never after a
  // reset or a step) leaves zero slots, as k_observe does
  uint32_t mlo = (uint32_t)s.am, mhi = (uint32_t)(s.am >> 32);
#pragma unroll
  for (int r = 0; r < C::R; ++r) {
    uint32_t flo, fhi;
    asm("v_ffbl_b32 %0, %1" : "=v"(flo) : "v"(mlo));   // 0xFFFFFFFF when empty
    asm("v_ffbl_b32 %0, %1" : "=v"(fhi) : "v"(mhi));
    const uint32_t j = __builtin_elementwise_min(
        __builtin_elementwise_min(flo, __builtin_elementwise_add_sat(fhi, 32u)), (uint32_t)C::P);
    const uint32_t rp = L.rtag(j).x;                        // pickup cell x | y << 16
    const uint32_t tb = L.target_byte(j, tid);              // target + 1 (row P: scratch)
    const uint32_t dc = L.dst_tb(tb);                       // x << 8 | y << 24 | 0x00FF00FF
    const uint32_t w = __builtin_amdgcn_perm(dc, rp, 0x07050200u);   // px | py << 8 | dx << 16 | dy << 24
    *reinterpret_cast<uint32_t*>(im + F::Q0 + 4 * r) = j < (uint32_t)C::P ? w : 0u;
    uint64_t m = ((uint64_t)mhi << 32) | mlo;
    m &= m - 1ull;
    mlo = (uint32_t)m;
    mhi = (uint32_t)(m >> 32);
  }
  O.lim[buf][tid] = n * (uint32_t)C::L | (fresh ? 0x80000000u : 0u);
}

// Rows of the workgroup's envs from image buffer `buf`: one contiguous [nenv x na x L] f32 region at
// `rows` (its first env's first float), float4 per lane over all 2 x BT lanes, q = tid + 2 BT i (na * L
// % 4 == 0 and 16-byte alignment: checked on the host).  (Chunks handed out from an LDS counter, so
// that the step lanes of a multi-step launch take less once they join late, measured 1.5 us slower
// on a 1-step launch and no faster on 20- and 100-step ones: profiles/r04_rows_ab.txt.)
// Every LDS read of a float4 is unconditional (a dead value reads a byte of the image, or past it,
// which LDS returns as 0 without a fault, and is then selected away): the conditional form compiled
// to one branch and one lgkmcnt(0) round trip per float, four serial LDS latencies per store.  The
// gather word of both tables is read beside lim, so a float4 costs two LDS round trips, and RU
// float4s per lane are in flight together.
template <class C, bool NTS, int NBUF>
__device__ __forceinline__ void write_rows(const SampLds<C, NBUF>& O, int buf, float* __restrict__ rows,
                                           uint32_t nenv, uint32_t qe, int tid) {
  stream_rows<2 * BT, SampLds<C, NBUF>::IMG, NTS>(O.lim[buf], O.src[0], O.src[1], &O.img[buf][0][0],
                                             reinterpret_cast<f32x4*>(rows), nenv, qe, tid);
}

// FAST: the fused rollout's steps (greedy/random policy, every env stepped, auto-reset): a.steps of
// them in one launch (wh_sampler_step: 1; wh_sampler_rollout: a rollout fragment), step k's rows
// going to obs + k * B * NA * L.  Iteration k of the launch loop: the step lanes compute step k and
// write its images into buffer k % 2 while the other lanes (and the step lanes, once done) stream
// step k-1's rows from buffer (k-1) % 2; one barrier per iteration.  So after the first step the
// simulation runs under the row stream, which is what binds (HBM writes).  State stays in registers
// across the steps, as in the fused rollout (reset slots from 8 steps on).
// Otherwise (FAST = false) wh_vector_step's single step: external actions in ascending or
// action-dict order (ORDERED), an optional env mask -- envs not stepped keep their state and still
// get their rows -- and the launch options of k_step's generic instance (episode metrics, odd agent
// counts).
template <class C, int POLICY, bool ORDERED, bool FAST, bool MULTI = false>
__global__ __launch_bounds__(2 * BT) void k_sampler(StepParams a, float* __restrict__ obs) {
  __shared__ Lds<C> L;
  __shared__ SampLds<C, MULTI ? 2 : 1> O;
  __shared__ std::conditional_t<MULTI, Slots<C>, NoSlots> RS;   // reset slots: multi-step launches
  __shared__ std::conditional_t<ORDERED, OKeys<C>, NoSlots> OK;   // dict-order move keys: ORDERED only
  const int tid = threadIdx.x;
  const bool stepper = tid < BT;
  const int64_t e0 = (int64_t)blockIdx.x * BT;
  const int64_t e = e0 + tid;
  const bool loaded = stepper && e < a.B;                              // its rows are written
  const bool stepped = loaded && (FAST || !a.mask || a.mask[e]);       // and it is stepped
  const int na = FAST ? C::NAM : a.na;
  RawEnv<C> raw;
  FastRun<C, POLICY, MULTI> run(a, e);
  // The step waves (stepper is wave-uniform: waves 0-3) issue the table loads (L2), then the state
  // planes (HBM), and write the table to LDS once it has landed, with the state still in flight --
  // all inside one uniform branch, so the waitcnt pass counts exactly (every step lane loads: a lane
  // past B re-reads env e0, which exists).  The row waves copy the gather table meanwhile.
  if (stepper) {
    const uint4 tv0 = issue_table_chunk<C>(a.tables, 0), tv1 = issue_table_chunk<C>(a.tables, 1);
    __builtin_amdgcn_sched_barrier(0);   // table loads ahead of the state loads, as in k_step
    load_env_issue<C>(raw, a.state, a.B, e0, loaded ? tid : 0, na);
    if constexpr (FAST) {
      if (loaded) run.load_actions(a, e);
    }
    commit_table_chunk<C>(L.tbl, 0, tv0);
    commit_table_chunk<C>(L.tbl, 1, tv1);
  } else {
    // all loads first, then the LDS writes: one memory latency, not one per strided iteration
    const uint32_t* srcg = &kObsSrcF<C::R, C::NAM>.w[0][0];
    constexpr int NS = 2 * SampLds<C>::SRCW, NSRC = (NS + BT - 1) / BT;
    uint32_t sv[NSRC];
#pragma unroll
    for (int i = 0; i < NSRC; ++i) sv[i] = tid - BT + i * BT < NS ? srcg[tid - BT + i * BT] : 0u;
#pragma unroll
    for (int i = 0; i < NSRC; ++i)
      if (tid - BT + i * BT < NS) (&O.src[0][0])[tid - BT + i * BT] = sv[i];
  }
  __syncthreads();
  const uint32_t nenv = (uint32_t)((a.B - e0) < BT ? (a.B - e0) : BT);
  const uint32_t qe = FAST ? (uint32_t)(C::NAM * C::L / 4) : (uint32_t)(na * C::L / 4);
  const Keys k{a.k0, a.k1};
  const uint32_t gid = (uint32_t)(a.env_offset + e);
  Regs<C> s;
  if (loaded) {
    load_env_finish<C>(s, L, raw, (uint32_t)a.W, tid);
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): drain the state loads before the step (k_step)
    if (stepped) {
#pragma unroll
      for (int y = 0; y < C::D; ++y) L.occ[y][tid] = 0u;
    }
  }
  if constexpr (FAST && MULTI) {
    if (loaded) RS.rs_ep[tid] = s.epi;   // reset slots start stale (!= epi + 1)
    const int64_t step_floats = a.B * (int64_t)(C::NAM * C::L);
#ifdef WH_ABLATION
    const int ablate = a.ablate;   // timing-only: 512 = no steps/images, 256 = no rows
#else
    constexpr int ablate = 0;
#endif
    for (int it = 0; it <= a.steps; ++it) {   // (every wave reaches every barrier)
      if (loaded && it < a.steps && !(ablate & 512)) {
        run.step(a, s, L, &RS, k, gid, e, tid, it);
        write_image<C>(s, L, O, tid, C::NAM, it & 1);
      }
      if (it > 0 && !(ablate & 256))
        write_rows<C, false>(O, (it - 1) & 1, obs + (int64_t)(it - 1) * step_floats + e0 * (int64_t)(4 * qe), nenv, qe, tid);
      __syncthreads();
    }
    if (loaded) store_env<C>(s, L, a.state, a.B, e0, na, tid);
  } else if constexpr (FAST) {   // one step
    if (loaded) {
      run.step(a, s, L, nullptr, k, gid, e, tid, 0);
      store_env<C>(s, L, a.state, a.B, e0, na, tid);
      write_image<C>(s, L, O, tid, C::NAM, 0);
    }
    __syncthreads();
    write_rows<C, rows_nt<C>()>(O, 0, obs + e0 * (int64_t)(4 * qe), nenv, qe, tid);
  } else {
    if (stepped) {
      if constexpr (ORDERED)
        run_steps<C, POLICY, ORDERED, PH_ALL>(a, s, L, k, gid, e, tid, &OK.k[0][0]);
      else
        run_steps<C, POLICY, ORDERED, PH_ALL>(a, s, L, k, gid, e, tid);
      store_env<C>(s, L, a.state, a.B, e0, na, tid);
    }
    if (loaded) write_image<C>(s, L, O, tid, na, 0);
    __syncthreads();
    write_rows<C, rows_nt<C>()>(O, 0, obs + e0 * (int64_t)(4 * qe), nenv, qe, tid);
  }
}

// canonical <-> packed (runtime dims; not on the hot path)
struct PackParams {
  uint32_t* state;
  const uint32_t* cstate;
  int64_t B;
  int32_t na, P, pw, D;
  int32_t *pos, *agent_target, *pickup_target, *pickup_timer, *t, *n;
  uint8_t* fresh;
  uint32_t* episode;
};

// delivery index -> (x, y) and back (core.py:177-188)
__device__ __forceinline__ uint32_t delivery_cell(int32_t d, int D) {
  const uint32_t v = 2 + ((uint32_t)d >> 2), side = (uint32_t)d & 3u;
  const uint32_t x = (side & 1u) ? (side == 3u ? (uint32_t)(D - 1) : 0u) : v;
  const uint32_t y = (side & 1u) ? v : (side == 2u ? (uint32_t)(D - 1) : 0u);
  return x | (y << 16);
}
__device__ __forceinline__ int32_t delivery_index(uint32_t x, uint32_t y, int D) {
  if (y == 0) return 4 * ((int32_t)x - 2);
  if (x == 0) return 4 * ((int32_t)y - 2) + 1;
  if (y == (uint32_t)(D - 1)) return 4 * ((int32_t)x - 2) + 2;
  return 4 * ((int32_t)y - 2) + 3;
}

__global__ __launch_bounds__(BT) void k_pack(PackParams a) {
  const int64_t e = (int64_t)blockIdx.x * BT + threadIdx.x;
  if (e >= a.B) return;
  const int64_t B = a.B;
  // out-of-range canonical values are clamped so packed state always indexes inside the grid
  const uint32_t n = min((uint32_t)max(a.n[e], 0), (uint32_t)a.na);
  a.state[e] = ((uint32_t)a.t[e] & 0xFFFFu) | (n << 16) | (a.fresh[e] ? (1u << 24) : 0u);
  a.state[B + e] = a.episode[e];
  const int32_t DP = 4 * (a.D - 4);
  for (int i = 0; i < a.na; ++i) {
    uint32_t w = IDLE;
    if (i < (int)n) {
      const int32_t tg = a.agent_target[e * a.na + i];
      const uint32_t x = (uint32_t)min(max(a.pos[(e * a.na + i) * 2], 0), a.D - 1);
      const uint32_t y = (uint32_t)min(max(a.pos[(e * a.na + i) * 2 + 1], 0), a.D - 1);
      w = x | (y << 16) | ((tg >= 0 && tg < DP) ? (delivery_cell(tg, a.D) << 8) : IDLE);
    }
    a.state[(2 + i) * B + e] = w;
  }
  for (int w = 0; w < a.pw; ++w) {
    uint32_t tw = 0, mw = 0;
    for (int b = 0; b < 4; ++b) {
      const int j = 4 * w + b;
      const int32_t tg = a.pickup_target[e * a.P + j];
      if (tg >= 0 && tg < DP) {
        tw |= (uint32_t)(tg + 1) << (8 * b);
        mw |= (((uint32_t)a.t[e] + (uint32_t)a.pickup_timer[e * a.P + j]) & 0xFFu) << (8 * b);   // expiry step
      }
    }
    a.state[(2 + a.na + w) * B + e] = tw;
    a.state[(2 + a.na + a.pw + w) * B + e] = mw;
  }
}

__global__ __launch_bounds__(BT) void k_unpack(PackParams a) {
  const int64_t e = (int64_t)blockIdx.x * BT + threadIdx.x;
  if (e >= a.B) return;
  const int64_t B = a.B;
  const uint32_t h = a.cstate[e];
  const uint32_t n = (h >> 16) & 0xFFu;
  a.t[e] = (int32_t)(h & 0xFFFFu);
  a.n[e] = (int32_t)n;
  a.fresh[e] = (uint8_t)((h >> 24) & 1u);
  a.episode[e] = a.cstate[B + e];
  for (int i = 0; i < a.na; ++i) {
    const uint32_t w = a.cstate[(2 + i) * B + e];
    const bool live = i < (int)n;
    a.pos[(e * a.na + i) * 2] = live ? (int32_t)(w & 0xFFu) : 0;
    a.pos[(e * a.na + i) * 2 + 1] = live ? (int32_t)((w >> 16) & 0xFFu) : 0;
    const bool carry = live && (w & 0xFF00u) != 0xFF00u;
    a.agent_target[e * a.na + i] = carry ? delivery_index((w >> 8) & 0xFFu, w >> 24, a.D) : -1;
  }
  for (int w = 0; w < a.pw; ++w) {
    const uint32_t tw = a.cstate[(2 + a.na + w) * B + e];
    const uint32_t mw = a.cstate[(2 + a.na + a.pw + w) * B + e];
    for (int b = 0; b < 4; ++b) {
      const int j = 4 * w + b;
      const uint32_t tg = (tw >> (8 * b)) & 0xFFu;
      a.pickup_target[e * a.P + j] = (int32_t)tg - 1;
      a.pickup_timer[e * a.P + j] = tg ? (int32_t)(((mw >> (8 * b)) - h) & 0xFFu) : -1;   // steps left
    }
  }
}

// ----------------------------------------------------------------------------- host side
int hip_err(hipError_t e) { return e == hipSuccess ? WH_OK : WH_EHIP + (int)e; }

struct Geometry {
  int D, R, NR, NA, P, DP, T, W;
  int racks[WH_MAX_RACKS];
};

int validate(const wh_config* c, Geometry* g) {
  if (!c) return WH_EINVAL;
  g->D = c->area_dimension;
  g->R = c->num_requests;
  g->NR = c->num_racks;
  g->NA = c->agent_slots;
  g->T = c->episode_duration;
  g->W = c->pickup_wait_duration;
  if (g->NR < 1 || g->NR > WH_MAX_RACKS || g->D < 5 || g->D > 32) return WH_EINVAL;
  g->P = 4 * g->NR * g->NR;
  g->DP = 4 * (g->D - 4);
  if (g->NA < 1 || g->NA > g->R || g->R > g->P || g->R > g->DP) return WH_EINVAL;
  if (g->W < 1 || g->W > 255 || g->T < 0) return WH_EINVAL;
  for (int i = 0; i < g->NR; ++i) {
    g->racks[i] = c->racks[i];
    if (c->racks[i] < 2 || c->racks[i] > g->D - 2) return WH_ENOTSUP;  // pickups must be interior
  }
  return WH_OK;
}

// Host copy of the per-workgroup tables, same layout as TableLayout (core.py:170-199):
//   cell  [256*D] u8 : (x | y << 8) -> pickup index + 1, 0 = not a pickup cell
//   rp/tag [P+1] u32 pairs, interleaved (the policy reads both with one 8-byte LDS read):
//          rp  = pickup cell as x | y << 16; [P] = far-away cell (never nearest)
//          tag = pickup << 10 | x << 5 | y   (greedy argmin tag, solvers.py:53-58);
//                [P] = the null cell (D/2, D/2): where fresh-reset agents head (core.py:233-236)
//   dst   [Dp]   u32 : delivery cell in agent-word target bytes, x << 8 | y << 24 | 0x00FF00FF
//   mv    [12]   u32 : MOVES[a] as packed i16 (dx, dy) (core.py:38)
//   valid [NV]   u32 : interior non-pickup cells x | y << 16, ascending (x, y) (spawn, core.py:191-199)
std::vector<uint32_t> build_tables(const Geometry& g, int* bad) {
  const int D = g.D;
  *bad = 0;
  if (D > 32) { *bad = 1; return {}; }
  std::vector<uint8_t> cell(cell_bytes(D), 0);
  std::vector<uint32_t> rp(g.P + 1), tag(g.P + 1);
  rp[g.P] = 0x00FF00FFu;
  tag[g.P] = (63u << 10) | ((uint32_t)(D / 2) << 5) | (uint32_t)(D / 2);   // pickup << 10 | y << 5 | x
  for (int ix = 0; ix < g.NR; ++ix)
    for (int iy = 0; iy < g.NR; ++iy)
      for (int q = 0; q < 4; ++q) {
        const int j = (ix * g.NR + iy) * 4 + q;
        const int x = g.racks[ix] - 1 + (q & 1), y = g.racks[iy] - 1 + (q >> 1);
        const int ci = cell_index(x, y, D);
        if (cell[ci]) *bad = 1;  // overlapping racks
        cell[ci] = (uint8_t)(j + 1);
        rp[j] = (uint32_t)x | ((uint32_t)y << 16);
        tag[j] = ((uint32_t)j << 10) | ((uint32_t)y << 5) | (uint32_t)x;
      }
  std::vector<uint32_t> dst(g.DP);
  for (int d = 0; d < g.DP; ++d) {
    const int v = 2 + d / 4, side = d % 4;
    const int x = (side & 1) ? (side == 3 ? D - 1 : 0) : v;
    const int y = (side & 1) ? v : (side == 2 ? D - 1 : 0);
    dst[d] = ((uint32_t)x << 8) | ((uint32_t)y << 24) | XY16;
  }
  std::vector<uint32_t> mv(12, 0);
  for (int a = 0; a < 9; ++a) {
    const int dx = a / 3 - 1, dy = a % 3 - 1;
    mv[a] = (uint32_t)(uint16_t)(int16_t)dx | ((uint32_t)(uint16_t)(int16_t)dy << 16);
  }
  std::vector<uint32_t> valid;
  for (int x = 1; x < D - 1; ++x)
    for (int y = 1; y < D - 1; ++y)
      if (!cell[cell_index(x, y, D)]) valid.push_back((uint32_t)x | ((uint32_t)y << 16));
  std::vector<uint32_t> words(cell.size() / 4, 0);
  memcpy(words.data(), cell.data(), cell.size());
  for (int j = 0; j <= g.P; ++j) {
    words.push_back(rp[j]);
    words.push_back(tag[j]);
  }
  words.insert(words.end(), dst.begin(), dst.end());
  words.insert(words.end(), mv.begin(), mv.end());
  words.insert(words.end(), valid.begin(), valid.end());
  return words;
}

struct TableEntry {
  int device, D, NR, words;
  int racks[WH_MAX_RACKS];
  uint32_t* dev;
};
std::mutex g_tab_mu;
std::vector<TableEntry> g_tabs;

// Device copy of the tables for (device, geometry); allocated once per geometry and device.  The
// device is the launch stream's (not the calling thread's current device), so a kernel never reads
// tables that live on another GPU.
int device_tables(const Geometry& g, int expect_words, hipStream_t stream, const uint32_t** out) {
  int dev = 0;
  hipError_t he = stream ? hipStreamGetDevice(stream, &dev) : hipGetDevice(&dev);
  if (he != hipSuccess) return hip_err(he);
  std::lock_guard<std::mutex> lk(g_tab_mu);
  for (auto& t : g_tabs)
    if (t.device == dev && t.D == g.D && t.NR == g.NR && !memcmp(t.racks, g.racks, sizeof(int) * g.NR)) {
      *out = t.dev;
      return t.words == expect_words ? WH_OK : WH_ENOTSUP;
    }
  int bad = 0;
  std::vector<uint32_t> w = build_tables(g, &bad);
  if (bad || (int)w.size() != expect_words) return WH_ENOTSUP;
  int cur = 0;
  he = hipGetDevice(&cur);
  if (he != hipSuccess) return hip_err(he);
  if (cur != dev && (he = hipSetDevice(dev)) != hipSuccess) return hip_err(he);
  uint32_t* d = nullptr;
  const size_t padded = (w.size() + 3) / 4 * 16;   // load_tables reads whole 16-byte chunks
  he = hipMalloc(&d, padded);
  if (he == hipSuccess) he = hipMemset(d, 0, padded);
  if (he == hipSuccess) he = hipMemcpy(d, w.data(), w.size() * 4, hipMemcpyHostToDevice);
  if (cur != dev) (void)hipSetDevice(cur);
  if (he != hipSuccess) return hip_err(he);
  TableEntry t{dev, g.D, g.NR, (int)w.size(), {0}, d};
  memcpy(t.racks, g.racks, sizeof(int) * g.NR);
  g_tabs.push_back(t);
  *out = d;
  return WH_OK;
}

// ---- kernel registry: (D, R, NR, NAM) instances
struct Kernels {
  int D, R, NR, NAM;
  void (*step[3])(StepParams);
  void (*step_fast[3])(StepParams);   // [policy]: greedy / random fused rollouts (NAM even), else null
  void (*step_ordered)(StepParams);
  void (*sampler[3])(StepParams, float*);   // [policy]: fused step + rows (k_sampler), NAM even, else null
  void (*sampler_multi[3])(StepParams, float*);   // [policy]: the same, K steps per launch (greedy / random)
  void (*vsampler[2])(StepParams, float*);  // [ordered]: wh_vector_step's step + rows (external actions)
  void (*reset)(ResetParams);
  void (*observe[4])(const uint32_t*, int64_t, int, const uint32_t*, float*, int, uint4*);   // kObsEB[i] envs per WG
  void (*observe_chunk)(const uint32_t*, int64_t, int, const uint32_t*, float*, int, uint4*);   // kObsChunk float4s per WG
  int tblw, nv;
};

// Large (R = 16) dispatches no k_sampler: with 16 agent slots its rows (9.3 KB per env) pass the fuse
// limit, and with 2-8 slots the step code spills at two waves per SIMD (220-544 B of scratch,
// tools/kernel_resources.py), which fused_ok() refuses.  Those instances are not built (unless an A/B
// build raises the limit), so no kernel with a private segment is left in the dict-order route.
template <class C>
constexpr bool kSamplerBuilt = C::R < 16 || WH_FUSE_ROWS_MAX > 4096;

template <int D, int R, int NR, int NAM>
Kernels make_kernels() {
  using C = Cfg<D, R, NR, NAM>;
  Kernels k;
  k.D = D; k.R = R; k.NR = NR; k.NAM = NAM;
  k.step[0] = k_step<C, POL_EXTERNAL, false, false>;
  k.step[1] = k_step<C, POL_GREEDY, false, false>;
  k.step[2] = k_step<C, POL_RANDOM, false, false>;
  k.step_fast[0] = nullptr;   // (set below for even agent counts: wh_vector_step's common case)
  k.sampler[0] = k.sampler[1] = k.sampler[2] = nullptr;
  k.sampler_multi[0] = k.sampler_multi[1] = k.sampler_multi[2] = nullptr;
  // the multi-step sampler holds the step's LDS, its reset slots and two image buffers
  constexpr bool sampler_fits = sizeof(Lds<C>) + sizeof(Slots<C>) + sizeof(SampLds<C, 2>) <= 160 * 1024;
  if constexpr (NAM % 2 == 0) {
    k.step_fast[0] = k_step<C, POL_EXTERNAL, false, true>;
    k.step_fast[1] = k_step<C, POL_GREEDY, false, true>;
    k.step_fast[2] = k_step<C, POL_RANDOM, false, true>;
    if constexpr (kSamplerBuilt<C>) {
      k.sampler[0] = k_sampler<C, POL_EXTERNAL, false, true>;
      k.sampler[1] = k_sampler<C, POL_GREEDY, false, true>;
      k.sampler[2] = k_sampler<C, POL_RANDOM, false, true>;
    }
    if constexpr (sampler_fits && kSamplerBuilt<C>) {
      k.sampler_multi[1] = k_sampler<C, POL_GREEDY, false, true, true>;
      k.sampler_multi[2] = k_sampler<C, POL_RANDOM, false, true, true>;
    }
  } else {
    k.step_fast[1] = k.step_fast[2] = nullptr;
  }
  k.step_ordered = k_step<C, POL_EXTERNAL, true, false>;
  k.vsampler[0] = k.vsampler[1] = nullptr;
  if constexpr (kSamplerBuilt<C>) {
    k.vsampler[0] = k_sampler<C, POL_EXTERNAL, false, false>;
    // the dict-order instance also holds the entries' move keys (OKeys: 4 * NAM x 512 bytes)
    if constexpr (sizeof(Lds<C>) + sizeof(SampLds<C, 1>) + sizeof(OKeys<C>) <= 160 * 1024)
      k.vsampler[1] = k_sampler<C, POL_EXTERNAL, true, false>;
  }
  k.reset = k_reset<C>;
  k.observe[0] = k_observe<C, kObsEB[0]>;
  k.observe[1] = k_observe<C, kObsEB[1]>;
  k.observe[2] = k_observe<C, kObsEB[2]>;
  k.observe[3] = k_observe<C, kObsEB[3]>;
  k.observe_chunk = kObsChunk > 0 ? k_observe<C, kObsEB[0], kObsChunk> : nullptr;
  k.tblw = C::TBLW;
  k.nv = C::NV;
  return k;
}

const std::vector<Kernels>& registry() {
#ifdef WH_ONLY_MEDIUM8   // analysis builds (tools/lds_stalls.py): one instance, fast to compile
  static const std::vector<Kernels> r = {make_kernels<16, 9, 3, 8>()};
#elif defined(WH_ONLY_LARGE16)
  static const std::vector<Kernels> r = {make_kernels<20, 16, 4, 16>()};
#elif defined(WH_ONLY_SMALL4)
  static const std::vector<Kernels> r = {make_kernels<12, 4, 2, 4>()};
#else
  static const std::vector<Kernels> r = {
      // WarehouseSmall  (variants.py:19-32): D=12, R=4, racks [4, 8]
      make_kernels<12, 4, 2, 2>(), make_kernels<12, 4, 2, 4>(),
      // WarehouseMedium (variants.py:35-47): D=16, R=9, racks [4, 8, 12]
      make_kernels<16, 9, 3, 2>(), make_kernels<16, 9, 3, 4>(), make_kernels<16, 9, 3, 8>(),
      make_kernels<16, 9, 3, 9>(),
      // WarehouseLarge  (variants.py:50-62): D=20, R=16, racks [4, 8, 12, 16]
      make_kernels<20, 16, 4, 2>(), make_kernels<20, 16, 4, 4>(), make_kernels<20, 16, 4, 8>(),
      make_kernels<20, 16, 4, 16>(),
  };
#endif
  return r;
}

// A fused step + rows kernel (k_sampler) runs two waves per SIMD, so its step code gets 256
// registers instead of 512: configurations whose step needs more spill to scratch there (Large-16)
// and keep the two launches.  Decided once per kernel from its private segment size.
bool fused_ok(void (*kern)(StepParams, float*)) {
  static std::mutex mu;
  static std::vector<std::pair<const void*, bool>> seen;
  std::lock_guard<std::mutex> lk(mu);
  for (const auto& p : seen)
    if (p.first == reinterpret_cast<const void*>(kern)) return p.second;
  hipFuncAttributes at;
  const bool ok = hipFuncGetAttributes(&at, reinterpret_cast<const void*>(kern)) == hipSuccess && at.localSizeBytes == 0;
  seen.emplace_back(reinterpret_cast<const void*>(kern), ok);
  return ok;
}

// The fused step + rows launch pays while an env's rows are small: at Large-16 (9.3 KB of rows per
// env, one 512-lane workgroup per CU by LDS) it streams the rows slower than k_observe's small
// workgroups -- 165 vs 127 us per sampler step for the two launches (profiles/r06_l16fuse_ab.txt,
// with the fused instance free of scratch); Small-4 13.2 vs 15.1, Medium-8 34.7 vs 40.3
// (profiles/r05_step3_ab.txt).  So configurations with more than WH_FUSE_ROWS_MAX bytes of rows per
// env take the two launches.
bool fuse_rows(const Geometry& g) { return 4 * g.NA * (9 * g.R + 1) <= WH_FUSE_ROWS_MAX; }

const Kernels* pick(const Geometry& g) {
  const Kernels* best = nullptr;
  for (const auto& k : registry())
    if (k.D == g.D && k.R == g.R && k.NR == g.NR && k.NAM >= g.NA && (!best || k.NAM < best->NAM))
      best = &k;
  return best;
}

int prepare(const wh_config* cfg, int64_t B, void* stream, Geometry* g, const Kernels** kk,
            const uint32_t** tab) {
  int rc = validate(cfg, g);
  if (rc) return rc;
  if (B < 0) return WH_EINVAL;
  *kk = pick(*g);
  if (!*kk) return WH_ENOTSUP;
  *tab = nullptr;
  if (B == 0) return WH_OK;   // an empty batch launches nothing: no device, no tables
  return device_tables(*g, (*kk)->tblw, (hipStream_t)stream, tab);
}

inline dim3 grid_for(int64_t B) { return dim3((unsigned)((B + BT - 1) / BT)); }

}  // namespace

// =============================================================================== C ABI
extern "C" {

#ifdef WH_TIMING
int wh_debug_times(uint64_t* out, int32_t n) {   // timing builds only (not in the header)
  if (!out || n < 0 || n > kTimeWaves * kTimeSlots) return WH_EINVAL;
  hipError_t he = hipDeviceSynchronize();
  if (he == hipSuccess) he = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wh_times), (size_t)n * 8, 0, hipMemcpyDeviceToHost);
  return he == hipSuccess ? WH_OK : hip_err(he);
}
#endif

int wh_check_read(uint64_t* out, int32_t clear) {
#ifdef WH_CHECK
  if (!out) return WH_EINVAL;
  unsigned long long v[4];
  hipError_t he = hipDeviceSynchronize();
  if (he == hipSuccess) he = hipMemcpyFromSymbol(v, HIP_SYMBOL(g_wh_check), sizeof(v), 0, hipMemcpyDeviceToHost);
  if (he != hipSuccess) return hip_err(he);
  for (int i = 0; i < 4; ++i) out[i] = v[i];
  if (clear) {
    const unsigned long long z[4] = {0, 0, 0, 0};
    he = hipMemcpyToSymbol(HIP_SYMBOL(g_wh_check), z, sizeof(z), 0, hipMemcpyHostToDevice);
    if (he != hipSuccess) return hip_err(he);
  }
  return WH_OK;
#elif defined(WH_COUNT_REV)
  if (!out) return WH_EINVAL;
  unsigned long long v[2];
  hipError_t he = hipDeviceSynchronize();
  if (he == hipSuccess) he = hipMemcpyFromSymbol(v, HIP_SYMBOL(g_wh_revcount), sizeof(v), 0, hipMemcpyDeviceToHost);
  if (he != hipSuccess) return hip_err(he);
  out[0] = v[0];
  out[1] = v[1];
  out[2] = out[3] = 0;
  if (clear) {
    const unsigned long long z[2] = {0, 0};
    he = hipMemcpyToSymbol(HIP_SYMBOL(g_wh_revcount), z, sizeof(z), 0, hipMemcpyHostToDevice);
    if (he != hipSuccess) return hip_err(he);
  }
  return WH_OK;
#else
  (void)out;
  (void)clear;
  return WH_ENOTSUP;
#endif
}

int wh_query(const wh_config* cfg, wh_layout* out) {
  Geometry g;
  int rc = validate(cfg, &g);
  if (rc) return rc;
  const Kernels* k = pick(g);
  if (!k) return WH_ENOTSUP;
  if (out) {
    out->words_per_env = 2 + g.NA + 2 * (g.P / 4);
    out->num_pickups = g.P;
    out->num_deliveries = g.DP;
    out->obs_len = 9 * g.R + 1;
    out->kernel_agents = k->NAM;
  }
  return WH_OK;
}

int wh_pack(const wh_config* cfg, int64_t B, const int32_t* pos, const int32_t* agent_target,
            const int32_t* pickup_target, const int32_t* pickup_timer, const int32_t* t,
            const int32_t* n, const uint8_t* fresh, const uint32_t* episode, uint32_t* state,
            void* stream) {
  Geometry g;
  int rc = validate(cfg, &g);
  if (rc) return rc;
  if (B == 0) return WH_OK;
  if (B < 0 || !pos || !agent_target || !pickup_target || !pickup_timer || !t || !n || !fresh ||
      !episode || !state)
    return WH_EINVAL;
  PackParams a{state, nullptr, B, g.NA, g.P, g.P / 4, g.D, const_cast<int32_t*>(pos),
               const_cast<int32_t*>(agent_target), const_cast<int32_t*>(pickup_target),
               const_cast<int32_t*>(pickup_timer), const_cast<int32_t*>(t), const_cast<int32_t*>(n),
               const_cast<uint8_t*>(fresh), const_cast<uint32_t*>(episode)};
  hipLaunchKernelGGL(k_pack, grid_for(B), dim3(BT), 0, (hipStream_t)stream, a);
  return hip_err(hipGetLastError());
}

int wh_unpack(const wh_config* cfg, int64_t B, const uint32_t* state, int32_t* pos,
              int32_t* agent_target, int32_t* pickup_target, int32_t* pickup_timer, int32_t* t,
              int32_t* n, uint8_t* fresh, uint32_t* episode, void* stream) {
  Geometry g;
  int rc = validate(cfg, &g);
  if (rc) return rc;
  if (B == 0) return WH_OK;
  if (B < 0 || !pos || !agent_target || !pickup_target || !pickup_timer || !t || !n || !fresh ||
      !episode || !state)
    return WH_EINVAL;
  PackParams a{nullptr, state, B, g.NA, g.P, g.P / 4, g.D, pos, agent_target, pickup_target,
               pickup_timer, t, n, fresh, episode};
  hipLaunchKernelGGL(k_unpack, grid_for(B), dim3(BT), 0, (hipStream_t)stream, a);
  return hip_err(hipGetLastError());
}

int wh_reset(const wh_config* cfg, int64_t B, uint32_t* state, const uint8_t* mask,
             const wh_reset_draws* draws, int32_t variable_n, uint64_t seed, int64_t env_offset,
             void* stream) {
  Geometry g;
  const Kernels* k;
  const uint32_t* tab;
  int rc = prepare(cfg, B, stream, &g, &k, &tab);
  if (rc) return rc;
  if (B == 0) return WH_OK;
  if (!state) return WH_EINVAL;
  if (draws && (!draws->spawn || !draws->pickups || !draws->targets)) return WH_EINVAL;
  ResetParams a{state, B, g.NA, g.W, tab, mask,
                draws ? draws->spawn : nullptr, draws ? draws->pickups : nullptr,
                draws ? draws->targets : nullptr, draws ? draws->n : nullptr,
                draws ? 1 : 0, variable_n ? 1 : 0,
                (uint32_t)(seed & 0xFFFFFFFFu), (uint32_t)(seed >> 32), env_offset};
  hipLaunchKernelGGL(k->reset, grid_for(B), dim3(BT), 0, (hipStream_t)stream, a);
  return hip_err(hipGetLastError());
}

}  // extern "C"

// A step launch with every argument resolved: what launch_step enqueues, and what a prepared
// launch (wh_rollout_prepare / wh_launch_run) replays without re-validating anything.
struct wh_launch {
  void (*kern)(StepParams);
  dim3 grid;
  hipStream_t stream;
  StepParams a;
};

// Live handles of wh_rollout_prepare: run / free of anything else (a freed or foreign pointer) is
// refused with WH_EINVAL instead of being dereferenced.
static std::mutex g_launch_mu;
static std::unordered_set<const wh_launch*> g_launches;
static bool launch_live(const wh_launch* l) {
  std::lock_guard<std::mutex> lk(g_launch_mu);
  return g_launches.count(l) != 0;
}

static int resolve_step(const wh_config* cfg, int64_t B, uint32_t* state, int policy, StepParams a,
                        void* stream, wh_launch* out) {
  Geometry g;
  const Kernels* k;
  const uint32_t* tab;
  // host-side argument checks first (no device needed to refuse them)
  int rc = validate(cfg, &g);
  if (rc) return rc;
  if (policy < 0 || policy > 2) return WH_EINVAL;
  if (B > 0 && !state) return WH_EINVAL;
  // order rows: 0 = NA entries, else 1 .. 4 * NA (every key form of every agent, core.py:280)
  if (a.ol == 0) a.ol = g.NA;
  if (a.ol < 1 || a.ol > 4 * g.NA) return WH_EINVAL;
  rc = prepare(cfg, B, stream, &g, &k, &tab);
  if (rc) return rc;
  a.state = state;
  a.B = B;
  a.na = g.NA;
  a.T = g.T;
  a.W = g.W;
  a.tables = tab;
#ifdef WH_ABLATION
  const char* abl = getenv("WH_ABLATE");   // timing experiments only (tools/ablate.py)
  a.ablate = abl ? atoi(abl) : 0;
#endif
  void (*kern)(StepParams) = (a.order != nullptr && policy == POL_EXTERNAL) ? k->step_ordered : k->step[policy];
  // the fused rollout's common case (run_steps_fast); rows of 16 (NAM % 4 == 0) or 8 bytes
  const uintptr_t ralign = (k->NAM % 4 == 0) ? 15u : 7u;
  if (k->step_fast[policy] && a.phase == PH_ALL && a.rewards && a.dones && !a.returns &&
      !a.stats.episode_return && !a.mask && !a.order && !a.regen && !a.n_inactive && a.autoreset &&
      g.NA == k->NAM && ((uintptr_t)a.rewards & ralign) == 0)
    kern = k->step_fast[policy];
  out->kern = kern;
  out->grid = grid_for(B);
  out->stream = (hipStream_t)stream;
  out->a = a;
  return WH_OK;
}

static int enqueue(const wh_launch& l) {
  if (l.a.B == 0) return WH_OK;
  hipLaunchKernelGGL(l.kern, l.grid, dim3(BT), 0, l.stream, l.a);
  return hip_err(hipGetLastError());
}

static int launch_step(const wh_config* cfg, int64_t B, uint32_t* state, int policy,
                       StepParams a, void* stream) {
  wh_launch l;
  const int rc = resolve_step(cfg, B, state, policy, a, stream, &l);
  return rc ? rc : enqueue(l);
}

extern "C" {

int wh_step(const wh_config* cfg, int64_t B, uint32_t* state, const int32_t* actions,
            const int32_t* order, int32_t order_len, float* rewards, uint8_t* dones, const int32_t* regen,
            int32_t* n_inactive, int32_t phase, uint64_t seed, int64_t env_offset, void* stream) {
  if (phase < WH_PHASE_ALL || phase > WH_PHASE_REGEN) return WH_EINVAL;
  if (B > 0 && phase != WH_PHASE_REGEN && !actions) return WH_EINVAL;
  StepParams a{};
  a.actions = actions;
  a.order = order;
  a.ol = order_len;
  a.rewards = rewards;
  a.dones = dones;
  a.regen = regen;
  a.n_inactive = n_inactive;
  a.k0 = (uint32_t)(seed & 0xFFFFFFFFu);
  a.k1 = (uint32_t)(seed >> 32);
  a.env_offset = env_offset;
  a.steps = 1;
  a.phase = phase;
  return launch_step(cfg, B, state, POL_EXTERNAL, a, stream);
}

int wh_policy(const wh_config* cfg, int64_t B, const uint32_t* state, int32_t policy, float p,
              int32_t* actions, uint64_t seed, int64_t env_offset, void* stream) {
  if ((policy != WH_POLICY_GREEDY && policy != WH_POLICY_RANDOM) || (B > 0 && !actions)) return WH_EINVAL;
  if (!(p >= 0.0f && p <= 1.0f)) return WH_EINVAL;
  StepParams a{};
  a.actions_out = actions;
  a.p = p;
  a.k0 = (uint32_t)(seed & 0xFFFFFFFFu);
  a.k1 = (uint32_t)(seed >> 32);
  a.env_offset = env_offset;
  a.steps = 0;
  a.phase = PH_POLICY;
  return launch_step(cfg, B, const_cast<uint32_t*>(state), policy, a, stream);
}

static bool stats_ok(const wh_episode_stats* st) {
  return !st || st->episode_return || (!st->return_sum && !st->episodes && !st->return_min && !st->return_max);
}

int wh_rollout(const wh_config* cfg, int64_t B, uint32_t* state, int32_t steps, int32_t policy,
               float p, float* rewards, uint8_t* dones, float* returns, const wh_episode_stats* stats,
               int32_t autoreset, int32_t variable_n, uint64_t seed, int64_t env_offset, void* stream) {
  if ((policy != WH_POLICY_GREEDY && policy != WH_POLICY_RANDOM) || steps < 0) return WH_EINVAL;
  if (!(p >= 0.0f && p <= 1.0f) || !stats_ok(stats)) return WH_EINVAL;
  StepParams a{};
  if (stats) a.stats = *stats;
  a.rewards = rewards;
  a.dones = dones;
  a.returns = returns;
  a.p = p;
  a.k0 = (uint32_t)(seed & 0xFFFFFFFFu);
  a.k1 = (uint32_t)(seed >> 32);
  a.env_offset = env_offset;
  a.steps = steps;
  a.phase = PH_ALL;
  a.autoreset = autoreset ? 1 : 0;
  a.variable_n = variable_n ? 1 : 0;
  return launch_step(cfg, B, state, policy, a, stream);
}

int wh_rollout_prepare(const wh_config* cfg, int64_t B, uint32_t* state, int32_t steps, int32_t policy,
                       float p, float* rewards, uint8_t* dones, float* returns, const wh_episode_stats* stats,
                       int32_t autoreset, int32_t variable_n, uint64_t seed, int64_t env_offset, void* stream,
                       wh_launch** out) {
  if (!out) return WH_EINVAL;
  *out = nullptr;
  if ((policy != WH_POLICY_GREEDY && policy != WH_POLICY_RANDOM) || steps < 0) return WH_EINVAL;
  if (!(p >= 0.0f && p <= 1.0f) || !stats_ok(stats)) return WH_EINVAL;
  StepParams a{};
  if (stats) a.stats = *stats;
  a.rewards = rewards;
  a.dones = dones;
  a.returns = returns;
  a.p = p;
  a.k0 = (uint32_t)(seed & 0xFFFFFFFFu);
  a.k1 = (uint32_t)(seed >> 32);
  a.env_offset = env_offset;
  a.steps = steps;
  a.phase = PH_ALL;
  a.autoreset = autoreset ? 1 : 0;
  a.variable_n = variable_n ? 1 : 0;
  wh_launch* l = new (std::nothrow) wh_launch;
  if (!l) return WH_EINVAL;
  const int rc = resolve_step(cfg, B, state, policy, a, stream, l);
  if (rc) {
    delete l;
    return rc;
  }
  {
    std::lock_guard<std::mutex> lk(g_launch_mu);
    g_launches.insert(l);
  }
  *out = l;
  return WH_OK;
}

int wh_launch_run(const wh_launch* l) { return launch_live(l) ? enqueue(*l) : WH_EINVAL; }

int wh_launch_run_timed(const wh_launch* l, void* start_event, void* stop_event) {
  if (!launch_live(l)) return WH_EINVAL;
  if (l->a.B == 0) return WH_OK;
  StepParams a = l->a;
  void* args[] = {&a};
  return hip_err(hipExtLaunchKernel(reinterpret_cast<const void*>(l->kern), l->grid, dim3(BT), args, 0,
                                    l->stream, (hipEvent_t)start_event, (hipEvent_t)stop_event, 0));
}

int wh_launch_free(wh_launch* l) {
  if (!l) return WH_OK;
  {
    std::lock_guard<std::mutex> lk(g_launch_mu);
    if (!g_launches.erase(l)) return WH_EINVAL;   // not a live handle: never prepared, or freed already
  }
  delete l;
  return WH_OK;
}

static int observe_impl(const wh_config* cfg, int64_t B, const uint32_t* state, float* obs, void* xfrag,
                        void* stream) {
  Geometry g;
  const Kernels* k;
  const uint32_t* tab;
  int rc = prepare(cfg, B, stream, &g, &k, &tab);
  if (rc) return rc;
  if (B == 0) return WH_OK;
  if (!state || (!obs && !xfrag)) return WH_EINVAL;
  const int quads = ((g.NA * (9 * g.R + 1)) % 4 == 0) && ((uintptr_t)obs % 16 == 0);
  // envs per workgroup (same-box A/Bs, tools/obs_bench.py and tools/sampler_probe.py): f32 rows 64
  // for Small-4's 592 B/env rows, 16 for Medium-8's 2.6 KB, 4 for Large-16's 9.3 KB
  // (profiles/r05_obseb0_ab.txt: 8 -> 4 is 119.5 -> 115.2 us, and 133 -> 130 us for the sampler
  // route, profiles/r05_obseb1_ab.txt 120.6 -> 114.8 us); the fragment operand alone 64 / 16 / 8
  // (Large-16: 16 is 3 % and 4 is 20 % slower than 8, profiles/r05_obseb1_ab.txt / r05_obseb0_ab.txt)
  const int row_bytes = 4 * g.NA * (9 * g.R + 1);
  int sel = row_bytes <= 1024 ? 3 : (row_bytes <= 4096 ? 2 : (obs ? 0 : 1));
  if (xfrag && (uintptr_t)xfrag % 16 != 0) return WH_EINVAL;
  // the fragment operand is written in whole 32-row tiles per workgroup: groups of 64 envs hold
  // 64 * NA rows, a multiple of 32 for every agent count (e.g. Medium with 9 agents, whose f32-row
  // grouping of 16 envs = 144 rows does not)
  if (xfrag && (kObsEB[sel] * g.NA) % 32 != 0) sel = 3;
  const int ebx = kObsEB[sel];
  const int64_t qe = (int64_t)g.NA * (9 * g.R + 1) / 4;
  if (sel == 0 && !xfrag && quads && k->observe_chunk && kObsChunk <= (ebx - 1) * qe + 1) {
    hipLaunchKernelGGL(k->observe_chunk, dim3((unsigned)((B * qe + kObsChunk - 1) / kObsChunk)), dim3(BT), 0,
                       (hipStream_t)stream, state, B, g.NA, tab, obs, quads, static_cast<uint4*>(xfrag));
    return hip_err(hipGetLastError());
  }
  hipLaunchKernelGGL(k->observe[sel], dim3((unsigned)((B + ebx - 1) / ebx)), dim3(BT), 0,
                     (hipStream_t)stream, state, B, g.NA, tab, obs, quads, static_cast<uint4*>(xfrag));
  return hip_err(hipGetLastError());
}

int wh_observe(const wh_config* cfg, int64_t B, const uint32_t* state, float* obs, void* stream) {
  return observe_impl(cfg, B, state, obs, nullptr, stream);
}

int wh_observe_x(const wh_config* cfg, int64_t B, const uint32_t* state, float* obs, void* xfrag, void* stream) {
  return observe_impl(cfg, B, state, obs, xfrag, stream);
}

int wh_vector_step(const wh_config* cfg, int64_t B, uint32_t* state, const int32_t* actions,
                   const int32_t* order, int32_t order_len, const uint8_t* mask, float* rewards, uint8_t* dones,
                   float* obs, const wh_episode_stats* stats, int32_t autoreset, int32_t variable_n,
                   uint64_t seed, int64_t env_offset, void* stream) {
  if (B > 0 && !actions) return WH_EINVAL;
  if (!stats_ok(stats)) return WH_EINVAL;
  StepParams a{};
  a.actions = actions;
  a.order = order;   // non-NULL: the action-dict order path (k_step<..., ORDERED>), as wh_step
  a.ol = order_len;
  a.mask = mask;
  a.rewards = rewards;
  a.dones = dones;
  a.k0 = (uint32_t)(seed & 0xFFFFFFFFu);
  a.k1 = (uint32_t)(seed >> 32);
  a.env_offset = env_offset;
  a.steps = 1;
  a.phase = PH_ALL;
  a.autoreset = autoreset ? 1 : 0;
  a.variable_n = variable_n ? 1 : 0;
  if (stats) a.stats = *stats;
  wh_launch l;
  int rc = resolve_step(cfg, B, state, POL_EXTERNAL, a, stream, &l);
  if (rc) return rc;
  // one launch (k_sampler's generic instance: the step on half of each workgroup, every env's rows
  // by all of it) when its step code keeps its registers and the rows are whole float4s
  static const bool unfused = getenv("WH_SAMPLER_UNFUSED") != nullptr;
  Geometry g;
  const Kernels* k = nullptr;
  const uint32_t* tab = nullptr;
  if (obs && !unfused && B > 0 && prepare(cfg, B, stream, &g, &k, &tab) == WH_OK && fuse_rows(g)) {
    // the fast instance when the step resolved to it (every env stepped in ascending order, no
    // metrics, auto-reset: RLlib's common case), else the generic one
    void (*fk)(StepParams, float*) = (l.kern == k->step_fast[0] && k->sampler[0]) ? k->sampler[0] : k->vsampler[order ? 1 : 0];
    if (fk && fused_ok(fk) && (g.NA * (9 * g.R + 1)) % 4 == 0 && (uintptr_t)obs % 16 == 0) {
      hipLaunchKernelGGL(fk, grid_for(B), dim3(2 * BT), 0, l.stream, l.a, obs);
      return hip_err(hipGetLastError());
    }
  }
  rc = enqueue(l);
  if (rc || !obs) return rc;
  return wh_observe(cfg, B, state, obs, stream);
}

// wh_vector_step with the rows written as the policy network's fragment-order operand (the policy
// route, scripts/rollout.py:72 -> env.step): the step launch, then wh_observe_x.  (k_sampler writing
// the operand from its images in the step launch ran 1.8 % slower per policy step than the two
// launches, profiles/r05_vsx_ab.txt: the operand's per-byte gathers at 8 waves per CU against
// k_observe's full occupancy.)
int wh_vector_step_x(const wh_config* cfg, int64_t B, uint32_t* state, const int32_t* actions,
                     const int32_t* order, int32_t order_len, const uint8_t* mask, float* rewards, uint8_t* dones,
                     void* xfrag, const wh_episode_stats* stats, int32_t autoreset, int32_t variable_n,
                     uint64_t seed, int64_t env_offset, void* stream) {
  if (B > 0 && (!actions || !xfrag)) return WH_EINVAL;
  if ((uintptr_t)xfrag % 16 != 0 || !stats_ok(stats)) return WH_EINVAL;
  StepParams a{};
  a.actions = actions;
  a.order = order;
  a.ol = order_len;
  a.mask = mask;
  a.rewards = rewards;
  a.dones = dones;
  a.k0 = (uint32_t)(seed & 0xFFFFFFFFu);
  a.k1 = (uint32_t)(seed >> 32);
  a.env_offset = env_offset;
  a.steps = 1;
  a.phase = PH_ALL;
  a.autoreset = autoreset ? 1 : 0;
  a.variable_n = variable_n ? 1 : 0;
  if (stats) a.stats = *stats;
  wh_launch l;
  int rc = resolve_step(cfg, B, state, POL_EXTERNAL, a, stream, &l);
  if (rc) return rc;
  if (B == 0) return WH_OK;
  rc = enqueue(l);
  if (rc) return rc;
  return wh_observe_x(cfg, B, state, nullptr, xfrag, stream);
}

int wh_sampler_step(const wh_config* cfg, int64_t B, uint32_t* state, int32_t policy, float p,
                    float* rewards, uint8_t* dones, float* obs, const wh_episode_stats* stats,
                    int32_t variable_n, uint64_t seed, int64_t env_offset, void* stream) {
  if (policy != WH_POLICY_GREEDY && policy != WH_POLICY_RANDOM) return WH_EINVAL;
  if (!(p >= 0.0f && p <= 1.0f) || !stats_ok(stats)) return WH_EINVAL;
  StepParams a{};
  if (stats) a.stats = *stats;
  a.rewards = rewards;
  a.dones = dones;
  a.p = p;
  a.k0 = (uint32_t)(seed & 0xFFFFFFFFu);
  a.k1 = (uint32_t)(seed >> 32);
  a.env_offset = env_offset;
  a.steps = 1;
  a.phase = PH_ALL;
  a.autoreset = 1;
  a.variable_n = variable_n ? 1 : 0;
  wh_launch l;
  int rc = resolve_step(cfg, B, state, policy, a, stream, &l);
  if (rc) return rc;
  // One launch (k_sampler: the fused rollout's step on half of each workgroup, then the rows by
  // all of it) when the fast step instance applies and the rows are whole float4s; otherwise the
  // step launch and k_observe.  WH_SAMPLER_UNFUSED=1 forces the two launches (A/B runs).
  static const bool unfused = getenv("WH_SAMPLER_UNFUSED") != nullptr;
  Geometry g;
  const Kernels* k = nullptr;
  const uint32_t* tab = nullptr;
  if (obs && !unfused && B > 0 && prepare(cfg, B, stream, &g, &k, &tab) == WH_OK && fuse_rows(g) && l.kern == k->step_fast[policy] &&
      k->sampler[policy] && fused_ok(k->sampler[policy]) && (g.NA * (9 * g.R + 1)) % 4 == 0 && (uintptr_t)obs % 16 == 0) {
    hipLaunchKernelGGL(k->sampler[policy], grid_for(B), dim3(2 * BT), 0, l.stream, l.a, obs);
    return hip_err(hipGetLastError());
  }
  rc = enqueue(l);
  if (rc || !obs) return rc;
  return wh_observe(cfg, B, state, obs, stream);
}

int wh_sampler_rollout(const wh_config* cfg, int64_t B, uint32_t* state, int32_t steps, int32_t policy, float p,
                       float* rewards, uint8_t* dones, float* obs, const wh_episode_stats* stats, int32_t variable_n,
                       uint64_t seed, int64_t env_offset, void* stream) {
  if (policy != WH_POLICY_GREEDY && policy != WH_POLICY_RANDOM) return WH_EINVAL;
  if (steps < 0 || !(p >= 0.0f && p <= 1.0f) || !stats_ok(stats)) return WH_EINVAL;
  if (B > 0 && steps > 0 && !obs) return WH_EINVAL;
  StepParams a{};
  if (stats) a.stats = *stats;
  a.rewards = rewards;
  a.dones = dones;
  a.p = p;
  a.k0 = (uint32_t)(seed & 0xFFFFFFFFu);
  a.k1 = (uint32_t)(seed >> 32);
  a.env_offset = env_offset;
  a.steps = steps;
  a.phase = PH_ALL;
  a.autoreset = 1;
  a.variable_n = variable_n ? 1 : 0;
  wh_launch l;
  int rc = resolve_step(cfg, B, state, policy, a, stream, &l);
  if (rc || B == 0 || steps == 0) return rc;
  Geometry g;
  const Kernels* k = nullptr;
  const uint32_t* tab = nullptr;
  if ((rc = prepare(cfg, B, stream, &g, &k, &tab)) != WH_OK) return rc;
  static const bool unfused = getenv("WH_SAMPLER_UNFUSED") != nullptr;
  void (*fk)(StepParams, float*) = steps == 1 ? k->sampler[policy] : k->sampler_multi[policy];
  if (!unfused && fuse_rows(g) && l.kern == k->step_fast[policy] && fk && fused_ok(fk) && (g.NA * (9 * g.R + 1)) % 4 == 0 &&
      (uintptr_t)obs % 16 == 0) {
    hipLaunchKernelGGL(fk, grid_for(B), dim3(2 * BT), 0, l.stream, l.a, obs);
    return hip_err(hipGetLastError());
  }
  // otherwise: the same steps one launch (pair) at a time
  const int64_t rows = B * (int64_t)g.NA * (9 * g.R + 1);
  for (int32_t t = 0; t < steps && rc == WH_OK; ++t)
    rc = wh_sampler_step(cfg, B, state, policy, p, rewards ? rewards + (int64_t)t * B * g.NA : nullptr,
                         dones ? dones + (int64_t)t * B : nullptr, obs + (int64_t)t * rows, stats, variable_n, seed,
                         env_offset, stream);
  return rc;
}

int wh_sampler_step_to(const wh_config* cfg, int64_t B, const uint32_t* state_in, uint32_t* state_out,
                       int32_t policy, float p, float* rewards, uint8_t* dones, const wh_episode_stats* stats,
                       int32_t variable_n, uint64_t seed, int64_t env_offset, void* stream) {
  if (policy != WH_POLICY_GREEDY && policy != WH_POLICY_RANDOM) return WH_EINVAL;
  if (!(p >= 0.0f && p <= 1.0f) || !stats_ok(stats)) return WH_EINVAL;
  if (B > 0 && !state_out) return WH_EINVAL;
  StepParams a{};
  if (stats) a.stats = *stats;
  a.rewards = rewards;
  a.dones = dones;
  a.p = p;
  a.k0 = (uint32_t)(seed & 0xFFFFFFFFu);
  a.k1 = (uint32_t)(seed >> 32);
  a.env_offset = env_offset;
  a.steps = 1;
  a.phase = PH_ALL;
  a.autoreset = 1;
  a.variable_n = variable_n ? 1 : 0;
  a.state_out = state_out;   // every env is live (no mask): each lane stores its whole state
  return launch_step(cfg, B, const_cast<uint32_t*>(state_in), policy, a, stream);
}

}  // extern "C"
