// warehouse_amd.hip -- gfx950 kernels + C ABI for the batched warehouse hot path.
//
// Design (DESIGN.md has the full rationale and measurements):
//  * ONE LANE PER ENV.  The per-env work of core.py:262-442 is a short, mostly serial integer
//    program (sequential collision resolution over agents, core.py:279-300).  Putting one env on
//    one lane and the batch across lanes makes every HBM access a fully coalesced word-plane
//    (state[w * B + e]) and shares each issued instruction among 64 envs.
//  * SWAR on packed bytes.  Pickup tables are 1 byte per point, 4 per register: expiry
//    (core.py:303-306), pickup clearing and regeneration masks (core.py:330-351) run 4 points per
//    VALU op; active/inactive sets are 64-bit masks (P <= 64).
//  * v_sad_u8 for the greedy policy: |dx|+|dy| of byte-packed (x,y) in one instruction
//    (solvers.py:53-58), argmin-first-wins as a v_min over (dist << 24 | index << 16 | xy).
//  * Per-lane LDS scratch for the few data-dependent lookups (occupancy grid bits core.py:275-291,
//    pickup target bytes core.py:327-329), laid out [word][lane] so every lane hits its own bank.
//  * Counter-based Philox streams (no RNG state in HBM) or injected draws (parity mode).
#include <hip/hip_runtime.h>

#include <mutex>
#include <stdint.h>
#include <string.h>
#include <vector>

#include "warehouse_amd.h"

namespace {

constexpr int BT = 256;  // lanes (= envs) per workgroup

enum Policy { POL_EXTERNAL = 0, POL_GREEDY = 1, POL_RANDOM = 2 };
enum Purpose : uint32_t { PUR_RESET = 1, PUR_REGEN = 2, PUR_POLICY = 3, PUR_RANDOM = 4 };
constexpr int PH_ALL = 0, PH_PRE = 1, PH_REGEN = 2, PH_POLICY = 3;

template <int D_, int R_, int NR_, int NAM_>
struct Cfg {
  static constexpr int D = D_, R = R_, NR = NR_, NAM = NAM_;
  static constexpr int P = 4 * NR * NR;
  static constexpr int DP = 4 * (D - 4);
  static constexpr int PW = P / 4;
  static constexpr int GRIDW = (D * D + 31) / 32;
  static constexpr int NV = (D - 2) * (D - 2) - P;      // interior cells that are not pickups
  static constexpr int CELLB = (D * D + 3) & ~3;         // table bytes: cell -> pickup+1
  static constexpr int TBL_BYTES = CELLB + 2 * P + 2 * NV;
  static constexpr int TBLW = (TBL_BYTES + 3) / 4;
  static constexpr int L = 9 * R + 1;                    // observation row length
  static_assert(P <= 64 && DP <= 64, "bitmask sets hold at most 64 points");
  static_assert(NAM <= R, "agents <= requests (core.py:89)");
};

// ----------------------------------------------------------------------------- small helpers
__device__ __forceinline__ uint4 philox10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;   // one v_mad_u64_u32 each
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    c = make_uint4((uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1,
                   (uint32_t)p0);
  }
  return c;
}

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

__device__ __forceinline__ int select_bit64(uint64_t m, uint32_t r) {
  uint32_t w = (uint32_t)m;
  int base = 0;
  uint32_t c = __popc(w);
  if (r >= c) { r -= c; w = (uint32_t)(m >> 32); base = 32; }
  c = __popc(w & 0xFFFFu);
  if (r >= c) { r -= c; w >>= 16; base += 16; }
  c = __popc(w & 0xFFu);
  if (r >= c) { r -= c; w >>= 8; base += 8; }
  c = __popc(w & 0xFu);
  if (r >= c) { r -= c; w >>= 4; base += 4; }
  c = __popc(w & 0x3u);
  if (r >= c) { r -= c; w >>= 2; base += 2; }
  if (r >= (w & 1u)) base += 1;
  return base;
}

// high bit of every nonzero byte
__device__ __forceinline__ uint32_t nz_hi(uint32_t x) {
  return (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
}
// 4 byte-flags (bit 7 of each byte) -> 4-bit nibble
__device__ __forceinline__ uint32_t nib_of(uint32_t hi) { return ((hi >> 7) * 0x00204081u) >> 21 & 0xFu; }
// 4-bit nibble -> 0xFF byte mask
__device__ __forceinline__ uint32_t expand_nib(uint32_t nib) {
  return ((nib * 0x00204081u) & 0x01010101u) * 0xFFu;
}

template <int D>
__device__ __forceinline__ uint32_t delivery_xy(uint32_t d) {  // core.py:178-187
  const uint32_t v = 2 + (d >> 2), side = d & 3u;
  const uint32_t x = (side & 1u) ? (side == 3u ? (uint32_t)(D - 1) : 0u) : v;
  const uint32_t y = (side & 1u) ? v : (side == 2u ? (uint32_t)(D - 1) : 0u);
  return x | (y << 8);
}

template <class C>
struct Regs {
  uint32_t hdr, epi;
  uint32_t ag[C::NAM];
  uint32_t pt[C::PW];
  uint32_t pm[C::PW];
};

template <class C>
struct Lds {
  uint32_t tbl[C::TBLW];
  uint32_t occ[C::GRIDW][BT];
  uint32_t ptl[C::PW][BT];
  uint32_t agl[C::NAM][BT];
  __device__ __forceinline__ uint32_t cell_pickup(uint32_t cell) const {
    return reinterpret_cast<const uint8_t*>(tbl)[cell];
  }
  __device__ __forceinline__ uint32_t pickup_xy(uint32_t j) const {
    return reinterpret_cast<const uint16_t*>(reinterpret_cast<const uint8_t*>(tbl) + C::CELLB)[j];
  }
  __device__ __forceinline__ uint32_t valid_cell(uint32_t v) const {
    return reinterpret_cast<const uint16_t*>(reinterpret_cast<const uint8_t*>(tbl) + C::CELLB +
                                             2 * C::P)[v];
  }
  __device__ __forceinline__ uint8_t* ptl_byte(uint32_t j, int tid) {
    return reinterpret_cast<uint8_t*>(&ptl[j >> 2][tid]) + (j & 3u);
  }
};

template <class C>
__device__ __forceinline__ void load_tables(Lds<C>& L, const uint32_t* __restrict__ tables) {
  for (int w = threadIdx.x; w < C::TBLW; w += BT) L.tbl[w] = tables[w];
}

template <class C>
__device__ __forceinline__ void load_env(Regs<C>& s, const uint32_t* __restrict__ st, int64_t B,
                                         int64_t e, int na) {
  s.hdr = st[e];
  s.epi = st[B + e];
#pragma unroll
  for (int i = 0; i < C::NAM; ++i) s.ag[i] = (i < na) ? st[(2 + i) * B + e] : 0u;
  const int wpt = 2 + na;
#pragma unroll
  for (int w = 0; w < C::PW; ++w) s.pt[w] = st[(wpt + w) * B + e];
#pragma unroll
  for (int w = 0; w < C::PW; ++w) s.pm[w] = st[(wpt + C::PW + w) * B + e];
}

template <class C>
__device__ __forceinline__ void store_env(const Regs<C>& s, uint32_t* __restrict__ st, int64_t B,
                                          int64_t e, int na) {
  st[e] = s.hdr;
  st[B + e] = s.epi;
#pragma unroll
  for (int i = 0; i < C::NAM; ++i)
    if (i < na) st[(2 + i) * B + e] = s.ag[i];
  const int wpt = 2 + na;
#pragma unroll
  for (int w = 0; w < C::PW; ++w) st[(wpt + w) * B + e] = s.pt[w];
#pragma unroll
  for (int w = 0; w < C::PW; ++w) st[(wpt + C::PW + w) * B + e] = s.pm[w];
}

template <class C>
__device__ __forceinline__ uint64_t active_mask(const Regs<C>& s) {
  uint64_t am = 0;
#pragma unroll
  for (int w = 0; w < C::PW; ++w) am |= (uint64_t)nib_of(nz_hi(s.pt[w])) << (4 * w);
  return am;
}

template <int N>
__device__ __forceinline__ uint64_t low_mask() {
  return N >= 64 ? ~0ull : ((1ull << N) - 1ull);
}

// ----------------------------------------------------------------------------- reset
// core.py:167-221 (philox draws): spawn on interior non-pickup cells, open R requests.
template <class C>
__device__ __forceinline__ void reset_philox(Regs<C>& s, Lds<C>& L, const Keys& k, uint32_t gid, int na,
                             int variable_n, uint32_t W, int tid) {
  const uint32_t ep = s.epi + 1u;
  Reader rd(k, gid, ep, 0u, PUR_RESET);
  const uint32_t n = variable_n ? 1u + __umulhi(rd.word(0), (uint32_t)na) : (uint32_t)na;
#pragma unroll
  for (int i = 0; i < C::NAM; ++i) {
    uint32_t a = 0;
    if (i < na) {
      const uint32_t v = __umulhi(rd.word(1 + i), (uint32_t)C::NV);
      a = (i < (int)n) ? L.valid_cell(v) : 0u;
    }
    s.ag[i] = a;
  }
#pragma unroll
  for (int w = 0; w < C::PW; ++w) L.ptl[w][tid] = 0u;
  uint64_t remP = low_mask<C::P>(), remD = low_mask<C::DP>();
  for (int j = 0; j < C::R; ++j) {
    const uint32_t r1 = __umulhi(rd.word(1 + na + 2 * j), (uint32_t)(C::P - j));
    const int sel = select_bit64(remP, r1);
    remP &= ~(1ull << sel);
    const uint32_t r2 = __umulhi(rd.word(2 + na + 2 * j), (uint32_t)(C::DP - j));
    const int tg = select_bit64(remD, r2);
    remD &= ~(1ull << tg);
    *L.ptl_byte((uint32_t)sel, tid) = (uint8_t)(tg + 1);
  }
  const uint64_t opened = low_mask<C::P>() & ~remP;
  const uint32_t wb = W * 0x01010101u;
#pragma unroll
  for (int w = 0; w < C::PW; ++w) {
    s.pt[w] = L.ptl[w][tid];
    s.pm[w] = expand_nib((uint32_t)(opened >> (4 * w)) & 0xFu) & wb;
  }
  s.hdr = (n << 16) | (1u << 24);
  s.epi = ep;
}

template <class C>
__device__ __forceinline__ void reset_injected(Regs<C>& s, Lds<C>& L, int64_t e, int na, const int32_t* spawn,
                               const int32_t* pickups, const int32_t* targets, const int32_t* nn,
                               uint32_t W, int tid) {
  const uint32_t n = nn ? min((uint32_t)nn[e], (uint32_t)na) : (uint32_t)na;
#pragma unroll
  for (int i = 0; i < C::NAM; ++i) {
    uint32_t a = 0;
    if (i < na && i < (int)n) {
      const uint32_t x = min((uint32_t)spawn[(e * na + i) * 2], (uint32_t)(C::D - 1));
      const uint32_t y = min((uint32_t)spawn[(e * na + i) * 2 + 1], (uint32_t)(C::D - 1));
      a = x | (y << 8);
    }
    s.ag[i] = a;
  }
#pragma unroll
  for (int w = 0; w < C::PW; ++w) L.ptl[w][tid] = 0u;
  uint64_t opened = 0;
  for (int j = 0; j < C::R; ++j) {
    const uint32_t sel = (uint32_t)pickups[e * C::R + j];
    const uint32_t tg = (uint32_t)targets[e * C::R + j];
    if (sel >= (uint32_t)C::P || tg >= (uint32_t)C::DP) continue;   // invalid injected draw: ignored
    opened |= 1ull << sel;
    *L.ptl_byte(sel, tid) = (uint8_t)(tg + 1);
  }
  const uint32_t wb = W * 0x01010101u;
#pragma unroll
  for (int w = 0; w < C::PW; ++w) {
    s.pt[w] = L.ptl[w][tid];
    s.pm[w] = expand_nib((uint32_t)(opened >> (4 * w)) & 0xFu) & wb;
  }
  s.hdr = (n << 16) | (1u << 24);
  s.epi = s.epi + 1u;
}

// ----------------------------------------------------------------------------- policy
// baseline/solvers.py:27-58 evaluated on the state: availability 0 (fresh reset or carrying)
// -> head for the own delivery target (the null cell after reset), else for the nearest open
// request by Manhattan distance, first (lowest pickup index) minimum wins; one step = clip(-1,1).
template <class C, int POLICY>
__device__ __forceinline__ void policy_actions(const Regs<C>& s, const Lds<C>& L, const Keys& k,
                                               uint32_t gid, float p, uint32_t (&act)[C::NAM]) {
  const uint32_t t = s.hdr & 0xFFFFu;
  const uint32_t n = (s.hdr >> 16) & 0xFFu;
  if (POLICY == POL_RANDOM) {
#pragma unroll
    for (int b = 0; b < (C::NAM + 3) / 4; ++b) {
      const uint4 blk = stream_block(k, gid, s.epi, t, PUR_RANDOM, (uint32_t)b);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int i = 4 * b + c;
        if (i < C::NAM) act[i] = (i < (int)n) ? __umulhi(comp(blk, c), 9u) : 4u;
      }
    }
    return;
  }
  const bool fresh = (s.hdr >> 24) & 1u;
  // open requests in ascending pickup order (core.py:409-418): tag = index << 16 | xy
  uint32_t rtag[C::R];
  uint64_t m = active_mask(s);
#pragma unroll
  for (int r = 0; r < C::R; ++r) {
    const int j = m ? __builtin_ctzll(m) : 0;
    rtag[r] = m ? (((uint32_t)j << 16) | L.pickup_xy((uint32_t)j)) : 0x00FFFFFFu;
    m &= m - 1ull;
  }
  constexpr uint32_t null_xy = (uint32_t)(C::D / 2) | ((uint32_t)(C::D / 2) << 8);
#pragma unroll
  for (int i = 0; i < C::NAM; ++i) {
    const uint32_t a = s.ag[i];
    const uint32_t pos = a & 0xFFFFu;
    const uint32_t carry = (a >> 16) & 0xFFu;
    uint32_t best = 0xFFFFFFFFu;
#pragma unroll
    for (int r = 0; r < C::R; ++r) {
      const uint32_t d = __builtin_amdgcn_sad_u8(pos, rtag[r] & 0xFFFFu, 0u);
      best = min(best, (d << 24) | rtag[r]);
    }
    uint32_t goal = best & 0xFFFFu;
    if (carry) goal = delivery_xy<C::D>(carry - 1u);
    if (fresh) goal = null_xy;
    const int x = (int)(pos & 0xFFu), y = (int)(pos >> 8);
    const int gx = (int)(goal & 0xFFu), gy = (int)(goal >> 8);
    const int sx = (gx > x) - (gx < x), sy = (gy > y) - (gy < y);
    act[i] = (uint32_t)((sx + 1) * 3 + (sy + 1));
  }
  if (p > 0.0f) {
#pragma unroll
    for (int b = 0; b < (C::NAM + 1) / 2; ++b) {
      const uint4 blk = stream_block(k, gid, s.epi, t, PUR_POLICY, (uint32_t)b);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int i = 2 * b + h;
        if (i < C::NAM) {
          const float u = (float)(comp(blk, 2 * h) >> 8) * (1.0f / 16777216.0f);
          if (u < p) act[i] = __umulhi(comp(blk, 2 * h + 1), 9u);
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < C::NAM; ++i)
    if (i >= (int)n) act[i] = 4u;
}

// ----------------------------------------------------------------------------- step
struct StepOut {
  float* rewards;
  uint8_t* dones;
  int32_t* n_inactive;
};

// core.py:267-368 on one env held in registers.  Returns done.
template <class C>
__device__ __forceinline__ bool step_env(Regs<C>& s, Lds<C>& L, const uint32_t (&act)[C::NAM],
                                         const int32_t* __restrict__ order,
                                         const int32_t* __restrict__ actions_g,
                                         const int32_t* __restrict__ regen, const Keys& k,
                                         uint32_t gid, int64_t e, int na, int phase, uint32_t T,
                                         uint32_t W, float (&rew)[C::NAM], int32_t* n_inactive,
                                         int tid) {
  constexpr int D = C::D;
  const uint32_t n = (s.hdr >> 16) & 0xFFu;
  uint32_t t = s.hdr & 0xFFFFu;

  if (phase != PH_REGEN) {
    t = (t + 1u) & 0xFFFFu;                                 // core.py:267
#pragma unroll
    for (int i = 0; i < C::NAM; ++i) rew[i] = 0.0f;

    // ---- move + collision, sequential in action-dict order (core.py:275-300)
#pragma unroll
    for (int w = 0; w < C::GRIDW; ++w) L.occ[w][tid] = 0u;
#pragma unroll
    for (int i = 0; i < C::NAM; ++i) {
      if (i < (int)n) {
        const uint32_t c = (s.ag[i] & 0xFFu) * D + ((s.ag[i] >> 8) & 0xFFu);
        atomicOr(&L.occ[c >> 5][tid], 1u << (c & 31u));
      }
    }
    const bool ordered = order != nullptr;
    if (ordered) {
#pragma unroll
      for (int i = 0; i < C::NAM; ++i) L.agl[i][tid] = s.ag[i];
    }
    uint32_t kk[3 * C::NAM];
#pragma unroll
    for (int j = 0; j < 3 * C::NAM; ++j) kk[j] = 0xFFFFFFFFu;
#pragma unroll
    for (int sidx = 0; sidx < C::NAM; ++sidx) {
      bool live;
      uint32_t a, mv;
      int who = sidx;
      if (ordered) {
        who = (sidx < na) ? order[e * na + sidx] : -1;
        live = who >= 0 && who < (int)n && who < C::NAM;
        who = live ? who : 0;
        a = L.agl[who][tid];
        mv = live ? (uint32_t)actions_g[e * na + who] : 4u;
      } else {
        live = sidx < (int)n;
        a = s.ag[sidx];
        mv = act[sidx];
      }
      mv = mv > 8u ? 4u : mv;
      const int px = (int)(a & 0xFFu), py = (int)((a >> 8) & 0xFFu);
      const int q = (int)((mv * 11u) >> 5);                 // mv / 3 for mv <= 8
      int x = px + q - 1, y = py + (int)mv - 3 * q - 1;     // MOVES[a] = (a//3-1, a%3-1)
      if ((unsigned)x >= (unsigned)D) x = px;
      if ((unsigned)y >= (unsigned)D) y = py;
      const uint32_t cn = (uint32_t)(x * D + y);
      const bool occupied = (L.occ[cn >> 5][tid] >> (cn & 31u)) & 1u;
      const uint32_t key = (uint32_t)px | ((uint32_t)py << 8) | ((uint32_t)x << 16) | ((uint32_t)y << 24);
      bool forbidden = false;
#pragma unroll
      for (int j = 0; j < 3 * sidx; ++j) forbidden |= (kk[j] == key);
      if (live && !occupied && !forbidden) {
        const uint32_t co = (uint32_t)(px * D + py);
        atomicAnd(&L.occ[co >> 5][tid], ~(1u << (co & 31u)));
        atomicOr(&L.occ[cn >> 5][tid], 1u << (cn & 31u));
        kk[3 * sidx] = (uint32_t)x | ((uint32_t)y << 8) | ((uint32_t)px << 16) | ((uint32_t)py << 24);
        if (x != px && y != py) {
          kk[3 * sidx + 1] = (uint32_t)x | ((uint32_t)py << 8) | ((uint32_t)px << 16) | ((uint32_t)y << 24);
          kk[3 * sidx + 2] = (uint32_t)px | ((uint32_t)y << 8) | ((uint32_t)x << 16) | ((uint32_t)py << 24);
        }
        const uint32_t na_ = (a & 0xFFFF0000u) | (uint32_t)x | ((uint32_t)y << 8);
        if (ordered)
          L.agl[who][tid] = na_;
        else
          s.ag[sidx] = na_;
      }
    }
    if (ordered) {
#pragma unroll
      for (int i = 0; i < C::NAM; ++i) s.ag[i] = L.agl[i][tid];
    }

    // ---- request expiry (core.py:303-306), 4 pickup points per op
#pragma unroll
    for (int w = 0; w < C::PW; ++w) {
      const uint32_t live = nz_hi(s.pt[w]);
      uint32_t tm = s.pm[w] - (live >> 7);
      const uint32_t zero = ~((((tm & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | tm)) & 0x80808080u;
      const uint32_t m = ((zero & live) >> 7) * 0xFFu;
      s.pt[w] &= ~m;
      s.pm[w] = tm & ~m;
    }

    // ---- pickups: gather for every agent against the pre-pickup table, then clear
    //      (core.py:309-335; two agents on one point both pick it up)
#pragma unroll
    for (int w = 0; w < C::PW; ++w) L.ptl[w][tid] = s.pt[w];
    uint64_t picked = 0;
#pragma unroll
    for (int i = 0; i < C::NAM; ++i) {
      const uint32_t a = s.ag[i];
      const uint32_t cell = (a & 0xFFu) * D + ((a >> 8) & 0xFFu);
      const uint32_t cp = L.cell_pickup(cell);
      if (i < (int)n && cp != 0u && ((a >> 16) & 0xFFu) == 0u) {
        const uint32_t tg = *L.ptl_byte(cp - 1u, tid);
        if (tg) {
          s.ag[i] = a | (tg << 16);
          picked |= 1ull << (cp - 1u);
          rew[i] = 1.0f;
        }
      }
    }
#pragma unroll
    for (int w = 0; w < C::PW; ++w) {
      const uint32_t m = expand_nib((uint32_t)(picked >> (4 * w)) & 0xFu);
      s.pt[w] &= ~m;
      s.pm[w] &= ~m;
    }
  }

  // ---- regeneration: reopen k = R - P + |inactive| points (core.py:338-351)
  {
    const uint64_t inactive = ~active_mask(s) & low_mask<C::P>();
    const uint32_t nin = (uint32_t)__popcll(inactive);
    const int kreq = C::R - C::P + (int)nin;
    if (phase == PH_PRE) {
      if (n_inactive) n_inactive[e] = (int32_t)nin;
    } else {
      uint64_t rem = inactive, used = 0, opened = 0;
      const uint32_t tnew = t;
      uint4 blk = make_uint4(0u, 0u, 0u, 0u);   // words 2j (pickup) and 2j+1 (target) share a block
#pragma unroll
      for (int j = 0; j < C::R; ++j) {
        if (j < kreq) {
          int sel, tg;
          if (regen) {
            const uint32_t rp = (uint32_t)regen[e * 2 * C::R + j];
            sel = rp < nin ? select_bit64(inactive, rp) : C::P;       // out-of-range draw: ignored
            tg = regen[e * 2 * C::R + C::R + j];
            if ((uint32_t)tg >= (uint32_t)C::DP) sel = C::P;
          } else {
            if ((j & 1) == 0) blk = stream_block(k, gid, s.epi, tnew, PUR_REGEN, (uint32_t)(j >> 1));
            const uint32_t w1 = comp(blk, (2 * j) & 3), w2 = comp(blk, (2 * j + 1) & 3);
            sel = select_bit64(rem, __umulhi(w1, nin - (uint32_t)j));
            rem &= ~(1ull << sel);
            tg = select_bit64(~used & low_mask<C::DP>(), __umulhi(w2, (uint32_t)(C::DP - j)));
            used |= 1ull << tg;
          }
          if (sel < C::P) {
            opened |= 1ull << sel;
            *L.ptl_byte((uint32_t)sel, tid) = (uint8_t)(tg + 1);
          }
        }
      }
      if (opened) {
        const uint32_t wb = W * 0x01010101u;
#pragma unroll
        for (int w = 0; w < C::PW; ++w) {
          const uint32_t m = expand_nib((uint32_t)(opened >> (4 * w)) & 0xFu);
          if (m) {
            s.pt[w] = (s.pt[w] & ~m) | (L.ptl[w][tid] & m);
            s.pm[w] = (s.pm[w] & ~m) | (wb & m);
          }
        }
      }
    }
  }

  bool done = false;
  if (phase != PH_REGEN) {
    // ---- deliveries (core.py:354-368)
#pragma unroll
    for (int i = 0; i < C::NAM; ++i) {
      const uint32_t a = s.ag[i];
      const uint32_t carry = (a >> 16) & 0xFFu;
      if (carry && delivery_xy<C::D>(carry - 1u) == (a & 0xFFFFu)) {
        s.ag[i] = a & 0xFF00FFFFu;
        rew[i] += 1.0f;
      }
    }
    done = t >= T;                                            // core.py:438
    s.hdr = t | (n << 16);                                    // clears `fresh`
  }
  return done;
}

// ----------------------------------------------------------------------------- kernels
struct StepParams {
  uint32_t* state;
  int64_t B;
  int32_t na, T, W;
  const uint32_t* tables;
  const int32_t* actions;
  const int32_t* order;
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
};

template <class C, int POLICY>
__global__ __launch_bounds__(BT) void k_step(StepParams a) {
  __shared__ Lds<C> L;
  load_tables<C>(L, a.tables);
  __syncthreads();
  const int tid = threadIdx.x;
  const int64_t e = (int64_t)blockIdx.x * BT + tid;
  if (e >= a.B) return;
  const Keys k{a.k0, a.k1};
  const uint32_t gid = (uint32_t)(a.env_offset + e);
  Regs<C> s;
  load_env<C>(s, a.state, a.B, e, a.na);

  if (a.phase == PH_POLICY) {
    uint32_t act[C::NAM];
    policy_actions<C, POLICY>(s, L, k, gid, a.p, act);
#pragma unroll
    for (int i = 0; i < C::NAM; ++i)
      if (i < a.na) a.actions_out[e * a.na + i] = (int32_t)act[i];
    return;
  }

  float ret = 0.0f;
  for (int stp = 0; stp < a.steps; ++stp) {
    uint32_t act[C::NAM];
    if (POLICY == POL_EXTERNAL) {
      const bool have = a.phase != PH_REGEN && a.order == nullptr;   // REGEN reads no actions
#pragma unroll
      for (int i = 0; i < C::NAM; ++i) act[i] = (have && i < a.na) ? (uint32_t)a.actions[e * a.na + i] : 4u;
    } else {
      policy_actions<C, POLICY>(s, L, k, gid, a.p, act);
    }
    float rew[C::NAM];
    const bool done = step_env<C>(s, L, act, a.order, a.actions, a.regen, k, gid, e, a.na, a.phase,
                                  (uint32_t)a.T, (uint32_t)a.W, rew, a.n_inactive, tid);
    if (a.phase != PH_REGEN) {
      if (a.rewards) {
        float* rp = a.rewards + ((int64_t)stp * a.B + e) * a.na;
#pragma unroll
        for (int i = 0; i < C::NAM; ++i)
          if (i < a.na) rp[i] = rew[i];
      }
      if (a.dones) a.dones[(int64_t)stp * a.B + e] = done ? 1 : 0;
      if (a.returns) {
#pragma unroll
        for (int i = 0; i < C::NAM; ++i) ret += rew[i];
      }
      if (done && a.autoreset) reset_philox<C>(s, L, k, gid, a.na, a.variable_n, (uint32_t)a.W, tid);
    }
  }
  if (a.returns) a.returns[e] += ret;
  store_env<C>(s, a.state, a.B, e, a.na);
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
  load_tables<C>(L, a.tables);
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
  store_env<C>(s, a.state, a.B, e, a.na);
}

// Observation rows: build a per-env byte image whose layout equals one row's value pool, then
// every output float is img[desc(f) + row-adjust(i)] -- no per-feature branching.
//   image bytes: [0] n, [1..R] availability, then R x (x,y) delivery targets, R x (x,y)
//   positions, R x (px,py,dx,dy) requests.
constexpr int OBS_EB = 64;  // envs per workgroup

template <class C>
struct ObsLds {
  static constexpr int IMG = (C::L + 3) & ~3;
  uint8_t img[OBS_EB][IMG];
  uint8_t fresh[OBS_EB];
  uint32_t desc[C::L];
};

template <class C>
__global__ __launch_bounds__(BT) void k_observe(const uint32_t* __restrict__ state, int64_t B, int na,
                                                const uint32_t* __restrict__ tables,
                                                float* __restrict__ obs) {
  __shared__ ObsLds<C> O;
  __shared__ uint32_t tbl[C::TBLW];
  constexpr int R = C::R, D = C::D;
  constexpr int A0 = 1, G0 = 1 + R, P0 = 1 + 3 * R, Q0 = 1 + 5 * R;
  const int tid = threadIdx.x;
  for (int w = tid; w < C::TBLW; w += BT) tbl[w] = tables[w];
  // feature descriptors: base | stride << 10 | mode << 14 | j << 16
  //   mode 0: fixed byte; 1: other row skip i; 2: other row skip (fresh ? i : 1); 3: own row
  for (int f = tid; f < C::L; f += BT) {
    uint32_t base, stride = 0, mode = 0, j = 0;
    if (f == 0) { base = 0; }
    else if (f < R) { j = f - 1; base = A0; stride = 1; mode = 1; }
    else if (f < 3 * R - 2) { j = (f - R) >> 1; base = G0 + ((f - R) & 1); stride = 2; mode = 2; }
    else if (f < 5 * R - 4) { j = (f - (3 * R - 2)) >> 1; base = P0 + ((f - (3 * R - 2)) & 1); stride = 2; mode = 1; }
    else if (f < 9 * R - 4) { base = Q0 + (f - (5 * R - 4)); }
    else if (f == 9 * R - 4) { base = A0; stride = 1; mode = 3; }
    else if (f < 9 * R - 1) { base = G0 + (f - (9 * R - 3)); stride = 2; mode = 3; }
    else { base = P0 + (f - (9 * R - 1)); stride = 2; mode = 3; }
    O.desc[f] = base | (stride << 10) | (mode << 14) | (j << 16);
  }
  __syncthreads();
  const int64_t e0 = (int64_t)blockIdx.x * OBS_EB;
  if (tid < OBS_EB && e0 + tid < B) {
    const int64_t e = e0 + tid;
    const uint32_t hdr = state[e];
    const uint32_t n = (hdr >> 16) & 0xFFu;
    const bool fresh = (hdr >> 24) & 1u;
    uint8_t* im = O.img[tid];
    const uint8_t nul = (uint8_t)(D / 2);
    im[0] = (uint8_t)n;
    for (int r = 0; r < R; ++r) {
      uint32_t a = (r < na && r < (int)n) ? state[(2 + r) * B + e] : 0u;
      const bool live = r < (int)n;
      const uint32_t carry = (a >> 16) & 0xFFu;
      im[A0 + r] = (uint8_t)((live && !fresh && !carry) ? 1 : 0);
      uint32_t dxy = (uint32_t)nul | ((uint32_t)nul << 8);
      if (live && !fresh && carry) dxy = delivery_xy<D>(carry - 1u);
      im[G0 + 2 * r] = (uint8_t)(dxy & 0xFFu);
      im[G0 + 2 * r + 1] = (uint8_t)(dxy >> 8);
      im[P0 + 2 * r] = live ? (uint8_t)(a & 0xFFu) : nul;
      im[P0 + 2 * r + 1] = live ? (uint8_t)((a >> 8) & 0xFFu) : nul;
    }
    const int wpt = 2 + na;
    int r = 0;
    for (int w = 0; w < C::PW; ++w) {
      const uint32_t pt = state[(wpt + w) * B + e];
      for (int b = 0; b < 4; ++b) {
        const uint32_t tg = (pt >> (8 * b)) & 0xFFu;
        if (tg && r < R) {
          const uint32_t j = 4u * w + b;
          const uint32_t pxy = reinterpret_cast<const uint16_t*>(reinterpret_cast<const uint8_t*>(tbl) + C::CELLB)[j];
          const uint32_t dxy = delivery_xy<D>(tg - 1u);
          im[Q0 + 4 * r] = (uint8_t)(pxy & 0xFFu);
          im[Q0 + 4 * r + 1] = (uint8_t)(pxy >> 8);
          im[Q0 + 4 * r + 2] = (uint8_t)(dxy & 0xFFu);
          im[Q0 + 4 * r + 3] = (uint8_t)(dxy >> 8);
          ++r;
        }
      }
    }
    O.fresh[tid] = fresh ? 1 : 0;
  }
  __syncthreads();
  const int64_t nenv = (B - e0) < OBS_EB ? (B - e0) : OBS_EB;
  const int64_t total = nenv * na * C::L;   // floats this block writes
  float* out = obs + e0 * na * C::L;
  for (int64_t o = tid; o < total; o += BT) {
    const int el = (int)(o / (na * C::L));
    const int rem = (int)(o - (int64_t)el * na * C::L);
    const int i = rem / C::L;
    const int f = rem - i * C::L;
    const uint32_t d = O.desc[f];
    const uint32_t base = d & 0x3FFu, stride = (d >> 10) & 0xFu, mode = (d >> 14) & 3u, j = d >> 16;
    uint32_t row = 0;
    if (mode == 1) row = (j < (uint32_t)i) ? j : j + 1;
    else if (mode == 2) { const uint32_t drop = O.fresh[el] ? (uint32_t)i : 1u; row = (j < drop) ? j : j + 1; }
    else if (mode == 3) row = (uint32_t)i;
    const uint8_t* im = O.img[el];
    const float v = (i < (int)im[0]) ? (float)im[base + stride * row] : 0.0f;
    out[o] = v;
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

__global__ __launch_bounds__(BT) void k_pack(PackParams a) {
  const int64_t e = (int64_t)blockIdx.x * BT + threadIdx.x;
  if (e >= a.B) return;
  const int64_t B = a.B;
  // out-of-range canonical values are clamped so packed state always indexes inside the grid
  const uint32_t n = min((uint32_t)max(a.n[e], 0), (uint32_t)a.na);
  a.state[e] = ((uint32_t)a.t[e] & 0xFFFFu) | (n << 16) | (a.fresh[e] ? (1u << 24) : 0u);
  a.state[B + e] = a.episode[e];
  for (int i = 0; i < a.na; ++i) {
    uint32_t w = 0;
    if (i < (int)n) {
      const int32_t tg = a.agent_target[e * a.na + i];
      const uint32_t x = (uint32_t)min(max(a.pos[(e * a.na + i) * 2], 0), a.D - 1);
      const uint32_t y = (uint32_t)min(max(a.pos[(e * a.na + i) * 2 + 1], 0), a.D - 1);
      w = x | (y << 8) | ((uint32_t)min(max(tg + 1, 0), 255) << 16);
    }
    a.state[(2 + i) * B + e] = w;
  }
  for (int w = 0; w < a.pw; ++w) {
    uint32_t tw = 0, mw = 0;
    for (int b = 0; b < 4; ++b) {
      const int j = 4 * w + b;
      const int32_t tg = a.pickup_target[e * a.P + j];
      if (tg >= 0) {
        tw |= (uint32_t)min(tg + 1, 255) << (8 * b);
        mw |= ((uint32_t)a.pickup_timer[e * a.P + j] & 0xFFu) << (8 * b);
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
    a.pos[(e * a.na + i) * 2] = (int32_t)(w & 0xFFu);
    a.pos[(e * a.na + i) * 2 + 1] = (int32_t)((w >> 8) & 0xFFu);
    a.agent_target[e * a.na + i] = (int32_t)((w >> 16) & 0xFFu) - 1;
  }
  for (int w = 0; w < a.pw; ++w) {
    const uint32_t tw = a.cstate[(2 + a.na + w) * B + e];
    const uint32_t mw = a.cstate[(2 + a.na + a.pw + w) * B + e];
    for (int b = 0; b < 4; ++b) {
      const int j = 4 * w + b;
      const uint32_t tg = (tw >> (8 * b)) & 0xFFu;
      a.pickup_target[e * a.P + j] = (int32_t)tg - 1;
      a.pickup_timer[e * a.P + j] = tg ? (int32_t)((mw >> (8 * b)) & 0xFFu) : -1;
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
  if (g->NR < 1 || g->NR > WH_MAX_RACKS || g->D < 5 || g->D > 255) return WH_EINVAL;
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

// host tables: cell -> pickup + 1, pickup xy, valid spawn cells (core.py:170-199)
std::vector<uint32_t> build_tables(const Geometry& g, int* bad) {
  const int cellb = (g.D * g.D + 3) & ~3;
  std::vector<uint8_t> cell(cellb, 0);
  std::vector<uint16_t> pxy(g.P);
  *bad = 0;
  for (int ix = 0; ix < g.NR; ++ix)
    for (int iy = 0; iy < g.NR; ++iy)
      for (int q = 0; q < 4; ++q) {
        const int j = (ix * g.NR + iy) * 4 + q;
        const int x = g.racks[ix] - 1 + (q & 1), y = g.racks[iy] - 1 + (q >> 1);
        if (cell[x * g.D + y]) *bad = 1;  // overlapping racks
        cell[x * g.D + y] = (uint8_t)(j + 1);
        pxy[j] = (uint16_t)(x | (y << 8));
      }
  std::vector<uint16_t> valid;
  for (int x = 1; x < g.D - 1; ++x)
    for (int y = 1; y < g.D - 1; ++y)
      if (!cell[x * g.D + y]) valid.push_back((uint16_t)(x | (y << 8)));
  std::vector<uint8_t> bytes(cell);
  for (uint16_t v : pxy) { bytes.push_back(v & 0xFF); bytes.push_back(v >> 8); }
  for (uint16_t v : valid) { bytes.push_back(v & 0xFF); bytes.push_back(v >> 8); }
  while (bytes.size() % 4) bytes.push_back(0);
  std::vector<uint32_t> words(bytes.size() / 4);
  memcpy(words.data(), bytes.data(), bytes.size());
  return words;
}

struct TableEntry {
  int device, D, NR, words;
  int racks[WH_MAX_RACKS];
  uint32_t* dev;
};
std::mutex g_tab_mu;
std::vector<TableEntry> g_tabs;

// Device copy of the tables for (device, geometry); allocated once per geometry and device.
int device_tables(const Geometry& g, int expect_words, const uint32_t** out) {
  int dev = 0;
  hipError_t he = hipGetDevice(&dev);
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
  uint32_t* d = nullptr;
  he = hipMalloc(&d, w.size() * 4);
  if (he != hipSuccess) return hip_err(he);
  he = hipMemcpy(d, w.data(), w.size() * 4, hipMemcpyHostToDevice);
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
  void (*reset)(ResetParams);
  void (*observe)(const uint32_t*, int64_t, int, const uint32_t*, float*);
  int tblw, nv;
};

template <int D, int R, int NR, int NAM>
Kernels make_kernels() {
  using C = Cfg<D, R, NR, NAM>;
  Kernels k;
  k.D = D; k.R = R; k.NR = NR; k.NAM = NAM;
  k.step[0] = k_step<C, POL_EXTERNAL>;
  k.step[1] = k_step<C, POL_GREEDY>;
  k.step[2] = k_step<C, POL_RANDOM>;
  k.reset = k_reset<C>;
  k.observe = k_observe<C>;
  k.tblw = C::TBLW;
  k.nv = C::NV;
  return k;
}

const std::vector<Kernels>& registry() {
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
  return r;
}

const Kernels* pick(const Geometry& g) {
  const Kernels* best = nullptr;
  for (const auto& k : registry())
    if (k.D == g.D && k.R == g.R && k.NR == g.NR && k.NAM >= g.NA && (!best || k.NAM < best->NAM))
      best = &k;
  return best;
}

int prepare(const wh_config* cfg, int64_t B, Geometry* g, const Kernels** kk, const uint32_t** tab) {
  int rc = validate(cfg, g);
  if (rc) return rc;
  if (B < 0) return WH_EINVAL;
  *kk = pick(*g);
  if (!*kk) return WH_ENOTSUP;
  return device_tables(*g, (*kk)->tblw, tab);
}

inline dim3 grid_for(int64_t B) { return dim3((unsigned)((B + BT - 1) / BT)); }

}  // namespace

// =============================================================================== C ABI
extern "C" {

const char* wh_version(void) { return "warehouse_amd gfx950 lane-per-env v1 " __DATE__; }

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
  int rc = prepare(cfg, B, &g, &k, &tab);
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

static int launch_step(const wh_config* cfg, int64_t B, uint32_t* state, int policy,
                       StepParams a, void* stream) {
  Geometry g;
  const Kernels* k;
  const uint32_t* tab;
  int rc = prepare(cfg, B, &g, &k, &tab);
  if (rc) return rc;
  if (policy < 0 || policy > 2) return WH_EINVAL;
  if (B == 0) return WH_OK;
  if (!state) return WH_EINVAL;
  a.state = state;
  a.B = B;
  a.na = g.NA;
  a.T = g.T;
  a.W = g.W;
  a.tables = tab;
  hipLaunchKernelGGL(k->step[policy], grid_for(B), dim3(BT), 0, (hipStream_t)stream, a);
  return hip_err(hipGetLastError());
}

int wh_step(const wh_config* cfg, int64_t B, uint32_t* state, const int32_t* actions,
            const int32_t* order, float* rewards, uint8_t* dones, const int32_t* regen,
            int32_t* n_inactive, int32_t phase, uint64_t seed, int64_t env_offset, void* stream) {
  if (phase < WH_PHASE_ALL || phase > WH_PHASE_REGEN) return WH_EINVAL;
  if (B > 0 && phase != WH_PHASE_REGEN && !actions) return WH_EINVAL;
  StepParams a{};
  a.actions = actions;
  a.order = order;
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

int wh_rollout(const wh_config* cfg, int64_t B, uint32_t* state, int32_t steps, int32_t policy,
               float p, float* rewards, uint8_t* dones, float* returns, int32_t autoreset,
               int32_t variable_n, uint64_t seed, int64_t env_offset, void* stream) {
  if ((policy != WH_POLICY_GREEDY && policy != WH_POLICY_RANDOM) || steps < 0) return WH_EINVAL;
  if (!(p >= 0.0f && p <= 1.0f)) return WH_EINVAL;
  StepParams a{};
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

int wh_observe(const wh_config* cfg, int64_t B, const uint32_t* state, float* obs, void* stream) {
  Geometry g;
  const Kernels* k;
  const uint32_t* tab;
  int rc = prepare(cfg, B, &g, &k, &tab);
  if (rc) return rc;
  if (B == 0) return WH_OK;
  if (!state || !obs) return WH_EINVAL;
  hipLaunchKernelGGL(k->observe, dim3((unsigned)((B + OBS_EB - 1) / OBS_EB)), dim3(BT), 0,
                     (hipStream_t)stream, state, B, g.NA, tab, obs);
  return hip_err(hipGetLastError());
}

}  // extern "C"
