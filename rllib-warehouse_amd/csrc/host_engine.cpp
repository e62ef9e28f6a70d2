// host_engine.cpp -- the warehouse transition on host cores (g++), behind the same C ABI as the
// gfx950 library (include/warehouse_amd.h): libwarehouse_host.so.
//
// What it is for: BASELINE config 1 ("1 env ... via baseline/run.py on CPU, no GPU").  The drop-in
// `warehouse.Warehouse` runs on this engine when no HIP device is present, so baseline/run.py and
// scripts/train.py work unchanged on a GPU-less host.  It is product code written from the
// reference (warehouse/core.py:167-442, baseline/solvers.py:27-58) and the header's contracts
// (packed state layout, injected draws, the philox draw contract of the device kernels) -- not a
// translation of the test oracle, which it never calls.  Every pointer is host memory and `stream`
// is ignored.  Entry points the CPU has no use for (the policy network, the fragment operand, the
// two-stream sampler step wh_sampler_step_to, prepared launches, assert mode) return WH_ENOTSUP;
// wh_sampler_step / wh_sampler_rollout run as policy + vector step per env.
//
// The state is the device's packed word planes (state[w * B + e]), so a state can move between the
// two engines with a plain copy, and the philox draws follow the device's stream layout word for
// word: a CPU rollout equals a GPU rollout bit for bit (tests/test_host_engine.py, tests/test_gpu_host_engine.py).
// Envs are independent; batches of many envs are split over host threads (OpenMP).
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "warehouse_amd.h"

namespace {

constexpr uint32_t IDLE = 0xFF00FF00u;   // target bytes of an agent word that carries nothing
constexpr int kMaxP = 64, kMaxA = 64;     // pickup / delivery points and agent slots per env (64-bit sets)
constexpr int kMaxD = 32;

enum Purpose : uint32_t { PUR_RESET = 1, PUR_REGEN = 2, PUR_POLICY = 3, PUR_RANDOM = 4 };

// ----------------------------------------------------------------------------- geometry
struct Geo {
  int D, R, NR, NA, P, DP, T, W, NV, words, L;
  int racks[WH_MAX_RACKS];
  int8_t cell[kMaxD][kMaxD];   // [x][y]: pickup index, -1 for other cells
  int px[kMaxP], py[kMaxP];    // pickup point cells (core.py:171-175)
  int dxc[kMaxP], dyc[kMaxP];  // delivery point cells (core.py:178-188)
  int vx[kMaxD * kMaxD], vy[kMaxD * kMaxD];   // spawn cells: interior, not a pickup, ascending (x, y)
};

int make_geo(const wh_config* c, Geo* g) {
  if (!c) return WH_EINVAL;
  g->D = c->area_dimension;
  g->R = c->num_requests;
  g->NR = c->num_racks;
  g->NA = c->agent_slots;
  g->T = c->episode_duration;
  g->W = c->pickup_wait_duration;
  if (g->NR < 1 || g->NR > WH_MAX_RACKS || g->D < 5 || g->D > kMaxD) return WH_EINVAL;
  g->P = 4 * g->NR * g->NR;
  g->DP = 4 * (g->D - 4);
  if (g->NA < 1 || g->NA > g->R || g->R > g->P || g->R > g->DP) return WH_EINVAL;
  if (g->W < 1 || g->W > 255 || g->T < 0) return WH_EINVAL;
  if (g->P > kMaxP || g->DP > kMaxP || g->NA > kMaxA) return WH_ENOTSUP;
  for (int i = 0; i < g->NR; ++i) {
    g->racks[i] = c->racks[i];
    if (c->racks[i] < 2 || c->racks[i] > g->D - 2) return WH_ENOTSUP;   // pickups must be interior
  }
  memset(g->cell, -1, sizeof(g->cell));
  // pickup points: for x in racks, for y in racks: (x-1, y-1), (x, y-1), (x-1, y), (x, y)
  int j = 0;
  for (int ix = 0; ix < g->NR; ++ix)
    for (int iy = 0; iy < g->NR; ++iy)
      for (int q = 0; q < 4; ++q, ++j) {
        const int x = g->racks[ix] - 1 + (q & 1), y = g->racks[iy] - 1 + (q >> 1);
        if (g->cell[x][y] >= 0) return WH_ENOTSUP;   // overlapping racks
        g->cell[x][y] = (int8_t)j;
        g->px[j] = x;
        g->py[j] = y;
      }
  // delivery points: for v in 2..D-3: (v, 0), (0, v), (v, D-1), (D-1, v)
  for (int d = 0; d < g->DP; ++d) {
    const int v = 2 + d / 4, side = d % 4;
    g->dxc[d] = (side & 1) ? (side == 3 ? g->D - 1 : 0) : v;
    g->dyc[d] = (side & 1) ? v : (side == 2 ? g->D - 1 : 0);
  }
  g->NV = 0;
  for (int x = 1; x < g->D - 1; ++x)
    for (int y = 1; y < g->D - 1; ++y)
      if (g->cell[x][y] < 0) {
        g->vx[g->NV] = x;
        g->vy[g->NV] = y;
        ++g->NV;
      }
  g->words = 2 + g->NA + 2 * (g->P / 4);
  g->L = 9 * g->R + 1;
  return WH_OK;
}

// delivery cell -> delivery index (the inverse of the table above)
int delivery_index(int x, int y, int D) {
  if (y == 0) return 4 * (x - 2);
  if (x == 0) return 4 * (y - 2) + 1;
  if (y == D - 1) return 4 * (x - 2) + 2;
  return 4 * (y - 2) + 3;
}

// ----------------------------------------------------------------------------- philox
// Philox4x32-10 (Salmon et al., SC'11); the device streams (include/warehouse_amd.h, RNG MODES):
// key (seed lo, seed hi), counter (global env id, episode, t, purpose << 24 | block).
struct U4 {
  uint32_t v[4];
};
U4 philox10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c0 = n0;
    c1 = (uint32_t)p1;
    c2 = n2;
    c3 = (uint32_t)p0;
  }
  return U4{{c0, c1, c2, c3}};
}
inline uint32_t umulhi(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }

struct Stream {   // words of one (env, episode, t, purpose) stream, one block cached
  uint32_t k0, k1, env, ep, t, purpose;
  int cur = -1;
  U4 blk{};
  uint32_t word(int j) {
    if ((j >> 2) != cur) {
      cur = j >> 2;
      blk = philox10(env, ep, t, (purpose << 24) | (uint32_t)cur, k0, k1);
    }
    return blk.v[j & 3];
  }
};

// ----------------------------------------------------------------------------- one env, unpacked
struct Env {
  uint32_t t, n, fresh, epi;
  int x[kMaxA], y[kMaxA], tg[kMaxA];   // position, delivery target index (-1: carries nothing)
  int pt[kMaxP];                        // request target of pickup point j (-1: none)
  uint32_t pe[kMaxP];                   // expiry byte of point j (the packed plane keeps it when closed)
};

void load(const Geo& g, const uint32_t* st, int64_t B, int64_t e, Env& s) {
  const uint32_t h = st[e];
  s.t = h & 0xFFFFu;
  s.n = std::min<uint32_t>((h >> 16) & 0xFFu, (uint32_t)g.NA);
  s.fresh = (h >> 24) & 1u;
  s.epi = st[B + e];
  for (int i = 0; i < g.NA; ++i) {
    const uint32_t w = st[(int64_t)(2 + i) * B + e];
    s.x[i] = (int)(w & 0xFFu);
    s.y[i] = (int)((w >> 16) & 0xFFu);
    const uint32_t dx = (w >> 8) & 0xFFu, dy = w >> 24;
    s.tg[i] = (dx == 0xFFu) ? -1 : delivery_index((int)dx, (int)dy, g.D);
  }
  const int PW = g.P / 4;
  for (int w = 0; w < PW; ++w) {
    const uint32_t tw = st[(int64_t)(2 + g.NA + w) * B + e], mw = st[(int64_t)(2 + g.NA + PW + w) * B + e];
    for (int b = 0; b < 4; ++b) {
      const uint32_t tb = (tw >> (8 * b)) & 0xFFu;
      s.pt[4 * w + b] = (tb == 0u || tb > (uint32_t)g.DP) ? -1 : (int)tb - 1;
      s.pe[4 * w + b] = (mw >> (8 * b)) & 0xFFu;
    }
  }
}

void store(const Geo& g, uint32_t* st, int64_t B, int64_t e, const Env& s) {
  st[e] = (s.t & 0xFFFFu) | (s.n << 16) | (s.fresh << 24);
  st[B + e] = s.epi;
  for (int i = 0; i < g.NA; ++i) {
    uint32_t w = IDLE;
    if ((uint32_t)i < s.n) {
      w = (uint32_t)s.x[i] | ((uint32_t)s.y[i] << 16);
      w |= s.tg[i] >= 0 ? ((uint32_t)g.dxc[s.tg[i]] << 8) | ((uint32_t)g.dyc[s.tg[i]] << 24) : IDLE;
    }
    st[(int64_t)(2 + i) * B + e] = w;
  }
  const int PW = g.P / 4;
  for (int w = 0; w < PW; ++w) {
    uint32_t tw = 0, mw = 0;
    for (int b = 0; b < 4; ++b) {
      const int j = 4 * w + b;
      tw |= (uint32_t)(s.pt[j] + 1) << (8 * b);
      mw |= (s.pe[j] & 0xFFu) << (8 * b);
    }
    st[(int64_t)(2 + g.NA + w) * B + e] = tw;
    st[(int64_t)(2 + g.NA + PW + w) * B + e] = mw;
  }
}

// ----------------------------------------------------------------------------- reset
// core.py:167-221; Train variants draw n first (variants.py:73-74).
void clear_requests(const Geo& g, Env& s) {
  for (int j = 0; j < g.P; ++j) {
    s.pt[j] = -1;
    s.pe[j] = 0;
  }
}

// Injected draws: accepted spawn cells, the R opened points and their targets in draw order.
void reset_injected(const Geo& g, Env& s, int64_t e, const wh_reset_draws& d) {
  const uint32_t n = d.n ? std::min<uint32_t>((uint32_t)d.n[e], (uint32_t)g.NA) : (uint32_t)g.NA;
  for (int i = 0; i < g.NA; ++i) {
    const bool live = (uint32_t)i < n;
    s.x[i] = live ? std::min<int>((int)(uint32_t)d.spawn[(e * g.NA + i) * 2], g.D - 1) : 0;
    s.y[i] = live ? std::min<int>((int)(uint32_t)d.spawn[(e * g.NA + i) * 2 + 1], g.D - 1) : 0;
    s.tg[i] = -1;
  }
  clear_requests(g, s);
  for (int j = 0; j < g.R; ++j) {
    const uint32_t sel = (uint32_t)d.pickups[e * g.R + j], tg = (uint32_t)d.targets[e * g.R + j];
    if (sel >= (uint32_t)g.P || tg >= (uint32_t)g.DP) continue;   // invalid injected draw: ignored
    s.pt[sel] = (int)tg;
    s.pe[sel] = (uint32_t)g.W & 0xFFu;   // opened at t = 0 with wait W
  }
  s.t = 0;
  s.n = n;
  s.fresh = 1;
  s.epi += 1;
}

// Philox draws, the device's word layout (RESET purpose, episode epi + 1, t = 0): word 0 the agent
// count (variable_n), words 1..NA the spawn cells (uniform over the NV spawn cells: the law of the
// reference's rejection loop, core.py:191-201), then per request j the pair (point, target): the
// points a uniform R-subset by Floyd's algorithm, the targets a uniform ordered R-tuple of distinct
// delivery points (core.py:213-221: choice(P, R) paired with choice(Dp, R)).
void reset_philox(const Geo& g, Env& s, uint32_t k0, uint32_t k1, uint32_t gid, bool variable_n) {
  const uint32_t ep = s.epi + 1u;
  Stream w{k0, k1, gid, ep, 0u, PUR_RESET};
  const int na = g.NA;
  const uint32_t n = variable_n ? 1u + umulhi(w.word(0), (uint32_t)na) : (uint32_t)na;
  for (int i = 0; i < na; ++i) {
    const uint32_t v = umulhi(w.word(1 + i), (uint32_t)g.NV);
    const bool live = (uint32_t)i < n;
    s.x[i] = live ? g.vx[v] : 0;
    s.y[i] = live ? g.vy[v] : 0;
    s.tg[i] = -1;
  }
  clear_requests(g, s);
  uint64_t taken = 0;
  uint32_t sel[kMaxP], rank[kMaxP];
  for (int j = 0; j < g.R; ++j) {
    const uint32_t m = (uint32_t)(g.P - g.R + j);
    const uint32_t r = umulhi(w.word(1 + na + 2 * j), m + 1u);
    sel[j] = (j > 0 && ((taken >> r) & 1ull)) ? m : r;
    taken |= 1ull << sel[j];
    rank[j] = umulhi(w.word(2 + na + 2 * j), (uint32_t)(g.DP - j));
  }
  // item j's target: the rank[j]-th delivery point not taken by items < j
  uint64_t used = 0;
  for (int j = 0; j < g.R; ++j) {
    uint32_t r = rank[j];
    int d = 0;
    for (;; ++d)
      if (!((used >> d) & 1ull) && r-- == 0) break;
    used |= 1ull << d;
    s.pt[sel[j]] = d;
    s.pe[sel[j]] = (uint32_t)g.W & 0xFFu;
  }
  s.t = 0;
  s.n = n;
  s.fresh = 1;
  s.epi = ep;
}

// ----------------------------------------------------------------------------- step
// core.py:267-368.  Entries: the action dict in iteration order (agent | (own action + 1) << 8; an
// entry without its own action takes actions[agent]; -1 = no entry), or every live agent in
// ascending order when `ord` is NULL.  Actions > 8 act as 4 (stay); the host binding wraps negative
// actions like Python's list indexing and rejects >= 9 before it gets here.
struct StepOut {
  float rew[kMaxA];
  bool done;
  int nin;
};

constexpr int PH_ALL = WH_PHASE_ALL, PH_PRE = WH_PHASE_PRE_REGEN, PH_REGEN = WH_PHASE_REGEN;

inline int move_dx(uint32_t a) { return (int)(a / 3u) - 1; }   // MOVES[a] = (a // 3 - 1, a % 3 - 1), core.py:38
inline int move_dy(uint32_t a) { return (int)(a % 3u) - 1; }

void move_phase(const Geo& g, Env& s, const int32_t* acts, const int32_t* ord, int ol) {
  bool occ[kMaxD][kMaxD] = {};   // rebuilt from the positions every step (core.py:275-276)
  for (uint32_t i = 0; i < s.n; ++i) occ[s.x[i]][s.y[i]] = true;
  // invalid moves (core.py:277, 293-297) as (from x, from y, to x, to y) bytes
  std::vector<uint32_t> invalid;
  auto key = [](int a, int b, int c, int d) { return (uint32_t)a | ((uint32_t)b << 8) | ((uint32_t)c << 16) | ((uint32_t)d << 24); };
  const int count = ord ? ol : (int)s.n;
  for (int k = 0; k < count; ++k) {
    int who;
    uint32_t a;
    if (ord) {
      const int32_t raw = ord[k];
      if (raw < 0) continue;
      who = raw & 0xFF;
      const uint32_t own = ((uint32_t)raw >> 8) & 0xFFu;
      if ((uint32_t)who >= s.n) continue;
      a = own ? own - 1u : (uint32_t)acts[who];
    } else {
      who = k;
      a = (uint32_t)acts[k];
    }
    if (a > 8u) a = 4u;
    const int px = s.x[who], py = s.y[who];
    int x = px + move_dx(a), y = py + move_dy(a);
    if (!(0 <= x && x < g.D)) x = px;   // core.py:284-287
    if (!(0 <= y && y < g.D)) y = py;
    if (occ[x][y] || std::find(invalid.begin(), invalid.end(), key(px, py, x, y)) != invalid.end()) continue;
    occ[px][py] = false;
    occ[x][y] = true;
    invalid.push_back(key(x, y, px, py));
    if (x != px && y != py) {
      invalid.push_back(key(x, py, px, y));
      invalid.push_back(key(px, y, x, py));
    }
    s.x[who] = x;
    s.y[who] = y;
  }
}

// the r-th (0-based) member of set m, ascending
int select_bit(uint64_t m, uint32_t r) {
  for (int j = 0; j < 64; ++j)
    if ((m >> j) & 1ull) {
      if (r == 0) return j;
      --r;
    }
  return -1;
}

void regenerate(const Geo& g, Env& s, const int32_t* regen, uint32_t k0, uint32_t k1, uint32_t gid) {
  uint64_t inactive = 0;
  int nin = 0;
  for (int j = 0; j < g.P; ++j)
    if (s.pt[j] < 0) {
      inactive |= 1ull << j;
      ++nin;
    }
  const int k = g.R - g.P + nin;   // core.py:339-341 (draws are consumed even when k = 0)
  const uint32_t exp = (s.t + (uint32_t)g.W) & 0xFFu;
  if (regen) {
    // injected: R positions into the ascending inactive list, then R targets (core.py:339-350)
    for (int j = 0; j < k && j < g.R; ++j) {
      const uint32_t rpos = (uint32_t)regen[j], tgi = (uint32_t)regen[g.R + j];
      if (rpos >= (uint32_t)nin || tgi >= (uint32_t)g.DP) continue;   // invalid draws are ignored
      const int sel = select_bit(inactive, rpos);
      s.pt[sel] = (int)tgi;
      s.pe[sel] = exp;
    }
    return;
  }
  // philox (REGEN purpose, words 2j / 2j + 1 = item j's point / target): an ordered k-subset of the
  // inactive points and k distinct targets, each uniform over what earlier items left
  Stream w{k0, k1, gid, s.epi, s.t, PUR_REGEN};
  uint64_t left = inactive, used = 0;
  for (int j = 0; j < k && j < g.R; ++j) {
    const int sel = select_bit(left, umulhi(w.word(2 * j), (uint32_t)(nin - j)));
    const int tgi = select_bit(~used & (g.DP >= 64 ? ~0ull : ((1ull << g.DP) - 1ull)), umulhi(w.word(2 * j + 1), (uint32_t)(g.DP - j)));
    left &= ~(1ull << sel);
    used |= 1ull << tgi;
    s.pt[sel] = tgi;
    s.pe[sel] = exp;
  }
}

StepOut step_env(const Geo& g, Env& s, const int32_t* acts, const int32_t* ord, int ol, const int32_t* regen,
                 uint32_t k0, uint32_t k1, uint32_t gid, int phase) {
  StepOut o{};
  for (int i = 0; i < g.NA; ++i) o.rew[i] = 0.0f;
  if (phase != PH_REGEN) {
    s.t = (s.t + 1u) & 0xFFFFu;                         // core.py:267
    move_phase(g, s, acts, ord, ol);                    // core.py:275-300
    for (int j = 0; j < g.P; ++j)                       // core.py:303-306: timers count to the expiry step
      if (s.pt[j] >= 0 && s.pe[j] == (s.t & 0xFFu)) s.pt[j] = -1;
    // pickups (core.py:309-335): every agent decides against the pre-pickup table, then the points
    // are cleared (two agents on one point both take its request)
    int taken[kMaxA];
    for (uint32_t i = 0; i < s.n; ++i) {
      const int c = g.cell[s.x[i]][s.y[i]];
      taken[i] = (c >= 0 && s.tg[i] < 0 && s.pt[c] >= 0) ? c : -1;
    }
    for (uint32_t i = 0; i < s.n; ++i)
      if (taken[i] >= 0) {
        s.tg[i] = s.pt[taken[i]];
        o.rew[i] = 1.0f;
      }
    for (uint32_t i = 0; i < s.n; ++i)
      if (taken[i] >= 0) s.pt[taken[i]] = -1;
    o.nin = 0;
    for (int j = 0; j < g.P; ++j) o.nin += s.pt[j] < 0;
  }
  if (phase != PH_PRE) regenerate(g, s, regen, k0, k1, gid);   // core.py:338-351
  if (phase != PH_REGEN) {
    for (uint32_t i = 0; i < s.n; ++i)                 // deliveries, core.py:354-368
      if (s.tg[i] >= 0 && s.x[i] == g.dxc[s.tg[i]] && s.y[i] == g.dyc[s.tg[i]]) {
        s.tg[i] = -1;
        o.rew[i] = 1.0f;   // (a pickup, interior, and a delivery, on the border, never share a step)
      }
    o.done = s.t >= (uint32_t)g.T;                     // core.py:438
    s.fresh = 0;
  }
  return o;
}

// ----------------------------------------------------------------------------- policy
// baseline/solvers.py:27-58 on the state: availability 0 (fresh reset, or carrying) -> the own
// delivery target (the null cell (D/2, D/2) after a reset, core.py:233-236), else the nearest open
// request (Manhattan, first minimum = lowest pickup index wins); step = clip(goal - pos, -1, 1).
// With probability p the action is uniform over the 9 moves (POLICY stream: word 2i the coin,
// 2i + 1 the move of agent i).  Random policy: RANDOM stream word i.
void policy_env(const Geo& g, const Env& s, int policy, float p, uint32_t k0, uint32_t k1, uint32_t gid,
                int32_t* out) {
  for (int i = 0; i < g.NA; ++i) out[i] = 4;
  if (policy == WH_POLICY_RANDOM) {
    Stream w{k0, k1, gid, s.epi, s.t, PUR_RANDOM};
    for (uint32_t i = 0; i < s.n; ++i) out[i] = (int32_t)umulhi(w.word((int)i), 9u);
    return;
  }
  const int nul = g.D / 2;
  Stream w{k0, k1, gid, s.epi, s.t, PUR_POLICY};
  for (uint32_t i = 0; i < s.n; ++i) {
    int gx = nul, gy = nul;
    if (!s.fresh) {
      if (s.tg[i] >= 0) {
        gx = g.dxc[s.tg[i]];
        gy = g.dyc[s.tg[i]];
      } else {
        int best = 1 << 30;
        for (int j = 0; j < g.P; ++j)
          if (s.pt[j] >= 0) {
            const int dist = std::abs(g.px[j] - s.x[i]) + std::abs(g.py[j] - s.y[i]);
            if (dist < best) {
              best = dist;
              gx = g.px[j];
              gy = g.py[j];
            }
          }
      }
    }
    const int sx = std::max(-1, std::min(1, gx - s.x[i])), sy = std::max(-1, std::min(1, gy - s.y[i]));
    out[i] = (sx + 1) * 3 + (sy + 1);
    if (p > 0.0f) {
      const float u = (float)(w.word(2 * (int)i) >> 8) * (1.0f / 16777216.0f);
      if (u < p) out[i] = (int32_t)umulhi(w.word(2 * (int)i + 1), 9u);
    }
  }
}

// ----------------------------------------------------------------------------- observation rows
// core.py:224-260 (fresh) / 371-432, in sorted gym-Dict key order: num_agents,
// other_availabilities, other_delivery_targets, other_positions, requests, self_availability,
// self_delivery_target, self_position.  other_delivery_targets drops row 1 for every agent after a
// step (core.py:428) and row i after a reset (core.py:256).  Rows of slots >= n are zero.
void observe_env(const Geo& g, const Env& s, float* rows) {
  const int R = g.R, L = g.L;
  const float nul = (float)(g.D / 2);
  float av[kMaxP], dt[kMaxP][2], ps[kMaxP][2], rq[kMaxP][4];
  for (int r = 0; r < R; ++r) {
    const bool live = (uint32_t)r < s.n;
    const bool carry = live && s.tg[r] >= 0;
    av[r] = (live && !s.fresh && !carry) ? 1.0f : 0.0f;
    dt[r][0] = (carry && !s.fresh) ? (float)g.dxc[s.tg[r]] : nul;
    dt[r][1] = (carry && !s.fresh) ? (float)g.dyc[s.tg[r]] : nul;
    ps[r][0] = live ? (float)s.x[r] : nul;
    ps[r][1] = live ? (float)s.y[r] : nul;
  }
  int q = 0;
  for (int j = 0; j < g.P && q < R; ++j)
    if (s.pt[j] >= 0) {
      rq[q][0] = (float)g.px[j];
      rq[q][1] = (float)g.py[j];
      rq[q][2] = (float)g.dxc[s.pt[j]];
      rq[q][3] = (float)g.dyc[s.pt[j]];
      ++q;
    }
  for (; q < R; ++q) rq[q][0] = rq[q][1] = rq[q][2] = rq[q][3] = 0.0f;
  for (int i = 0; i < g.NA; ++i) {
    float* o = rows + (int64_t)i * L;
    if ((uint32_t)i >= s.n) {
      memset(o, 0, sizeof(float) * L);
      continue;
    }
    int f = 0;
    o[f++] = (float)s.n;
    for (int r = 0; r < R; ++r)
      if (r != i) o[f++] = av[r];
    const int drop = s.fresh ? i : 1;
    for (int r = 0; r < R; ++r)
      if (r != drop) {
        o[f++] = dt[r][0];
        o[f++] = dt[r][1];
      }
    for (int r = 0; r < R; ++r)
      if (r != i) {
        o[f++] = ps[r][0];
        o[f++] = ps[r][1];
      }
    for (int r = 0; r < R; ++r)
      for (int c = 0; c < 4; ++c) o[f++] = rq[r][c];
    o[f++] = av[i];
    o[f++] = dt[i][0];
    o[f++] = dt[i][1];
    o[f++] = ps[i][0];
    o[f++] = ps[i][1];
  }
}

// ----------------------------------------------------------------------------- episode metrics
void fold_episode(const wh_episode_stats* st, uint32_t n, uint32_t ret) {
  if (!st) return;
#pragma omp critical(wh_host_stats)
  {
    if (st->return_sum) st->return_sum[n] += ret;
    if (st->episodes) st->episodes[n] += 1;
    if (st->return_min) st->return_min[n] = std::min(st->return_min[n], ret);
    if (st->return_max) st->return_max[n] = std::max(st->return_max[n], ret);
  }
}

bool stats_ok(const wh_episode_stats* st) {
  return !st || st->episode_return || (!st->return_sum && !st->episodes && !st->return_min && !st->return_max);
}

uint32_t keys_lo(uint64_t seed) { return (uint32_t)(seed & 0xFFFFFFFFu); }
uint32_t keys_hi(uint64_t seed) { return (uint32_t)(seed >> 32); }

// order rows: 0 = agent_slots entries per env, else 1 .. 4 * agent_slots
int order_width(const Geo& g, int32_t order_len) {
  if (order_len == 0) return g.NA;
  return (order_len >= 1 && order_len <= 4 * g.NA) ? order_len : -1;
}

}  // namespace

// =============================================================================== C ABI
extern "C" {

int wh_query(const wh_config* cfg, wh_layout* out) {
  Geo g;
  const int rc = make_geo(cfg, &g);
  if (rc) return rc;
  if (out) {
    out->words_per_env = g.words;
    out->num_pickups = g.P;
    out->num_deliveries = g.DP;
    out->obs_len = g.L;
    out->kernel_agents = g.NA;
  }
  return WH_OK;
}

int wh_pack(const wh_config* cfg, int64_t B, const int32_t* pos, const int32_t* agent_target,
            const int32_t* pickup_target, const int32_t* pickup_timer, const int32_t* t, const int32_t* n,
            const uint8_t* fresh, const uint32_t* episode, uint32_t* state, void* stream) {
  (void)stream;
  Geo g;
  const int rc = make_geo(cfg, &g);
  if (rc) return rc;
  if (B == 0) return WH_OK;
  if (B < 0 || !pos || !agent_target || !pickup_target || !pickup_timer || !t || !n || !fresh || !episode || !state)
    return WH_EINVAL;
  for (int64_t e = 0; e < B; ++e) {   // out-of-range canonical values are clamped (as wh_pack on the device)
    Env s{};
    s.t = (uint32_t)t[e] & 0xFFFFu;
    s.n = (uint32_t)std::min(std::max(n[e], 0), g.NA);
    s.fresh = fresh[e] ? 1u : 0u;
    s.epi = episode[e];
    for (int i = 0; i < g.NA; ++i) {
      s.x[i] = std::min(std::max(pos[(e * g.NA + i) * 2], 0), g.D - 1);
      s.y[i] = std::min(std::max(pos[(e * g.NA + i) * 2 + 1], 0), g.D - 1);
      const int32_t tg = agent_target[e * g.NA + i];
      s.tg[i] = (tg >= 0 && tg < g.DP) ? tg : -1;
    }
    for (int j = 0; j < g.P; ++j) {
      const int32_t tg = pickup_target[e * g.P + j];
      s.pt[j] = (tg >= 0 && tg < g.DP) ? tg : -1;
      s.pe[j] = s.pt[j] >= 0 ? ((uint32_t)t[e] + (uint32_t)pickup_timer[e * g.P + j]) & 0xFFu : 0u;
    }
    store(g, state, B, e, s);
  }
  return WH_OK;
}

int wh_unpack(const wh_config* cfg, int64_t B, const uint32_t* state, int32_t* pos, int32_t* agent_target,
              int32_t* pickup_target, int32_t* pickup_timer, int32_t* t, int32_t* n, uint8_t* fresh,
              uint32_t* episode, void* stream) {
  (void)stream;
  Geo g;
  const int rc = make_geo(cfg, &g);
  if (rc) return rc;
  if (B == 0) return WH_OK;
  if (B < 0 || !pos || !agent_target || !pickup_target || !pickup_timer || !t || !n || !fresh || !episode || !state)
    return WH_EINVAL;
  for (int64_t e = 0; e < B; ++e) {
    Env s;
    load(g, state, B, e, s);
    t[e] = (int32_t)s.t;
    n[e] = (int32_t)((state[e] >> 16) & 0xFFu);
    fresh[e] = (uint8_t)s.fresh;
    episode[e] = s.epi;
    for (int i = 0; i < g.NA; ++i) {
      const bool live = (uint32_t)i < s.n;
      pos[(e * g.NA + i) * 2] = live ? s.x[i] : 0;
      pos[(e * g.NA + i) * 2 + 1] = live ? s.y[i] : 0;
      agent_target[e * g.NA + i] = live ? s.tg[i] : -1;
    }
    for (int j = 0; j < g.P; ++j) {
      pickup_target[e * g.P + j] = s.pt[j];
      pickup_timer[e * g.P + j] = s.pt[j] >= 0 ? (int32_t)((s.pe[j] - s.t) & 0xFFu) : -1;   // steps left
    }
  }
  return WH_OK;
}

int wh_reset(const wh_config* cfg, int64_t B, uint32_t* state, const uint8_t* mask, const wh_reset_draws* draws,
             int32_t variable_n, uint64_t seed, int64_t env_offset, void* stream) {
  (void)stream;
  Geo g;
  const int rc = make_geo(cfg, &g);
  if (rc) return rc;
  if (B < 0) return WH_EINVAL;
  if (B == 0) return WH_OK;
  if (!state) return WH_EINVAL;
  if (draws && (!draws->spawn || !draws->pickups || !draws->targets)) return WH_EINVAL;
#pragma omp parallel for schedule(static) if (B >= 1024)
  for (int64_t e = 0; e < B; ++e) {
    if (mask && !mask[e]) continue;
    Env s;
    load(g, state, B, e, s);
    if (draws)
      reset_injected(g, s, e, *draws);
    else
      reset_philox(g, s, keys_lo(seed), keys_hi(seed), (uint32_t)(env_offset + e), variable_n != 0);
    store(g, state, B, e, s);
  }
  return WH_OK;
}

int wh_step(const wh_config* cfg, int64_t B, uint32_t* state, const int32_t* actions, const int32_t* order,
            int32_t order_len, float* rewards, uint8_t* dones, const int32_t* regen, int32_t* n_inactive,
            int32_t phase, uint64_t seed, int64_t env_offset, void* stream) {
  (void)stream;
  if (phase < WH_PHASE_ALL || phase > WH_PHASE_REGEN) return WH_EINVAL;
  if (B > 0 && phase != WH_PHASE_REGEN && !actions) return WH_EINVAL;
  Geo g;
  const int rc = make_geo(cfg, &g);
  if (rc) return rc;
  const int ol = order_width(g, order_len);
  if (B < 0 || ol < 0) return WH_EINVAL;
  if (B == 0) return WH_OK;
  if (!state) return WH_EINVAL;
#pragma omp parallel for schedule(static) if (B >= 1024)
  for (int64_t e = 0; e < B; ++e) {
    Env s;
    load(g, state, B, e, s);
    const StepOut o = step_env(g, s, actions ? actions + e * g.NA : nullptr, order ? order + e * ol : nullptr, ol,
                               regen ? regen + e * 2 * g.R : nullptr, keys_lo(seed), keys_hi(seed),
                               (uint32_t)(env_offset + e), phase);
    if (phase != WH_PHASE_REGEN) {
      if (rewards)
        for (int i = 0; i < g.NA; ++i) rewards[e * g.NA + i] = o.rew[i];
      if (dones) dones[e] = o.done ? 1 : 0;
    }
    if (phase == WH_PHASE_PRE_REGEN && n_inactive) n_inactive[e] = o.nin;
    store(g, state, B, e, s);
  }
  return WH_OK;
}

int wh_observe(const wh_config* cfg, int64_t B, const uint32_t* state, float* obs, void* stream) {
  (void)stream;
  Geo g;
  const int rc = make_geo(cfg, &g);
  if (rc) return rc;
  if (B < 0) return WH_EINVAL;
  if (B == 0) return WH_OK;
  if (!state || !obs) return WH_EINVAL;
#pragma omp parallel for schedule(static) if (B >= 1024)
  for (int64_t e = 0; e < B; ++e) {
    Env s;
    load(g, state, B, e, s);
    observe_env(g, s, obs + e * g.NA * g.L);
  }
  return WH_OK;
}

int wh_observe_x(const wh_config* cfg, int64_t B, const uint32_t* state, float* obs, void* xfrag, void* stream) {
  (void)cfg, (void)B, (void)state, (void)obs, (void)xfrag, (void)stream;
  return WH_ENOTSUP;   // the policy network's MFMA operand: a device format
}

int wh_policy(const wh_config* cfg, int64_t B, const uint32_t* state, int32_t policy, float p, int32_t* actions,
              uint64_t seed, int64_t env_offset, void* stream) {
  (void)stream;
  if ((policy != WH_POLICY_GREEDY && policy != WH_POLICY_RANDOM) || (B > 0 && !actions)) return WH_EINVAL;
  if (!(p >= 0.0f && p <= 1.0f)) return WH_EINVAL;
  Geo g;
  const int rc = make_geo(cfg, &g);
  if (rc) return rc;
  if (B < 0) return WH_EINVAL;
  if (B == 0) return WH_OK;
  if (!state) return WH_EINVAL;
#pragma omp parallel for schedule(static) if (B >= 1024)
  for (int64_t e = 0; e < B; ++e) {
    Env s;
    load(g, state, B, e, s);
    policy_env(g, s, policy, p, keys_lo(seed), keys_hi(seed), (uint32_t)(env_offset + e), actions + e * g.NA);
  }
  return WH_OK;
}

int wh_rollout(const wh_config* cfg, int64_t B, uint32_t* state, int32_t steps, int32_t policy, float p,
               float* rewards, uint8_t* dones, float* returns, const wh_episode_stats* stats, int32_t autoreset,
               int32_t variable_n, uint64_t seed, int64_t env_offset, void* stream) {
  (void)stream;
  if ((policy != WH_POLICY_GREEDY && policy != WH_POLICY_RANDOM) || steps < 0) return WH_EINVAL;
  if (!(p >= 0.0f && p <= 1.0f) || !stats_ok(stats)) return WH_EINVAL;
  Geo g;
  const int rc = make_geo(cfg, &g);
  if (rc) return rc;
  if (B < 0) return WH_EINVAL;
  if (B == 0) return WH_OK;
  if (!state) return WH_EINVAL;
  const bool st = stats && stats->episode_return;
#pragma omp parallel for schedule(static) if (B >= 256)
  for (int64_t e = 0; e < B; ++e) {
    Env s;
    load(g, state, B, e, s);
    const uint32_t gid = (uint32_t)(env_offset + e);
    uint32_t epr = st ? stats->episode_return[e] : 0u;
    float ret = 0.0f;
    int32_t acts[kMaxA];
    for (int k = 0; k < steps; ++k) {
      policy_env(g, s, policy, p, keys_lo(seed), keys_hi(seed), gid, acts);
      const StepOut o = step_env(g, s, acts, nullptr, 0, nullptr, keys_lo(seed), keys_hi(seed), gid, WH_PHASE_ALL);
      if (rewards)
        for (int i = 0; i < g.NA; ++i) rewards[((int64_t)k * B + e) * g.NA + i] = o.rew[i];
      if (dones) dones[(int64_t)k * B + e] = o.done ? 1 : 0;
      float r = 0.0f;
      for (int i = 0; i < g.NA; ++i) r += o.rew[i];
      ret += r;
      if (st) {
        epr += (uint32_t)r;
        if (o.done) {
          fold_episode(stats, s.n, epr);
          epr = 0;
        }
      }
      if (o.done && autoreset) reset_philox(g, s, keys_lo(seed), keys_hi(seed), gid, variable_n != 0);
    }
    if (returns) returns[e] += ret;
    if (st) stats->episode_return[e] = epr;
    store(g, state, B, e, s);
  }
  return WH_OK;
}

int wh_vector_step(const wh_config* cfg, int64_t B, uint32_t* state, const int32_t* actions, const int32_t* order,
                   int32_t order_len, const uint8_t* mask, float* rewards, uint8_t* dones, float* obs,
                   const wh_episode_stats* stats, int32_t autoreset, int32_t variable_n, uint64_t seed,
                   int64_t env_offset, void* stream) {
  (void)stream;
  if (B > 0 && !actions) return WH_EINVAL;
  if (!stats_ok(stats)) return WH_EINVAL;
  Geo g;
  const int rc = make_geo(cfg, &g);
  if (rc) return rc;
  const int ol = order_width(g, order_len);
  if (B < 0 || ol < 0) return WH_EINVAL;
  if (B == 0) return WH_OK;
  if (!state) return WH_EINVAL;
  const bool st = stats && stats->episode_return;
#pragma omp parallel for schedule(static) if (B >= 1024)
  for (int64_t e = 0; e < B; ++e) {
    Env s;
    load(g, state, B, e, s);
    if (!mask || mask[e]) {
      const uint32_t gid = (uint32_t)(env_offset + e);
      const StepOut o = step_env(g, s, actions + e * g.NA, order ? order + e * ol : nullptr, ol, nullptr, keys_lo(seed),
                                 keys_hi(seed), gid, WH_PHASE_ALL);
      if (rewards)
        for (int i = 0; i < g.NA; ++i) rewards[e * g.NA + i] = o.rew[i];
      if (dones) dones[e] = o.done ? 1 : 0;
      if (st) {
        float r = 0.0f;
        for (int i = 0; i < g.NA; ++i) r += o.rew[i];
        uint32_t epr = stats->episode_return[e] + (uint32_t)r;
        if (o.done) {
          fold_episode(stats, s.n, epr);
          epr = 0;
        }
        stats->episode_return[e] = epr;
      }
      if (o.done && autoreset) reset_philox(g, s, keys_lo(seed), keys_hi(seed), gid, variable_n != 0);
      store(g, state, B, e, s);
    }
    if (obs) observe_env(g, s, obs + e * g.NA * g.L);
  }
  return WH_OK;
}

int wh_vector_step_x(const wh_config* cfg, int64_t B, uint32_t* state, const int32_t* actions, const int32_t* order,
                     int32_t order_len, const uint8_t* mask, float* rewards, uint8_t* dones, void* xfrag,
                     const wh_episode_stats* stats, int32_t autoreset, int32_t variable_n, uint64_t seed,
                     int64_t env_offset, void* stream) {
  (void)cfg, (void)B, (void)state, (void)actions, (void)order, (void)order_len, (void)mask, (void)rewards,
      (void)dones, (void)xfrag, (void)stats, (void)autoreset, (void)variable_n, (void)seed, (void)env_offset,
      (void)stream;
  return WH_ENOTSUP;
}

int wh_sampler_step(const wh_config* cfg, int64_t B, uint32_t* state, int32_t policy, float p, float* rewards,
                    uint8_t* dones, float* obs, const wh_episode_stats* stats, int32_t variable_n, uint64_t seed,
                    int64_t env_offset, void* stream) {
  if (policy != WH_POLICY_GREEDY && policy != WH_POLICY_RANDOM) return WH_EINVAL;
  if (!(p >= 0.0f && p <= 1.0f) || !stats_ok(stats)) return WH_EINVAL;
  Geo g;
  const int rc = make_geo(cfg, &g);
  if (rc) return rc;
  if (B < 0) return WH_EINVAL;
  if (B == 0) return WH_OK;
  std::vector<int32_t> acts((size_t)B * g.NA);
  int r = wh_policy(cfg, B, state, policy, p, acts.data(), seed, env_offset, stream);
  if (r) return r;
  return wh_vector_step(cfg, B, state, acts.data(), nullptr, 0, nullptr, rewards, dones, obs, stats, 1, variable_n,
                        seed, env_offset, stream);
}

int wh_sampler_rollout(const wh_config* cfg, int64_t B, uint32_t* state, int32_t steps, int32_t policy, float p,
                       float* rewards, uint8_t* dones, float* obs, const wh_episode_stats* stats, int32_t variable_n,
                       uint64_t seed, int64_t env_offset, void* stream) {
  if (steps < 0) return WH_EINVAL;
  if (B > 0 && steps > 0 && !obs) return WH_EINVAL;
  Geo g;
  const int rc = make_geo(cfg, &g);
  if (rc) return rc;
  int r = WH_OK;
  for (int32_t k = 0; k < steps && r == WH_OK; ++k)
    r = wh_sampler_step(cfg, B, state, policy, p, rewards ? rewards + (int64_t)k * B * g.NA : nullptr,
                        dones ? dones + (int64_t)k * B : nullptr, obs + (int64_t)k * B * g.NA * g.L, stats, variable_n,
                        seed, env_offset, stream);
  return r;
}

int wh_sampler_step_to(const wh_config* cfg, int64_t B, const uint32_t* state_in, uint32_t* state_out, int32_t policy,
                       float p, float* rewards, uint8_t* dones, const wh_episode_stats* stats, int32_t variable_n,
                       uint64_t seed, int64_t env_offset, void* stream) {
  (void)cfg, (void)B, (void)state_in, (void)state_out, (void)policy, (void)p, (void)rewards, (void)dones, (void)stats,
      (void)variable_n, (void)seed, (void)env_offset, (void)stream;
  return WH_ENOTSUP;   // a two-stream device pipeline
}

int wh_rollout_prepare(const wh_config* cfg, int64_t B, uint32_t* state, int32_t steps, int32_t policy, float p,
                       float* rewards, uint8_t* dones, float* returns, const wh_episode_stats* stats, int32_t autoreset,
                       int32_t variable_n, uint64_t seed, int64_t env_offset, void* stream, wh_launch** out) {
  (void)cfg, (void)B, (void)state, (void)steps, (void)policy, (void)p, (void)rewards, (void)dones, (void)returns,
      (void)stats, (void)autoreset, (void)variable_n, (void)seed, (void)env_offset, (void)stream;
  if (out) *out = nullptr;
  return WH_ENOTSUP;   // prepared device launches
}
int wh_launch_run(const wh_launch* launch) { return launch ? WH_EINVAL : WH_EINVAL; }
int wh_launch_run_timed(const wh_launch* launch, void* start_event, void* stop_event) {
  (void)launch, (void)start_event, (void)stop_event;
  return WH_EINVAL;
}
int wh_launch_free(wh_launch* launch) { return launch ? WH_EINVAL : WH_OK; }

int wh_mlp_query(const wh_mlp_desc* d, int64_t* packed_bytes) {
  (void)d, (void)packed_bytes;
  return WH_ENOTSUP;   // the policy network runs on the device only
}
int wh_mlp_pack(const wh_mlp_desc* d, const float* w0, const float* b0, const float* w1, const float* b1,
                const float* w2, const float* b2, void* packed) {
  (void)d, (void)w0, (void)b0, (void)w1, (void)b1, (void)w2, (void)b2, (void)packed;
  return WH_ENOTSUP;
}
int wh_mlp_forward(const wh_mlp_desc* d, const void* packed, int64_t rows, const float* obs, float* logits,
                   int32_t* actions, int32_t explore, uint64_t seed, uint32_t step, void* stream) {
  (void)d, (void)packed, (void)rows, (void)obs, (void)logits, (void)actions, (void)explore, (void)seed, (void)step,
      (void)stream;
  return WH_ENOTSUP;
}
int wh_mlp_forward_x(const wh_mlp_desc* d, const void* packed, int64_t rows, const void* xfrag, float* logits,
                     int32_t* actions, int32_t explore, uint64_t seed, uint32_t step, void* stream) {
  (void)d, (void)packed, (void)rows, (void)xfrag, (void)logits, (void)actions, (void)explore, (void)seed, (void)step,
      (void)stream;
  return WH_ENOTSUP;
}
int wh_check_read(uint64_t* out, int32_t clear) {
  (void)out, (void)clear;
  return WH_ENOTSUP;
}

}  // extern "C"
