// The host engine (csrc/host_engine.cpp) under AddressSanitizer + UndefinedBehaviorSanitizer: every
// computing entry point over the three variants, with ragged batches, Train agent counts, masks, dict
// orders of up to 4*NA entries, injected and philox draws, rollouts across episode ends and
// episode metrics -- all buffers exactly the sizes the header states, so any read or write past
// them, any shift or overflow UB and any leak is reported.  Built and run by `make asan-host`
// (tests/test_asan_host.py); prints "ASAN HOST ENGINE OK" on a clean run.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "warehouse_amd.h"

namespace {

int fails = 0;
#define EXPECT(c)                                                  \
  do {                                                             \
    if (!(c)) {                                                    \
      fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                     \
    }                                                              \
  } while (0)

wh_config variant(int D, int R, std::vector<int> racks, int na) {
  wh_config c{};
  c.area_dimension = D;
  c.num_requests = R;
  c.num_racks = (int32_t)racks.size();
  for (size_t i = 0; i < racks.size(); ++i) c.racks[i] = racks[i];
  c.agent_slots = na;
  c.episode_duration = 200;
  c.pickup_wait_duration = 200;
  return c;
}

void exercise(const wh_config& cfg, int64_t B, bool train, uint64_t seed) {
  wh_layout L{};
  EXPECT(wh_query(&cfg, &L) == WH_OK);
  const int NA = cfg.agent_slots, R = cfg.num_requests, OBS = L.obs_len;
  std::vector<uint32_t> state((size_t)L.words_per_env * B);
  std::vector<float> rew((size_t)B * NA), obs((size_t)B * NA * OBS);
  std::vector<uint8_t> done(B), mask(B);
  std::vector<int32_t> acts((size_t)B * NA), ninact(B);
  std::mt19937 rng((uint32_t)seed);

  // philox reset, then injected resets of half the envs
  EXPECT(wh_reset(&cfg, B, state.data(), nullptr, nullptr, train, seed, 0, nullptr) == WH_OK);
  std::vector<int32_t> spawn((size_t)B * NA * 2), pk((size_t)B * R), tg((size_t)B * R), nn(B);
  for (int64_t e = 0; e < B; ++e) {
    for (int i = 0; i < NA; ++i) {
      spawn[(e * NA + i) * 2] = 1 + (int)(rng() % (cfg.area_dimension - 2));
      spawn[(e * NA + i) * 2 + 1] = 1 + (int)(rng() % (cfg.area_dimension - 2));
    }
    for (int j = 0; j < R; ++j) {
      pk[e * R + j] = j * (L.num_pickups / R);          // distinct pickup points
      tg[e * R + j] = (int)(rng() % L.num_deliveries);
    }
    nn[e] = 1 + (int)(rng() % NA);
    mask[e] = (uint8_t)(e & 1);
  }
  wh_reset_draws dr{spawn.data(), pk.data(), tg.data(), train ? nn.data() : nullptr};
  EXPECT(wh_reset(&cfg, B, state.data(), mask.data(), &dr, train, seed, 0, nullptr) == WH_OK);
  EXPECT(wh_observe(&cfg, B, state.data(), obs.data(), nullptr) == WH_OK);

  // wh_step: ascending, dict orders of every length 1 .. 4*NA, phases with injected regeneration
  for (int s = 0; s < 60; ++s) {
    for (auto& a : acts) a = (int32_t)(rng() % 9);
    const int ol = 1 + (int)(rng() % (4 * NA));
    std::vector<int32_t> order((size_t)B * ol);
    for (auto& o : order) {
      const uint32_t r = rng();
      o = (r % 7 == 0) ? -1 : (int32_t)((r % NA) | ((r >> 8) % 10 << 8));   // entry action 0 = actions[]
    }
    const bool use_order = s % 3 != 0;
    if (s % 2) {
      EXPECT(wh_step(&cfg, B, state.data(), acts.data(), use_order ? order.data() : nullptr, use_order ? ol : 0,
                     rew.data(), done.data(), nullptr, nullptr, WH_PHASE_ALL, seed, 0, nullptr) == WH_OK);
    } else {
      EXPECT(wh_step(&cfg, B, state.data(), acts.data(), use_order ? order.data() : nullptr, use_order ? ol : 0,
                     rew.data(), done.data(), nullptr, ninact.data(), WH_PHASE_PRE_REGEN, seed, 0, nullptr) == WH_OK);
      std::vector<int32_t> regen((size_t)B * 2 * R);
      for (int64_t e = 0; e < B; ++e)
        for (int j = 0; j < R; ++j) {
          regen[e * 2 * R + j] = ninact[e] > 0 ? (int32_t)(rng() % (uint32_t)ninact[e]) : 0;
          regen[e * 2 * R + R + j] = (int32_t)(rng() % L.num_deliveries);
        }
      EXPECT(wh_step(&cfg, B, state.data(), nullptr, nullptr, 0, nullptr, nullptr, regen.data(), nullptr,
                     WH_PHASE_REGEN, seed, 0, nullptr) == WH_OK);
    }
  }
  EXPECT(wh_observe(&cfg, B, state.data(), obs.data(), nullptr) == WH_OK);

  // episode metrics, rollouts across episode ends (greedy with coins, random), policy alone
  std::vector<uint32_t> eret(B), rmin(NA + 1, 0xFFFFFFFFu), rmax(NA + 1);
  std::vector<uint64_t> rsum(NA + 1), neps(NA + 1);
  wh_episode_stats st{eret.data(), rsum.data(), neps.data(), rmin.data(), rmax.data()};
  const int K = 230;
  std::vector<float> krew((size_t)K * B * NA), ret(B);
  std::vector<uint8_t> kdone((size_t)K * B);
  EXPECT(wh_rollout(&cfg, B, state.data(), K, WH_POLICY_GREEDY, 0.2f, krew.data(), kdone.data(), ret.data(), &st,
                    1, train, seed, 0, nullptr) == WH_OK);
  EXPECT(wh_rollout(&cfg, B, state.data(), 30, WH_POLICY_RANDOM, 0.0f, nullptr, nullptr, nullptr, nullptr, 1, train,
                    seed, 0, nullptr) == WH_OK);
  EXPECT(wh_policy(&cfg, B, state.data(), WH_POLICY_GREEDY, 0.5f, acts.data(), seed, 0, nullptr) == WH_OK);

  // the sampler routes: masked dict-order vector steps with rows and metrics, sampler steps, a fragment
  for (int s = 0; s < 40; ++s) {
    for (auto& a : acts) a = (int32_t)(rng() % 9);
    for (auto& m : mask) m = (uint8_t)(rng() & 1);
    const int ol = 1 + (int)(rng() % (4 * NA));
    std::vector<int32_t> order((size_t)B * ol);
    for (auto& o : order) o = (rng() % 5 == 0) ? -1 : (int32_t)(rng() % NA);
    EXPECT(wh_vector_step(&cfg, B, state.data(), acts.data(), s % 2 ? order.data() : nullptr, s % 2 ? ol : 0,
                          s % 3 ? mask.data() : nullptr, rew.data(), done.data(), obs.data(), &st, 1, train, seed, 0,
                          nullptr) == WH_OK);
    EXPECT(wh_sampler_step(&cfg, B, state.data(), s % 2 ? WH_POLICY_GREEDY : WH_POLICY_RANDOM, 0.1f, rew.data(),
                           done.data(), obs.data(), &st, train, seed, 0, nullptr) == WH_OK);
  }
  const int F = 7;
  std::vector<float> frew((size_t)F * B * NA), fobs((size_t)F * B * NA * OBS);
  std::vector<uint8_t> fdone((size_t)F * B);
  EXPECT(wh_sampler_rollout(&cfg, B, state.data(), F, WH_POLICY_GREEDY, 0.0f, frew.data(), fdone.data(), fobs.data(),
                            &st, train, seed, 0, nullptr) == WH_OK);

  // canonical round trip
  const int P = L.num_pickups;
  std::vector<int32_t> pos((size_t)B * NA * 2), at((size_t)B * NA), pt((size_t)B * P), ptm((size_t)B * P), t(B), n(B);
  std::vector<uint8_t> fresh(B);
  std::vector<uint32_t> ep(B), state2(state.size());
  EXPECT(wh_unpack(&cfg, B, state.data(), pos.data(), at.data(), pt.data(), ptm.data(), t.data(), n.data(),
                   fresh.data(), ep.data(), nullptr) == WH_OK);
  EXPECT(wh_pack(&cfg, B, pos.data(), at.data(), pt.data(), ptm.data(), t.data(), n.data(), fresh.data(), ep.data(),
                 state2.data(), nullptr) == WH_OK);
  std::vector<float> obs2(obs.size());
  EXPECT(wh_observe(&cfg, B, state.data(), obs.data(), nullptr) == WH_OK);
  EXPECT(wh_observe(&cfg, B, state2.data(), obs2.data(), nullptr) == WH_OK);
  EXPECT(memcmp(obs.data(), obs2.data(), obs.size() * sizeof(float)) == 0);

  // argument checks: an order row longer than 4*NA, a policy id out of range
  EXPECT(wh_step(&cfg, B, state.data(), acts.data(), acts.data(), 4 * NA + 1, nullptr, nullptr, nullptr, nullptr,
                 WH_PHASE_ALL, seed, 0, nullptr) == WH_EINVAL);
  EXPECT(wh_policy(&cfg, B, state.data(), 7, 0.0f, acts.data(), seed, 0, nullptr) == WH_EINVAL);
}

}  // namespace

int main() {
  exercise(variant(12, 4, {4, 8}, 4), 37, false, 11);          // Small-4
  exercise(variant(12, 4, {4, 8}, 4), 5, true, 12);            // SmallTrain
  exercise(variant(16, 9, {4, 8, 12}, 8), 29, false, 13);      // Medium-8
  exercise(variant(16, 9, {4, 8, 12}, 9), 17, true, 14);       // MediumTrain
  exercise(variant(20, 16, {4, 8, 12, 16}, 16), 9, false, 15); // Large-16
  exercise(variant(20, 16, {4, 8, 12, 16}, 3), 11, true, 16);  // Large, 3 slots, Train
  if (fails) {
    fprintf(stderr, "%d check(s) failed\n", fails);
    return 1;
  }
  printf("ASAN HOST ENGINE OK\n");
  return 0;
}
