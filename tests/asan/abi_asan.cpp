// Host-side AddressSanitizer run of the C ABI (SURVEY.md §5 "Race detection / sanitizers": a debug build
// with -fsanitize=address on the host C++).  Built by `make -C rllib-warehouse_amd/csrc asan` against
// an ASan-instrumented, host-only compile of the library's sources (the kernels are not in it: nothing
// here launches one), run by tests/test_asan_host.py on a machine without a GPU.  Exercises every
// host path that runs before a device is needed: config validation (wh_query and each entry point's
// own argument checks), the launch-handle lifecycle (prepare / run / free, double free and foreign
// handles refused, error paths that must not leak), pack/unpack/observe/step argument checks and the
// MLP descriptor checks.  Exit status 0 and "ASAN ABI OK" = every expectation held and ASan (with
// LeakSanitizer) reported nothing.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "warehouse_amd.h"

static int g_fail = 0;
#define EXPECT(cond)                                                    \
  do {                                                                  \
    if (!(cond)) {                                                      \
      fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++g_fail;                                                         \
    }                                                                   \
  } while (0)

static wh_config variant(int D, int R, std::vector<int> racks, int na) {
  wh_config c;
  memset(&c, 0, sizeof(c));
  c.area_dimension = D;
  c.num_requests = R;
  c.num_racks = (int)racks.size();
  for (size_t i = 0; i < racks.size(); ++i) c.racks[i] = racks[i];
  c.agent_slots = na;
  c.episode_duration = 200;
  c.pickup_wait_duration = 200;
  return c;
}

int main() {
  EXPECT(wh_version() != nullptr && strstr(wh_version(), "sha=") != nullptr);

  // ---- config validation: the variants of warehouse/variants.py:25-62 and every agent count
  const wh_config small = variant(12, 4, {4, 8}, 4), medium = variant(16, 9, {4, 8, 12}, 8),
                  large = variant(20, 16, {4, 8, 12, 16}, 16);
  for (const wh_config* c : {&small, &medium, &large}) {
    for (int na = 1; na <= c->num_requests; ++na) {
      wh_config v = *c;
      v.agent_slots = na;
      wh_layout L;
      memset(&L, 0xAB, sizeof(L));
      EXPECT(wh_query(&v, &L) == WH_OK);
      EXPECT(L.kernel_agents >= na && L.obs_len == 9 * v.num_requests + 1);
      EXPECT(L.words_per_env == 2 + na + 2 * (L.num_pickups / 4));
      EXPECT(wh_query(&v, nullptr) == WH_OK);
    }
  }
  EXPECT(wh_query(nullptr, nullptr) == WH_EINVAL);
  {
    wh_config c = medium;
    c.agent_slots = 10;   // > R (core.py:89)
    EXPECT(wh_query(&c, nullptr) == WH_EINVAL);
    c = medium; c.agent_slots = 0; EXPECT(wh_query(&c, nullptr) == WH_EINVAL);
    c = medium; c.area_dimension = 4; EXPECT(wh_query(&c, nullptr) == WH_EINVAL);
    c = medium; c.area_dimension = 33; EXPECT(wh_query(&c, nullptr) == WH_EINVAL);
    c = medium; c.num_racks = 0; EXPECT(wh_query(&c, nullptr) == WH_EINVAL);
    c = medium; c.num_racks = WH_MAX_RACKS + 1; EXPECT(wh_query(&c, nullptr) == WH_EINVAL);
    c = medium; c.racks[0] = 1; EXPECT(wh_query(&c, nullptr) == WH_ENOTSUP);     // not interior
    c = medium; c.racks[2] = 15; EXPECT(wh_query(&c, nullptr) == WH_ENOTSUP);
    c = medium; c.pickup_wait_duration = 0; EXPECT(wh_query(&c, nullptr) == WH_EINVAL);
    c = medium; c.pickup_wait_duration = 256; EXPECT(wh_query(&c, nullptr) == WH_EINVAL);
    c = medium; c.episode_duration = -1; EXPECT(wh_query(&c, nullptr) == WH_EINVAL);
    c = variant(14, 9, {4, 8, 12}, 8);    // a geometry this build has no kernel for
    EXPECT(wh_query(&c, nullptr) == WH_ENOTSUP);
  }

  // ---- the launch-handle lifecycle (wh_rollout_prepare / wh_launch_run / wh_launch_free)
  uint32_t dummy_state[4] = {0, 0, 0, 0};
  float rew[8];
  uint8_t dn[1];
  wh_launch* h = reinterpret_cast<wh_launch*>(0x1);
  EXPECT(wh_rollout_prepare(&medium, 0, dummy_state, 20, WH_POLICY_GREEDY, 0.0f, rew, dn, nullptr, nullptr, 1, 0,
                            1234, 0, nullptr, nullptr) == WH_EINVAL);                       // no out
  EXPECT(wh_rollout_prepare(&medium, 0, dummy_state, 20, 7, 0.0f, rew, dn, nullptr, nullptr, 1, 0, 1234, 0, nullptr,
                            &h) == WH_EINVAL && h == nullptr);                              // bad policy
  EXPECT(wh_rollout_prepare(&medium, 0, dummy_state, -1, WH_POLICY_GREEDY, 0.0f, rew, dn, nullptr, nullptr, 1, 0,
                            1234, 0, nullptr, &h) == WH_EINVAL && h == nullptr);            // steps < 0
  EXPECT(wh_rollout_prepare(&medium, 0, dummy_state, 20, WH_POLICY_GREEDY, 1.5f, rew, dn, nullptr, nullptr, 1, 0,
                            1234, 0, nullptr, &h) == WH_EINVAL && h == nullptr);            // p > 1
  EXPECT(wh_rollout_prepare(&medium, -5, dummy_state, 20, WH_POLICY_GREEDY, 0.0f, rew, dn, nullptr, nullptr, 1, 0,
                            1234, 0, nullptr, &h) == WH_EINVAL && h == nullptr);            // B < 0
  {
    wh_episode_stats st;
    memset(&st, 0, sizeof(st));
    uint64_t sums[17];
    st.return_sum = sums;   // bins without the per-env return accumulator
    EXPECT(wh_rollout_prepare(&medium, 0, dummy_state, 20, WH_POLICY_GREEDY, 0.0f, rew, dn, nullptr, &st, 1, 0,
                              1234, 0, nullptr, &h) == WH_EINVAL && h == nullptr);
  }
  wh_config bad = medium;
  bad.agent_slots = 12;
  EXPECT(wh_rollout_prepare(&bad, 0, dummy_state, 20, WH_POLICY_GREEDY, 0.0f, rew, dn, nullptr, nullptr, 1, 0, 1234,
                            0, nullptr, &h) == WH_EINVAL && h == nullptr);                  // invalid config
  // B > 0 needs the device's tables: without a GPU the HIP error comes back and nothing leaks
  const int rc_dev = wh_rollout_prepare(&medium, 64, dummy_state, 20, WH_POLICY_GREEDY, 0.0f, rew, dn, nullptr,
                                        nullptr, 1, 0, 1234, 0, nullptr, &h);
  EXPECT(rc_dev >= WH_EHIP && h == nullptr);
  // B = 0: a valid handle that launches nothing
  for (int rep = 0; rep < 3; ++rep) {
    wh_launch* a = nullptr;
    wh_launch* b = nullptr;
    EXPECT(wh_rollout_prepare(&medium, 0, nullptr, 20, WH_POLICY_GREEDY, 0.0f, nullptr, nullptr, nullptr, nullptr, 1,
                              0, 1234, 0, nullptr, &a) == WH_OK && a != nullptr);
    EXPECT(wh_rollout_prepare(&large, 0, nullptr, 200, WH_POLICY_RANDOM, 0.5f, nullptr, nullptr, nullptr, nullptr, 1,
                              1, 7, 0, nullptr, &b) == WH_OK && b != nullptr && b != a);
    EXPECT(wh_launch_run(a) == WH_OK);
    EXPECT(wh_launch_run_timed(b, nullptr, nullptr) == WH_OK);
    EXPECT(wh_launch_free(a) == WH_OK);
    EXPECT(wh_launch_free(a) == WH_EINVAL);         // double free refused
    EXPECT(wh_launch_run(a) == WH_EINVAL);          // use after free refused
    EXPECT(wh_launch_run_timed(a, nullptr, nullptr) == WH_EINVAL);
    EXPECT(wh_launch_run(b) == WH_OK);               // the other handle is untouched
    EXPECT(wh_launch_free(b) == WH_OK);
  }
  EXPECT(wh_launch_free(nullptr) == WH_OK);
  EXPECT(wh_launch_run(nullptr) == WH_EINVAL);
  {
    int not_a_handle[16] = {0};
    EXPECT(wh_launch_free(reinterpret_cast<wh_launch*>(not_a_handle)) == WH_EINVAL);
    EXPECT(wh_launch_run(reinterpret_cast<wh_launch*>(not_a_handle)) == WH_EINVAL);
  }

  // ---- argument checks of the other entry points (empty batches run nothing)
  EXPECT(wh_step(&medium, 0, nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr, nullptr, 7, 0, 0, nullptr) == WH_EINVAL);
  EXPECT(wh_step(&medium, 4, dummy_state, nullptr, nullptr, 0, rew, dn, nullptr, nullptr, WH_PHASE_ALL, 0, 0, nullptr) == WH_EINVAL);
  EXPECT(wh_step(&medium, 4, dummy_state, (const int32_t*)dummy_state, (const int32_t*)dummy_state, 37, rew, dn, nullptr, nullptr, WH_PHASE_ALL, 0, 0, nullptr) == WH_EINVAL);   // order rows > 4 NA
  EXPECT(wh_step(&medium, 0, nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr, nullptr, WH_PHASE_ALL, 0, 0, nullptr) == WH_OK);
  EXPECT(wh_policy(&medium, 0, nullptr, 9, 0.0f, nullptr, 0, 0, nullptr) == WH_EINVAL);
  EXPECT(wh_policy(&medium, 0, nullptr, WH_POLICY_GREEDY, -0.1f, nullptr, 0, 0, nullptr) == WH_EINVAL);
  EXPECT(wh_policy(&medium, 0, nullptr, WH_POLICY_GREEDY, 0.0f, nullptr, 0, 0, nullptr) == WH_OK);
  EXPECT(wh_rollout(&medium, 0, nullptr, 20, WH_POLICY_GREEDY, 0.0f, nullptr, nullptr, nullptr, nullptr, 1, 0, 0, 0, nullptr) == WH_OK);
  EXPECT(wh_rollout(&bad, 0, nullptr, 20, WH_POLICY_GREEDY, 0.0f, nullptr, nullptr, nullptr, nullptr, 1, 0, 0, 0, nullptr) == WH_EINVAL);
  EXPECT(wh_reset(&medium, 0, nullptr, nullptr, nullptr, 0, 0, 0, nullptr) == WH_OK);
  EXPECT(wh_reset(&bad, 0, nullptr, nullptr, nullptr, 0, 0, 0, nullptr) == WH_EINVAL);
  EXPECT(wh_pack(&medium, 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) == WH_OK);
  EXPECT(wh_pack(&medium, 4, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) == WH_EINVAL);
  EXPECT(wh_unpack(&medium, 4, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) == WH_EINVAL);
  EXPECT(wh_observe(&medium, 0, nullptr, nullptr, nullptr) == WH_OK);
  EXPECT(wh_observe(&bad, 0, nullptr, nullptr, nullptr) == WH_EINVAL);
  EXPECT(wh_vector_step(&medium, 4, dummy_state, nullptr, nullptr, 0, nullptr, rew, dn, nullptr, nullptr, 1, 0, 0, 0, nullptr) == WH_EINVAL);
  EXPECT(wh_vector_step(&medium, 0, nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr, nullptr, nullptr, 1, 0, 0, 0, nullptr) == WH_OK);
  const int32_t acts[32] = {0};
  alignas(16) unsigned char xbuf[64];
  EXPECT(wh_vector_step_x(&medium, 4, dummy_state, nullptr, nullptr, 0, nullptr, rew, dn, rew, nullptr, 1, 0, 0, 0, nullptr) == WH_EINVAL);
  EXPECT(wh_vector_step_x(&medium, 4, dummy_state, acts, nullptr, 0, nullptr, rew, dn, nullptr, nullptr, 1, 0, 0, 0, nullptr) == WH_EINVAL);
  EXPECT(wh_vector_step_x(&medium, 4, dummy_state, acts, nullptr, 0, nullptr, rew, dn, xbuf + 4, nullptr, 1, 0, 0, 0, nullptr) == WH_EINVAL);
  EXPECT(wh_vector_step_x(&medium, 0, nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr, nullptr, nullptr, 1, 0, 0, 0, nullptr) == WH_OK);
  EXPECT(wh_sampler_step(&medium, 0, nullptr, 5, 0.0f, nullptr, nullptr, nullptr, nullptr, 0, 0, 0, nullptr) == WH_EINVAL);
  EXPECT(wh_sampler_rollout(&medium, 4, dummy_state, 3, WH_POLICY_GREEDY, 0.0f, rew, dn, nullptr, nullptr, 0, 0, 0, nullptr) == WH_EINVAL);
  EXPECT(wh_sampler_rollout(&medium, 0, nullptr, 3, WH_POLICY_GREEDY, 0.0f, nullptr, nullptr, nullptr, nullptr, 0, 0, 0, nullptr) == WH_OK);
  EXPECT(wh_sampler_step_to(&medium, 4, dummy_state, nullptr, WH_POLICY_GREEDY, 0.0f, rew, dn, nullptr, 0, 0, 0, nullptr) == WH_EINVAL);
  uint64_t chk[4];
  EXPECT(wh_check_read(chk, 0) == WH_ENOTSUP);      // production build: no assert-mode counters

  // ---- MLP descriptors (scripts/experiments/warehouse-*-sac policy_model shapes)
  const wh_mlp_desc dm{82, 512, 512, 9, WH_MLP_BF16}, dl{145, 1024, 256, 9, WH_MLP_F32}, ds{37, 256, 256, 9, WH_MLP_BF16};
  for (const wh_mlp_desc* d : {&dm, &dl, &ds}) {
    int64_t bytes = -1;
    EXPECT(wh_mlp_query(d, &bytes) == WH_OK && bytes > 0 && bytes % 16 == 0);
  }
  const wh_mlp_desc odd{83, 512, 512, 9, WH_MLP_BF16}, badp{82, 512, 512, 9, 7};
  int64_t bytes = 0;
  EXPECT(wh_mlp_query(&odd, &bytes) == WH_ENOTSUP);
  EXPECT(wh_mlp_query(&badp, &bytes) != WH_OK);
  EXPECT(wh_mlp_query(nullptr, &bytes) != WH_OK);
  EXPECT(wh_mlp_forward(&dm, nullptr, 0, nullptr, nullptr, nullptr, 0, 0, 0, nullptr) == WH_OK);
  EXPECT(wh_mlp_forward(&dm, nullptr, -1, nullptr, nullptr, nullptr, 0, 0, 0, nullptr) == WH_EINVAL);
  EXPECT(wh_mlp_forward(&dm, nullptr, 32, nullptr, nullptr, nullptr, 0, 0, 0, nullptr) == WH_EINVAL);

  if (g_fail) {
    fprintf(stderr, "%d expectation(s) failed\n", g_fail);
    return 1;
  }
  printf("ASAN ABI OK\n");
  return 0;
}
