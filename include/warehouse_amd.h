/*
 * warehouse_amd.h -- C ABI of the MI355X (gfx950) batched warehouse simulator.
 *
 * Drop-in boundary for the hot path of ffahleraz/rllib-warehouse: `Warehouse.reset()` /
 * `Warehouse.step()` (warehouse/core.py:167-442) and the greedy baseline policy
 * (baseline/solvers.py:27-58), run for B independent episodes on one GPU.  Plain pointers and
 * sizes only; every pointer named "device" is HIP device memory, `stream` is a hipStream_t
 * (NULL = the default stream).  The host engine (libwarehouse_host.so, csrc/host_engine.cpp: the
 * same entry points on host cores, for hosts without a GPU) takes host memory for every "device"
 * pointer, ignores `stream`, runs synchronously, and returns WH_ENOTSUP for the device-only entry
 * points (policy network, fragment operand, two-stream and prepared launches, assert mode).
 * All calls are asynchronous on `stream` except where noted, return
 * WH_OK (0) or a WH_E* code, and never throw.  The reference is Python, so the binding a maintainer
 * adds on the reference side is ctypes; `warehouse/_native.py` is that binding.
 *
 * PACKED STATE (device, struct-of-arrays across the batch, word-plane major):
 *   state[w * B + e] is 32-bit word w of env e, 0 <= w < wh_layout.words_per_env:
 *     w = 0            header : bits 0-15 t (episode time, core.py:165), bits 16-23 n (live agents),
 *                               bit 24 fresh (set by reset: observation availabilities read 0,
 *                               core.py:233)
 *     w = 1            episode counter (bumped by every reset; keys the philox streams)
 *     w = 2 .. 2+NA-1  agent slot i: byte0 x, byte1 dx, byte2 y, byte3 dy (core.py:153-154), where
 *                      (dx, dy) is the cell of the agent's delivery target and 0xFF,0xFF when it
 *                      carries nothing; slots >= n hold 0xFF00FF00 (idle at (0,0))
 *     next P/4 words   pickup point j, byte j%4 of word j/4: (request target + 1, 0 = no request)
 *                      (core.py:158)
 *     next P/4 words   pickup point j: low 8 bits of the step at which its request expires
 *                      (opened at step t0: t0 + W; steps left = (byte - t) mod 256, core.py:159;
 *                      don't-care when the point has no request)
 *   NA = cfg.agent_slots, P = 4 * num_racks^2.
 *
 * RNG MODES.  Every draw the reference takes from numpy's global MT19937 stream can either be
 * INJECTED (explicit arrays below: bit-exact parity with the reference given its draws) or taken
 * from the PHILOX contract: Philox4x32-10 keyed by `seed`, counter (env_offset + e, episode, t,
 * purpose << 24 | block); purposes RESET=1, REGEN=2, POLICY=3, RANDOM=4 (word layout in
 * DESIGN.md §RNG and oracle/philox.py).  Philox trajectories depend only on the global env id,
 * so any sharding of env ids over GPUs reproduces them exactly.
 */
#ifndef WAREHOUSE_AMD_H
#define WAREHOUSE_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WH_OK 0
#define WH_EINVAL 22      /* bad pointer / size / value */
#define WH_ENOTSUP 95     /* a layout this build has no kernel for */
#define WH_EHIP 1000      /* + hipError_t: a HIP runtime error */

#define WH_MAX_RACKS 8

/* Variant geometry.  Mirrors the constructor of warehouse/core.py:78-86
 * (the variant table is warehouse/variants.py:25-62). */
typedef struct wh_config {
  int32_t area_dimension;        /* D                          core.py:82 */
  int32_t num_requests;          /* R (always-open requests)   core.py:81 */
  int32_t num_racks;             /* len(pickup_racks_arrangement) */
  int32_t racks[WH_MAX_RACKS];   /* pickup_racks_arrangement   core.py:83 */
  int32_t agent_slots;           /* NA: agent records per env (num_agents, or max_num_agents for
                                    the Train variants, variants.py:65-98); 1 <= NA <= R */
  int32_t episode_duration;      /* T                          core.py:84 */
  int32_t pickup_wait_duration;  /* W (<= 255)                 core.py:85 */
} wh_config;

typedef struct wh_layout {
  int32_t words_per_env;   /* packed state words per env */
  int32_t num_pickups;     /* P  = 4 * num_racks^2        core.py:96 */
  int32_t num_deliveries;  /* Dp = 4 * (D - 4)            core.py:97 */
  int32_t obs_len;         /* 9R + 1 floats per agent row, sorted gym.spaces.Dict key order */
  int32_t kernel_agents;   /* compile-time agent bound of the kernel chosen for this config */
} wh_layout;

/* Validate `cfg` and describe its packed layout.  Host only, synchronous. */
int wh_query(const wh_config* cfg, wh_layout* out);

/* Canonical <-> packed state.  Canonical arrays are int32 device tensors:
 *   pos [B,NA,2], agent_target [B,NA] (-1 idle), pickup_target [B,P] (-1 none),
 *   pickup_timer [B,P] (-1 none), t [B], n [B]; fresh [B] uint8; episode [B] uint32.
 * (the reference's own state arrays, core.py:150-165) */
int wh_pack(const wh_config* cfg, int64_t B, const int32_t* pos, const int32_t* agent_target,
            const int32_t* pickup_target, const int32_t* pickup_timer, const int32_t* t,
            const int32_t* n, const uint8_t* fresh, const uint32_t* episode, uint32_t* state,
            void* stream);
int wh_unpack(const wh_config* cfg, int64_t B, const uint32_t* state, int32_t* pos,
              int32_t* agent_target, int32_t* pickup_target, int32_t* pickup_timer, int32_t* t,
              int32_t* n, uint8_t* fresh, uint32_t* episode, void* stream);

/* Injected reset draws (core.py:191-221): accepted spawn cells, the R opened pickups and their
 * targets in draw order, and (Train variants, variants.py:73-74) the agent count. */
typedef struct wh_reset_draws {
  const int32_t* spawn;    /* [B,NA,2] */
  const int32_t* pickups;  /* [B,R]    distinct pickup indices */
  const int32_t* targets;  /* [B,R]    delivery indices */
  const int32_t* n;        /* [B] or NULL (= NA) */
} wh_reset_draws;

/* Warehouse.reset()  (warehouse/core.py:167-260; Train variants variants.py:69-71).
 * mask [B] uint8 or NULL (all); draws NULL = philox; variable_n != 0 draws n ~ U{1..NA}. */
int wh_reset(const wh_config* cfg, int64_t B, uint32_t* state, const uint8_t* mask,
             const wh_reset_draws* draws, int32_t variable_n, uint64_t seed, int64_t env_offset,
             void* stream);

#define WH_PHASE_ALL 0        /* the whole of core.py:262-442 */
#define WH_PHASE_PRE_REGEN 1  /* everything but regeneration (core.py:267-335, 354-442);
                                 writes n_inactive so a host can draw the reference's
                                 np.random.choice(inactive, k) before WH_PHASE_REGEN */
#define WH_PHASE_REGEN 2      /* regeneration only (core.py:338-351) */

/* Warehouse.step(action_dict)  (warehouse/core.py:262-442).
 *   actions   [B,NA] int32 in 0..8 (MOVES index, core.py:38; the host wraps -9..-1 like Python)
 *   order     [B,OL] int32 or NULL: action-dict iteration order (core.py:279), -1 entries skipped
 *             (rows are -1 padded); agents not listed do not move.  NULL = ascending agent id.
 *             Entry = agent id in bits 0-7, optionally (bits 8-15) that dict entry's own action + 1,
 *             0 = actions[e,id]: a dict naming one agent under several keys ('0', 0, '-n', -n: int(key)
 *             indexes like numpy, core.py:280) moves it once per entry with that entry's action.
 *   order_len OL, the order row length: 0 = NA, else 1 .. 4*NA (a dict may name every agent under
 *             all four of its key forms); anything else is WH_EINVAL.
 *   rewards   [B,NA] float32 (core.py:334-368), dones [B] uint8 (core.py:438); either may be NULL
 *   regen     [B,2R] int32 or NULL (philox): R positions into the ascending list of inactive
 *             pickups (the index np.random.choice(inactive,k) picked), then R delivery targets;
 *             only the first k = R - P + |inactive| of each are read.
 *   n_inactive [B] int32 or NULL: |inactive| before regeneration (core.py:338). */
int wh_step(const wh_config* cfg, int64_t B, uint32_t* state, const int32_t* actions,
            const int32_t* order, int32_t order_len, float* rewards, uint8_t* dones, const int32_t* regen,
            int32_t* n_inactive, int32_t phase, uint64_t seed, int64_t env_offset, void* stream);

/* Per-agent observation rows (core.py:224-260 after reset, 371-432 after a step, including the
 * row-1 quirk of core.py:428), flattened in sorted-key order:
 *   num_agents, other_availabilities, other_delivery_targets, other_positions, requests,
 *   self_availability, self_delivery_target, self_position
 * obs [B,NA,9R+1] float32; rows of slots >= n are zero. */
int wh_observe(const wh_config* cfg, int64_t B, const uint32_t* state, float* obs, void* stream);
/* wh_observe plus (xfrag != NULL) the same rows as the SAC policy network's layer-0 operand, for
 * wh_mlp_forward_x: bf16 in MFMA fragment order, ceil(B*NA/32) tiles of 32 agent rows x KQ =
 * ceil((9R+3)/16) k-steps x 64 lanes x 16 bytes; 16-byte chunk ((tile*KQ + q)*64 + lane) = features
 * 16q + 8(lane>>5) + j, j < 8, of row tile*32 + (lane&31), features 9R+1 and 9R+2 = 1.0, padding 0
 * (rows past B*NA: zero features but the two 1.0 columns).  obs may be NULL.  Every agent count
 * is supported; xfrag must be 16-byte aligned. */
int wh_observe_x(const wh_config* cfg, int64_t B, const uint32_t* state, float* obs, void* xfrag, void* stream);

#define WH_POLICY_GREEDY 1    /* baseline/solvers.py:27-58 with random_action_prob p */
#define WH_POLICY_RANDOM 2    /* uniform over the 9 moves (action_space.sample()) */

/* WarehouseRandomGreedySolver.compute_action (baseline/solvers.py:27-58) evaluated on the state,
 * or uniform random actions: writes actions [B,NA] int32 (slots >= n get 4 = stay). */
int wh_policy(const wh_config* cfg, int64_t B, const uint32_t* state, int32_t policy, float p,
              int32_t* actions, uint64_t seed, int64_t env_offset, void* stream);

/* Episode metrics of scripts/train.py:18-23 (on_episode_end: avg_agent_reward = episode return
 * summed over agents / n, reported overall and per n), accumulated on the device.  Rewards are
 * whole numbers, so returns are kept as integers and every total is exact and order-independent:
 * the mean avg_agent_reward of the episodes with n agents is return_sum[n] / (n * episodes[n]).
 * Bins are indexed by n (arrays of agent_slots + 1); the caller zeroes them (return_min to
 * 0xFFFFFFFF).  `episode_return` is required when any bin pointer is set; others may be NULL.
 * An episode is counted at the step whose done flag is set; continuing a done env without a reset
 * counts it again (the reference has no guard after done either, core.py:438). */
typedef struct wh_episode_stats {
  uint32_t* episode_return;  /* [B]      running return of each env's current episode (read+write) */
  uint64_t* return_sum;      /* [NA + 1] += return of every finished episode, binned by its n */
  uint64_t* episodes;        /* [NA + 1] += finished episodes */
  uint32_t* return_min;      /* [NA + 1] min= episode return */
  uint32_t* return_max;      /* [NA + 1] max= episode return */
} wh_episode_stats;

/* Device-resident rollout: `steps` iterations of {policy, step, auto-reset at t >= T} in one
 * launch (the loop of baseline/run.py:42-62 without the host).  State stays in registers between
 * iterations.  rewards [steps,B,NA] / dones [steps,B] / returns [B] (+= sum of rewards) / stats
 * may each be NULL.  Philox draws only. */
int wh_rollout(const wh_config* cfg, int64_t B, uint32_t* state, int32_t steps, int32_t policy,
               float p, float* rewards, uint8_t* dones, float* returns, const wh_episode_stats* stats,
               int32_t autoreset, int32_t variable_n, uint64_t seed, int64_t env_offset, void* stream);

/* One step of an RLlib-style vectorised sampler (the route scripts/train.py's workload takes:
 * policy actions in, {obs, rewards, dones} out, done episodes restarted): wh_step with philox
 * draws, then (autoreset != 0) a philox reset of every env whose episode ended -- Train variants
 * (variable_n != 0) redraw n there, variants.py:69-71 -- then wh_observe into obs (NULL = skip).
 * With autoreset the obs rows of a done env are the first rows of its next episode.
 *   actions [B,NA] int32 0..8 (others act as 4 = stay)
 *   order   [B,OL] int32 or NULL (OL = order_len as in wh_step): each env's action-dict iteration
 *           order (core.py:279), -1 padded; agents not listed are skipped -- they neither move nor
 *           re-mark their cell (core.py:279-300 only visits the dict's keys).  NULL = every agent,
 *           ascending id.  Entries as wh_step's (bits 8-15: the entry's own action + 1, for repeated
 *           agents).
 *   mask [B] uint8 or NULL: only envs with mask != 0 are stepped (the others keep their state;
 *   their rewards/dones are not written); rewards [B,NA] / dones [B] / obs [B,NA,9R+1] / stats
 *   may be NULL. */
int wh_vector_step(const wh_config* cfg, int64_t B, uint32_t* state, const int32_t* actions,
                   const int32_t* order, int32_t order_len, const uint8_t* mask, float* rewards, uint8_t* dones, float* obs,
                   const wh_episode_stats* stats, int32_t autoreset, int32_t variable_n,
                   uint64_t seed, int64_t env_offset, void* stream);

/* wh_vector_step writing the rows as wh_observe_x's fragment-order operand (xfrag, 16-byte
 * aligned, [ceil(B*NA/32), KQ, 64, 16] bytes, KQ = (9R+1+2+15)/16) instead of f32 rows: the step of
 * the policy route of scripts/rollout.py:72 (network forward on the operand -> env.step -> next
 * operand).  The same transitions and operand bytes as wh_vector_step(obs = NULL) followed by
 * wh_observe_x (which is what it runs). */
int wh_vector_step_x(const wh_config* cfg, int64_t B, uint32_t* state, const int32_t* actions,
                     const int32_t* order, int32_t order_len, const uint8_t* mask, float* rewards, uint8_t* dones, void* xfrag,
                     const wh_episode_stats* stats, int32_t autoreset, int32_t variable_n,
                     uint64_t seed, int64_t env_offset, void* stream);

/* One step of the sampler route with the device policy (the greedy solver of baseline/solvers.py:27-58
 * standing in for the learner's policy, or uniform random actions): policy + step + auto-reset
 * (Train variants redraw n) in one step launch, then the observation rows (wh_observe); the same
 * philox draws and results as wh_policy followed by wh_vector_step(autoreset = 1), one launch
 * fewer.  rewards [B,NA] / dones [B] / obs [B,NA,9R+1] / stats may be NULL. */
int wh_sampler_step(const wh_config* cfg, int64_t B, uint32_t* state, int32_t policy, float p,
                    float* rewards, uint8_t* dones, float* obs, const wh_episode_stats* stats,
                    int32_t variable_n, uint64_t seed, int64_t env_offset, void* stream);

/* `steps` consecutive wh_sampler_step's in ONE launch (a rollout fragment of the sampler route):
 * rewards [steps,B,NA] / dones [steps,B] / obs [steps,B,NA,9R+1] (obs required), step k's outputs at
 * index k; the same draws, transitions and rows as `steps` calls of wh_sampler_step.  In the fused
 * launch the simulation of step k runs while step k-1's rows stream out, the state staying in
 * registers; configurations it does not cover run the steps one call at a time. */
int wh_sampler_rollout(const wh_config* cfg, int64_t B, uint32_t* state, int32_t steps, int32_t policy, float p,
                       float* rewards, uint8_t* dones, float* obs, const wh_episode_stats* stats, int32_t variable_n,
                       uint64_t seed, int64_t env_offset, void* stream);

/* wh_sampler_step's step launch with the state double-buffered and no observation rows: reads
 * state_in, writes the stepped state to state_out (a distinct [words, B] buffer, or state_in itself).
 * With two state buffers, wh_observe of step s (reading its output buffer) can run on another stream
 * while step s + 1 reads the same buffer and writes the other one (warehouse/vector.py
 * SamplerPipeline); the results are those of wh_sampler_step. */
int wh_sampler_step_to(const wh_config* cfg, int64_t B, const uint32_t* state_in, uint32_t* state_out,
                       int32_t policy, float p, float* rewards, uint8_t* dones, const wh_episode_stats* stats,
                       int32_t variable_n, uint64_t seed, int64_t env_offset, void* stream);

/* A prepared wh_rollout: the same arguments resolved once (config validated, kernel and tables
 * chosen) into an opaque handle, so a loop that launches the same rollout repeatedly pays one
 * cheap call per launch (wh_launch_run enqueues exactly what wh_rollout would).  The buffers must
 * stay valid while the handle is used; free it with wh_launch_free. */
typedef struct wh_launch wh_launch;
int wh_rollout_prepare(const wh_config* cfg, int64_t B, uint32_t* state, int32_t steps, int32_t policy,
                       float p, float* rewards, uint8_t* dones, float* returns, const wh_episode_stats* stats,
                       int32_t autoreset, int32_t variable_n, uint64_t seed, int64_t env_offset, void* stream,
                       wh_launch** out);
int wh_launch_run(const wh_launch* launch);
/* wh_launch_run with HIP events (hipEvent_t, created by the caller with timing enabled) attached to
 * the kernel dispatch itself (hipExtLaunchKernel): start/stop are stamped when the kernel starts and
 * ends, so their span is the kernel's duration and no separate marker packets sit in the stream.
 * Either event may be NULL (e.g. start on the first of several launches, stop on the last). */
int wh_launch_run_timed(const wh_launch* launch, void* start_event, void* stop_event);
/* Frees a handle of wh_rollout_prepare.  Handles are tracked: run / run_timed / free of a pointer that
 * is not a live handle (never prepared, or already freed) return WH_EINVAL and touch nothing, so a
 * double free is refused instead of corrupting the heap -- as long as no later wh_rollout_prepare
 * has been handed the same address: a freed handle whose address the allocator reuses is live again
 * (it names the new launch), so a stale pointer must not be used after a further prepare.  NULL is
 * a no-op (WH_OK).  A prepare with B = 0 needs no device and no tables: its handle launches nothing. */
int wh_launch_free(wh_launch* launch);

/* SAC policy network forward (the policy_model of scripts/experiments/warehouse-{small,medium,large}-sac: a
 * ReLU MLP, hidden_layer_sizes [256,256] Small / [512,512] Medium / [1024,256] Large, 9 action
 * logits), i.e. trainer.compute_action(obs) of scripts/rollout.py:72 for every agent row of a
 * batch.  precision WH_MLP_BF16: bf16 MFMA with f32 accumulation, activations rounded to bf16
 * between layers (fast); WH_MLP_F32: exact f32 (v_mfma_f32_32x32x2_f32, an fmaf chain per output:
 * logits equal a float32 reference up to summation order), like the reference's TF fp32 policy.
 * Supported: in_dim = 9R+1 of a variant with its hidden sizes, out_dim = 9 (else WH_ENOTSUP).
 * Blobs are precision-specific: pack and forward with the same desc. */
#define WH_MLP_BF16 0
#define WH_MLP_F32 1
typedef struct wh_mlp_desc {
  int32_t in_dim, hidden0, hidden1, out_dim;
  int32_t precision; /* WH_MLP_BF16 or WH_MLP_F32 */
} wh_mlp_desc;

/* Size of the packed weight blob (device bytes).  Host only. */
int wh_mlp_query(const wh_mlp_desc* d, int64_t* packed_bytes);

/* Pack host f32 weights in torch nn.Linear layout (w0 [hidden0, in_dim], b0 [hidden0],
 * w1 [hidden1, hidden0], b1 [hidden1], w2 [out_dim, hidden1], b2 [out_dim]) into the device blob
 * `packed` (wh_mlp_query bytes, 16-byte aligned).  Synchronous. */
int wh_mlp_pack(const wh_mlp_desc* d, const float* w0, const float* b0, const float* w1,
                const float* b1, const float* w2, const float* b2, void* packed);

/* obs [rows, in_dim] f32 -> logits [rows, 9] f32 and/or actions [rows] int32 (either may be NULL,
 * not both).  explore = 0: argmax, first maximum wins; explore = 1: Gumbel-max sample of
 * Categorical(logits), noise from philox (seed; counter row, step, purpose 5). */
int wh_mlp_forward(const wh_mlp_desc* d, const void* packed, int64_t rows, const float* obs,
                   float* logits, int32_t* actions, int32_t explore, uint64_t seed, uint32_t step,
                   void* stream);
/* wh_mlp_forward with the observation rows given as wh_observe_x's fragment-order operand (bf16
 * precision only; the same logits as wh_mlp_forward on the f32 rows, which it rounds to bf16
 * exactly so): one coalesced 16-byte load per k-step and lane instead of strided f32 rows. */
int wh_mlp_forward_x(const wh_mlp_desc* d, const void* packed, int64_t rows, const void* xfrag,
                     float* logits, int32_t* actions, int32_t explore, uint64_t seed, uint32_t step,
                     void* stream);

/* Library build identification (e.g. "warehouse_amd gfx950 <date>"). */
const char* wh_version(void);

/* Assert-mode builds (-DWH_CHECK) check SURVEY §5's invariants inside the kernels after every
 * state load, step and reset: exactly R open requests, live agents inside the grid, carried
 * targets on delivery cells, request bytes valid delivery indices, open mask == table, n <= slots.
 * out[4] = {violations, first failing env id, its failed-check bits, env-states checked}; clear
 * != 0 zeroes the counters.  Synchronises the current device.  WH_ENOTSUP in production builds. */
int wh_check_read(uint64_t* out, int32_t clear);

#ifdef __cplusplus
}
#endif
#endif /* WAREHOUSE_AMD_H */
