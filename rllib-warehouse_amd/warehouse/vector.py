"""RLlib-facing batched adapters over `BatchedWarehouse` (the route scripts/train.py's workload
takes, scripts/train.py:29-43): many warehouse episodes on one MI355X presented to a sampler.

* `WarehouseVectorEnv` -- the tensor fast path, shaped like ray.rllib.env.vector_env.VectorEnv
  (`num_envs`, `observation_space`, `action_space`, `vector_reset()`, `reset_at()`,
  `vector_step()`): actions [B,NA] in, flat observation rows [B,NA,9R+1] float32 / rewards [B,NA]
  / dones [B] out, one wh_vector_step call per step, done episodes restarted on the device.
* `WarehouseBaseEnv` -- the dict surface of ray.rllib.env.base_env.BaseEnv (`poll()`,
  `send_actions()`, `try_reset()`), with per-agent ids str(i) like warehouse/core.py:248-260,
  435-442, for samplers that speak MultiEnvDicts.  It does not auto-reset: like RLlib's
  MultiAgentEnvWrapper, an env whose "__all__" is done waits for try_reset(env_id).

Both report the on_episode_end metrics of scripts/train.py:18-23 from device counters
(`custom_metrics()`).

Observation rows are the gym Dict observation (warehouse/core.py:118-148) flattened the way a
Dict-flattening preprocessor does: keys in sorted order, each value flattened row-major, as
float32.  ray is not installed here, so that flat layout is "parity unpinned" against RLlib itself;
every value is pinned against the reference's per-agent dicts (tests/test_gpu_parity.py).
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import numpy as np
import torch

from ._compat import spaces
from ._geometry import GEOMETRY
from .batched import BatchedWarehouse
from .core import agent_index

# sorted gym.spaces.Dict key order and each key's flattened width, R = num_requests
OBS_KEYS = ("num_agents", "other_availabilities", "other_delivery_targets", "other_positions",
            "requests", "self_availability", "self_delivery_target", "self_position")


def obs_key_widths(R: int) -> Dict[str, int]:
    return {"num_agents": 1, "other_availabilities": R - 1, "other_delivery_targets": 2 * (R - 1),
            "other_positions": 2 * (R - 1), "requests": 4 * R, "self_availability": 1,
            "self_delivery_target": 2, "self_position": 2}


def flat_observation_space(R: int, D: int):
    """Box of one flattened observation row, bounds taken from core.py:118-148."""
    lo, hi = [], []
    bounds = {"num_agents": (1, R), "other_availabilities": (0, 1), "other_delivery_targets": (0, D),
              "other_positions": (0, D), "requests": (0, D), "self_availability": (0, 1),
              "self_delivery_target": (0, D), "self_position": (0, D)}
    for k, w in obs_key_widths(R).items():
        lo += [bounds[k][0]] * w
        hi += [bounds[k][1]] * w
    return spaces.Box(low=np.array(lo, np.float32), high=np.array(hi, np.float32), shape=(9 * R + 1,),
                      dtype=np.float32)


def unflatten_row(row: np.ndarray, R: int) -> Dict[str, np.ndarray]:
    """One flat row back to the reference's observation dict (core.py:248-260 / 421-432)."""
    row = np.asarray(row)
    out, o = {}, 0
    shapes = {"num_agents": (1,), "other_availabilities": (R - 1,), "other_delivery_targets": (R - 1, 2),
              "other_positions": (R - 1, 2), "requests": (R, 4), "self_availability": (1,),
              "self_delivery_target": (2,), "self_position": (2,)}
    for k, w in obs_key_widths(R).items():
        dt = np.int8 if k in ("other_availabilities", "self_availability") else np.int32
        out[k] = row[o:o + w].astype(dt).reshape(shapes[k])
        o += w
    return out


class WarehouseVectorEnv:
    """`num_envs` episodes of one variant as a vectorised sampler env (tensor API).  Train
    variants (default, like scripts/train.py:11-15) draw each episode's agent count n on the
    device; rows and rewards of slots >= n are zero and `agent_mask()` marks the live ones."""

    def __init__(self, variant: str = "medium", num_envs: int = 1024, num_agents: Optional[int] = None,
                 *, train: bool = True, seed: int = 0, env_offset: int = 0, device=None,
                 autoreset: bool = True):
        self.env = BatchedWarehouse(variant, num_envs, num_agents, train=train, seed=seed,
                                    env_offset=env_offset, device=device)
        geo = GEOMETRY[variant]
        self.variant = variant
        self.num_envs = self.env.B
        self.num_agents = self.env.agent_slots
        self.num_requests = geo["R"]
        self.autoreset = bool(autoreset)
        self.observation_space = flat_observation_space(geo["R"], geo["D"])
        self.action_space = spaces.Discrete(9)
        self.stats = self.env.enable_episode_stats()
        self._slot = torch.arange(self.num_agents, device=self.env.device, dtype=torch.int32)

    @property
    def device(self):
        return self.env.device

    def vector_reset(self) -> torch.Tensor:
        self.env.reset()
        return self.env.observe()

    def reset_at(self, index=None, mask=None) -> torch.Tensor:
        """Restart env `index` (or every env in the [B] bool `mask`); returns the full obs tensor,
        whose rows of the restarted envs are their first observations."""
        if mask is None:
            mask = torch.zeros(self.num_envs, dtype=torch.bool, device=self.device)
            mask[int(index)] = True
        self.env.reset(mask=mask)
        return self.env.observe()

    def vector_step(self, actions, mask=None, order=None) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, dict]:
        """actions [B,NA] int in 0..8 (values outside act as 4 = stay); `mask` [B] bool limits the
        step to some envs; `order` [B,OL] int (OL <= 4 NA, -1 padded) is each env's action-dict order --
        agents it leaves out are skipped as in the reference (core.py:279-300), None = every agent
        in ascending id order.  Returns env-owned (obs [B,NA,9R+1], rewards [B,NA], dones [B]
        bool, infos)."""
        obs, rew, done = self.env.vector_step(actions, autoreset=self.autoreset, mask=mask, order=order)
        return obs, rew, done.bool(), {}

    def agent_mask(self) -> torch.Tensor:
        """[B,NA] bool: slot i is a live agent of its env's current episode (i < n)."""
        n = (self.env.state[0] >> 16) & 0xFF
        return self._slot[None, :] < n[:, None]

    def custom_metrics(self) -> Dict[str, Dict[str, float]]:
        return self.stats.custom_metrics()


class WarehouseBaseEnv:
    """MultiEnvDict surface (ray.rllib.env.base_env.BaseEnv) over one batch on the device."""

    def __init__(self, variant: str = "medium", num_envs: int = 4, num_agents: Optional[int] = None,
                 *, train: bool = True, seed: int = 0, env_offset: int = 0, device=None):
        self.vec = WarehouseVectorEnv(variant, num_envs, num_agents, train=train, seed=seed,
                                      env_offset=env_offset, device=device, autoreset=False)
        self.num_envs = self.vec.num_envs
        self.observation_space = self.vec.observation_space
        self.action_space = self.vec.action_space
        self._n = np.zeros(self.num_envs, np.int64)   # agents of each env's episode (host copy)
        obs = self.vec.vector_reset()
        self._pending = self._pack(obs, None, None, range(self.num_envs))

    def _pack(self, obs, rew, done, env_ids):
        # Only the rows of `env_ids` leave the device, gathered there and brought back in ONE
        # download: [n | rewards | done | obs rows] as f32 per env (n <= 255 and done in {0, 1} are
        # exact in f32).  try_reset of one env therefore copies one env's rows, not the batch's.
        env_ids = list(env_ids)
        if not env_ids:
            return ({}, {}, {}, {}, {})
        B, NA, L = obs.shape
        sel = torch.as_tensor(env_ids, dtype=torch.long, device=obs.device)
        cols = [((self.vec.env.state[0, sel] >> 16) & 0xFF).float()[:, None]]
        if rew is not None:
            cols.append(rew[sel].float())
        if done is not None:
            cols.append(done[sel].float()[:, None])
        cols.append(obs[sel].reshape(len(env_ids), NA * L))
        h = torch.cat(cols, 1).cpu().numpy()
        n = h[:, 0].astype(np.int64)
        c = 1
        r = None if rew is None else h[:, c:c + NA]
        c += 0 if rew is None else NA
        d = None if done is None else h[:, c] != 0
        c += 0 if done is None else 1
        o = h[:, c:].reshape(len(env_ids), NA, L)
        agent_ids = [str(i) for i in range(NA)]
        rl = None if r is None else r.tolist()
        dl = [False] * len(env_ids) if d is None else d.tolist()
        self._n[env_ids] = n
        res = ({}, {}, {}, {}, {})
        for k, e in enumerate(env_ids):
            nk = int(n[k])
            ids = agent_ids[:nk]
            res[0][e] = dict(zip(ids, o[k, :nk]))
            res[1][e] = dict.fromkeys(ids, 0.0) if rl is None else dict(zip(ids, rl[k][:nk]))
            dd = dl[k]
            res[2][e] = dict.fromkeys(ids, dd)
            res[2][e]["__all__"] = dd
            res[3][e] = {a: {} for a in ids}
            res[4][e] = {}
        return res

    def poll(self):
        """(obs, rewards, dones, infos, off_policy_actions), each {env_id: {agent_id: value}},
        for every env with results not yet polled."""
        out, self._pending = self._pending, ({}, {}, {}, {}, {})
        return out

    def send_actions(self, action_dict: Dict[int, Dict[str, int]]) -> None:
        """Step the envs named in `action_dict` (other envs are untouched) with the reference's
        dict semantics (core.py:279-300): each env's agents are resolved in its dict's iteration
        order, and an agent missing from the dict is skipped -- it neither moves nor re-marks its
        cell (a "stay" would), so a later agent may enter a cell a co-located agent just left.
        Actions wrap like Python indexing; >= 9 raises IndexError (MOVES[action], core.py:281),
        and so does an agent id outside [-n, n) (agent_positions[idx], core.py:280); negative keys
        name agent n + key as numpy indexing does, and an agent named under two keys ('0' and 0)
        moves once per entry with that entry's action (each order entry carries its own action).
        Up to 4n entries per env dict (every agent under the four key forms '0', 0, '-n', -n); a
        longer dict (int() accepts more spellings, '00') raises ValueError where the reference runs it."""
        NA = self.vec.num_agents
        width = max([NA] + [len(ad) for ad in action_dict.values()])
        acts = np.full((self.num_envs, NA), 4, np.int32)
        order = np.full((self.num_envs, width), -1, np.int32)
        mask = np.zeros(self.num_envs, bool)
        ascending = True            # every dict lists all agents of its env in ascending order
        for e, ad in action_dict.items():
            mask[e] = True
            n = int(self._n[e])
            if len(ad) > 4 * n:
                raise ValueError(f"env {e}: {len(ad)} action-dict entries: at most 4 per agent ({4 * n}) are supported")
            for s, (a, v) in enumerate(ad.items()):
                idx, v = agent_index(a, n), int(v)
                if not -9 <= v < 9:
                    raise IndexError("list index out of range")   # MOVES[a], core.py:281
                acts[e, idx] = v % 9
                order[e, s] = idx | ((v % 9 + 1) << 8)
                ascending = ascending and idx == s
            ascending = ascending and len(ad) == n
        # the ascending kernel when every dict is full and in id order (the common sampler case),
        # else the dict-order kernel
        obs, rew, done, _ = self.vec.vector_step(acts, mask=mask, order=None if ascending else order)
        self._pending = self._pack(obs, rew, done, sorted(action_dict))

    def try_reset(self, env_id: int) -> Dict[str, np.ndarray]:
        obs = self.vec.reset_at(env_id)
        return self._pack(obs, None, None, [env_id])[0][env_id]

    def get_sub_environments(self):
        return []   # the envs live on the device as one batch, not as Python objects

    def custom_metrics(self) -> Dict[str, Dict[str, float]]:
        return self.vec.custom_metrics()


class SamplerPipeline:
    """The sampler route with the device policy (BatchedWarehouse.sampler_step) as a two-stream
    pipeline: the observation rows of step s are written on a side stream while step s + 1 runs on
    the current stream.  Both only READ the state step s produced, so the state is double-buffered
    (wh_sampler_step_to reads one buffer and writes the other) and so are the outputs: step s
    writes rewards[s % 2] / dones[s % 2], its rows land in obs[s % 2].  Step s + 2 writes the buffer
    observe(s) reads, so it waits for that observe (an event); nothing else is ordered, so the step
    kernel (one workgroup per CU) and the observation kernel (HBM-write bound) share the chip.
    Results equal sampler_step's: the same launches on the same states (tests/test_gpu_vector.py).

    step() returns (obs, rewards, dones) of that step; obs is complete once `ready(s)` has been
    waited on (or after synchronize()); use it before step s + 2 reuses its buffer.  env.state
    always names the newest state buffer.  Inside a CUDA-graph capture call begin() first and end()
    last (the side stream forks from and joins the capturing stream)."""

    def __init__(self, env: BatchedWarehouse, policy: str = "greedy", p: float = 0.0):
        from . import _native as nat
        from .batched import POLICIES

        self.env, self.policy, self.p = env, POLICIES[policy], float(p)
        self._nat = nat
        dev = env.device
        self.bufs = [env.state, torch.empty_like(env.state)]
        shape = (env.B, env.agent_slots, env.obs_len)
        self.obs = [torch.empty(shape, dtype=torch.float32, device=dev) for _ in range(2)]
        self.rewards = [torch.zeros((env.B, env.agent_slots), dtype=torch.float32, device=dev) for _ in range(2)]
        self.dones = [torch.zeros(env.B, dtype=torch.uint8, device=dev) for _ in range(2)]
        self.side = torch.cuda.Stream(device=dev)
        self.step_ev = [torch.cuda.Event(), torch.cuda.Event()]
        self.obs_ev = [torch.cuda.Event(), torch.cuda.Event()]
        self.pending = [False, False]   # obs_ev[k] recorded and not yet waited on by the main stream
        self.s = 0
        self.cur = 0                    # bufs[cur] holds the newest state

    def begin(self) -> None:
        """Fork the side stream from the current stream (start of a capture / after a sync)."""
        self.side.wait_stream(torch.cuda.current_stream(self.env.device))
        self.pending = [False, False]

    def end(self) -> None:
        """Join: the current stream waits for every observation launched so far."""
        torch.cuda.current_stream(self.env.device).wait_stream(self.side)
        self.pending = [False, False]

    def step(self):
        env, nat = self.env, self._nat
        i, o = self.cur, 1 - self.cur
        k = self.s % 2
        main = torch.cuda.current_stream(env.device)
        if self.pending[k]:              # observe(s - 2) read bufs[o]: let it finish first
            main.wait_event(self.obs_ev[k])
            self.pending[k] = False
        nat.check(nat.lib().wh_sampler_step_to(
            env._cfgp, env.B, self.bufs[i].data_ptr(), self.bufs[o].data_ptr(), self.policy, self.p,
            self.rewards[k].data_ptr(), self.dones[k].data_ptr(),
            None if env.stats is None else env.stats.ref, int(env.train), env.seed, env.env_offset,
            nat.stream_of(env.device)), "wh_sampler_step_to")
        self.step_ev[k].record(main)
        with torch.cuda.stream(self.side):
            self.side.wait_event(self.step_ev[k])
            nat.check(nat.lib().wh_observe(env._cfgp, env.B, self.bufs[o].data_ptr(), self.obs[k].data_ptr(),
                                           nat.stream_of(env.device)), "wh_observe")
            self.obs_ev[k].record(self.side)
        self.pending[k] = True
        self.cur = o
        env.state = self.bufs[o]
        self.s += 1
        return self.obs[k], self.rewards[k], self.dones[k]

    def ready(self, s: int) -> torch.cuda.Event:
        """Event after which step s's observation rows are written (valid until step s + 2)."""
        return self.obs_ev[s % 2]
