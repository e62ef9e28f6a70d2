"""Drop-in `Warehouse` (RLlib MultiAgentEnv) backed by the gfx950 kernels.

Same constructor, attributes and reset()/step() contract as the reference class
(warehouse/core.py:73-442), so baseline/run.py and scripts/train.py run unchanged.  One env is a
B=1 batch of `BatchedWarehouse`; every transition runs on the GPU -- or, on a host without a HIP
device, on the host engine (csrc/host_engine.cpp, the same C ABI on host cores: BASELINE config 1,
"baseline/run.py on CPU").  WAREHOUSE_DEVICE names the device explicitly ("cuda", "cuda:1", "cpu").

RNG parity.  The reference draws from numpy's GLOBAL stream (core.py:196-197, 215-220, 339-350),
interleaved with whatever else the process draws (e.g. the greedy solver's per-agent coin,
solvers.py:44).  To keep seeded trajectories identical, this class takes exactly those draws from
np.random on the host, in the same order, and injects them into the kernels:
  reset(): spawn rejection loop + choice(P, R) + choice(Dp, R)        -> wh_reset (injected)
  step():  wh_step(WH_PHASE_PRE_REGEN) reports |inactive|, then
           choice(|inactive|, k) + choice(Dp, k) on the host          -> wh_step(WH_PHASE_REGEN)
For thousands of envs use `warehouse.batched.BatchedWarehouse` (device philox draws) instead.
"""
from __future__ import annotations

import os
import time
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from . import _native as nat
from ._compat import MultiAgentEnv, spaces
from ._geometry import pickup_cells
from .batched import BatchedWarehouse

__all__ = ["Warehouse"]

ANIMATE_FRAMES_PER_STEP: int = 10     # core.py:69-70
ANIMATE_STEPS_PER_SECOND: float = 6.0

OBS_KEYS = ("num_agents", "other_availabilities", "other_delivery_targets", "other_positions",
            "requests", "self_availability", "self_delivery_target", "self_position")


def _default_device():
    return os.environ.get("WAREHOUSE_DEVICE") or ("cuda" if torch.cuda.is_available() else "cpu")


def agent_index(key, n: int) -> int:
    """The agent a dict key names, as core.py:280-281 indexes with it: int(key), negative values
    wrapping like numpy (-n..-1 -> 0..n-1); IndexError outside [-n, n)."""
    idx = int(key)
    if not -n <= idx < n:
        raise IndexError("index %d is out of bounds for axis 0 with size %d" % (idx, n))
    return idx + n if idx < 0 else idx


class Warehouse(MultiAgentEnv):
    metadata = {"render.modes": ["human", "ansi", "rgb_array"]}

    def __init__(self, num_agents: int, num_requests: int, area_dimension: int,
                 pickup_racks_arrangement: List[int], episode_duration: int,
                 pickup_wait_duration: int) -> None:
        super(Warehouse, self).__init__()
        assert num_agents <= num_requests

        self._area_dimension = int(area_dimension)
        self._pickup_racks_arrangement = list(pickup_racks_arrangement)
        self._num_agents = int(num_agents)
        self._num_requests = int(num_requests)
        self._num_pickup_points = 4 * len(self._pickup_racks_arrangement) ** 2
        self._num_delivery_points = 4 * int(self._area_dimension - 4)
        self._episode_duration = int(episode_duration)
        self._pickup_wait_duration = int(pickup_wait_duration)
        self._null_position = self._area_dimension // 2

        self.num_agents = self._num_agents
        self.num_requests = self._num_requests
        self.animate_frames_per_step = ANIMATE_FRAMES_PER_STEP
        self.animate_steps_per_second = ANIMATE_STEPS_PER_SECOND

        R, D = self._num_requests, self._area_dimension
        self.reward_range = (0.0, 1.0)
        self.action_space = spaces.Discrete(9)
        self.observation_space = spaces.Dict({
            "num_agents": spaces.Box(low=1, high=R, shape=(1,), dtype=np.int32),
            "self_position": spaces.Box(low=0, high=D, shape=(2,), dtype=np.int32),
            "self_availability": spaces.MultiBinary(1),
            "self_delivery_target": spaces.Box(low=0, high=D, shape=(2,), dtype=np.int32),
            "other_positions": spaces.Box(low=0, high=D, shape=(R - 1, 2), dtype=np.int32),
            "other_availabilities": spaces.MultiBinary(R - 1),
            "other_delivery_targets": spaces.Box(low=0, high=D, shape=(R - 1, 2), dtype=np.int32),
            "requests": spaces.Box(low=0, high=D, shape=(R, 4), dtype=np.int32),
        })

        self._pickup_set = set(pickup_cells(D, self._pickup_racks_arrangement))
        w = {k: n for k, n in zip(OBS_KEYS, (1, R - 1, 2 * (R - 1), 2 * (R - 1), 4 * R, 1, 2, 2))}
        ends = np.cumsum([w[k] for k in OBS_KEYS])
        self._obs_slices = [slice(int(a), int(b)) for a, b in zip(np.r_[0, ends[:-1]], ends)]
        self._done = False
        self._prev = None          # host snapshot before the last step (core.py:270-272), kept
        self._rendering = False    # only once render() has been called: it costs a device copy
        # The device engine and its buffers, per configuration.  The Train variants re-run
        # __init__ at every reset with a new agent count (variants.py:69-71); the engine, its
        # result block and the pinned upload buffers of an agent count are built once per env object
        # and reused by every later episode with that count (pinning host memory is slow).
        geo = dict(D=D, R=R, racks=tuple(self._pickup_racks_arrangement), T=self._episode_duration,
                   W=self._pickup_wait_duration, max_agents=self._num_agents)
        cache = self.__dict__.setdefault("_engine_cache", {})
        key = (self._num_agents, D, R, geo["racks"], geo["T"], geo["W"])
        if key not in cache:
            cache[key] = self._build_engine(geo)
        self._engine, self._blob, self._r_off, self._d_off, io = cache[key]
        self._io = io              # per-step upload buffers (pinned), created at the first step

    def _build_engine(self, geo):
        eng = BatchedWarehouse(num_envs=1, num_agents=self._num_agents, geometry=geo, device=_default_device())
        # The engine's observation, reward and done buffers as views of ONE device block, so a step's
        # results come back in a single download with no gather kernel (offsets 256-aligned: the
        # kernels store rows with 16-byte writes).
        o_bytes = 4 * self._num_agents * eng.obs_len
        r_off = -(-o_bytes // 256) * 256
        d_off = r_off + 256 * (-(-4 * self._num_agents // 256))
        blob = torch.zeros(d_off + 256, dtype=torch.uint8, device=eng.device)
        eng._obs = blob[:o_bytes].view(torch.float32).view(1, self._num_agents, eng.obs_len)
        eng.rewards = blob[r_off:r_off + 4 * self._num_agents].view(torch.float32).view(1, self._num_agents)
        eng.dones = blob[d_off:d_off + 1]
        return [eng, blob, r_off, d_off, None]

    # ------------------------------------------------------------------ helpers
    def _io_buffers(self):
        """Host and device buffers for the per-step uploads (allocated on first step; pinned for a
        HIP device): io = [actions (n) | dict-order entries (4n)], regen [1, 2R]."""
        if self._io is None:
            n, R, dev = self._num_agents, self._num_requests, self._engine.device
            pin = (lambda t: t) if dev.type == "cpu" else (lambda t: t.pin_memory())
            h_io = pin(torch.empty((1, 5 * n), dtype=torch.int32))
            h_regen = pin(torch.empty((1, 2 * R), dtype=torch.int32))
            self._io = (h_io, torch.empty_like(h_io, device=dev), h_regen, torch.empty_like(h_regen, device=dev))
            for entry in self._engine_cache.values():   # kept with the engine for later episodes
                if entry[0] is self._engine:
                    entry[4] = self._io
        return self._io

    def _obs_dicts(self, rows: Optional[np.ndarray] = None) -> Dict[str, Dict[str, np.ndarray]]:
        if rows is None:
            rows = self._engine.observe()[0].cpu().numpy().astype(np.int32)
        R = self._num_requests
        out = {}
        for i in range(self._num_agents):
            row = rows[i]
            p = [row[sl] for sl in self._obs_slices]
            out[str(i)] = {
                "num_agents": p[0],
                "self_position": p[7],
                "self_availability": p[5].astype(np.int8),
                "self_delivery_target": p[6],
                "other_positions": p[3].reshape(R - 1, 2),
                "other_availabilities": p[1].astype(np.int8),
                "other_delivery_targets": p[2].reshape(R - 1, 2),
                "requests": p[4].reshape(R, 4),
            }
        return out

    # ------------------------------------------------------------------ MultiAgentEnv
    def reset(self) -> Dict[str, Dict[str, np.ndarray]]:
        D, R, n = self._area_dimension, self._num_requests, self._num_agents
        spawn = []
        for _ in range(n):                                  # core.py:191-201, same draw order
            while True:
                cell = (np.random.randint(1, D - 1), np.random.randint(1, D - 1))
                if cell not in self._pickup_set:
                    spawn.append(cell)
                    break
        sel = np.random.choice(self._num_pickup_points, R, replace=False)      # core.py:215-217
        tgt = np.random.choice(self._num_delivery_points, R, replace=False)    # core.py:218-220
        self._engine.reset(draws=dict(spawn=np.array(spawn, np.int32).reshape(1, n, 2),
                                      pickups=sel.reshape(1, R), targets=tgt.reshape(1, R)))
        return self._obs_dicts()

    def step(self, action_dict: Dict[str, int]
             ) -> Tuple[Dict[str, dict], Dict[str, float], Dict[str, bool], Dict[str, dict]]:
        """core.py:262-442 for one env.  Each dict entry moves its agent in iteration order; an agent
        named under several key forms ('0', 0, '-n', -n: int(key) indexes like numpy, core.py:280)
        moves once per entry, with that entry's action.  Up to 4n entries -- every agent under all
        four of those forms; int() accepts yet more spellings of a number ('00', ' 0'), and a dict
        with more than 4n entries raises ValueError where the reference would run it."""
        n, R = self._num_agents, self._num_requests
        h_io, d_io, h_regen, d_regen = self._io_buffers()
        io = h_io.numpy()[0]                                 # [actions (n) | dict order (4n)]
        io[:n] = 4
        io[n:] = -1
        if len(action_dict) > 4 * n:
            raise ValueError(f"{len(action_dict)} action-dict entries: at most 4 per agent ({4 * n}) are supported")
        for s, (key, action) in enumerate(action_dict.items()):
            idx = agent_index(key, n)
            a = int(action)
            if not -9 <= a <= 8:                            # MOVES[action] (core.py:282)
                raise IndexError("list index out of range")
            io[n + s] = idx | ((a % 9 + 1) << 8)            # the entry's own action (a repeated agent)
            io[idx] = a % 9                                  # Python's negative-index wrap
        ol = max(n, len(action_dict))
        eng = self._engine
        if self._rendering:
            self._prev = self._snapshot()                    # core.py:270-272
        # One step costs two host round trips: the reference draws the regeneration on the host
        # from the post-pickup count of free points (core.py:339-350), so n_inactive must come
        # back; then observations, rewards and dones come back in one copy.  Uploads are async
        # from pinned buffers on the launch stream (each is rewritten only after a later sync).
        d_io.copy_(h_io, non_blocking=True)
        eng.step(d_io[:, :n], order=d_io[:, n:n + ol], phase=nat.WH_PHASE_PRE_REGEN)
        n_in = int(eng.n_inactive[0].item())
        k = R - self._num_pickup_points + n_in
        rpos = np.random.choice(n_in, k, replace=False)                       # core.py:339-343
        rtgt = np.random.choice(self._num_delivery_points, k, replace=False)  # core.py:346-350
        regen = h_regen.numpy()
        regen[:] = -1
        regen[0, :k] = rpos
        regen[0, R:R + k] = rtgt
        d_regen.copy_(h_regen, non_blocking=True)
        eng.step(None, regen=d_regen, phase=nat.WH_PHASE_REGEN)
        eng.observe()
        h = self._blob.cpu().numpy()
        L = eng.obs_len
        obs = self._obs_dicts(h[:4 * n * L].view(np.float32).reshape(n, L).astype(np.int32))
        rew = h[self._r_off:self._r_off + 4 * n].view(np.float32)
        done = bool(h[self._d_off])
        rewards = {str(i): rew[i] for i in range(n)}
        dones = {str(i): done for i in range(n)}
        dones["__all__"] = done
        return obs, rewards, dones, {str(i): {} for i in range(n)}

    # ------------------------------------------------------------------ rendering
    def _snapshot(self) -> Dict[str, np.ndarray]:
        c = self._engine.to_canonical()
        return dict(pos=c["pos"][0].cpu().numpy(), agent_target=c["agent_target"][0].cpu().numpy(),
                    pickup_target=c["pickup_target"][0].cpu().numpy())

    def _frame_text(self, snap: Dict[str, np.ndarray]) -> str:
        """One frame as text, row y = D-1 at the top (the reference's viewer has y up):
        '.' floor, '#' pickup point, 'P' pickup point with an open request, 'D' delivery point,
        agents 'a', 'b', ... when idle and 'A', 'B', ... when carrying, '*' for a shared cell."""
        D = self._area_dimension
        grid = [["." for _ in range(D)] for _ in range(D)]
        pk = pickup_cells(D, self._pickup_racks_arrangement)
        for j, (x, y) in enumerate(pk):
            grid[y][x] = "P" if snap["pickup_target"][j] >= 0 else "#"
        for v in range(2, D - 2):                             # core.py:177-188
            for x, y in ((v, 0), (0, v), (v, D - 1), (D - 1, v)):
                grid[y][x] = "D"
        for i, (x, y) in enumerate(snap["pos"]):
            ch = chr((ord("A") if snap["agent_target"][i] >= 0 else ord("a")) + i % 26)
            grid[y][x] = "*" if grid[y][x] not in ".#PD" else ch
        return "\n".join("".join(row) for row in reversed(grid))

    def _frame_rgb(self, pos: np.ndarray, snap: Dict[str, np.ndarray], px: int = 12) -> np.ndarray:
        D = self._area_dimension
        img = np.full((D * px, D * px, 3), 235, np.uint8)
        def fill(x, y, c, m=0):
            img[(D - 1 - y) * px + m:(D - y) * px - m, x * px + m:(x + 1) * px - m] = c
        for j, (x, y) in enumerate(pickup_cells(D, self._pickup_racks_arrangement)):
            fill(x, y, (230, 160, 40) if snap["pickup_target"][j] >= 0 else (170, 170, 170))
        for v in range(2, D - 2):
            for x, y in ((v, 0), (0, v), (v, D - 1), (D - 1, v)):
                fill(x, y, (90, 160, 230))
        for i, (x, y) in enumerate(np.rint(pos).astype(int)):
            fill(int(x), int(y), (200, 40, 40) if snap["agent_target"][i] >= 0 else (40, 150, 60), m=2)
        return img

    def render(self, mode: str = "human", animate: bool = False):
        """Headless rendering of the device state (the reference draws the same scene with a gym
        pyglet Viewer, core.py:444-617).  mode "human" prints the frame, "ansi" returns it as
        text, "rgb_array" returns an RGB image -- with animate=True a list of
        animate_frames_per_step images moving the agents from their previous cells
        (core.py:449-469); "human" then keeps the reference's pacing of
        animate_steps_per_second."""
        if mode not in self.metadata["render.modes"]:
            raise NotImplementedError(f"render mode {mode!r}")
        self._rendering = True
        snap = self._snapshot()
        prev = self._prev if self._prev is not None else snap
        if mode == "rgb_array":
            if not animate:
                return self._frame_rgb(snap["pos"], snap)
            f = self.animate_frames_per_step
            return [self._frame_rgb(prev["pos"] + (snap["pos"] - prev["pos"]) / f * i, prev) for i in range(f)]
        text = self._frame_text(snap)
        if mode == "ansi":
            return text
        print(text, flush=True)
        if animate:
            time.sleep(1.0 / self.animate_steps_per_second)
        return None
