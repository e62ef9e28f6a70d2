"""B independent warehouse episodes resident on one MI355X (or, without a GPU, on host cores).

`BatchedWarehouse` owns the packed struct-of-arrays state (include/warehouse_amd.h, "PACKED
STATE") as one int32 tensor `state[words, B]` and drives an engine through the C ABI: the HIP
kernels (libwarehouse_amd.so) for a batch on a HIP device, the host engine (libwarehouse_host.so,
csrc/host_engine.cpp) for a batch on "cpu" -- the device the caller names, or the host when no HIP
device is visible (BASELINE config 1).  Same entry points, state layout and draws either way:

    reset()    -> wh_reset    Warehouse.reset()              warehouse/core.py:167-260
    step()     -> wh_step     Warehouse.step()               warehouse/core.py:262-442
    observe()  -> wh_observe  per-agent observation rows     warehouse/core.py:224-260, 371-432
    policy()   -> wh_policy   greedy / random actions        baseline/solvers.py:27-58
    rollout()  -> wh_rollout  device-resident rollout loop   baseline/run.py:42-62
    vector_step() -> wh_vector_step  sampler step: step + auto-reset + observation rows
    EpisodeStats     on_episode_end metrics kept on the device  scripts/train.py:18-23

Global env ids are `env_offset + e`; with philox draws a shard of env ids reproduces exactly the
trajectories those ids have in any other sharding (multi-GPU is a straight per-device shard).
"""
from __future__ import annotations

import ctypes
import weakref
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from . import _native as nat
from ._geometry import GEOMETRY

POLICIES = {"greedy": nat.WH_POLICY_GREEDY, "random": nat.WH_POLICY_RANDOM}


def resolve_device(device=None) -> torch.device:
    """The device a batch lives on: a HIP device (the gfx950 kernels) or the host ("cpu": the host
    engine).  None = the current HIP device, or the host when no HIP device is visible.  Naming a
    HIP device on a host without one raises -- nothing silently moves to the host engine."""
    if device is None:
        device = "cuda" if torch.cuda.is_available() else "cpu"
    dev = torch.device(device)
    if dev.type == "cpu":
        return dev
    return require_device(dev)


def require_device(device=None) -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("warehouse: no HIP device visible -- the gfx950 kernels need an MI355X; there "
                           "is no CPU fallback (device='cpu' selects the host engine explicitly)")
    dev = torch.device(device if device is not None else "cuda")
    if dev.type != "cuda":
        raise RuntimeError(f"warehouse: device {dev} is not a HIP device")
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    return dev


def _check_out(t, shape, dtype, device):
    """A caller-supplied output tensor the kernel writes: exact shape, dtype and device, contiguous --
    a tensor of the right shape but a narrower dtype, or on another GPU, would be written past its
    end or into the wrong device's memory."""
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f"expected shape {tuple(shape)}, got {tuple(t.shape)}")
    if t.dtype != dtype:
        raise ValueError(f"expected dtype {dtype}, got {t.dtype}")
    if t.device != device:
        raise ValueError(f"expected a tensor on {device}, got {t.device}")
    if not t.is_contiguous():
        raise ValueError("warehouse kernels take contiguous tensors")
    return t


def _dev_mask(mask, device, B):
    """An env mask [B] as the uint8 device operand the kernels read (mask[e] for every e < B): any
    bool/int array or tensor of exactly B entries; another length would be read past its end."""
    if mask is None:
        return None
    m = torch.as_tensor(np.asarray(mask) if not torch.is_tensor(mask) else mask)
    if tuple(m.shape) != (B,):
        raise ValueError(f"mask: expected shape ({B},), got {tuple(m.shape)}")
    return m.to(device=device, dtype=torch.uint8).contiguous()


def _dev_i32(x, device, shape=None):
    if x is None:
        return None
    if torch.is_tensor(x) and x.dtype == torch.int32 and x.device == device and x.is_contiguous() \
            and (shape is None or tuple(x.shape) == tuple(shape)):
        return x                         # already a device operand: no conversion ops per launch
    t = torch.as_tensor(np.asarray(x) if not torch.is_tensor(x) else x)
    t = t.to(device=device, dtype=torch.int32).contiguous()
    if shape is not None:
        t = t.reshape(shape)
    return t


class EpisodeStats:
    """Device-side episode metrics of scripts/train.py:18-23 (`on_episode_end`): for every
    finished episode avg_agent_reward = (episode return summed over agents) / n, reported over all
    episodes ("avg_agent_reward_all") and per agent count n ("avg_agent_reward_{n}").  The kernels
    bin integer returns by n (wh_episode_stats), so every figure here is exact."""

    def __init__(self, num_envs: int, agent_slots: int, device):
        z = dict(device=device)
        self.agent_slots = int(agent_slots)
        self.episode_return = torch.zeros(num_envs, dtype=torch.int32, **z)
        self.return_sum = torch.zeros(agent_slots + 1, dtype=torch.int64, **z)
        self.episodes = torch.zeros(agent_slots + 1, dtype=torch.int64, **z)
        self.return_min = torch.full((agent_slots + 1,), -1, dtype=torch.int32, **z)   # 0xFFFFFFFF
        self.return_max = torch.zeros(agent_slots + 1, dtype=torch.int32, **z)
        self._c = nat.WhEpisodeStats(self.episode_return.data_ptr(), self.return_sum.data_ptr(),
                                     self.episodes.data_ptr(), self.return_min.data_ptr(),
                                     self.return_max.data_ptr())

    @property
    def ref(self):
        return ctypes.byref(self._c)

    def clear(self) -> None:
        """Forget finished episodes (running episode returns are kept)."""
        self.return_sum.zero_()
        self.episodes.zero_()
        self.return_min.fill_(-1)
        self.return_max.zero_()

    def bins(self) -> Dict[str, np.ndarray]:
        return dict(return_sum=self.return_sum.cpu().numpy(), episodes=self.episodes.cpu().numpy(),
                    return_min=self.return_min.cpu().numpy().view(np.uint32),
                    return_max=self.return_max.cpu().numpy().view(np.uint32))

    def custom_metrics(self) -> Dict[str, Dict[str, float]]:
        return custom_metrics_from_bins(**self.bins())


def custom_metrics_from_bins(return_sum, episodes, return_min, return_max) -> Dict[str, Dict[str, float]]:
    """RLlib's custom_metrics summary (mean / min / max / count over episodes) of the
    avg_agent_reward values on_episode_end records (scripts/train.py:18-23), from n-binned totals."""
    out: Dict[str, Dict[str, float]] = {}
    tot_avg, tot_cnt, lo, hi = 0.0, 0, np.inf, -np.inf
    for n in range(1, len(episodes)):
        c = int(episodes[n])
        if c == 0:
            continue
        mean = int(return_sum[n]) / (n * c)
        mn, mx = int(return_min[n]) / n, int(return_max[n]) / n
        out[f"avg_agent_reward_{n}"] = dict(mean=mean, min=mn, max=mx, count=c)
        tot_avg += int(return_sum[n]) / n
        tot_cnt += c
        lo, hi = min(lo, mn), max(hi, mx)
    if tot_cnt:
        out["avg_agent_reward_all"] = dict(mean=tot_avg / tot_cnt, min=lo, max=hi, count=tot_cnt)
    return out


class BatchedWarehouse:
    """`num_envs` episodes of one variant.  `train=True` gives the Train variants' per-episode
    agent count n ~ U{1..max_num_agents} (warehouse/variants.py:65-98) with max_num_agents slots."""

    def __init__(self, variant: str = "medium", num_envs: int = 1, num_agents: Optional[int] = None,
                 *, train: bool = False, seed: int = 0, env_offset: int = 0, device=None,
                 geometry: Optional[dict] = None):
        geo = dict(GEOMETRY[variant] if geometry is None else geometry)
        self.geometry = geo
        self.variant = variant if geometry is None else None
        self.train = bool(train)
        nmax = int(geo["max_agents"])
        slots = nmax if train or num_agents is None else int(num_agents)
        if not 1 <= slots <= geo["R"]:
            raise AssertionError("num_agents <= num_requests (core.py:89)")
        self.agent_slots = slots
        self.cfg = nat.make_config(geo["D"], geo["R"], geo["racks"], slots, geo["T"], geo["W"])
        self.device = resolve_device(device)
        self.host = self.device.type == "cpu"          # the host engine (no HIP device)
        self._lib = nat.host_lib() if self.host else nat.lib()
        self.layout = nat.query(self.cfg, self._lib)
        self.B = int(num_envs)
        self.seed = int(seed)
        self.env_offset = int(env_offset)
        self.R, self.P, self.Dp = geo["R"], self.layout.num_pickups, self.layout.num_deliveries
        self.obs_len = self.layout.obs_len
        self.state = torch.zeros((self.layout.words_per_env, self.B), dtype=torch.int32, device=self.device)
        self.rewards = torch.zeros((self.B, slots), dtype=torch.float32, device=self.device)
        self.dones = torch.zeros(self.B, dtype=torch.uint8, device=self.device)
        self.actions = torch.full((self.B, slots), 4, dtype=torch.int32, device=self.device)
        self.n_inactive = torch.zeros(self.B, dtype=torch.int32, device=self.device)
        self._obs = None
        self._cfgp = ctypes.byref(self.cfg)
        self.stats: Optional[EpisodeStats] = None

    def enable_episode_stats(self) -> EpisodeStats:
        """Track on_episode_end metrics in rollout() / vector_step() from now on."""
        if self.stats is None:
            self.stats = EpisodeStats(self.B, self.agent_slots, self.device)
        return self.stats

    # ------------------------------------------------------------------ plumbing
    @property
    def stream(self) -> int:
        return nat.stream_of(self.device)

    def _call(self, name, *args):
        nat.check(getattr(self._lib, name)(self._cfgp, self.B, *args), name)

    def _ptr(self, t):
        return nat.ptr(t, self.host)

    def _order(self, order):
        """An action-dict order operand [B, OL] (OL = 1 .. 4 * agent_slots, -1 padded; see
        include/warehouse_amd.h wh_step) and its row length, or (None, 0)."""
        if order is None:
            return None, 0
        o = _dev_i32(order, self.device)
        if o.dim() == 1 and self.B == 1:
            o = o.reshape(1, -1)
        if o.dim() != 2 or o.shape[0] != self.B or not 1 <= o.shape[1] <= 4 * self.agent_slots:
            raise ValueError(f"order: expected shape ({self.B}, 1..{4 * self.agent_slots}), got {tuple(o.shape)}")
        return o, int(o.shape[1])

    # ------------------------------------------------------------------ API
    def reset(self, mask=None, draws: Optional[Dict[str, object]] = None) -> None:
        """Reset the envs selected by `mask` ([B] bool; None = all).  `draws` injects the
        reference's reset draws: spawn [B,NA,2], pickups [B,R], targets [B,R], n [B] (optional)."""
        m = _dev_mask(mask, self.device, self.B)
        keep = []
        dp = None
        if draws is not None:
            sp = _dev_i32(draws["spawn"], self.device, (self.B, self.agent_slots, 2))
            pk = _dev_i32(draws["pickups"], self.device, (self.B, self.R))
            tg = _dev_i32(draws["targets"], self.device, (self.B, self.R))
            nn = _dev_i32(draws.get("n"), self.device, (self.B,))
            keep = [sp, pk, tg, nn]
            dp = ctypes.byref(nat.WhResetDraws(sp.data_ptr(), pk.data_ptr(), tg.data_ptr(),
                                               None if nn is None else nn.data_ptr()))
        self._call("wh_reset", self.state.data_ptr(), self._ptr(m), dp, int(self.train),
                   self.seed, self.env_offset, self.stream)
        if self.stats is not None:   # a reset starts a new episode return
            if m is None:
                self.stats.episode_return.zero_()
            else:
                self.stats.episode_return.masked_fill_(m.bool(), 0)
        del keep

    def step(self, actions, order=None, regen=None, phase: int = nat.WH_PHASE_ALL
             ) -> Tuple[torch.Tensor, torch.Tensor]:
        """One transition for every env.  actions [B,NA] in 0..8; order [B,OL] (OL up to 4 NA, -1
        padded) is the action-dict iteration order; regen [B,2R] injects the regeneration draws.
        Returns the env-owned (rewards [B,NA] float32, dones [B] uint8) buffers, overwritten next call."""
        a = None if actions is None else _dev_i32(actions, self.device, (self.B, self.agent_slots))
        o, ol = self._order(order)
        r = _dev_i32(regen, self.device, (self.B, 2 * self.R))
        self._call("wh_step", self.state.data_ptr(), self._ptr(a), self._ptr(o), ol, self.rewards.data_ptr(),
                   self.dones.data_ptr(), self._ptr(r), self.n_inactive.data_ptr(), int(phase),
                   self.seed, self.env_offset, self.stream)
        return self.rewards, self.dones

    def observe(self) -> torch.Tensor:
        """[B, NA, 9R+1] float32 rows in sorted-key order (env-owned buffer)."""
        if self._obs is None:
            self._obs = torch.empty((self.B, self.agent_slots, self.obs_len), dtype=torch.float32,
                                    device=self.device)
        self._call("wh_observe", self.state.data_ptr(), self._obs.data_ptr(), self.stream)
        return self._obs

    def _xfrag_buffer(self) -> torch.Tensor:
        kq = (self.obs_len + 2 + 15) // 16
        tiles = (self.B * self.agent_slots + 31) // 32
        if getattr(self, "_xfrag", None) is None or self._xfrag.shape[0] != tiles:
            self._xfrag = torch.empty((tiles, kq, 64, 16), dtype=torch.uint8, device=self.device)
        return self._xfrag

    def observe_x(self, obs: bool = False):
        """The observation rows as the policy network's layer-0 operand (wh_observe_x: bf16, MFMA
        fragment order, for MLPPolicy.forward_x), optionally also the f32 rows.  Returns the
        env-owned uint8 buffer [tiles, KQ, 64, 16] (and the obs tensor when obs=True)."""
        self._xfrag_buffer()
        if obs and self._obs is None:
            self._obs = torch.empty((self.B, self.agent_slots, self.obs_len), dtype=torch.float32,
                                    device=self.device)
        self._call("wh_observe_x", self.state.data_ptr(), self._obs.data_ptr() if obs else None,
                   self._xfrag.data_ptr(), self.stream)
        return (self._xfrag, self._obs) if obs else self._xfrag

    def vector_step(self, actions, autoreset: bool = True, observe: bool = True, mask=None, order=None
                    ) -> Tuple[Optional[torch.Tensor], torch.Tensor, torch.Tensor]:
        """Sampler step (wh_vector_step): step every env (or those in the [B] bool `mask`) with
        `actions` [B,NA] (philox draws), restart the envs whose episode ended (autoreset; Train
        variants redraw n), then write the observation rows.  `order` [B,NA] (-1 terminated) is
        each env's action-dict iteration order; agents it does not list are skipped like agents
        absent from the reference's action dict (core.py:279-300); None = all, ascending.
        Returns env-owned (obs [B,NA,9R+1] or None, rewards [B,NA], dones [B]); with autoreset the
        obs rows of a done env already belong to its next episode.  Rewards/dones of envs outside
        `mask` are stale."""
        a = _dev_i32(actions, self.device, (self.B, self.agent_slots))
        o, ol = self._order(order)
        m = _dev_mask(mask, self.device, self.B)
        if observe and self._obs is None:
            self._obs = torch.empty((self.B, self.agent_slots, self.obs_len), dtype=torch.float32,
                                    device=self.device)
        obs = self._obs if observe else None
        self._call("wh_vector_step", self.state.data_ptr(), a.data_ptr(), self._ptr(o), ol, self._ptr(m),
                   self.rewards.data_ptr(), self.dones.data_ptr(), self._ptr(obs),
                   None if self.stats is None else self.stats.ref,
                   int(bool(autoreset)), int(self.train), self.seed, self.env_offset, self.stream)
        return obs, self.rewards, self.dones

    def vector_step_x(self, actions, autoreset: bool = True, mask=None, order=None):
        """vector_step with the rows written as the policy network's fragment-order operand
        (wh_vector_step_x: the step, then observe_x()'s buffer).  Returns env-owned
        (fragments [tiles, KQ, 64, 16] uint8, rewards [B,NA], dones [B])."""
        a = _dev_i32(actions, self.device, (self.B, self.agent_slots))
        o, ol = self._order(order)
        m = _dev_mask(mask, self.device, self.B)
        xf = self._xfrag_buffer()
        self._call("wh_vector_step_x", self.state.data_ptr(), a.data_ptr(), self._ptr(o), ol, self._ptr(m),
                   self.rewards.data_ptr(), self.dones.data_ptr(), xf.data_ptr(),
                   None if self.stats is None else self.stats.ref, int(bool(autoreset)), int(self.train),
                   self.seed, self.env_offset, self.stream)
        return xf, self.rewards, self.dones

    def sampler_step(self, policy: str = "greedy", p: float = 0.0, observe: bool = True
                     ) -> Tuple[Optional[torch.Tensor], torch.Tensor, torch.Tensor]:
        """vector_step(self.policy(policy, p), autoreset=True) with the device policy fused into
        the step launch (wh_sampler_step: policy + step + auto-reset, then the observation rows),
        with the same transitions and rows and one launch fewer.
        Returns env-owned (obs [B,NA,9R+1] or None, rewards [B,NA], dones [B])."""
        if observe and self._obs is None:
            self._obs = torch.empty((self.B, self.agent_slots, self.obs_len), dtype=torch.float32,
                                    device=self.device)
        obs = self._obs if observe else None
        self._call("wh_sampler_step", self.state.data_ptr(), POLICIES[policy], float(p),
                   self.rewards.data_ptr(), self.dones.data_ptr(), self._ptr(obs),
                   None if self.stats is None else self.stats.ref, int(self.train), self.seed,
                   self.env_offset, self.stream)
        return obs, self.rewards, self.dones

    def sampler_rollout(self, steps: int, policy: str = "greedy", p: float = 0.0, obs=None, rewards=None,
                        dones=None):
        """`steps` sampler_step's in one launch (wh_sampler_rollout: a rollout fragment): obs
        [steps,B,NA,9R+1] f32, rewards [steps,B,NA] f32, dones [steps,B] uint8, step k at index k
        (allocated when None).  Returns (obs, rewards, dones)."""
        NA, L = self.agent_slots, self.obs_len
        shapes = ((steps, self.B, NA, L), (steps, self.B, NA), (steps, self.B))
        dt = (torch.float32, torch.float32, torch.uint8)
        out = []
        for t, shape, d in zip((obs, rewards, dones), shapes, dt):
            t = torch.empty(shape, dtype=d, device=self.device) if t is None else _check_out(t, shape, d, self.device)
            out.append(t)
        self._call("wh_sampler_rollout", self.state.data_ptr(), int(steps), POLICIES[policy], float(p),
                   self._ptr(out[1]), self._ptr(out[2]), self._ptr(out[0]),
                   None if self.stats is None else self.stats.ref, int(self.train), self.seed, self.env_offset,
                   self.stream)
        return tuple(out)

    def policy(self, kind: str = "greedy", p: float = 0.0) -> torch.Tensor:
        self._call("wh_policy", self.state.data_ptr(), POLICIES[kind], float(p), self.actions.data_ptr(),
                   self.seed, self.env_offset, self.stream)
        return self.actions

    def rollout(self, steps: int, policy: str = "greedy", p: float = 0.0, rewards=None, dones=None,
                returns=None, autoreset: bool = True) -> None:
        """`steps` fused iterations of {policy, step, auto-reset}.  rewards [steps,B,NA] float32,
        dones [steps,B] uint8 and returns [B] float32 (+=) are optional device tensors."""
        for t, shape, d in ((rewards, (steps, self.B, self.agent_slots), torch.float32),
                            (dones, (steps, self.B), torch.uint8), (returns, (self.B,), torch.float32)):
            if t is not None:
                _check_out(t, shape, d, self.device)
        self._call("wh_rollout", self.state.data_ptr(), int(steps), POLICIES[policy], float(p),
                   self._ptr(rewards), self._ptr(dones), self._ptr(returns),
                   None if self.stats is None else self.stats.ref, int(bool(autoreset)),
                   int(self.train), self.seed, self.env_offset, self.stream)

    def stagger(self, offsets, policy: str = "greedy", p: float = 0.0) -> None:
        """Desynchronise episodes the way independent RLlib workers do: env e takes offsets[e]
        extra steps (policy actions, auto-reset) while the others wait, via masked sampler steps
        (wh_policy + wh_vector_step with an env mask).  Afterwards the envs' episode clocks differ, so
        a fused rollout meets episode ends, resets and expiry passes on every step instead of all
        at once.  Exactly the reference's per-env semantics: an env is only ever stepped or reset."""
        off = torch.as_tensor(np.asarray(offsets) if not torch.is_tensor(offsets) else offsets)
        off = off.to(device=self.device, dtype=torch.int32).reshape(self.B)
        for s in range(int(off.max().item()) if self.B else 0):
            self.vector_step(self.policy(policy, p), autoreset=True, observe=False, mask=off > s)

    def rollout_launcher(self, steps: int, policy: str = "greedy", p: float = 0.0, rewards=None,
                         dones=None, returns=None, autoreset: bool = True, events=None):
        """rollout() with every argument bound once (wh_rollout_prepare): returns a zero-argument
        callable that launches the same fused rollout through one cheap wh_launch_run call (the
        callable keeps the output tensors alive; the state tensor must stay in place).
        events=(start, stop) (torch.cuda.Event with enable_timing=True, either may be None): every
        launch stamps them at the kernel's own start and end (wh_launch_run_timed), so
        start.elapsed_time(stop) is the kernel's duration, with no marker packets around it."""
        for t, shape, d in ((rewards, (steps, self.B, self.agent_slots), torch.float32),
                            (dones, (steps, self.B), torch.uint8), (returns, (self.B,), torch.float32)):
            if t is not None:
                _check_out(t, shape, d, self.device)
        if self.host:
            raise nat.WarehouseNativeError("rollout_launcher: prepared launches are a device feature "
                                           "(the host engine runs rollout() directly)")
        lib = nat.lib()
        handle = ctypes.c_void_p()
        nat.check(lib.wh_rollout_prepare(self._cfgp, self.B, self.state.data_ptr(), int(steps), POLICIES[policy],
                                         float(p), nat.ptr(rewards), nat.ptr(dones), nat.ptr(returns),
                                         None if self.stats is None else self.stats.ref, int(bool(autoreset)),
                                         int(self.train), self.seed, self.env_offset, self.stream,
                                         ctypes.byref(handle)), "wh_rollout_prepare")
        h = handle.value
        if events is None:
            run = lib.wh_launch_run

            def launch() -> None:
                rc = run(h)
                if rc:
                    nat.check(rc, "wh_launch_run")
        else:
            run = lib.wh_launch_run_timed
            s = torch.cuda.current_stream(self.device)
            for ev in events:        # torch creates the HIP event at its first record
                if ev is not None:
                    ev.record(s)
            e0, e1 = (ctypes.c_void_p(None if ev is None else int(ev.cuda_event)) for ev in events)
            if any(ev is not None and not c.value for ev, c in zip(events, (e0, e1))):
                raise RuntimeError("rollout_launcher: an event has no HIP event handle")

            def launch() -> None:
                rc = run(h, e0, e1)
                if rc:
                    nat.check(rc, "wh_launch_run_timed")
        # everything the handle points into: the output buffers and the state tensor (held through
        # the env; reassigning env.state while the launcher lives is not supported -- the handle
        # keeps the old tensor alive and writes it).  The launch stream is the one current at
        # prepare time, for every launch of the handle.
        launch.keep = (rewards, dones, returns, self.stats, events, self.state, self)
        launch.stream = self.stream
        weakref.finalize(launch, lib.wh_launch_free, h)
        return launch

    # ------------------------------------------------------------------ canonical state
    def to_canonical(self) -> Dict[str, torch.Tensor]:
        B, NA, P = self.B, self.agent_slots, self.P
        z = dict(pos=torch.empty((B, NA, 2), dtype=torch.int32, device=self.device),
                 agent_target=torch.empty((B, NA), dtype=torch.int32, device=self.device),
                 pickup_target=torch.empty((B, P), dtype=torch.int32, device=self.device),
                 pickup_timer=torch.empty((B, P), dtype=torch.int32, device=self.device),
                 t=torch.empty(B, dtype=torch.int32, device=self.device),
                 n=torch.empty(B, dtype=torch.int32, device=self.device),
                 fresh=torch.empty(B, dtype=torch.uint8, device=self.device),
                 episode=torch.empty(B, dtype=torch.int32, device=self.device))
        self._call("wh_unpack", self.state.data_ptr(), *(z[k].data_ptr() for k in
                   ("pos", "agent_target", "pickup_target", "pickup_timer", "t", "n", "fresh", "episode")),
                   self.stream)
        return z

    def from_canonical(self, c: Dict[str, object]) -> None:
        B, NA, P = self.B, self.agent_slots, self.P
        d = self.device
        t = dict(pos=_dev_i32(c["pos"], d, (B, NA, 2)), agent_target=_dev_i32(c["agent_target"], d, (B, NA)),
                 pickup_target=_dev_i32(c["pickup_target"], d, (B, P)),
                 pickup_timer=_dev_i32(c["pickup_timer"], d, (B, P)), t=_dev_i32(c["t"], d, (B,)),
                 n=_dev_i32(c.get("n", np.full(B, NA)), d, (B,)),
                 fresh=torch.as_tensor(np.asarray(c.get("fresh", np.zeros(B, bool)))).to(d, torch.uint8).contiguous(),
                 episode=_dev_i32(c.get("episode", np.zeros(B, np.int64)), d, (B,)))
        self._call("wh_pack", *(t[k].data_ptr() for k in
                   ("pos", "agent_target", "pickup_target", "pickup_timer", "t", "n", "fresh", "episode")),
                   self.state.data_ptr(), self.stream)
