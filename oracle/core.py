"""Single-env numpy restatement of the reference hot path -- TEST INFRASTRUCTURE ONLY.

Restates, with the reference's exact integer semantics and draw order:
  * the static layout built in `warehouse/core.py:170-188` (pickup and delivery point tables),
  * `Warehouse.reset()`  `warehouse/core.py:167-260`,
  * `Warehouse.step()`   `warehouse/core.py:262-442`,
  * the greedy policy    `baseline/solvers.py:27-58`,
  * the variant table    `warehouse/variants.py:19-98`.

Draws go through a *draw source* object so the same transition code can be driven by
  * `GlobalNumpyDraws` -- the global legacy MT19937 stream, in the reference's call order
    (`core.py:196-197` spawn, `:215-220` reset requests, `:339-350` regeneration,
    `solvers.py:44` policy coin, `variants.py:73-74` Train agent count), or
  * `InjectedDraws`    -- recorded draws (the GPU kernels' parity mode).

Pinned against fixtures produced by the reference itself (tests/golden/make_golden.py) in
tests/test_oracle_golden.py.  Never imported by the product package.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

# (D, R, racks, T, W, max agents) per size -- warehouse/variants.py:25-62
VARIANTS: Dict[str, dict] = {
    "small": dict(D=12, R=4, racks=(4, 8), T=200, W=200, nmax=4),
    "medium": dict(D=16, R=9, racks=(4, 8, 12), T=200, W=200, nmax=9),
    "large": dict(D=20, R=16, racks=(4, 8, 12, 16), T=200, W=200, nmax=16),
}

# sorted gym.spaces.Dict key order (gym sorts plain-dict keys; core.py:119-148)
OBS_KEYS: Tuple[str, ...] = (
    "num_agents",
    "other_availabilities",
    "other_delivery_targets",
    "other_positions",
    "requests",
    "self_availability",
    "self_delivery_target",
    "self_position",
)


def move_delta(action: int) -> Tuple[int, int]:
    """MOVES[action] of core.py:38 including Python's negative-index wrap; IndexError otherwise."""
    a = int(action)
    if a < -9 or a > 8:
        raise IndexError("list index out of range")
    a %= 9
    return a // 3 - 1, a % 3 - 1


@dataclass(frozen=True)
class Layout:
    """Static per-variant geometry (core.py:92-107, 170-188)."""

    D: int
    R: int
    racks: Tuple[int, ...]
    T: int
    W: int

    @property
    def P(self) -> int:
        return 4 * len(self.racks) ** 2

    @property
    def Dp(self) -> int:
        return 4 * (self.D - 4)

    @property
    def null(self) -> int:
        return self.D // 2

    @property
    def obs_len(self) -> int:
        return 9 * self.R + 1

    def pickup_xy(self) -> np.ndarray:
        # rack-major, then the four cells around the rack corner: (-1,-1), (0,-1), (-1,0), (0,0)
        out = np.zeros((self.P, 2), np.int32)
        nr = len(self.racks)
        for idx in range(self.P):
            blk, q = divmod(idx, 4)
            ix, iy = divmod(blk, nr)
            out[idx] = (self.racks[ix] - 1 + (q & 1), self.racks[iy] - 1 + (q >> 1))
        return out

    def delivery_xy(self) -> np.ndarray:
        # for v in 2..D-3: bottom, left, top, right border cells
        out = np.zeros((self.Dp, 2), np.int32)
        for idx in range(self.Dp):
            v, side = 2 + idx // 4, idx % 4
            out[idx] = [(v, 0), (0, v), (v, self.D - 1), (self.D - 1, v)][side]
        return out

    def cell_pickup(self) -> np.ndarray:
        grid = np.full((self.D, self.D), -1, np.int32)
        for idx, (x, y) in enumerate(self.pickup_xy()):
            grid[x, y] = idx
        return grid

    def obs_slices(self) -> Dict[str, slice]:
        R = self.R
        widths = dict(num_agents=1, other_availabilities=R - 1, other_delivery_targets=2 * (R - 1),
                      other_positions=2 * (R - 1), requests=4 * R, self_availability=1,
                      self_delivery_target=2, self_position=2)
        out, o = {}, 0
        for k in OBS_KEYS:
            out[k] = slice(o, o + widths[k])
            o += widths[k]
        assert o == self.obs_len
        return out


def layout_for(variant: str) -> Layout:
    v = VARIANTS[variant]
    return Layout(D=v["D"], R=v["R"], racks=tuple(v["racks"]), T=v["T"], W=v["W"])


@dataclass
class State:
    """Canonical per-env state (core.py:150-165 without the render-only prev_* copies)."""

    pos: np.ndarray          # (n, 2) int32
    agent_tgt: np.ndarray    # (n,) int32, delivery index or -1
    pk_tgt: np.ndarray       # (P,) int32, delivery index or -1
    pk_timer: np.ndarray     # (P,) int32, remaining wait or -1
    t: int = 0
    fresh: bool = True       # True right after reset(): observation availabilities are 0 (core.py:233)

    def copy(self) -> "State":
        return State(self.pos.copy(), self.agent_tgt.copy(), self.pk_tgt.copy(),
                     self.pk_timer.copy(), int(self.t), bool(self.fresh))


# --------------------------------------------------------------------------- draw sources
class GlobalNumpyDraws:
    """The reference's draws, taken from the global legacy numpy stream in the reference's order."""

    def __init__(self, space_rng: Optional[np.random.RandomState] = None):
        # gym's Discrete.sample uses the space's own generator (solvers.py:45), never np.random
        self.space_rng = space_rng if space_rng is not None else np.random.RandomState(0)

    def num_agents(self, nmax: int) -> int:                       # variants.py:73-74
        return int(np.random.randint(1, nmax + 1))

    def spawn(self, L: Layout, n: int) -> np.ndarray:             # core.py:191-201
        blocked = {tuple(c) for c in L.pickup_xy().tolist()}
        cells = []
        while len(cells) < n:
            x = np.random.randint(1, L.D - 1)
            y = np.random.randint(1, L.D - 1)
            if (x, y) not in blocked:
                cells.append((x, y))
        return np.array(cells, np.int32).reshape(n, 2)

    def reset_requests(self, L: Layout) -> Tuple[np.ndarray, np.ndarray]:   # core.py:215-220
        sel = np.random.choice(L.P, L.R, replace=False)
        tgt = np.random.choice(L.Dp, L.R, replace=False)
        return sel.astype(np.int32), tgt.astype(np.int32)

    def regen(self, L: Layout, n_inactive: int, k: int) -> Tuple[np.ndarray, np.ndarray]:
        # choice(inactive, k) == inactive[permutation(len(inactive))[:k]]  (core.py:339-350)
        pos = np.random.choice(n_inactive, k, replace=False)
        tgt = np.random.choice(L.Dp, k, replace=False)
        return pos.astype(np.int32), tgt.astype(np.int32)

    def policy_coin(self) -> float:                              # solvers.py:44
        return float(np.random.uniform())

    def random_action(self) -> int:                              # solvers.py:45
        return int(self.space_rng.randint(9))


class InjectedDraws:
    """Replays recorded draws (the kernels' `injected` mode)."""

    def __init__(self, spawn=None, reset_sel=None, reset_tgt=None, regen=None, coins=None,
                 actions=None, nagents=None):
        self._spawn = spawn
        self._reset = (reset_sel, reset_tgt)
        self._regen = list(regen or [])       # list of (rpos[k], rtgt[k])
        self._coins = list(coins or [])
        self._actions = list(actions or [])
        self._nagents = list(nagents or [])

    def num_agents(self, nmax):
        return int(self._nagents.pop(0))

    def spawn(self, L, n):
        return np.asarray(self._spawn, np.int32).reshape(n, 2)

    def reset_requests(self, L):
        return np.asarray(self._reset[0], np.int32), np.asarray(self._reset[1], np.int32)

    def regen(self, L, n_inactive, k):
        rpos, rtgt = self._regen.pop(0)
        rpos = np.asarray(rpos, np.int32)[:k]
        rtgt = np.asarray(rtgt, np.int32)[:k]
        assert len(rpos) == k and (k == 0 or rpos.max() < n_inactive)
        return rpos, rtgt

    def policy_coin(self):
        return float(self._coins.pop(0))

    def random_action(self):
        return int(self._actions.pop(0))


# --------------------------------------------------------------------------- transition
def reset(L: Layout, n: int, draws) -> State:
    """core.py:167-221: spawn agents off the pickup cells, then open R requests."""
    assert 1 <= n <= L.R, "num_agents <= num_requests (core.py:89)"
    pos = draws.spawn(L, n)
    sel, tgt = draws.reset_requests(L)
    pk_tgt = np.full(L.P, -1, np.int32)
    pk_timer = np.full(L.P, -1, np.int32)
    pk_tgt[sel] = tgt
    pk_timer[sel] = L.W
    return State(pos=pos, agent_tgt=np.full(n, -1, np.int32), pk_tgt=pk_tgt, pk_timer=pk_timer,
                 t=0, fresh=True)


@dataclass
class StepResult:
    rewards: np.ndarray      # (n,) float32
    done: bool
    n_inactive: int          # regeneration population (core.py:338)
    k: int                   # requests regenerated this step (core.py:341)
    regen_pos: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))
    regen_tgt: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))


def resolve_moves(L: Layout, pos: np.ndarray, actions: Sequence[int], order: Sequence[int]) -> None:
    """core.py:274-300, in place.  `order` lists agent ids in action-dict iteration order; agents
    not listed do not move.  An entry may be an (id, action) pair -- a dict entry with its own
    action, as core.py:279-281 reads them (int(key) indexes like numpy, so '-1' is agent n-1 and
    one agent named under two keys moves twice); a plain id takes actions[id].  Occupancy is a set of cells (a cell is freed when ANY agent leaves it,
    even if another agent still stands there); `forbidden` holds (from, to) cell pairs that later
    movers may not take (reverse of every accepted move, plus both crossing diagonals)."""
    occupied = {(int(x), int(y)) for x, y in pos}
    forbidden = set()
    for i in order:
        i, a = (i if isinstance(i, tuple) else (i, actions[i]))
        dx, dy = move_delta(a)
        px, py = int(pos[i, 0]), int(pos[i, 1])
        x, y = px + dx, py + dy
        if not 0 <= x < L.D:
            x = px
        if not 0 <= y < L.D:
            y = py
        if (x, y) in occupied or ((px, py), (x, y)) in forbidden:
            continue
        occupied.discard((px, py))
        occupied.add((x, y))
        forbidden.add(((x, y), (px, py)))
        if x != px and y != py:
            forbidden.add(((x, py), (px, y)))
            forbidden.add(((px, y), (x, py)))
        pos[i] = (x, y)


def step(L: Layout, st: State, actions: Sequence[int], order: Optional[Sequence[int]],
         draws) -> StepResult:
    """One transition of core.py:262-442 (state updated in place)."""
    n = len(st.pos)
    st.t += 1
    st.fresh = False
    resolve_moves(L, st.pos, actions, range(n) if order is None else order)

    # request expiry (core.py:303-306)
    live = st.pk_tgt > -1
    st.pk_timer[live] -= 1
    gone = st.pk_timer == 0
    st.pk_tgt[gone] = -1
    st.pk_timer[gone] = -1

    # pickups: every agent decides against the pre-pickup table, then the table is cleared
    cellmap = L.cell_pickup()
    c = cellmap[st.pos[:, 0], st.pos[:, 1]]
    picks = (c >= 0) & (st.agent_tgt == -1)
    picks &= np.where(c >= 0, st.pk_tgt[np.maximum(c, 0)] > -1, False)
    rewards = np.zeros(n, np.float32)
    if picks.any():
        st.agent_tgt[picks] = st.pk_tgt[c[picks]]
        st.pk_tgt[c[picks]] = -1
        st.pk_timer[c[picks]] = -1
        rewards[picks] += np.float32(1.0)

    # regeneration: keep exactly R open requests (core.py:338-351)
    inactive = np.flatnonzero(st.pk_tgt == -1)
    k = L.R - L.P + len(inactive)
    rpos, rtgt = draws.regen(L, len(inactive), k)
    chosen = inactive[rpos]
    st.pk_timer[chosen] = L.W
    st.pk_tgt[chosen] = rtgt

    # deliveries (core.py:354-368)
    dl = L.delivery_xy()
    carrying = np.flatnonzero(st.agent_tgt > -1)
    arrived = carrying[np.all(dl[st.agent_tgt[carrying]] == st.pos[carrying], axis=1)]
    st.agent_tgt[arrived] = -1
    rewards[arrived] += np.float32(1.0)

    done = st.t >= L.T
    return StepResult(rewards=rewards, done=bool(done), n_inactive=len(inactive), k=int(k),
                      regen_pos=np.asarray(rpos, np.int32), regen_tgt=np.asarray(rtgt, np.int32))


def observe(L: Layout, st: State) -> np.ndarray:
    """Per-agent observation rows in sorted-key order, (n, 9R+1) int32 (core.py:224-260, 371-432)."""
    n, R, D = len(st.pos), L.R, L.D
    null = L.null
    apos = np.full((R, 2), null, np.int32)
    apos[:n] = st.pos
    avail = np.zeros(R, np.int32)
    dtg = np.full((R, 2), null, np.int32)
    if not st.fresh:
        carrying = st.agent_tgt > -1
        avail[:n] = np.where(carrying, 0, 1)
        dl = L.delivery_xy()
        rows = np.flatnonzero(carrying)
        dtg[rows] = dl[st.agent_tgt[rows]]
    active = np.flatnonzero(st.pk_tgt > -1)
    req = np.concatenate([L.pickup_xy()[active], L.delivery_xy()[st.pk_tgt[active]]], axis=1)
    out = np.zeros((n, L.obs_len), np.int32)
    for i in range(n):
        drop_dtg = i if st.fresh else 1   # core.py:256 vs the step-time row-1 quirk at core.py:428
        parts = [
            [n],
            np.delete(avail, i),
            np.delete(dtg, drop_dtg, axis=0).ravel(),
            np.delete(apos, i, axis=0).ravel(),
            req.ravel(),
            [avail[i]],
            dtg[i],
            apos[i],
        ]
        out[i] = np.concatenate([np.asarray(p, np.int32).ravel() for p in parts])
    return out


def obs_dicts(L: Layout, flat: np.ndarray) -> Dict[str, Dict[str, np.ndarray]]:
    """Split flat rows back into the reference's per-agent dicts (dtypes as core.py:224-260)."""
    sl = L.obs_slices()
    R = L.R
    out = {}
    for i, row in enumerate(np.asarray(flat)):
        out[str(i)] = {
            "num_agents": row[sl["num_agents"]].astype(np.int32),
            "self_position": row[sl["self_position"]].astype(np.int32),
            "self_availability": row[sl["self_availability"]].astype(np.int8),
            "self_delivery_target": row[sl["self_delivery_target"]].astype(np.int32),
            "other_positions": row[sl["other_positions"]].astype(np.int32).reshape(R - 1, 2),
            "other_availabilities": row[sl["other_availabilities"]].astype(np.int8),
            "other_delivery_targets": row[sl["other_delivery_targets"]].astype(np.int32).reshape(R - 1, 2),
            "requests": row[sl["requests"]].astype(np.int32).reshape(R, 4),
        }
    return out


def greedy(L: Layout, flat_obs: np.ndarray, p: float, draws) -> np.ndarray:
    """baseline/solvers.py:27-58 on flat observation rows; one coin per agent, always drawn."""
    sl = L.obs_slices()
    acts = np.zeros(len(flat_obs), np.int32)
    for i, row in enumerate(np.asarray(flat_obs)):
        me = row[sl["self_position"]]
        if row[sl["self_availability"]][0] == 0:
            goal = row[sl["self_delivery_target"]]
        else:
            req = row[sl["requests"]].reshape(L.R, 4)[:, :2]
            goal = req[int(np.argmin(np.abs(req - me).sum(axis=1)))]
        sx, sy = np.clip(goal - me, -1, 1)
        if draws.policy_coin() < p:
            acts[i] = draws.random_action()
        else:
            acts[i] = (sx + 1) * 3 + (sy + 1)
    return acts


# --------------------------------------------------------------------------- reference-shaped env
class OracleWarehouse:
    """Reference-shaped wrapper (same call surface as warehouse/core.py:73) around the restatement.
    Used as the CPU baseline `warehouse.core.Warehouse.step()` in bench.py and by the C1 tests."""

    def __init__(self, variant: str, num_agents: int, draws=None, train: bool = False):
        self.layout = layout_for(variant)
        self.nmax = VARIANTS[variant]["nmax"]
        self.train = train
        self.draws = draws if draws is not None else GlobalNumpyDraws()
        self.num_agents = self.draws.num_agents(self.nmax) if train else num_agents
        self.num_requests = self.layout.R
        self.state: Optional[State] = None

    def reset(self):
        if self.train:
            self.num_agents = self.draws.num_agents(self.nmax)
        self.state = reset(self.layout, self.num_agents, self.draws)
        return obs_dicts(self.layout, observe(self.layout, self.state))

    def step(self, action_dict: Dict[str, int]):
        # every entry with its own key and action, as core.py:279-281 reads them
        order = [(int(k), int(a)) for k, a in action_dict.items()]
        acts = np.zeros(self.num_agents, np.int64)
        res = step(self.layout, self.state, acts, order, self.draws)
        obs = obs_dicts(self.layout, observe(self.layout, self.state))
        rewards = {str(i): res.rewards[i] for i in range(self.num_agents)}
        dones = {str(i): res.done for i in range(self.num_agents)}
        dones["__all__"] = res.done
        return obs, rewards, dones, {str(i): {} for i in range(self.num_agents)}
