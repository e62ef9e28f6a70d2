"""Vectorised (B envs) numpy restatement of the hot path -- TEST INFRASTRUCTURE ONLY.

Same transition as `oracle.core` (itself pinned to the reference: warehouse/core.py:167-442,
baseline/solvers.py:27-58), written over struct-of-arrays [B, ...] so the GPU kernels can be
checked at B in the thousands in seconds.  It is cross-checked against `oracle.core` per env in
tests/test_oracle_batched.py.  Agent slots are fixed at NA per env with a per-env agent count n
(the Train variants, warehouse/variants.py:65-98); slots >= n hold pos (0, 0), target -1.

Draw sources:
  * `Injected(...)`  -- explicit draws (spawns, request picks, regeneration picks as positions in
                        the ascending inactive list, exactly what the reference's
                        np.random.choice(inactive, k) returns an index into, core.py:339-343).
  * `PhiloxDraws(seed, env_ids)` -- the device's counter-based contract (oracle/philox.py).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import philox as ph
from .core import Layout

U64 = np.uint64


def tables(L: Layout):
    pk = L.pickup_xy()
    dl = L.delivery_xy()
    cell = L.cell_pickup().reshape(-1)
    interior = [(x, y) for x in range(1, L.D - 1) for y in range(1, L.D - 1) if cell[x * L.D + y] < 0]
    valid = np.array(interior, np.int32)
    return pk, dl, cell, valid


@dataclass
class BState:
    pos: np.ndarray        # [B, NA, 2] int32
    agent_tgt: np.ndarray  # [B, NA] int32
    pk_tgt: np.ndarray     # [B, P] int32
    pk_timer: np.ndarray   # [B, P] int32
    t: np.ndarray          # [B] int64
    n: np.ndarray          # [B] int32
    fresh: np.ndarray      # [B] bool
    episode: np.ndarray    # [B] uint32

    @staticmethod
    def zeros(L: Layout, B: int, NA: int) -> "BState":
        return BState(pos=np.zeros((B, NA, 2), np.int32), agent_tgt=np.full((B, NA), -1, np.int32),
                      pk_tgt=np.full((B, L.P), -1, np.int32), pk_timer=np.full((B, L.P), -1, np.int32),
                      t=np.zeros(B, np.int64), n=np.zeros(B, np.int32), fresh=np.zeros(B, bool),
                      episode=np.zeros(B, np.uint32))

    def copy(self) -> "BState":
        return BState(*(np.array(getattr(self, f), copy=True) for f in
                        ("pos", "agent_tgt", "pk_tgt", "pk_timer", "t", "n", "fresh", "episode")))

    @property
    def B(self):
        return self.pos.shape[0]

    @property
    def NA(self):
        return self.pos.shape[1]


class Injected:
    def __init__(self, spawn=None, reset_sel=None, reset_tgt=None, n=None, rpos=None, rtgt=None,
                 coins=None, rand_actions=None):
        self.spawn, self.reset_sel, self.reset_tgt, self.n = spawn, reset_sel, reset_tgt, n
        self.rpos, self.rtgt = rpos, rtgt
        self.coins, self.rand_actions = coins, rand_actions


class PhiloxDraws:
    def __init__(self, seed: int, env_ids: np.ndarray):
        self.streams = ph.Streams(seed)
        self.env_ids = np.asarray(env_ids, np.uint64)

    def word(self, ep, t, purpose, j):
        return self.streams.word(self.env_ids, np.asarray(ep, U64), np.asarray(t, U64), purpose, j)


def _bits(idx):
    return np.left_shift(U64(1), np.asarray(idx, np.int64).astype(U64))


def _choose_without_replacement(avail_mask, count, words_fn, k_needed, first_word, stride=2):
    """Sequential r-th-remaining selection used by the philox contract (word first + stride*j)."""
    B = avail_mask.shape[0]
    R = k_needed.max(initial=0)
    sel = np.full((B, max(R, 0)), -1, np.int64)
    rem = avail_mask.copy()
    for j in range(R):
        act = j < k_needed
        w = words_fn(first_word + stride * j)
        r = ph.uniform_int(np.maximum(count - j, 1), w)
        s = ph.select_bit(rem, r)
        s = np.where(act, s, -1)
        sel[:, j] = s
        rem = np.where(act, rem & ~_bits(np.maximum(s, 0)), rem)
    return sel


def _floyd_subset(P, R, words_fn, first_word, B, stride=2):
    """Floyd's R-subset of range(P) as the philox contract draws it (word first + stride*j):
    item j takes r = uniform_int(m+1) with m = P-R+j, or m when r is already taken."""
    S = np.zeros(B, U64)
    sel = np.zeros((B, R), np.int64)
    for j in range(R):
        m = P - R + j
        r = ph.uniform_int(m + 1, words_fn(first_word + stride * j))
        taken = ((S >> r.astype(U64)) & U64(1)).astype(bool)
        s = np.where(taken, m, r)
        S |= _bits(s)
        sel[:, j] = s
    return sel


# --------------------------------------------------------------------------- reset
def reset(L: Layout, S: BState, draws, mask: Optional[np.ndarray] = None, nmax: Optional[int] = None,
          n_fixed: Optional[int] = None) -> None:
    """core.py:167-221 per env (mask selects which envs reset).  Philox mode bumps the episode."""
    B, NA = S.B, S.NA
    m = np.ones(B, bool) if mask is None else np.asarray(mask, bool)
    pk, dl, cell, valid = tables(L)
    ep = S.episode.astype(np.int64) + 1
    if isinstance(draws, PhiloxDraws):
        wf = lambda j: draws.word(ep, 0, ph.RESET, j)  # noqa: E731
        if nmax is not None:
            n = 1 + ph.uniform_int(nmax, wf(0))
        else:
            n = np.full(B, n_fixed if n_fixed is not None else NA, np.int64)
        spawn = np.zeros((B, NA, 2), np.int32)
        for i in range(NA):
            spawn[:, i] = valid[ph.uniform_int(len(valid), wf(1 + i))]
        full_d = np.full(B, U64((1 << L.Dp) - 1 if L.Dp < 64 else 0xFFFFFFFFFFFFFFFF), U64)
        kR = np.full(B, L.R)
        sel = _floyd_subset(L.P, L.R, wf, 1 + NA, B)
        tgt = _choose_without_replacement(full_d, L.Dp, wf, kR, 2 + NA)
    else:
        n = np.asarray(draws.n if draws.n is not None else np.full(B, n_fixed or NA), np.int64)
        spawn = np.asarray(draws.spawn, np.int32)
        sel = np.asarray(draws.reset_sel, np.int64)
        tgt = np.asarray(draws.reset_tgt, np.int64)
    slot = np.arange(NA)[None, :]
    live = slot < n[:, None]
    pos = np.where(live[..., None], spawn, 0).astype(np.int32)
    pk_tgt = np.full((B, L.P), -1, np.int32)
    pk_timer = np.full((B, L.P), -1, np.int32)
    rows = np.repeat(np.arange(B), L.R)
    pk_tgt[rows, sel.reshape(-1)] = tgt.reshape(-1)
    pk_timer[rows, sel.reshape(-1)] = L.W
    S.pos[m] = pos[m]
    S.agent_tgt[m] = -1
    S.pk_tgt[m] = pk_tgt[m]
    S.pk_timer[m] = pk_timer[m]
    S.t[m] = 0
    S.n[m] = n[m]
    S.fresh[m] = True
    S.episode[m] = ep[m].astype(np.uint32)   # every reset bumps the episode counter


# --------------------------------------------------------------------------- step
def _pack(a, b, c, d):
    return (a.astype(np.int64) | (b.astype(np.int64) << 8) | (c.astype(np.int64) << 16)
            | (d.astype(np.int64) << 24))


def step(L: Layout, S: BState, actions: np.ndarray, draws, order: Optional[np.ndarray] = None):
    """One transition for all B envs (core.py:262-442); returns rewards [B,NA] f32, done [B],
    n_inactive [B], k [B].  `actions` must already be in 0..8 (the host wraps negatives)."""
    B, NA, D, P, R = S.B, S.NA, L.D, L.P, L.R
    pk, dl, cell, valid = tables(L)
    b = np.arange(B)
    t_new = S.t + 1
    acts = np.asarray(actions, np.int64)
    assert acts.shape == (B, NA) and acts.min(initial=0) >= 0 and acts.max(initial=0) <= 8

    # -- move + collision, sequential in processing order (core.py:275-300)
    occ = np.zeros((B, D * D), bool)
    for i in range(NA):
        li = i < S.n
        occ[b[li], S.pos[li, i, 0] * D + S.pos[li, i, 1]] = True
    keys = np.full((B, 3 * NA), -1, np.int64)
    for s in range(NA):
        if order is None:
            idx = np.full(B, s)
            act = s < S.n
            a = acts[b, idx]
        else:
            # entry = agent id (bits 0-7) | the entry's own action + 1 (bits 8-15, 0: actions[id]),
            # -1 terminated (include/warehouse_amd.h, wh_step)
            raw = np.asarray(order[:, s], np.int64)
            act = raw >= 0
            idx = np.where(act, raw & 0xFF, 0)
            sact = np.where(act, (raw >> 8) & 0xFF, 0)
            a = np.where(sact > 0, sact - 1, acts[b, idx])
        px, py = S.pos[b, idx, 0].astype(np.int64), S.pos[b, idx, 1].astype(np.int64)
        x, y = px + a // 3 - 1, py + a % 3 - 1
        x = np.where((x >= 0) & (x < D), x, px)
        y = np.where((y >= 0) & (y < D), y, py)
        blocked = occ[b, x * D + y] | np.any(keys == _pack(px, py, x, y)[:, None], axis=1)
        ok = act & ~blocked
        occ[b[ok], (px * D + py)[ok]] = False
        occ[b[ok], (x * D + y)[ok]] = True
        keys[:, 3 * s] = np.where(ok, _pack(x, y, px, py), -1)
        diag = ok & (x != px) & (y != py)
        keys[:, 3 * s + 1] = np.where(diag, _pack(x, py, px, y), -1)
        keys[:, 3 * s + 2] = np.where(diag, _pack(px, y, x, py), -1)
        S.pos[b[ok], idx[ok], 0] = x[ok]
        S.pos[b[ok], idx[ok], 1] = y[ok]

    # -- expiry (core.py:303-306)
    live = S.pk_tgt > -1
    S.pk_timer[live] -= 1
    gone = S.pk_timer == 0
    S.pk_tgt[gone] = -1
    S.pk_timer[gone] = -1

    # -- pickups: gather for all agents, then scatter (core.py:309-335)
    slot_live = np.arange(NA)[None, :] < S.n[:, None]
    c = cell[S.pos[..., 0] * D + S.pos[..., 1]]
    cc = np.maximum(c, 0)
    picks = slot_live & (c >= 0) & (S.agent_tgt == -1) & (np.take_along_axis(S.pk_tgt, cc, 1) > -1)
    got = np.take_along_axis(S.pk_tgt, cc, 1)
    S.agent_tgt = np.where(picks, got, S.agent_tgt).astype(np.int32)
    rb, ra = np.nonzero(picks)
    S.pk_tgt[rb, c[rb, ra]] = -1
    S.pk_timer[rb, c[rb, ra]] = -1
    rewards = picks.astype(np.float32)

    # -- regeneration (core.py:338-351)
    inact = S.pk_tgt == -1
    n_in = inact.sum(1)
    k = R - P + n_in
    imask = np.zeros(B, U64)
    for j in range(P):
        imask |= np.where(inact[:, j], U64(1) << U64(j), U64(0))
    if isinstance(draws, PhiloxDraws):
        wf = lambda j: draws.word(S.episode, t_new, ph.REGEN, j)  # noqa: E731
        sel = _choose_without_replacement(imask, n_in, wf, k, 0)
        full_d = np.full(B, U64((1 << L.Dp) - 1 if L.Dp < 64 else 0xFFFFFFFFFFFFFFFF), U64)
        tg = _choose_without_replacement(full_d, L.Dp, wf, k, 1)
    else:
        rpos = np.asarray(draws.rpos, np.int64)
        tg = np.asarray(draws.rtgt, np.int64)
        sel = np.full(rpos.shape, -1, np.int64)
        for j in range(rpos.shape[1]):
            act = j < k
            sel[:, j] = np.where(act, ph.select_bit(imask, np.where(act, rpos[:, j], 0)), -1)
    for j in range(sel.shape[1]):
        act = j < k
        S.pk_timer[b[act], sel[act, j]] = L.W
        S.pk_tgt[b[act], sel[act, j]] = tg[act, j]

    # -- deliveries (core.py:354-368)
    carrying = slot_live & (S.agent_tgt > -1)
    dxy = dl[np.maximum(S.agent_tgt, 0)]
    arrived = carrying & np.all(dxy == S.pos, axis=2)
    S.agent_tgt = np.where(arrived, -1, S.agent_tgt).astype(np.int32)
    rewards += arrived.astype(np.float32)

    S.t = t_new
    S.fresh[:] = False
    done = S.t >= L.T
    return rewards.astype(np.float32), done, n_in, k


# --------------------------------------------------------------------------- observation
def observe(L: Layout, S: BState) -> np.ndarray:
    """[B, NA, 9R+1] int32 rows in sorted-key order; slots >= n are zero rows."""
    B, NA, R = S.B, S.NA, L.R
    pk, dl, cell, valid = tables(L)
    null = L.null
    slot = np.arange(R)[None, :]
    nn = S.n[:, None]
    apos = np.full((B, R, 2), null, np.int32)
    apos[:, :NA][slot[:, :NA] < nn] = S.pos[slot[:, :NA] < nn]
    carry = np.zeros((B, R), bool)
    carry[:, :NA] = (S.agent_tgt > -1) & (slot[:, :NA] < nn)
    avail = np.where((slot < nn) & ~S.fresh[:, None], (~carry).astype(np.int32), 0)
    dtg = np.full((B, R, 2), null, np.int32)
    tg = np.zeros((B, R), np.int64)
    tg[:, :NA] = np.maximum(S.agent_tgt, 0)
    showing = carry & ~S.fresh[:, None]
    dtg[showing] = dl[tg[showing]]
    order = np.argsort(S.pk_tgt < 0, axis=1, kind="stable")[:, :R]
    act_t = np.take_along_axis(S.pk_tgt, order, 1)
    req = np.concatenate([pk[order], dl[np.maximum(act_t, 0)]], axis=2)
    out = np.zeros((B, NA, L.obs_len), np.int32)
    rows_all = np.arange(R)
    for i in range(NA):
        keep_i = rows_all[rows_all != i]
        keep_1 = rows_all[rows_all != 1]
        dsel = np.where(S.fresh[:, None], keep_i[None, :], keep_1[None, :])
        parts = [
            S.n[:, None],
            avail[:, keep_i],
            np.take_along_axis(dtg, dsel[..., None], 1).reshape(B, -1),
            apos[:, keep_i].reshape(B, -1),
            req.reshape(B, -1),
            avail[:, i:i + 1],
            dtg[:, i],
            apos[:, i],
        ]
        row = np.concatenate([np.asarray(p, np.int32) for p in parts], axis=1)
        out[:, i] = np.where((i < S.n)[:, None], row, 0)
    return out


# --------------------------------------------------------------------------- policies
def greedy(L: Layout, S: BState, p: float, draws=None) -> np.ndarray:
    """baseline/solvers.py:27-58 evaluated on the state (equivalent to its observation)."""
    B, NA, R = S.B, S.NA, L.R
    pk, dl, cell, valid = tables(L)
    order = np.argsort(S.pk_tgt < 0, axis=1, kind="stable")[:, :R]
    req = pk[order]                                            # [B, R, 2]
    acts = np.zeros((B, NA), np.int32)
    for i in range(NA):
        me = S.pos[:, i].astype(np.int64)
        dist = np.abs(req - me[:, None, :]).sum(2)
        near = req[np.arange(B), np.argmin(dist, axis=1)]
        carrying = S.agent_tgt[:, i] > -1
        goal = np.where(carrying[:, None], dl[np.maximum(S.agent_tgt[:, i], 0)], near)
        goal = np.where(S.fresh[:, None], L.null, goal)
        st = np.clip(goal - me, -1, 1)
        a = (st[:, 0] + 1) * 3 + (st[:, 1] + 1)
        if p > 0:
            if isinstance(draws, PhiloxDraws):
                coin = (draws.word(S.episode, S.t, ph.POLICY, 2 * i) >> U64(8)).astype(np.float64) / 2.0 ** 24
                ra = ph.uniform_int(9, draws.word(S.episode, S.t, ph.POLICY, 2 * i + 1))
            else:
                coin, ra = draws.coins[:, i], draws.rand_actions[:, i]
            a = np.where(coin < np.float32(p), ra, a)
        acts[:, i] = np.where(i < S.n, a, 4)
    return acts


def random_actions(S: BState, draws: PhiloxDraws) -> np.ndarray:
    NA = S.NA
    acts = np.zeros((S.B, NA), np.int32)
    for i in range(NA):
        acts[:, i] = ph.uniform_int(9, draws.word(S.episode, S.t, ph.RANDOM, i))
    return acts
