"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

Run in the build container only (it imports /root/reference through `ref_stubs`):

    python tests/golden/make_golden.py

It never runs on the GPU box and nothing imports it at test time; the tests read only the
`.npz` files it writes.  What it records:

* G1 `g1_<variant>_n<N>_s<seed>.npz` -- full 200-step episodes with random actions drawn from a
  separate RandomState (so the env's global MT19937 stream is untouched), recording every draw
  the env makes (`warehouse/core.py:195-220` at reset, `:339-350` per step), the canonical state
  after reset and after every step, per-agent observations flattened in sorted-key order, rewards
  and dones.  `ord_*` files do the same with shuffled/partial action dicts (`core.py:279`);
  `keys_*` with the key forms `int(key)` accepts beyond "0".."n-1" (`core.py:280`): int keys,
  negative keys (numpy wraps them to n + key) and one agent named under two keys in one dict
  (moved once per entry, each with its own action); `long_*` with dicts of up to 4n entries
  (agents under several of the four forms at once: several moves of one agent in one step).
* G2 `g2_<variant>.npz` -- single transitions from adversarial hand-built states (agents packed
  on a few cells, on pickup cells, carrying next to their delivery cell, timers about to expire,
  t about to reach T) with random actions and dict orders.
* G3 `g3_greedy.npz` -- seeded greedy rollouts through `baseline/solvers.py` exactly as
  `baseline/run.py:15-76` drives them, plus the total-reward line `run.main` prints.
"""
from __future__ import annotations

import contextlib
import io
import os
import sys

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ref_stubs  # noqa: E402

ref_wh, ref_solvers, ref_run = ref_stubs.import_reference()

VARIANTS = {
    "small": ref_wh.WarehouseSmall,
    "medium": ref_wh.WarehouseMedium,
    "large": ref_wh.WarehouseLarge,
}
OBS_KEYS = [
    "num_agents",
    "other_availabilities",
    "other_delivery_targets",
    "other_positions",
    "requests",
    "self_availability",
    "self_delivery_target",
    "self_position",
]


class DrawRecorder:
    """Pass-through wrappers around np.random.choice / randint that log what the env drew."""

    def __init__(self):
        self.log = []
        self._choice = np.random.choice
        self._randint = np.random.randint

    def __enter__(self):
        rec = self

        def choice(a, size=None, replace=True, p=None):
            out = rec._choice(a, size, replace, p)
            rec.log.append(("choice", np.array(a, copy=True), np.array(out, copy=True)))
            return out

        def randint(low, high=None, size=None, dtype=int):
            out = rec._randint(low, high, size, dtype)
            rec.log.append(("randint", low, high, out))
            return out

        np.random.choice = choice
        np.random.randint = randint
        return self

    def __exit__(self, *exc):
        np.random.choice = self._choice
        np.random.randint = self._randint
        return False

    def take(self):
        out, self.log = self.log, []
        return out


def canon_state(env):
    return dict(
        pos=np.array(env._agent_positions, dtype=np.int32).reshape(env._num_agents, 2),
        agent_tgt=np.array(env._agent_delivery_targets, dtype=np.int32),
        pk_tgt=np.array(env._pickup_point_targets, dtype=np.int32),
        pk_timer=np.array(env._pickup_point_timers, dtype=np.int32),
        t=np.int32(env._episode_time),
    )


def flat_obs(obs, n):
    rows = []
    for i in range(n):
        d = obs[str(i)]
        rows.append(np.concatenate([np.asarray(d[k]).ravel().astype(np.int32) for k in OBS_KEYS]))
    return np.stack(rows).astype(np.int16)


def reset_draws(log, R):
    """Split the reset-time draws into accepted spawns, the pickup choice and the target choice."""
    ints = [e for e in log if e[0] == "randint"]
    chs = [e for e in log if e[0] == "choice"]
    assert len(chs) == 2, chs
    pairs = [(int(ints[i][3]), int(ints[i + 1][3])) for i in range(0, len(ints), 2)]
    return pairs, chs[0][2].astype(np.int32), chs[1][2].astype(np.int32)


def step_draws(log, R):
    chs = [e for e in log if e[0] == "choice"]
    assert len(chs) == 2 and not [e for e in log if e[0] == "randint"], log
    inactive, sel = chs[0][1], chs[0][2]
    tg = chs[1][2]
    k = len(sel)
    # positions of the selected pickups inside the ascending inactive list
    posn = np.searchsorted(inactive, sel).astype(np.int32)
    assert np.array_equal(inactive[posn], sel)
    rpos = np.full(R, -1, np.int32)
    rtgt = np.full(R, -1, np.int32)
    rpos[:k] = posn
    rtgt[:k] = tg
    return len(inactive), k, rpos, rtgt, sel


def spawn_valid(env, pairs):
    pick = set()
    for x in env._pickup_racks_arrangement:
        for y in env._pickup_racks_arrangement:
            pick.update([(x - 1, y - 1), (x, y - 1), (x - 1, y), (x, y)])
    return [p for p in pairs if p not in pick]


def run_g1(variant, n, seed, steps=200, shuffle=False):
    cls = VARIANTS[variant]
    np.random.seed(seed)
    act_rng = np.random.RandomState(10_000 + 97 * seed + n)
    env = cls(n)
    R, P = env._num_requests, env._num_pickup_points
    with DrawRecorder() as rec:
        obs0 = env.reset()
        pairs, rsel, rtgt0 = reset_draws(rec.take(), R)
    spawn = np.array(spawn_valid(env, pairs), dtype=np.int32)
    assert spawn.shape == (n, 2)
    assert np.array_equal(spawn, env._agent_positions)
    out = {k: [] for k in ("actions", "order", "n_inactive", "k", "rpos", "rtgt", "rsel",
                           "pos", "agent_tgt", "pk_tgt", "pk_timer", "t", "obs", "rewards", "done")}
    s0 = canon_state(env)
    for s in range(steps):
        acts = act_rng.randint(0, 9, size=n).astype(np.int32)
        order = np.arange(n)
        if shuffle:
            order = act_rng.permutation(n)
            keep = act_rng.rand(n) > 0.15
            order = order[keep]
            neg = act_rng.rand(n) < 0.1
            acts = np.where(neg, acts - 9, acts).astype(np.int32)  # python-style wrap: -9..-1
        action_dict = {str(int(i)): int(acts[i]) for i in order}
        with DrawRecorder() as rec:
            obs, rew, dones, infos = env.step(action_dict)
            nin, k, rpos, rtgt, ssel = step_draws(rec.take(), R)
        ordv = np.full(n, -1, np.int32)
        ordv[: len(order)] = order
        st = canon_state(env)
        out["actions"].append(acts)
        out["order"].append(ordv)
        out["n_inactive"].append(nin)
        out["k"].append(k)
        out["rpos"].append(rpos)
        out["rtgt"].append(rtgt)
        sel = np.full(R, -1, np.int32)
        sel[:k] = ssel
        out["rsel"].append(sel)
        for key in ("pos", "agent_tgt", "pk_tgt", "pk_timer", "t"):
            out[key].append(st[key])
        out["obs"].append(flat_obs(obs, n))
        out["rewards"].append(np.array([rew[str(i)] for i in range(n)], np.float32))
        assert all(dones[str(i)] == dones["__all__"] for i in range(n))
        out["done"].append(bool(dones["__all__"]))
    arr = {k: np.stack([np.asarray(v) for v in vals]) for k, vals in out.items()}
    arr.update(
        variant=np.array(variant), n=np.int32(n), seed=np.int32(seed),
        spawn_pairs=np.array(pairs, np.int32), spawn=spawn, reset_sel=rsel, reset_tgt=rtgt0,
        reset_obs=flat_obs(obs0, n),
        **{"reset_" + k: v for k, v in s0.items()},
    )
    return arr


def run_keys(variant, n, seed, steps=200, long=False):
    """A G1 episode whose action dicts mix key forms: str(a), int a, str(a - n), int(a - n), so some
    dicts name an agent under two keys (both entries act).  Per step the dict's entries are recorded
    as key_form (0 str, 1 int, 2 negative str, 3 negative int; -1 = no entry), key_agent (the agent
    the key names) and key_act (the entry's action, -9..8).  long=True (`long_*` fixtures): dicts of
    up to 4n entries -- agents named under several, up to all four, key forms, so one agent moves
    several times in one step -- and every 10th dict holds all 4n keys."""
    cls = VARIANTS[variant]
    np.random.seed(seed)
    act_rng = np.random.RandomState(20_000 + 31 * seed + n + (7_777 if long else 0))
    width = 4 * n if long else n
    env = cls(n)
    R = env._num_requests
    with DrawRecorder() as rec:
        obs0 = env.reset()
        pairs, rsel, rtgt0 = reset_draws(rec.take(), R)
    spawn = np.array(spawn_valid(env, pairs), dtype=np.int32)
    assert np.array_equal(spawn, env._agent_positions)
    out = {k: [] for k in ("key_form", "key_agent", "key_act", "n_inactive", "k", "rpos", "rtgt", "rsel",
                           "pos", "agent_tgt", "pk_tgt", "pk_timer", "t", "obs", "rewards", "done")}
    s0 = canon_state(env)
    dup_steps = 0
    for s in range(steps):
        m = int(act_rng.randint(1, width + 1)) if not (long and s % 10 == 9) else 64 * width
        form = np.full(width, -1, np.int32)
        agent = np.full(width, -1, np.int32)
        act = np.zeros(width, np.int32)
        action_dict = {}
        for j in range(m):
            if len(action_dict) == width:
                break
            a, f, v = int(act_rng.randint(0, n)), int(act_rng.randint(0, 4)), int(act_rng.randint(-9, 9))
            key = [str(a), a, str(a - n), a - n][f]
            if key in action_dict:
                continue
            form[len(action_dict)], agent[len(action_dict)], act[len(action_dict)] = f, a, v
            action_dict[key] = v
        dup_steps += len({int(k) % n for k in action_dict}) < len(action_dict)
        with DrawRecorder() as rec:
            obs, rew, dones, infos = env.step(action_dict)
            nin, k, rpos, rtgt, ssel = step_draws(rec.take(), R)
        st = canon_state(env)
        out["key_form"].append(form)
        out["key_agent"].append(agent)
        out["key_act"].append(act)
        out["n_inactive"].append(nin)
        out["k"].append(k)
        out["rpos"].append(rpos)
        out["rtgt"].append(rtgt)
        sel = np.full(R, -1, np.int32)
        sel[:k] = ssel
        out["rsel"].append(sel)
        for key in ("pos", "agent_tgt", "pk_tgt", "pk_timer", "t"):
            out[key].append(st[key])
        out["obs"].append(flat_obs(obs, n))
        out["rewards"].append(np.array([rew[str(i)] for i in range(n)], np.float32))
        out["done"].append(bool(dones["__all__"]))
    assert dup_steps > 10, dup_steps
    arr = {k: np.stack([np.asarray(v) for v in vals]) for k, vals in out.items()}
    arr.update(
        variant=np.array(variant), n=np.int32(n), seed=np.int32(seed),
        spawn_pairs=np.array(pairs, np.int32), spawn=spawn, reset_sel=rsel, reset_tgt=rtgt0,
        reset_obs=flat_obs(obs0, n),
        **{"reset_" + k: v for k, v in s0.items()},
    )
    return arr


def dense_state(env, rng):
    """An adversarial pre-step state: agents crowded on a few cells near pickups/deliveries."""
    D, n = env._area_dimension, env._num_agents
    P, Dp, R, W = env._num_pickup_points, env._num_delivery_points, env._num_requests, env._pickup_wait_duration
    pk = env._pickup_point_positions
    dl = env._delivery_point_positions
    mode = rng.randint(4)
    if mode == 0:  # a 3x3 window somewhere
        cx, cy = rng.randint(0, D - 2, size=2)
        pos = np.stack([cx + rng.randint(0, 3, n), cy + rng.randint(0, 3, n)], 1)
    elif mode == 1:  # around a pickup block
        c = pk[rng.randint(P)]
        pos = np.clip(np.stack([c[0] + rng.randint(-1, 2, n), c[1] + rng.randint(-1, 2, n)], 1), 0, D - 1)
    elif mode == 2:  # hugging the border next to delivery points
        c = dl[rng.randint(Dp)]
        pos = np.clip(np.stack([c[0] + rng.randint(-1, 2, n), c[1] + rng.randint(-1, 2, n)], 1), 0, D - 1)
    else:  # anywhere, including corners
        pos = rng.randint(0, D, size=(n, 2))
    pos = pos.astype(np.int32)
    n_active = rng.randint(max(0, R - n), R + 1)
    tgt = np.full(P, -1, np.int32)
    tim = np.full(P, -1, np.int32)
    sel = rng.choice(P, n_active, replace=False)
    tgt[sel] = rng.randint(0, Dp, n_active)
    tim[sel] = np.where(rng.rand(n_active) < 0.3, 1, rng.randint(1, W + 1, n_active))
    atg = np.where(rng.rand(n) < 0.4, rng.randint(0, Dp, n), -1).astype(np.int32)
    # some carriers stand on / next to their own delivery cell
    for i in range(n):
        if atg[i] >= 0 and rng.rand() < 0.5:
            pos[i] = np.clip(dl[atg[i]] + rng.randint(-1, 2, 2), 0, D - 1)
    t = int(rng.choice([0, 5, env._episode_duration - 1, env._episode_duration, 150]))
    return pos, atg, tgt, tim, t


def run_g2(variant, count, seed):
    cls = VARIANTS[variant]
    rng = np.random.RandomState(seed)
    recs = {k: [] for k in ("n", "pre_pos", "pre_agent_tgt", "pre_pk_tgt", "pre_pk_timer", "pre_t",
                            "actions", "order", "n_inactive", "k", "rpos", "rtgt",
                            "pos", "agent_tgt", "pk_tgt", "pk_timer", "t", "obs", "rewards", "done")}
    nmax = cls.max_num_agents
    for c in range(count):
        n = int(rng.choice([1, 2, nmax, nmax, rng.randint(1, nmax + 1)]))
        env = cls(n)
        np.random.seed(seed * 1000 + c)
        env.reset()
        R, P = env._num_requests, env._num_pickup_points
        pos, atg, tgt, tim, t = dense_state(env, rng)
        env._agent_positions = pos.copy()
        env._agent_delivery_targets = atg.copy()
        env._pickup_point_targets = tgt.copy()
        env._pickup_point_timers = tim.copy()
        env._episode_time = t
        acts = rng.randint(0, 9, n).astype(np.int32)
        order = rng.permutation(n) if rng.rand() < 0.5 else np.arange(n)
        if rng.rand() < 0.2:
            order = order[rng.rand(n) > 0.3]
        with DrawRecorder() as rec:
            obs, rew, dones, _ = env.step({str(int(i)): int(acts[i]) for i in order})
            nin, k, rpos, rtgt, _ = step_draws(rec.take(), R)
        st = canon_state(env)
        pad = lambda a, fill, shape: np.concatenate([a, np.full((nmax - len(a),) + shape, fill, a.dtype)])  # noqa: E731
        ordv = np.full(nmax, -1, np.int32)
        ordv[: len(order)] = order
        recs["n"].append(n)
        recs["pre_pos"].append(pad(pos, 0, (2,)))
        recs["pre_agent_tgt"].append(pad(atg, -1, ()))
        recs["pre_pk_tgt"].append(tgt)
        recs["pre_pk_timer"].append(tim)
        recs["pre_t"].append(t)
        recs["actions"].append(pad(acts, 4, ()))
        recs["order"].append(ordv)
        recs["n_inactive"].append(nin)
        recs["k"].append(k)
        recs["rpos"].append(rpos)
        recs["rtgt"].append(rtgt)
        recs["pos"].append(pad(st["pos"], 0, (2,)))
        recs["agent_tgt"].append(pad(st["agent_tgt"], -1, ()))
        recs["pk_tgt"].append(st["pk_tgt"])
        recs["pk_timer"].append(st["pk_timer"])
        recs["t"].append(st["t"])
        ob = flat_obs(obs, n)
        recs["obs"].append(np.concatenate([ob, np.zeros((nmax - n, ob.shape[1]), ob.dtype)]))
        recs["rewards"].append(pad(np.array([rew[str(i)] for i in range(n)], np.float32), 0, ()))
        recs["done"].append(bool(dones["__all__"]))
    return {k: np.stack([np.asarray(v) for v in vals]) for k, vals in recs.items()}


def run_g3():
    """Greedy rollouts driven like baseline/run.py:35-62 (solver draws interleaved with env draws)."""
    cases = [("small", 2, 0.0, s) for s in range(5)] + [
        ("medium", 8, 0.0, 0), ("medium", 8, 0.0, 1), ("large", 16, 0.0, 0), ("large", 16, 0.0, 1),
        ("small", 4, 0.25, 7), ("medium", 5, 0.1, 3),
    ]
    out = {}
    for ci, (variant, n, p, seed) in enumerate(cases):
        np.random.seed(seed)
        env = VARIANTS[variant](n)
        solver = ref_solvers.WarehouseRandomGreedySolver(
            num_agents=env.num_agents, num_requests=env.num_requests,
            random_action_prob=p, action_space=env.action_space)
        obs = env.reset()
        acc = np.zeros(n, np.float64)
        actions, rewards = [], []
        done = False
        while not done:
            ad = solver.compute_action(obs)
            actions.append(np.array([int(ad[str(i)]) for i in range(n)], np.int32))
            obs, rew, dones, _ = env.step(ad)
            for _, o in obs.items():
                assert env.observation_space.contains(o)
            r = np.array([rew[str(i)] for i in range(n)], np.float32)
            rewards.append(r)
            acc += r
            done = dones["__all__"]
        pre = f"c{ci}_"
        out[pre + "meta"] = np.array([variant, str(n), repr(p), str(seed)])
        out[pre + "actions"] = np.stack(actions)
        out[pre + "rewards"] = np.stack(rewards)
        out[pre + "final_pos"] = np.array(env._agent_positions, np.int32)
        out[pre + "total"] = np.float64(acc.sum())
    # the exact line run.main prints for seed 0 (82.0 = 42.0 + 40.0)
    totals = []
    for s in range(3):
        np.random.seed(s)
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            ref_run.main("small", 2, 0.0, False)
        line = [ln for ln in buf.getvalue().splitlines() if ln.startswith("Total:")][-1]
        totals.append(float(line.split(",")[0].split(":")[1]))
    out["run_main_totals"] = np.array(totals)
    return out


def main_keys():
    for variant, n in (("small", 4), ("medium", 8), ("large", 16)):
        arr = run_keys(variant, n, 7)
        np.savez_compressed(os.path.join(HERE, f"keys_{variant}_n{n}_s7.npz"), **arr)
    print("wrote keys_* fixtures to", HERE)


def main_long():
    for variant, n in (("small", 4), ("medium", 8), ("large", 16)):
        arr = run_keys(variant, n, 9, long=True)
        np.savez_compressed(os.path.join(HERE, f"long_{variant}_n{n}_s9.npz"), **arr)
    print("wrote long_* fixtures to", HERE)


def main():
    os.makedirs(HERE, exist_ok=True)
    for variant, nmax in (("small", 4), ("medium", 9), ("large", 16)):
        for n in sorted({1, 2, nmax} | ({8} if variant == "medium" else set())):
            for seed in (0, 1):
                arr = run_g1(variant, n, seed)
                np.savez_compressed(os.path.join(HERE, f"g1_{variant}_n{n}_s{seed}.npz"), **arr)
        arr = run_g1(variant, nmax, 5, shuffle=True)
        np.savez_compressed(os.path.join(HERE, f"ord_{variant}_n{nmax}_s5.npz"), **arr)
        g2 = run_g2(variant, 400, {"small": 11, "medium": 12, "large": 13}[variant])
        np.savez_compressed(os.path.join(HERE, f"g2_{variant}.npz"), **g2)
    np.savez_compressed(os.path.join(HERE, "g3_greedy.npz"), **run_g3())
    print("wrote fixtures to", HERE)


if __name__ == "__main__":
    if sys.argv[1:] == ["keys"]:   # (added in round 4: only the keys_* fixtures)
        main_keys()
    elif sys.argv[1:] == ["long"]:   # (added in round 6: only the long_* fixtures)
        main_long()
    else:
        main()
        main_keys()
        main_long()
