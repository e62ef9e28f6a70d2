"""The vectorised oracle agrees with the reference fixtures env-by-env (so it can check the GPU at
B in the thousands), and its philox draw contract behaves as documented."""
import glob
import os

import numpy as np
import pytest

from oracle import batched as ob
from oracle import core as oc
from oracle import philox as ph

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def load_g1_batch(variant):
    paths = sorted(glob.glob(os.path.join(GOLDEN, f"g1_{variant}_*.npz"))
                   + glob.glob(os.path.join(GOLDEN, f"ord_{variant}_*.npz")))
    return [dict(np.load(p)) for p in paths]


def batch_inputs(runs, nmax, R):
    B = len(runs)
    spawn = np.zeros((B, nmax, 2), np.int32)
    n = np.array([int(g["n"]) for g in runs])
    for e, g in enumerate(runs):
        spawn[e, : n[e]] = g["spawn"]
    sel = np.stack([g["reset_sel"] for g in runs])
    tgt = np.stack([g["reset_tgt"] for g in runs])
    return B, n, spawn, sel, tgt


def step_inputs(runs, nmax, s):
    B = len(runs)
    acts = np.full((B, nmax), 4, np.int64)
    order = np.full((B, nmax), -1, np.int64)
    for e, g in enumerate(runs):
        n = int(g["n"])
        acts[e, :n] = np.mod(g["actions"][s], 9)  # host-side python-style wrap of -9..-1
        order[e, :n] = g["order"][s]
    rpos = np.stack([g["rpos"][s] for g in runs])
    rtgt = np.stack([g["rtgt"][s] for g in runs])
    return acts, order, rpos, rtgt


def check_env(L, S, e, g, s, obs, rew):
    n = int(g["n"])
    np.testing.assert_array_equal(S.pos[e, :n], g["pos"][s])
    np.testing.assert_array_equal(S.agent_tgt[e, :n], g["agent_tgt"][s])
    np.testing.assert_array_equal(S.pk_tgt[e], g["pk_tgt"][s])
    np.testing.assert_array_equal(S.pk_timer[e], g["pk_timer"][s])
    np.testing.assert_array_equal(obs[e, :n], g["obs"][s])
    assert not obs[e, n:].any()
    np.testing.assert_array_equal(rew[e, :n], g["rewards"][s])
    assert not rew[e, n:].any()


@pytest.mark.parametrize("variant", ["small", "medium", "large"])
def test_batched_matches_g1(variant):
    runs = load_g1_batch(variant)
    L = oc.layout_for(variant)
    nmax = oc.VARIANTS[variant]["nmax"]
    B, n, spawn, sel, tgt = batch_inputs(runs, nmax, L.R)
    S = ob.BState.zeros(L, B, nmax)
    ob.reset(L, S, ob.Injected(spawn=spawn, reset_sel=sel, reset_tgt=tgt, n=n))
    obs = ob.observe(L, S)
    for e, g in enumerate(runs):
        np.testing.assert_array_equal(obs[e, : int(g["n"])], g["reset_obs"])
    for s in range(200):
        acts, order, rpos, rtgt = step_inputs(runs, nmax, s)
        rew, done, n_in, k = ob.step(L, S, acts, ob.Injected(rpos=rpos, rtgt=rtgt), order=order)
        obs = ob.observe(L, S)
        for e, g in enumerate(runs):
            check_env(L, S, e, g, s, obs, rew)
            assert n_in[e] == g["n_inactive"][s] and k[e] == g["k"][s]
            assert done[e] == g["done"][s]


@pytest.mark.parametrize("variant", ["small", "medium", "large"])
def test_batched_matches_g2(variant):
    g = np.load(os.path.join(GOLDEN, f"g2_{variant}.npz"))
    L = oc.layout_for(variant)
    B = len(g["n"])
    nmax = g["pre_pos"].shape[1]
    S = ob.BState(pos=g["pre_pos"].copy(), agent_tgt=g["pre_agent_tgt"].copy(),
                  pk_tgt=g["pre_pk_tgt"].copy(), pk_timer=g["pre_pk_timer"].copy(),
                  t=g["pre_t"].astype(np.int64), n=g["n"].astype(np.int32),
                  fresh=np.zeros(B, bool), episode=np.zeros(B, np.uint32))
    rew, done, n_in, k = ob.step(L, S, g["actions"], ob.Injected(rpos=g["rpos"], rtgt=g["rtgt"]),
                                 order=g["order"])
    np.testing.assert_array_equal(S.pos, g["pos"])
    np.testing.assert_array_equal(S.agent_tgt, g["agent_tgt"])
    np.testing.assert_array_equal(S.pk_tgt, g["pk_tgt"])
    np.testing.assert_array_equal(S.pk_timer, g["pk_timer"])
    np.testing.assert_array_equal(rew, g["rewards"])
    np.testing.assert_array_equal(done, g["done"])
    np.testing.assert_array_equal(k, g["k"])
    np.testing.assert_array_equal(ob.observe(L, S), g["obs"])


def test_batched_greedy_matches_core_greedy():
    """Greedy on state == reference solver on the observation dicts (solvers.py:27-58)."""
    g = np.load(os.path.join(GOLDEN, "g3_greedy.npz"))
    for ci in (5, 7):   # medium-8, large-16, p = 0
        variant, n, p, seed = g[f"c{ci}_meta"]
        n, seed = int(n), int(seed)
        L = oc.layout_for(variant)
        np.random.seed(seed)
        env = oc.OracleWarehouse(variant, n)
        env.reset()
        for s in range(len(g[f"c{ci}_actions"])):
            st = env.state
            S = ob.BState(pos=st.pos[None].copy(), agent_tgt=st.agent_tgt[None].copy(),
                          pk_tgt=st.pk_tgt[None].copy(), pk_timer=st.pk_timer[None].copy(),
                          t=np.array([st.t]), n=np.array([n], np.int32), fresh=np.array([st.fresh]),
                          episode=np.zeros(1, np.uint32))
            acts = ob.greedy(L, S, 0.0)
            np.testing.assert_array_equal(acts[0], g[f"c{ci}_actions"][s])
            np.random.uniform(size=n)  # the solver's per-agent coins (solvers.py:44) precede env draws
            env.step({str(i): int(acts[0, i]) for i in range(n)})


def test_select_bit():
    rng = np.random.RandomState(0)
    masks = rng.randint(0, 2**62, size=200, dtype=np.int64).astype(np.uint64) | np.uint64(1 << 63)
    for m in masks[:50]:
        bits = [b for b in range(64) if (int(m) >> b) & 1]
        got = ph.select_bit(np.full(len(bits), m), np.arange(len(bits)))
        assert list(got) == bits


@pytest.mark.parametrize("variant", ["small", "medium", "large"])
def test_philox_mode_invariants_and_shard_invariance(variant):
    L = oc.layout_for(variant)
    nmax = oc.VARIANTS[variant]["nmax"]
    B = 64
    S = ob.BState.zeros(L, B, nmax)
    d = ob.PhiloxDraws(1234, np.arange(B))
    ob.reset(L, S, d, nmax=nmax)
    # two shards of the same env ids reproduce the same trajectory
    S1, S2 = ob.BState.zeros(L, B // 2, nmax), ob.BState.zeros(L, B // 2, nmax)
    d1, d2 = ob.PhiloxDraws(1234, np.arange(B // 2)), ob.PhiloxDraws(1234, np.arange(B // 2, B))
    ob.reset(L, S1, d1, nmax=nmax)
    ob.reset(L, S2, d2, nmax=nmax)
    _, _, cell, valid = ob.tables(L)
    for s in range(60):
        acts = ob.greedy(L, S, 0.2, d)
        a1, a2 = ob.greedy(L, S1, 0.2, d1), ob.greedy(L, S2, 0.2, d2)
        np.testing.assert_array_equal(np.concatenate([a1, a2]), acts)
        ob.step(L, S, acts, d)
        ob.step(L, S1, a1, d1)
        ob.step(L, S2, a2, d2)
        assert ((S.pk_tgt > -1).sum(1) == L.R).all()
        assert ((S.pk_tgt > -1) == (S.pk_timer > -1)).all()
        assert S.pos.min() >= 0 and S.pos.max() < L.D
    np.testing.assert_array_equal(np.concatenate([S1.pos, S2.pos]), S.pos)
    np.testing.assert_array_equal(np.concatenate([S1.pk_tgt, S2.pk_tgt]), S.pk_tgt)


def test_philox_reset_distribution():
    """Spawns are uniform over interior non-pickup cells (what the reference's rejection loop at
    core.py:191-201 produces), n is uniform on 1..nmax, reset requests are R distinct pickups."""
    L = oc.layout_for("medium")
    B = 20000
    S = ob.BState.zeros(L, B, 9)
    ob.reset(L, S, ob.PhiloxDraws(7, np.arange(B)), nmax=9)
    _, _, cell, valid = ob.tables(L)
    c = S.pos[:, 0, 0] * L.D + S.pos[:, 0, 1]
    assert (cell[c] < 0).all()
    counts = np.bincount(c, minlength=L.D * L.D)[valid[:, 0] * L.D + valid[:, 1]]
    exp = B / len(valid)
    chi2 = ((counts - exp) ** 2 / exp).sum()
    assert chi2 < len(valid) + 6 * np.sqrt(2 * len(valid))
    nc = np.bincount(S.n, minlength=10)[1:]
    assert (np.abs(nc - B / 9) < 6 * np.sqrt(B / 9)).all()
    assert ((S.pk_tgt > -1).sum(1) == L.R).all()


def test_philox_reset_subset_and_pairing_law():
    """The philox reset's request law (Floyd subset + ordered targets) equals the reference's
    choice(P, R, replace=False) paired with choice(Dp, R, replace=False): every R-subset of pickup
    points equally likely, and the lowest open point's target uniform over the delivery points."""
    from math import comb

    from scipy import stats

    L = oc.layout_for("small")
    B = 60000
    S = ob.BState.zeros(L, B, 4)
    ob.reset(L, S, ob.PhiloxDraws(11, np.arange(B)))
    open_ = S.pk_tgt > -1
    assert (open_.sum(1) == L.R).all()
    code = (open_.astype(np.int64) << np.arange(L.P)).sum(1)
    counts = np.unique(code, return_counts=True)[1]
    assert len(counts) == comb(L.P, L.R)
    exp = B / comb(L.P, L.R)
    assert stats.chi2.sf(((counts - exp) ** 2 / exp).sum(), len(counts) - 1) > 1e-6
    first = S.pk_tgt[np.arange(B), open_.argmax(1)]
    c = np.bincount(first, minlength=L.Dp)
    assert stats.chi2.sf(((c - B / L.Dp) ** 2 / (B / L.Dp)).sum(), L.Dp - 1) > 1e-6
