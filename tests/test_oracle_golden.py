"""Pin the CPU oracle to fixtures produced by the reference itself (tests/golden/make_golden.py)."""
import glob
import os

import numpy as np
import pytest

from oracle import core as oc

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
G1 = sorted(glob.glob(os.path.join(GOLDEN, "g1_*.npz")) + glob.glob(os.path.join(GOLDEN, "ord_*.npz")))


def _order(row):
    return [int(i) for i in row if i >= 0]


@pytest.mark.parametrize("path", G1, ids=[os.path.basename(p) for p in G1])
@pytest.mark.parametrize("mode", ["injected", "global_mt19937"])
def test_g1_trajectory(path, mode):
    g = np.load(path)
    L = oc.layout_for(str(g["variant"]))
    n = int(g["n"])
    if mode == "injected":
        regen = [(g["rpos"][s], g["rtgt"][s]) for s in range(len(g["t"]))]
        draws = oc.InjectedDraws(spawn=g["spawn"], reset_sel=g["reset_sel"], reset_tgt=g["reset_tgt"],
                                 regen=regen)
    else:
        np.random.seed(int(g["seed"]))
        draws = oc.GlobalNumpyDraws()
    st = oc.reset(L, n, draws)
    np.testing.assert_array_equal(st.pos, g["reset_pos"])
    np.testing.assert_array_equal(st.pk_tgt, g["reset_pk_tgt"])
    np.testing.assert_array_equal(st.pk_timer, g["reset_pk_timer"])
    np.testing.assert_array_equal(oc.observe(L, st), g["reset_obs"])
    for s in range(len(g["t"])):
        res = oc.step(L, st, g["actions"][s], _order(g["order"][s]), draws)
        assert res.n_inactive == g["n_inactive"][s] and res.k == g["k"][s]
        np.testing.assert_array_equal(st.pos, g["pos"][s])
        np.testing.assert_array_equal(st.agent_tgt, g["agent_tgt"][s])
        np.testing.assert_array_equal(st.pk_tgt, g["pk_tgt"][s])
        np.testing.assert_array_equal(st.pk_timer, g["pk_timer"][s])
        assert st.t == g["t"][s] and res.done == bool(g["done"][s])
        np.testing.assert_array_equal(res.rewards, g["rewards"][s])
        np.testing.assert_array_equal(oc.observe(L, st), g["obs"][s])


KEYS = sorted(glob.glob(os.path.join(GOLDEN, "keys_*.npz")))


@pytest.mark.parametrize("path", KEYS, ids=[os.path.basename(p) for p in KEYS])
@pytest.mark.parametrize("mode", ["injected", "global_mt19937"])
def test_keys_trajectory(path, mode):
    """keys_*: dicts keyed by int, negative (numpy wrap) and repeated agents, through the oracle's
    dict-taking step (OracleWarehouse.step, as core.py:279-281 reads the dict) and through the
    batched oracle with the C ABI's encoded order entries (agent | (action + 1) << 8)."""
    from keyforms import encoded_order, key_dict
    from oracle import batched as ob

    g = np.load(path)
    L = oc.layout_for(str(g["variant"]))
    n = int(g["n"])
    steps = len(g["t"])
    if mode == "injected":
        draws = oc.InjectedDraws(spawn=g["spawn"], reset_sel=g["reset_sel"], reset_tgt=g["reset_tgt"],
                                 regen=[(g["rpos"][s], g["rtgt"][s]) for s in range(steps)])
    else:
        np.random.seed(int(g["seed"]))
        draws = oc.GlobalNumpyDraws()
    env = oc.OracleWarehouse(str(g["variant"]), n, draws=draws)
    env.reset()
    dicts = [key_dict(g["key_form"][s], g["key_agent"][s], g["key_act"][s], n) for s in range(steps)]
    assert sum(len({int(k) % n for k in d}) < len(d) for d in dicts) > 10      # repeated agents
    assert sum(any(int(k) < 0 for k in d) for d in dicts) > 10                 # negative keys
    for s in range(steps):
        pre_pos = env.state.pos.copy()
        _, rew, dones, _ = env.step(dicts[s])
        st = env.state
        np.testing.assert_array_equal(st.pos, g["pos"][s], err_msg=f"step {s}")
        np.testing.assert_array_equal(st.pk_tgt, g["pk_tgt"][s])
        assert [rew[str(i)] for i in range(n)] == list(g["rewards"][s])
        np.testing.assert_array_equal(oc.observe(L, st), g["obs"][s])
        # the move phase alone through the batched oracle's encoded order entries
        pos = pre_pos[None].copy()
        S = ob.BState.zeros(L, 1, n)
        S.pos[:] = pos
        S.n[:] = n
        order = np.array([encoded_order(dicts[s], n, n)], np.int32)
        ob_pos = _batched_moves(L, S, order)
        np.testing.assert_array_equal(ob_pos[0], g["pos"][s], err_msg=f"batched moves, step {s}")


def _batched_moves(L, S, order):
    """Positions after the batched oracle's move phase (the rest of its step is irrelevant here)."""
    from oracle import batched as ob

    ob.step(L, S, np.full((S.B, S.NA), 4, np.int32), ob.PhiloxDraws(0, np.arange(S.B)), order=order)
    return S.pos


@pytest.mark.parametrize("variant", ["small", "medium", "large"])
def test_g2_dense_transitions(variant):
    g = np.load(os.path.join(GOLDEN, f"g2_{variant}.npz"))
    L = oc.layout_for(variant)
    for c in range(len(g["n"])):
        n = int(g["n"][c])
        st = oc.State(pos=g["pre_pos"][c][:n].copy(), agent_tgt=g["pre_agent_tgt"][c][:n].copy(),
                      pk_tgt=g["pre_pk_tgt"][c].copy(), pk_timer=g["pre_pk_timer"][c].copy(),
                      t=int(g["pre_t"][c]), fresh=False)
        draws = oc.InjectedDraws(regen=[(g["rpos"][c], g["rtgt"][c])])
        res = oc.step(L, st, g["actions"][c][:n], _order(g["order"][c]), draws)
        assert res.k == g["k"][c] and res.n_inactive == g["n_inactive"][c]
        np.testing.assert_array_equal(st.pos, g["pos"][c][:n])
        np.testing.assert_array_equal(st.agent_tgt, g["agent_tgt"][c][:n])
        np.testing.assert_array_equal(st.pk_tgt, g["pk_tgt"][c])
        np.testing.assert_array_equal(st.pk_timer, g["pk_timer"][c])
        np.testing.assert_array_equal(res.rewards, g["rewards"][c][:n])
        assert res.done == bool(g["done"][c])
        np.testing.assert_array_equal(oc.observe(L, st), g["obs"][c][:n])


def test_g3_greedy_rollouts_global_stream():
    """Solver coins interleaved with env draws on the global stream (baseline/run.py:42-62)."""
    g = np.load(os.path.join(GOLDEN, "g3_greedy.npz"))
    assert list(g["run_main_totals"]) == [82.0, 49.0, 7.0]
    ci = 0
    while f"c{ci}_meta" in g:
        variant, n, p, seed = g[f"c{ci}_meta"]
        n, p, seed = int(n), float(p), int(seed)
        np.random.seed(seed)
        env = oc.OracleWarehouse(variant, n)
        obs = env.reset()
        total = 0.0
        for s in range(len(g[f"c{ci}_actions"])):
            flat = np.stack([np.concatenate([np.asarray(obs[str(i)][k]).ravel() for k in oc.OBS_KEYS])
                             for i in range(n)])
            acts = oc.greedy(env.layout, flat, p, env.draws)
            np.testing.assert_array_equal(acts, g[f"c{ci}_actions"][s])
            obs, rew, dones, _ = env.step({str(i): int(acts[i]) for i in range(n)})
            total += sum(float(rew[str(i)]) for i in range(n))
        assert dones["__all__"]
        assert total == float(g[f"c{ci}_total"])
        np.testing.assert_array_equal(env.state.pos, g[f"c{ci}_final_pos"])
        ci += 1
    assert ci == 11
