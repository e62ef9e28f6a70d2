"""GPU parity: the HIP kernels (through the C ABI) against the reference fixtures and the oracle.

Bar: bit-exact for every integer state field, assignment, observation value and done flag; rewards
are sums of 1.0f terms and must match exactly too (tolerance 0, tighter than north_star's 1e-6).
"""
import glob
import os

import numpy as np
import pytest

from oracle import batched as ob
from oracle import core as oc

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def wh():
    import torch

    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    import warehouse

    return warehouse


def canon(env):
    c = env.to_canonical()
    return {k: v.cpu().numpy() for k, v in c.items()}


def g1_runs(variant):
    paths = sorted(glob.glob(os.path.join(GOLDEN, f"g1_{variant}_*.npz"))
                   + glob.glob(os.path.join(GOLDEN, f"ord_{variant}_*.npz")))
    return [dict(np.load(p)) for p in paths]


@pytest.mark.parametrize("variant", ["small", "medium", "large"])
@pytest.mark.parametrize("ordered", [True, False])
def test_g1_episodes_injected(wh, variant, ordered):
    """Whole 200-step reference episodes, all (variant, N, seed) runs batched as B envs."""
    runs = g1_runs(variant)
    if not ordered:
        runs = [g for g in runs if np.all(g["order"] == np.arange(int(g["n"])))]
    nmax = oc.VARIANTS[variant]["nmax"]
    L = oc.layout_for(variant)
    B = len(runs)
    n = np.array([int(g["n"]) for g in runs], np.int32)
    spawn = np.zeros((B, nmax, 2), np.int32)
    for e, g in enumerate(runs):
        spawn[e, : n[e]] = g["spawn"]
    env = wh.BatchedWarehouse(variant, B, train=True)
    env.reset(draws=dict(spawn=spawn, pickups=np.stack([g["reset_sel"] for g in runs]),
                         targets=np.stack([g["reset_tgt"] for g in runs]), n=n))
    obs = env.observe().cpu().numpy()
    for e, g in enumerate(runs):
        np.testing.assert_array_equal(obs[e, : n[e]], g["reset_obs"])
        assert not obs[e, n[e]:].any()
    for s in range(200):
        acts = np.full((B, nmax), 4, np.int32)
        order = np.full((B, nmax), -1, np.int32)
        for e, g in enumerate(runs):
            acts[e, : n[e]] = np.mod(g["actions"][s], 9)
            order[e, : n[e]] = g["order"][s]
        regen = np.concatenate([np.stack([g["rpos"][s] for g in runs]),
                                np.stack([g["rtgt"][s] for g in runs])], axis=1)
        rew, done = env.step(acts, order=order if ordered else None, regen=regen)
        rew, done = rew.cpu().numpy(), done.cpu().numpy()
        c = canon(env)
        obs = env.observe().cpu().numpy()
        for e, g in enumerate(runs):
            k = n[e]
            np.testing.assert_array_equal(c["pos"][e, :k], g["pos"][s], err_msg=f"env {e} step {s}")
            np.testing.assert_array_equal(c["agent_target"][e, :k], g["agent_tgt"][s])
            np.testing.assert_array_equal(c["pickup_target"][e], g["pk_tgt"][s])
            np.testing.assert_array_equal(c["pickup_timer"][e], g["pk_timer"][s])
            assert c["t"][e] == g["t"][s]
            np.testing.assert_array_equal(rew[e, :k], g["rewards"][s])
            assert bool(done[e]) == bool(g["done"][s])
            np.testing.assert_array_equal(obs[e, :k], g["obs"][s])


@pytest.mark.parametrize("variant", ["small", "medium", "large"])
def test_g2_dense_transitions(wh, variant):
    g = np.load(os.path.join(GOLDEN, f"g2_{variant}.npz"))
    B = len(g["n"])
    env = wh.BatchedWarehouse(variant, B, train=True)
    env.from_canonical(dict(pos=g["pre_pos"], agent_target=g["pre_agent_tgt"], pickup_target=g["pre_pk_tgt"],
                            pickup_timer=g["pre_pk_timer"], t=g["pre_t"], n=g["n"]))
    regen = np.concatenate([g["rpos"], g["rtgt"]], axis=1)
    rew, done = env.step(g["actions"], order=g["order"], regen=regen)
    c = canon(env)
    np.testing.assert_array_equal(c["pos"], g["pos"])
    np.testing.assert_array_equal(c["agent_target"], g["agent_tgt"])
    np.testing.assert_array_equal(c["pickup_target"], g["pk_tgt"])
    np.testing.assert_array_equal(c["pickup_timer"], g["pk_timer"])
    np.testing.assert_array_equal(rew.cpu().numpy(), g["rewards"])
    np.testing.assert_array_equal(done.cpu().numpy().astype(bool), g["done"])
    np.testing.assert_array_equal(env.observe().cpu().numpy(), g["obs"])


def test_pack_unpack_roundtrip(wh):
    g = np.load(os.path.join(GOLDEN, "g2_large.npz"))
    env = wh.BatchedWarehouse("large", len(g["n"]), train=True)
    src = dict(pos=g["pos"], agent_target=g["agent_tgt"], pickup_target=g["pk_tgt"],
               pickup_timer=g["pk_timer"], t=g["t"], n=g["n"])
    env.from_canonical(src)
    c = canon(env)
    for k in ("pos", "agent_target", "pickup_target", "pickup_timer", "t", "n"):
        np.testing.assert_array_equal(c[k], src[k] if k != "t" else g["t"])


def oracle_state(c, L):
    return ob.BState(pos=c["pos"].copy(), agent_tgt=c["agent_target"].copy(), pk_tgt=c["pickup_target"].copy(),
                     pk_timer=c["pickup_timer"].copy(), t=c["t"].astype(np.int64), n=c["n"].copy(),
                     fresh=c["fresh"].astype(bool), episode=c["episode"].astype(np.uint32))


def assert_same(c, S, msg=""):
    np.testing.assert_array_equal(c["pos"], S.pos, err_msg=msg)
    np.testing.assert_array_equal(c["agent_target"], S.agent_tgt, err_msg=msg)
    np.testing.assert_array_equal(c["pickup_target"], S.pk_tgt, err_msg=msg)
    np.testing.assert_array_equal(c["pickup_timer"], S.pk_timer, err_msg=msg)
    np.testing.assert_array_equal(c["t"], S.t, err_msg=msg)
    np.testing.assert_array_equal(c["n"], S.n, err_msg=msg)
    np.testing.assert_array_equal(c["fresh"].astype(bool), S.fresh, err_msg=msg)
    np.testing.assert_array_equal(c["episode"].astype(np.uint32), S.episode, err_msg=msg)


def test_c2_small_random_actions_philox(wh):
    """Config 2: B=4096 Small envs x 4 agents, random actions, step kernel vs oracle, 210 steps
    (crosses the t=T boundary; no auto-reset in wh_step)."""
    B, seed = 4096, 99
    L = oc.layout_for("small")
    env = wh.BatchedWarehouse("small", B, 4, seed=seed)
    env.reset()
    S = ob.BState.zeros(L, B, 4)
    d = ob.PhiloxDraws(seed, np.arange(B))
    ob.reset(L, S, d, n_fixed=4)
    assert_same(canon(env), S, "reset")
    rng = np.random.RandomState(0)
    for s in range(210):
        acts = rng.randint(0, 9, size=(B, 4)).astype(np.int32)
        rew, done = env.step(acts)
        orew, odone, _, _ = ob.step(L, S, acts, d)
        np.testing.assert_array_equal(rew.cpu().numpy(), orew)
        np.testing.assert_array_equal(done.cpu().numpy().astype(bool), odone)
        if s % 10 == 0 or s > 195:
            assert_same(canon(env), S, f"step {s}")
            np.testing.assert_array_equal(env.observe().cpu().numpy(), ob.observe(L, S))


@pytest.mark.parametrize("variant,na,train,p", [("medium", 8, False, 0.0), ("large", 16, False, 0.0),
                                                ("medium", 9, True, 0.3), ("small", 4, True, 0.1)])
def test_policy_step_and_autoreset_vs_oracle(wh, variant, na, train, p):
    """wh_policy + wh_step + masked wh_reset, against the oracle with the philox contract."""
    B, seed = 2048, 7
    L = oc.layout_for(variant)
    env = wh.BatchedWarehouse(variant, B, na, train=train, seed=seed)
    env.reset()
    S = ob.BState.zeros(L, B, na)
    d = ob.PhiloxDraws(seed, np.arange(B))
    ob.reset(L, S, d, nmax=na if train else None)
    for s in range(230):
        a = env.policy("greedy", p).cpu().numpy()
        oa = ob.greedy(L, S, p, d)
        np.testing.assert_array_equal(a, oa, err_msg=f"step {s}")
        rew, done = env.step(a)
        orew, odone, _, _ = ob.step(L, S, oa, d)
        np.testing.assert_array_equal(rew.cpu().numpy(), orew)
        dn = done.cpu().numpy().astype(bool)
        np.testing.assert_array_equal(dn, odone)
        if dn.any():
            env.reset(mask=dn)
            ob.reset(L, S, d, mask=dn, nmax=na if train else None)
        if s % 25 == 0:
            assert_same(canon(env), S, f"step {s}")
    assert_same(canon(env), S, "end")


@pytest.mark.parametrize("variant,na,policy,p", [("medium", 8, "greedy", 0.0), ("large", 16, "greedy", 0.05),
                                                  ("small", 4, "random", 0.0)])
def test_fused_rollout_equals_stepwise(wh, variant, na, policy, p):
    """wh_rollout (K steps in one launch, auto-reset) == policy/step/reset launches == oracle."""
    import torch

    B, seed, K = 1024, 3, 230
    L = oc.layout_for(variant)
    a = wh.BatchedWarehouse(variant, B, na, seed=seed)
    a.reset()
    rew = torch.zeros((K, B, na), device=a.device)
    dn = torch.zeros((K, B), dtype=torch.uint8, device=a.device)
    ret = torch.zeros(B, device=a.device)
    a.rollout(K, policy, p, rewards=rew, dones=dn, returns=ret)
    S = ob.BState.zeros(L, B, na)
    d = ob.PhiloxDraws(seed, np.arange(B))
    ob.reset(L, S, d)
    tot = np.zeros(B, np.float32)
    for s in range(K):
        acts = ob.greedy(L, S, p, d) if policy == "greedy" else ob.random_actions(S, d)
        orew, odone, _, _ = ob.step(L, S, acts, d)
        np.testing.assert_array_equal(rew[s].cpu().numpy(), orew, err_msg=f"step {s}")
        np.testing.assert_array_equal(dn[s].cpu().numpy().astype(bool), odone)
        tot += orew.sum(1)
        if odone.any():
            ob.reset(L, S, d, mask=odone)
    assert_same(canon(a), S, "after rollout")
    np.testing.assert_allclose(ret.cpu().numpy(), tot, rtol=0, atol=0)


def test_c3_full_size_shard_invariance_and_spot_check(wh):
    """Config 3 size (B=65536 Medium x 8, greedy, fused): 2 shards == 1 batch bit-exactly; a sampled
    subset of env ids equals the oracle; request/timer invariants hold for every env."""
    import torch

    B, seed, K = 65536, 11, 40
    L = oc.layout_for("medium")
    full = wh.BatchedWarehouse("medium", B, 8, seed=seed)
    full.reset()
    full.rollout(K, "greedy", 0.0)
    halves = []
    for h in range(2):
        e = wh.BatchedWarehouse("medium", B // 2, 8, seed=seed, env_offset=h * (B // 2))
        e.reset()
        e.rollout(K, "greedy", 0.0)
        halves.append(e.state)
    torch.testing.assert_close(torch.cat(halves, dim=1), full.state, rtol=0, atol=0)
    c = canon(full)
    active = c["pickup_target"] >= 0
    assert (active.sum(1) == L.R).all()
    assert ((c["pickup_timer"] >= 0) == active).all()
    assert c["pos"].min() >= 0 and c["pos"].max() < L.D
    ids = np.random.RandomState(5).choice(B, 256, replace=False)
    S = ob.BState.zeros(L, len(ids), 8)
    d = ob.PhiloxDraws(seed, ids)
    ob.reset(L, S, d)
    for _ in range(K):
        ob.step(L, S, ob.greedy(L, S, 0.0, d), d)
    sub = {k: v[ids] for k, v in c.items()}
    assert_same(sub, S, "subset")
    np.testing.assert_array_equal(full.observe().cpu().numpy()[ids], ob.observe(L, S))


def test_c4_full_size_shard_invariance_and_spot_check(wh):
    """Config 4 size (B=65536 Large x 16 agents, greedy, fused fast instance: the dense collision and
    assignment path): 200 steps across an episode end; two shards of 32,768 == one batch
    bit-exactly (rewards every step and the final state); a sampled subset of env ids equals the
    oracle step by step; request/timer invariants hold for every env."""
    import torch

    B, seed, K = 65536, 19, 210
    L = oc.layout_for("large")
    full = wh.BatchedWarehouse("large", B, 16, seed=seed)
    full.reset()
    full.rollout(185, "greedy", 0.0)                 # untimed prefix: the window below crosses t = T
    rew = torch.zeros((K - 185, B, 16), device=full.device)
    dn = torch.zeros((K - 185, B), dtype=torch.uint8, device=full.device)
    full.rollout(K - 185, "greedy", 0.0, rewards=rew, dones=dn)
    assert int(dn.sum()) == B                         # every env ended its episode in the window
    for h in range(2):
        e = wh.BatchedWarehouse("large", B // 2, 16, seed=seed, env_offset=h * (B // 2))
        e.reset()
        e.rollout(185, "greedy", 0.0)
        r = torch.zeros((K - 185, B // 2, 16), device=e.device)
        d = torch.zeros((K - 185, B // 2), dtype=torch.uint8, device=e.device)
        e.rollout(K - 185, "greedy", 0.0, rewards=r, dones=d)
        sl = slice(h * (B // 2), (h + 1) * (B // 2))
        torch.testing.assert_close(e.state, full.state[:, sl], rtol=0, atol=0)
        assert torch.equal(r, rew[:, sl]) and torch.equal(d, dn[:, sl])
        del e, r, d
    c = canon(full)
    active = c["pickup_target"] >= 0
    assert (active.sum(1) == L.R).all()
    assert ((c["pickup_timer"] >= 0) == active).all()
    assert c["pos"].min() >= 0 and c["pos"].max() < L.D
    ids = np.concatenate([np.random.RandomState(6).choice(B - 64, 192, replace=False), np.arange(B - 64, B)])
    S = ob.BState.zeros(L, len(ids), 16)
    d = ob.PhiloxDraws(seed, ids)
    ob.reset(L, S, d)
    rw = rew.cpu().numpy()
    for s in range(K):
        orew, odone, _, _ = ob.step(L, S, ob.greedy(L, S, 0.0, d), d)
        if s >= 185:
            np.testing.assert_array_equal(rw[s - 185][ids], orew, err_msg=f"step {s}")
        if odone.any():
            ob.reset(L, S, d, mask=odone)
    assert_same({k: v[ids] for k, v in c.items()}, S, "subset")
    np.testing.assert_array_equal(full.observe().cpu().numpy()[ids], ob.observe(L, S))


def test_dropin_single_env_matches_reference_greedy_runs(wh):
    """Config 1 through the drop-in class on the GPU: baseline/run.py's loop, the reference solver
    (restated in oracle.core.greedy on the obs dicts), global numpy stream -> seed 0 gives 82.0."""
    g = np.load(os.path.join(GOLDEN, "g3_greedy.npz"))
    for ci in range(11):
        variant, n, p, seed = g[f"c{ci}_meta"]
        n, p, seed = int(n), float(p), int(seed)
        cls = {"small": wh.WarehouseSmall, "medium": wh.WarehouseMedium, "large": wh.WarehouseLarge}[variant]
        np.random.seed(seed)
        env = cls(n)
        L = oc.layout_for(variant)
        obs = env.reset()
        for o in obs.values():
            assert env.observation_space.contains(o)
        draws = oc.GlobalNumpyDraws()
        total, steps, done = 0.0, 0, False
        while not done:
            flat = np.stack([np.concatenate([np.asarray(obs[str(i)][k]).ravel() for k in oc.OBS_KEYS])
                             for i in range(n)])
            acts = oc.greedy(L, flat, p, draws)
            np.testing.assert_array_equal(acts, g[f"c{ci}_actions"][steps])
            obs, rew, dones, infos = env.step({str(i): int(acts[i]) for i in range(n)})
            for o in obs.values():
                assert env.observation_space.contains(o)
            total += sum(float(rew[str(i)]) for i in range(n))
            done = dones["__all__"]
            steps += 1
        assert steps == 200 and total == float(g[f"c{ci}_total"])
    assert float(g["c0_total"]) == 82.0


def test_dropin_dict_order_negative_actions(wh):
    """ord_* fixtures: shuffled/partial action dicts and negative actions via the drop-in class."""
    g = np.load(os.path.join(GOLDEN, "ord_medium_n9_s5.npz"))
    np.random.seed(int(g["seed"]))
    env = wh.WarehouseMedium(9)
    obs = env.reset()
    for s in range(200):
        order = [int(i) for i in g["order"][s] if i >= 0]
        obs, rew, dones, _ = env.step({str(i): int(g["actions"][s][i]) for i in order})
        flat = np.stack([np.concatenate([np.asarray(obs[str(i)][k]).ravel() for k in oc.OBS_KEYS])
                         for i in range(9)])
        np.testing.assert_array_equal(flat, g["obs"][s])
        np.testing.assert_array_equal(np.array([rew[str(i)] for i in range(9)]), g["rewards"][s])
    with pytest.raises(IndexError):
        env.step({"0": 9})


@pytest.mark.parametrize("variant,n", [("small", 4), ("medium", 8), ("large", 16)])
def test_dropin_key_forms_match_reference(wh, variant, n):
    """keys_* fixtures (the reference run with int keys, negative keys and one agent named under
    two keys in a dict, core.py:279-281): the drop-in class, global numpy stream, equals the
    reference's observations, rewards and dones at every step."""
    from keyforms import key_dict

    g = np.load(os.path.join(GOLDEN, f"keys_{variant}_n{n}_s7.npz"))
    np.random.seed(int(g["seed"]))
    env = {"small": wh.WarehouseSmall, "medium": wh.WarehouseMedium, "large": wh.WarehouseLarge}[variant](n)
    env.reset()
    dup = 0
    for s in range(len(g["t"])):
        d = key_dict(g["key_form"][s], g["key_agent"][s], g["key_act"][s], n)
        dup += len({int(k) % n for k in d}) < len(d)
        obs, rew, dones, _ = env.step(d)
        flat = np.stack([np.concatenate([np.asarray(obs[str(i)][k]).ravel() for k in oc.OBS_KEYS])
                         for i in range(n)])
        np.testing.assert_array_equal(flat, g["obs"][s], err_msg=f"step {s}")
        np.testing.assert_array_equal(np.array([rew[str(i)] for i in range(n)]), g["rewards"][s])
        assert dones["__all__"] == bool(g["done"][s])
    assert dup > 10
    with pytest.raises(IndexError):
        env.step({str(-n - 1): 0})
    with pytest.raises(IndexError):
        env.step({str(n): 0})
    # up to 4n entries (every agent under its four key forms) run; a fifth spelling of a number
    # ('00': int() accepts it) is past the documented limit and raises ValueError
    full = {k: 4 for i in range(n) for k in (str(i), i, str(i - n), i - n)}
    env.step(full)
    full["00"] = 4
    with pytest.raises(ValueError):
        env.step(full)


def test_dropin_train_variant_matches_oracle(wh):
    """Train variants re-draw N from the global stream at construction and every reset."""
    def run(make):
        np.random.seed(3)
        env = make()
        trace = []
        for ep in range(3):
            obs = env.reset()
            trace.append((env.num_agents, obs, None))
            for s in range(30):
                rs = np.random.RandomState(100 * ep + s)
                acts = {str(i): int(rs.randint(9)) for i in range(env.num_agents)}
                obs, rew, dones, _ = env.step(acts)
                trace.append((env.num_agents, obs, rew))
        return trace

    got = run(wh.WarehouseLargeTrain)
    exp = run(lambda: oc.OracleWarehouse("large", 0, train=True))
    assert len(got) == len(exp)
    for (n1, o1, r1), (n2, o2, r2) in zip(got, exp):
        assert n1 == n2
        for i in range(n1):
            for k in oc.OBS_KEYS:
                np.testing.assert_array_equal(o1[str(i)][k], o2[str(i)][k])
            if r1 is not None:
                assert r1[str(i)] == r2[str(i)]


def test_edge_empty_batch_and_bad_config(wh):
    from warehouse import _native as nat

    e = wh.BatchedWarehouse("small", 0, 4)
    e.reset()
    e.step(np.zeros((0, 4), np.int32))
    with pytest.raises(ValueError):
        nat.query(nat.make_config(12, 4, (4, 8), 5, 200, 200))   # agents > requests
    with pytest.raises(ValueError):
        nat.query(nat.make_config(12, 4, (4, 8), 2, 200, 300))   # W > 255 not representable


def test_c5_eight_shards_equal_one_batch_of_524288(wh):
    """Config 5 on one GPU: B = 524,288 Medium x 8 envs as ONE batch equals the 8 per-GPU shards of
    65,536 (env_offset = rank * B) that bench.py runs on an 8-GPU node -- bit-exact state,
    rewards and observation rows; plus request/timer invariants over all 524,288 envs."""
    import torch

    B, G, seed, K = 524288, 8, 5, 30
    L = oc.layout_for("medium")
    full = wh.BatchedWarehouse("medium", B, 8, seed=seed)
    full.reset()
    rew = torch.zeros((K, B, 8), device=full.device)
    full.rollout(K, "greedy", 0.0, rewards=rew)
    for g in range(G):
        sh = wh.BatchedWarehouse("medium", B // G, 8, seed=seed, env_offset=g * (B // G))
        sh.reset()
        r = torch.zeros((K, B // G, 8), device=sh.device)
        sh.rollout(K, "greedy", 0.0, rewards=r)
        sl = slice(g * (B // G), (g + 1) * (B // G))
        torch.testing.assert_close(sh.state, full.state[:, sl], rtol=0, atol=0)
        torch.testing.assert_close(r, rew[:, sl], rtol=0, atol=0)
        if g == G - 1:
            torch.testing.assert_close(sh.observe(), full.observe()[sl], rtol=0, atol=0)
        del sh, r
    c = canon(full)
    active = c["pickup_target"] >= 0
    assert (active.sum(1) == L.R).all()
    assert ((c["pickup_timer"] >= 0) == active).all()
    assert c["pos"].min() >= 0 and c["pos"].max() < L.D
    assert float(rew.sum()) > 0


def test_dropin_render_headless(wh):
    """Rendering (core.py:444-617) from a host copy of the device state: the text
    frame puts every agent on its cell and every open request on its pickup point; animate=True
    yields animate_frames_per_step RGB frames from the previous cells (core.py:270-272, 449-469)."""
    np.random.seed(3)
    env = wh.WarehouseSmall(2)
    env.reset()
    D = 12
    txt = env.render(mode="ansi")
    rows = txt.split("\n")
    assert len(rows) == D and all(len(r) == D for r in rows)
    snap = env._snapshot()
    for i, (x, y) in enumerate(snap["pos"]):
        assert rows[D - 1 - y][x] in (chr(ord("a") + i), "*")
    covered = {tuple(p) for p in snap["pos"]}
    from warehouse._geometry import pickup_cells

    open_cells = [c for j, c in enumerate(pickup_cells(D, (4, 8))) if snap["pickup_target"][j] >= 0]
    assert len(open_cells) == 4
    assert txt.count("P") == sum(1 for c in open_cells if c not in covered)
    env.step({"0": 4, "1": 5})
    frames = env.render(mode="rgb_array", animate=True)
    assert len(frames) == env.animate_frames_per_step and frames[0].shape == (D * 12, D * 12, 3)
    assert env.render(mode="rgb_array").dtype == np.uint8
    with pytest.raises(NotImplementedError):
        env.render(mode="bogus")


def test_max_size_batch_2m_envs(wh):
    """2,097,152 Medium x 8 envs on one GPU (32x the per-GPU C3 batch): 64-bit offsets in the
    step, reward, observation and policy paths.  A sampled subset of env ids (including the last
    ones) equals the oracle after a fused greedy rollout, and the observation rows match."""
    import torch

    B, seed, K = 1 << 21, 21, 6
    L = oc.layout_for("medium")
    env = wh.BatchedWarehouse("medium", B, 8, seed=seed)
    env.reset()
    rew = torch.zeros((K, B, 8), device=env.device)
    env.rollout(K, "greedy", 0.0, rewards=rew)
    ids = np.concatenate([np.random.RandomState(2).choice(B - 64, 192, replace=False), np.arange(B - 64, B)])
    S = ob.BState.zeros(L, len(ids), 8)
    d = ob.PhiloxDraws(seed, ids)
    ob.reset(L, S, d)
    orew = []
    for _ in range(K):
        r, _, _, _ = ob.step(L, S, ob.greedy(L, S, 0.0, d), d)
        orew.append(r)
    c = canon(env)
    assert_same({k: v[ids] for k, v in c.items()}, S, "subset")
    np.testing.assert_array_equal(rew[:, torch.as_tensor(ids, device=env.device)].cpu().numpy(), np.stack(orew))
    obs = env.observe()
    np.testing.assert_array_equal(obs[torch.as_tensor(ids, device=env.device)].cpu().numpy(), ob.observe(L, S))
    acts = env.policy("greedy", 0.0)
    np.testing.assert_array_equal(acts[torch.as_tensor(ids, device=env.device)].cpu().numpy(),
                                  ob.greedy(L, S, 0.0, d))


def test_prepared_launch_equals_rollout(wh):
    """wh_rollout_prepare + wh_launch_run (BatchedWarehouse.rollout_launcher, bench.py's timed
    launches) enqueue exactly wh_rollout: same rewards, dones and state after 3 launches."""
    import torch

    B, na, K = 2048, 8, 90
    a = wh.BatchedWarehouse("medium", B, na, seed=31)
    b = wh.BatchedWarehouse("medium", B, na, seed=31)
    a.reset()
    b.reset()
    ra = torch.zeros((K, B, na), device=a.device)
    rb = torch.zeros_like(ra)
    da = torch.zeros((K, B), dtype=torch.uint8, device=a.device)
    db = torch.zeros_like(da)
    launch = b.rollout_launcher(K, "greedy", 0.0, rewards=rb, dones=db)
    for _ in range(3):
        a.rollout(K, "greedy", 0.0, rewards=ra, dones=da)
        launch()
        assert torch.equal(ra, rb) and torch.equal(da, db)
    assert torch.equal(a.state, b.state)


def test_timed_launch_equals_rollout_and_stamps_events(wh):
    """wh_launch_run_timed (events attached to the dispatch, bench.py's fused window) enqueues exactly
    wh_rollout, and its start/stop events bracket the kernel: a positive span that grows with K."""
    import torch

    B, na = 4096, 8
    spans = {}
    for K in (5, 60):
        a = wh.BatchedWarehouse("medium", B, na, seed=37)
        b = wh.BatchedWarehouse("medium", B, na, seed=37)
        a.reset()
        b.reset()
        ra = torch.zeros((K, B, na), device=a.device)
        rb = torch.zeros_like(ra)
        da = torch.zeros((K, B), dtype=torch.uint8, device=a.device)
        db = torch.zeros_like(da)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        launch = b.rollout_launcher(K, "greedy", 0.0, rewards=rb, dones=db, events=(e0, e1))
        for _ in range(4):
            a.rollout(K, "greedy", 0.0, rewards=ra, dones=da)
            launch()
            torch.cuda.synchronize()
            assert torch.equal(ra, rb) and torch.equal(da, db)
        assert torch.equal(a.state, b.state)
        spans[K] = e0.elapsed_time(e1)
        assert spans[K] > 0.0
    assert spans[60] > spans[5]


@pytest.mark.parametrize("variant,na,policy,p", [("medium", 8, "greedy", 0.0), ("large", 16, "greedy", 0.0),
                                                  ("medium", 8, "greedy", 0.25), ("large", 16, "greedy", 0.1),
                                                  ("medium", 8, "random", 0.0), ("small", 4, "random", 0.0)])
def test_fast_rollout_co_located_agents_vs_oracle(wh, variant, na, policy, p):
    """The fast fused instance (rewards + dones only, auto-reset: lazy occupancy grid, unclamped
    greedy steps, random moves converted to the steps they take) on states where agents share
    cells.  A co-located agent leaving clears the cell under the one that stays (core.py:289-291)
    until the next step's rebuild (core.py:275-276); the fast instance rebuilds only for lanes
    whose co-located agents moved, so this is its exactness case: up to half the agents start in
    pairs on shared cells (pairs that stay put keep sharing), and the rollout crosses two episode
    ends (fresh spawns share cells again).  Greedy with p > 0 and the random policy put random
    moves (including off-grid ones, core.py:282-287) through the same path."""
    import torch

    B, seed, K = 2048, 17, 430
    L = oc.layout_for(variant)
    env = wh.BatchedWarehouse(variant, B, na, seed=seed)
    env.reset()
    env.rollout(13, "greedy", 0.0)
    c = canon(env)
    rng = np.random.RandomState(1)
    pos = c["pos"].copy()
    for e in range(B):
        k = rng.randint(1, na // 2 + 1)                         # k pairs share a cell
        slots = rng.permutation(na)[: 2 * k]
        pos[e, slots[1::2]] = pos[e, slots[0::2]]
    c["pos"] = pos
    env.from_canonical(c)
    S = oracle_state(canon(env), L)
    rew = torch.zeros((K, B, na), device=env.device)
    dn = torch.zeros((K, B), dtype=torch.uint8, device=env.device)
    env.rollout(K, policy, p, rewards=rew, dones=dn)          # no returns/stats: the fast instance
    d = ob.PhiloxDraws(seed, np.arange(B))
    for s in range(K):
        acts = ob.greedy(L, S, p, d) if policy == "greedy" else ob.random_actions(S, d)
        orew, odone, _, _ = ob.step(L, S, acts, d)
        np.testing.assert_array_equal(rew[s].cpu().numpy(), orew, err_msg=f"step {s}")
        np.testing.assert_array_equal(dn[s].cpu().numpy().astype(bool), odone, err_msg=f"step {s}")
        if odone.any():
            ob.reset(L, S, d, mask=odone)
    assert_same(canon(env), S, "after rollout")


@pytest.mark.parametrize("variant,na", [("medium", 5), ("large", 7)])
def test_ordered_path_na_below_kernel_slots_vs_oracle(wh, variant, na):
    """The action-dict-order kernel (wh_step with `order`) at B = 2048 with fewer agents than the
    kernel's compile-time slots (Medium-5 runs the 8-slot instance, Large-7 the 8-slot one): the
    odd-NA reward rows are staged in LDS inside each wave's own columns (the path that carried
    round 2's cross-wave race), shuffled and partial dicts, philox regeneration; 120 steps across
    t = T (no auto-reset in wh_step) vs the oracle."""
    B, seed, K = 2048, 23, 205
    L = oc.layout_for(variant)
    env = wh.BatchedWarehouse(variant, B, na, seed=seed)
    env.reset()
    S = ob.BState.zeros(L, B, na)
    d = ob.PhiloxDraws(seed, np.arange(B))
    ob.reset(L, S, d, n_fixed=na)
    rng = np.random.RandomState(8)
    for s in range(K):
        acts = rng.randint(0, 9, size=(B, na)).astype(np.int32)
        order = np.full((B, na), -1, np.int32)
        for e in range(B):
            k = na if rng.rand() < 0.4 else rng.randint(0, na + 1)
            order[e, :k] = rng.permutation(na)[:k]
        rew, done = env.step(acts, order=order)
        orew, odone, _, _ = ob.step(L, S, acts, d, order=order)
        np.testing.assert_array_equal(rew.cpu().numpy(), orew, err_msg=f"step {s}")
        np.testing.assert_array_equal(done.cpu().numpy().astype(bool), odone, err_msg=f"step {s}")
        if s % 20 == 0 or s >= 195:
            assert_same(canon(env), S, f"step {s}")
    np.testing.assert_array_equal(env.observe().cpu().numpy(), ob.observe(L, S))
