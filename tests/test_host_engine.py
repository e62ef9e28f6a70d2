"""The host engine (csrc/host_engine.cpp -> libwarehouse_host.so): the C ABI on host cores, the
engine `warehouse.Warehouse` runs on when no HIP device is present (BASELINE config 1,
"baseline/run.py on CPU").  CPU tests: every case replays the reference's own fixtures
(tests/golden/, generated from /root/reference by make_golden.py) or the fixture-pinned oracle at
tolerance 0, through `BatchedWarehouse(device="cpu")`, the drop-in class and the RLlib adapters.
The engine itself never imports or calls oracle/ (tests/test_host_engine.py checks that too)."""
import contextlib
import glob
import importlib
import io
import os
import re
import subprocess
import sys
import types

import numpy as np
import pytest

from oracle import batched as ob
from oracle import core as oc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
REF = "/root/reference"
CPU = "cpu"


@pytest.fixture(scope="module")
def wh():
    import warehouse
    import warehouse.vector  # noqa: F401

    return warehouse


@pytest.fixture()
def host_device(monkeypatch):
    """The drop-in classes on the host engine whatever this machine has (WAREHOUSE_DEVICE)."""
    monkeypatch.setenv("WAREHOUSE_DEVICE", CPU)


def canon(env):
    return {k: v.cpu().numpy() for k, v in env.to_canonical().items()}


def flat(obs, n):
    return np.stack([np.concatenate([np.asarray(obs[str(i)][k]).ravel() for k in oc.OBS_KEYS]) for i in range(n)])


def test_host_library_exports_every_declared_symbol_and_is_from_this_tree():
    from test_native_abi import declared_symbols

    from warehouse import _native

    lib = _native.host_lib()
    out = subprocess.run(["nm", "-D", "--defined-only", _native.HOST_LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    assert set(re.findall(r" T (wh_[a-z_]+)$", out, flags=re.M)) == set(declared_symbols())
    assert lib.wh_version().startswith(b"warehouse_host cpu host-engine v1")
    assert _native.verify_host_provenance() == _native.tree_source_sha()
    src = open(os.path.join(ROOT, "rllib-warehouse_amd", "csrc", "host_engine.cpp")).read()
    assert "oracle" not in src.replace("test oracle", "")   # product code: nothing from oracle/


def test_host_engine_refuses_device_only_entry_points(wh):
    import ctypes

    from warehouse import _native

    env = wh.BatchedWarehouse("medium", 8, 8, device=CPU)
    env.reset()
    with pytest.raises(_native.WarehouseNativeError, match="ENOTSUP"):
        env.observe_x()
    with pytest.raises(_native.WarehouseNativeError):
        env.rollout_launcher(4)
    n = ctypes.c_int64()
    d = _native.WhMlpDesc(82, 512, 512, 9, _native.WH_MLP_BF16)
    assert _native.host_lib().wh_mlp_query(ctypes.byref(d), ctypes.byref(n)) == _native.WH_ENOTSUP
    with pytest.raises(ValueError):                       # order rows past 4 * NA
        env.step(np.full((8, 8), 4, np.int32), order=np.full((8, 33), -1, np.int32))
    acts = np.full((8, 8), 4, np.int32)
    for bad in (np.ones(7, bool), np.ones((8, 1), bool)):   # env masks of the wrong shape
        with pytest.raises(ValueError):
            env.vector_step(acts, mask=bad)
        with pytest.raises(ValueError):
            env.reset(mask=bad)


def g1_runs(variant):
    paths = sorted(glob.glob(os.path.join(GOLDEN, f"g1_{variant}_*.npz"))
                   + glob.glob(os.path.join(GOLDEN, f"ord_{variant}_*.npz")))
    return [dict(np.load(p)) for p in paths]


@pytest.mark.parametrize("variant", ["small", "medium", "large"])
@pytest.mark.parametrize("ordered", [True, False])
def test_g1_episodes_injected(wh, variant, ordered):
    """Whole 200-step reference episodes (G1 and the shuffled/partial-dict ord_* runs), every
    (N, seed) batched as B envs of a Train-shaped batch: state, rewards, dones and observation rows
    equal the reference's at every step."""
    runs = g1_runs(variant)
    if not ordered:
        runs = [g for g in runs if np.all(g["order"] == np.arange(int(g["n"])))]
    nmax = oc.VARIANTS[variant]["nmax"]
    B = len(runs)
    n = np.array([int(g["n"]) for g in runs], np.int32)
    spawn = np.zeros((B, nmax, 2), np.int32)
    for e, g in enumerate(runs):
        spawn[e, : n[e]] = g["spawn"]
    env = wh.BatchedWarehouse(variant, B, train=True, device=CPU)
    env.reset(draws=dict(spawn=spawn, pickups=np.stack([g["reset_sel"] for g in runs]),
                         targets=np.stack([g["reset_tgt"] for g in runs]), n=n))
    obs = env.observe().numpy()
    for e, g in enumerate(runs):
        np.testing.assert_array_equal(obs[e, : n[e]], g["reset_obs"])
        assert not obs[e, n[e]:].any()
    for s in range(200):
        acts = np.full((B, nmax), 4, np.int32)
        order = np.full((B, nmax), -1, np.int32)
        for e, g in enumerate(runs):
            acts[e, : n[e]] = np.mod(g["actions"][s], 9)
            order[e, : n[e]] = g["order"][s]
        regen = np.concatenate([np.stack([g["rpos"][s] for g in runs]), np.stack([g["rtgt"][s] for g in runs])], axis=1)
        rew, done = env.step(acts, order=order if ordered else None, regen=regen)
        rew, done = rew.numpy().copy(), done.numpy().copy()
        c = canon(env)
        obs = env.observe().numpy()
        for e, g in enumerate(runs):
            k = n[e]
            msg = f"env {e} step {s}"
            np.testing.assert_array_equal(c["pos"][e, :k], g["pos"][s], err_msg=msg)
            np.testing.assert_array_equal(c["agent_target"][e, :k], g["agent_tgt"][s], err_msg=msg)
            np.testing.assert_array_equal(c["pickup_target"][e], g["pk_tgt"][s], err_msg=msg)
            np.testing.assert_array_equal(c["pickup_timer"][e], g["pk_timer"][s], err_msg=msg)
            assert c["t"][e] == g["t"][s]
            np.testing.assert_array_equal(rew[e, :k], g["rewards"][s], err_msg=msg)
            assert bool(done[e]) == bool(g["done"][s])
            np.testing.assert_array_equal(obs[e, :k], g["obs"][s], err_msg=msg)


@pytest.mark.parametrize("variant", ["small", "medium", "large"])
def test_g2_dense_transitions(wh, variant):
    """G2: 400 single transitions from adversarial hand-built states (stacked agents, carriers at
    their delivery cells, expiring timers, t at T) with shuffled dicts, exact."""
    g = np.load(os.path.join(GOLDEN, f"g2_{variant}.npz"))
    env = wh.BatchedWarehouse(variant, len(g["n"]), train=True, device=CPU)
    env.from_canonical(dict(pos=g["pre_pos"], agent_target=g["pre_agent_tgt"], pickup_target=g["pre_pk_tgt"],
                            pickup_timer=g["pre_pk_timer"], t=g["pre_t"], n=g["n"]))
    rew, done = env.step(g["actions"], order=g["order"], regen=np.concatenate([g["rpos"], g["rtgt"]], axis=1))
    c = canon(env)
    np.testing.assert_array_equal(c["pos"], g["pos"])
    np.testing.assert_array_equal(c["agent_target"], g["agent_tgt"])
    np.testing.assert_array_equal(c["pickup_target"], g["pk_tgt"])
    np.testing.assert_array_equal(c["pickup_timer"], g["pk_timer"])
    np.testing.assert_array_equal(rew.numpy(), g["rewards"])
    np.testing.assert_array_equal(done.numpy().astype(bool), g["done"])
    np.testing.assert_array_equal(env.observe().numpy(), g["obs"])


def test_dropin_config1_greedy_runs_match_reference(wh, host_device):
    """BASELINE config 1 on the host engine: baseline/run.py's loop through the drop-in class with
    the reference solver (restated by the oracle on the obs dicts), numpy's global stream: every G3
    rollout's actions and total equal the reference's (seed 0 -> 82.0)."""
    g = np.load(os.path.join(GOLDEN, "g3_greedy.npz"))
    for ci in range(11):
        variant, n, p, seed = g[f"c{ci}_meta"]
        n, p, seed = int(n), float(p), int(seed)
        np.random.seed(seed)
        env = {"small": wh.WarehouseSmall, "medium": wh.WarehouseMedium, "large": wh.WarehouseLarge}[variant](n)
        assert env._engine.host
        L = oc.layout_for(variant)
        obs = env.reset()
        draws = oc.GlobalNumpyDraws()
        total, steps, done = 0.0, 0, False
        while not done:
            acts = oc.greedy(L, flat(obs, n), p, draws)
            np.testing.assert_array_equal(acts, g[f"c{ci}_actions"][steps], err_msg=f"run {ci} step {steps}")
            obs, rew, dones, _ = env.step({str(i): int(acts[i]) for i in range(n)})
            for o in obs.values():
                assert env.observation_space.contains(o)
            total += sum(float(rew[str(i)]) for i in range(n))
            done = dones["__all__"]
            steps += 1
        assert steps == 200 and total == float(g[f"c{ci}_total"]), ci
    assert float(g["c0_total"]) == 82.0


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "baseline")), reason="the reference is not on this machine")
def test_reference_run_main_unchanged_on_host_engine(wh, host_device, monkeypatch):
    """`np.random.seed(0); run.main('small', 2, 0.0, False)` with the reference's own, unchanged
    baseline/run.py and baseline/solvers.py on the path, importing this package as `warehouse`:
    the printed rewards are 42.0 / 40.0.  solvers.py imports gym only for a type
    annotation; gym is not installed here, so a stand-in module carries this package's spaces."""
    from warehouse import _compat

    gym = types.ModuleType("gym")
    gym.Space, gym.spaces = object, _compat.spaces
    monkeypatch.setitem(sys.modules, "gym", gym)
    monkeypatch.syspath_prepend(os.path.join(REF, "baseline"))
    for m in ("run", "solvers"):
        sys.modules.pop(m, None)
    run = importlib.import_module("run")
    assert os.path.dirname(run.__file__) == os.path.join(REF, "baseline")
    assert run.WarehouseSmall is wh.WarehouseSmall          # this package, not the reference's
    for seed, want in ((0, "Rewards: 42.0 40.0"), (1, None), (2, None)):
        np.random.seed(seed)
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            run.main("small", 2, 0.0, False)
        text = buf.getvalue()
        total = float(re.search(r"Total: ([0-9.]+)", text).group(1))
        assert total == {0: 82.0, 1: 49.0, 2: 7.0}[seed], text
        if want:
            assert want in text, text
    for m in ("run", "solvers"):
        sys.modules.pop(m, None)


def test_dropin_dict_order_and_key_forms(wh, host_device):
    """ord_* (shuffled/partial dicts, negative actions), keys_* (int, negative and repeated keys)
    and long_* (dicts of up to 4n entries: agents under up to all four key forms, moving several
    times in one step) through the drop-in class on the global numpy stream: observations, rewards
    and dones equal the reference's at every step."""
    from keyforms import key_dict

    g = np.load(os.path.join(GOLDEN, "ord_medium_n9_s5.npz"))
    np.random.seed(int(g["seed"]))
    env = wh.WarehouseMedium(9)
    env.reset()
    for s in range(200):
        order = [int(i) for i in g["order"][s] if i >= 0]
        obs, rew, _, _ = env.step({str(i): int(g["actions"][s][i]) for i in order})
        np.testing.assert_array_equal(flat(obs, 9), g["obs"][s])
        np.testing.assert_array_equal(np.array([rew[str(i)] for i in range(9)]), g["rewards"][s])
    for pat in ("keys_*.npz", "long_*.npz"):
        for path in sorted(glob.glob(os.path.join(GOLDEN, pat))):
            g = np.load(path)
            n = int(g["n"])
            np.random.seed(int(g["seed"]))
            env = {"small": wh.WarehouseSmall, "medium": wh.WarehouseMedium, "large": wh.WarehouseLarge}[str(g["variant"])](n)
            env.reset()
            longest = 0
            for s in range(len(g["t"])):
                d = key_dict(g["key_form"][s], g["key_agent"][s], g["key_act"][s], n)
                longest = max(longest, len(d))
                obs, rew, dones, _ = env.step(d)
                np.testing.assert_array_equal(flat(obs, n), g["obs"][s], err_msg=f"{path} step {s}")
                np.testing.assert_array_equal(np.array([rew[str(i)] for i in range(n)]), g["rewards"][s])
                assert dones["__all__"] == bool(g["done"][s])
            assert longest == (4 * n if pat.startswith("long") else n) or pat.startswith("keys")
    with pytest.raises(IndexError):
        env.step({"0": 9})
    too_long = {k: 4 for i in range(n) for k in (str(i), i, str(i - n), i - n)}
    too_long["00"] = 4                                      # int("00") == 0: a fifth key form
    with pytest.raises(ValueError):
        env.step(too_long)


def test_base_env_long_dicts_match_reference(wh):
    """long_* through WarehouseBaseEnv.send_actions as one batch (env s holds the reference's state
    before step s): positions, carried targets, rewards and dones equal the reference's."""
    from keyforms import key_dict
    from test_gpu_vector import fixture_pre_states

    from warehouse.vector import WarehouseBaseEnv

    for path in sorted(glob.glob(os.path.join(GOLDEN, "long_*.npz"))):
        g = np.load(path)
        n, variant = int(g["n"]), str(g["variant"])
        steps = len(g["t"])
        be = WarehouseBaseEnv(variant, steps, n, train=False, seed=9, device=CPU)
        be.vec.env.from_canonical(fixture_pre_states(g))
        be._n[:] = n
        be.send_actions({s: key_dict(g["key_form"][s], g["key_agent"][s], g["key_act"][s], n) for s in range(steps)})
        _, rew, dones, _, _ = be.poll()
        c = canon(be.vec.env)
        for s in range(steps):
            msg = f"{path} step {s}"
            np.testing.assert_array_equal(c["pos"][s], g["pos"][s], err_msg=msg)
            np.testing.assert_array_equal(c["agent_target"][s], g["agent_tgt"][s], err_msg=msg)
            assert [rew[s][str(i)] for i in range(n)] == list(g["rewards"][s]), msg
            assert dones[s]["__all__"] == bool(g["done"][s]), msg


@pytest.mark.parametrize("variant,na,policy,p,train", [("medium", 8, "greedy", 0.0, False), ("large", 16, "greedy", 0.05, False),
                                                       ("small", 4, "random", 0.0, False), ("medium", 9, "greedy", 0.2, True)])
def test_philox_rollout_vs_oracle(wh, variant, na, policy, p, train):
    """wh_rollout on the host engine (device philox contract: policy coins, regeneration, auto-reset
    with n redrawn for the Train variants) equals the oracle's philox model step by step, with
    returns and the n-binned episode metrics."""
    import torch

    B, seed, K = 192, 3, 230
    L = oc.layout_for(variant)
    env = wh.BatchedWarehouse(variant, B, na, train=train, seed=seed, device=CPU)
    st = env.enable_episode_stats()
    env.reset()
    rew = torch.zeros((K, B, na))
    dn = torch.zeros((K, B), dtype=torch.uint8)
    ret = torch.zeros(B)
    env.rollout(K, policy, p, rewards=rew, dones=dn, returns=ret)
    S = ob.BState.zeros(L, B, na)
    d = ob.PhiloxDraws(seed, np.arange(B))
    nmax = na if train else None
    ob.reset(L, S, d, nmax=nmax)
    tot = np.zeros(B, np.float32)
    epr, cnt = np.zeros(B, np.int64), np.zeros(na + 1, np.int64)
    for s in range(K):
        acts = ob.greedy(L, S, p, d) if policy == "greedy" else ob.random_actions(S, d)
        orew, odone, _, _ = ob.step(L, S, acts, d)
        np.testing.assert_array_equal(rew[s].numpy(), orew, err_msg=f"step {s}")
        np.testing.assert_array_equal(dn[s].numpy().astype(bool), odone)
        tot += orew.sum(1)
        epr += orew.sum(1).astype(np.int64)
        np.add.at(cnt, S.n[odone], 1)
        epr[odone] = 0
        if odone.any():
            ob.reset(L, S, d, mask=odone, nmax=nmax)
    c = canon(env)
    for f, k in (("pos", "pos"), ("agent_target", "agent_tgt"), ("pickup_target", "pk_tgt"),
                 ("pickup_timer", "pk_timer"), ("t", "t"), ("n", "n")):
        np.testing.assert_array_equal(c[f], getattr(S, k), err_msg=f)
    np.testing.assert_array_equal(ret.numpy(), tot)
    np.testing.assert_array_equal(st.episodes.numpy(), cnt)
    np.testing.assert_array_equal(st.episode_return.numpy(), epr)
    np.testing.assert_array_equal(env.observe().numpy(), ob.observe(L, S))


@pytest.mark.parametrize("variant,na,train", [("medium", 9, True), ("large", 16, False)])
def test_vector_step_masked_dict_order_autoreset_vs_oracle(wh, variant, na, train):
    """wh_vector_step on the host engine: shuffled/partial dicts, env masks, auto-reset (n redrawn for
    Train), observation rows every step, equal to the oracle."""
    from test_gpu_vector import put, take

    B, seed, K = 128, 29, 215
    L = oc.layout_for(variant)
    venv = wh.vector.WarehouseVectorEnv(variant, B, na, train=train, seed=seed, device=CPU)
    venv.vector_reset()
    S = ob.BState.zeros(L, B, na)
    ob.reset(L, S, ob.PhiloxDraws(seed, np.arange(B)), nmax=na if train else None)
    rng = np.random.RandomState(3)
    for s in range(K):
        acts = rng.randint(0, 9, size=(B, na)).astype(np.int32)
        order = np.full((B, na), -1, np.int32)
        for e in range(B):
            k = int(S.n[e]) if rng.rand() < 0.3 else rng.randint(0, int(S.n[e]) + 1)
            order[e, :k] = rng.permutation(int(S.n[e]))[:k]
        m = np.ones(B, bool) if s % 5 else rng.rand(B) < 0.6
        obs, rew, done, _ = venv.vector_step(acts, mask=None if m.all() else m, order=order)
        idx = np.flatnonzero(m)
        sub = take(S, idx)
        d = ob.PhiloxDraws(seed, idx)
        orew, odone, _, _ = ob.step(L, sub, acts[idx], d, order=order[idx])
        np.testing.assert_array_equal(rew.numpy()[idx], orew, err_msg=f"step {s}")
        np.testing.assert_array_equal(done.numpy()[idx], odone, err_msg=f"step {s}")
        if odone.any():
            ob.reset(L, sub, d, mask=odone, nmax=na if train else None)
        put(S, idx, sub)
        np.testing.assert_array_equal(obs.numpy(), ob.observe(L, S), err_msg=f"obs step {s}")


def test_pack_unpack_roundtrip_and_policy(wh):
    """Canonical <-> packed round trip on the G2 states; wh_policy equals the oracle's greedy
    policy (with coins) on them."""
    g = np.load(os.path.join(GOLDEN, "g2_large.npz"))
    env = wh.BatchedWarehouse("large", len(g["n"]), train=True, device=CPU, seed=4)
    src = dict(pos=g["pos"], agent_target=g["agent_tgt"], pickup_target=g["pk_tgt"], pickup_timer=g["pk_timer"],
               t=g["t"], n=g["n"])
    env.from_canonical(src)
    c = canon(env)
    for k in ("pos", "agent_target", "pickup_target", "pickup_timer", "t", "n"):
        np.testing.assert_array_equal(c[k], src[k])
    L = oc.layout_for("large")
    from test_gpu_parity import oracle_state

    S = oracle_state(c, L)
    d = ob.PhiloxDraws(4, np.arange(len(g["n"])))
    for p in (0.0, 0.3):
        np.testing.assert_array_equal(env.policy("greedy", p).numpy(), ob.greedy(L, S, p, d))
