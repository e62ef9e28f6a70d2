"""GPU: the gfx950 kernels against the host engine (csrc/host_engine.cpp, itself pinned to the
reference fixtures by tests/test_host_engine.py) on identical inputs -- packed state words,
rewards, dones, observation rows and episode metrics bit for bit -- and the dict-order kernel on
dicts of up to 4n entries (the reference's long_* fixtures, and random long dicts at batch size).
"""
import glob
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def wh():
    import torch

    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    import warehouse
    import warehouse.vector  # noqa: F401

    return warehouse


def pair(wh, variant, B, na, train, seed):
    dev = wh.BatchedWarehouse(variant, B, na, train=train, seed=seed)
    host = wh.BatchedWarehouse(variant, B, na, train=train, seed=seed, device="cpu")
    assert not dev.host and host.host
    return dev, host


def same_state(dev, host, msg=""):
    import torch

    assert torch.equal(dev.state.cpu(), host.state), f"packed state differs {msg}"


@pytest.mark.parametrize("variant,na,policy,p,train,B,K", [
    ("medium", 8, "greedy", 0.0, False, 4096, 230),     # C3's shape (fast fused instance, reset slots)
    ("large", 16, "greedy", 0.05, False, 2048, 215),    # C4's shape with random-action coins
    ("small", 4, "random", 0.0, False, 4096, 210),      # C2's shape, random policy
    ("medium", 9, "greedy", 0.2, True, 2048, 220),      # Train variant: n redrawn at every reset
])
def test_rollout_device_equals_host_engine(wh, variant, na, policy, p, train, B, K):
    """wh_rollout (one launch of K steps: policy, step, auto-reset) on the device and on the host
    engine: rewards and dones of every step, returns, episode metrics and the final packed state
    are identical."""
    import torch

    dev, host = pair(wh, variant, B, na, train, 17)
    sd, sh = dev.enable_episode_stats(), host.enable_episode_stats()
    dev.reset()
    host.reset()
    same_state(dev, host, "after reset")
    out = []
    for e in (dev, host):
        r = torch.zeros((K, B, na), device=e.device)
        d = torch.zeros((K, B), dtype=torch.uint8, device=e.device)
        ret = torch.zeros(B, device=e.device)
        e.rollout(K, policy, p, rewards=r, dones=d, returns=ret)
        out.append((r.cpu(), d.cpu(), ret.cpu()))
    for a, b in zip(out[0], out[1]):
        assert torch.equal(a, b)
    same_state(dev, host, "after the rollout")
    for k in ("return_sum", "episodes", "return_min", "return_max", "episode_return"):
        assert torch.equal(getattr(sd, k).cpu(), getattr(sh, k)), k
    assert torch.equal(dev.observe().cpu(), host.observe())


def long_orders(rng, n, B, width, NA):
    """Random action dicts of up to `width` entries per env as order rows: agents named under
    several key forms (repeated entries, each with its own action), shuffled, partial."""
    order = np.full((B, width), -1, np.int32)
    for e in range(B):
        k = int(rng.randint(0, width + 1))
        who = rng.randint(0, n[e], size=k)
        act = rng.randint(0, 9, size=k)
        order[e, :k] = who | ((act + 1) << 8)
    return order


@pytest.mark.parametrize("variant,na,train", [("medium", 8, False), ("large", 16, False), ("small", 4, True)])
def test_vector_step_long_dicts_device_equals_host_engine(wh, variant, na, train):
    """wh_vector_step with dict orders of up to 4 NA entries per env (the dict-order kernel's LDS key
    list; Medium/Small also through the fused step + rows launch), env masks and auto-reset, against
    the host engine: rewards, dones, observation rows and packed state every step."""
    import torch

    B = 2048 + 37
    dev, host = pair(wh, variant, B, na, train, 23)
    dev.reset()
    host.reset()
    rng = np.random.RandomState(5)
    for s in range(60):
        n = ((host.state[0] >> 16) & 0xFF).numpy()
        acts = rng.randint(0, 9, size=(B, na)).astype(np.int32)
        width = [na, 2 * na, 4 * na][s % 3]
        order = long_orders(rng, n, B, width, na)
        mask = None if s % 4 else rng.rand(B) < 0.6
        od, rd, dd = dev.vector_step(acts, autoreset=True, mask=mask, order=order)
        oh, rh, dh = host.vector_step(acts, autoreset=True, mask=mask, order=order)
        keep = np.ones(B, bool) if mask is None else mask
        assert torch.equal(rd.cpu()[keep], rh[keep]), f"rewards step {s}"
        assert torch.equal(dd.cpu()[keep], dh[keep]), f"dones step {s}"
        assert torch.equal(od.cpu(), oh), f"obs step {s}"
        same_state(dev, host, f"step {s}")


def test_step_long_orders_injected_device_equals_host_engine(wh):
    """wh_step (the drop-in's kernel: dict order, injected regeneration, split phases) with orders of
    4 NA entries: every phase's result equals the host engine's."""
    import torch

    B, na = 1024, 9
    dev, host = pair(wh, "medium", B, na, False, 2)
    dev.reset()
    host.reset()
    rng = np.random.RandomState(8)
    for s in range(40):
        n = ((host.state[0] >> 16) & 0xFF).numpy()
        acts = rng.randint(0, 9, size=(B, na)).astype(np.int32)
        order = long_orders(rng, n, B, 4 * na, na)
        dev.step(acts, order=order, phase=1)
        host.step(acts, order=order, phase=1)
        assert torch.equal(dev.n_inactive.cpu(), host.n_inactive)
        assert torch.equal(dev.rewards.cpu(), host.rewards) and torch.equal(dev.dones.cpu(), host.dones)
        nin = host.n_inactive.numpy()
        regen = np.full((B, 2 * 9), -1, np.int32)
        for e in range(B):
            k = 9 - 36 + int(nin[e])
            regen[e, :k] = rng.permutation(int(nin[e]))[:k]
            regen[e, 9:9 + k] = rng.permutation(48)[:k]
        dev.step(None, regen=regen, phase=2)
        host.step(None, regen=regen, phase=2)
        same_state(dev, host, f"step {s}")


def test_long_dict_fixtures_through_dropin_and_base_env(wh):
    """long_* (the reference run with dicts of up to 4n entries) through the drop-in class on the GPU
    (global numpy stream) and through WarehouseBaseEnv.send_actions as one batch."""
    from keyforms import key_dict
    from test_gpu_vector import fixture_pre_states

    from oracle import core as oc
    from warehouse.vector import WarehouseBaseEnv

    paths = sorted(glob.glob(os.path.join(GOLDEN, "long_*.npz")))
    assert len(paths) == 3
    for path in paths:
        g = np.load(path)
        n, variant = int(g["n"]), str(g["variant"])
        np.random.seed(int(g["seed"]))
        env = {"small": wh.WarehouseSmall, "medium": wh.WarehouseMedium, "large": wh.WarehouseLarge}[variant](n)
        assert not env._engine.host
        env.reset()
        dicts = [key_dict(g["key_form"][s], g["key_agent"][s], g["key_act"][s], n) for s in range(len(g["t"]))]
        assert max(len(d) for d in dicts) == 4 * n
        for s, d in enumerate(dicts):
            obs, rew, dones, _ = env.step(d)
            flat = np.stack([np.concatenate([np.asarray(obs[str(i)][k]).ravel() for k in oc.OBS_KEYS]) for i in range(n)])
            np.testing.assert_array_equal(flat, g["obs"][s], err_msg=f"{path} step {s}")
            np.testing.assert_array_equal(np.array([rew[str(i)] for i in range(n)]), g["rewards"][s])
            assert dones["__all__"] == bool(g["done"][s])
        steps = len(dicts)
        be = WarehouseBaseEnv(variant, steps, n, train=False, seed=9)
        be.vec.env.from_canonical(fixture_pre_states(g))
        be._n[:] = n
        be.send_actions(dict(enumerate(dicts)))
        _, rew, dones, _, _ = be.poll()
        c = {k: v.cpu().numpy() for k, v in be.vec.env.to_canonical().items()}
        for s in range(steps):
            np.testing.assert_array_equal(c["pos"][s], g["pos"][s], err_msg=f"{path} step {s}")
            np.testing.assert_array_equal(c["agent_target"][s], g["agent_tgt"][s])
            assert [rew[s][str(i)] for i in range(n)] == list(g["rewards"][s])
            assert dones[s]["__all__"] == bool(g["done"][s])
