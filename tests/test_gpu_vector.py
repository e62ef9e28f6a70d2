"""GPU parity of the sampler path (wh_vector_step, episode metrics) and the RLlib-facing adapters
(warehouse.vector) against the oracle with the philox draw contract.  Bit-exact throughout."""
import numpy as np
import pytest

from oracle import batched as ob
from oracle import core as oc

pytestmark = pytest.mark.gpu
FIELDS = ("pos", "agent_tgt", "pk_tgt", "pk_timer", "t", "n", "fresh", "episode")


@pytest.fixture(scope="module")
def wh():
    import torch

    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    import warehouse
    import warehouse.vector  # noqa: F401

    return warehouse


def take(S, idx):
    return ob.BState(*(getattr(S, f)[idx].copy() for f in FIELDS))


def put(S, idx, sub):
    for f in FIELDS:
        getattr(S, f)[idx] = getattr(sub, f)


class Bins:
    """Oracle of wh_episode_stats: on_episode_end (scripts/train.py:18-23) binned by n."""

    def __init__(self, na):
        self.sum = np.zeros(na + 1, np.int64)
        self.cnt = np.zeros(na + 1, np.int64)
        self.mn = np.full(na + 1, 0xFFFFFFFF, np.int64)
        self.mx = np.zeros(na + 1, np.int64)

    def fold(self, ret, n, done):
        for e in np.flatnonzero(done):
            b, r = int(n[e]), int(ret[e])
            self.sum[b] += r
            self.cnt[b] += 1
            self.mn[b] = min(self.mn[b], r)
            self.mx[b] = max(self.mx[b], r)

    def check(self, stats):
        got = stats.bins()
        np.testing.assert_array_equal(got["return_sum"], self.sum)
        np.testing.assert_array_equal(got["episodes"], self.cnt)
        np.testing.assert_array_equal(got["return_min"].astype(np.int64), self.mn)
        np.testing.assert_array_equal(got["return_max"].astype(np.int64), self.mx)


@pytest.mark.parametrize("variant,na,train", [("medium", 9, True), ("large", 16, False), ("small", 4, True)])
def test_vector_step_autoreset_obs_stats_vs_oracle(wh, variant, na, train):
    """wh_vector_step: external actions, some steps masked to a subset of envs, auto-reset with n
    redrawn (Train), observation rows every step, n-binned episode metrics; 420 steps = two
    episode boundaries."""
    B, seed, K = 1024, 21, 420
    L = oc.layout_for(variant)
    venv = wh.vector.WarehouseVectorEnv(variant, B, na, train=train, seed=seed)
    obs = venv.vector_reset().cpu().numpy()
    S = ob.BState.zeros(L, B, na)
    ids = np.arange(B)
    ob.reset(L, S, ob.PhiloxDraws(seed, ids), nmax=na if train else None)
    np.testing.assert_array_equal(obs, ob.observe(L, S))
    bins, epret = Bins(na), np.zeros(B, np.int64)
    rng = np.random.RandomState(1)
    for s in range(K):
        acts = rng.randint(0, 9, size=(B, na)).astype(np.int32)
        m = np.ones(B, bool) if s % 7 else rng.rand(B) < 0.5
        obs, rew, done, _ = venv.vector_step(acts, mask=None if m.all() else m)
        idx = np.flatnonzero(m)
        sub = take(S, idx)
        d = ob.PhiloxDraws(seed, idx)
        orew, odone, _, _ = ob.step(L, sub, acts[idx], d)
        np.testing.assert_array_equal(rew.cpu().numpy()[idx], orew, err_msg=f"step {s}")
        np.testing.assert_array_equal(done.cpu().numpy()[idx], odone, err_msg=f"step {s}")
        epret[idx] += orew.sum(1).astype(np.int64)
        full_done = np.zeros(B, bool)
        full_done[idx] = odone
        bins.fold(epret, S.n, full_done)          # n of the episode that ended (before the reset)
        epret[full_done] = 0
        if odone.any():
            ob.reset(L, sub, d, mask=odone, nmax=na if train else None)
        put(S, idx, sub)
        np.testing.assert_array_equal(obs.cpu().numpy(), ob.observe(L, S), err_msg=f"obs step {s}")
    bins.check(venv.stats)
    np.testing.assert_array_equal(venv.stats.episode_return.cpu().numpy(), epret)
    assert venv.custom_metrics()["avg_agent_reward_all"]["count"] == int(bins.cnt.sum())



@pytest.mark.parametrize("variant,na,train,p", [("medium", 9, True, 0.1), ("medium", 8, False, 0.0)])
def test_rollout_episode_stats_vs_oracle(wh, variant, na, train, p):
    """wh_rollout with wh_episode_stats over two launches (the running returns persist between
    them) == the oracle's greedy rollout folded into n bins; custom_metrics == on_episode_end."""
    import torch

    B, seed, K1, K2 = 2048, 13, 250, 190
    L = oc.layout_for(variant)
    env = wh.BatchedWarehouse(variant, B, na, train=train, seed=seed)
    st = env.enable_episode_stats()
    env.reset()
    ret = torch.zeros(B, device=env.device)
    env.rollout(K1, "greedy", p, returns=ret)
    env.rollout(K2, "greedy", p, returns=ret)
    S = ob.BState.zeros(L, B, na)
    d = ob.PhiloxDraws(seed, np.arange(B))
    nmax = na if train else None
    ob.reset(L, S, d, nmax=nmax)
    bins, epret = Bins(na), np.zeros(B, np.int64)
    per_episode = []
    for _ in range(K1 + K2):
        orew, odone, _, _ = ob.step(L, S, ob.greedy(L, S, p, d), d)
        epret += orew.sum(1).astype(np.int64)
        bins.fold(epret, S.n, odone)
        for e in np.flatnonzero(odone):
            per_episode.append((int(S.n[e]), epret[e] / S.n[e]))
        epret[odone] = 0
        if odone.any():
            ob.reset(L, S, d, mask=odone, nmax=nmax)
    bins.check(st)
    np.testing.assert_array_equal(st.episode_return.cpu().numpy(), epret)
    cm = st.custom_metrics()
    avgs = np.array([a for _, a in per_episode])
    assert cm["avg_agent_reward_all"]["count"] == len(per_episode)
    assert cm["avg_agent_reward_all"]["mean"] == pytest.approx(avgs.mean(), rel=1e-12)
    assert cm["avg_agent_reward_all"]["min"] == avgs.min() and cm["avg_agent_reward_all"]["max"] == avgs.max()
    for n in sorted({n for n, _ in per_episode}):
        a = np.array([v for k, v in per_episode if k == n])
        assert cm[f"avg_agent_reward_{n}"]["mean"] == pytest.approx(a.mean(), rel=1e-12)
        assert cm[f"avg_agent_reward_{n}"]["count"] == len(a)


def test_base_env_poll_send_try_reset(wh):
    """The MultiEnvDict surface: agent ids str(i) for i < n, rows equal the oracle's, "__all__"
    dones at t = T, try_reset restarts one env (Train: n redrawn), actions wrap like Python and
    >= 9 raise IndexError (core.py:281)."""
    from warehouse.vector import WarehouseBaseEnv, unflatten_row

    B, seed, na = 3, 5, 4
    L = oc.layout_for("small")
    be = WarehouseBaseEnv("small", B, train=True, seed=seed)
    S = ob.BState.zeros(L, B, na)
    d = ob.PhiloxDraws(seed, np.arange(B))
    ob.reset(L, S, d, nmax=na)
    rng = np.random.RandomState(2)
    obs, rew, dones, infos, _ = be.poll()
    ended = 0
    for s in range(260):
        ref = ob.observe(L, S)
        assert sorted(obs) == list(range(B)) if s == 0 else True
        for e, od in obs.items():
            assert list(od) == [str(i) for i in range(int(S.n[e]))]
            for a, row in od.items():
                np.testing.assert_array_equal(row, ref[e, int(a)])
                assert be.observation_space.contains(row)
                assert unflatten_row(row, L.R)["num_agents"][0] == S.n[e]
        acts = rng.randint(-9, 9, size=(B, na))
        be.send_actions({e: {str(i): int(acts[e, i]) for i in range(int(S.n[e]))} for e in range(B)})
        obs, rew, dones, infos, _ = be.poll()
        orew, odone, _, _ = ob.step(L, S, np.where(np.arange(na) < S.n[:, None], acts % 9, 4), d)
        for e in range(B):
            assert dones[e]["__all__"] == bool(odone[e])
            for a, r in rew[e].items():
                assert r == orew[e, int(a)]
        for e in np.flatnonzero(odone):
            ended += 1
            first = be.try_reset(int(e))
            m = np.zeros(B, bool)
            m[e] = True
            ob.reset(L, S, d, mask=m, nmax=na)
            obs[e] = first
    assert ended == B
    with pytest.raises(IndexError):
        be.send_actions({0: {"0": 9}})


@pytest.mark.parametrize("variant,na,train", [("medium", 8, False), ("large", 16, False), ("large", 16, True),
                                              ("small", 4, True)])
def test_staggered_episodes_fused_rollout_vs_oracle(wh, variant, na, train):
    """Desynchronised episodes (BatchedWarehouse.stagger: env e takes e*7 % 200 extra masked greedy
    steps), then a 260-step fused rollout: every step some envs end, reset and run the expiry pass
    while their wave-mates do not (one env per wave: the wave-wide single-env reset and expiry).
    Train variants redraw n at every reset.  Rewards and dones every step, and the final state,
    equal the oracle's (philox draws, auto-reset per env)."""
    import torch

    B, seed, K = 1024, 13, 260
    L = oc.layout_for(variant)
    nmax = na if train else None
    env = wh.BatchedWarehouse(variant, B, None if train else na, train=train, seed=seed)
    env.reset()
    S = ob.BState.zeros(L, B, na)
    ids = np.arange(B)
    ob.reset(L, S, ob.PhiloxDraws(seed, ids), nmax=nmax)
    off = (ids * 7) % 200
    env.stagger(off)
    for s in range(int(off.max())):
        idx = np.flatnonzero(off > s)
        sub = take(S, idx)
        d = ob.PhiloxDraws(seed, idx)
        _, odone, _, _ = ob.step(L, sub, ob.greedy(L, sub, 0.0, d), d)
        if odone.any():
            ob.reset(L, sub, d, mask=odone, nmax=nmax)
        put(S, idx, sub)
    assert len(np.unique(S.t)) > 150                       # episode clocks are spread out
    rew = torch.zeros((K, B, na), device=env.device)
    dn = torch.zeros((K, B), dtype=torch.uint8, device=env.device)
    env.rollout(K, "greedy", 0.0, rewards=rew, dones=dn)
    d = ob.PhiloxDraws(seed, ids)
    ends = 0
    for s in range(K):
        orew, odone, _, _ = ob.step(L, S, ob.greedy(L, S, 0.0, d), d)
        np.testing.assert_array_equal(rew[s].cpu().numpy(), orew, err_msg=f"step {s}")
        np.testing.assert_array_equal(dn[s].cpu().numpy().astype(bool), odone, err_msg=f"step {s}")
        ends += int(odone.sum())
        if odone.any():
            ob.reset(L, S, d, mask=odone, nmax=nmax)
    assert ends >= B                                        # every env crossed an episode end
    c = {k: v.cpu().numpy() for k, v in env.to_canonical().items()}
    np.testing.assert_array_equal(c["pos"], S.pos)
    np.testing.assert_array_equal(c["pickup_target"], S.pk_tgt)
    np.testing.assert_array_equal(c["t"], S.t)
    np.testing.assert_array_equal(c["n"], S.n)
