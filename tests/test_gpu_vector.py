"""GPU parity of the sampler path (wh_vector_step, episode metrics) and the RLlib-facing adapters
(warehouse.vector) against the oracle with the philox draw contract.  Bit-exact throughout."""
import os

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



@pytest.mark.parametrize("na,B", [(16, 7), (12, 333), (16, 1000), (8, 129)])
def test_chunked_large_rows_vs_oracle(wh, na, B):
    """Large f32 rows are written in 1,024-float4 chunks per workgroup (k_observe's CHUNK form), each
    imaging the envs its chunk touches: chunks that start mid-env and span three (16 agents) or four
    (12 agents) envs, a ragged last chunk, a batch smaller than one chunk; 8 agents (rows of 290
    float4s: more envs per chunk than the instance images) takes the per-group form.  Rows vs the
    oracle after resets and every external-action step."""
    L = oc.layout_for("large")
    seed = 5
    venv = wh.vector.WarehouseVectorEnv("large", B, na, train=False, seed=seed)
    obs = venv.vector_reset().cpu().numpy()
    S = ob.BState.zeros(L, B, na)
    ids = np.arange(B)
    ob.reset(L, S, ob.PhiloxDraws(seed, ids))
    np.testing.assert_array_equal(obs, ob.observe(L, S))
    rng = np.random.RandomState(2)
    d = ob.PhiloxDraws(seed, ids)
    for s in range(30):
        acts = rng.randint(0, 9, size=(B, na)).astype(np.int32)
        obs, rew, done, _ = venv.vector_step(acts)
        orew, odone, _, _ = ob.step(L, S, acts, d)
        np.testing.assert_array_equal(rew.cpu().numpy(), orew, err_msg=f"step {s}")
        if odone.any():
            ob.reset(L, S, d, mask=odone)
        np.testing.assert_array_equal(obs.cpu().numpy(), ob.observe(L, S), err_msg=f"obs step {s}")


def test_large_rows_unaligned_output_equal_the_chunked_rows(wh):
    """An f32 row buffer that is not 16-byte aligned cannot take the chunked float4 writer: the
    per-group scalar form writes it, with the same rows."""
    import torch
    from warehouse import _native as nat

    env = wh.BatchedWarehouse("large", 300, 16, seed=4)
    env.reset()
    env.rollout(17, "greedy", 0.0)
    ref = env.observe().clone()
    buf = torch.zeros(ref.numel() + 1, device=env.device)
    nat.check(nat.lib().wh_observe(env._cfgp, env.B, env.state.data_ptr(), buf.data_ptr() + 4, env.stream),
              "wh_observe")
    torch.cuda.synchronize()
    assert torch.equal(buf[1:].view_as(ref), ref)


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


@pytest.mark.parametrize("variant,na,train,policy,p,group", [("medium", 8, False, "greedy", 0.0, 1),
                                                              ("large", 16, False, "greedy", 0.0, 1),
                                                              ("large", 16, True, "greedy", 0.0, 1),
                                                              ("small", 4, True, "greedy", 0.0, 1),
                                                              ("medium", 8, False, "greedy", 0.2, 1),
                                                              ("medium", 8, False, "random", 0.0, 1),
                                                              ("medium", 8, False, "greedy", 0.0, 4),
                                                              ("large", 16, True, "greedy", 0.0, 8),
                                                              ("medium", 9, True, "greedy", 0.1, 16),
                                                              ("medium", 8, False, "greedy", 0.0, -5),
                                                              ("large", 16, True, "greedy", 0.1, -1)])
def test_staggered_episodes_fused_rollout_vs_oracle(wh, variant, na, train, policy, p, group):
    """Desynchronised episodes (BatchedWarehouse.stagger: env e takes e*7 % 200 extra masked greedy
    steps; with group > 1 the lanes l, l + 64/group, ... of a wave share an offset), then a 260-step
    fused rollout: every step some envs end, reset and run the expiry pass while their wave-mates do
    not -- `group` envs of a wave at a time: the wave-wide resets from the reset slots (one lane
    each, up to kSlotResetMax), the slot refill, and past that the all-lane reset.  Train variants
    redraw n at every reset.  Rewards and dones every step, and the final state, equal the oracle's
    (philox draws, auto-reset per env).  group < 0: the same 260 steps as launches of -group steps
    (shorter than kSlotMinSteps: single lanes reset from scratch, the sampler's 1-step case)."""
    import torch

    B, seed, K = 1024, 13, 260
    L = oc.layout_for(variant)
    nmax = na if train else None
    env = wh.BatchedWarehouse(variant, B, None if train else na, train=train, seed=seed)
    env.reset()
    S = ob.BState.zeros(L, B, na)
    ids = np.arange(B)
    ob.reset(L, S, ob.PhiloxDraws(seed, ids), nmax=nmax)
    off = (ids * 7) % 200 if group <= 1 else ((ids % (64 // group)) * 7 + (ids // 64) * 3) % 200
    env.stagger(off)
    for s in range(int(off.max())):
        idx = np.flatnonzero(off > s)
        sub = take(S, idx)
        d = ob.PhiloxDraws(seed, idx)
        _, odone, _, _ = ob.step(L, sub, ob.greedy(L, sub, 0.0, d), d)
        if odone.any():
            ob.reset(L, sub, d, mask=odone, nmax=nmax)
        put(S, idx, sub)
    assert len(np.unique(S.t)) > (150 if group <= 1 else 40)   # episode clocks are spread out
    rew = torch.zeros((K, B, na), device=env.device)
    dn = torch.zeros((K, B), dtype=torch.uint8, device=env.device)
    step = K if group > 0 else -group
    for s0 in range(0, K, step):
        s1 = min(K, s0 + step)
        env.rollout(s1 - s0, policy, p, rewards=rew[s0:s1], dones=dn[s0:s1])
    d = ob.PhiloxDraws(seed, ids)
    ends = 0
    for s in range(K):
        acts = ob.greedy(L, S, p, d) if policy == "greedy" else ob.random_actions(S, d)
        orew, odone, _, _ = ob.step(L, S, acts, d)
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


# ----------------------------------------------------------------------------- action-dict order
def fixture_pre_states(g):
    """The fixture's state before each of its 200 steps (reset state, then the state after step
    s-1) as canonical arrays [200, ...]."""
    n = int(g["n"])
    pos = np.concatenate([g["reset_pos"][None], g["pos"][:-1]])
    atg = np.concatenate([g["reset_agent_tgt"][None], g["agent_tgt"][:-1]])
    ptg = np.concatenate([g["reset_pk_tgt"][None], g["pk_tgt"][:-1]])
    ptm = np.concatenate([g["reset_pk_timer"][None], g["pk_timer"][:-1]])
    t = np.concatenate([[int(g["reset_t"])], g["t"][:-1]]).astype(np.int32)
    return dict(pos=pos, agent_target=atg, pickup_target=ptg, pickup_timer=ptm, t=t,
                n=np.full(len(t), n, np.int32))


@pytest.mark.parametrize("variant", ["small", "medium", "large"])
def test_base_env_replays_reference_dict_order_fixtures(wh, variant):
    """tests/golden/ord_*: the reference's own episodes driven by shuffled and partial action dicts
    with negative actions (core.py:279-300), replayed through WarehouseBaseEnv.send_actions as one
    batch -- env s holds the reference's state before step s and gets that step's dict, in two
    masked halves (odd envs first).  Everything the regeneration draws do not touch equals the
    reference bit for bit (positions, carried targets, rewards, dones, every request not reopened
    this step, the count reopened); the whole transition including the philox regeneration and
    the observation rows equals the oracle's."""
    from warehouse.vector import WarehouseBaseEnv

    L = oc.layout_for(variant)
    import glob
    import os

    paths = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", f"ord_{variant}_*.npz")))
    assert paths
    for path in paths:
        g = np.load(path)
        n = int(g["n"])
        steps = len(g["t"])
        pre = fixture_pre_states(g)
        be = WarehouseBaseEnv(variant, steps, n, train=False, seed=9)
        be.vec.env.from_canonical(pre)
        be._n[:] = n
        dicts = {s: {str(int(i)): int(g["actions"][s][int(i)]) for i in g["order"][s] if i >= 0}
                 for s in range(steps)}
        assert any(len(d) < n for d in dicts.values()) and any(list(d) != sorted(d, key=int) for d in dicts.values())
        got_rew, got_done = {}, {}
        for half in (1, 0):
            be.send_actions({s: dicts[s] for s in range(steps) if s % 2 == half})
            _, rew, dones, _, _ = be.poll()
            assert sorted(rew) == [s for s in range(steps) if s % 2 == half]
            got_rew.update(rew)
            got_done.update(dones)
        c = {k: v.cpu().numpy() for k, v in be.vec.env.to_canonical().items()}
        W = L.W
        for s in range(steps):
            msg = f"{path} step {s}"
            np.testing.assert_array_equal(c["pos"][s], g["pos"][s], err_msg=msg)
            np.testing.assert_array_equal(c["agent_target"][s], g["agent_tgt"][s], err_msg=msg)
            assert [got_rew[s][str(i)] for i in range(n)] == list(g["rewards"][s]), msg
            assert got_done[s]["__all__"] == bool(g["done"][s]), msg
            ro, rf = c["pickup_timer"][s] == W, g["pk_timer"][s] == W       # reopened this step
            assert ro.sum() == rf.sum(), msg
            keep = ~(ro | rf)
            np.testing.assert_array_equal(c["pickup_target"][s][keep], g["pk_tgt"][s][keep], err_msg=msg)
            np.testing.assert_array_equal(c["pickup_timer"][s][keep], g["pk_timer"][s][keep], err_msg=msg)
            assert (c["pickup_target"][s][rf & ~ro] == -1).all() and (g["pk_tgt"][s][ro & ~rf] == -1).all()
        # the whole transition, philox regeneration included, against the oracle
        S = ob.BState(pos=pre["pos"].copy(), agent_tgt=pre["agent_target"].copy(),
                      pk_tgt=pre["pickup_target"].copy(), pk_timer=pre["pickup_timer"].copy(),
                      t=pre["t"].astype(np.int64), n=pre["n"].copy(), fresh=np.zeros(steps, bool),
                      episode=np.zeros(steps, np.uint32))
        acts = np.full((steps, n), 4, np.int32)
        order = np.full((steps, n), -1, np.int32)
        for s, d in dicts.items():
            for k, (a, v) in enumerate(d.items()):
                acts[s, int(a)] = v % 9
                order[s, k] = int(a)
        orew, odone, _, _ = ob.step(L, S, acts, ob.PhiloxDraws(9, np.arange(steps)), order=order)
        np.testing.assert_array_equal(np.array([[got_rew[s][str(i)] for i in range(n)] for s in range(steps)]), orew)
        for f, k in (("pos", "pos"), ("agent_target", "agent_tgt"), ("pickup_target", "pk_tgt"),
                     ("pickup_timer", "pk_timer"), ("t", "t")):
            np.testing.assert_array_equal(c[f], getattr(S, k), err_msg=f)
        np.testing.assert_array_equal(be.vec.env.observe().cpu().numpy(), ob.observe(L, S))


@pytest.mark.parametrize("variant,n", [("small", 4), ("medium", 8), ("large", 16)])
def test_base_env_key_forms_match_reference(wh, variant, n):
    """keys_* fixtures (int, negative and repeated keys in one dict, core.py:279-281) replayed through
    WarehouseBaseEnv.send_actions as one batch (env s holds the reference's state before step s):
    positions, carried targets, rewards and dones equal the reference's; the whole transition with
    the philox regeneration and the rows equals the batched oracle's on the encoded order entries."""
    from keyforms import encoded_order, key_dict

    from warehouse.vector import WarehouseBaseEnv

    L = oc.layout_for(variant)
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", f"keys_{variant}_n{n}_s7.npz"))
    steps = len(g["t"])
    pre = fixture_pre_states(g)
    be = WarehouseBaseEnv(variant, steps, n, train=False, seed=9)
    be.vec.env.from_canonical(pre)
    be._n[:] = n
    dicts = {s: key_dict(g["key_form"][s], g["key_agent"][s], g["key_act"][s], n) for s in range(steps)}
    be.send_actions(dicts)
    _, rew, dones, _, _ = be.poll()
    c = {k: v.cpu().numpy() for k, v in be.vec.env.to_canonical().items()}
    for s in range(steps):
        msg = f"step {s}"
        np.testing.assert_array_equal(c["pos"][s], g["pos"][s], err_msg=msg)
        np.testing.assert_array_equal(c["agent_target"][s], g["agent_tgt"][s], err_msg=msg)
        assert [rew[s][str(i)] for i in range(n)] == list(g["rewards"][s]), msg
        assert dones[s]["__all__"] == bool(g["done"][s]), msg
    S = ob.BState(pos=pre["pos"].copy(), agent_tgt=pre["agent_target"].copy(),
                  pk_tgt=pre["pickup_target"].copy(), pk_timer=pre["pickup_timer"].copy(),
                  t=pre["t"].astype(np.int64), n=pre["n"].copy(), fresh=np.zeros(steps, bool),
                  episode=np.zeros(steps, np.uint32))
    order = np.array([encoded_order(dicts[s], n, n) for s in range(steps)], np.int32)
    orew, _, _, _ = ob.step(L, S, np.full((steps, n), 4, np.int32), ob.PhiloxDraws(9, np.arange(steps)), order=order)
    np.testing.assert_array_equal(np.array([[rew[s][str(i)] for i in range(n)] for s in range(steps)]), orew)
    for f, k in (("pos", "pos"), ("agent_target", "agent_tgt"), ("pickup_target", "pk_tgt"),
                 ("pickup_timer", "pk_timer"), ("t", "t")):
        np.testing.assert_array_equal(c[f], getattr(S, k), err_msg=f)
    np.testing.assert_array_equal(be.vec.env.observe().cpu().numpy(), ob.observe(L, S))


def test_base_env_absent_agent_does_not_remark_its_cell(wh):
    """Known-answer test of core.py:279-300's dict semantics on co-located agents (Small, 3
    agents; 0 and 1 share cell (2,2), agent 2 at (3,2); action 1 = move -x):
      env 0  {"0": 1, "2": 1}          agent 0 leaves (clearing the shared cell), agent 1 is absent
                                       and does not re-mark it, so agent 2 enters: 1 and 2 share it
      env 1  {"0": 1, "1": 4, "2": 1}  agent 1's "stay" re-marks the cell: agent 2 is blocked
      env 2  {"2": 1, "0": 1}          agent 2 goes first and is blocked, then agent 0 leaves
      env 3  {}                        nobody moves
    and the same through the oracle for every env."""
    from warehouse.vector import WarehouseBaseEnv

    L = oc.layout_for("small")
    B, n = 4, 3
    pos = np.tile(np.array([[2, 2], [2, 2], [3, 2]], np.int32), (B, 1, 1))
    ptg = np.full((B, L.P), -1, np.int32)
    ptm = np.full((B, L.P), -1, np.int32)
    ptg[:, :L.R] = np.arange(L.R)
    ptm[:, :L.R] = 150
    state = dict(pos=pos, agent_target=np.full((B, n), -1, np.int32), pickup_target=ptg, pickup_timer=ptm,
                 t=np.full(B, 10, np.int32), n=np.full(B, n, np.int32))
    be = WarehouseBaseEnv("small", B, n, train=False, seed=4)
    be.vec.env.from_canonical(state)
    be._n[:] = n
    dicts = {0: {"0": 1, "2": 1}, 1: {"0": 1, "1": 4, "2": 1}, 2: {"2": 1, "0": 1}, 3: {}}
    be.send_actions(dicts)
    be.poll()
    got = be.vec.env.to_canonical()["pos"].cpu().numpy()
    np.testing.assert_array_equal(got[0], [[1, 2], [2, 2], [2, 2]])
    np.testing.assert_array_equal(got[1], [[1, 2], [2, 2], [3, 2]])
    np.testing.assert_array_equal(got[2], [[1, 2], [2, 2], [3, 2]])
    np.testing.assert_array_equal(got[3], [[2, 2], [2, 2], [3, 2]])
    S = ob.BState(pos=pos.copy(), agent_tgt=state["agent_target"].copy(), pk_tgt=ptg.copy(), pk_timer=ptm.copy(),
                  t=state["t"].astype(np.int64), n=state["n"].copy(), fresh=np.zeros(B, bool),
                  episode=np.zeros(B, np.uint32))
    acts = np.full((B, n), 4, np.int32)
    order = np.full((B, n), -1, np.int32)
    for e, d in dicts.items():
        for k, (a, v) in enumerate(d.items()):
            acts[e, int(a)] = v
            order[e, k] = int(a)
    ob.step(L, S, acts, ob.PhiloxDraws(4, np.arange(B)), order=order)
    np.testing.assert_array_equal(got, S.pos)
    with pytest.raises(IndexError):
        be.send_actions({0: {"3": 4}})                    # no agent 3 in a 3-agent episode


@pytest.mark.parametrize("variant,na,train", [("medium", 9, True), ("large", 16, False), ("small", 4, False)])
def test_vector_step_dict_order_masked_autoreset_vs_oracle(wh, variant, na, train):
    """wh_vector_step with an action-dict order per env (random permutations of random subsets of
    the live agents: shuffled and partial dicts), env masks and auto-reset, 230 steps: rewards,
    dones and observation rows equal the oracle's every step."""
    B, seed, K = 1024, 29, 230
    L = oc.layout_for(variant)
    venv = wh.vector.WarehouseVectorEnv(variant, B, na, train=train, seed=seed)
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
        np.testing.assert_array_equal(rew.cpu().numpy()[idx], orew, err_msg=f"step {s}")
        np.testing.assert_array_equal(done.cpu().numpy()[idx], odone, err_msg=f"step {s}")
        if odone.any():
            ob.reset(L, sub, d, mask=odone, nmax=na if train else None)
        put(S, idx, sub)
        np.testing.assert_array_equal(obs.cpu().numpy(), ob.observe(L, S), err_msg=f"obs step {s}")


@pytest.mark.parametrize("variant,na,train,p", [("medium", 8, False, 0.0), ("medium", 9, True, 0.2), ("large", 16, False, 0.0)])
def test_sampler_step_equals_policy_then_vector_step(wh, variant, na, train, p):
    """BatchedWarehouse.sampler_step (the device policy fused into a 1-step wh_rollout launch, then
    wh_observe) == wh_policy + wh_vector_step(autoreset) step by step: rewards, dones, observation
    rows, episode metrics and the final state, over 230 steps (an episode end), and both == the
    oracle's greedy rollout."""
    import torch

    B, seed, K = 1024, 41, 230
    L = oc.layout_for(variant)
    a = wh.BatchedWarehouse(variant, B, None if train else na, train=train, seed=seed)
    b = wh.BatchedWarehouse(variant, B, None if train else na, train=train, seed=seed)
    sa, sb = a.enable_episode_stats(), b.enable_episode_stats()
    a.reset()
    b.reset()
    S = ob.BState.zeros(L, B, na)
    d = ob.PhiloxDraws(seed, np.arange(B))
    nmax = na if train else None
    ob.reset(L, S, d, nmax=nmax)
    for s in range(K):
        oa, ra, da = a.sampler_step("greedy", p)
        ob_, rb, db = b.vector_step(b.policy("greedy", p), autoreset=True)
        assert torch.equal(ra, rb) and torch.equal(da, db) and torch.equal(oa, ob_), f"step {s}"
        orew, odone, _, _ = ob.step(L, S, ob.greedy(L, S, p, d), d)
        np.testing.assert_array_equal(ra.cpu().numpy(), orew, err_msg=f"step {s}")
        if odone.any():
            ob.reset(L, S, d, mask=odone, nmax=nmax)
        if s % 50 == 0 or s == K - 1:
            np.testing.assert_array_equal(oa.cpu().numpy(), ob.observe(L, S), err_msg=f"obs step {s}")
    assert torch.equal(a.state, b.state)
    for k in ("return_sum", "episodes", "return_min", "return_max", "episode_return"):
        assert torch.equal(getattr(sa, k), getattr(sb, k)), k


@pytest.mark.parametrize("variant,na,train,policy,p,B", [
    ("medium", 8, False, "greedy", 0.0, 65536), ("medium", 8, False, "greedy", 0.3, 1000),
    ("large", 16, False, "greedy", 0.0, 777), ("small", 4, True, "greedy", 0.1, 2049),
    ("medium", 4, False, "random", 0.0, 513), ("large", 16, True, "greedy", 0.0, 300)])
def test_fused_sampler_step_equals_two_launch_route_and_oracle(wh, variant, na, train, policy, p, B):
    """wh_sampler_step without episode metrics takes the fused launch (k_sampler: the step on half of
    each 512-lane workgroup, the rows by all of it, images written from the step's registers).  Its
    rewards, dones and observation rows equal the two-launch route's (wh_policy + wh_vector_step
    with auto-reset = step kernel + k_observe) at every step over 210 steps (episode ends, fresh
    reset rows, a Train variant's new n), full-size and ragged batches (a partial last workgroup);
    the final states are equal; and a sample of envs equals the oracle's rollout."""
    import torch

    seed, K = 17, 210
    L = oc.layout_for(variant)
    a = wh.BatchedWarehouse(variant, B, None if train else na, train=train, seed=seed)
    b = wh.BatchedWarehouse(variant, B, None if train else na, train=train, seed=seed)
    a.reset()
    b.reset()
    ids = np.unique(np.r_[np.arange(min(B, 64)), np.linspace(0, B - 1, 64).astype(np.int64)])
    S = ob.BState.zeros(L, len(ids), na)
    d = ob.PhiloxDraws(seed, ids)
    nmax = na if train else None
    ob.reset(L, S, d, nmax=nmax)
    for s in range(K):
        oa, ra, da = a.sampler_step(policy, p)
        ob_, rb, db = b.vector_step(b.policy(policy, p), autoreset=True)
        assert torch.equal(ra, rb) and torch.equal(da, db), f"step {s}"
        assert torch.equal(oa, ob_), f"obs step {s}"
        acts = ob.greedy(L, S, p, d) if policy == "greedy" else ob.random_actions(S, d)
        orew, odone, _, _ = ob.step(L, S, acts, d)
        np.testing.assert_array_equal(ra.cpu().numpy()[ids], orew, err_msg=f"step {s}")
        if odone.any():
            ob.reset(L, S, d, mask=odone, nmax=nmax)
        if s % 40 == 0 or s == K - 1:
            np.testing.assert_array_equal(oa.cpu().numpy()[ids], ob.observe(L, S), err_msg=f"obs step {s}")
    assert torch.equal(a.state, b.state)


@pytest.mark.parametrize("variant,na,train,policy,p,B,K,stagger,stats", [
    ("medium", 8, False, "greedy", 0.0, 65536, 24, False, False), ("medium", 8, False, "greedy", 0.0, 4096, 40, True, False),
    ("medium", 8, False, "greedy", 0.3, 1000, 7, True, False), ("small", 4, True, "greedy", 0.1, 2049, 12, False, False),
    ("medium", 4, False, "random", 0.0, 513, 9, False, False), ("large", 16, False, "greedy", 0.0, 777, 10, True, False),
    ("medium", 8, False, "greedy", 0.0, 300, 5, False, True)])
def test_sampler_rollout_equals_sampler_steps(wh, variant, na, train, policy, p, B, K, stagger, stats):
    """wh_sampler_rollout (K sampler steps in one launch: the simulation of step k under the row stream
    of step k-1, state in registers, reset slots from 8 steps on) == K calls of wh_sampler_step:
    rewards, dones and observation rows of every step, episode metrics and the final state; launches
    across episode ends with desynchronised episodes (several lanes of a wave ending on one step),
    Train variants, p > 0, random actions, ragged batches; configurations outside the fused kernel
    (Large-16: the step would spill at two waves per SIMD; episode metrics) take the per-step path.
    A sample of envs equals the oracle."""
    import torch

    seed = 29
    L = oc.layout_for(variant)
    a = wh.BatchedWarehouse(variant, B, None if train else na, train=train, seed=seed)
    b = wh.BatchedWarehouse(variant, B, None if train else na, train=train, seed=seed)
    if stats:
        sa, sb = a.enable_episode_stats(), b.enable_episode_stats()
    a.reset()
    b.reset()
    if stagger:
        off = (np.arange(B, dtype=np.int64) * 37) % 200
        a.stagger(off, policy, p)
        b.stagger(off, policy, p)
    ids = np.unique(np.linspace(0, B - 1, 48).astype(np.int64))
    c0 = {kk: v.cpu().numpy()[ids] for kk, v in a.to_canonical().items()}
    for rep in range(2):   # two launches back to back (the second starts from the first's state)
        obs, rew, dn = a.sampler_rollout(K, policy, p)
        for t in range(K):
            ob_, rb, db = b.sampler_step(policy, p)
            assert torch.equal(rew[t], rb) and torch.equal(dn[t], db), f"launch {rep} step {t}"
            assert torch.equal(obs[t], ob_), f"obs launch {rep} step {t}"
    assert torch.equal(a.state, b.state)
    if stats:
        for kk in ("return_sum", "episodes", "return_min", "return_max", "episode_return"):
            assert torch.equal(getattr(sa, kk), getattr(sb, kk)), kk
    # the last launch's final rows for a sample of envs against the oracle, from their start state
    S = ob.BState(pos=c0["pos"].copy(), agent_tgt=c0["agent_target"].copy(), pk_tgt=c0["pickup_target"].copy(),
                  pk_timer=c0["pickup_timer"].copy(), t=c0["t"].astype(np.int64), n=c0["n"].copy(),
                  fresh=c0["fresh"].astype(bool), episode=c0["episode"].astype(np.uint32))
    d = ob.PhiloxDraws(seed, ids)
    nmax = a.agent_slots if train else None
    for t in range(2 * K):
        acts = ob.greedy(L, S, p, d) if policy == "greedy" else ob.random_actions(S, d)
        orew, odone, _, _ = ob.step(L, S, acts, d)
        if odone.any():
            ob.reset(L, S, d, mask=odone, nmax=nmax)
    np.testing.assert_array_equal(obs[K - 1].cpu().numpy()[ids], ob.observe(L, S))
    np.testing.assert_array_equal(rew[K - 1].cpu().numpy()[ids], orew)



def test_sampler_rollout_refuses_wrong_dtype_or_device(wh):
    """Caller-supplied outputs of sampler_rollout / rollout must match the kernel's dtype and device
    exactly: a float16 obs buffer of the right shape would be written past its end."""
    import torch

    env = wh.BatchedWarehouse("small", 64, 4, seed=3, device="cuda:0")
    env.reset()
    K, L = 2, env.obs_len
    with pytest.raises(ValueError):
        env.sampler_rollout(K, obs=torch.empty((K, 64, 4, L), dtype=torch.float16, device="cuda:0"))
    with pytest.raises(ValueError):
        env.sampler_rollout(K, rewards=torch.empty((K, 64, 4), dtype=torch.float32))   # host tensor
    with pytest.raises(ValueError):
        env.sampler_rollout(K, dones=torch.empty((K, 64), dtype=torch.int32, device="cuda:0"))
    with pytest.raises(ValueError):
        env.rollout(K, rewards=torch.empty((K, 64, 4), dtype=torch.bfloat16, device="cuda:0"))
    with pytest.raises(ValueError):
        env.rollout_launcher(K, dones=torch.empty((K, 64), dtype=torch.float32, device="cuda:0"))
    obs, rew, dn = env.sampler_rollout(K)     # allocated by the env: accepted
    assert obs.dtype == torch.float32 and dn.dtype == torch.uint8

@pytest.mark.parametrize("variant,na,train,B,masked,ordered,stats", [
    ("medium", 8, False, 65536, False, False, False), ("medium", 8, False, 1000, True, True, True),
    ("small", 4, True, 2049, True, False, True), ("medium", 4, False, 513, False, True, False),
    ("medium", 2, False, 300, True, True, False)])
def test_fused_vector_step_equals_two_launch_route(wh, variant, na, train, B, masked, ordered, stats):
    """wh_vector_step with observation rows takes one launch (k_sampler's generic instance: external
    actions, optional env mask and action-dict order, episode metrics) where its step code keeps its
    registers; it must equal the two launches it replaces -- the step alone (observe=False) then
    wh_observe -- in rewards, dones (stepped envs), rows of EVERY env (masked-out envs keep theirs),
    episode metrics and state, over 210 steps with auto-reset.  Without mask, order and metrics the
    fused launch runs the fast (fused-rollout) step instance with external actions; the comparison
    then steps b with an all-true mask, i.e. through the generic instance."""
    import torch

    seed, K = 23, 210
    a = wh.BatchedWarehouse(variant, B, None if train else na, train=train, seed=seed)
    b = wh.BatchedWarehouse(variant, B, None if train else na, train=train, seed=seed)
    if stats:
        sa, sb = a.enable_episode_stats(), b.enable_episode_stats()
    a.reset()
    b.reset()
    NA = a.agent_slots
    rng = np.random.default_rng(5)
    for s in range(K):
        acts = torch.from_numpy(rng.integers(0, 9, (B, NA), dtype=np.int32))
        mask = torch.from_numpy(rng.random(B) < 0.6) if masked and s % 2 else None
        order = None
        if ordered and s % 3:
            perm = np.argsort(rng.random((B, NA)), axis=1).astype(np.int32)
            drop = rng.random((B, NA)) < 0.2
            order = torch.from_numpy(np.where(np.cumsum(drop, axis=1) > 0, -1, perm).astype(np.int32))
        oa, ra, da = a.vector_step(acts, autoreset=True, mask=mask, order=order)
        # b: the two launches, and with an all-true mask where a has none, so that b's step is the
        # generic instance while a's (no mask, no order, no metrics) is the fast one
        mb = torch.ones(B, dtype=torch.bool) if mask is None else mask
        _, rb, db = b.vector_step(acts, autoreset=True, mask=mb, order=order, observe=False)
        ob_ = b.observe()
        live = slice(None) if mask is None else mask.to(ra.device)
        assert torch.equal(ra[live], rb[live]) and torch.equal(da[live], db[live]), f"step {s}"
        assert torch.equal(oa, ob_), f"obs step {s}"
    assert torch.equal(a.state, b.state)
    if stats:
        for k in ("return_sum", "episodes", "return_min", "return_max", "episode_return"):
            assert torch.equal(getattr(sa, k), getattr(sb, k)), k


@pytest.mark.parametrize("variant,na,train,B", [("medium", 8, False, 4096), ("medium", 9, True, 1000),
                                                ("large", 16, False, 777), ("large", 5, False, 300),
                                                ("small", 4, True, 2049), ("small", 3, False, 129)])
def test_sampler_observation_rows_equal_wh_observe(wh, variant, na, train, B):
    """The observation rows wh_vector_step and wh_sampler_step return are wh_observe's on the
    state they leave: masked steps, ragged batches (a partial last workgroup), odd agent counts
    (rows not a multiple of 4 floats), Train variants, fresh resets."""
    import torch

    env = wh.BatchedWarehouse(variant, B, None if train else na, train=train, seed=3)
    env.reset()
    g = torch.Generator(device=env.device).manual_seed(1)
    NA = env.agent_slots
    for s in range(260):
        if s % 3 == 0:
            acts = torch.randint(0, 9, (B, NA), device=env.device, dtype=torch.int32, generator=g)
            mask = (torch.rand(B, device=env.device, generator=g) < 0.5) if s % 2 else None
            obs, _, _ = env.vector_step(acts, autoreset=True, mask=mask)
        else:
            obs, _, _ = env.sampler_step("greedy", 0.1 if s % 2 else 0.0)
        fused = obs.clone()
        ref = env.observe()
        assert torch.equal(fused, ref), f"step {s}"



@pytest.mark.parametrize("variant,na,train,B", [("medium", 8, False, 4096), ("medium", 9, True, 1000),
                                                ("large", 16, False, 777), ("small", 4, True, 2049),
                                                ("small", 3, False, 129), ("small", 1, False, 150),
                                                ("medium", 2, False, 333)])
def test_vector_step_x_equals_vector_step_then_observe_x(wh, variant, na, train, B):
    """wh_vector_step_x (the step launch writing the policy's fragment-order operand) == the same
    wh_vector_step without rows followed by wh_observe_x, byte for byte, with equal rewards, dones
    and states: the fast instance (every env stepped, ascending order), masked steps and dict order
    (the generic instance), ragged batches, odd agent counts, Train variants, Large-16 (two
    launches: its step code does not fit the fused launch)."""
    import torch

    a = wh.BatchedWarehouse(variant, B, None if train else na, train=train, seed=3)
    b = wh.BatchedWarehouse(variant, B, None if train else na, train=train, seed=3)
    a.reset()
    b.reset()
    g = torch.Generator(device=a.device).manual_seed(1)
    NA = a.agent_slots
    for s in range(230):
        acts = torch.randint(0, 9, (B, NA), device=a.device, dtype=torch.int32, generator=g)
        mask = (torch.rand(B, device=a.device, generator=g) < 0.5) if s % 5 == 1 else None
        order = None
        if s % 7 == 3:
            order = torch.argsort(torch.rand((B, NA), device=a.device, generator=g), dim=1).to(torch.int32)
        xa, ra, da = a.vector_step_x(acts, autoreset=True, mask=mask, order=order)
        _, rb, db = b.vector_step(acts, autoreset=True, observe=False, mask=mask, order=order)
        xb = b.observe_x()
        assert torch.equal(xa, xb), f"step {s}"
        keep = torch.ones(B, dtype=torch.bool, device=a.device) if mask is None else mask
        assert torch.equal(ra[keep], rb[keep]) and torch.equal(da[keep], db[keep]), f"step {s}"
        assert torch.equal(a.state, b.state), f"step {s}"


@pytest.mark.parametrize("variant,na,train,p,graph", [("medium", 8, False, 0.0, False), ("medium", 9, True, 0.2, False),
                                                      ("large", 16, False, 0.0, True), ("small", 4, True, 0.1, True)])
def test_sampler_pipeline_equals_sampler_step(wh, variant, na, train, p, graph):
    """SamplerPipeline (wh_sampler_step_to into the other state buffer on the current stream, the
    observation rows of step s on a side stream while step s + 1 runs) == sampler_step step by
    step: rewards, dones, observation rows, episode metrics and the final state over 216 steps
    (an episode end), eagerly and as a captured CUDA graph of 4-step blocks (the bench's form: an
    even block, so every replay starts from the same state buffer)."""
    import torch

    from warehouse.vector import SamplerPipeline

    B, seed, K, G = 2048 + 77, 5, 216, 4
    a = wh.BatchedWarehouse(variant, B, None if train else na, train=train, seed=seed)
    b = wh.BatchedWarehouse(variant, B, None if train else na, train=train, seed=seed)
    sa, sb = a.enable_episode_stats(), b.enable_episode_stats()
    a.reset()
    b.reset()
    pipe = SamplerPipeline(a, "greedy", p)
    dev = a.device
    if graph:
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize(dev)
        with torch.cuda.graph(g):   # capture launches nothing: replays start from the reset state
            pipe.begin()
            outs = [pipe.step() for _ in range(G)]
            pipe.end()
        torch.cuda.synchronize(dev)
    s = 0
    while s < K:
        if graph:
            g.replay()
            got = outs
        else:
            got = [pipe.step()]
        torch.cuda.synchronize(dev)
        for j, (oa, ra, da) in enumerate(got):
            ob_, rb, db = b.sampler_step("greedy", p)
            s += 1
            if j < len(got) - 2:   # its buffers were reused by step j + 2 of the block
                continue
            assert torch.equal(ra, rb), f"rewards step {s}"
            assert torch.equal(da, db), f"dones step {s}"
            assert torch.equal(oa, ob_), f"obs step {s}"
    assert torch.equal(a.state, b.state)   # (every step's rewards also enter the episode metrics)
    for k in ("return_sum", "episodes", "return_min", "return_max", "episode_return"):
        assert torch.equal(getattr(sa, k), getattr(sb, k)), k
