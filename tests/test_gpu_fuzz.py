"""GPU fuzz parity: one transition from many random adversarial states (the G2 recipe --
agents crowded on a few cells, on pickup blocks, hugging delivery cells, overlapping; timers about
to expire; t at T-1/T) with random actions and random (possibly partial) action-dict orders,
kernel vs the oracle (which the reference's own fixtures pin).  Regeneration draws are injected
the way the drop-in class does it: phase PRE_REGEN reports |inactive|, the host draws, phase
REGEN finishes.  Bit-exact state, rewards, dones and observation rows."""
import numpy as np
import pytest

from oracle import batched as ob
from oracle import core as oc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def wh():
    import torch

    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    import warehouse

    return warehouse


def random_states(L, B, nmax, rng, ts=None, full=False):
    P, Dp, R, W, D = L.P, L.Dp, L.R, L.W, L.D
    pk, dl, _, _ = ob.tables(L)
    n = rng.randint(1, nmax + 1, size=B)
    pos = np.zeros((B, nmax, 2), np.int32)
    atg = np.full((B, nmax), -1, np.int32)
    tgt = np.full((B, P), -1, np.int32)
    tim = np.full((B, P), -1, np.int32)
    t = rng.choice(ts if ts is not None else [0, 5, L.T - 1, L.T, 150], size=B).astype(np.int64)
    for e in range(B):
        k = n[e]
        mode = rng.randint(4)
        if mode == 0:
            cx, cy = rng.randint(0, D - 2, size=2)
            p = np.stack([cx + rng.randint(0, 3, k), cy + rng.randint(0, 3, k)], 1)
        elif mode == 1:
            c = pk[rng.randint(P)]
            p = np.stack([c[0] + rng.randint(-1, 2, k), c[1] + rng.randint(-1, 2, k)], 1)
        elif mode == 2:
            c = dl[rng.randint(Dp)]
            p = np.stack([c[0] + rng.randint(-1, 2, k), c[1] + rng.randint(-1, 2, k)], 1)
        else:
            p = rng.randint(0, D, size=(k, 2))
        pos[e, :k] = np.clip(p, 0, D - 1)
        na = R if full else rng.randint(max(0, R - k), R + 1)
        sel = rng.choice(P, na, replace=False)
        tgt[e, sel] = rng.randint(0, Dp, na)
        tim[e, sel] = np.where(rng.rand(na) < 0.3, 1, rng.randint(1, W + 1, na))
        a = np.where(rng.rand(k) < 0.4, rng.randint(0, Dp, k), -1)
        for i in range(k):
            if a[i] >= 0 and rng.rand() < 0.5:
                pos[e, i] = np.clip(dl[a[i]] + rng.randint(-1, 2, 2), 0, D - 1)
        atg[e, :k] = a
    return n.astype(np.int32), pos, atg, tgt, tim, t


def run_fuzz(wh, variant, ordered, seed, ts=None, B=3000):
    L = oc.layout_for(variant)
    nmax = oc.VARIANTS[variant]["nmax"]
    rng = np.random.RandomState(seed)
    n, pos, atg, tgt, tim, t = random_states(L, B, nmax, rng, ts)
    env = wh.BatchedWarehouse(variant, B, train=True)
    env.from_canonical(dict(pos=pos, agent_target=atg, pickup_target=tgt, pickup_timer=tim, t=t, n=n))
    S = ob.BState(pos=pos.copy(), agent_tgt=atg.copy(), pk_tgt=tgt.copy(), pk_timer=tim.copy(), t=t.copy(),
                  n=n.copy(), fresh=np.zeros(B, bool), episode=np.zeros(B, np.uint32))
    acts = rng.randint(0, 9, size=(B, nmax)).astype(np.int32)
    order = np.full((B, nmax), -1, np.int32)
    for e in range(B):
        perm = rng.permutation(n[e]) if ordered else np.arange(n[e])
        if ordered and rng.rand() < 0.3:
            perm = perm[: rng.randint(0, n[e] + 1)]            # agents missing from the dict
        order[e, : len(perm)] = perm
    env.step(acts, order=order if ordered else None, phase=1)           # PRE_REGEN
    nin = env.n_inactive.cpu().numpy()
    regen = np.zeros((B, 2 * L.R), np.int32)
    for e in range(B):
        k = L.R - L.P + int(nin[e])
        if k > 0:
            regen[e, :k] = rng.permutation(int(nin[e]))[:k]
            regen[e, L.R:L.R + k] = rng.permutation(L.Dp)[:k]
    rew, done = env.step(None, regen=regen, phase=2)                       # REGEN
    orew, odone, on_in, ok = ob.step(L, S, acts, ob.Injected(rpos=regen[:, :L.R], rtgt=regen[:, L.R:]),
                                     order=order if ordered else None)
    np.testing.assert_array_equal(nin, on_in)
    c = {k: v.cpu().numpy() for k, v in env.to_canonical().items()}
    np.testing.assert_array_equal(c["pos"], S.pos)
    np.testing.assert_array_equal(c["agent_target"], S.agent_tgt)
    np.testing.assert_array_equal(c["pickup_target"], S.pk_tgt)
    np.testing.assert_array_equal(c["pickup_timer"], S.pk_timer)
    np.testing.assert_array_equal(c["t"], S.t)
    np.testing.assert_array_equal(rew.cpu().numpy(), orew)
    np.testing.assert_array_equal(done.cpu().numpy().astype(bool), odone)
    np.testing.assert_array_equal(env.observe().cpu().numpy(), ob.observe(L, S))


@pytest.mark.parametrize("variant", ["small", "medium", "large"])
@pytest.mark.parametrize("ordered", [False, True])
def test_fuzz_single_transitions(wh, variant, ordered):
    nmax = oc.VARIANTS[variant]["nmax"]
    run_fuzz(wh, variant, ordered, 100 + nmax + (7 if ordered else 0))


@pytest.mark.parametrize("variant", ["small", "medium", "large"])
def test_fuzz_expiry_far_below_w(wh, variant):
    """Whole waves at t < W holding requests about to expire (states no episode reaches: a request
    opened at t0 >= 0 lives W steps).  The kernel must not assume reachability to skip expiry."""
    nmax = oc.VARIANTS[variant]["nmax"]
    run_fuzz(wh, variant, False, 300 + nmax, ts=[0, 5, 150])


@pytest.mark.parametrize("variant", ["small", "medium", "large"])
def test_fused_rollout_from_fuzzed_states(wh, variant):
    """wh_rollout (greedy, philox regeneration and auto-reset, K steps in one launch) started from
    fuzzed states -- t far below W with requests about to expire, crowded agents, t at T-1 -- against
    the oracle stepping the same philox contract.  Every state holds R open requests, as every
    reachable pre-step state does (the solver reads exactly R request rows, solvers.py:53-58)."""
    import torch

    L = oc.layout_for(variant)
    nmax = oc.VARIANTS[variant]["nmax"]
    B, K, seed = 2048, 40, 11
    rng = np.random.RandomState(500 + nmax)
    n, pos, atg, tgt, tim, t = random_states(L, B, nmax, rng, ts=[0, 5, 150, L.T - 1], full=True)
    env = wh.BatchedWarehouse(variant, B, train=True, seed=seed)
    env.from_canonical(dict(pos=pos, agent_target=atg, pickup_target=tgt, pickup_timer=tim, t=t, n=n))
    S = ob.BState(pos=pos.copy(), agent_tgt=atg.copy(), pk_tgt=tgt.copy(), pk_timer=tim.copy(), t=t.copy(),
                  n=n.copy(), fresh=np.zeros(B, bool), episode=np.zeros(B, np.uint32))
    rew = torch.zeros((K, B, nmax), device=env.device)
    dn = torch.zeros((K, B), dtype=torch.uint8, device=env.device)
    env.rollout(K, "greedy", 0.0, rewards=rew, dones=dn)
    d = ob.PhiloxDraws(seed, np.arange(B))
    for s in range(K):
        orew, odone, _, _ = ob.step(L, S, ob.greedy(L, S, 0.0, d), d)
        np.testing.assert_array_equal(rew[s].cpu().numpy(), orew, err_msg=f"step {s}")
        np.testing.assert_array_equal(dn[s].cpu().numpy().astype(bool), odone, err_msg=f"step {s}")
        if odone.any():
            ob.reset(L, S, d, mask=odone, nmax=nmax)
    c = {k: v.cpu().numpy() for k, v in env.to_canonical().items()}
    np.testing.assert_array_equal(c["pos"], S.pos)
    np.testing.assert_array_equal(c["agent_target"], S.agent_tgt)
    np.testing.assert_array_equal(c["pickup_target"], S.pk_tgt)
    np.testing.assert_array_equal(c["pickup_timer"], S.pk_timer)
    np.testing.assert_array_equal(c["t"], S.t)
