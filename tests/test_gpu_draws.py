"""Statistical parity of the device's philox draws with the reference's draw LAWS (philox
mode is validated statistically; the bit-exact stream is the injected-draw mode's job).

The reference draws every random choice from numpy's global MT19937 stream:
  * reset (core.py:191-221): spawn cells uniform over interior non-pickup cells (rejection loop),
    choice(P, R, replace=False) pickups, choice(Dp, R, replace=False) targets; Train variants draw
    n ~ randint(1, Nmax+1) (variants.py:73-74);
  * regeneration (core.py:338-351): inactive[permutation(|inactive|)[:k]] points and
    permutation(Dp)[:k] targets, i.e. uniformly random ORDERED k-subsets of each;
  * the greedy solver's coin (solvers.py:44): uniform() < p, then action_space.sample().
These tests run the HIP kernels (through the C ABI) on 65,536 independent env ids and check the
observed frequencies with chi-square / binomial tests at a 1e-6 significance floor (the seeds are
fixed, so the outcome is deterministic; the floor only keeps the test far from the edge).
"""
import itertools

import numpy as np
import pytest
from scipy import stats

from oracle import core as oc

pytestmark = pytest.mark.gpu
ALPHA = 1e-6


@pytest.fixture(scope="module")
def wh():
    import torch

    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    import warehouse

    return warehouse


def canon(env):
    return {k: v.cpu().numpy() for k, v in env.to_canonical().items()}


def chi2_uniform(counts):
    counts = np.asarray(counts, np.float64).ravel()
    exp = counts.sum() / len(counts)
    chi2 = ((counts - exp) ** 2 / exp).sum()
    return stats.chi2.sf(chi2, len(counts) - 1)


def test_device_reset_law(wh):
    """Train-variant reset: n uniform on 1..Nmax, live agents' spawn cells uniform over the interior
    non-pickup cells, R distinct pickups and R distinct targets, each point / target equally likely."""
    B = 65536
    env = wh.BatchedWarehouse("medium", B, train=True, seed=99)
    env.reset()
    c = canon(env)
    L = oc.layout_for("medium")
    nmax = 9
    n = c["n"]
    assert n.min() >= 1 and n.max() <= nmax
    assert chi2_uniform(np.bincount(n, minlength=nmax + 1)[1:]) > ALPHA
    live = np.arange(nmax)[None, :] < n[:, None]
    cells = c["pos"][live]
    pick = {(int(x), int(y)) for x, y in L.pickup_xy()}
    valid = [(x, y) for x in range(1, L.D - 1) for y in range(1, L.D - 1) if (x, y) not in pick]
    idx = {v: i for i, v in enumerate(valid)}
    ci = np.array([idx[(int(x), int(y))] for x, y in cells])     # KeyError = spawn outside the law's support
    assert chi2_uniform(np.bincount(ci, minlength=len(valid))) > ALPHA
    pt = c["pickup_target"]
    assert ((pt > -1).sum(1) == L.R).all()
    assert chi2_uniform((pt > -1).sum(0)) > ALPHA                 # each point open with prob R/P
    tg = np.sort(np.where(pt > -1, pt, 10 ** 6), axis=1)[:, : L.R]
    assert (np.diff(tg, axis=1) > 0).all()                         # targets distinct at reset
    assert chi2_uniform(np.bincount(tg.ravel(), minlength=L.Dp)) > ALPHA


def test_device_reset_subset_law(wh):
    """Reset requests (Small, P=16, R=4): all C(16,4) subsets equally likely (Floyd's algorithm on
    the device is the law of choice(P, R, replace=False)), and the target of the lowest open point
    uniform over the delivery points (pairing with a uniform ordered target tuple)."""
    from math import comb

    B = 65536
    env = wh.BatchedWarehouse("small", B, 4, seed=123)
    env.reset()
    c = canon(env)
    L = oc.layout_for("small")
    open_ = c["pickup_target"] > -1
    assert (open_.sum(1) == L.R).all()
    code = (open_.astype(np.int64) << np.arange(L.P)).sum(1)
    counts = np.unique(code, return_counts=True)[1]
    assert len(counts) == comb(L.P, L.R)
    assert chi2_uniform(counts) > ALPHA
    first = c["pickup_target"][np.arange(B), open_.argmax(1)]
    assert chi2_uniform(np.bincount(first, minlength=L.Dp)) > ALPHA


def _regen_state(wh, k, B, seed):
    """B copies of one Medium state (one idle agent far from every pickup, staying put) with R-k open
    requests, so the next step's only random event is regeneration of exactly k requests."""
    L = oc.layout_for("medium")
    env = wh.BatchedWarehouse("medium", B, 1, seed=seed)
    rng = np.random.default_rng(3)
    open_pts = np.sort(rng.choice(L.P, L.R - k, replace=False))
    pk_tgt = np.full((B, L.P), -1, np.int32)
    pk_tgt[:, open_pts] = rng.choice(L.Dp, L.R - k, replace=False)
    timer = np.where(pk_tgt > -1, 150, -1).astype(np.int32)
    env.from_canonical(dict(pos=np.ones((B, 1, 2), np.int32), agent_target=np.full((B, 1), -1, np.int32),
                            pickup_target=pk_tgt, pickup_timer=timer, t=np.full(B, 10, np.int32),
                            n=np.ones(B, np.int32), episode=np.full(B, 5, np.int64)))
    return env, L, open_pts


@pytest.mark.parametrize("k", [1, 2])
def test_device_regeneration_law(wh, k):
    """core.py:338-351 with philox draws: exactly k points reopen, each inactive point equally likely
    (for k = 2 every unordered pair equally likely), targets distinct and uniform; for k = 2 the
    (lower point's target, higher point's target) pair is uniform over ordered distinct pairs."""
    B = 65536
    env, L, open_pts = _regen_state(wh, k, B, seed=11 + k)
    env.step(np.full((B, 1), 4, np.int32))                        # stay: no pickup, no delivery
    c = canon(env)
    pt = c["pickup_target"]
    new = (pt > -1)
    new[:, open_pts] = False
    assert (new.sum(1) == k).all()
    inactive = np.setdiff1d(np.arange(L.P), open_pts)
    assert not new[:, open_pts].any()
    assert chi2_uniform(new[:, inactive].sum(0)) > ALPHA
    assert (c["pickup_timer"][new] == L.W).all()                  # a reopened request waits W steps
    pts = np.nonzero(new)[1].reshape(B, k)                         # ascending point index per env
    tgs = pt[np.arange(B)[:, None], pts]
    if k == 1:
        assert chi2_uniform(np.bincount(tgs[:, 0], minlength=L.Dp)) > ALPHA
    else:
        assert (tgs[:, 0] != tgs[:, 1]).all()
        pair_id = {p: i for i, p in enumerate(itertools.combinations(inactive, 2))}
        pc = np.bincount([pair_id[(a, b)] for a, b in pts], minlength=len(pair_id))
        assert chi2_uniform(pc) > ALPHA
        ordered = tgs[:, 0] * L.Dp + tgs[:, 1]
        cnt = np.bincount(ordered, minlength=L.Dp * L.Dp).reshape(L.Dp, L.Dp)
        off = ~np.eye(L.Dp, dtype=bool)
        assert chi2_uniform(cnt[off]) > ALPHA
        for j in range(2):
            assert chi2_uniform(np.bincount(tgs[:, j], minlength=L.Dp)) > ALPHA


@pytest.mark.parametrize("p", [0.1, 0.5])
def test_device_greedy_coin(wh, p):
    """solvers.py:44: every agent flips its own coin; with probability p the action is uniform over
    the 9 moves (so it differs from the greedy one with probability 8p/9), independently per agent
    slot, and a replaced action is uniform over the 8 others."""
    B = 65536
    env = wh.BatchedWarehouse("medium", B, 8, seed=21)
    env.reset()
    env.rollout(37, "greedy", 0.0)                                  # agents spread over the grid
    g = env.policy("greedy", 0.0).cpu().numpy().copy()
    a = env.policy("greedy", p).cpu().numpy().copy()
    diff = a != g
    N = diff.size
    exp = N * p * 8 / 9
    assert abs(diff.sum() - exp) < 6 * np.sqrt(exp * (1 - p * 8 / 9))
    per_slot = diff.sum(0)
    assert chi2_uniform(per_slot) > ALPHA
    # replaced actions: uniform over the 8 actions other than the greedy one
    pv = []
    for ga in range(9):
        sel = diff & (g == ga)
        if sel.sum() < 400:
            continue
        cnt = np.bincount(a[sel], minlength=9)
        assert cnt[ga] == 0
        pv.append(chi2_uniform(np.delete(cnt, ga)))
    assert pv and min(pv) > ALPHA


def test_device_random_policy_uniform(wh):
    """The random policy (RANDOM stream) draws each agent's action uniformly over the 9 moves."""
    B = 65536
    env = wh.BatchedWarehouse("small", B, 4, seed=5)
    env.reset()
    a = env.policy("random").cpu().numpy()
    assert chi2_uniform(np.bincount(a.ravel(), minlength=9)) > ALPHA
    assert chi2_uniform(np.bincount(a[:, 0] * 9 + a[:, 1], minlength=81)) > ALPHA   # slots independent
