"""GPU numerics of the SAC policy kernel (wh_mlp_forward) against a plain PyTorch reference of the
same network (scripts/experiments/warehouse-*-sac policy_model shapes).

Tolerances (stated here, checked below):
  * logits vs the float64 reference that rounds weights, inputs and hidden activations to bf16
    exactly where the kernel does: |d| <= 2e-3 + 2e-3 |ref|  (left: f32 accumulation order and the
    rare bf16 rounding flip of a hidden unit).
  * logits vs the plain fp32 network (no bf16 anywhere): |d| <= 3e-2 max|ref|  (the bf16 error).
  * argmax actions equal the reference's wherever its top-2 margin exceeds 1e-2.
  * explore=1 samples follow softmax(logits): chi-square over 9 bins below the 1e-4 quantile.
  * precision="f32" (exact f32 MFMA): logits vs the float64 network (the reference policy is fp32)
    |d| <= 1e-5 max|ref| per row (measured ~1e-7: f32 rounding in a different summation order), and
    argmax equal to the float64 reference's on EVERY row whose top-2 margin exceeds 1e-5 max|ref|
    (a closer pair is a tie at fp32 precision; the test reports how many such rows exist).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def wh():
    import torch

    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    import warehouse
    import warehouse.policy  # noqa: F401

    return warehouse


def reference_logits(w, x, bf16):
    import torch

    def q(a):
        t = torch.as_tensor(np.asarray(a), dtype=torch.float32)
        return (t.to(torch.bfloat16) if bf16 else t).to(torch.float64)

    h = q(x)
    h = torch.relu(h @ q(w["w0"]).T + torch.as_tensor(w["b0"], dtype=torch.float64))
    h = q(h.to(torch.float32)) if bf16 else h
    h = torch.relu(h @ q(w["w1"]).T + torch.as_tensor(w["b1"], dtype=torch.float64))
    h = q(h.to(torch.float32)) if bf16 else h
    return (h @ q(w["w2"]).T + torch.as_tensor(w["b2"], dtype=torch.float64)).numpy()


def observation_rows(wh, variant, na, B, extra_random):
    import torch

    env = wh.BatchedWarehouse(variant, B, na, seed=4)
    env.reset()
    env.rollout(23, "greedy", 0.1)
    rows = env.observe().reshape(-1, env.obs_len)
    g = torch.Generator(device="cpu").manual_seed(1)
    rnd = (torch.randn((extra_random, env.obs_len), generator=g) * 6).to(rows.device)
    return torch.cat([rows, rnd]).contiguous()


@pytest.mark.parametrize("variant,na", [("small", 4), ("medium", 8), ("large", 16)])
def test_mlp_logits_and_argmax_vs_torch(wh, variant, na):
    net = wh.policy.MLPPolicy(variant, seed=11)
    x = observation_rows(wh, variant, na, 61, 203)          # ragged row count
    acts, lg = net(x, logits=True)
    lg, acts = lg.cpu().numpy(), acts.cpu().numpy()
    xc = x.cpu().numpy()
    ref = reference_logits(net.weights, xc, bf16=True)
    np.testing.assert_array_less(np.abs(lg - ref), 2e-3 + 2e-3 * np.abs(ref))
    ref32 = reference_logits(net.weights, xc, bf16=False)
    assert np.abs(lg - ref32).max() <= 3e-2 * np.abs(ref32).max()
    srt = np.sort(ref, axis=1)
    clear = srt[:, -1] - srt[:, -2] > 1e-2
    assert clear.mean() > 0.9
    np.testing.assert_array_equal(acts[clear], ref.argmax(1)[clear])
    # actions-only launch gives the same argmax
    a2, none = net(x)
    assert none is None
    np.testing.assert_array_equal(a2.cpu().numpy(), acts)


def test_mlp_explore_samples_softmax(wh):
    import torch

    net = wh.policy.MLPPolicy("medium", seed=3)
    x = observation_rows(wh, "medium", 8, 1, 0)[:1]
    rows = 1 << 17
    xx = x.expand(rows, -1).contiguous()
    _, lg = net(xx[:1], logits=True)
    p = torch.softmax(lg[0].double(), 0).cpu().numpy()
    acts, _ = net(xx, explore=True, seed=9, step=5)
    cnt = np.bincount(acts.cpu().numpy(), minlength=9)
    exp = p * rows
    chi2 = ((cnt - exp) ** 2 / exp).sum()
    assert chi2 < 37.0      # chi-square, 8 dof, p = 1e-5
    acts2, _ = net(xx, explore=True, seed=9, step=5)
    np.testing.assert_array_equal(acts.cpu().numpy(), acts2.cpu().numpy())      # counter-based: reproducible
    acts3, _ = net(xx, explore=True, seed=9, step=6)
    assert (acts3.cpu().numpy() != acts.cpu().numpy()).any()


def test_mlp_edge_cases(wh):
    import ctypes

    import torch
    from warehouse import _native as nat

    net = wh.policy.MLPPolicy("small", seed=1)
    empty = torch.empty((0, net.in_dim), device=net.device)
    a, _ = net(empty)
    assert a.numel() == 0
    one = torch.zeros((1, net.in_dim), device=net.device)
    _, lg = net(one, logits=True)
    ref = reference_logits(net.weights, np.zeros((1, net.in_dim), np.float32), bf16=True)
    np.testing.assert_allclose(lg.cpu().numpy(), ref, atol=2e-3, rtol=2e-3)
    bad = nat.WhMlpDesc(net.in_dim, 128, 128, 9, 0)
    assert nat.lib().wh_mlp_forward(ctypes.byref(bad), net.packed.data_ptr(), 1, one.data_ptr(), None,
                                    None, 0, 0, 0, None) == nat.WH_ENOTSUP


@pytest.mark.parametrize("variant,na,train,operand", [("medium", 8, False, "fragments"), ("medium", 8, False, "rows"),
                                                       ("medium", 9, False, "auto"), ("medium", None, True, "auto"),
                                                       ("large", 5, False, "auto"), ("small", None, True, "auto")])
def test_policy_rollout_transitions_vs_oracle(wh, variant, na, train, operand):
    """The device policy loop (network forward -> wh_vector_step with auto-reset) for 230 steps, on
    the fragment-order operand and on the f32 rows: actions equal a separate forward on the same
    rows, and every transition equals the oracle's given those actions (philox draws).  Includes
    the default BatchedWarehouse('medium', B) (9 agent slots), the Train variants (per-episode n)
    and agent counts whose observation workgroups do not hold whole 32-row fragment tiles."""
    import torch

    from oracle import batched as ob
    from oracle import core as oc

    B, seed = 512, 17
    L = oc.layout_for(variant)
    env = wh.BatchedWarehouse(variant, B, na, train=train, seed=seed)
    na = env.agent_slots
    env.reset()
    net = wh.policy.MLPPolicy(variant, seed=2)
    S = ob.BState.zeros(L, B, na)
    d = ob.PhiloxDraws(seed, np.arange(B))
    nmax = na if train else None
    ob.reset(L, S, d, nmax=nmax)
    log = []

    def record(s, acts, rew, done):
        log.append((acts.cpu().numpy().copy(), rew.cpu().numpy().copy(), done.cpu().numpy().copy()))

    obs0 = env.observe().clone()
    ref_a0, _ = net(obs0.view(B * na, -1), explore=True, seed=1, step=0)
    wh.policy.policy_rollout(env, net, 230, explore=True, seed=1, record=record, operand=operand)
    np.testing.assert_array_equal(log[0][0].reshape(-1), ref_a0.cpu().numpy())
    for s, (a, rew, done) in enumerate(log):
        orew, odone, _, _ = ob.step(L, S, a, d)
        np.testing.assert_array_equal(rew, orew, err_msg=f"step {s}")
        np.testing.assert_array_equal(done.astype(bool), odone)
        if odone.any():
            ob.reset(L, S, d, mask=odone, nmax=nmax)
    np.testing.assert_array_equal(env.observe().cpu().numpy(), ob.observe(L, S))
    assert len({int(x) for x in np.unique(np.concatenate([a.reshape(-1) for a, _, _ in log]))}) > 1


@pytest.mark.parametrize("variant,na", [("small", 4), ("medium", 8), ("large", 16)])
def test_mlp_f32_matches_fp32_reference(wh, variant, na):
    net = wh.policy.MLPPolicy(variant, seed=11, precision="f32")
    x = observation_rows(wh, variant, na, 509, 3001)        # ragged row count, observation + random rows
    acts, lg = net(x, logits=True)
    lg, acts = lg.cpu().numpy().astype(np.float64), acts.cpu().numpy()
    ref = reference_logits(net.weights, x.cpu().numpy(), bf16=False)          # float64 network
    scale = np.abs(ref).max(axis=1, keepdims=True)
    rel = np.abs(lg - ref) / scale
    assert rel.max() <= 1e-5, rel.max()
    srt = np.sort(ref, axis=1)
    tie = (srt[:, -1] - srt[:, -2]) <= 1e-5 * scale[:, 0]
    assert tie.sum() <= 2                                     # ties at fp32 precision are rare
    np.testing.assert_array_equal(acts[~tie], ref.argmax(1)[~tie])
    # and against torch's own float32 network on the same rows
    import torch

    t = {k: torch.as_tensor(v) for k, v in net.weights.items()}
    xc = x.cpu()
    h = torch.relu(xc @ t["w0"].T + t["b0"])
    h = torch.relu(h @ t["w1"].T + t["b1"])
    z32 = (h @ t["w2"].T + t["b2"]).numpy().astype(np.float64)
    assert (np.abs(lg - z32) / scale).max() <= 1e-5
    a2, _ = net(x)
    np.testing.assert_array_equal(a2.cpu().numpy(), acts)


def test_mlp_f32_edge_cases(wh):
    import torch

    net = wh.policy.MLPPolicy("medium", seed=5, precision="f32")
    a, _ = net(torch.empty((0, net.in_dim), device=net.device))
    assert a.numel() == 0
    for rows in (1, 31, 33, 127):
        x = torch.randn((rows, net.in_dim), device=net.device) * 4
        _, lg = net(x, logits=True)
        ref = reference_logits(net.weights, x.cpu().numpy(), bf16=False)
        assert np.abs(lg.cpu().numpy() - ref).max() <= 1e-5 * np.abs(ref).max()
    with pytest.raises(ValueError):
        wh.policy.MLPPolicy("medium", precision="fp16")


def frag_reference(rows_f32, kq):
    """numpy: f32 rows [N, L] -> wh_observe_x's layout [tiles, kq, 64 lanes, 8] bf16 bits."""
    import torch

    N, L = rows_f32.shape
    tiles = (N + 31) // 32
    X = np.zeros((tiles * 32, 16 * kq), np.float32)
    X[:N, :L] = rows_f32
    X[:, L:L + 2] = 1.0
    bits = torch.as_tensor(X).to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)
    out = np.zeros((tiles, kq, 64, 8), np.uint16)
    for h in range(2):
        for q in range(kq):
            out[:, q, 32 * h:32 * h + 32, :] = bits.reshape(tiles, 32, 16 * kq)[:, :, 16 * q + 8 * h:16 * q + 8 * h + 8]
    return out


@pytest.mark.parametrize("variant,na,B", [("small", 4, 100), ("medium", 8, 61), ("large", 16, 37),
                                          ("medium", 9, 150), ("large", 5, 70), ("small", 3, 131),
                                          ("small", 1, 130), ("medium", 1, 70), ("large", 1, 200),
                                          ("medium", 2, 99), ("large", 2, 77)])
def test_observe_x_fragments_and_forward_x(wh, variant, na, B):
    """wh_observe_x writes exactly the bf16 fragment image of wh_observe's rows (bias columns 1.0,
    padding 0, ragged last tile), and wh_mlp_forward_x on it gives bit-identical logits and actions
    to wh_mlp_forward on the f32 rows (the kernel rounds those to bf16 the same way)."""
    import torch

    env = wh.BatchedWarehouse(variant, B, na, seed=8)
    env.reset()
    env.rollout(31, "greedy", 0.1)
    xf, obs = env.observe_x(obs=True)
    rows = obs.reshape(-1, env.obs_len)
    kq = (env.obs_len + 2 + 15) // 16
    ref = frag_reference(rows.cpu().numpy(), kq)
    got = xf.cpu().numpy().view(np.uint16).reshape(ref.shape)
    real = np.zeros(ref.shape[:1] + (32,), bool)
    real.reshape(-1)[:rows.shape[0]] = True
    for q in range(kq):        # rows past B*NA: not compared (never emitted by the MLP)
        for h in range(2):
            np.testing.assert_array_equal(got[:, q, 32 * h:32 * h + 32][real], ref[:, q, 32 * h:32 * h + 32][real])
    np.testing.assert_array_equal(env.observe().cpu().numpy(), obs.cpu().numpy())
    net = wh.policy.MLPPolicy(variant, seed=13)
    a1, l1 = net(rows, logits=True, step=0)
    a2, l2 = net.forward_x(xf, rows.shape[0], logits=True, step=0)
    assert torch.equal(l1, l2) and torch.equal(a1, a2)
    a3, _ = net(rows, explore=True, seed=5, step=9)
    a4, _ = net.forward_x(xf, rows.shape[0], explore=True, seed=5, step=9)
    assert torch.equal(a3, a4)
