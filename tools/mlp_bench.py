"""Time wh_mlp_forward (SAC policy forward, argmax) on B=65536 envs' agent rows per variant.
Prints us/launch and dense bf16 TFLOP/s (2 * rows * (in*h0 + h0*h1 + h1*9))."""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rllib-warehouse_amd")]
import torch  # noqa: E402
import warehouse  # noqa: E402
import warehouse.policy as wp  # noqa: E402

B = int(os.environ.get("MLP_B", 65536))
VARIANTS = os.environ.get("MLP_VARIANTS", "small,medium,large").split(",")
for abl, variant, na in [(a, v, n) for a in os.environ.get("MLP_ABLATE", "0").split(",")
                         for v, n in (("small", 4), ("medium", 8), ("large", 16)) if v in VARIANTS]:
    os.environ["WH_MLP_ABLATE"] = abl
    net = wp.MLPPolicy(variant, seed=1)
    rows = B * na
    x = torch.randn((rows, net.in_dim), device="cuda") * 4
    acts = torch.empty(rows, dtype=torch.int32, device="cuda")
    if os.environ.get("MLP_X") == "1":
        # the fragment-order operand (wh_observe_x's layout): random bf16 of magnitude [0.5, 1)
        kq = (net.in_dim + 2 + 15) // 16
        bits = torch.randint(0, 1 << 15, ((rows + 31) // 32, kq, 64, 8), device="cuda", dtype=torch.int32)
        xf = ((bits & 0x807F) | 0x3F00).to(torch.int16).view(torch.uint8).contiguous()
        fwd = lambda: net.forward_x(xf, rows, actions=acts, step=0)   # noqa: E731
    else:
        fwd = lambda: net(x, actions=acts, step=0)   # noqa: E731
    for _ in range(3):
        fwd()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    t0.record()
    for _ in range(reps):
        fwd()
    t1.record()
    torch.cuda.synchronize()
    us = t0.elapsed_time(t1) / reps * 1e3
    h0, h1 = net.hidden
    flop = 2.0 * rows * (net.in_dim * h0 + h0 * h1 + h1 * 9)
    print(f"ablate={abl} {variant:6s} rows={rows:8d} [{net.in_dim},{h0},{h1},9] {us:9.1f} us  {flop / us / 1e6:7.1f} TFLOP/s",
          flush=True)
