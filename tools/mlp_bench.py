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
    for _ in range(3):
        net(x, actions=acts, step=0)
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    t0.record()
    for _ in range(reps):
        net(x, actions=acts, step=0)
    t1.record()
    torch.cuda.synchronize()
    us = t0.elapsed_time(t1) / reps * 1e3
    h0, h1 = net.hidden
    flop = 2.0 * rows * (net.in_dim * h0 + h0 * h1 + h1 * 9)
    print(f"ablate={abl} {variant:6s} rows={rows:8d} [{net.in_dim},{h0},{h1},9] {us:9.1f} us  {flop / us / 1e6:7.1f} TFLOP/s",
          flush=True)
