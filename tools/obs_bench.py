"""Time wh_observe (f32 rows) and wh_observe_x (the policy's bf16 fragment-order operand) at
B=65536.  Prints us/launch and the achieved write bandwidth.  OBS_SHAPES="medium:8 large:16" picks
the shapes (default: small:4 medium:8 large:16)."""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rllib-warehouse_amd")]
import torch  # noqa: E402
import warehouse  # noqa: E402

B = int(os.environ.get("OBS_B", 65536))
SHAPES = [(v, int(n)) for v, n in (x.split(":") for x in os.environ.get("OBS_SHAPES", "small:4 medium:8 large:16").split())]


def timed(fn, reps=50):
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(5):
        fn()
    t0.record()
    for _ in range(reps):
        fn()
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) / reps * 1e3


for variant, na in SHAPES:
    env = warehouse.BatchedWarehouse(variant, B, na, seed=3)
    env.reset()
    env.rollout(37, "greedy", 0.0)
    obs = env.observe()
    xf = env.observe_x()
    torch.cuda.synchronize()
    o = env.observe()
    w = (torch.arange(o.numel(), device=o.device, dtype=torch.float64) % 9973 + 1).view(o.shape)
    print(f"{variant:6s} na={na:2d} observe rows fingerprint {float((o.double() * w).sum()):.1f} "
          f"(sum {float(o.double().sum()):.1f})", flush=True)
    us = timed(env.observe)
    nbytes = obs.numel() * 4 + env.state.numel() * 4
    print(f"{variant:6s} na={na:2d} observe   {us:8.2f} us  {nbytes / us / 1e3:7.1f} GB/s "
          f"(rows {obs.numel() * 4 / 1e6:.1f} MB + state {env.state.numel() * 4 / 1e6:.1f} MB)", flush=True)
    xb = env.observe_x().view(-1).to(torch.int64)
    print(f"{variant:6s} na={na:2d} observe_x operand fingerprint "
          f"{int(((xb & 0xFF) * (torch.arange(xb.numel(), device=xb.device) % 9973 + 1)).sum())}", flush=True)
    us = timed(env.observe_x)
    nbytes = xf.numel() + env.state.numel() * 4
    print(f"{variant:6s} na={na:2d} observe_x {us:8.2f} us  {nbytes / us / 1e3:7.1f} GB/s "
          f"(fragments {xf.numel() / 1e6:.1f} MB + state {env.state.numel() * 4 / 1e6:.1f} MB)", flush=True)
