"""Time wh_observe (and the step + observe pair) at B=65536 for the three variants.
Prints us/launch and the achieved write bandwidth of the observation rows."""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rllib-warehouse_amd")]
import torch  # noqa: E402
import warehouse  # noqa: E402

B = int(os.environ.get("OBS_B", 65536))
for variant, na in (("small", 4), ("medium", 8), ("large", 16)):
    env = warehouse.BatchedWarehouse(variant, B, na, seed=3)
    env.reset()
    env.rollout(37, "greedy", 0.0)
    obs = env.observe()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    reps = 50
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(5):
        env.observe()
    t0.record()
    for _ in range(reps):
        env.observe()
    t1.record()
    torch.cuda.synchronize()
    us = t0.elapsed_time(t1) / reps * 1e3
    nbytes = obs.numel() * 4 + env.state.numel() * 4
    print(f"{variant:6s} na={na:2d} observe {us:8.2f} us  {nbytes / us / 1e3:7.1f} GB/s "
          f"(rows {obs.numel() * 4 / 1e6:.1f} MB + state {env.state.numel() * 4 / 1e6:.1f} MB)", flush=True)
