"""Identical fused-rollout launches for kernel studies under rocprofv3 (every k_step dispatch has the
same shape, so --stats averages and per-dispatch counters describe exactly one launch shape).

    python tools/step_probe.py [--variant medium --agents 8 --envs 65536 --steps 200 --launches 6]
Prints the HIP-event time per launch and per step (median over launches after the first).
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rllib-warehouse_amd")]

import torch  # noqa: E402

import warehouse  # noqa: E402


def positioning(T, steps, launches, cross):
    """Untimed positioning steps before each timed launch (0 = none): with cross, t + K/2 = T (mod T),
    so the launch's middle step ends the episode."""
    t, out = 0, []
    for _ in range(launches):
        pos = (T - steps // 2 - t) % T if cross else 0
        out.append(pos)
        t = (t + pos + steps) % T
    return out


def timed_dispatches(T, steps, launches, cross):
    """Indices, among this probe's k_step dispatches in issue order, of the timed launches (each
    positioning rollout is one k_step dispatch of its own)."""
    idx, i = [], 0
    for pos in positioning(T, steps, launches, cross):
        i += pos > 0
        idx.append(i)
        i += 1
    return idx


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="medium")
    ap.add_argument("--agents", type=int, default=8)
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--launches", type=int, default=6)
    ap.add_argument("--policy", default="greedy")
    ap.add_argument("--train", action="store_true")
    ap.add_argument("--stagger", action="store_true", help="desynchronised episodes (bench.py's desync leg)")
    ap.add_argument("--cross", action="store_true",
                    help="place every timed launch across an episode end, as bench.py's window (untimed "
                         "positioning steps before each launch)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    env = warehouse.BatchedWarehouse(a.variant, a.envs, None if a.train else a.agents, train=a.train,
                                     seed=3, device=dev)
    env.reset()
    if a.stagger:
        env.stagger((torch.arange(a.envs, dtype=torch.int64) * 37) % 200)
    NA = env.agent_slots
    rew = torch.zeros((a.steps, a.envs, NA), device=dev)
    dn = torch.zeros((a.steps, a.envs), dtype=torch.uint8, device=dev)
    launch = env.rollout_launcher(a.steps, a.policy, 0.0, rewards=rew, dones=dn)
    s = torch.cuda.current_stream(dev)
    times = []
    T = int(env.geometry["T"])
    for pos in positioning(T, a.steps, a.launches, a.cross):
        if pos:
            env.rollout(pos, a.policy, 0.0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        launch()
        e1.record(s)
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1) * 1e3)
    med = statistics.median(times[1:] if len(times) > 1 else times)
    print(f"{a.variant} N={NA} B={a.envs} steps/launch={a.steps}: {med:.1f} us per launch, "
          f"{med / a.steps:.3f} us per step, {a.envs * NA * a.steps / med * 1e6:.3e} agent-steps/s "
          f"(launch times {', '.join(f'{t:.1f}' for t in times)})")


if __name__ == "__main__":
    main()
