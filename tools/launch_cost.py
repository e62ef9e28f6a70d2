"""Where the fixed cost of a short timed window goes (bench.py --steps 20): host call, launch
latency, kernel prologue/epilogue, completion/sync latency.  Medium-8, B = 65,536, greedy fused.

    python tools/launch_cost.py
Prints medians (us) over repetitions:
  sync_idle      torch.cuda.synchronize() on an idle device
  tiny_op        a one-element torch op + sync (launch + completion latency of a trivial kernel)
  call_K         the bound wh_rollout call alone (host time, no sync)
  wall_K         call + sync (what bench.py's window sees for one launch of K steps)
  event_K        HIP-event span around the launch on its stream
  plain_K        wall of the launch + sync with no events at all
  ext_K          wall / span with the events attached to the dispatch (wh_launch_run_timed)
"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rllib-warehouse_amd")]

import torch  # noqa: E402

import warehouse  # noqa: E402


def med(xs):
    return statistics.median(xs) * 1e6


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B, NA = int(os.environ.get("B", 65536)), 8
    env = warehouse.BatchedWarehouse("medium", B, NA, seed=1, device=dev)
    env.reset()
    x = torch.zeros(1, device=dev)
    s = torch.cuda.current_stream(dev)
    torch.cuda.synchronize()
    r = []
    for _ in range(50):
        t0 = time.perf_counter(); torch.cuda.synchronize(); r.append(time.perf_counter() - t0)
    print(f"sync_idle {med(r):8.1f}")
    r = []
    for _ in range(50):
        torch.cuda.synchronize()
        t0 = time.perf_counter(); x.add_(1); torch.cuda.synchronize(); r.append(time.perf_counter() - t0)
    print(f"tiny_op   {med(r):8.1f}")
    r = []
    for _ in range(50):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(s); x.add_(1); e1.record(s)
        torch.cuda.synchronize()
        r.append(e0.elapsed_time(e1) * 1e-3)
    print(f"tiny_op_event {med(r):8.1f}")
    Ks = (20,) if "--quick" in sys.argv else (0, 1, 2, 5, 20, 200)
    for K in Ks:
        rew = torch.zeros((K, B, NA), device=dev)
        dn = torch.zeros((K, B), dtype=torch.uint8, device=dev)
        launch = env.rollout_launcher(K, "greedy", 0.0, rewards=rew, dones=dn)
        for _ in range(3):
            launch()
        torch.cuda.synchronize()
        call, wall, span = [], [], []
        for _ in range(30):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record(s)
            launch()
            e1.record(s)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            call.append(t1 - t0); wall.append(t2 - t0); span.append(e0.elapsed_time(e1) * 1e-3)
        print(f"K={K:4d} call {med(call):8.1f}  wall {med(wall):8.1f}  event {med(span):8.1f}  "
              f"wall-event {med(wall) - med(span):7.1f}  event/step {med(span) / max(K, 1):7.2f}")
        plain = []
        for _ in range(30):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            launch()
            torch.cuda.synchronize()
            plain.append(time.perf_counter() - t0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        tl = env.rollout_launcher(K, "greedy", 0.0, rewards=rew, dones=dn, events=(e0, e1))
        tl()
        torch.cuda.synchronize()
        wall, span = [], []
        for _ in range(30):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tl()
            torch.cuda.synchronize()
            wall.append(time.perf_counter() - t0)
            span.append(e0.elapsed_time(e1) * 1e-3)
        print(f"K={K:4d} plain wall {med(plain):8.1f}  ext wall {med(wall):8.1f}  ext span {med(span):8.1f}  "
              f"wall-span {med(wall) - med(span):7.1f}")


if __name__ == "__main__":
    main()
