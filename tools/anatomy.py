"""Launch anatomy of the fused step kernel: kernel duration as a function of steps per launch, with
and without an episode end inside the launch, for the fast fused instance (greedy, rewards + dones,
auto-reset; bench.py's timed launch).  Every k_step dispatch of this script is labelled in order;
run it under `rocprofv3 --kernel-trace` and join the labels with the trace:

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/anatomy.py > labels.json
    python tools/anatomy.py --join OUT/run_kernel_trace.csv labels.json

Without the profiler it prints HIP-event times (they add ~2 us per launch).  The fixed cost of a
launch is the intercept of duration vs steps; the episode-end cost is the crossing launch minus a
mid-episode launch of the same length.
"""
import argparse
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rllib-warehouse_amd")]


def join(trace, labels_path):
    # a 0-step launch has empty reward/done buffers (NULL pointers): it runs the generic instance
    labels = [x for x in json.load(open(labels_path))["labels"] if not x.endswith("_k0")]
    # the fast fused instance only (k_step<Cfg, POLICY, false, true>): wh_policy / wh_vector_step
    # launches (stagger) are other instances of k_step
    import re

    fast = re.compile(r"k_step<.*,\s*\d\s*,\s*false\s*,\s*true\s*>")
    rows = [r for r in csv.DictReader(open(trace)) if fast.search(r["Kernel_Name"])]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    if len(rows) != len(labels):
        print(f"warning: {len(rows)} k_step dispatches, {len(labels)} labels")
    by = {}
    for r, lab in zip(rows, labels):
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
        by.setdefault(lab, []).append(d)
    out = {}
    for lab, ds in by.items():
        if lab.startswith("pos"):
            continue
        v = sorted(ds)
        out[lab] = dict(median_us=statistics.median(v), min_us=v[0], n=len(v))
        print(f"{lab:28s} median {statistics.median(v):9.2f} us  min {v[0]:9.2f}  n={len(v)}")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--join", nargs=2, metavar=("TRACE_CSV", "LABELS_JSON"))
    ap.add_argument("--variant", default="medium")
    ap.add_argument("--agents", type=int, default=8)
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--ks", default="0,1,2,5,10,20,40,100")
    ap.add_argument("--stagger", action="store_true", help="desynchronised episodes first")
    ap.add_argument("--tscan", action="store_true", help="1- and 20-step launches at several episode "
                    "times, cold (after a host sync) and warm (queued behind another launch)")
    a = ap.parse_args()
    if a.join:
        json.dump(join(*a.join), open(a.join[1].replace(".json", "_joined.json"), "w"), indent=1)
        return
    import torch

    import warehouse

    dev = torch.device("cuda", 0)
    env = warehouse.BatchedWarehouse(a.variant, a.envs, a.agents, seed=3, device=dev)
    env.reset()
    B, NA = env.B, env.agent_slots
    T = int(env.geometry["T"])
    KMAX = 240
    rew = torch.zeros((KMAX, B, NA), device=dev)
    dn = torch.zeros((KMAX, B), dtype=torch.uint8, device=dev)
    labels, ev = [], {}
    t = 0   # episode clock of every env (synchronised episodes)
    if a.stagger:
        import numpy as np

        env.stagger((np.arange(B, dtype=np.int64) * 37) % T)   # (other k_step instances)

    def run(k, lab):
        nonlocal t
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        env.rollout(k, "greedy", 0.0, rewards=rew[:k], dones=dn[:k])
        e1.record()
        torch.cuda.synchronize()
        labels.append(lab)
        ev.setdefault(lab, []).append(e0.elapsed_time(e1) * 1e3)
        t = (t + k) % T

    def goto(target):
        k = (target - t) % T
        while k:
            c = min(k, KMAX)
            run(c, "pos")
            k -= c

    def run_warm(k, lab):
        """`k`-step launch queued right behind a 40-step one (no host gap, the GPU busy)."""
        nonlocal t
        env.rollout(40, "greedy", 0.0, rewards=rew[:40], dones=dn[:40])
        labels.append("pos")
        env.rollout(k, "greedy", 0.0, rewards=rew[40:40 + k], dones=dn[40:40 + k])
        labels.append(lab)
        torch.cuda.synchronize()
        t = (t + 40 + k) % T

    ks = [int(x) for x in a.ks.split(",")]
    if a.tscan:
        for _ in range(a.reps):
            for t0 in (0, 1, 5, 20, 60, 100, 140, 180, 198, 199):
                goto(t0)
                run(1, f"k1_t{t0}")
            for t0 in (0, 20, 60, 100, 140, 180):
                goto(t0)
                run(20, f"k20_t{t0}")
            for t0 in (20, 180):
                goto((t0 - 40) % T)
                run_warm(20, f"warm_k20_t{t0}")
                goto((t0 - 40) % T)
                run_warm(1, f"warm_k1_t{t0}")
        print(json.dumps({"labels": labels}))
        return
    for _ in range(a.reps):
        for k in ks:
            goto(20)                       # mid-episode: no end inside any of these launches
            run(k, f"mid_k{k}")
        for k in (2, 10, 20, 40):
            goto(T - k // 2)               # crossing: the episode end in the middle of the launch
            run(k, f"cross_k{k}")
        goto(T - 1)
        run(1, "end_k1")                   # the done step alone: auto-reset of every env
        run(1, "first_k1")                 # the first step of the new episode
    print(json.dumps({"labels": labels, "events_us": {k: statistics.median(v) for k, v in ev.items()
                                                      if not k.startswith("pos")}}))


if __name__ == "__main__":
    main()
