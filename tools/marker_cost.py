"""Host cost of the bench window's two timing markers: the driver's 20-step launch timed as
bench.py's run() does it (torch.cuda.Event.record around the prepared launch) against the same two
markers recorded with one ctypes call each to hipEventRecord, and against no markers at all.
Median window (sync -> markers + launch -> sync) over many repetitions, interleaved.

    python tools/marker_cost.py [--reps 200]
"""
import argparse
import ctypes
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rllib-warehouse_amd")]

import torch  # noqa: E402

import warehouse  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    env = warehouse.BatchedWarehouse("medium", 65536, 8, seed=3, device=dev)
    env.reset()
    K = 20
    rew = torch.zeros((K, env.B, 8), device=dev)
    dn = torch.zeros((K, env.B), dtype=torch.uint8, device=dev)
    launch = env.rollout_launcher(K, "greedy", 0.0, rewards=rew, dones=dn)
    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    hip = ctypes.CDLL("libamdhip64.so.7")   # the soname torch loaded (a bare "libamdhip64.so" loads a second runtime)
    hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    rec = hip.hipEventRecord
    ev0.record(stream)                 # torch creates the HIP events at their first record
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    h0, h1, hs = ev0.cuda_event, ev1.cuda_event, stream.cuda_stream
    assert h0 and h1

    def torch_markers():
        ev0.record(stream)
        launch()
        ev1.record(stream)

    def ctypes_markers():
        rec(h0, hs)
        launch()
        rec(h1, hs)

    def none():
        launch()

    forms = {"torch markers (bench.py)": torch_markers, "ctypes hipEventRecord": ctypes_markers, "no markers": none}
    times = {k: [] for k in forms}
    spans = {k: [] for k in forms}
    for _ in range(5):
        for f in forms.values():
            f()
    torch.cuda.synchronize(dev)
    for r in range(a.reps):
        for name, f in forms.items():
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            f()
            torch.cuda.synchronize(dev)
            times[name].append((time.perf_counter() - t0) * 1e6)
            if name != "no markers":
                spans[name].append(ev0.elapsed_time(ev1) * 1e3)
    for name in forms:
        sp = f", marker span {statistics.median(spans[name]):.1f} us" if spans[name] else ""
        print(f"{name:26s} window median {statistics.median(times[name]):.1f} us "
              f"(p10 {sorted(times[name])[len(times[name]) // 10]:.1f}){sp}", flush=True)


if __name__ == "__main__":
    main()
