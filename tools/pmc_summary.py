"""Summarise a tools/profile_round.sh (or tools/sq_probe.sh) output directory into profiles/ (committed evidence).

    python tools/pmc_summary.py gpurun_out/prof_<tag> <tag> [--kernel k_step]

Writes profiles/<round>_<tag>_kernel_stats.csv (rocprofv3 --stats table, unchanged) and merges
{tag: {...}} into profiles/pmc_traffic.json:
  avg_ns           rocprofv3 kernel-trace average duration of the kernel
  fetch_kb/write_kb  per-dispatch averages of FETCH_SIZE / WRITE_SIZE (KB)
  bytes_per_launch (2 * FETCH_SIZE + WRITE_SIZE) * 1024: MI355X_MICROARCH.md §HBM -- on gfx950
                   FETCH_SIZE reports half the bytes of a coalesced streaming read, WRITE_SIZE is exact.
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(path, kernel, keep=None):
    """Per-dispatch averages of every counter of `kernel`; keep = indices (in dispatch order among that
    kernel's dispatches) to average over, None = all."""
    rows = [r for r in csv.DictReader(open(path)) if r["Kernel_Name"].startswith(kernel)]
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})
    chosen = set(ids if keep is None else [ids[i] for i in keep])
    vals = collections.defaultdict(list)
    for r in rows:
        if int(r["Dispatch_Id"]) in chosen:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("tag")
    ap.add_argument("--kernel", default="k_step")
    ap.add_argument("--round", default="r02")
    ap.add_argument("--steps-per-launch", type=int, default=None)
    ap.add_argument("--probe", default=None, metavar="T,LAUNCHES",
                    help="the directory holds tools/step_probe.py --cross runs of --launches LAUNCHES over "
                         "episodes of T steps: average only its timed launches, not the positioning rollouts")
    a = ap.parse_args()
    keep = None
    if a.probe:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from step_probe import timed_dispatches
        T, n = (int(x) for x in a.probe.split(","))
        keep = timed_dispatches(T, a.steps_per_launch, n, True)
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = os.path.join(a.prof_dir, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(prof, f"{a.round}_{a.tag}_kernel_stats.csv"))
    avg_ns = None
    for r in csv.DictReader(open(stats)):
        if r["Name"].startswith(a.kernel):
            avg_ns = float(r["AverageNs"])
    if keep is not None:   # the timed launches' own durations, from the trace
        tr = [r for r in csv.DictReader(open(os.path.join(a.prof_dir, "trace", "run_kernel_trace.csv")))
              if r["Kernel_Name"].startswith(a.kernel)]
        tr.sort(key=lambda r: int(r["Dispatch_Id"]))
        durs = [int(tr[i]["End_Timestamp"]) - int(tr[i]["Start_Timestamp"]) for i in keep]
        avg_ns = sum(durs) / len(durs)
    sys.path.insert(0, ROOT)
    import bench

    out = {"kernel": a.kernel, "avg_ns": avg_ns, "avg_ns_of": "all dispatches" if keep is None else
           f"the {len(keep)} timed step_probe launches (dispatches {keep} of the kernel)", "round": a.round, "source_sha": bench.source_sha(),
           "steps_per_launch": a.steps_per_launch}
    fetch, n_f = counters(os.path.join(a.prof_dir, "fetch", "run_counter_collection.csv"), a.kernel, keep)
    write, n_w = counters(os.path.join(a.prof_dir, "write", "run_counter_collection.csv"), a.kernel, keep)
    out["fetch_kb"] = fetch.get("FETCH_SIZE")
    out["write_kb"] = write.get("WRITE_SIZE")
    out["dispatches"] = {"fetch": n_f.get("FETCH_SIZE"), "write": n_w.get("WRITE_SIZE")}
    if out["fetch_kb"] is not None and out["write_kb"] is not None:
        out["bytes_per_launch"] = (2 * out["fetch_kb"] + out["write_kb"]) * 1024
    for sub in ("sq", "sq2"):
        extra = os.path.join(a.prof_dir, sub, "run_counter_collection.csv")
        if os.path.exists(extra):
            sq, _ = counters(extra, a.kernel, keep)
            out.setdefault("sq", {}).update(sq)
    path = os.path.join(prof, "pmc_traffic.json")
    d = json.load(open(path)) if os.path.exists(path) else {}
    d[a.tag] = out
    json.dump(d, open(path, "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
