"""Report of tools/wait_attrib.py's rocprofv3 --pmc run: per (K, WH_ABLATE mask) the SQ counters per
wave-step of the fused step kernel, and what each removed phase saves against the full kernel.

    python tools/wait_attrib_report.py gpurun_out/wattr [--out profiles/r05_wait_attribution.json]

SQ_WAVE_CYCLES / SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_BUSY_CYCLES are quad-cycles (MI355X_MICROARCH.md);
counts are summed over the dispatch and divided by SQ_WAVES and K.
"""
import argparse
import collections
import csv
import glob
import json
import os

NAMES = {0: "full kernel", 1: "-policy", 2: "-move", 4: "-expiry", 8: "-pickup", 16: "-regeneration",
         32: "-delivery", 64: "-reward/done stores", 128: "-auto-reset", 255: "-everything"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--plan", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    plan = json.load(open(a.plan or os.path.join(os.path.dirname(a.dir.rstrip("/")), "wattr_plan.json")))
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    csvs = glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True)
    if csvs:
        path = csvs[0]
        for r in csv.DictReader(open(path)):
            if r["Kernel_Name"].startswith("k_step"):
                per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    else:   # rocprofv3's default rocpd (SQLite) output
        import sqlite3
        path = glob.glob(os.path.join(a.dir, "**", "*.db"), recursive=True)[0]
        db = sqlite3.connect(path)
        names = {d: n for d, n in db.execute("select dispatch_id, name from kernels")}
        for d, cn, v in db.execute("select dispatch_id, counter_name, counter_value from pmc_events"):
            if "k_step<" in names.get(d, ""):
                per[int(d)][cn] += float(v)
    ids = sorted(per)
    need = sum(p["launches"] for p in plan["plan"])
    assert len(ids) == need, (len(ids), need)
    res, i = {}, 0
    for p in plan["plan"]:
        grp = [per[d] for d in ids[i:i + p["launches"]]][1:]   # first launch of a group: warm-up
        i += p["launches"]
        K = p["K"]
        avg = {c: sum(g[c] for g in grp) / len(grp) for c in grp[0]}
        waves = avg["SQ_WAVES"]
        res[f"K{K}_m{p['mask']}"] = {"K": K, "mask": p["mask"], "what": NAMES.get(p["mask"], str(p["mask"])),
                                     **{c: round(v / waves / K, 1) for c, v in avg.items() if c != "SQ_WAVES"}}
    print(f"{'K':>4} {'mask':>5} {'what':22s} {'WAVE_CYC':>9} {'WAIT_ANY':>9} {'VALU':>7} {'LDS':>6} {'W_INST':>7} {'W_LDS':>6}")
    for k, v in res.items():
        print(f"{v['K']:4d} {v['mask']:5d} {v['what']:22s} {v['SQ_WAVE_CYCLES']:9.1f} {v['SQ_WAIT_ANY']:9.1f} "
              f"{v['SQ_INSTS_VALU']:7.1f} {v['SQ_INSTS_LDS']:6.1f} {v['SQ_WAIT_INST_ANY']:7.1f} {v['SQ_WAIT_INST_LDS']:6.1f}")
    if a.out:
        json.dump({"source": os.path.relpath(path), "units": "per wave-step (per wave for the fixed part); cycle "
                   "counters in quad-cycles", "variant": plan["variant"], "agents": plan["agents"], "rows": res},
                  open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
