"""Per-wave, per-step view of tools/sq_counters.sh output.  python tools/sq_report.py DIR STEPS_PER_LAUNCH"""
import collections
import csv
import glob
import sys

d, spl = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1
KERNEL = sys.argv[3] if len(sys.argv) > 3 else "k_step"
vals = collections.defaultdict(list)
for f in glob.glob(f"{d}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith(KERNEL):
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
avg = {k: sum(v) / len(v) for k, v in vals.items()}
waves = avg.get("SQ_WAVES", 1024.0)
for k in sorted(avg):
    print(f"{k:28s} per launch {avg[k]:16.1f}   per wave-step {avg[k] / waves / spl:12.2f}")
