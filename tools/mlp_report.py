"""Per-wave view of tools/mlp_counters.sh output: python tools/mlp_report.py gpurun_out/mlpc_<variant>"""
import collections
import csv
import glob
import sys

vals = collections.defaultdict(list)
for f in glob.glob(f"{sys.argv[1]}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("k_mlp"):
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
a = {k: sum(v) / len(v) for k, v in vals.items()}
w = a.get("SQ_WAVES", 1.0)
for k in sorted(a):
    print(f"{k:28s} per launch {a[k]:16.1f}   per wave {a[k] / w:12.1f}")
if "SQ_VALU_MFMA_BUSY_CYCLES" in a and "GRBM_GUI_ACTIVE" in a:
    print("MFMA busy / (GUI_ACTIVE x SIMDs):", a["SQ_VALU_MFMA_BUSY_CYCLES"] / (a["GRBM_GUI_ACTIVE"] * 1024))
