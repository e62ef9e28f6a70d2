"""Side-by-side table of tools/anat_ab.sh results: python tools/anat_table.py VARIANT_MODE lib1 lib2 ..."""
import os
import sys

tag, libs = sys.argv[1], sys.argv[2:]
cols = []
for lib in libs:
    p = os.path.join("gpurun_out", f"anat_{lib}_{tag}.txt")
    d = {}
    if os.path.exists(p):
        for line in open(p):
            f = line.split()
            if len(f) >= 3 and f[1] == "median":
                d[f[0]] = float(f[2])
    cols.append(d)
keys = [k for k in (cols[0] if cols else {})]
print(f"{tag:22s}" + "".join(f"{l:>10s}" for l in libs))
for k in keys:
    print(f"{k:22s}" + "".join(f"{c.get(k, float('nan')):10.2f}" for c in cols))
