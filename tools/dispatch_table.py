"""Per-dispatch table of one kernel from a rocprofv3 kernel trace (the --stats summary averages
every launch shape together; this lists each dispatch so the timed one can be read off).

    python tools/dispatch_table.py gpurun_out/prof_<tag>/trace/run_kernel_trace.csv [--kernel k_step] [--out CSV]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="k_step")
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if r["Kernel_Name"].startswith(a.kernel)]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    out = []
    for i, r in enumerate(rows):
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
        out.append(dict(index=i, dispatch_id=r["Dispatch_Id"], kernel=r["Kernel_Name"][:80], duration_us=f"{d:.2f}",
                        grid=r["Grid_Size_X"], workgroup=r["Workgroup_Size_X"], vgpr=r["VGPR_Count"],
                        sgpr=r["SGPR_Count"], lds=r["LDS_Block_Size"]))
        print(f"{i:4d} {d:10.2f} us  grid {r['Grid_Size_X']:>7s}  {r['Kernel_Name'][:60]}")
    if a.out:
        with open(a.out, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(out[0].keys()))
            w.writeheader()
            w.writerows(out)


if __name__ == "__main__":
    main()
