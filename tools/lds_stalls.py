"""Static estimate of the LDS-latency stalls in the fused step loop (tools/ analysis aid).

    make -C rllib-warehouse_amd/csrc asm EXTRA=-DWH_ONLY_MEDIUM8
    python tools/lds_stalls.py [rllib-warehouse_amd/csrc/warehouse_amd.s] [--lat 13] [--all]

Walks the last top-level loop of k_step<Medium-8, greedy> (the PH_ALL step loop) in program order,
counts one issue slot (quad-cycle) per instruction, and for every `s_waitcnt lgkmcnt(N)` estimates
the stall as max(0, lat - slots since the newest LDS op it waits for) (LDS ops retire in order).
Prints per-phase instruction counts and stall estimates, and the worst waits with their line.
Straight-line approximation: both sides of branches are walked (expiry / reset blocks are reported
under their phase and can be discounted).
"""
import re
import sys

KERNEL = "_ZN12_GLOBAL__N_16k_stepINS_3CfgILi16ELi9ELi3ELi8EEELi1ELb0EEEvNS_10StepParamsE"


def main():
    argv = sys.argv[1:]
    args = [a for j, a in enumerate(argv) if not a.startswith("--") and (j == 0 or argv[j - 1] not in ("--lat", "--kernel"))]
    path = args[0] if args else "rllib-warehouse_amd/csrc/warehouse_amd.s"
    lat = 13
    if "--lat" in sys.argv:
        lat = int(sys.argv[sys.argv.index("--lat") + 1])
    kernel = KERNEL
    if "--kernel" in sys.argv:
        kernel = sys.argv[sys.argv.index("--kernel") + 1]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(kernel + ":"))
    end = next(i for i in range(start, len(lines)) if "codeLenInByte" in lines[i])
    heads = [i for i in range(start, end) if "Loop Header: Depth=1" in lines[i]]
    lo = heads[-1]
    phase = "head"
    slots = 0
    queue = []          # issue slot of each outstanding LDS op, oldest first
    per = {}
    waits = []
    for i in range(lo, end):
        l = lines[i].strip()
        m = re.search(r"; PHASE (\w+)", l)
        if m:
            phase = m.group(1)
            continue
        if not l or l.startswith((";", ".")):
            continue
        op = l.split()[0]
        st = per.setdefault(phase, {"inst": 0, "valu": 0, "lds": 0, "stall": 0, "waits": 0})
        if op.startswith("s_waitcnt"):
            m = re.search(r"lgkmcnt\((\d+)\)", l)
            if m:
                keep = int(m.group(1))
                if len(queue) > keep:
                    need = queue[len(queue) - keep - 1]
                    stall = max(0, lat - (slots - need))
                    st["stall"] += stall
                    st["waits"] += 1
                    waits.append((stall, i + 1, phase, l))
                    slots += stall
                    queue = queue[len(queue) - keep:] if keep else []
            continue
        st["inst"] += 1
        if op.startswith("v_"):
            st["valu"] += 1
        if op.startswith("ds_"):
            st["lds"] += 1
            queue.append(slots)
        slots += 1
    tot = {"inst": 0, "valu": 0, "lds": 0, "stall": 0, "waits": 0}
    print(f"{'phase':16s} {'inst':>6s} {'valu':>6s} {'lds':>5s} {'waits':>6s} {'stall':>6s}")
    for k, v in per.items():
        print(f"{k:16s} {v['inst']:6d} {v['valu']:6d} {v['lds']:5d} {v['waits']:6d} {v['stall']:6d}")
        for f in tot:
            tot[f] += v[f]
    print(f"{'total':16s} {tot['inst']:6d} {tot['valu']:6d} {tot['lds']:5d} {tot['waits']:6d} {tot['stall']:6d}")
    print("\nworst waits (est. stall quad-cycles, line, phase):")
    for w in sorted(waits, reverse=True)[:25]:
        print(f"  {w[0]:3d}  line {w[1]:6d}  {w[2]:14s} {w[3]}")


if __name__ == "__main__":
    main()
