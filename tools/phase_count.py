"""Static instruction counts per WH_PHASE_MARK region of one kernel in the device assembly
(`make -C rllib-warehouse_amd/csrc asm` -> warehouse_amd.s).  Counts every instruction between a
"; PHASE name" label and the next one (straight-line view: both sides of a branch are counted).

    python tools/phase_count.py [SYMBOL_SUBSTRING]   (default: the Medium-8 greedy fast instance)
"""
import collections
import re
import sys

SYM = next((a for a in sys.argv[1:] if not a.startswith("-")), None) or "k_stepINS_3CfgILi16ELi9ELi3ELi8EEELi1ELb0ELb1EE"
import os
lines = open(os.environ.get("WH_ASM", "rllib-warehouse_amd/csrc/warehouse_amd.s")).read().splitlines()
start = next(i for i, l in enumerate(lines) if l.startswith("_ZN") and SYM in l and l.split(";")[0].rstrip().endswith(":"))
end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
phase = "prologue"
cnt = collections.defaultdict(collections.Counter)
order = [phase]
for l in lines[start + 1:end]:
    s = l.strip()
    m = re.match(r";\s*PHASE (\w+)", s)
    if m:
        phase = m.group(1)
        if phase not in order:
            order.append(phase)
        continue
    if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
        continue
    op = s.split()[0]
    cls = ("branch" if op.startswith("s_cbranch") or op == "s_branch" else
           "valu" if op.startswith("v_") else "salu" if op.startswith("s_") else
           "lds" if op.startswith("ds_") else "vmem" if op.startswith(("global_", "buffer_", "flat_")) else "other")
    cnt[phase][cls] += 1
    if op.startswith("v_"):
        cnt[phase]["op:" + op] += 1
tot = collections.Counter()
for p in order:
    c = cnt[p]
    tot.update({k: v for k, v in c.items() if not k.startswith("op:")})
    print(f"{p:16s} valu {c['valu']:5d}  salu {c['salu']:4d}  lds {c['lds']:4d}  vmem {c['vmem']:3d}  branch {c['branch']:3d}")
print(f"{'total':16s} valu {tot['valu']:5d}  salu {tot['salu']:4d}  lds {tot['lds']:4d}  vmem {tot['vmem']:3d}  branch {tot['branch']:3d}")
if "-v" in sys.argv:
    for p in order:
        print(p, cnt[p].most_common(25))
