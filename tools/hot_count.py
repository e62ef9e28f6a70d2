"""Static instruction counts of the fused rollout's hot loop, per basic block, from device assembly
(quick feedback for step-kernel edits without a GPU):

    hipcc ... -DWH_ONLY_MEDIUM8 --cuda-device-only -S warehouse_amd.hip -o /tmp/m8.s
    python tools/hot_count.py /tmp/m8.s [SYMBOL_SUBSTRING]

Blocks are listed in layout order with their VALU / LDS / SALU / s_waitcnt counts and the phase
marks (WH_PHASE_MARK) they contain; `hot` sums the blocks of the loop's common path (the blocks that
hold the policy, move, pickup and delivery marks plus the blocks between them in layout order)."""
import re
import sys

path = sys.argv[1]
SYM = sys.argv[2] if len(sys.argv) > 2 else "k_stepINS_3CfgILi16ELi9ELi3ELi8EEELi1ELb0ELb1EE"
lines = open(path).read().splitlines()
start = next(i for i, l in enumerate(lines) if l.startswith("_ZN") and SYM in l and l.split(";")[0].rstrip().endswith(":"))
end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
blocks = [dict(label="entry", n=0, v=0, lds=0, s=0, w=0, ph=[])]
for i in range(start + 1, end):
    s = lines[i].strip()
    m = re.match(r"^(\.LBB\d+_\d+):", s)
    if m:
        blocks.append(dict(label=m.group(1), n=0, v=0, lds=0, s=0, w=0, ph=[]))
        continue
    m = re.match(r";\s*PHASE (\w+)", s)
    if m:
        blocks[-1]["ph"].append(m.group(1))
    if not s or s.startswith(";") or s.startswith("."):
        continue
    op = s.split()[0]
    b = blocks[-1]
    b["n"] += 1
    if op.startswith("v_"):
        b["v"] += 1
    elif op.startswith("ds_"):
        b["lds"] += 1
    elif op == "s_waitcnt":
        b["w"] += 1
    elif op.startswith("s_"):
        b["s"] += 1
idx = [k for k, b in enumerate(blocks) if set(b["ph"]) & {"policy_rtag", "policy_agents", "move", "pickup", "deliver"}]
lo, hi = (min(idx), max(idx)) if idx else (0, -1)
hot = dict(v=0, lds=0, s=0, w=0)
for k, b in enumerate(blocks):
    if b["n"] == 0:
        continue
    tag = "*" if lo <= k <= hi else " "
    if tag == "*":
        for f in hot:
            hot[f] += b[f]
    print(f"{tag} {b['label']:12s} v{b['v']:5d} lds{b['lds']:4d} s{b['s']:4d} w{b['w']:3d} {','.join(b['ph'])}")
print(f"hot path (static, both sides of its branches): valu {hot['v']}  lds {hot['lds']}  salu {hot['s']}  waitcnt {hot['w']}")
