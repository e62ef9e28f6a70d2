"""BASELINE config 1 -- `baseline/run.py` on CPU, one env -- timed with the reference's own
`warehouse` package and with this package's drop-in on the host engine, the same unchanged
`baseline/run.py` + `baseline/solvers.py` driving both (build container only: it imports
/root/reference through tests/golden/ref_stubs.py; nothing here runs on the GPU box).

    python tools/c1_compare.py [--seeds 10]

Each side runs in its own process: `np.random.seed(s); run.main('small', 2, 0.0, False)` for
s = 0 .. seeds-1 (one 200-step episode each), printed totals compared, wall time of the loop.
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"

CHILD = r'''
import contextlib, io, json, os, re, sys, time, types
import numpy as np
side, seeds, ROOT, REF = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4]
if side == "reference":
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import ref_stubs
    _, _, run = ref_stubs.import_reference(REF)
else:
    os.environ["WAREHOUSE_DEVICE"] = "cpu"
    sys.path.insert(0, os.path.join(ROOT, "rllib-warehouse_amd"))
    from warehouse import _compat
    gym = types.ModuleType("gym")
    gym.Space, gym.spaces = object, _compat.spaces
    sys.modules["gym"] = gym
    sys.path.insert(0, os.path.join(REF, "baseline"))
    import run
totals = []
np.random.seed(100); buf = io.StringIO()
with contextlib.redirect_stdout(buf):
    run.main("small", 2, 0.0, False)          # warm-up (imports, library load)
t0 = time.perf_counter()
for s in range(seeds):
    np.random.seed(s)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        run.main("small", 2, 0.0, False)
    totals.append(float(re.search(r"Total: ([0-9.]+)", buf.getvalue()).group(1)))
dt = time.perf_counter() - t0
print(json.dumps({"side": side, "totals": totals, "wall_s": dt, "agent_steps_per_s": seeds * 200 * 2 / dt}))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=10)
    a = ap.parse_args()
    out = {}
    for side in ("reference", "host_engine"):
        r = subprocess.run([sys.executable, "-c", CHILD, side, str(a.seeds), ROOT, REF], capture_output=True,
                           text=True, timeout=600)
        if r.returncode:
            print(r.stderr[-2000:], file=sys.stderr)
            return r.returncode
        out[side] = json.loads(r.stdout.strip().splitlines()[-1])
    same = out["reference"]["totals"] == out["host_engine"]["totals"]
    print(json.dumps({"config": "C1: baseline/run.py small 2 0.0 (greedy solver, one env), CPU",
                      "seeds": a.seeds, "totals_identical": same,
                      "reference_agent_steps_per_s": out["reference"]["agent_steps_per_s"],
                      "host_engine_agent_steps_per_s": out["host_engine"]["agent_steps_per_s"],
                      "speedup": out["host_engine"]["agent_steps_per_s"] / out["reference"]["agent_steps_per_s"],
                      "totals": out["reference"]["totals"]}))
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
