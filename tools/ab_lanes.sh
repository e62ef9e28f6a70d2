#!/bin/bash
# A/B of the kernel families (lane pair vs one lane per env) on the bench workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for v in "medium 8" "large 16" "small 4"; do
  set -- $v
  for L in 2 1; do
    if [ $L = 1 ]; then export WH_LANES=1; else unset WH_LANES; fi
    timeout -k 10 300 python bench.py --variant $1 --agents $2 --no-cpu-baseline --steps 1000 --warmup 100 > gpurun_out/ab_$1_$L.log 2>&1 || exit $?
    python - "$1" "$L" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab_{sys.argv[1]}_{sys.argv[2]}.log").read().strip().splitlines()[-1])
a = d["alt_launch_mode"]
print(f"{sys.argv[1]:6s} lanes={sys.argv[2]} fused {d['value']/1e9:7.2f} G/s {d['ms_per_step']*1e3:6.2f} us/step | graph {a['value']/1e9:7.2f} G/s {a['ms_per_step']*1e3:6.2f} us/step frac {a['roofline_frac']:.3f}")
PY
  done
done
