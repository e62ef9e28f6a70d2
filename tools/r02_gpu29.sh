#!/bin/bash
# per-launch time of consecutive 20-step launches from a fresh reset (episode phase profile), per
# phase ablation (timing only, -DWH_ABLATION build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for m in 0 1 2 8 16 32; do
  WH_ABLATE=$m WAREHOUSE_AMD_LIB=build_ab/ablation.so timeout -k 10 120 python tools/step_probe.py --steps 20 --launches 21 > gpurun_out/phase_$m.log 2>&1 || exit $?
done
