#!/bin/bash
# where the waits are: SQ counters of the ablation build with one phase skipped at a time
# (WH_ABLATE bits: 1 policy, 2 move, 8 pickup, 16 regeneration; 200-step Medium-8 launches)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp WAREHOUSE_AMD_LIB=build_ab/ablation.so
mkdir -p gpurun_out/abl_sq
for m in 0 1 2 8 16 3; do
  WH_ABLATE=$m timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAIT_INST_ANY \
    -T --output-format csv -d gpurun_out/abl_sq/m$m -o run -- python3 tools/step_probe.py --steps 200 --launches 3 > gpurun_out/abl_sq/m$m.log 2>&1 || exit $?
  echo "m$m done"
done
unset WAREHOUSE_AMD_LIB
for i in 1 2; do
  timeout -k 10 120 python3 tools/step_probe.py --steps 200 --launches 6 > gpurun_out/abl_sq/cur_$i.log 2>&1 || exit $?
  WAREHOUSE_AMD_LIB=build_ab/ahead2.so timeout -k 10 120 python3 tools/step_probe.py --steps 200 --launches 6 > gpurun_out/abl_sq/a2_$i.log 2>&1 || exit $?
done
