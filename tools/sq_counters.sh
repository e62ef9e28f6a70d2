#!/bin/bash
# Issue/stall counter passes for the step kernel (GPU box).  Usage: bash tools/sq_counters.sh TAG [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/sq_$TAG
mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_INT64 SQ_IFETCH SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P3="SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SMEM"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $P -T --output-format csv -d $OUT/p$i -o run -- python3 bench.py --no-cpu-baseline --steps 400 --warmup 20 "$@" > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc" | tee -a $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
done
