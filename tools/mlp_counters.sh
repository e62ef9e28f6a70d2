#!/bin/bash
# MFMA/LDS counters for the policy kernel (GPU box).  Usage: bash tools/mlp_counters.sh [small|medium|large]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
V=${1:-medium}
OUT=gpurun_out/mlpc_$V
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/avail.txt 2>&1
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA"
P3="SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_MFMA_BF16"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  MLP_VARIANTS=$V MLP_B=16384 timeout -k 10 300 rocprofv3 --pmc $P -T --output-format csv -d $OUT/p$i -o run -- python3 tools/mlp_bench.py > $OUT/p$i.log 2>&1
  echo "pass $i rc=$?" >> $OUT/status.txt
done
exit 0
