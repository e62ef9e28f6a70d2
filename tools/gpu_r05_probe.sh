#!/bin/bash
# Round-5 probe batch (GPU box): the occupancy-ahead x pickup-plane A/B, per-phase SQ attribution of the fused step
# kernel (Medium-8, Large-16; tools/wait_attrib.py) and the bare 16x16x32 MFMA loop ceiling.
# Each step under its own time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 840 python tools/abrun.py run tools/ab/r05_occ.json > gpurun_out/abrun.log 2>&1 &&
WAREHOUSE_AMD_LIB=$PWD/build_ab/ablm8.so WAREHOUSE_AMD_AB=1 timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d gpurun_out/wattr_m8 -o run -- python3 tools/wait_attrib.py > gpurun_out/wattr_m8.log 2>&1 &&
cp gpurun_out/wattr_plan.json gpurun_out/wattr_m8_plan.json &&
timeout -k 10 120 ./build_ab/mfma16_ceiling > gpurun_out/mfma16_ceiling.txt 2>&1 &&
WATTR_VARIANT=large WATTR_AGENTS=16 WAREHOUSE_AMD_LIB=$PWD/build_ab/abll16.so WAREHOUSE_AMD_AB=1 timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/wattr_l16 -o run -- python3 tools/wait_attrib.py > gpurun_out/wattr_l16.log 2>&1 &&
cp gpurun_out/wattr_plan.json gpurun_out/wattr_l16_plan.json
