#!/bin/bash
# Round-5 probe batch 2 (GPU box): pickup-lookup distance A/B and the MFMA loop ceilings by waves
# per SIMD and sample tiles per A operand.  Each step under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 120 ./build_ab/mfma16_ceiling > gpurun_out/mfma16_ceiling.txt 2>&1 &&
timeout -k 10 700 python tools/abrun.py run tools/ab/r05_pick.json > gpurun_out/abrun.log 2>&1
