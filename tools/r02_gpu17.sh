#!/bin/bash
# MLP: where the time goes (same box): normal build (staging on/off), ablation build (relu, barriers, obs loads)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_round.sh \
  "MLP_ABLATE=0,1 python tools/mlp_bench.py" \
  "WAREHOUSE_AMD_LIB=build_ab/mlpabl.so MLP_ABLATE=0,1,3,5,9,15 python tools/mlp_bench.py" \
  "bash tools/mlp_counters.sh medium" "bash tools/mlp_counters.sh large"
