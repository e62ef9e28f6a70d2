#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_round.sh \
  "MLP_VARIANTS=medium,large MLP_ABLATE=0,1 python tools/mlp_bench.py" \
  "WAREHOUSE_AMD_LIB=build_ab/mlpabl.so MLP_VARIANTS=medium,large MLP_ABLATE=0,16,1,9,17,25 python tools/mlp_bench.py"
