#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_round.sh \
  "MLP_ABLATE=0,1 python tools/mlp_bench.py" \
  "bash tools/mlp_counters.sh"
