#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_round.sh "bash tools/mlp_counters.sh medium" "bash tools/mlp_counters.sh large"
