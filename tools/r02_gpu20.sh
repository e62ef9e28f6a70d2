#!/bin/bash
# phase ablations (timing only) of the fused step kernel, Medium-8 and Large-16
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_round.sh \
  "WAREHOUSE_AMD_LIB=build_ab/ablation.so python tools/ablate.py medium 8" \
  "WAREHOUSE_AMD_LIB=build_ab/ablation.so python tools/ablate.py large 16"
