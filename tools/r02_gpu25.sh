#!/bin/bash
# desynchronised episodes: where the extra time goes (expiry, reset: lane-parallel vs per-lane)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_round.sh \
  "ABL_STAGGER=1 ABL_MASKS=0,4 WAREHOUSE_AMD_LIB=build_ab/ablation.so python tools/ablate.py medium 8" \
  "ABL_MASKS=0,4 WAREHOUSE_AMD_LIB=build_ab/ablation.so python tools/ablate.py medium 8" \
  "ABL_STAGGER=1 ABL_MASKS=0 WAREHOUSE_AMD_LIB=build_ab/nolane.so python tools/ablate.py medium 8" \
  "ABL_STAGGER=1 ABL_MASKS=0 python tools/ablate.py medium 8" \
  "ABL_MASKS=0 python tools/ablate.py medium 8"
