#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_round.sh \
  "python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread" \
  "ABL_STAGGER=1 ABL_MASKS=0 python tools/ablate.py medium 8" \
  "ABL_STAGGER=1 ABL_MASKS=0 WAREHOUSE_AMD_LIB=build_ab/nolane.so python tools/ablate.py medium 8" \
  "ABL_MASKS=0 python tools/ablate.py medium 8" \
  "ABL_MASKS=0 WAREHOUSE_AMD_LIB=build_ab/nolane.so python tools/ablate.py medium 8" \
  "python bench.py --gpus 1 --steps 20 --warmup 5 --no-alt --no-sampler --no-policy --no-cpu-baseline"
