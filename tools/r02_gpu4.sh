#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_round.sh \
  "python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread" \
  "WAREHOUSE_AMD_LIB=build_ab/ablation.so python tools/ablate.py medium 8 && WAREHOUSE_AMD_LIB=build_ab/ablation.so python tools/ablate.py large 16" \
  "bash tools/sq_probe.sh large_n16_k200 --variant large --agents 16 --steps 200 --launches 5" \
  "bash tools/sq_probe.sh medium_n8_k20 --steps 20 --launches 20" \
  "python bench.py --gpus 1 --steps 20 --warmup 5"
