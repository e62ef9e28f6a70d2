#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_round.sh \
  "python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread" \
  "tools/oprate5_bin" "python tools/launch_cost.py" \
  "python bench.py --gpus 1 --steps 20 --warmup 5" \
  "python bench.py"
