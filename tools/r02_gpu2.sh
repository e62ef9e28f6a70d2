#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_round.sh "tools/oprate5_bin" "python tools/launch_cost.py" \
  "python -u -m pytest tests/test_gpu_draws.py tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread" \
  "python bench.py --gpus 1 --steps 20 --warmup 5" \
  "bash tools/prof_driver.sh r02_driver"
