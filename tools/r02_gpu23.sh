#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_round.sh \
  "python -u -m pytest tests/test_gpu_policy.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread" \
  "python bench.py --gpus 1 --steps 200 --warmup 5 --no-alt --no-desync --no-sampler --no-cpu-baseline" \
  "python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
