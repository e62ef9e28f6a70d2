#!/bin/bash
# policy MLP without layer-0 recompute: policy tests, timing per variant, SQ MFMA counters (Medium)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_round.sh \
  "python -u -m pytest tests/test_gpu_policy.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread" \
  "python tools/mlp_bench.py" \
  "python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
