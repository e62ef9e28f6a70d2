#!/bin/bash
# BaseEnv one-download _pack: GPU vector/drop-in tests, then same-box A/B of the dict sampler route (old package first) x3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_round.sh \
  "python -u -m pytest tests/test_gpu_vector.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread" \
  "for i in 1 2 3; do WH_PKG_DIR=build_ab/old_pkg python tools/baseenv_bench.py && python tools/baseenv_bench.py || exit 3; done"
