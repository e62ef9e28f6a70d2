#!/bin/bash
# BaseEnv dict building from lists: GPU vector tests, then B=2048 medium A/B (old package first) x3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export BE_ENVS=2048 BE_STEPS=240 BE_VARIANT=medium
bash tools/gpu_round.sh \
  "python -u -m pytest tests/test_gpu_vector.py -x -q -p no:cacheprovider -k base_env --timeout 300 --timeout-method thread" \
  "for i in 1 2 3; do WH_PKG_DIR=build_ab/old_pkg python tools/baseenv_bench.py && python tools/baseenv_bench.py || exit 3; done"
