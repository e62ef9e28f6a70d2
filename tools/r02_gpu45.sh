#!/bin/bash
# BaseEnv dict route A/B at B=2048 medium (try_reset of one env: whole-batch download before, one env's rows now), old package first, x2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export BE_ENVS=2048 BE_STEPS=240 BE_VARIANT=medium
bash tools/gpu_round.sh \
  "for i in 1 2; do WH_PKG_DIR=build_ab/old_pkg python tools/baseenv_bench.py && python tools/baseenv_bench.py || exit 3; done"
