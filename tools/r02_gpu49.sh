#!/bin/bash
# whole GPU suite, then C1 A/B (old = HEAD package, first) x3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export C1_WARM=1 C1_EPISODES=20
bash tools/gpu_round.sh \
  "python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread" \
  "for i in 1 2 3; do WH_PKG_DIR=build_ab/old_pkg python tools/dropin_c1.py && python tools/dropin_c1.py || exit 3; done"
