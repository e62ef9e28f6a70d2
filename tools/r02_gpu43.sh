#!/bin/bash
# same-box C1 A/B of the drop-in step (old: 4 downloads + 3 sync uploads per step; new: 2 downloads), warmed, 20 episodes each, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export C1_WARM=1 C1_EPISODES=20
bash tools/gpu_round.sh \
  "for i in 1 2 3; do WH_PKG_DIR=build_ab/old_pkg python tools/dropin_c1.py && python tools/dropin_c1.py || exit 3; done"
