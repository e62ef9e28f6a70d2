#!/bin/bash
# where the drop-in single-env step spends its time (cProfile of tools/dropin_c1.py, warmed, 20 episodes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export C1_WARM=1 C1_EPISODES=20
bash tools/gpu_round.sh "python -m cProfile -s tottime tools/dropin_c1.py 2>&1 | head -45"
