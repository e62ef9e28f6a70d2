#!/bin/bash
# drop-in outputs as views of one device block (no gather kernel): drop-in parity tests, then C1 A/B vs the cat+float version (old first) x3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export C1_WARM=1 C1_EPISODES=20
bash tools/gpu_round.sh \
  "python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider -k dropin --timeout 300 --timeout-method thread" \
  "for i in 1 2 3; do WH_PKG_DIR=build_ab/old_pkg python tools/dropin_c1.py && python tools/dropin_c1.py || exit 3; done"
