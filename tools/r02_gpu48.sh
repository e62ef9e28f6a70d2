#!/bin/bash
# drop-in C1 A/B (old = HEAD package) with the parity and stream tests first; reused for successive host-side changes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export C1_WARM=1 C1_EPISODES=20
bash tools/gpu_round.sh \
  "python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_parity.py -x -q -p no:cacheprovider -k 'dropin or stream' --timeout 300 --timeout-method thread" \
  "for i in 1 2 3; do WH_PKG_DIR=build_ab/old_pkg python tools/dropin_c1.py && python tools/dropin_c1.py || exit 3; done"
