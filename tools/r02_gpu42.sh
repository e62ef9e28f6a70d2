#!/bin/bash
# drop-in (single env) step with one download per step: parity tests, then same-box C1 A/B (old vs new)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_round.sh \
  "python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider -k dropin --timeout 300 --timeout-method thread" \
  "WH_PKG_DIR=build_ab/old_pkg python tools/dropin_c1.py && python tools/dropin_c1.py && WH_PKG_DIR=build_ab/old_pkg python tools/dropin_c1.py && python tools/dropin_c1.py"
