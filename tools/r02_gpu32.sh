#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_round.sh \
  "python -u -m pytest tests/test_gpu_policy.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread" \
  "python tools/obs_bench.py" \
  "WAREHOUSE_AMD_LIB=build_ab/obsnt.so python tools/obs_bench.py" \
  "python tools/obs_bench.py" \
  "WAREHOUSE_AMD_LIB=build_ab/obsnt.so python tools/obs_bench.py" \
  "python tools/write_ceiling.py"
