#!/bin/bash
# lazy rebuild v2 (co-located slots): co-location parity test, GPU suite, lazy vs eager A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
E=build_ab/eager.so
P="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
bash tools/gpu_round.sh \
  "$P tests/test_gpu_parity.py -k co_located" \
  "$P tests -m gpu" \
  "python tools/step_probe.py --steps 200 --launches 6" \
  "WAREHOUSE_AMD_LIB=$E python tools/step_probe.py --steps 200 --launches 6" \
  "python tools/step_probe.py --steps 200 --launches 6" \
  "WAREHOUSE_AMD_LIB=$E python tools/step_probe.py --steps 200 --launches 6" \
  "python tools/step_probe.py --variant large --agents 16 --steps 200 --launches 6" \
  "WAREHOUSE_AMD_LIB=$E python tools/step_probe.py --variant large --agents 16 --steps 200 --launches 6" \
  "python bench.py --gpus 1 --steps 20 --warmup 5" \
  "WAREHOUSE_AMD_LIB=$E python bench.py --gpus 1 --steps 20 --warmup 5" \
  "python bench.py --gpus 1 --steps 20 --warmup 5" \
  "WAREHOUSE_AMD_LIB=$E python bench.py --gpus 1 --steps 20 --warmup 5"
