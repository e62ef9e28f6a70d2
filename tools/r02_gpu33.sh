#!/bin/bash
# lazy occupancy rebuild: GPU tests, then lazy (default build) vs eager (-DWH_EAGER_GRID) A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
E=build_ab/eager.so
bash tools/gpu_round.sh \
  "python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread" \
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
