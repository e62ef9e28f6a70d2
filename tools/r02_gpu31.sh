#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_round.sh \
  "python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread" \
  "python tools/step_probe.py --steps 20 --launches 21" \
  "WAREHOUSE_AMD_LIB=build_ab/nolane.so python tools/step_probe.py --steps 20 --launches 21" \
  "python tools/step_probe.py --steps 200 --launches 5" \
  "python bench.py --gpus 1 --steps 20 --warmup 5 --no-alt --no-sampler --no-policy --no-cpu-baseline"
