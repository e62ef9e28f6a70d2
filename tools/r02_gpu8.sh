#!/bin/bash
# Round 2 re-entry: GPU tests, the driver's bench command, its rocprof trace, SQ probes at HEAD.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_round.sh \
  "python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread" \
  "python bench.py --gpus 1 --steps 20 --warmup 5" \
  "bash tools/prof_driver.sh driver" \
  "bash tools/sq_probe.sh medium_n8_k20 --steps 20 --launches 20" \
  "bash tools/sq_probe.sh medium_n8_k200 --steps 200 --launches 5" \
  "python tools/launch_cost.py"
