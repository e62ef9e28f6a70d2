#!/bin/bash
# final round-2 evidence: GPU tests, the driver's bench command + its rocprof trace, SQ/PMC probes
# of the timed launch shape (K=20) and of 200-step launches (Medium-8, Large-16), full default bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_round.sh \
  "python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread" \
  "python bench.py --gpus 1 --steps 20 --warmup 5" \
  "bash tools/prof_driver.sh driver" \
  "bash tools/sq_probe.sh medium_n8_k20 --steps 20 --launches 20" \
  "bash tools/sq_probe.sh medium_n8_k200 --steps 200 --launches 5" \
  "bash tools/sq_probe.sh large_n16_k200 --variant large --agents 16 --steps 200 --launches 5" \
  "python tools/launch_cost.py"
