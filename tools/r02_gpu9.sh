#!/bin/bash
# Table-load prologue fix + dispatch-attached events: GPU tests, launch costs, driver bench, probes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_round.sh \
  "python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread" \
  "python tools/launch_cost.py" \
  "python bench.py --gpus 1 --steps 20 --warmup 5" \
  "python tools/step_probe.py --steps 20 --launches 20" \
  "python tools/step_probe.py --steps 200 --launches 5" \
  "python tools/step_probe.py --variant large --agents 16 --steps 200 --launches 5"
