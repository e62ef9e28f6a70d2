#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_round.sh \
  "python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread" \
  "python tools/step_probe.py --steps 200 --launches 5" \
  "python tools/step_probe.py --variant large --agents 16 --steps 200 --launches 5"
