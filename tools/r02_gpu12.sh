#!/bin/bash
# greedy steps without the off-grid clamp, perm/bfe decode of goals: tests, probes, SQ counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_round.sh \
  "python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread" \
  "python bench.py --gpus 1 --steps 20 --warmup 5 --no-alt --no-sampler --no-policy --no-cpu-baseline" \
  "python tools/step_probe.py --steps 200 --launches 5" \
  "python tools/step_probe.py --variant large --agents 16 --steps 200 --launches 5" \
  "bash tools/sq_probe.sh medium_n8_k200 --steps 200 --launches 5"
