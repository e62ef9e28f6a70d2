#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_round.sh \
  "python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread" \
  "python tools/launch_cost.py" \
  "python bench.py --gpus 1 --steps 20 --warmup 5" \
  "python tools/step_probe.py --variant small --agents 4 --envs 4096 --steps 200 && python tools/step_probe.py --variant large --agents 16 --steps 200 && python tools/step_probe.py --variant medium --agents 8 --steps 200" \
  "bash tools/prof_driver.sh r02_driver" \
  "bash tools/sq_probe.sh medium_n8_k200 --steps 200 --launches 5"
