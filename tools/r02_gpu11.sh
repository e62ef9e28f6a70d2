#!/bin/bash
# Floyd reset + open-request expiry walk: GPU tests, driver bench, probes (sync + desync), trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_round.sh \
  "python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread" \
  "python bench.py --gpus 1 --steps 20 --warmup 5" \
  "python tools/step_probe.py --steps 20 --launches 20" \
  "python tools/step_probe.py --steps 200 --launches 5" \
  "python tools/step_probe.py --variant large --agents 16 --steps 200 --launches 5" \
  "python bench.py --gpus 1 --steps 200 --warmup 20 --no-alt --no-sampler --no-policy --no-cpu-baseline"
