#!/bin/bash
# BASELINE.json configs 1-4 on one GPU (config 5 = config 3 x 8 GPUs is the driver's scaling run):
# one JSON line each into gpurun_out/configs.jsonl.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
OUT=gpurun_out/configs.jsonl
: > $OUT
run() { timeout -k 10 600 "$@" 2>/dev/null | tail -1 >> $OUT; }
run python tools/dropin_c1.py && \
run python bench.py --variant small --agents 4 --envs 4096 --policy random --no-alt --no-sampler --no-policy --no-cpu-baseline && \
run python bench.py --no-alt --no-sampler --no-policy --no-cpu-baseline && \
run python bench.py --variant large --agents 16 --no-alt --no-sampler --no-policy --no-cpu-baseline
