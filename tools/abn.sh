#!/bin/bash
# Same-box comparison of N library builds (run on the GPU box):
#   bash tools/abn.sh "python tools/ablate.py medium 8" ROUNDS A.so B.so C.so ...
# Alternates the builds round-robin so clock/thermal drift hits all; prints one line per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
CMD=$1; N=$2; shift 2
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for lib in "$@"; do
    out=$(WAREHOUSE_AMD_LIB=$lib ABL_MASKS=0 timeout -k 10 300 $CMD 2>/dev/null | tail -1) || exit $?
    echo "$lib $out" | tee -a gpurun_out/abn.log
  done
done
