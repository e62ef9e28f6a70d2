#!/bin/bash
# Same-box A/B of two builds of the library (run on the GPU box):
#   bash tools/ab.sh A.so B.so "python tools/ablate.py medium 8" [rounds]
# Alternates A, B, A, B ... so clock/thermal drift hits both; each run's output goes to
# gpurun_out/ab_<A|B>_<i>.log.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
A=$1; B=$2; CMD=$3; N=${4:-3}
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    WAREHOUSE_AMD_LIB=$lib timeout -k 10 300 $CMD > gpurun_out/ab_${v}_$i.log 2>&1 || exit $?
  done
done
