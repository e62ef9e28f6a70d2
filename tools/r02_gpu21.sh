#!/bin/bash
# same-box A/B of the desync leg: previous commit (build_ab/prev.so) vs the working tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for i in 1 2; do
  for v in prev cur; do
    lib=build_ab/prev.so; [ $v = cur ] && lib=rllib-warehouse_amd/warehouse/_lib/libwarehouse_amd.so
    WAREHOUSE_AMD_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-alt --no-sampler --no-policy --no-cpu-baseline > gpurun_out/ab_${v}_$i.log 2>&1 || exit $?
  done
done
