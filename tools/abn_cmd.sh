#!/bin/bash
# Same-box A/B/... of library builds, interleaved so clock and thermal drift hit all of them:
#   bash tools/abn_cmd.sh "tree obsu2 obsu4" "python tools/obs_bench.py" [rounds]
# ("tree" = the in-tree library, otherwise build_ab/<name>.so); output gpurun_out/abn_<name>.txt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for i in $(seq 1 ${3:-3}); do
  for lib in $1; do
    so=build_ab/$lib.so; [ "$lib" = tree ] && so=rllib-warehouse_amd/warehouse/_lib/libwarehouse_amd.so
    WAREHOUSE_AMD_LIB=$so timeout -k 10 300 $2 >> gpurun_out/abn_$lib.txt 2>&1 || exit $?
  done
done
