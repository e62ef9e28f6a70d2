#!/bin/bash
# rocprofv3 kernel trace + stats of the driver's exact bench command (BENCH_rNN.json's cmd), then a
# per-dispatch table of k_step from the same trace (tools/dispatch_table.py) so the timed launch's
# duration can be read next to the bench line's kernel_ms.
# Usage: bash tools/prof_driver.sh TAG [bench args...]   (default args: the driver's command)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=${1:-driver}; shift
ARGS=${*:---gpus 1 --steps 20 --warmup 5}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/bench.log 2>&1
rc=$?
echo "trace rc=$rc"
exit $rc
