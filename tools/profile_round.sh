#!/bin/bash
# rocprofv3 passes for the bench kernel (run on the GPU box).  Kernel trace + stats in one pass,
# then FETCH_SIZE and WRITE_SIZE in separate counter passes (they do not fit one TCC pass).
# Usage: bash tools/profile_round.sh TAG [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
run() { local name=$1 limit=$2; shift 2
  timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" | tee -a $OUT/status.txt
  [ $rc -eq 0 ] || exit $rc; }
run trace 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 bench.py --no-cpu-baseline "$@"
run fetch 600 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $OUT/fetch -o run -- python3 bench.py --no-cpu-baseline --steps 300 --warmup 20 "$@"
run write 600 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $OUT/write -o run -- python3 bench.py --no-cpu-baseline --steps 300 --warmup 20 "$@"
if [ -n "$SQ" ]; then
  run sq 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -T --output-format csv -d $OUT/sq -o run -- python3 bench.py --no-cpu-baseline --steps 300 --warmup 20 "$@"
fi
