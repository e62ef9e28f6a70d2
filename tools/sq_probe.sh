#!/bin/bash
# rocprofv3 passes over tools/step_probe.py (identical fused launches): kernel trace + stats, then
# FETCH_SIZE, WRITE_SIZE and the SQ issue counters, each in its own pass.
# Usage: bash tools/sq_probe.sh TAG [step_probe args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
run() { local name=$1; shift
  timeout -k 10 120 "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" | tee -a $OUT/status.txt
  [ $rc -eq 0 ] || exit $rc; }
run probe python3 tools/step_probe.py "$@"
run trace rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 tools/step_probe.py "$@"
run fetch rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $OUT/fetch -o run -- python3 tools/step_probe.py "$@"
run write rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $OUT/write -o run -- python3 tools/step_probe.py "$@"
run sq rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -T --output-format csv -d $OUT/sq -o run -- python3 tools/step_probe.py "$@"
run sq2 rocprofv3 --pmc SQ_WAVES SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS -T --output-format csv -d $OUT/sq2 -o run -- python3 tools/step_probe.py "$@"
