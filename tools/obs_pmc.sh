#!/bin/bash
# Large-16 observation rows (the chunked k_observe) under rocprofv3: kernel trace, FETCH_SIZE and
# WRITE_SIZE, each pass its own run (GPU box):  bash tools/obs_pmc.sh TAG  -> gpurun_out/obs_TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp OBS_SHAPES="large:16"
OUT=gpurun_out/obs_${1:?usage: obs_pmc.sh TAG}
mkdir -p $OUT
run() { local name=$1; shift; timeout -k 10 180 "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc; }
run trace rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 tools/obs_bench.py
run fetch rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $OUT/fetch -o run -- python3 tools/obs_bench.py
run write rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $OUT/write -o run -- python3 tools/obs_bench.py
echo done >> $OUT/status.txt
