#!/bin/bash
# Round-3 evidence passes (GPU box).  1) rocprofv3 kernel trace + stats of the driver's bench command;
# 2) per launch shape (identical fused launches of tools/step_probe.py): kernel trace, FETCH_SIZE,
# WRITE_SIZE and SQ issue counters in separate passes, laid out for tools/pmc_summary.py.
#   bash tools/profile_r03.sh ["medium:8:20 medium:8:200 large:16:200"]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/prof_r03
mkdir -p $OUT
run() { local name=$1 limit=$2; shift 2
  timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" | tee -a $OUT/status.txt
  [ $rc -eq 0 ] || exit $rc; }
run driver 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/driver -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"
for shape in ${1:-medium:8:20 medium:8:200 large:16:200}; do
  IFS=: read v n k <<< "$shape"
  P="python3 tools/step_probe.py --variant $v --agents $n --steps $k --launches 6"
  D=$OUT/${v}_n${n}_fused_k$k
  mkdir -p $D
  run ${v}${n}k${k}_trace 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $D/trace -o run -- $P
  run ${v}${n}k${k}_fetch 120 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $D/fetch -o run -- $P
  run ${v}${n}k${k}_write 120 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $D/write -o run -- $P
  run ${v}${n}k${k}_sq 120 rocprofv3 --pmc $SQ -T --output-format csv -d $D/sq -o run -- $P
done
