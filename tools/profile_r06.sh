#!/bin/bash
# Round-6 evidence passes (GPU box), laid out for tools/pmc_summary.py (one directory per launch shape):
#  1) rocprofv3 kernel trace + stats of the driver's bench command;
#  2) per step-kernel launch shape (tools/step_probe.py, identical launches placed across an episode end
#     like the bench window): kernel trace, FETCH_SIZE, WRITE_SIZE and the SQ issue counters, each in its
#     own pass.  Shapes: C3 (medium:8:greedy:65536), C4 (large:16:greedy:65536), C2 (small:4:random:4096)
#     at the driver's 20 steps per launch, and C3/C4 at 200.
#   bash tools/profile_r06.sh TAG ["medium:8:greedy:65536:20 ..."]   -> gpurun_out/prof_TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=${1:?usage: profile_r06.sh TAG [shapes]}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
run() { local name=$1 limit=$2; shift 2
  timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" | tee -a $OUT/status.txt
  [ $rc -eq 0 ] || exit $rc; }
if [ -z "$NO_DRIVER" ]; then
  run driver 500 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/driver -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5
fi
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"
SQ2="SQ_WAVES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES"
for shape in ${2:-medium:8:greedy:65536:20 medium:8:greedy:65536:200 large:16:greedy:65536:20 large:16:greedy:65536:200 small:4:random:4096:20}; do
  IFS=: read v n pol envs k <<< "$shape"
  P="python3 tools/step_probe.py --variant $v --agents $n --policy $pol --envs $envs --steps $k --launches 6 --cross"
  if [ "$pol" = greedy ] && [ "$envs" = 65536 ]; then D=$OUT/${v}_n${n}_fused_k$k; else D=$OUT/${v}_n${n}_${pol}_b${envs}_fused_k$k; fi
  mkdir -p $D
  nm=$(basename $D)
  run ${nm}_trace 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $D/trace -o run -- $P
  run ${nm}_fetch 120 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $D/fetch -o run -- $P
  run ${nm}_write 120 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $D/write -o run -- $P
  run ${nm}_sq 120 rocprofv3 --pmc $SQ -T --output-format csv -d $D/sq -o run -- $P
  run ${nm}_sq2 120 rocprofv3 --pmc $SQ2 -T --output-format csv -d $D/sq2 -o run -- $P
done
echo done | tee -a $OUT/status.txt
