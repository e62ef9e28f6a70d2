#!/bin/bash
# A round's evidence passes (GPU box), laid out for tools/pmc_summary.py:
#  1) rocprofv3 kernel trace + stats of the driver's bench command;
#  2) per step-kernel launch shape (identical fused launches, tools/step_probe.py): kernel trace, FETCH_SIZE,
#     WRITE_SIZE, SQ issue counters and an SQ wait/LDS breakdown, each in its own pass;
#  3) the fused sampler step (tools/sampler_probe.py, k_sampler): trace, FETCH_SIZE, WRITE_SIZE;
#  4) the policy kernel (tools/mlp_bench.py, Medium, fragment operand): trace + GRBM_GUI_ACTIVE (clock).
#   bash tools/profile_round.sh TAG ["medium:8:20 medium:8:200 large:16:20"]   -> gpurun_out/prof_TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=${1:?usage: profile_round.sh TAG [shapes]}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
run() { local name=$1 limit=$2; shift 2
  timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" | tee -a $OUT/status.txt
  [ $rc -eq 0 ] || exit $rc; }
run driver 500 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/driver -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"
SQ2="SQ_WAVES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES"
for shape in ${2:-medium:8:20 medium:8:200 large:16:20}; do
  IFS=: read v n k <<< "$shape"
  P="python3 tools/step_probe.py --variant $v --agents $n --steps $k --launches 6"
  D=$OUT/${v}_n${n}_fused_k$k
  mkdir -p $D
  run ${v}${n}k${k}_trace 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $D/trace -o run -- $P
  run ${v}${n}k${k}_fetch 120 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $D/fetch -o run -- $P
  run ${v}${n}k${k}_write 120 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $D/write -o run -- $P
  run ${v}${n}k${k}_sq 120 rocprofv3 --pmc $SQ -T --output-format csv -d $D/sq -o run -- $P
  run ${v}${n}k${k}_sq2 120 rocprofv3 --pmc $SQ2 -T --output-format csv -d $D/sq2 -o run -- $P
done
D=$OUT/medium_n8_sampler
mkdir -p $D
P="python3 tools/sampler_probe.py --replays 2"
run sampler_trace 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $D/trace -o run -- $P
run sampler_fetch 120 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $D/fetch -o run -- $P
run sampler_write 120 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $D/write -o run -- $P
D=$OUT/medium_n8_mlp
mkdir -p $D
P="python3 tools/mlp_bench.py"
export MLP_VARIANTS=medium MLP_X=1
run mlp_trace 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $D/trace -o run -- $P
run mlp_grbm 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -T --output-format csv -d $D/grbm -o run -- $P
echo done | tee -a $OUT/status.txt
