# Large-16 at 200-step launches (C4 steady state) on this round's kernels: kernel trace, FETCH_SIZE,
# WRITE_SIZE, SQ issue counters and the SQ wait/LDS breakdown, each pass on its own (tools/pmc_summary.py)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/prof_r04
mkdir -p $OUT
run() { local name=$1 limit=$2; shift 2
  timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || exit $rc; }
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"
SQ2="SQ_WAVES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES"
P="python3 tools/step_probe.py --variant large --agents 16 --steps 200 --launches 6"
D=$OUT/large_n16_fused_k200
rm -rf $D && mkdir -p $D
run large16k200_trace 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $D/trace -o run -- $P
run large16k200_fetch 120 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $D/fetch -o run -- $P
run large16k200_write 120 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $D/write -o run -- $P
run large16k200_sq 120 rocprofv3 --pmc $SQ -T --output-format csv -d $D/sq -o run -- $P
run large16k200_sq2 120 rocprofv3 --pmc $SQ2 -T --output-format csv -d $D/sq2 -o run -- $P
echo done
