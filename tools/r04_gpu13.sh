# SQ counters of the policy kernel (k_mlp16, Medium, fragment operand): where its non-MFMA time goes
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/prof_mlp
mkdir -p $OUT
export MLP_VARIANTS=medium,large MLP_X=1
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS -T --output-format csv -d $OUT/sq1 -o run -- python3 tools/mlp_bench.py > $OUT/sq1.log 2>&1 || { tail -20 $OUT/sq1.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -T --output-format csv -d $OUT/sq2 -o run -- python3 tools/mlp_bench.py > $OUT/sq2.log 2>&1 || { tail -20 $OUT/sq2.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 tools/mlp_bench.py > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
echo done
