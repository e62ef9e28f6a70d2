# Policy kernel: chunk staging by alternating wave halves (one wave of each SIMD stages, the other
# keeps the MFMA pipe busy) -- parity (test_gpu_policy) + same-box A/B against the previous build
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_policy.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04_gpu15_tests.log 2>&1 || { tail -30 gpurun_out/r04_gpu15_tests.log; exit 1; }
tail -1 gpurun_out/r04_gpu15_tests.log
: > gpurun_out/r04_mlp_stage_ab.txt
for i in 1 2; do
  for lib in build_ab/mlp_base.so rllib-warehouse_amd/warehouse/_lib/libwarehouse_amd.so; do
    echo "lib=$lib" >> gpurun_out/r04_mlp_stage_ab.txt
    MLP_X=1 WAREHOUSE_AMD_AB=1 WAREHOUSE_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/mlp_bench.py >> gpurun_out/r04_mlp_stage_ab.txt 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/r04_mlp_stage_ab.txt
