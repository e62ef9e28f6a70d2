# MLP on 16x16x32 tiles: policy tests, then same-box A/B against the 32x32x16 kernel (WH_MLP_LEGACY=1)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_policy.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04_mlp_tests.log 2>&1 || { tail -40 gpurun_out/r04_mlp_tests.log; exit 1; }
tail -3 gpurun_out/r04_mlp_tests.log
: > gpurun_out/r04_mlp16_ab.txt
for i in 1 2; do
  for legacy in 1 0; do
    echo "WH_MLP_LEGACY=$legacy (1: 32x32x16 kernel)" >> gpurun_out/r04_mlp16_ab.txt
    if [ $legacy = 1 ]; then export WH_MLP_LEGACY=1; else unset WH_MLP_LEGACY; fi
    MLP_X=1 timeout -k 10 120 python tools/mlp_bench.py >> gpurun_out/r04_mlp16_ab.txt 2>&1 || exit $?
    timeout -k 10 120 python tools/mlp_bench.py >> gpurun_out/r04_mlp16_ab.txt 2>&1 || exit $?
  done
done
unset WH_MLP_LEGACY
grep -v amdgpu.ids gpurun_out/r04_mlp16_ab.txt
