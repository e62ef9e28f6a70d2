# Same-box A/B: previous build (prebank), bank-conflict-free table copies with 16-bit pickup cells (pk16),
# table copies + 32-bit pickup cells (current); then the policy MLP against the vendor-library route
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r04_pk_ab.txt
for i in 1 2; do
  for lib in build_ab/prebank.so build_ab/pk16.so rllib-warehouse_amd/warehouse/_lib/libwarehouse_amd.so; do
    echo "lib=$lib" >> gpurun_out/r04_pk_ab.txt
    for args in "--steps 200" "--steps 20 --launches 8" "--variant large --agents 16 --steps 200" "--variant large --agents 16 --steps 20 --launches 8"; do
      WAREHOUSE_AMD_AB=1 WAREHOUSE_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/step_probe.py $args >> gpurun_out/r04_pk_ab.txt 2>&1 || exit $?
    done
    WAREHOUSE_AMD_AB=1 WAREHOUSE_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/sampler_probe.py >> gpurun_out/r04_pk_ab.txt 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/r04_pk_ab.txt
WH_MLP_WG4=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_policy.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04_mlp_wg4_tests.log 2>&1 || { tail -30 gpurun_out/r04_mlp_wg4_tests.log; exit 1; }
tail -1 gpurun_out/r04_mlp_wg4_tests.log
: > gpurun_out/r04_mlp_wg4_ab.txt
for i in 1 2; do
  for wg in 0 1; do
    echo "WH_MLP_WG4=$wg" >> gpurun_out/r04_mlp_wg4_ab.txt
    if [ $wg = 1 ]; then export WH_MLP_WG4=1; else unset WH_MLP_WG4; fi
    MLP_X=1 timeout -k 10 120 python tools/mlp_bench.py >> gpurun_out/r04_mlp_wg4_ab.txt 2>&1 || exit $?
  done
done
unset WH_MLP_WG4
grep -v amdgpu.ids gpurun_out/r04_mlp_wg4_ab.txt
MLP_LIB=1 timeout -k 10 300 python tools/mlp_bench.py > gpurun_out/r04_mlp_lib.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r04_mlp_lib.txt
