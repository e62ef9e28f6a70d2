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
MLP_LIB=1 timeout -k 10 300 python tools/mlp_bench.py > gpurun_out/r04_mlp_lib.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r04_mlp_lib.txt
