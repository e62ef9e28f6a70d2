# LDS bank-conflict-free table copies + 32-bit pickup cells: parity tests, then same-box A/B against the
# previous build (build_ab/prebank.so), Medium-8 / Large-16 at 200- and 20-step launches, desync, sampler
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_vector.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04_gpu8_tests.log 2>&1 || { tail -40 gpurun_out/r04_gpu8_tests.log; exit 1; }
tail -2 gpurun_out/r04_gpu8_tests.log
: > gpurun_out/r04_bank_ab.txt
for i in 1 2; do
  for lib in build_ab/prebank.so rllib-warehouse_amd/warehouse/_lib/libwarehouse_amd.so; do
    echo "lib=$lib" >> gpurun_out/r04_bank_ab.txt
    for args in "--steps 200" "--steps 200 --stagger" "--steps 20 --launches 8" "--variant large --agents 16 --steps 200" "--variant large --agents 16 --steps 20 --launches 8"; do
      WAREHOUSE_AMD_AB=1 WAREHOUSE_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/step_probe.py $args >> gpurun_out/r04_bank_ab.txt 2>&1 || exit $?
    done
    WAREHOUSE_AMD_AB=1 WAREHOUSE_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/sampler_probe.py >> gpurun_out/r04_bank_ab.txt 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/r04_bank_ab.txt
