# The move loop's blocked-move test as precomputed pair flags (two v_bitop3 levels per agent on the
# serial chain): parity tests, then same-box A/B against the serial key test (-DWH_SERIAL_KEYS)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_vector.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04_gpu12_tests.log 2>&1 || { tail -40 gpurun_out/r04_gpu12_tests.log; exit 1; }
tail -2 gpurun_out/r04_gpu12_tests.log
: > gpurun_out/r04_flags_ab.txt
for i in 1 2; do
  for lib in build_ab/serial.so rllib-warehouse_amd/warehouse/_lib/libwarehouse_amd.so; do
    echo "lib=$lib" >> gpurun_out/r04_flags_ab.txt
    for args in "--steps 200" "--steps 200 --stagger" "--steps 20 --launches 8" "--variant large --agents 16 --steps 200" "--variant large --agents 16 --steps 20 --launches 8" "--variant small --agents 4 --steps 200"; do
      WAREHOUSE_AMD_AB=1 WAREHOUSE_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/step_probe.py $args >> gpurun_out/r04_flags_ab.txt 2>&1 || exit $?
    done
    WAREHOUSE_AMD_AB=1 WAREHOUSE_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/sampler_probe.py >> gpurun_out/r04_flags_ab.txt 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/r04_flags_ab.txt
