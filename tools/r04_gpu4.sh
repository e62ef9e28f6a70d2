# sampler rollout tests + probe; FastRun refactor A/B vs HEAD library
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_vector.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "sampler_rollout or fused" > gpurun_out/r04_gpu4_tests.log 2>&1 || { tail -40 gpurun_out/r04_gpu4_tests.log; exit 1; }
tail -4 gpurun_out/r04_gpu4_tests.log
timeout -k 10 120 python tools/sampler_probe.py --fragment 20 > gpurun_out/r04_sampler_probe2.txt 2>&1 || exit $?
timeout -k 10 120 python tools/sampler_probe.py --fragment 100 --replays 3 >> gpurun_out/r04_sampler_probe2.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r04_sampler_probe2.txt
: > gpurun_out/r04_fastrun_ab.txt
for i in 1 2; do
  for lib in build_ab/head.so rllib-warehouse_amd/warehouse/_lib/libwarehouse_amd.so; do
    echo "lib=$lib" >> gpurun_out/r04_fastrun_ab.txt
    WAREHOUSE_AMD_AB=1 WAREHOUSE_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/step_probe.py --steps 200 --launches 6 >> gpurun_out/r04_fastrun_ab.txt 2>&1 || exit $?
    WAREHOUSE_AMD_AB=1 WAREHOUSE_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/step_probe.py --steps 200 --launches 6 --stagger >> gpurun_out/r04_fastrun_ab.txt 2>&1 || exit $?
    WAREHOUSE_AMD_AB=1 WAREHOUSE_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/step_probe.py --steps 20 --launches 8 >> gpurun_out/r04_fastrun_ab.txt 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/r04_fastrun_ab.txt
: > gpurun_out/r04_sampler_ab.txt
for i in 1 2; do
  for lib in build_ab/head.so rllib-warehouse_amd/warehouse/_lib/libwarehouse_amd.so; do
    echo "lib=$lib" >> gpurun_out/r04_sampler_ab.txt
    WAREHOUSE_AMD_AB=1 WAREHOUSE_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/sampler_probe.py >> gpurun_out/r04_sampler_ab.txt 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/r04_sampler_ab.txt
