# sampler: 1-step instance restored to a single step (no slots, one image buffer), multi-step instance separate
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_vector.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04_gpu7_tests.log 2>&1 || { tail -40 gpurun_out/r04_gpu7_tests.log; exit 1; }
tail -2 gpurun_out/r04_gpu7_tests.log
: > gpurun_out/r04_sampler_ab2.txt
for i in 1 2; do
  for lib in build_ab/head.so rllib-warehouse_amd/warehouse/_lib/libwarehouse_amd.so; do
    echo "lib=$lib" >> gpurun_out/r04_sampler_ab2.txt
    F=20; [ $lib = build_ab/head.so ] && F=0
    WAREHOUSE_AMD_AB=1 WAREHOUSE_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/sampler_probe.py --fragment $F >> gpurun_out/r04_sampler_ab2.txt 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/r04_sampler_ab2.txt
