# round 4: fused vector step tests, sampler/vector probes, desync A/B against the round-3 library, bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_vector.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04_gpu2_tests.log 2>&1 || { tail -40 gpurun_out/r04_gpu2_tests.log; exit 1; }
tail -4 gpurun_out/r04_gpu2_tests.log
: > gpurun_out/r04_desync_ab.txt
for i in 1 2 3; do
  for lib in build_ab/r03.so rllib-warehouse_amd/warehouse/_lib/libwarehouse_amd.so; do
    echo "lib=$lib" >> gpurun_out/r04_desync_ab.txt
    WAREHOUSE_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/step_probe.py --steps 200 --launches 6 --stagger >> gpurun_out/r04_desync_ab.txt 2>&1 || exit $?
    WAREHOUSE_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/step_probe.py --steps 200 --launches 6 >> gpurun_out/r04_desync_ab.txt 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/r04_desync_ab.txt
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04_bench2.json 2> gpurun_out/r04_bench2.err || { tail -20 gpurun_out/r04_bench2.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r04_bench2.json').read().strip().splitlines()[-1])
print('value', d['value'], 'kernel_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'], 'bound', d['roofline']['bound'])
print('sampler', d['sampler_path']['value'], d['sampler_path']['kernel_split_ms'])
print('vector', d['vector_path']['value'], d['vector_path']['roofline']['kernel_ms'])
print('desync', d['desync_episodes']['kernel_time_vs_synchronised'])
"
