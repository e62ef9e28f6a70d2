# desync at the driver's launch shape (20 steps), round-3 library vs this tree's, interleaved
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r04_desync20_ab.txt
for i in 1 2 3; do
  for lib in build_ab/r03.so rllib-warehouse_amd/warehouse/_lib/libwarehouse_amd.so; do
    echo "lib=$lib" >> gpurun_out/r04_desync20_ab.txt
    WAREHOUSE_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/step_probe.py --steps 20 --launches 8 --stagger >> gpurun_out/r04_desync20_ab.txt 2>&1 || exit $?
    WAREHOUSE_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/step_probe.py --steps 20 --launches 8 >> gpurun_out/r04_desync20_ab.txt 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/r04_desync20_ab.txt
for i in 1 2; do
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --no-policy --no-sampler --no-alt --no-cpu-baseline > gpurun_out/r04_bench3_$i.json 2> gpurun_out/r04_bench3.err || { tail -20 gpurun_out/r04_bench3.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r04_bench3_$i.json').read().strip().splitlines()[-1])
print('value', d['value'], 'kernel_ms', d['roofline']['kernel_ms'], 'desync', d['desync_episodes']['kernel_ms'], d['desync_episodes']['kernel_time_vs_synchronised'])
"
done
