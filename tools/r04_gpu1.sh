# round 4: new parity tests (fused sampler, key forms) + the sampler route probe + the fused-launch split
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_vector.py tests/test_gpu_parity.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "fused_sampler or key_forms or sampler" > gpurun_out/r04_gpu1_tests.log 2>&1 || { tail -30 gpurun_out/r04_gpu1_tests.log; exit 1; }
tail -15 gpurun_out/r04_gpu1_tests.log
timeout -k 10 120 python tools/sampler_probe.py > gpurun_out/r04_sampler_probe.txt 2>&1 || exit $?
WH_SAMPLER_UNFUSED=1 timeout -k 10 120 python tools/sampler_probe.py >> gpurun_out/r04_sampler_probe.txt 2>&1 || exit $?
cat gpurun_out/r04_sampler_probe.txt
