# same-box A/B of the sampler write-phase work split: head.so (1-step k_sampler, static), rows_static.so (multi-step,
# static share), this tree (multi-step, row chunks from an LDS counter); 1-step route and 20/100-step fragments
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r04_rows_ab.txt
for i in 1 2; do
  for lib in build_ab/head.so build_ab/rows_static.so rllib-warehouse_amd/warehouse/_lib/libwarehouse_amd.so; do
    echo "lib=$lib" >> gpurun_out/r04_rows_ab.txt
    F=20; [ $lib = build_ab/head.so ] && F=0
    WAREHOUSE_AMD_AB=1 WAREHOUSE_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/sampler_probe.py --fragment $F >> gpurun_out/r04_rows_ab.txt 2>&1 || exit $?
    [ $F = 20 ] && { WAREHOUSE_AMD_AB=1 WAREHOUSE_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/sampler_probe.py --fragment 100 --replays 3 2>&1 | grep rollout >> gpurun_out/r04_rows_ab.txt || exit $?; }
  done
done
grep -v amdgpu.ids gpurun_out/r04_rows_ab.txt
timeout -k 10 300 python tools/step_probe.py --steps 200 --launches 6 > gpurun_out/r04_step_check.txt 2>&1 || exit $?
timeout -k 10 300 python tools/step_probe.py --steps 20 --launches 8 >> gpurun_out/r04_step_check.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r04_step_check.txt
