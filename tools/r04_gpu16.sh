# Scheduler strategy of the step/sampler object (SCHED_warehouse_amd): same-box A/B of the production
# iterative-ilp build against max-ilp, iterative-minreg, max-memory-clause builds of the same sources
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r04_sched_ab.txt
for i in 1 2; do
  for lib in rllib-warehouse_amd/warehouse/_lib/libwarehouse_amd.so build_ab/sched_max-ilp.so build_ab/sched_iterative-minreg.so build_ab/sched_max-memory-clause.so; do
    echo "lib=$lib" >> gpurun_out/r04_sched_ab.txt
    for args in "--steps 200" "--steps 20 --launches 8" "--variant large --agents 16 --steps 200"; do
      WAREHOUSE_AMD_AB=1 WAREHOUSE_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/step_probe.py $args >> gpurun_out/r04_sched_ab.txt 2>&1 || exit $?
    done
    WAREHOUSE_AMD_AB=1 WAREHOUSE_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/sampler_probe.py >> gpurun_out/r04_sched_ab.txt 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/r04_sched_ab.txt
