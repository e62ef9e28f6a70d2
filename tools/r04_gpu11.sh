# Timing-only probes of the move loop's serial chain (wrong results): no occupancy test / no
# forbidden-move test / neither, against the production build; Medium-8 and Large-16
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r04_chain_probe.txt
for i in 1 2; do
  for lib in rllib-warehouse_amd/warehouse/_lib/libwarehouse_amd.so build_ab/noocc.so build_ab/nokey.so build_ab/nokeyocc.so; do
    echo "lib=$lib" >> gpurun_out/r04_chain_probe.txt
    for args in "--steps 200" "--variant large --agents 16 --steps 200"; do
      WAREHOUSE_AMD_AB=1 WAREHOUSE_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/step_probe.py $args >> gpurun_out/r04_chain_probe.txt 2>&1 || exit $?
    done
  done
done
grep -v amdgpu.ids gpurun_out/r04_chain_probe.txt
