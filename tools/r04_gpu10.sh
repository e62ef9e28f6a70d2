# Timing probe: cost of the greedy policy's per-agent loop, measured by running it again for 4 or 8
# agents with identical results (-DWH_POLICY_DUP=4/8) -- what a second wave computing half the agents'
# policy could take off the step's single wave
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r04_policy_dup.txt
for i in 1 2; do
  for lib in rllib-warehouse_amd/warehouse/_lib/libwarehouse_amd.so build_ab/dup4.so build_ab/dup8.so; do
    echo "lib=$lib" >> gpurun_out/r04_policy_dup.txt
    for args in "--steps 200" "--steps 20 --launches 8"; do
      WAREHOUSE_AMD_AB=1 WAREHOUSE_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/step_probe.py $args >> gpurun_out/r04_policy_dup.txt 2>&1 || exit $?
    done
  done
done
grep -v amdgpu.ids gpurun_out/r04_policy_dup.txt
