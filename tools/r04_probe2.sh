cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./tools/obs_write_probe_bin > gpurun_out/r04_obs_write_probe.txt 2>&1 || exit $?
timeout -k 10 120 python tools/write_ceiling.py >> gpurun_out/r04_obs_write_probe.txt 2>&1 || exit $?
cat gpurun_out/r04_obs_write_probe.txt
