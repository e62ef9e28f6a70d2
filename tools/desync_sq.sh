cd "${GRAFT_REPO_ROOT:-.}" || exit 2
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_BRANCH"
for k in 20 200; do
  for st in "" "--stagger"; do
    tag=k${k}${st:+_stagger}
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/dsq/$tag/trace -o run -- python3 tools/step_probe.py --steps $k --launches 6 $st > gpurun_out/dsq/$tag.log 2>&1 || exit 3
    timeout -k 10 200 rocprofv3 --pmc $SQ -T --output-format csv -d gpurun_out/dsq/$tag/sq -o run -- python3 tools/step_probe.py --steps $k --launches 6 $st >> gpurun_out/dsq/$tag.log 2>&1 || exit 3
  done
done
