cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for spec in "medium 8 65536" "medium 8 131072" "medium 8 262144" "large 16 65536" "large 16 131072"; do
  set -- $spec
  timeout -k 10 120 python tools/step_probe.py --variant $1 --agents $2 --envs $3 --steps 200 --launches 6 >> gpurun_out/r04_bscale.txt 2>&1 || exit $?
done
cat gpurun_out/r04_bscale.txt
