# Rehearsal of the driver's N = 2 command on one card (both ranks share it: the per-rank numbers are
# not a scaling measurement; this checks the multi-rank path end to end -- gloo barriers, max over
# ranks, one rank-0 line with cpu_baseline)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/r04_n2_rehearsal.json 2> gpurun_out/r04_n2_rehearsal.err || { tail -30 gpurun_out/r04_n2_rehearsal.err; exit 1; }
python -c "
import json; lines=[l for l in open('gpurun_out/r04_n2_rehearsal.json').read().splitlines() if l.startswith('{')]
print(len(lines), 'json line(s)')
d=json.loads(lines[-1]); print('n_gpus', d['n_gpus'], 'value', d['value'], 'cpu_baseline' in d, d.get('cpu_baseline',{}).get('cores'))
"
