# full -m gpu suite + smoke + the driver's bench command; each step under its own limit, stop at the first failure
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04_pytest.log 2>&1 || { tail -40 gpurun_out/r04_pytest.log; exit 1; }
tail -3 gpurun_out/r04_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke.log 2>&1 || { tail -20 gpurun_out/r04_smoke.log; exit 1; }
tail -1 gpurun_out/r04_smoke.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04_bench.json 2> gpurun_out/r04_bench.err || { tail -20 gpurun_out/r04_bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r04_bench.json').read().strip().splitlines()[-1])
r=d['roofline']
print('value', d['value'], 'kernel_ms', r['kernel_ms'], 'frac', r['frac'], 'bound', r['bound'], 'valu', (r.get('valu') or {}).get('frac'))
print('sampler', d['sampler_path']['value'], d['sampler_path']['kernel_split_ms'], 'step share', d['sampler_path'].get('step_share_ms'))
print('fragments', (d.get('sampler_fragments') or {}).get('value'), 'vector', (d.get('vector_path') or {}).get('value'))
print('policy', d['policy_path']['value'], d['policy_path']['roofline']['frac'])
print('desync', d['desync_episodes']['kernel_time_vs_synchronised'])
print('cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores'])
"
