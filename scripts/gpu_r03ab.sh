# Round 3 (re-entry, rebuilt container): smoke, the driver's bench command and the reference
# configurations' rates (best of 3) at HEAD -- the baseline for the multi-wave wavefront.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03ab_smoke.log 2>&1 || { tail -20 gpurun_out/r03ab_smoke.log; exit 1; }
tail -2 gpurun_out/r03ab_smoke.log
timeout -k 10 300 python -u -c "
import json, sys
sys.path[:0] = ['.', 'radiative-transfer_amd']
import bench, rtsn
pdir = bench.REPO / 'tests' / 'golden' / 'prm'
for rep in range(3):
    for name in bench.REFERENCE_CONFIGS:
        ph = rtsn.ParameterHandler(pdir / name, table_dir=str(pdir) + '/')
        q = ph.params
        g = bench.gpu_rate(q, q['ts_method'], 1000)
        print(json.dumps(dict(config=name, rep=rep, **g)), flush=True)
" > gpurun_out/r03ab_rates.jsonl 2>&1 || { tail -20 gpurun_out/r03ab_rates.jsonl; exit 1; }
grep '^{' gpurun_out/r03ab_rates.jsonl
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03ab_bench.log 2>&1 || { tail -30 gpurun_out/r03ab_bench.log; exit 1; }
grep "^{" gpurun_out/r03ab_bench.log | tail -1 > gpurun_out/r03ab_bench.json
python3 -c "
import json; d=json.load(open('gpurun_out/r03ab_bench.json')); r=d['roofline']
print('value', d['value'], 'ms/step', d['ms_per_step'], 'kern', r['kernel_ms'], 'frac', r['frac'], 'finite', d['state_finite'])
print('gather', d['gather']); print('llnl', d.get('llnl_slab_test'))"
