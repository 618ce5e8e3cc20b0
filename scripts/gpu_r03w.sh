# Round 3: wavefront kernel with component 0 of the carried state from the previous tick
# (one lane shift fewer) and no per-lane padding branch (non-reflective chains): its tests
# (incl. 150-step runs through the unmasked stretch), the reference configurations' parity,
# then their rates (best of 3).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_wavefront_gpu.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "wavefront or reference_configs or llnl_full or gray" > gpurun_out/r03w_tests.log 2>&1 || { tail -60 gpurun_out/r03w_tests.log; exit 1; }
tail -2 gpurun_out/r03w_tests.log
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
" > gpurun_out/r03w_rates.jsonl 2>&1 || { tail -20 gpurun_out/r03w_rates.jsonl; exit 1; }
grep '^{' gpurun_out/r03w_rates.jsonl
