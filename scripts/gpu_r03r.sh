# Round 3: wavefront kernel, line-map loads in flight together: its tests, then the reference
# configurations' rates.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_wavefront_gpu.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "wavefront or reference_configs or llnl_full or gray" > gpurun_out/r03r_tests.log 2>&1 || { tail -60 gpurun_out/r03r_tests.log; exit 1; }
tail -2 gpurun_out/r03r_tests.log
timeout -k 10 300 python -u -c "
import json, sys
sys.path[:0] = ['.', 'radiative-transfer_amd']
import bench, rtsn
pdir = bench.REPO / 'tests' / 'golden' / 'prm'
for name in bench.REFERENCE_CONFIGS:
    ph = rtsn.ParameterHandler(pdir / name, table_dir=str(pdir) + '/')
    q = ph.params
    g = bench.gpu_rate(q, q['ts_method'], 1000)
    print(json.dumps(dict(config=name, **g)))
" > gpurun_out/r03r_rates.jsonl 2>&1 || { tail -20 gpurun_out/r03r_rates.jsonl; exit 1; }
cat gpurun_out/r03r_rates.jsonl
