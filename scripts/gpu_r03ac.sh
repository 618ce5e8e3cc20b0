# Round 3: wavefront chains over up to 8 waves (LDS hand-over, one barrier per 8 ticks): the
# wavefront tests (one wave vs the chain vs the pipelined schedule, bitwise), the reference
# configurations' oracle parity, then their rates with the chain (default) and with one wave
# per chain (RTSN_WAVE_WAVES=1, the previous kernel's geometry), interleaved, 3 rounds.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_wavefront_gpu.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "wavefront or reference_configs or llnl_full or gray" > gpurun_out/r03ac_tests.log 2>&1 || { tail -60 gpurun_out/r03ac_tests.log; exit 1; }
tail -2 gpurun_out/r03ac_tests.log
cat > scripts/wave_rates.py <<'PY'
import json, os, sys
sys.path[:0] = ['.', 'radiative-transfer_amd']
import bench, rtsn
pdir = bench.REPO / 'tests' / 'golden' / 'prm'
for name in bench.REFERENCE_CONFIGS:
    ph = rtsn.ParameterHandler(pdir / name, table_dir=str(pdir) + '/')
    q = ph.params
    g = bench.gpu_rate(q, q['ts_method'], 1000)
    print(json.dumps(dict(config=name, rep=int(sys.argv[1]), waves_max=int(os.environ.get('RTSN_WAVE_WAVES', 8)), **g)), flush=True)
PY
for rep in 0 1 2; do
  timeout -k 10 120 python -u scripts/wave_rates.py $rep >> gpurun_out/r03ac_rates.jsonl 2>&1 || { tail -20 gpurun_out/r03ac_rates.jsonl; exit 1; }
  RTSN_WAVE_WAVES=1 timeout -k 10 120 python -u scripts/wave_rates.py $rep >> gpurun_out/r03ac_rates.jsonl 2>&1 || { tail -20 gpurun_out/r03ac_rates.jsonl; exit 1; }
done
grep '^{' gpurun_out/r03ac_rates.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['config'][:28].ljust(28), d['waves_max'], d.get('cells_per_lane'), d.get('waves_per_chain'), '%.1f us' % (1e3*d['ms']), '%.3g steps/s' % d['bdf2_steps_per_s'])"
