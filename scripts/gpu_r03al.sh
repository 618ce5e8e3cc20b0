# Round 3: the chain plan (one wave while 1-2 cells per lane fit, reflective 1-4; else <= 4
# waves; else <= 8): wavefront tests + reference configurations' parity, then one wave
# (RTSN_WAVE_WAVES=1) vs the plan for 129-512-cell lines (and reflective 100-256).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_wavefront_gpu.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "wavefront or reference_configs or llnl_full or gray" > gpurun_out/r03al_tests.log 2>&1 || { tail -60 gpurun_out/r03al_tests.log; exit 1; }
tail -2 gpurun_out/r03al_tests.log
for NB in "129 0" "200 0" "256 0" "300 0" "400 0" "512 0" "100 2" "129 2" "200 2" "256 2"; do
  for v in 8 1; do
    RTSN_WAVE_WAVES=$v timeout -k 10 60 python -u tools/wave_ablation.py $NB | sed "s/^{/{\"max_waves\": $v, /" >> gpurun_out/r03al_plan.jsonl || exit 1
  done
done
grep '^{' gpurun_out/r03al_plan.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['N'], d['bc_left'], d['max_waves'], d['cells_per_lane'], d['waves'], '%.1f us' % d['us'])"
timeout -k 10 120 python -u scripts/wave_rates.py 0 > gpurun_out/r03al_rates.jsonl 2>&1 || { tail -20 gpurun_out/r03al_rates.jsonl; exit 1; }
grep '^{' gpurun_out/r03al_rates.jsonl | cut -c1-150
