# Round 3 full check at HEAD (after the wavefront chains and their plan): every -m gpu test,
# smoke(), then one wave (RTSN_WAVE_WAVES=1) vs the plan for 129-512-cell lines (and
# reflective 100-256), and the reference configurations' rates.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --durations=30 --timeout 300 --timeout-method thread > gpurun_out/r03an_tests.log 2>&1 || { tail -60 gpurun_out/r03an_tests.log; exit 1; }
tail -2 gpurun_out/r03an_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03an_smoke.log 2>&1 || { tail -20 gpurun_out/r03an_smoke.log; exit 1; }
tail -2 gpurun_out/r03an_smoke.log
for NB in "129 0" "200 0" "256 0" "300 0" "400 0" "512 0" "100 2" "129 2" "200 2" "256 2"; do
  for v in 8 1; do
    RTSN_WAVE_WAVES=$v timeout -k 10 60 python -u tools/wave_ablation.py $NB | sed "s/^{/{\"max_waves\": $v, /" >> gpurun_out/r03an_plan.jsonl || exit 1
  done
done
grep '^{' gpurun_out/r03an_plan.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['N'], d['bc_left'], d['max_waves'], d['cells_per_lane'], d['waves'], '%.1f us' % d['us'])"
timeout -k 10 120 python -u scripts/wave_rates.py 0 > gpurun_out/r03an_rates.jsonl 2>&1 || { tail -20 gpurun_out/r03an_rates.jsonl; exit 1; }
grep '^{' gpurun_out/r03an_rates.jsonl | cut -c1-150
