# Round 3: wavefront chains with the lane-63 store issued after the next tick's shifts (so the
# shifts' wait for the ring read never waits on a fresh store): wavefront tests, then rates
# of the chain (blocks of 8 ticks; variant blocks of 16) against one wave per chain.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_wavefront_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03ae_tests.log 2>&1 || { tail -60 gpurun_out/r03ae_tests.log; exit 1; }
tail -2 gpurun_out/r03ae_tests.log
for rep in 0 1; do
  timeout -k 10 120 python -u scripts/wave_rates.py $rep | sed 's/^{/{"lib": "default", /' >> gpurun_out/r03ae_rates.jsonl || exit 1
  RTSN_WAVE_WAVES=1 timeout -k 10 120 python -u scripts/wave_rates.py $rep | sed 's/^{/{"lib": "default", /' >> gpurun_out/r03ae_rates.jsonl || exit 1
  RTSN_LIB=radiative-transfer_amd/variants/blk16/librtsn.so timeout -k 10 120 python -u scripts/wave_rates.py $rep | sed 's/^{/{"lib": "blk16", /' >> gpurun_out/r03ae_rates.jsonl || exit 1
done
grep '^{' gpurun_out/r03ae_rates.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['lib'].ljust(8), d['config'][:28].ljust(28), d['waves_max'], d.get('cells_per_lane'), d.get('waves_per_chain'), '%.1f us' % (1e3*d['ms']), '%.3g steps/s' % d['bdf2_steps_per_s'])"
