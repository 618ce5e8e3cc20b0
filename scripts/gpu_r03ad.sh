# Round 3: where do the waves of a small workgroup run (tools/simd_placement), and the
# wavefront chain's rates with the register file claimed (one wave per SIMD: variant
# RT_WAVE_SPREAD=1, chains of <= 4 waves) against the default and one wave per chain.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 ./tools/simd_placement > gpurun_out/r03ad_placement.txt 2>&1 || { tail -20 gpurun_out/r03ad_placement.txt; exit 1; }
cat gpurun_out/r03ad_placement.txt
for rep in 0 1; do
  timeout -k 10 120 python -u scripts/wave_rates.py $rep | sed 's/^{/{"lib": "default", /' >> gpurun_out/r03ad_rates.jsonl || exit 1
  RTSN_WAVE_WAVES=1 timeout -k 10 120 python -u scripts/wave_rates.py $rep | sed 's/^{/{"lib": "default", /' >> gpurun_out/r03ad_rates.jsonl || exit 1
  RTSN_LIB=radiative-transfer_amd/variants/spread/librtsn.so RTSN_WAVE_WAVES=4 timeout -k 10 120 python -u scripts/wave_rates.py $rep | sed 's/^{/{"lib": "spread", /' >> gpurun_out/r03ad_rates.jsonl || exit 1
done
grep '^{' gpurun_out/r03ad_rates.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['lib'].ljust(8), d['config'][:28].ljust(28), d['waves_max'], d.get('cells_per_lane'), d.get('waves_per_chain'), '%.1f us' % (1e3*d['ms']), '%.3g steps/s' % d['bdf2_steps_per_s'])"
