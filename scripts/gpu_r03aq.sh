# Round 3: issue priority for wave 0 of the level-split pass as the default: the split-pass
# parity tests, then the driver's T = 20 window and the bench's default T = 40 window (four
# waves per segment) with and without it (variant noprio), interleaved, 2 rounds.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "level_split or headline or timed_kernels or large_time or full_size or time_block" > gpurun_out/r03aq_tests.log 2>&1 || { tail -60 gpurun_out/r03aq_tests.log; exit 1; }
tail -1 gpurun_out/r03aq_tests.log
for rep in 0 1; do
  for W in "--steps 20 --warmup 5" "--steps 0"; do
    for v in default noprio; do
      if [ $v = default ]; then unset RTSN_LIB; else export RTSN_LIB=radiative-transfer_amd/variants/$v/librtsn.so; fi
      timeout -k 10 200 python -u bench.py $W --no-cpu-baseline --side-legs 0 --material-steps 0 > gpurun_out/r03aq_$v.log 2>&1 || { tail -20 gpurun_out/r03aq_$v.log; exit 1; }
      grep '^{' gpurun_out/r03aq_$v.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print(json.dumps({'lib': '$v', 'rep': $rep, 'steps': d['steps'], 'T': d['config']['steps_per_pass'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': r['kernel_ms'], 'frac': r['frac'], 'finite': d['state_finite']}))" | tee -a gpurun_out/r03aq_prio.jsonl
    done
  done
done
