# Round 3: with issue priority for wave 0, an uneven level split of the T = 20 pass again
# (RT_SPLIT_BIAS 1: wave 0 runs 9 of the 20 levels, -1: 11) against the even split -- the
# driver's window, headline leg only, interleaved, 3 rounds.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
B="bench.py --steps 20 --warmup 5 --no-cpu-baseline --side-legs 0 --material-steps 0"
for rep in 0 1 2; do
  for v in default biasp1 biasm1; do
    if [ $v = default ]; then unset RTSN_LIB; else export RTSN_LIB=radiative-transfer_amd/variants/$v/librtsn.so; fi
    timeout -k 10 200 python -u $B > gpurun_out/r03as_$v.log 2>&1 || { tail -20 gpurun_out/r03as_$v.log; exit 1; }
    grep '^{' gpurun_out/r03as_$v.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print(json.dumps({'lib': '$v', 'rep': $rep, 'ms_per_step': d['ms_per_step'], 'kernel_ms': r['kernel_ms'], 'frac': r['frac'], 'finite': d['state_finite']}))" | tee -a gpurun_out/r03as_prio.jsonl
  done
done
# and graded issue priority for the four-wave T = 40 pass (variant graded: waves 0-3 at
# priority 3-0) against wave 0 alone -- the bench's default window (two T = 40 passes)
for rep in 0 1 2; do
  for v in default graded; do
    if [ $v = default ]; then unset RTSN_LIB; else export RTSN_LIB=radiative-transfer_amd/variants/$v/librtsn.so; fi
    timeout -k 10 200 python -u bench.py --steps 0 --no-cpu-baseline --side-legs 0 --material-steps 0 > gpurun_out/r03as_t40_$v.log 2>&1 || { tail -20 gpurun_out/r03as_t40_$v.log; exit 1; }
    grep '^{' gpurun_out/r03as_t40_$v.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print(json.dumps({'lib': '$v', 'rep': $rep, 'T': d['config']['steps_per_pass'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': r['kernel_ms'], 'frac': r['frac'], 'finite': d['state_finite']}))" | tee -a gpurun_out/r03as_graded.jsonl
  done
done
