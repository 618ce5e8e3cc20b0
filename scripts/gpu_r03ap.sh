# Round 3: static issue priority in the T = 20 level-split pass (variants: s_setprio 1 for
# wave 0, which streams the rows in, or for wave 1, which stores them) against none --
# the driver's window (20 steps), headline leg only, interleaved, 3 rounds.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
B="bench.py --steps 20 --warmup 5 --no-cpu-baseline --side-legs 0 --material-steps 0"
for rep in 0 1 2; do
  for v in default prio1 prio2; do
    if [ $v = default ]; then unset RTSN_LIB; else export RTSN_LIB=radiative-transfer_amd/variants/$v/librtsn.so; fi
    timeout -k 10 200 python -u $B > gpurun_out/r03ap_$v.log 2>&1 || { tail -20 gpurun_out/r03ap_$v.log; exit 1; }
    grep '^{' gpurun_out/r03ap_$v.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print(json.dumps({'lib': '$v', 'rep': $rep, 'ms_per_step': d['ms_per_step'], 'kernel_ms': r['kernel_ms'], 'frac': r['frac'], 'finite': d['state_finite']}))" | tee -a gpurun_out/r03ap_prio.jsonl
  done
done
