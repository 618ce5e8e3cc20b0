# Round 3: the headline at dt = 1e-9 (finite at every GPU count): the driver's command at
# N = 1, then the two-rank rehearsal (both ranks on cuda:0, gloo), whose 320-step fill
# overflowed the state at dt = 1e-7.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03v_bench.log 2>&1 || { tail -30 gpurun_out/r03v_bench.log; exit 1; }
grep "^{" gpurun_out/r03v_bench.log | tail -1 > gpurun_out/r03v_bench.json
python3 -c "
import json; d=json.load(open('gpurun_out/r03v_bench.json')); r=d['roofline']
print('N=1 value', d['value'], 'ms/step', d['ms_per_step'], 'kern', r['kernel_ms'], 'frac', r['frac'], 'finite', d['state_finite'], d['config']['workload'])
print({k:(d[k]['ms_per_step'], d[k]['state_finite']) for k in ['hbm_pass_t1','overflow_control','variant_corr']})"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 20 --warmup 5 --backend gloo --share-device > gpurun_out/r03v_rehearsal2.log 2>&1 || { tail -30 gpurun_out/r03v_rehearsal2.log; exit 1; }
grep '^{' gpurun_out/r03v_rehearsal2.log | tail -1 > gpurun_out/r03v_rehearsal2.json
python3 -c "
import json; d=json.load(open('gpurun_out/r03v_rehearsal2.json'))
print('N=2', d['value'], d['ms_per_step'], d['state_finite'], d['config']['parallelism'], d['schedule']['warmup_steps'])
print({k:(d[k]['ms_per_step'], d[k]['state_finite']) for k in ['hbm_pass_t1','overflow_control','variant_corr']})"
