# T = 20 (the driver's window) with two vs four waves per segment, alternating, same box.
# EXTRA: more bench.py arguments (e.g. --groups 16, the 8-GPU strong-scaling shard).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/lw20.jsonl
for rep in 1 2; do
  for lw in 2 4; do
    RTSN_LEVEL_WAVES=$lw timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --side-legs 0 --material-steps 0 $EXTRA > gpurun_out/lw20_$lw.log 2>&1 || { tail -20 gpurun_out/lw20_$lw.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/lw20_$lw.log').read().strip().splitlines()[-1]); print(json.dumps({'level_waves': $lw, 'rep': $rep, 'ms_per_step': d['ms_per_step'], 'frac': d['roofline']['frac'], 'kernel': d['roofline']['kernel'], 'e2e': d['schedule']['end_to_end_updates_per_s']/d['value']}))" | tee -a gpurun_out/lw20.jsonl
  done
done
