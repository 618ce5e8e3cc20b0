# Round 3: (1) the driver's window, interleaved: default vs four waves per segment with 16 /
# 32 workgroups per CU, on finite states (dt = 1e-7 for the default's short fill, dt = 1e-9
# for all); (2) rt_solve planned vs round-2 rule at dt = 1e-9.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r03k_window_ab.jsonl
for round in 0 1 2; do
  for cfg in "- - 1e-7" "- - 1e-9" "4 16 1e-9" "4 32 1e-9"; do
    set -- $cfg
    env_lw=""; env_w=""
    [ "$1" != "-" ] && env_lw="RTSN_LEVEL_WAVES=$1"
    [ "$2" != "-" ] && env_w="RTSN_WAVES_PER_CU=$2"
    env $env_lw $env_w timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --dt $3 --no-cpu-baseline --side-legs 0 --material-steps 0 > gpurun_out/r03k_b.log 2>&1 || { tail -20 gpurun_out/r03k_b.log; exit 1; }
    python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/r03k_b.log') if l.startswith('{')][-1]
print(json.dumps({'round': $round, 'level_waves': '$1', 'wgs_per_cu': '$2', 'dt': $3, 'ms_per_step': d['ms_per_step'], 'kernel': d['roofline']['kernel'], 'kernel_ms': d['roofline']['kernel_ms'], 'segments': d['config']['tiles_per_step'], 'warmup': d['warmup'], 'state_finite': d['state_finite']}))" >> gpurun_out/r03k_window_ab.jsonl
    tail -1 gpurun_out/r03k_window_ab.jsonl
  done
done
timeout -k 10 500 python -u tools/run_solve_plan.py 16,128 100,300,1000 1 > gpurun_out/r03k_solve_plan.jsonl 2> gpurun_out/r03k_solve_plan.err || { tail -20 gpurun_out/r03k_solve_plan.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r03k_solve_plan.jsonl'):
    d=json.loads(l); print(d['groups'], d['steps'], d['mode'], round(d['ms']), d['finite'], d['time_block'], d['level_waves'], d['segments'], round(d['plan']['estimated_ms']))"
