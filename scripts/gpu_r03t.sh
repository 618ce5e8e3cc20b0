# Round 3: the driver's window with four waves per segment at the default segment count
# (same fill as the two-wave default) and at twice it, interleaved with the default and the
# 16-workgroups-per-CU point of r03k; finite states.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r03t_window_ab.jsonl
for round in 0 1; do
  for cfg in "- - 1e-7" "4 4 1e-7" "4 6 1e-8" "4 8 1e-8" "4 16 1e-9"; do
    set -- $cfg
    env_lw=""; env_w=""
    [ "$1" != "-" ] && env_lw="RTSN_LEVEL_WAVES=$1"
    [ "$2" != "-" ] && env_w="RTSN_WAVES_PER_CU=$2"
    env $env_lw $env_w timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --dt $3 --no-cpu-baseline --side-legs 0 --material-steps 0 > gpurun_out/r03t_b.log 2>&1 || { tail -20 gpurun_out/r03t_b.log; exit 1; }
    python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/r03t_b.log') if l.startswith('{')][-1]
print(json.dumps({'round': $round, 'level_waves': '$1', 'wgs_per_cu': '$2', 'dt': $3, 'ms_per_step': d['ms_per_step'], 'kernel': d['roofline']['kernel'], 'kernel_ms': d['roofline']['kernel_ms'], 'segments': d['config']['tiles_per_step'], 'warmup': d['warmup'], 'state_finite': d['state_finite']}))" >> gpurun_out/r03t_window_ab.jsonl
    tail -1 gpurun_out/r03t_window_ab.jsonl
  done
done
