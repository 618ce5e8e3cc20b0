# Round 3: interleaved same-box A/B of the driver's window (T = 20, K = 20, finite state):
# waves per segment (RTSN_LEVEL_WAVES) x target workgroups per CU for the segmentation
# (RTSN_WAVES_PER_CU; unset = the kernel's occupancy), three rounds.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r03h_window_ab.jsonl
for round in 0 1 2; do
  for cfg in "- -" "4 16" "4 32" "2 16"; do
    set -- $cfg
    env_lw=""; env_w=""
    [ "$1" != "-" ] && env_lw="RTSN_LEVEL_WAVES=$1"
    [ "$2" != "-" ] && env_w="RTSN_WAVES_PER_CU=$2"
    env $env_lw $env_w timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --side-legs 0 --material-steps 0 > gpurun_out/r03h_b.log 2>&1 || { tail -20 gpurun_out/r03h_b.log; exit 1; }
    python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/r03h_b.log') if l.startswith('{')][-1]
print(json.dumps({'round': $round, 'level_waves': '$1', 'wgs_per_cu': '$2', 'ms_per_step': d['ms_per_step'], 'kernel': d['roofline']['kernel'], 'kernel_ms': d['roofline']['kernel_ms'], 'segments': d['config']['tiles_per_step'], 'state_finite': d['state_finite']}))" >> gpurun_out/r03h_window_ab.jsonl
    tail -1 gpurun_out/r03h_window_ab.jsonl
  done
done
