# Round 3: the planned rt_solve schedule vs the round-2 rule, whole runs, 16-group shard and
# all 128 groups; then the window A/B (waves per segment x segmentation).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/run_solve_plan.py 16,128 100,300,1000 2 > gpurun_out/r03i_solve_plan.jsonl 2> gpurun_out/r03i_solve_plan.err || { tail -20 gpurun_out/r03i_solve_plan.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r03i_solve_plan.jsonl'):
    d=json.loads(l); print(d['groups'], d['steps'], d['round'], d['mode'], round(d['ms']), d['time_block'], d['level_waves'], d['segments'], round(d['plan']['estimated_ms']))"
bash scripts/gpu_r03h.sh
