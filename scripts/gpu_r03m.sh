# Round 3: rt_solve with the planned schedule vs the round-2 rule (finite states), 16-group
# shard and all 128 groups, 100 / 300 / 1000 steps, two rounds.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u tools/run_solve_plan.py 16,128 100,300,1000 2 > gpurun_out/r03m_solve_plan.jsonl 2> gpurun_out/r03m_solve_plan.err || { tail -20 gpurun_out/r03m_solve_plan.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r03m_solve_plan.jsonl'):
    d=json.loads(l); print(d['groups'], d['steps'], d['round'], d['mode'], round(d['ms']), d['finite'], d['time_block'], d['level_waves'], d['segments'], round(d['plan']['estimated_ms']))"
