# Round 3: whole rt_solve runs of lines beyond the wavefront (5000-50000 cells, few groups):
# rt_solve's plan vs fixed pipelined / aligned schedules.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/solve_mid.py > gpurun_out/r03ao_solve_mid.jsonl 2>&1 || { tail -20 gpurun_out/r03ao_solve_mid.jsonl; exit 1; }
grep '^{' gpurun_out/r03ao_solve_mid.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['N'], d['G'], d['schedule'].ljust(8), '%.1f ms' % d['ms'], d['plan'], d['finite'])"
