# bench.py at several (K, W) windows (lean: no side legs, material or CPU baseline).
# Run from the repo root on the GPU box; one JSON line per window in gpurun_out/windows.jsonl.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/windows.jsonl
for kw in ${WINDOWS:-"2 1" "20 5" "10 2" "100 10" "50 0"}; do
  set -- $kw
  timeout -k 10 300 python bench.py --no-cpu-baseline --side-legs 0 --material-steps 0 --steps $1 --warmup $2 > gpurun_out/win_$1_$2.log 2>&1 || { tail -20 gpurun_out/win_$1_$2.log; exit 1; }
  grep "^{" gpurun_out/win_$1_$2.log | tail -1 >> gpurun_out/windows.jsonl
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/windows.jsonl').read().splitlines()[-1]); print(d['steps'], d['warmup'], d['schedule']['steps_per_pass'], round(d['ms_per_step'],3), '%.3g' % d['value'])"
done
