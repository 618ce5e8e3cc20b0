# Round 3: more segments per line for whole runs (16-group shard and all 128 groups), and
# the driver's bench window with four waves per segment and 8 / 16 target workgroups per CU.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/run_grid.py 16 300,1000 16,20,32,40 4 8,16,32 > gpurun_out/r03g_grid16.jsonl 2> gpurun_out/r03g_grid16.err || { tail -20 gpurun_out/r03g_grid16.err; exit 1; }
cat gpurun_out/r03g_grid16.jsonl
timeout -k 10 300 python -u tools/run_grid.py 128 300,1000 20,32,40 4 16,32 > gpurun_out/r03g_grid128.jsonl 2> gpurun_out/r03g_grid128.err || { tail -20 gpurun_out/r03g_grid128.err; exit 1; }
cat gpurun_out/r03g_grid128.jsonl
for cfg in "0 0" "4 4" "4 8" "4 16" "2 8"; do
  set -- $cfg
  RTSN_LEVEL_WAVES=$1 RTSN_WAVES_PER_CU=$2 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --side-legs 0 --material-steps 0 > gpurun_out/r03g_bench_$1_$2.log 2>&1 || { tail -20 gpurun_out/r03g_bench_$1_$2.log; exit 1; }
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/r03g_bench_$1_$2.log') if l.startswith('{')][-1]
print('lw=$1 w=$2', round(d['ms_per_step'],3), d['roofline']['kernel'], round(d['roofline']['kernel_ms'],2), d['config']['tiles_per_step'], d['schedule']['end_to_end_ms'])"
done
