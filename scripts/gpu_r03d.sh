# Round 3: the driver's bench command (finite-state headline, gather breakdown, llnl_slab_test
# key), its rocprofv3 kernel trace, and the kernel trace of a whole 1000-step run of the
# 16-group shard (one rank of an 8-GPU strong-scaling run) for the fill / drain analysis.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03d_bench.log 2>&1 || { tail -30 gpurun_out/r03d_bench.log; exit 1; }
grep "^{" gpurun_out/r03d_bench.log | tail -1 > gpurun_out/r03d_bench.json
python3 -c "
import json; d=json.load(open('gpurun_out/r03d_bench.json')); r=d['roofline']
print('value', d['value'], 'ms/step', d['ms_per_step'], 'kern', r['kernel_ms'], 'frac', r['frac'], 'finite', d['state_finite'])
print('gather', d['gather'])
print('llnl', d['llnl_slab_test'])
print('overflow', d['overflow_control']['ms_per_step'], 'hbm', d['hbm_pass_t1']['hbm'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r03d_kt -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --side-legs 0 --material-steps 0 > gpurun_out/r03d_kt.log 2>&1 || { tail -20 gpurun_out/r03d_kt.log; exit 1; }
python3 scripts/trace_summary.py gpurun_out/r03d_kt/run_kernel_trace.csv gpurun_out/r03d_trace_summary.json
cp gpurun_out/r03d_kt/run_kernel_stats.csv gpurun_out/r03d_kernel_stats.csv
grep "^{" gpurun_out/r03d_kt.log | tail -1 > gpurun_out/r03d_kt_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r03d_run16 -o run --output-format csv -- python3 tools/run_once.py 16 1000 20 > gpurun_out/r03d_run16.log 2>&1 || { tail -20 gpurun_out/r03d_run16.log; exit 1; }
python3 scripts/launch_sequence.py gpurun_out/r03d_run16/run_kernel_trace.csv gpurun_out/r03d_run16_launches.jsonl
rm -rf gpurun_out/r03d_run16 gpurun_out/r03d_kt/run_kernel_trace.csv
tail -2 gpurun_out/r03d_run16.log
