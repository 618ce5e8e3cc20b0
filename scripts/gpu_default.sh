# The bench's default window (two T = 40 passes) in full, and a kernel trace of it.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r02i}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_def -o run --output-format csv -- python3 bench.py --no-cpu-baseline --side-legs 0 --material-steps 0 > gpurun_out/prof_def.log 2>&1 || { tail -20 gpurun_out/prof_def.log; exit 1; }
cp gpurun_out/prof_def/run_kernel_stats.csv gpurun_out/${TAG}_default_kernel_stats.csv
python3 scripts/trace_summary.py gpurun_out/prof_def/run_kernel_trace.csv gpurun_out/${TAG}_default_trace_summary.json
timeout -k 10 900 python bench.py > gpurun_out/${TAG}_default.log 2>&1 || { tail -20 gpurun_out/${TAG}_default.log; exit 1; }
tail -1 gpurun_out/${TAG}_default.log > gpurun_out/${TAG}_bench_default.json
python3 - <<PY
import json
d = json.load(open("gpurun_out/${TAG}_bench_default.json")); r = d["roofline"]
print(d["value"], d["ms_per_step"], d["steps"], r["kernel"], r["kernel_ms"], r["frac"], r["traffic"])
print("e2e", d["schedule"]["end_to_end_updates_per_s"] / d["value"], "hbm t1", d["hbm_pass_t1"]["hbm"]["frac"])
print("cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["sample"])
PY
