# Full GPU check (run from the repo root on the GPU box): every -m gpu test, smoke(), a
# kernel-trace profile of the driver's bench command and its bench line.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r02}
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_kt.log 2>&1 || { tail -20 gpurun_out/prof_kt.log; exit 1; }
cp gpurun_out/prof_kt/run_kernel_stats.csv gpurun_out/${TAG}_kernel_stats.csv
python3 scripts/trace_summary.py gpurun_out/prof_kt/run_kernel_trace.csv gpurun_out/${TAG}_trace_summary.json
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_full.log 2>&1 || { tail -20 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log > gpurun_out/${TAG}_bench.json
python3 - <<PY
import json
d = json.load(open("gpurun_out/${TAG}_bench.json"))
r = d["roofline"]
print(d["value"], d["ms_per_step"], r["kernel"], r["kernel_ms"], r["frac"], r["traffic"])
print("e2e ratio", d["schedule"]["end_to_end_updates_per_s"] / d["value"], "drain", d["schedule"]["drain_ms"])
c = d["cpu_baseline"]; print("cpu", c["value"], c["reference_shaped_value"], c["single_thread_value"], c["threads"])
print("material", d["material"]["ms_per_step"], d["material"]["allreduce"][:40])
PY
