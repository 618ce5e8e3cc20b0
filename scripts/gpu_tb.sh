# Parity tests, then a bench line per time block (run from the repo root on the GPU box).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
for tb in 1 2 3 4; do
  timeout -k 10 600 python bench.py --no-cpu-baseline --time-block $tb --steps 12 --warmup 4 > gpurun_out/bench_tb$tb.log 2>&1 || { tail -20 gpurun_out/bench_tb$tb.log; exit 1; }
  python3 -c "import json;l=json.loads(open('gpurun_out/bench_tb$tb.log').read().strip().splitlines()[-1]);print($tb, '%.4g'%l['value'], '%.2f ms/step'%l['ms_per_step'], '%.2f ms/pass'%l['roofline']['kernel_ms'], '%.0f GB/s'%l['roofline']['achieved'], l['absorption_allreduce_finite'])"
done
