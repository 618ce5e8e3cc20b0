# GPU tests, then a kernel-trace profile of a lean bench run (headline sweep + gather).
# Run from the repo root on the GPU box; output under gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_q -o run --output-format csv -- python3 bench.py --no-cpu-baseline --side-legs 0 ${BENCH_ARGS} > gpurun_out/prof_q.log 2>&1 || { tail -20 gpurun_out/prof_q.log; exit 1; }
cp gpurun_out/prof_q/run_kernel_stats.csv gpurun_out/${TAG}_kernel_stats.csv
cut -c1-160 gpurun_out/${TAG}_kernel_stats.csv | head -14
