set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --cells 100000 --no-cpu-baseline > gpurun_out/bench_small.log 2>&1 || { tail -20 gpurun_out/bench_small.log; exit 1; }
tail -2 gpurun_out/bench_small.log
timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2>&1 || { tail -20 gpurun_out/bench_full.log; exit 1; }
tail -2 gpurun_out/bench_full.log
