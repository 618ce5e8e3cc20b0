# bench + rocprofv3 kernel trace (run from the repo root on the GPU box)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2>&1 || { tail -20 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 4 > gpurun_out/prof_kt.log 2>&1 || { tail -20 gpurun_out/prof_kt.log; exit 1; }
find gpurun_out/prof_kt -name "*stats*" | head
