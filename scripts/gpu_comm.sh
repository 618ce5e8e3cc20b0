set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_comm_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/comm_tests.log 2>&1 || { tail -60 gpurun_out/comm_tests.log; exit 1; }
tail -12 gpurun_out/comm_tests.log
NCCL_DEBUG=WARN timeout -k 10 120 python tools/debug/rccl_two_ranks.py > gpurun_out/rccl_two.log 2>&1; echo "two-rank probe rc=$?"; tail -20 gpurun_out/rccl_two.log
