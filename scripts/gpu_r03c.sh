# Round 3: the wavefront tests, then the interleaved overflow / finite A/B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_wavefront_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r03c_tests.log 2>&1 || { tail -60 gpurun_out/r03c_tests.log; exit 1; }
tail -2 gpurun_out/r03c_tests.log
timeout -k 10 240 python -u tools/ab_finite.py 20 3 > gpurun_out/r03c_ab_finite.jsonl 2> gpurun_out/r03c_ab_finite.err || { tail -20 gpurun_out/r03c_ab_finite.err; exit 1; }
cat gpurun_out/r03c_ab_finite.jsonl
