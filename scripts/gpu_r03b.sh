# Round 3: the rest of the -m gpu suite after r03a stopped (T = 40 multi-line-group cases,
# C client, material, wavefront), then the interleaved overflow / finite A/B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "multi_line_group and 40-" > gpurun_out/r03b_tests1.log 2>&1 || { tail -60 gpurun_out/r03b_tests1.log; exit 1; }
tail -2 gpurun_out/r03b_tests1.log
timeout -k 10 600 python -u -m pytest tests/test_host.py tests/test_material_gpu.py tests/test_wavefront_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r03b_tests2.log 2>&1 || { tail -60 gpurun_out/r03b_tests2.log; exit 1; }
tail -2 gpurun_out/r03b_tests2.log
timeout -k 10 240 python -u tools/ab_finite.py 20 3 > gpurun_out/r03b_ab_finite.jsonl 2> gpurun_out/r03b_ab_finite.err || { tail -20 gpurun_out/r03b_ab_finite.err; exit 1; }
cat gpurun_out/r03b_ab_finite.jsonl
