# Round 3: one wave per chain whenever the line fits (multi-wave chains only beyond it, auto
# only while the chains leave one wave per SIMD): the wavefront tests and the reference
# configurations' parity, then mid-length lines (300-4000 cells) as wavefront chains vs the
# segment pipeline, and the reference configurations' rates.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_wavefront_gpu.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "wavefront or reference_configs or llnl_full or gray" > gpurun_out/r03ai_tests.log 2>&1 || { tail -60 gpurun_out/r03ai_tests.log; exit 1; }
tail -2 gpurun_out/r03ai_tests.log
timeout -k 10 300 python -u tools/wave_mid_rates.py > gpurun_out/r03ai_mid.jsonl 2>&1 || { tail -20 gpurun_out/r03ai_mid.jsonl; exit 1; }
grep '^{' gpurun_out/r03ai_mid.jsonl
timeout -k 10 120 python -u scripts/wave_rates.py 0 > gpurun_out/r03ai_rates.jsonl 2>&1 || { tail -20 gpurun_out/r03ai_rates.jsonl; exit 1; }
grep '^{' gpurun_out/r03ai_rates.jsonl | cut -c1-200
