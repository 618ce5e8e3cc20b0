# Round 3 final: smoke() and the wavefront + split-pass tests at HEAD (after dropping the
# experiment-only knobs).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03at_smoke.log 2>&1 || { tail -20 gpurun_out/r03at_smoke.log; exit 1; }
tail -2 gpurun_out/r03at_smoke.log
timeout -k 10 600 python -u -m pytest tests/test_wavefront_gpu.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "wavefront or level_split or headline or reference_configs" > gpurun_out/r03at_tests.log 2>&1 || { tail -60 gpurun_out/r03at_tests.log; exit 1; }
tail -1 gpurun_out/r03at_tests.log
