# Round 3: every -m gpu test (the new multi-line-group, full-size T = 16/20/40, wavefront,
# C-client and rank-failure tests among them), then the interleaved overflow / finite A/B
# of the headline pass.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "$@" \
  > gpurun_out/r03a_tests.log 2>&1 || { tail -80 gpurun_out/r03a_tests.log; exit 1; }
tail -5 gpurun_out/r03a_tests.log
timeout -k 10 240 python -u tools/ab_finite.py 20 3 > gpurun_out/r03a_ab_finite.jsonl 2> gpurun_out/r03a_ab_finite.err || { tail -20 gpurun_out/r03a_ab_finite.err; exit 1; }
cat gpurun_out/r03a_ab_finite.jsonl
