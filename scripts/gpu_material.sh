# Material-coupling GPU tests, then a kernel trace of scripts/material_perf.py (BE and BDF2).
# Run from the repo root on the GPU box; output under gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
timeout -k 10 600 python -u -m pytest tests/test_material_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/material_tests.log 2>&1 || { tail -40 gpurun_out/material_tests.log; exit 1; }
tail -1 gpurun_out/material_tests.log
for ts in 1 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mat$ts -o run --output-format csv -- python3 scripts/material_perf.py --ts $ts > gpurun_out/mat$ts.log 2>&1 || { tail -20 gpurun_out/mat$ts.log; exit 1; }
  grep "^{" gpurun_out/mat$ts.log
  cp gpurun_out/prof_mat$ts/run_kernel_stats.csv gpurun_out/${TAG}_material_ts${ts}_kernel_stats.csv
  cut -d, -f1-4 gpurun_out/${TAG}_material_ts${ts}_kernel_stats.csv | head -8
done
