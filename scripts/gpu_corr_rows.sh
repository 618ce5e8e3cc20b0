# BDF2 correction share by tabulated rows: material parity tests (rows vs walk vs oracle),
# then kernel traces of the BDF2 coupled step with the rows kernel and with the walk.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_material_gpu.py -m gpu > gpurun_out/rows_tests.log 2>&1 || { tail -30 gpurun_out/rows_tests.log; exit 1; }
tail -2 gpurun_out/rows_tests.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rows -o run --output-format csv -- python3 tools/material_steps.py 3 3 > gpurun_out/prof_rows.log 2>&1 || { tail -20 gpurun_out/prof_rows.log; exit 1; }
RTSN_PHI_WALK=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rwalk -o run --output-format csv -- python3 tools/material_steps.py 3 3 > gpurun_out/prof_rwalk.log 2>&1 || { tail -20 gpurun_out/prof_rwalk.log; exit 1; }
grep -h "phi_correction\|corr_rows" gpurun_out/prof_rows/run_kernel_stats.csv gpurun_out/prof_rwalk/run_kernel_stats.csv | cut -d, -f1-4
tail -2 gpurun_out/prof_rows.log gpurun_out/prof_rwalk.log
