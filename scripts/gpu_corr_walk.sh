# Correction walks without the zero columns: parity tests (all schedules, material), then
# kernel traces of the BDF2 coupled step (walk) and the aligned T = 4 pass.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_material_gpu.py -m gpu > gpurun_out/walk_tests.log 2>&1 || { tail -30 gpurun_out/walk_tests.log; exit 1; }
tail -2 gpurun_out/walk_tests.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_walk -o run --output-format csv -- python3 tools/material_steps.py 3 3 > gpurun_out/prof_walk.log 2>&1 || { tail -20 gpurun_out/prof_walk.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_al -o run --output-format csv -- python3 bench.py --steps 8 --warmup 4 --schedule aligned --no-cpu-baseline --side-legs 0 --material-steps 0 > gpurun_out/prof_al.log 2>&1 || { tail -20 gpurun_out/prof_al.log; exit 1; }
grep -h "phi_correction\|sweep_block_kernel<3, 1, 0, true>\|sweep_block_kernel<3, 4, 0" gpurun_out/prof_walk/run_kernel_stats.csv gpurun_out/prof_al/run_kernel_stats.csv | cut -d, -f1-4
grep '^{' gpurun_out/prof_al.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('aligned', d['ms_per_step'], d['roofline']['kernel'], d['roofline']['kernel_ms'])"
