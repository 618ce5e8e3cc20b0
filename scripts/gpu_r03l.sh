# Round 3: whole-run grids on finite states (dt = 1e-9, a fresh handle per configuration).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/run_grid.py 16 300,1000 8,16,20,24,32,40 4 8,16,32 > gpurun_out/r03l_grid16.jsonl 2> gpurun_out/r03l_grid16.err || { tail -20 gpurun_out/r03l_grid16.err; exit 1; }
cat gpurun_out/r03l_grid16.jsonl
timeout -k 10 500 python -u tools/run_grid.py 128 300,1000 20,24,32,40 4 4,8,16,32 > gpurun_out/r03l_grid128.jsonl 2> gpurun_out/r03l_grid128.err || { tail -20 gpurun_out/r03l_grid128.err; exit 1; }
cat gpurun_out/r03l_grid128.jsonl
