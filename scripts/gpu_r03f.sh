# Round 3: whole runs (300 and 1000 steps) over time block x segments per line, four waves
# per segment, for the 16-group shard and all 128 groups.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/run_grid.py 16 300,1000 8,16,20,24,32,40 4 2,4,8 > gpurun_out/r03f_grid16.jsonl 2> gpurun_out/r03f_grid16.err || { tail -20 gpurun_out/r03f_grid16.err; exit 1; }
cat gpurun_out/r03f_grid16.jsonl
timeout -k 10 400 python -u tools/run_grid.py 128 300,1000 20,24,32,40 4 4,8 > gpurun_out/r03f_grid128.jsonl 2> gpurun_out/r03f_grid128.err || { tail -20 gpurun_out/r03f_grid128.err; exit 1; }
cat gpurun_out/r03f_grid128.jsonl
