# Round 3: whole 1000-step runs of the 16-group shard (one rank of an 8-GPU run) and of all
# 128 groups over time block x waves per segment x segments per line.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/run_grid.py 16 1000 8,12,16,20 2,4 1,2,4 > gpurun_out/r03e_grid16.jsonl 2> gpurun_out/r03e_grid16.err || { tail -20 gpurun_out/r03e_grid16.err; exit 1; }
cat gpurun_out/r03e_grid16.jsonl
timeout -k 10 300 python -u tools/run_grid.py 128 1000 20,16 2,4 1,2,4 > gpurun_out/r03e_grid128.jsonl 2> gpurun_out/r03e_grid128.err || { tail -20 gpurun_out/r03e_grid128.err; exit 1; }
cat gpurun_out/r03e_grid128.jsonl
