# Round 3: how many BDF2 steps the SL state stays finite per dt.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/finite_horizon.py 128 1e-7,3e-8,1e-8,3e-9,1e-9 200 4000 > gpurun_out/r03j_finite_horizon.jsonl 2> gpurun_out/r03j_finite_horizon.err || { tail -20 gpurun_out/r03j_finite_horizon.err; exit 1; }
cat gpurun_out/r03j_finite_horizon.jsonl
