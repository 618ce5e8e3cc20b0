# Round 3: why a wavefront chain over 2 waves ticks slower than one wave with 2 cells per
# lane -- kernel durations and SQ counters of multi_group_equilibrium's 1000-step advance,
# chain (default) vs one wave per chain (RTSN_WAVE_WAVES=1).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 8 1; do
  RTSN_WAVE_WAVES=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r03ag_kt_$v -o run --output-format csv -- python3 tools/wave_profile.py > gpurun_out/r03ag_kt_$v.log 2>&1 || { tail -20 gpurun_out/r03ag_kt_$v.log; exit 1; }
  grep -i wavefront gpurun_out/r03ag_kt_$v/run_kernel_stats.csv | cut -c1-300
  RTSN_WAVE_WAVES=$v timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY -d gpurun_out/r03ag_pmc_$v -o run --output-format csv -- python3 tools/wave_profile.py > gpurun_out/r03ag_pmc_$v.log 2>&1 || { tail -20 gpurun_out/r03ag_pmc_$v.log; exit 1; }
  grep -i wavefront gpurun_out/r03ag_pmc_$v/run_counter_collection.csv | awk -F, '{print $(NF-1), $NF}' | tail -8
done
