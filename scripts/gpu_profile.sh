# Round profile: bench (default + corr variant), rocprofv3 kernel trace, PMC passes.
# Run from the repo root on the GPU box; results land in gpurun_out/ and profiles/.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out profiles
V=${VARIANT:-v0}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt_$V -o run --output-format csv -- python3 bench.py --no-cpu-baseline --variant $V > gpurun_out/prof_kt_$V.log 2>&1 || { tail -20 gpurun_out/prof_kt_$V.log; exit 1; }
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pmc -d gpurun_out/pmc_${V}_$i -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 0 --variant $V > gpurun_out/pmc_${V}_$i.log 2>&1 || { tail -5 gpurun_out/pmc_${V}_$i.log; exit 1; }
done
python3 scripts/pmc_summary.py $V gpurun_out/pmc_${V}_1 gpurun_out/pmc_${V}_2 gpurun_out/pmc_${V}_3 gpurun_out/pmc_${V}_4
cp gpurun_out/prof_kt_$V/run_kernel_stats.csv gpurun_out/r01_${V}_kernel_stats.csv
timeout -k 10 600 python bench.py --variant $V > gpurun_out/bench_$V.log 2>&1 || { tail -20 gpurun_out/bench_$V.log; exit 1; }
tail -1 gpurun_out/bench_$V.log | tee gpurun_out/r01_bench_$V.json
