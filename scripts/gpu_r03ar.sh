# Round 3 full check at HEAD (issue priority for wave 0 of the level-split pass): the driver's bench command, its
# rocprofv3 kernel trace (+ stats) and the PMC passes of the headline pass (all tests: r03an;
# split-pass tests: r03aq).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03ar_bench.log 2>&1 || { tail -30 gpurun_out/r03ar_bench.log; exit 1; }
grep "^{" gpurun_out/r03ar_bench.log | tail -1 > gpurun_out/r03ar_bench.json
python3 -c "
import json; d=json.load(open('gpurun_out/r03ar_bench.json')); r=d['roofline']
print('value', d['value'], 'ms/step', d['ms_per_step'], 'kern', r['kernel_ms'], 'frac', r['frac'], 'finite', d['state_finite'])
print('gather', d['gather']); print('llnl', d['llnl_slab_test'])"
B="bench.py --steps 20 --warmup 5 --no-cpu-baseline --side-legs 0 --material-steps 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r03ar_kt -o run --output-format csv -- python3 $B > gpurun_out/r03ar_kt.log 2>&1 || { tail -20 gpurun_out/r03ar_kt.log; exit 1; }
python3 scripts/trace_summary.py gpurun_out/r03ar_kt/run_kernel_trace.csv gpurun_out/r03ar_trace_summary.json
cp gpurun_out/r03ar_kt/run_kernel_stats.csv gpurun_out/r03ar_kernel_stats.csv
rm -f gpurun_out/r03ar_kt/run_kernel_trace.csv
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pmc -d gpurun_out/r03ar_pmc_$i -o run --output-format csv -- python3 $B > gpurun_out/r03ar_pmc_$i.log 2>&1 || { tail -5 gpurun_out/r03ar_pmc_$i.log; exit 1; }
done
python3 scripts/pmc_summary.py r03ar_v0_t20 gpurun_out/r03ar_pmc_1 gpurun_out/r03ar_pmc_2 gpurun_out/r03ar_pmc_3 gpurun_out/r03ar_pmc_4
cp profiles/pmc_r03ar_v0_t20.json gpurun_out/ 2>/dev/null || true
