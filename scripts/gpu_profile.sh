# Round profile of one bench window: rocprofv3 kernel trace, four PMC passes (HBM bytes,
# SQ counters, clock), the PMC summary and a bench line.  Run from the repo root on the
# GPU box; everything lands in gpurun_out/.  BENCHARGS: the window (default the driver's).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
V=${VARIANT:-v0}
TAG=${TAG:-r02}
WIN=${BENCHARGS:---steps 20 --warmup 5}
B="bench.py --no-cpu-baseline --side-legs 0 --material-steps 0 --variant $V $WIN"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt_$V -o run --output-format csv -- python3 $B > gpurun_out/prof_kt_$V.log 2>&1 || { tail -20 gpurun_out/prof_kt_$V.log; exit 1; }
T=$(python3 -c "import json;print([json.loads(l) for l in open('gpurun_out/prof_kt_$V.log') if l.startswith('{\"metric')][-1]['config']['steps_per_pass'])")
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pmc -d gpurun_out/pmc_${V}_$i -o run --output-format csv -- python3 $B > gpurun_out/pmc_${V}_$i.log 2>&1 || { tail -5 gpurun_out/pmc_${V}_$i.log; exit 1; }
done
python3 scripts/pmc_summary.py ${V}_t$T gpurun_out/pmc_${V}_1 gpurun_out/pmc_${V}_2 gpurun_out/pmc_${V}_3 gpurun_out/pmc_${V}_4
cp profiles/pmc_${V}_t$T.json gpurun_out/
cp gpurun_out/prof_kt_$V/run_kernel_stats.csv gpurun_out/${TAG}_${V}_t${T}_kernel_stats.csv
python3 scripts/trace_summary.py gpurun_out/prof_kt_$V/run_kernel_trace.csv gpurun_out/${TAG}_${V}_t${T}_trace_summary.json
timeout -k 10 600 python bench.py --variant $V $WIN > gpurun_out/bench_$V.log 2>&1 || { tail -20 gpurun_out/bench_$V.log; exit 1; }
grep "^{" gpurun_out/bench_$V.log | tail -1 > gpurun_out/${TAG}_bench_${V}_t${T}.json
python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_bench_${V}_t${T}.json')); r=d['roofline']
print(d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r['traffic'])"
cat gpurun_out/${TAG}_${V}_t${T}_trace_summary.json | head -30
