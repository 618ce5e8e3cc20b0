# bench + PMC counter passes for the sweep kernel (run from the repo root on the GPU box)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pmc -d gpurun_out/pmc$i -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 0 > gpurun_out/pmc$i.log 2>&1 || { tail -5 gpurun_out/pmc$i.log; exit 1; }
done
echo done
