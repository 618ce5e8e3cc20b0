# Round 3: the level-split pass with the loader wave's refills one cell late, pinned after
# their cell's FMAs, and the prologue loads waited for before the chunk loop (RT_SPLIT_PIN_LOADS,
# default) vs without (variants/nopin): parity of the split passes, then an interleaved
# same-box A/B of the driver's window (T = 20) and of the T = 40 window.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "level_split or headline or timed_kernels or full_size or large_time or pipeline_long or reference_configs or time_block_switching" \
  > gpurun_out/r03x_tests.log 2>&1 || { tail -60 gpurun_out/r03x_tests.log; exit 1; }
tail -2 gpurun_out/r03x_tests.log
B="--no-cpu-baseline --side-legs 0 --material-steps 0"
for rep in 1 2 3; do
  for v in pin nopin; do
    lib=$PWD/radiative-transfer_amd/lib/librtsn.so
    [ $v = nopin ] && lib=$PWD/radiative-transfer_amd/variants/nopin/librtsn.so
    for K in 20 40; do
      RTSN_LIB=$lib timeout -k 10 300 python bench.py --steps $K --warmup 5 $B > gpurun_out/r03x_${v}_${K}_$rep.log 2>&1 || { tail -5 gpurun_out/r03x_${v}_${K}_$rep.log; exit 1; }
      python3 -c "
import json;d=[json.loads(x) for x in open('gpurun_out/r03x_${v}_${K}_$rep.log') if x.startswith('{')][-1]; r=d['roofline']
print(json.dumps(dict(variant='$v', K=$K, rep=$rep, ms_per_step=d['ms_per_step'], kernel_ms=r['kernel_ms'], frac=r['frac'], value=d['value'], finite=d['state_finite'], kernel=r['kernel'])))" | tee -a gpurun_out/r03x_ab.jsonl
    done
  done
done
