# level-split pass: parity (new test + pipelined T >= 8 cases) then timing of
# the one-wave pass (RTSN_LEVEL_WAVES=1) vs the level-split pass; VARIANTS=c16 adds a
# build variant (make -C radiative-transfer_amd variant V=c16 RT_DEFS=-DRT_CHUNK_SPLIT=16)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "level_split or large_time_blocks or full_length or pipeline_long" > gpurun_out/split_tests.log 2>&1 \
  || { tail -30 gpurun_out/split_tests.log; exit 1; }
tail -2 gpurun_out/split_tests.log
for v in lw1 lw2 $VARIANTS; do
  lib=radiative-transfer_amd/lib/librtsn.so; lw=2
  [ "$v" = lw1 ] && lw=1
  [ -d radiative-transfer_amd/variants/$v ] && lib=radiative-transfer_amd/variants/$v/librtsn.so
  RTSN_LEVEL_WAVES=$lw RTSN_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --material-steps 0 \
    > gpurun_out/split_$v.log 2>&1 || { tail -5 gpurun_out/split_$v.log; exit 1; }
  echo "$v $(python3 -c "
import json;d=[json.loads(x) for x in open('gpurun_out/split_$v.log') if x.startswith('{')][-1]
print(round(d['ms_per_step'],3),'ms/step', round(d['roofline']['kernel_ms'],2),'ms/pass', round(d['roofline']['frac'],3), d['roofline']['kernel'], d['config'].get('sweep_workgroups'))")"
done
