# time build variants of librtsn.so (timing experiments; see radiative-transfer_amd/Makefile `variant`):
# the headline pass and the T = 1 (HBM-bound) side leg of bench.py per variant
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in base $VARIANTS; do
  if [ "$v" = base ]; then lib=radiative-transfer_amd/lib/librtsn.so; else lib=radiative-transfer_amd/variants/$v/librtsn.so; fi
  RTSN_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --material-steps 0 $BENCH_ARGS > gpurun_out/var_$v.log 2>&1 || { tail -5 gpurun_out/var_$v.log; exit 1; }
  echo "$v $(python3 -c "
import json;d=[json.loads(x) for x in open('gpurun_out/var_$v.log') if x.startswith('{')][-1]
t=d.get('hbm_pass_t1', {})
print(round(d['ms_per_step'],3),'ms/step', round(d['roofline']['kernel_ms'],2),'ms/pass', round(d['roofline']['frac'],3), '| T=1', round(t.get('kernel_ms',0),2),'ms', round(t.get('hbm',{}).get('frac',0),3))")"
done
