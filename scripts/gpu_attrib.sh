# time attribution of the sweep kernel (debug flags make results wrong; timing only)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for f in 0 1 2 3; do
  RTSN_DEBUG_FLAGS=$f timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/attrib_$f.log 2>&1 || { tail -5 gpurun_out/attrib_$f.log; exit 1; }
  echo "flags=$f $(python3 -c "import json;d=json.loads(open('gpurun_out/attrib_$f.log').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],2),'ms', d['config']['sweep_workgroups'],'wg')")"
done
