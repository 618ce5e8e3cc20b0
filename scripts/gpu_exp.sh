# Time-block experiment (repo root, GPU box): bench lines for the given T list.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for t in ${TS:-8 12 16}; do
  RTSN_TIME_BLOCK=$t timeout -k 10 600 python bench.py --no-cpu-baseline --time-block $t > gpurun_out/bench_t$t.log 2>&1 || { tail -20 gpurun_out/bench_t$t.log; exit 1; }
  python3 -c "import json;l=[json.loads(x) for x in open('gpurun_out/bench_t$t.log') if x.startswith('{')][-1];sc=l['schedule'];print('T $t', l['config']['tiles_per_step'], 'seg', '%.4g'%l['value'], '%.2f ms/step'%l['ms_per_step'], '%.2f ms/launch'%l['roofline']['kernel_ms'], 'warmup', sc['warmup_steps'], 'drain %.0f ms'%sc['drain_ms'], 'e2e %.4g upd/s'%sc['end_to_end_updates_per_s'])"
done
