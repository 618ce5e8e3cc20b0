# Segments-per-line experiment for the pipelined schedule (repo root, GPU box).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in 8 4 2; do
  RTSN_WAVES_PER_CU=$w timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_w$w.log 2>&1 || { tail -20 gpurun_out/bench_w$w.log; exit 1; }
  python3 -c "import json;l=[json.loads(x) for x in open('gpurun_out/bench_w$w.log') if x.startswith('{')][-1];sc=l['schedule'];print('waves/CU $w', l['config']['tiles_per_step'], 'seg', '%.4g'%l['value'], '%.2f ms/step'%l['ms_per_step'], '%.2f ms/launch'%l['roofline']['kernel_ms'], 'warmup', sc['warmup_steps'], 'drain %.0f ms'%sc['drain_ms'], 'e2e %.4g upd/s'%sc['end_to_end_updates_per_s'], l['state_finite'])"
done
