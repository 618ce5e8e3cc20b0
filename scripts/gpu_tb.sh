# Parity tests, then a bench line per time block and schedule (run from the repo root on the GPU box).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
IFS=, read -ra LIST <<< "${CFGS:-pipelined 4,pipelined 8,pipelined 16,aligned 4}"
for cfg in "${LIST[@]}"; do
  set -- $cfg
  timeout -k 10 600 python bench.py --no-cpu-baseline --schedule $1 --time-block $2 > gpurun_out/bench_$1_$2.log 2>&1 || { tail -20 gpurun_out/bench_$1_$2.log; exit 1; }
  python3 -c "import json;l=[json.loads(x) for x in open('gpurun_out/bench_$1_$2.log') if x.startswith('{')][-1];sc=l['schedule'];print('$1', $2, '%.4g'%l['value'], '%.2f ms/step'%l['ms_per_step'], '%.2f ms/launch'%l['roofline']['kernel_ms'], 'warmup', sc['warmup_steps'], 'drain %.0f ms'%sc['drain_ms'], 'e2e %.4g upd/s'%sc['end_to_end_updates_per_s'], l['state_finite'])"
done
