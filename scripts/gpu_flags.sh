# Flag hand-over in the level-split kernel: bitwise tests, then the driver's window A/B
# against the barrier build (variants/barrier/librtsn.so), alternating.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "level_split or level_waves or headline or large_time or pipeline_long" > gpurun_out/flags_tests.log 2>&1 || { tail -40 gpurun_out/flags_tests.log; exit 1; }
tail -2 gpurun_out/flags_tests.log
: > gpurun_out/flags.jsonl
B="python bench.py --no-cpu-baseline --side-legs 0 --material-steps 0"
for rep in 1 2; do
  for lib in flags barrier; do
    if [ $lib = barrier ]; then L=radiative-transfer_amd/variants/barrier/librtsn.so; else L=radiative-transfer_amd/lib/librtsn.so; fi
    for args in "--steps 20 --warmup 5" "--steps 80"; do
      RTSN_LIB=$L timeout -k 10 300 $B $args > gpurun_out/flags.log 2>&1 || { tail -20 gpurun_out/flags.log; exit 1; }
      echo "{\"lib\": \"$lib\", \"args\": \"$args\", \"line\": $(tail -1 gpurun_out/flags.log)}" >> gpurun_out/flags.jsonl
    done
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/flags.jsonl"):
    d = json.loads(l); L = d["line"]; r = L["roofline"]
    print(d["lib"], d["args"], f'{L["ms_per_step"]:.3f} ms/step', r["kernel"], f'{r["kernel_ms"]:.1f}', f'frac {r["frac"]:.3f}', f'e2e {L["schedule"]["end_to_end_updates_per_s"]/L["value"]:.3f}')
PY
