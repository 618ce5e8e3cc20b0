# T = 64 / 80 (eight waves per segment) against T = 40, same box, alternating.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/bigT2.jsonl
B="python bench.py --no-cpu-baseline --side-legs 0 --material-steps 0"
for rep in 1 2; do
  for args in "--steps 80 --time-block 40" "--steps 128 --time-block 64" "--steps 160 --time-block 80"; do
    timeout -k 10 300 $B $args > gpurun_out/bigT2.log 2>&1 || { tail -20 gpurun_out/bigT2.log; exit 1; }
    echo "{\"args\": \"$args\", \"line\": $(tail -1 gpurun_out/bigT2.log)}" >> gpurun_out/bigT2.jsonl
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/bigT2.jsonl"):
    d = json.loads(l); L = d["line"]; r = L["roofline"]
    print(d["args"], L["config"]["tiles_per_step"], f'{L["ms_per_step"]:.3f} ms/step', r["kernel"], f'{r["kernel_ms"]:.1f}', f'frac {r["frac"]:.3f}', f'e2e {L["schedule"]["end_to_end_updates_per_s"]/L["value"]:.3f}')
PY
