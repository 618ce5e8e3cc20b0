# T = 24 / 32 (four waves per segment) against T = 16 / 20, same box, alternating.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/bigT.jsonl
B="python bench.py --no-cpu-baseline --side-legs 0 --material-steps 0"
for rep in 1 2; do
  for args in "--steps 64 --time-block 16" "--steps 64 --time-block 32" "--steps 80 --time-block 40" "--steps 40 --time-block 20"; do
    timeout -k 10 300 $B $args > gpurun_out/bigT.log 2>&1 || { tail -20 gpurun_out/bigT.log; exit 1; }
    echo "{\"args\": \"$args\", \"line\": $(tail -1 gpurun_out/bigT.log)}" >> gpurun_out/bigT.jsonl
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/bigT.jsonl"):
    d = json.loads(l); L = d["line"]; r = L["roofline"]
    print(d["args"], L["config"]["tiles_per_step"], f'{L["ms_per_step"]:.3f} ms/step', r["kernel"], f'{r["kernel_ms"]:.1f}', f'frac {r["frac"]:.3f}', f'e2e {L["schedule"]["end_to_end_updates_per_s"]/L["value"]:.3f}')
PY
