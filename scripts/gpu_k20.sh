# The driver's window with 2 vs 4 waves per segment for the T = 20 pass, alternating.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/k20w.jsonl
B="python bench.py --no-cpu-baseline --side-legs 0 --material-steps 0 --steps 20 --warmup 5"
for rep in 1 2; do
  for lw in 2 4; do
    RTSN_LEVEL_WAVES=$lw timeout -k 10 300 $B > gpurun_out/k20w.log 2>&1 || { tail -20 gpurun_out/k20w.log; exit 1; }
    echo "{\"level_waves\": $lw, \"line\": $(tail -1 gpurun_out/k20w.log)}" >> gpurun_out/k20w.jsonl
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/k20w.jsonl"):
    d = json.loads(l); L = d["line"]; r = L["roofline"]
    print(d["level_waves"], L["config"]["tiles_per_step"], f'{L["ms_per_step"]:.3f} ms/step', r["kernel"], f'{r["kernel_ms"]:.1f}', f'frac {r["frac"]:.3f}', f'e2e {L["schedule"]["end_to_end_updates_per_s"]/L["value"]:.3f}')
PY
