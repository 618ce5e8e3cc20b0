# Pipeline fill/drain with the fill-split launches (default) vs without (RTSN_LEVEL_WAVES=2,
# the same T = 20 steady-state kernel), the driver's window; and T = 16 (K = 32).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/fill.jsonl
run() {  # tag, env, args
  tag=$1; envv=$2; shift 2
  env $envv timeout -k 10 300 python bench.py --no-cpu-baseline --side-legs 0 --material-steps 0 "$@" > gpurun_out/fill_$tag.log 2>&1 || { tail -20 gpurun_out/fill_$tag.log; exit 1; }
  echo "{\"tag\": \"$tag\", \"env\": \"$envv\", \"line\": $(tail -1 gpurun_out/fill_$tag.log)}" >> gpurun_out/fill.jsonl
}
for rep in 1 2; do
  run auto_k20 "RTSN_X=0" --steps 20 --warmup 5
  run lw2_k20 "RTSN_LEVEL_WAVES=2" --steps 20 --warmup 5
  run auto_k32 "RTSN_X=0" --steps 32
  run lw1_k32 "RTSN_LEVEL_WAVES=1" --steps 32
done
python3 - <<'PY'
import json
for l in open("gpurun_out/fill.jsonl"):
    d = json.loads(l); L = d["line"]; sc = L["schedule"]
    print(d["tag"], f'{L["ms_per_step"]:.3f} ms/step', f'warm+timed+drain {sc["end_to_end_ms"]:.0f} ms', f'drain {sc["drain_ms"]:.0f} ms',
          f'e2e {sc["end_to_end_updates_per_s"]:.3e}', f'ratio {sc["end_to_end_updates_per_s"]/L["value"]:.3f}')
PY
