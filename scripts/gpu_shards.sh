# Per-GPU rate of the shard each rank holds at N = 8/4/2/1 (strong scaling of the 128-group
# SL slab: 16/32/64/128 groups), driver's window, one GPU.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/shards.jsonl
for g in 16 32 64 128; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --side-legs 0 --material-steps 0 --steps 20 --warmup 5 --groups $g > gpurun_out/sh_$g.log 2>&1 || { tail -20 gpurun_out/sh_$g.log; exit 1; }
  echo "{\"groups\": $g, \"line\": $(tail -1 gpurun_out/sh_$g.log)}" >> gpurun_out/shards.jsonl
done
python3 - <<'PY'
import json
for l in open("gpurun_out/shards.jsonl"):
    d = json.loads(l); L = d["line"]; r = L["roofline"]
    print(d["groups"], L["config"]["tiles_per_step"], f'{L["value"]:.3e}', f'{L["ms_per_step"]:.3f} ms/step', r["kernel"], f'{r["kernel_ms"]:.2f} ms', f'e2e {L["schedule"]["end_to_end_updates_per_s"]/L["value"]:.3f}')
PY
