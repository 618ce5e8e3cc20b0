# T = 20 pass: one wave (AGPR-assisted) vs level-split over two waves, same box, alternating.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --side-legs 0 --material-steps 0 --steps 20 --warmup 5"
: > gpurun_out/split20.jsonl
for rep in 1 2; do
  for lw in 1 2; do
    RTSN_LEVEL_WAVES=$lw timeout -k 10 300 $B > gpurun_out/s20_$lw.log 2>&1 || { tail -20 gpurun_out/s20_$lw.log; exit 1; }
    echo "{\"level_waves\": $lw, \"rep\": $rep, \"line\": $(tail -1 gpurun_out/s20_$lw.log)}" >> gpurun_out/split20.jsonl
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/split20.jsonl"):
    d = json.loads(l); r = d["line"]["roofline"]
    print(d["level_waves"], d["rep"], r["kernel"], f'{d["line"]["ms_per_step"]:.3f} ms/step', f'kernel {r["kernel_ms"]:.1f}', f'frac {r["frac"]:.3f}')
PY
