# Driver window (--steps 20 --warmup 5) and others, each with segments sized for the time
# block it runs (run from the repo root on the GPU box).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --side-legs 0 --material-steps 0"
run() {  # name, args...
  n=$1; shift
  timeout -k 10 300 $B "$@" > gpurun_out/w_$n.log 2>&1 || { tail -20 gpurun_out/w_$n.log; exit 1; }
  tail -1 gpurun_out/w_$n.log > gpurun_out/w_$n.json
}
run k20 --steps 20 --warmup 5
run k20_t10 --steps 20 --warmup 5 --time-block 10
run k32 --steps 32
run k40 --steps 40
run k2 --steps 2 --warmup 1
python3 - <<'PY'
import json
for n in ("k20", "k20_t10", "k32", "k40", "k2"):
    d = json.load(open(f"gpurun_out/w_{n}.json"))
    r = d["roofline"]
    print(n, d["steps"], d["config"]["sweep_workgroups"], d["schedule"]["steps_per_pass"],
          f'{d["value"]:.3e}', f'{d["ms_per_step"]:.2f} ms/step', f'kernel {r["kernel_ms"]:.1f} ms', f'fp64 {r["fp64"]["frac"]:.3f}',
          f'e2e {d["schedule"]["end_to_end_updates_per_s"]:.3e}')
PY
