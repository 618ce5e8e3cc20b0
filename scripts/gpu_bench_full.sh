# The driver's bench command, in full (run from the repo root on the GPU box).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r02}
cat /sys/fs/cgroup/cpu.max 2>/dev/null; nproc; python -c "import os; print(len(os.sched_getaffinity(0)), os.environ.get('OMP_NUM_THREADS'))"
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2>&1 || { tail -30 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log > gpurun_out/${TAG}_bench.json
python3 - <<PY
import json
d = json.load(open("gpurun_out/${TAG}_bench.json"))
print({k: d[k] for k in ("value", "ms_per_step", "steps", "warmup")})
print("roofline", {k: d["roofline"][k] for k in ("frac", "achieved", "kernel", "kernel_ms", "traffic")})
print("schedule", d["schedule"])
print("hbm_t1", d["hbm_pass_t1"]["hbm"]["frac"], "finite ctl", d["finite_control"]["ms_per_step"])
print("material", d["material"])
print("cpu", d["cpu_baseline"])
for k, v in d["reference_config"].items():
    print(k, v["rate"])
PY
