# SQ/GRBM counters of the one-wave vs the level-split T = 16 pass (clock, issue, waits)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
B="bench.py --no-cpu-baseline --side-legs 0 --material-steps 0"
for lw in 1 2; do
  RTSN_LEVEL_WAVES=$lw timeout -k 10 300 python3 $B > gpurun_out/splitpmc_b$lw.log 2>&1 || { tail -5 gpurun_out/splitpmc_b$lw.log; exit 1; }
  RTSN_LEVEL_WAVES=$lw timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/splitpmc_$lw -o run --output-format csv -- python3 $B > gpurun_out/splitpmc_$lw.log 2>&1 || { tail -5 gpurun_out/splitpmc_$lw.log; exit 1; }
done
python3 - <<'PY'
import csv, json
from pathlib import Path
out = {}
for lw in (1, 2):
    b = [json.loads(l) for l in open(f"gpurun_out/splitpmc_b{lw}.log") if l.startswith('{"metric')][-1]
    ms = b["roofline"]["kernel_ms"]
    c = {}
    for f in Path(f"gpurun_out/splitpmc_{lw}").rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if ("sweep_split_kernel<3, 16>" in n or "sweep_block_kernel<3, 16, 2, false>" in n):
                c.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    m = {k: max(v) for k, v in c.items()}
    m["kernel_ms"] = ms
    m["clock_ghz"] = m["GRBM_GUI_ACTIVE"] / 8 / (ms * 1e-3) / 1e9
    m["valu_per_busy"] = m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVE_CYCLES"]
    out[f"level_waves_{lw}"] = m
print(json.dumps(out, indent=1))
json.dump(out, open("gpurun_out/split_pmc.json", "w"), indent=1)
PY
