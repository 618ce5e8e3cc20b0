#!/usr/bin/env python3
"""Per-dispatch view of a rocprofv3 --kernel-trace run of bench.py.

usage: trace_summary.py <run_kernel_trace.csv> <out.json>

The pipelined schedule's first and last launches (fill / drain) cover fewer
segments than a steady-state pass, so the kernel's plain average over all
dispatches is not the per-pass time bench.py reports.  Dispatches are
grouped by (kernel, grid size); for each group: count, mean and median
duration.  The steady-state pass is the sweep-kernel group (one-wave sweep_block_kernel or
level-split sweep_split_kernel) with the most workgroups -- every chain position active --
ties to the most time (the fill and drain launches may run a kernel with more waves per
workgroup and more total time over fewer workgroups).
"""
import csv
import json
import statistics
import sys
from collections import defaultdict


def main():
    src, out = sys.argv[1:3]
    groups = defaultdict(list)
    wg = {}
    for r in csv.DictReader(open(src)):
        dur_ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        key = (r["Kernel_Name"], int(r["Grid_Size_X"]))
        groups[key].append(dur_ms)
        wg[key] = int(r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or 0)
    rows = []
    for (name, grid), d in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        w = wg[(name, grid)]
        rows.append({"kernel": name, "grid_threads": grid, "workgroups": grid // w if w else None,
                     "dispatches": len(d), "total_ms": sum(d), "mean_ms": statistics.mean(d),
                     "median_ms": statistics.median(d)})
    # per sweep kernel its full-grid group; the headline pass is the one with the most time
    # (the material-coupled pass, `..., true>`, runs a larger grid but is not the headline)
    per_kernel = {}
    for r in rows:
        if "sweep_block_kernel" in r["kernel"] or "sweep_split_kernel" in r["kernel"]:
            best = per_kernel.get(r["kernel"])
            if best is None or r["grid_threads"] > best["grid_threads"]:
                per_kernel[r["kernel"]] = r
    total = defaultdict(float)
    for r in rows:
        total[r["kernel"]] += r["total_ms"]
    full = (max(per_kernel.values(), key=lambda r: (r["workgroups"] or 0, total[r["kernel"]]))
            if per_kernel else None)
    res = {"steady_state_pass": full, "full_grid_per_kernel": list(per_kernel.values()), "groups": rows}
    open(out, "w").write(json.dumps(res, indent=1) + "\n")
    print(json.dumps(full))


if __name__ == "__main__":
    main()
