#!/usr/bin/env python3
"""The sweep launches of a rocprofv3 --kernel-trace run in dispatch order: kernel, grid
(workgroups), waves per workgroup, duration -- the pipeline's fill, steady and drain
launches of a whole run side by side (the per-launch view behind DESIGN.md §5's fill /
drain analysis).  usage: launch_sequence.py run_kernel_trace.csv out.jsonl"""
import csv
import json
import sys


def main():
    src, out = sys.argv[1:3]
    rows = []
    for r in csv.DictReader(open(src)):
        name = r["Kernel_Name"]
        if "sweep_" not in name and "wavefront" not in name:
            continue
        wg = int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", "64")))
        rows.append({"start_ns": int(r["Start_Timestamp"]), "kernel": name.split("(")[0],
                     "workgroups": int(r["Grid_Size_X"]) // wg, "waves_per_wg": wg // 64,
                     "ms": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6})
    rows.sort(key=lambda x: x["start_ns"])
    t0 = rows[0]["start_ns"] if rows else 0
    with open(out, "w") as f:
        for i, r in enumerate(rows):
            r["i"] = i
            r["t_ms"] = (r.pop("start_ns") - t0) / 1e6
            f.write(json.dumps(r) + "\n")
    print(f"{len(rows)} sweep launches, {sum(r['ms'] for r in rows):.1f} ms of kernel time")


if __name__ == "__main__":
    main()
