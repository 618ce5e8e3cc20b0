#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes of the sweep kernel into profiles/pmc_<tag>.json.

usage: pmc_summary.py <tag> <fetch_dir> <write_dir> [<sq_dir> ...]
(tag = <variant>_t<time block>, the name bench.py looks up)

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a
16-B-per-lane streaming read, so it is doubled.
"""
import csv
import json
import sys
from pathlib import Path

KERNEL = "sweep_block_kernel"


def counters(d, names=None):
    """{counter: [values]} over the sweep passes' launches; `names` (a dict) receives
    {counter: [kernel names]} in the same order."""
    out = {}
    for f in Path(d).rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            targs = name.replace(" ", "").split("(")[0].split("<")[-1].rstrip(">").split(",")
            # a sweep pass: sweep_block_kernel<S, T, mode[, material]> with mode 0 aligned or 2
            # pipelined (1 = finalize), or the level-split sweep_split_kernel<S, T, waves>
            block = KERNEL in name and len(targs) >= 3 and targs[2] in ("0", "2") and "true" not in targs[3:]
            if block or "sweep_split_kernel" in name:
                out.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
                if names is not None:
                    names.setdefault(r["Counter_Name"], []).append(name.split("(")[0].strip())
    return out


def main():
    variant, fdir, wdir, *rest = sys.argv[1:]
    # the largest launch is a full pass (pipeline fill/drain launches cover fewer segments)
    names = {}
    fetch = counters(fdir, names)["FETCH_SIZE"]
    write = counters(wdir)["WRITE_SIZE"]
    rd = max(fetch) * 1024 * 2
    wr = max(write) * 1024
    # the kernel of the largest launch (the full pass the bytes are quoted for)
    kernel = names["FETCH_SIZE"][fetch.index(max(fetch))]
    res = {"variant": variant, "kernel": kernel, "launches": len(fetch),
           "fetch_size_kib_max": max(fetch), "write_size_kib_max": max(write),
           "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
           "hbm_bytes_per_launch": rd + wr,
           "correction": "FETCH_SIZE x 2 (gfx950 half-count of 16 B/lane streaming reads), KiB -> bytes"}
    for d in rest:
        for k, v in counters(d).items():
            res[k + "_max"] = max(v)
    out = Path(__file__).resolve().parent.parent / "profiles" / f"pmc_{variant}.json"
    out.write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
