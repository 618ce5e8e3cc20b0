"""Whole-run time of n BDF2 steps (advance + finish + sync, auto pipeline) per time block T,
on the SL slab with G groups -- the data behind rt_solve's run-length-aware block choice.
dt = 1e-7 keeps the state finite.  usage: python -u tools/run_blocks.py G n1,n2,... T1,T2,..."""
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import bench  # noqa: E402
import rtsn  # noqa: E402

G = int(sys.argv[1])
runs = [int(x) for x in sys.argv[2].split(",")]
blocks = [int(x) for x in sys.argv[3].split(",")]
p = bench.slab_params(G, "v0")
p["dt"] = 1e-7
with rtsn.Solver(p) as s:
    s.advance(2)
    s.finish()
    s.synchronize()
    for n in runs:
        for T in blocks:
            s.time_block = T
            s.advance(T)  # warm this block's kernels and segments
            s.finish()
            s.synchronize()
            t0 = time.perf_counter()
            s.advance(n)
            s.finish()
            s.synchronize()
            dt = time.perf_counter() - t0
            print(json.dumps({"groups": G, "steps": n, "T": T, "ms": 1e3 * dt, "ms_per_step": 1e3 * dt / n}), flush=True)
