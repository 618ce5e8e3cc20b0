"""Whole-run time of n BDF2 steps on the SL slab (advance + finish + sync) per schedule:
aligned (pipeline 0), auto (1) and pipelined (2).  dt = 1e-7 keeps the state finite."""
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import bench  # noqa: E402
import rtsn  # noqa: E402

p = bench.slab_params(128, "v0")
p["dt"] = 1e-7
out = []
with rtsn.Solver(p) as s:
    s.advance(2)
    s.finish()
    s.synchronize()
    for n in (4, 16, 32, 48, 100):
        for pipe in (0, 1, 2):
            s.pipeline = pipe
            s.synchronize()
            t0 = time.perf_counter()
            s.advance(n)
            s.finish()
            s.synchronize()
            dt = time.perf_counter() - t0
            r = {"steps": n, "pipeline": pipe, "ms": 1e3 * dt, "ms_per_step": 1e3 * dt / n}
            print(json.dumps(r), flush=True)
            out.append(r)
