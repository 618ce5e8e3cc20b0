"""Whole rt_solve time on the SL slab with G groups for runs of n BDF2 steps (handle created
and the block's kernels loaded outside the timer, on a 2000-cell run; rt_solve picks the block, rt_plan_time_block).
dt = 1e-7 keeps the state finite.  usage: python -u tools/run_solve.py G n1,n2,..."""
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import bench  # noqa: E402
import rtsn  # noqa: E402

G = int(sys.argv[1])
for n in [int(x) for x in sys.argv[2].split(",")]:
    p = bench.slab_params(G, "v0")
    p["dt"] = 1e-7
    p["max_timesteps"] = n
    T = rtsn.plan_time_block(3, n)
    with rtsn.Solver(dict(p, N=2000)) as w:  # load this block's kernels outside the timer
        w.solve()
    with rtsn.Solver(p) as s:
        s.synchronize()
        t0 = time.perf_counter()
        s.solve()
        dt = time.perf_counter() - t0
        print(json.dumps({"groups": G, "steps": n, "T": T, "time_block_after": s.time_block, "ms": 1e3 * dt,
                          "ms_per_step": 1e3 * dt / n}), flush=True)
