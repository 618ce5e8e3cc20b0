"""One whole run of n BDF2 steps (advance + finish + sync, the default auto pipeline) on
the SL slab with G groups at time block T -- for kernel traces of a run's fill, steady
and drain launches (scripts/launch_sequence.py).  dt = 1e-7 keeps the state finite.
usage: python -u tools/run_once.py G n T"""
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import bench  # noqa: E402
import rtsn  # noqa: E402

G, n, T = (int(x) for x in sys.argv[1:4])
p = bench.slab_params(G, "v0")
p["dt"] = 1e-7
with rtsn.Solver(p) as s:
    s.time_block = T
    s.advance(T)  # warm this block's kernels and segments
    s.finish()
    s.synchronize()
    t0 = time.perf_counter()
    s.advance(n)
    s.finish()
    s.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"groups": G, "steps": n, "T": T, "segments": s.sweep_geometry()[1], "ms": 1e3 * dt}), flush=True)
