"""The fixed cost around a short rt_solve: llnl_slab_test (the wavefront kernel, one launch)
for n = 1, 10, 100, 1000 BDF2 steps, median of 20 fresh handles each, timing rt_solve alone,
rt_solve + rt_finish + rt_synchronize (bench.py's rate), and the kernel by HIP events
(rt_set_profiling).  The intercept at n -> 0 is the launch + host path.
python tools/solve_overhead.py -> one JSON line per n."""
import json
import statistics
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import rtsn  # noqa: E402

pdir = REPO / "tests" / "golden" / "prm"
base = rtsn.ParameterHandler(pdir / "llnl_slab_test.prm", table_dir=str(pdir) + "/").params
with rtsn.Solver(dict(base, max_timesteps=10)) as s:  # warm: kernels loaded
    s.solve()
for n in (1, 10, 100, 1000):
    p = dict(base, max_timesteps=n)
    solve_us, full_us, kern_us = [], [], []
    for _ in range(20):
        with rtsn.Solver(p) as s:
            s.synchronize()
            t0 = time.perf_counter()
            s.solve()
            t1 = time.perf_counter()
            s.finish()
            s.synchronize()
            t2 = time.perf_counter()
            solve_us.append(1e6 * (t1 - t0))
            full_us.append(1e6 * (t2 - t0))
        with rtsn.Solver(p) as s:
            s.set_profiling(True)
            s.solve()
            s.finish()
            kern_us.append(1e3 * s.sweep_time()[0])
    print(json.dumps({"config": "llnl_slab_test", "steps": n, "solve_us": statistics.median(solve_us),
                      "solve_finish_sync_us": statistics.median(full_us),
                      "kernel_us_events": statistics.median(kern_us)}), flush=True)
