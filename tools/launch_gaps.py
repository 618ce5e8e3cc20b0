"""Is a whole run launch-bound?  rt_solve of 1000 BDF2 steps on long lines with few groups
(llnl_slab_test's material, G groups, vacuum) and of the 16-group SL shard (100 steps): the
host wall time of the solve (device sync on both sides, the second of two runs), the sweep
launches it made and the sum of their HIP-event durations (rt_set_profiling, on alternate
runs), so the unprofiled wall - sum is the time the GPU sat between launches.
  python tools/launch_gaps.py -> one JSON line per case."""
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import bench  # noqa: E402
import rtsn  # noqa: E402

pdir = REPO / "tests" / "golden" / "prm"
base = rtsn.ParameterHandler(pdir / "llnl_slab_test.prm", table_dir=str(pdir) + "/").params


def mid(N, G, steps=1000):
    q = dict(base, N=N, G=G, group_bounds=None, group_kappa=None, dt=1e-9, max_timesteps=steps,
             bc_left_indicator=0, bc_right_indicator=0)
    q["psi_source"] = np.ones((q["M"], G))
    return q


cases = [(f"llnl_material_N{N}_G4", mid(N, 4)) for N in (5000, 10000, 50000, 200000)]
cases.append(("SL_16_groups_100_steps", dict(bench.slab_params(16, "v0"), dt=1e-9, max_timesteps=100)))
for name, q in cases:
    with rtsn.Solver(q) as s:
        plan = s.plan_schedule(q["max_timesteps"])
        walls = []
        for rep in range(4):  # profiled (event pairs around every launch) on even reps
            prof = rep % 2 == 0
            s.synchronize()
            s.set_profiling(prof)
            t0 = time.perf_counter()
            s.solve()
            s.synchronize()
            walls.append((prof, time.perf_counter() - t0))
            if prof:
                kern_ms, nl = s.sweep_time()
            s.set_profiling(False)
    wall = min(w for p, w in walls[1:] if not p)  # unprofiled, after the first run
    print(json.dumps({"case": name, "plan": plan, "wall_ms": 1e3 * wall,
                      "wall_profiled_ms": 1e3 * min(w for p, w in walls if p), "launches": nl, "kernel_ms": kern_ms,
                      "gap_ms": 1e3 * wall - kern_ms, "gap_per_launch_us": (1e3 * wall - kern_ms) * 1e3 / max(nl, 1),
                      "gap_fraction": 1 - kern_ms / (1e3 * wall)}), flush=True)
