"""Reflective few-group lines: rt_solve's plan (1-2 workgroups per CU where the model puts them
3% ahead) against the previous plan's segmentation (T = 8, four waves, 4 workgroups per CU),
best of 3, 1000 BDF2 steps, 4 groups.  python tools/debug/plan_refl_check.py"""
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import rtsn  # noqa: E402

pdir = REPO / "tests" / "golden" / "prm"
base = rtsn.ParameterHandler(pdir / "llnl_slab_test.prm", table_dir=str(pdir) + "/").params
for N in (5000, 20000, 50000):
    q = dict(base, N=N, G=4, group_bounds=None, group_kappa=None, dt=1e-9, max_timesteps=1000, bc_left_indicator=2,
             bc_right_indicator=1)
    q["psi_source"] = np.ones((q["M"], 4))
    out = {"N": N, "bc_left": 2}
    for name, forced in (("plan", None), ("old_plan_w4", 4)):
        with rtsn.Solver(q) as s:
            if forced:
                s.time_block = 8
                s.pipeline = 2
                s.level_waves = 4
                s.set_segmentation(forced)
            else:
                out["plan"] = s.plan_schedule(1000)
            best = 1e9
            for _ in range(3):
                s.synchronize()
                t0 = time.perf_counter()
                s.solve()
                s.synchronize()
                best = min(best, time.perf_counter() - t0)
            out[name + "_ms"] = 1e3 * best
    print(json.dumps(out), flush=True)
