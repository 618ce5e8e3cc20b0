"""Mid-length lines (beyond one wave's chain): 1000 BDF2 steps of llnl_slab_test's material
on N cells with G groups, as the wavefront over a chain of waves (rt_set_wavefront 2) and as
the segment pipeline (0, at rt_solve's planned time block), and what auto (1) picks.
python tools/wave_mid_rates.py -> one JSON line per (N, G, bc_left, mode)."""
import json
import sys
import time

import numpy as np
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import rtsn  # noqa: E402

STEPS = 1000
pdir = REPO / "tests" / "golden" / "prm"
base = rtsn.ParameterHandler(pdir / "llnl_slab_test.prm", table_dir=str(pdir) + "/").params


def params(N, G, bc_left):
    q = dict(base, N=N, max_timesteps=STEPS, dt=1e-9, bc_left_indicator=bc_left, bc_right_indicator=1 if bc_left else 0)
    if G != base["G"]:
        q.update(G=G, group_bounds=None, group_kappa=None)
    q["psi_source"] = np.ones((q["M"], G))
    return q


def run(q, mode):
    with rtsn.Solver(q) as s:
        s.wavefront = mode
        if not s.wavefront_state()["active"]:
            s.time_block = rtsn.plan_time_block(3, STEPS)
        st = s.wavefront_state()
        s.advance(8)
        s.finish()
        s.synchronize()
        t0 = time.perf_counter()
        s.advance(STEPS)
        s.finish()
        s.synchronize()
        dt = time.perf_counter() - t0
        return dt, st, s.state_finite()


for N, G, bcl in [(300, 4, 2), (600, 4, 0), (1000, 4, 0), (1000, 4, 2), (2000, 4, 0), (4000, 4, 0),
                  (1000, 124, 0), (2000, 124, 0), (4000, 124, 0)]:
    q = params(N, G, bcl)
    for mode in (2, 0, 1):
        dt, st, fin = run(q, mode)
        print(json.dumps({"N": N, "G": G, "bc_left": bcl, "mode": mode, "ms": 1e3 * dt, "steps": STEPS,
                          "active": st["active"], "cells_per_lane": st["cells_per_lane"], "waves": st["waves"],
                          "finite": fin}), flush=True)
