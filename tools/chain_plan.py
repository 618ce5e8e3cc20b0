"""The wavefront plan's crossovers, re-measured on round 4's chain_kernel:
1000 BDF2 steps of llnl_slab_test's material on N-cell lines (4 groups, M = 2: 8 lines), every
feasible cells-per-lane choice C (rt_set_wavefront_cells; the chain spans ceil(lanes / 64)
waves), vacuum and reflective, median of 3 runs (advance + finish + sync after an 8-step warm
start).  python tools/chain_plan.py [vacuum|reflective] [N ...] -> one JSON line per (N, bc_left, C)."""
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import rtsn  # noqa: E402

STEPS = 1000
pdir = REPO / "tests" / "golden" / "prm"
base = rtsn.ParameterHandler(pdir / "llnl_slab_test.prm", table_dir=str(pdir) + "/").params


def params(N, bc_left, G=4):
    q = dict(base, N=N, max_timesteps=STEPS, dt=1e-9, bc_left_indicator=bc_left, bc_right_indicator=1 if bc_left else 0,
             G=G, group_bounds=None, group_kappa=None)
    q["psi_source"] = np.ones((q["M"], G))
    return q


def run(q, C):
    with rtsn.Solver(q) as s:
        s.wavefront = 2
        s.set_wavefront_cells(C)
        st = s.wavefront_state()
        if st["cells_per_lane"] != C:
            return None, st
        s.advance(8)
        s.finish()
        s.synchronize()
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            s.advance(STEPS)
            s.finish()
            s.synchronize()
            ts.append(time.perf_counter() - t0)
        return sorted(ts)[1], st


ARGS = sys.argv[1:]
KINDS = {"vacuum": (0,), "reflective": (2,)}.get(ARGS[0] if ARGS else "", (0, 2))
if ARGS and ARGS[0] in ("vacuum", "reflective"):
    ARGS = ARGS[1:]
LENGTHS = [int(a) for a in ARGS] or [65, 129, 192, 256, 320, 384, 448, 512, 640, 768, 1024, 1536, 2048]
for bcl in KINDS:
    for N in LENGTHS:
        q = params(N, bcl)
        with rtsn.Solver(q) as s:
            s.wavefront = 2
            auto = s.wavefront_state()
        for C in (1, 2, 4, 8):
            dt, st = run(q, C)
            if dt is None:
                continue
            lanes = -(-N // C) * (2 if bcl == 2 else 1)
            print(json.dumps({"N": N, "bc_left": bcl, "C": C, "waves": st["waves"], "us": round(1e6 * dt, 2),
                              "ticks": STEPS + lanes - 1, "ns_per_tick": round(1e9 * dt / (STEPS + lanes - 1), 2),
                              "plan_C": auto["cells_per_lane"], "plan_waves": auto["waves"]}), flush=True)
