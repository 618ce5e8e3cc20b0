"""rt_solve's plan against forced schedules on long few-group lines, where the plan's model
is furthest from the measured time (tools/launch_gaps.py: 4-group 5000-cell lines, 1000
steps, estimated 3.2 ms, run 7.3 ms).  For each N: the plan's run, then every (time block T,
waves per segment, workgroups per CU) the pipelined schedule takes, forced through
rt_set_time_block / rt_set_level_waves / rt_set_segmentation with rt_set_pipeline(2); the best
of 3 host-timed runs each.  python tools/plan_sweep_mid.py [N ...] -> one JSON line per run."""
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import rtsn  # noqa: E402

pdir = REPO / "tests" / "golden" / "prm"
base = rtsn.ParameterHandler(pdir / "llnl_slab_test.prm", table_dir=str(pdir) + "/").params
STEPS = 1000


def params(N, G=4):
    q = dict(base, N=N, G=G, group_bounds=None, group_kappa=None, dt=1e-9, max_timesteps=STEPS,
             bc_left_indicator=0, bc_right_indicator=0)
    q["psi_source"] = np.ones((q["M"], G))
    return q


def timed(q, setup):
    with rtsn.Solver(q) as s:
        info = setup(s)
        best = None
        for _ in range(3):
            s.synchronize()
            t0 = time.perf_counter()
            s.solve()
            s.synchronize()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        return 1e3 * best, info


for N in [int(a) for a in sys.argv[1:]] or [5000, 20000]:
    q = params(N)
    ms, plan = timed(q, lambda s: s.plan_schedule(STEPS))
    print(json.dumps({"N": N, "run": "plan", "ms": ms, "plan": plan}), flush=True)
    for T in (4, 8, 16, 20):
        for lw in (1, 2, 4):
            for w in (1, 2, 4, 8, 16):
                def setup(s, T=T, lw=lw, w=w):
                    s.time_block = T
                    s.pipeline = 2
                    s.level_waves = lw
                    s.set_segmentation(w)
                    return {"T": s.time_block, "level_waves": s.level_waves, "wgs_per_cu": w}
                try:
                    ms, info = timed(q, setup)
                except rtsn.RtError as e:  # a (T, waves) pair without a kernel
                    continue
                print(json.dumps({"N": N, "run": "forced", "ms": ms, **info}), flush=True)
