"""BDF2 steps/s of the reference's own small configs (single_group, multi_group_equilibrium,
llnl_slab_test) per time block and waves per segment: 1000 steps, advance + finish + sync,
handle created and warmed outside the timer.  usage: python -u tools/small_rates.py"""
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import rtsn  # noqa: E402

pdir = REPO / "tests" / "golden" / "prm"
STEPS = 1000
for name in ("single_group.prm", "multi_group_equilibrium.prm", "llnl_slab_test.prm"):
    ph = rtsn.ParameterHandler(pdir / name, table_dir=str(pdir) + "/")
    params = dict(ph.params, max_timesteps=STEPS)
    for T, lw in ((8, 0), (16, 0), (16, 2), (16, 4), (20, 0), (20, 4), (32, 0), (40, 0)):
        with rtsn.Solver(params) as s:
            s.time_block = T
            if lw:
                s.level_waves = lw
            s.advance(2 * T)
            s.finish()
            s.synchronize()
            best = None
            for _ in range(3):
                t0 = time.perf_counter()
                s.advance(STEPS)
                s.finish()
                s.synchronize()
                dt = time.perf_counter() - t0
                best = dt if best is None else min(best, dt)
            print(json.dumps({"config": name, "T": T, "level_waves": s.level_waves, "steps": STEPS,
                              "ms": 1e3 * best, "bdf2_steps_per_s": STEPS / best}), flush=True)
