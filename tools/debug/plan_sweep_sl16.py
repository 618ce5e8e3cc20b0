"""The 16-group SL shard's 100-step rt_solve (one rank of the 8-GPU strong-scaling run): the
plan against forced (T, four waves, workgroups per CU), best of 2 host-timed runs each.
  python tools/debug/plan_sweep_sl16.py -> one JSON line per run."""
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import bench  # noqa: E402
import rtsn  # noqa: E402

q = dict(bench.slab_params(16, "v0"), dt=1e-9, max_timesteps=100)
with rtsn.Solver(q) as s:
    plan = s.plan_schedule(100)
    runs = []
    for _ in range(2):
        s.synchronize()
        t0 = time.perf_counter()
        s.solve()
        s.synchronize()
        runs.append(1e3 * (time.perf_counter() - t0))
    print(json.dumps({"run": "plan", "plan": plan, "ms": min(runs)}), flush=True)
    for T in (8, 16, 20):
        for w in (2, 4, 8, 16, 32, 64):
            s.time_block = T
            s.pipeline = 2
            s.level_waves = 4
            s.set_segmentation(w)
            runs = []
            for _ in range(2):
                s.synchronize()
                t0 = time.perf_counter()
                s.solve()
                s.synchronize()
                runs.append(1e3 * (time.perf_counter() - t0))
            print(json.dumps({"run": "forced", "T": T, "level_waves": 4, "wgs_per_cu": w, "ms": min(runs)}), flush=True)
