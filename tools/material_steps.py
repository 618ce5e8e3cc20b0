"""A few material-coupled steps on the SL slab (128 groups) with a given time scheme, for a
kernel trace of the coupled pass and the correction's share: usage
python -u tools/material_steps.py ts steps   (ts 1 BE, 2 CN, 3 BDF2; V = 0, dt = 1e-7)."""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import bench  # noqa: E402
import rtsn  # noqa: E402

ts, steps = int(sys.argv[1]), int(sys.argv[2])
p = dict(bench.slab_params(128, "v0"), ts_method=ts, V=0.0, dt=1e-7)
with rtsn.Solver(p) as s:
    s.material_enable(1.0)
    s.material_step(steps)
    s.synchronize()
    print("ts", ts, "steps", steps, "T finite", bool((s.temperature() > 0).all()), flush=True)
