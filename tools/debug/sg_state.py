"""single_group.prm's wavefront plan (rt_wavefront_state) and its solve split into phases."""
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import rtsn  # noqa: E402

pdir = REPO / "tests" / "golden" / "prm"
for name in ("single_group.prm", "multi_group_equilibrium.prm", "llnl_slab_test.prm"):
    ph = rtsn.ParameterHandler(pdir / name, table_dir=str(pdir) + "/")
    for rep in range(3):
        with rtsn.Solver(ph) as s:
            st = s.wavefront_state()
            s.synchronize()
            t0 = time.perf_counter()
            s.advance(ph.params["max_timesteps"])
            t1 = time.perf_counter()
            s.finish()
            t2 = time.perf_counter()
            s.synchronize()
            t3 = time.perf_counter()
    print(json.dumps({"config": name, "wavefront": st, "advance_ms": 1e3 * (t1 - t0),
                      "finish_ms": 1e3 * (t2 - t1), "sync_ms": 1e3 * (t3 - t2)}), flush=True)
