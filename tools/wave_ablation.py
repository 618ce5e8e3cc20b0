"""1000 BDF2 steps of an N-cell x 4-group line set (default 600; argv[2] = 2: reflective left
boundary) on the wavefront (rt_set_wavefront 2), best of 5 -- for A/Bs of the chain's
geometry (RTSN_WAVE_WAVES) and of timing-only builds (RTSN_LIB).  One JSON line."""
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import rtsn  # noqa: E402

pdir = REPO / "tests" / "golden" / "prm"
q = rtsn.ParameterHandler(pdir / "llnl_slab_test.prm", table_dir=str(pdir) + "/").params
q.update(N=int(sys.argv[1]) if len(sys.argv) > 1 else 600, G=4, group_bounds=None, group_kappa=None, dt=1e-9,
         bc_left_indicator=int(sys.argv[2]) if len(sys.argv) > 2 else 0, bc_right_indicator=0)
q["psi_source"] = np.ones((q["M"], 4))
best = 1e9
for rep in range(5):
    with rtsn.Solver(q) as s:
        s.wavefront = 2
        st = s.wavefront_state()
        s.advance(8)
        s.synchronize()
        t0 = time.perf_counter()
        s.advance(1000)
        s.synchronize()
        best = min(best, time.perf_counter() - t0)
print(json.dumps({"lib": os.environ.get("RTSN_LIB", "default"), "N": q["N"], "bc_left": q["bc_left_indicator"], **st,
                  "us": 1e6 * best}), flush=True)
