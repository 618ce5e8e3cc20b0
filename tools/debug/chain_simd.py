"""Which SIMD each wave of a wavefront chain runs on (diagnostic stamps build: lane 0 of
every wave records its HW_ID register at entry).  Question: do the 2-4 waves of one chain
workgroup take distinct SIMDs of their CU, or share one (which would explain a 2-wave chain's
tick costing ~1.8x a single wave's: 141 vs 79 ns at one cell per lane)?
  RTSN_LIB=tools/debug/stamps/librtsn.so python tools/debug/chain_simd.py
One JSON line per config: per workgroup, the (SE, CU, SIMD) of each wave, and a count of
workgroups whose waves share a SIMD."""
import ctypes as C
import json
import sys
from collections import Counter
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import rtsn  # noqa: E402
from rtsn import api  # noqa: E402

pdir = REPO / "tests" / "golden" / "prm"
base = rtsn.ParameterHandler(pdir / "llnl_slab_test.prm", table_dir=str(pdir) + "/").params


def hwid(n):
    f = api.lib().rt_debug_wave_hwid
    f.argtypes = [C.POINTER(C.c_uint), C.c_int]
    f.restype = C.c_int
    out = (C.c_uint * n)()
    got = f(out, n)
    return [out[i] for i in range(max(got, 0))]


for N, bcl, Cc in ((128, 0, 1), (256, 0, 1), (100, 2, 2), (192, 0, 1), (64, 0, 1)):
    G = 4
    q = dict(base, N=N, G=G, group_bounds=None, group_kappa=None, dt=1e-9, bc_left_indicator=bcl,
             bc_right_indicator=1 if bcl else 0)
    q["psi_source"] = np.ones((q["M"], G))
    with rtsn.Solver(q) as s:
        s.wavefront = 2
        s.set_wavefront_cells(Cc)
        st = s.wavefront_state()
        s.advance(200)
        s.finish()
        s.synchronize()
        waves = st["waves"]
        wgs = G * (1 if bcl == 2 else 2)  # M = 2: one line per half and group (pairs: one per group)
        ids = hwid(wgs * waves)
    per_wg, shared = [], 0
    for b in range(wgs):
        ws = ids[b * waves:(b + 1) * waves]
        loc = [((h >> 13) & 7, (h >> 8) & 15, (h >> 4) & 3) for h in ws]
        per_wg.append(loc)
        simds = Counter((se, cu, sd) for se, cu, sd in loc)
        if max(simds.values()) > 1:
            shared += 1
    print(json.dumps({"N": N, "bc_left": bcl, "C": st["cells_per_lane"], "waves": waves, "workgroups": wgs,
                      "workgroups_sharing_a_simd": shared, "wave_locations_se_cu_simd": per_wg}), flush=True)
