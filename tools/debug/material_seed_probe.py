"""One-off: a random material case (tests/test_random_gpu.py _material_case) on the device and
in the oracle, printing per group the largest B difference, its cell, T and both values.
usage: python tools/debug/material_seed_probe.py SEED"""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO / "tests"), str(REPO / "oracle"), str(REPO / "radiative-transfer_amd")]
import oracle as om  # noqa: E402
import rtsn  # noqa: E402
import test_random_gpu as t  # noqa: E402
from test_material_gpu import run_pair  # noqa: E402

p, T0, rc, steps, w, (lo, hi) = t._material_case(om, int(sys.argv[1]))
print({k: p[k] for k in ("M", "G", "N", "ts_method", "bc_left", "bc_right", "kappa_grey", "T", "dt", "efirst", "elast")},
      "rho_cv", rc, "steps", steps, "wgs", w)
gpu, orc = run_pair(rtsn, om, p, steps, rho_cv=rc, T0=T0, g_lo=lo, g_hi=hi, wgs_per_cu=w)
with gpu:
    Tg, To = gpu.temperature(), orc.temperature()
    Bg, Bo = gpu.cell_planck(), orc.cell_planck()
    print("T gpu", Tg, "\nT orc", To)
    for g in range(Bg.shape[0]):
        d = np.abs(Bg[g] - Bo[g])
        c = int(np.argmax(d))
        print(g, "max|dB| %.3e at cell %d T %.17g  gpu %.17g orc %.17g  group max %.3e" % (d[c], c, To[c], Bg[g, c], Bo[g, c], np.abs(Bo[g]).max()))
    print("edges", orc.groups()["e_edge"])
