"""One-off check that a library change leaves the device Planck values bit for bit: the
per-cell B_g, the emission Beff_g, the [q, b] exchange (b = sum_g sigma_g dB_g/dT) and T
after three coupled BE steps, from cell temperatures spread over 1e-8 .. 50 keV (every
branch of the group integrals: Gauss, series, split, the remainder group), 128 groups.
usage: python tools/debug/planck_pair_bitwise.py OUT.npz   (RTSN_LIB selects the library)
       python tools/debug/planck_pair_bitwise.py --compare A.npz B.npz"""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]

if sys.argv[1] == "--compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    bad = [k for k in a.files if not np.array_equal(a[k], b[k], equal_nan=True)]
    for k in a.files:
        print(k, a[k].shape, "bitwise" if k not in bad else f"max |diff| {np.nanmax(np.abs(a[k] - b[k])):.3e}")
    sys.exit(1 if bad else 0)

import torch  # noqa: E402
import bench  # noqa: E402
import rtsn  # noqa: E402

N = 4096
p = bench.slab_params(128, "v0", N=N, M=8)
p.update(ts_method=1, dt=1e-9, use_correction=0)
T0 = np.logspace(-8, np.log10(50.0), N)
out = {}
with rtsn.Solver(p) as s:
    s.material_enable(1.0, T0)
    out["B0"], out["Beff0"] = s.cell_planck(), s.cell_emission()
    q = torch.zeros(2 * N, dtype=torch.float64, device="cuda")
    for k in range(3):
        s.material_sweep(q)
        torch.cuda.synchronize()
        out[f"qb{k}"] = q.cpu().numpy()
        s.material_update(q)
        out[f"T{k}"], out[f"Beff{k}"] = s.temperature(), s.cell_emission()
    out["B3"], out["transit"] = s.cell_planck(), s.material_transit()
np.savez(sys.argv[1], **out)
print("saved", sys.argv[1], {k: v.shape for k, v in out.items()})
