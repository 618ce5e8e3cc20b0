"""PCIe-inclusive read-out of the SL state through the reference-layout host getters
(C ABI, flat host buffers in the boundary's layout, no Python transposes timed):
rt_get_psi (psi, M G N doubles), rt_get_ends / rt_set_ends (2 M G N doubles),
rt_get_moments (phi, F, phi_plus: 3 G N doubles) -- after one BDF2 pass, dt = 1e-7.
Each host buffer is read twice: first into fresh pageable memory (first-touch page
faults included), then into the same, already-faulted buffer.

usage: python -u tools/pcie_readout.py [groups]   (16 = the SL headline state, 8.2 GB psi)"""
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import bench  # noqa: E402
import rtsn  # noqa: E402
from rtsn.api import _check, _dp, lib  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 16
p = bench.slab_params(G, "v0")
p["dt"] = 1e-7


def timed(what, fn):
    t0 = time.perf_counter()
    fn()
    t = time.perf_counter() - t0
    print(what, round(t, 3), "s", flush=True)
    return t


with rtsn.Solver(p) as s:
    s.advance(16)
    s.finish()
    s.synchronize()
    print("stepped", flush=True)
    h, L = s._h, lib()
    n = s.G * s.N
    mom = [np.empty(n) for _ in range(3)]
    t_mom = timed("moments", lambda: _check(L.rt_get_moments(h, *map(_dp, mom)), "m", h))
    nb = 8 * s.M * s.G * s.N
    psi = np.empty(nb // 8)
    t_psi = timed("psi (fresh)", lambda: _check(L.rt_get_psi(h, _dp(psi)), "psi", h))
    t_psi2 = timed("psi (touched)", lambda: _check(L.rt_get_psi(h, _dp(psi)), "psi", h))
    finite = bool(np.isfinite(psi[::1000]).all())
    del psi
    ends = np.empty(2 * nb // 8)
    t_ends = timed("ends (fresh)", lambda: _check(L.rt_get_ends(h, _dp(ends)), "ends", h))
    t_ends2 = timed("ends (touched)", lambda: _check(L.rt_get_ends(h, _dp(ends)), "ends", h))
    t_set = timed("set_ends", lambda: _check(L.rt_set_ends(h, _dp(ends)), "set", h))
    out = {"groups": G, "psi_bytes": nb, "psi_GBps_fresh": nb / t_psi / 1e9, "psi_GBps": nb / t_psi2 / 1e9,
           "ends_GBps_fresh": 2 * nb / t_ends / 1e9, "ends_GBps": 2 * nb / t_ends2 / 1e9,
           "set_ends_GBps": 2 * nb / t_set / 1e9, "moments_bytes": 3 * 8 * n,
           "moments_GBps": 3 * 8 * n / t_mom / 1e9, "psi_finite": finite}
    print(json.dumps(out), flush=True)
