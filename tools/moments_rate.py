"""moments_kernel on the SL slab (N = 1e6 x S64 x 128 groups, 131 GB of state): the read-out
that every real run ends with (solver.cpp:191-237).  Each repetition advances one step (a new
state version, so the moments are recomputed), then times rt_get_moments_device alone
(device sync on both sides): ms and the state bytes read per ms.  Run with RTSN_LIB to time
a variant.  python tools/moments_rate.py [groups] -> one JSON line."""
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import bench  # noqa: E402
import rtsn  # noqa: E402
import torch  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 128
p = dict(bench.slab_params(G, "v0"), dt=1e-9)
out = []
with rtsn.Solver(p) as s:
    s.time_block = 1
    s.pipeline = 0
    n = s.G * s.N
    phi = torch.empty(n, dtype=torch.float64, device="cuda")
    F = torch.empty_like(phi)
    pp = torch.empty_like(phi)
    for rep in range(6):
        s.advance(1)
        s.finish()
        s.synchronize()
        t0 = time.perf_counter()
        s.moments_device(phi, F, pp)
        s.synchronize()
        out.append(1e3 * (time.perf_counter() - t0))
    # the same bytes read by the finite scan (a plain streaming read of the state, no sums)
    scan = []
    for rep in range(6):
        s.synchronize()
        t0 = time.perf_counter()
        s.state_finite()
        scan.append(1e3 * (time.perf_counter() - t0))
state_bytes = 2 * 16.0 * p["M"] / 2 * G * p["N"]  # both halves' (e_in, e_out) rows
best = min(out[1:])
print(json.dumps({"what": "moments_kernel on SL (rt_get_moments_device, host-timed)", "groups": G,
                  "lib": os.environ.get("RTSN_LIB", "default"), "ms": out, "best_ms": best,
                  "state_gb": state_bytes / 1e9, "tb_per_s": state_bytes / (best * 1e-3) / 1e12,
                  "finite_scan_best_ms": min(scan[1:]),
                  "finite_scan_tb_per_s": state_bytes / (min(scan[1:]) * 1e-3) / 1e12}), flush=True)
