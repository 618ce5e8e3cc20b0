"""Same-box interleaved A/B of the headline pass on an overflowing vs a finite state
(verdict r02, item 4): the SL slab (128 groups) at dt = 1e-3 -- the reference's BDF2
(const_B from the full dt, solver.cpp:501) overflows it to inf within the pipeline fill --
and at dt = 1e-7, where it stays finite; the T-step pipelined pass after the fill, two
passes timed exactly as bench.py's headline, alternating A B A B ... on one process.
usage: python -u tools/ab_finite.py [T] [rounds]  -> one JSON line per leg"""
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 20
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
device = torch.device("cuda", 0)
info = (128, 0, 128)
for r in range(rounds):
    for dt in (1e-3, 1e-7):
        p = dict(bench.slab_params(128, "v0"), dt=dt, variant="v0")
        leg = bench.side_leg(p, info, 1, device, 0, "strong", T, f"A/B round {r}")
        print(json.dumps({"round": r, "dt": dt, "T": T, "ms_per_step": leg["ms_per_step"],
                          "kernel_ms": leg["kernel_ms"], "state_finite": leg["state_finite"],
                          "value": leg["value"]}), flush=True)
