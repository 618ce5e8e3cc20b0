"""Whole-run time of n BDF2 steps on the SL slab with G groups (advance + finish + sync,
pipelined) over a grid of time block T, waves per segment KW (rt_set_level_waves, used by
every launch of the run) and segments per line (rt_set_segmentation(w): Sg = CUs w / (2 Q)):
the data behind the small-shard schedule.  A fresh handle per configuration
at dt = 1e-9 (RTSN_GRID_DT), where the reference's BDF2 keeps the SL state finite for more
than 4000 steps (profiles/archive/r03j_finite_horizon.jsonl; at 1e-7 it overflows within 400 and
inf arithmetic runs faster).
usage: python -u tools/run_grid.py G n1,n2 T1,T2 KW1,KW2 w1,w2"""
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import bench  # noqa: E402
import rtsn  # noqa: E402

G, runs = int(sys.argv[1]), [int(x) for x in sys.argv[2].split(",")]
Ts, KWs, Ws = ([int(x) for x in a.split(",")] for a in sys.argv[3:6])
p = dict(bench.slab_params(G, "v0"), dt=float(os.environ.get("RTSN_GRID_DT", "1e-9")))
for w in Ws:
    for T in Ts:
        for kw in KWs:
            with rtsn.Solver(p) as s:
                s.set_segmentation(w)
                s.pipeline = 2
                try:
                    s.time_block = T
                    s.level_waves = kw
                except rtsn.RtError as e:
                    print(json.dumps({"T": T, "kw": kw, "w": w, "error": str(e)}), flush=True)
                    continue
                if s.level_waves != kw:
                    continue
                s.advance(T)  # warm this block's kernels and segments
                s.finish()
                s.synchronize()
                segs = s.sweep_geometry()[1]
                for n in runs:
                    t0 = time.perf_counter()
                    s.advance(n)
                    s.finish()
                    s.synchronize()
                    dt = time.perf_counter() - t0
                    print(json.dumps({"groups": G, "steps": n, "T": T, "kw": kw, "w": w, "segments": segs,
                                      "ms": 1e3 * dt, "ms_per_step": 1e3 * dt / n, "dt": p["dt"],
                                      "finite": s.state_finite()}), flush=True)
