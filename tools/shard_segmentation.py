"""The steady T = 20 pipelined pass of the SL slab at G groups per GPU against the segmentation
(rt_set_segmentation: workgroups per CU the segments are sized for; 0 = the default, the
kernel's occupancy).  Why: the 16-group shard (one rank of the 8-GPU strong-scaling run)
ran 5.6% slower per update than 128 groups with the same 1024 workgroups per pass
(profiles/archive/r04u_bench_1gpu_groups16.json): each workgroup then holds 8x less work, so a
fixed per-launch cost (the last workgroups' spread, the launch boundary) weighs 8x more.
For each (G, w): fill the pipeline, time `passes` steady passes (host clock between device
syncs, and the per-launch kernel time), one JSON line each.
  python tools/shard_segmentation.py [G,...] [w,...] [passes]"""
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import bench  # noqa: E402
import rtsn  # noqa: E402

GS = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "16").split(",")]
WS = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0,2,4,8,16").split(",")]
PASSES = int(sys.argv[3]) if len(sys.argv) > 3 else 4
T = 20
for G in GS:
    for w in WS:
        p = dict(bench.slab_params(G, "v0"), dt=1e-9)
        with rtsn.Solver(p) as s:
            s.time_block = T
            s.pipeline = 1
            if w:
                s.set_segmentation(w)
            wg, tiles = s.sweep_geometry()
            s.advance(tiles * T)  # the fill: every position running
            s.synchronize()
            before = s.pipeline_state()
            s.set_profiling(True)
            t0 = time.perf_counter()
            s.advance(PASSES * T)
            s.synchronize()
            wall = time.perf_counter() - t0
            kern_ms, nl = s.sweep_time()
            s.set_profiling(False)
            steady = s.pipeline_state() == before
            upd = 4.0 * p["M"] * G * p["N"] * PASSES * T
            print(json.dumps({"groups": G, "wgs_per_cu": w, "workgroups": wg, "positions": tiles,
                              "steady": steady, "ms_per_step": 1e3 * wall / (PASSES * T),
                              "kernel_ms_per_launch": kern_ms / max(nl, 1), "launches": nl,
                              "updates_per_s": upd / wall}), flush=True)
