"""rt_solve whole runs on the SL slab (dt = 1e-9: finite for > 4000 steps) with the planned schedule
(rt_plan_schedule: time block, four waves per segment, segmentation) against the round-2
rule (rt_set_time_block(rt_plan_time_block) with the default waves and occupancy-sized
segments) and against forced schedules, alternating, per group count and run length.
usage: python -u tools/run_solve_plan.py G1,G2 n1,n2 [rounds] [modes]
modes: comma-separated, "planned", "round2" or "T.lw.w" (time block T, lw waves per segment,
segments for w workgroups per CU, pipelined; advance + finish); default planned,round2."""
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import bench  # noqa: E402
import rtsn  # noqa: E402

Gs = [int(x) for x in sys.argv[1].split(",")]
runs = [int(x) for x in sys.argv[2].split(",")]
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 1
modes = sys.argv[4].split(",") if len(sys.argv) > 4 else ["planned", "round2"]
for G in Gs:
    for n in runs:
        p = dict(bench.slab_params(G, "v0"), dt=1e-9, max_timesteps=n)
        for r in range(rounds):
            for mode in modes:
                with rtsn.Solver(p) as s:
                    plan = s.plan_schedule(n)
                    forced = mode not in ("planned", "round2")
                    if mode == "round2":
                        s.time_block = rtsn.plan_time_block(3, n)
                    elif forced:
                        T, lw, w = (int(x) for x in mode.split("."))
                        s.pipeline = 2
                        s.time_block = T
                        s.level_waves = lw
                        s.set_segmentation(w)
                    s.synchronize()
                    t0 = time.perf_counter()
                    if forced:
                        s.advance(n)
                        s.finish()
                        s.synchronize()
                    else:
                        s.solve()
                    ms = 1e3 * (time.perf_counter() - t0)
                    print(json.dumps({"groups": G, "steps": n, "round": r, "mode": mode, "ms": ms,
                                      "finite": s.state_finite(),
                                      "time_block": s.time_block, "level_waves": s.level_waves,
                                      "segments": s.sweep_geometry()[1], "plan": plan}), flush=True)
