"""Whole 1000-step BDF2 runs of long lines with few groups (llnl_slab_test's material, 4
groups) -- rt_solve's plan against the same run advanced in chunks -- the aligned-schedule
cliff of round 3 (profiles/archive/r03ao_solve_mid.jsonl: chunked aligned runs 100-400x
rt_solve).  Modes:
  solve           rt_solve (the planned pipelined schedule)
  chunk7          143 x rt_advance(7) + rt_finish, auto schedule (fewer passes per call than
                  1/8 of the pipeline's depth: round 3 ran every call as aligned passes)
  chunk7_aligned  the same with rt_set_pipeline(0): aligned passes on their own segmentation
  readout50       20 x (rt_advance(50) + a moments read-out), auto schedule
python tools/solve_mid.py [N ...] -> one JSON line per (N, mode)."""
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import rtsn  # noqa: E402
import torch  # noqa: E402

pdir = REPO / "tests" / "golden" / "prm"
base = rtsn.ParameterHandler(pdir / "llnl_slab_test.prm", table_dir=str(pdir) + "/").params
STEPS = 1000


def params(N, G):
    q = dict(base, N=N, G=G, group_bounds=None, group_kappa=None, dt=1e-9, max_timesteps=STEPS,
             bc_left_indicator=0, bc_right_indicator=0)
    q["psi_source"] = np.ones((q["M"], G))
    return q


def run(s, mode, bufs):
    if mode == "solve":
        s.solve()
        return
    if mode == "chunk7_aligned":
        s.pipeline = 0
    chunk = 50 if mode == "readout50" else 7
    done = 0
    while done < STEPS:
        n = min(chunk, STEPS - done)
        s.advance(n)
        done += n
        if mode == "readout50":
            s.moments_device(*bufs)
    s.finish()


Ns = [int(a) for a in sys.argv[1:]] or [4000, 5000, 10000, 50000]
G = 4
for N in Ns:
    for mode in ("solve", "chunk7", "chunk7_aligned", "readout50"):
        best = None
        for rep in range(2):
            with rtsn.Solver(params(N, G)) as s:
                n = s.G * s.N
                bufs = [torch.empty(n, dtype=torch.float64, device="cuda") for _ in range(3)]
                s.synchronize()
                t0 = time.perf_counter()
                run(s, mode, bufs)
                s.synchronize()
                ms = 1e3 * (time.perf_counter() - t0)
                best = ms if best is None else min(best, ms)
                segs = s.sweep_geometry()[1]
                wave = s.wavefront_state()["active"]
                fin = s.state_finite()
        print(json.dumps({"N": N, "G": G, "steps": STEPS, "mode": mode, "ms": best, "segments": segs,
                          "wavefront": wave, "finite": fin}), flush=True)
