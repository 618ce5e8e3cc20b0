"""Time the material-coupled step (rt_material_step) on the SL slab, 1 GPU.

Usage (GPU box): python scripts/material_perf.py [--groups 128] [--cells 1000000] [--steps 3] [--T0 1.0]
Prints one JSON line: ms per coupled step (sweep + finalize + moments + q +
T update + Planck), from radiation at B(1 keV) and material at T0 (default 1 keV, the
uniform equilibrium; T0 = 0.1: every cell heats by many times T, the full-emission solve).
"""
import argparse
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "radiative-transfer_amd"))

import bench  # noqa: E402
import rtsn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=128)
    ap.add_argument("--cells", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--ts", type=int, default=1)
    ap.add_argument("--T0", type=float, default=1.0)
    a = ap.parse_args()
    p = bench.slab_params(a.groups, "v0", N=a.cells)
    p["ts_method"] = a.ts
    t0 = time.perf_counter()
    with rtsn.Solver(p) as s:
        t1 = time.perf_counter()
        s.material_enable(1.0, None if a.T0 == 1.0 else [a.T0] * a.cells)
        s.synchronize()
        t2 = time.perf_counter()
        s.material_step(1)  # warm-up (propagators for T = 1 are built here)
        s.synchronize()
        T1 = s.temperature()
        t3 = time.perf_counter()
        s.material_step(a.steps)
        s.synchronize()
        t4 = time.perf_counter()
        T = s.temperature()
    print(json.dumps({"groups": a.groups, "cells": a.cells, "ts_method": a.ts, "create_s": t1 - t0,
                      "enable_s": t2 - t1, "first_step_s": t3 - t2,
                      "ms_per_coupled_step": 1e3 * (t4 - t3) / a.steps,
                      "T0": a.T0, "T_after_first": [float(T1.min()), float(T1.max())],
                      "T_min": float(T.min()), "T_max": float(T.max())}))


if __name__ == "__main__":
    main()
