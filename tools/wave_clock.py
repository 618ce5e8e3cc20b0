"""Cycles per tick and the held shader clock of the wavefront kernel, from the diagnostic
build's in-kernel stamps (make -C radiative-transfer_amd variant V=stamps
RT_DEFS=-DRT_WAVE_STAMPS; lane 0 of every wave records s_memtime / s_memrealtime at entry,
before and after its tick stream).  Run with RTSN_LIB pointing at that build:
  RTSN_LIB=radiative-transfer_amd/variants/stamps/librtsn.so python tools/wave_clock.py
One JSON line per (config, steps): wall time of advance + finish + sync (best of 5), and from
the stamps of the last launch: cycles per tick, clock (memtime / memrealtime x 100 MHz),
prologue and epilogue cycles, the spread of the waves' start times and the in-kernel span."""
import ctypes as C
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import rtsn  # noqa: E402
from rtsn import api  # noqa: E402

pdir = REPO / "tests" / "golden" / "prm"
base = rtsn.ParameterHandler(pdir / "llnl_slab_test.prm", table_dir=str(pdir) + "/").params


def configs():
    yield "llnl_slab_test", dict(base)
    eq = rtsn.ParameterHandler(pdir / "multi_group_equilibrium.prm", table_dir=str(pdir) + "/").params
    yield "multi_group_equilibrium", dict(eq)
    for N, G in ((256, 4), (1000, 4)):
        q = dict(base, N=N, G=G, group_bounds=None, group_kappa=None, dt=1e-9)
        q["psi_source"] = np.ones((q["M"], G))
        yield f"llnl_material_N{N}_G{G}", q


def stamps(nwaves):
    L = api.lib()
    f = L.rt_debug_wave_stamps
    f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    buf = (C.c_ulonglong * (6 * nwaves))()
    n = f(buf, nwaves)
    if n < 0:
        raise RuntimeError("rt_debug_wave_stamps failed")
    return np.frombuffer(buf, dtype=np.uint64).reshape(nwaves, 6).astype(np.int64)


def main():
    if "stamps" not in os.environ.get("RTSN_LIB", ""):
        print("set RTSN_LIB to the stamps variant", file=sys.stderr)
        sys.exit(2)
    for name, q in configs():
        for steps in (1000, 2000):
            q = dict(q, max_timesteps=steps)
            with rtsn.Solver(q) as s:
                st = s.wavefront_state()
                if not st["active"]:
                    print(json.dumps({"config": name, "skip": "not a wavefront line"}), flush=True)
                    break
                s.advance(8)
                s.finish()
                s.synchronize()
                best = None
                for _ in range(5):
                    t0 = time.perf_counter()
                    s.advance(steps)
                    s.finish()
                    s.synchronize()
                    dt = time.perf_counter() - t0
                    best = dt if best is None else min(best, dt)
                bc2 = q["bc_left_indicator"] == 2
                lines = q["M"] // 2 * q["G"]
                grid = lines if bc2 else 2 * lines
                nw = grid * st["waves"]
                a = stamps(nw)
                lanes = -(-q["N"] // st["cells_per_lane"]) * (2 if bc2 else 1)
                ticks = steps + lanes - 1
                loop_cyc = a[:, 4] - a[:, 2]
                loop_real = (a[:, 5] - a[:, 3]) / 100e6
                clock = loop_cyc / np.maximum(loop_real, 1e-12)
                span = (a[:, 5].max() - a[:, 1].min()) / 100e6
                print(json.dumps({
                    "config": name, "steps": steps, "N": q["N"], "G": q["G"], "waves": st["waves"],
                    "cells_per_lane": st["cells_per_lane"], "ticks": ticks, "wall_us": 1e6 * best,
                    "span_us": 1e6 * span,
                    "cycles_per_tick": float(np.median(loop_cyc) / ticks),
                    "cycles_per_tick_max": float(loop_cyc.max() / ticks),
                    "clock_ghz": float(np.median(clock) / 1e9), "clock_min_ghz": float(clock.min() / 1e9),
                    "prologue_cyc": float(np.median(a[:, 2] - a[:, 0])),
                    "start_spread_us": float((a[:, 1].max() - a[:, 1].min()) / 100e6 * 1e6),
                    "loop_us": float(np.median(loop_real) * 1e6)}), flush=True)


if __name__ == "__main__":
    main()
