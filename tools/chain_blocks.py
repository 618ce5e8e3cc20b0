"""Where a chain's ticks go: per-block stamps of chain_kernel's workgroup 0 (diagnostic build
make -C radiative-transfer_amd variant V=stamps RT_DEFS=-DRT_WAVE_STAMPS; every wave's
s_memtime before and after each block's barrier).  For each wave: the cycles per tick it
computes in unmasked blocks (every lane at a level in [1, n)), in masked ones, and what it
waits at the barriers.  RTSN_LIB=.../variants/stamps/librtsn.so python tools/chain_blocks.py"""
import ctypes as C
import json
import os
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import rtsn  # noqa: E402
from rtsn import api  # noqa: E402

pdir = REPO / "tests" / "golden" / "prm"
base = rtsn.ParameterHandler(pdir / "llnl_slab_test.prm", table_dir=str(pdir) + "/").params
BLOCK, SKEW, NB, MAXW = 8, 16, 2048, 8


def block_stamps():
    f = api.lib().rt_debug_block_stamps
    f.argtypes = [C.POINTER(C.c_ulonglong)]
    buf = (C.c_ulonglong * (2 * MAXW * NB))()
    if f(buf) < 0:
        raise RuntimeError("rt_debug_block_stamps failed")
    return np.frombuffer(buf, dtype=np.uint64).reshape(MAXW, NB, 2).astype(np.int64)


def main():
    if "stamps" not in os.environ.get("RTSN_LIB", ""):
        sys.exit("set RTSN_LIB to the stamps variant")
    steps = 1000
    for N, bc in ((1000, 0), (2000, 0), (4000, 0), (600, 0), (1000, 2)):
        q = dict(base, N=N, G=4, group_bounds=None, group_kappa=None, dt=1e-9, bc_left_indicator=bc,
                 max_timesteps=steps)
        q["psi_source"] = np.ones((q["M"], 4))
        with rtsn.Solver(q) as s:
            st = s.wavefront_state()
            nw, Cc = st["waves"], st["cells_per_lane"]
            s.advance(steps)
            s.finish()
            s.synchronize()
            a = block_stamps()
        lanes = -(-N // Cc) * (2 if bc == 2 else 1)
        ticks = steps + lanes - 1
        nblocks = (ticks + (nw - 1) * SKEW + BLOCK - 1) // BLOCK
        out = {"N": N, "bc_left": bc, "waves": nw, "cells_per_lane": Cc, "ticks": ticks, "blocks": nblocks}
        total = a[0, nblocks - 1, 1] - a[0, 0, 0]
        out["cycles_per_wall_tick"] = float(total / (nblocks * BLOCK))
        per = []
        for w in range(nw):
            u_lo = min(64 * w + 63, lanes - 1) + 1
            u_hi = max(u_lo, steps + 64 * w)
            comp = a[w, 1:nblocks, 0] - a[w, 0:nblocks - 1, 1]
            wait = a[w, 1:nblocks, 1] - a[w, 1:nblocks, 0]
            kinds = []
            for b in range(1, nblocks):
                t0 = b * BLOCK - w * SKEW
                if t0 >= u_lo and t0 + BLOCK <= u_hi:
                    kinds.append("unmasked")
                elif t0 + BLOCK <= 64 * w or t0 >= ticks:
                    kinds.append("idle")
                else:
                    kinds.append("masked")
            kinds = np.array(kinds)
            d = {"wave": w}
            for k in ("unmasked", "masked", "idle"):
                m = kinds == k
                if m.any():
                    d[k] = {"blocks": int(m.sum()), "compute_per_tick": float(np.median(comp[m]) / BLOCK),
                            "wait_per_tick": float(np.median(wait[m]) / BLOCK)}
            per.append(d)
        out["per_wave"] = per
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
