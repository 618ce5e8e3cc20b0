"""Probe: where group 0's left group end differs between the GPU and the oracle in the
full-size SL check (test_full_size_sl_oracle_groups: M = 64, N = 1e6, dt = 1e-7, 22 BDF2
steps, T = 20 pipelined).  A one-group handle (bitwise the 128-group handle's group, by
test_full_size_sl_properties' shard check) against the oracle: per mu < 0 line, the exit
node (cell 0, node 0), its relative error, and the magnitude of the state in the cells
next to it, so the error can be set against the values it is computed from."""
import json
import sys
import time

import numpy as np

sys.path[:0] = ["oracle", "radiative-transfer_amd", "."]
import bench  # noqa: E402
import oracle  # noqa: E402
import rtsn  # noqa: E402

g = int(sys.argv[1]) if len(sys.argv) > 1 else 0
p = bench.slab_params(128, "v0")
p["dt"] = 1e-7
q = dict(p, bc_left=0, bc_right=0, dx=p["X"] / p["N"], have_group_bounds=0, have_group_kappa=1, prm_found=1,
         max_timesteps=22)
t0 = time.time()
o = oracle.OracleSolver(q, g_lo=g, g_hi=g + 1)
o.set_threads(bench.host_cpus()["threads"])
o.solve()
e_o = o.ends()[:, 0]  # (M, N, 2)
lo, ro = o.group_ends()
mu, _ = o.quad()
print(json.dumps({"oracle_s": time.time() - t0}), flush=True)
del o
with rtsn.Solver(p, g_lo=g, g_hi=g + 1) as s:
    s.pipeline = 2
    s.time_block = 20
    s.advance(22)
    s.finish()
    e_g = s.ends()[:, 0]
    lg, rg = s.compute_group_ends()
with rtsn.Solver(p) as s:  # the 128-group handle's group end
    s.pipeline = 2
    s.time_block = 20
    s.advance(22)
    s.finish()
    l128, r128 = s.compute_group_ends()
out = {"group": g, "left_oracle": float(lo[0]), "left_1grp": float(lg[0]), "left_128grp": float(l128[g]),
       "right_rel": float(abs(rg[0] - ro[0]) / abs(ro[0])), "left_rel": float(abs(lg[0] - lo[0]) / abs(lo[0])),
       "ends_max_rel_to_group_max": float(np.abs(e_g - e_o).max() / np.abs(e_o).max()), "lines": []}
for i in np.nonzero(mu < 0)[0]:
    ex_o, ex_g = e_o[i, 0, 0], e_g[i, 0, 0]
    near = np.abs(e_o[i, :8, :]).max()
    d8 = np.abs(e_g[i, :8, :] - e_o[i, :8, :]).max()
    out["lines"].append({"i": int(i), "mu": float(mu[i]), "exit_oracle": float(ex_o), "exit_gpu": float(ex_g),
                         "exit_rel": float(abs(ex_g - ex_o) / max(abs(ex_o), 1e-300)),
                         "cells0_7_max": float(near), "cells0_7_err_rel": float(d8 / near),
                         "line_max": float(np.abs(e_o[i]).max())})
print(json.dumps(out), flush=True)
