"""Probe: per-group group-end errors of the full-length SL pair (test_headline_kernel_full_length)."""
import sys
import numpy as np
sys.path[:0] = ["oracle", "radiative-transfer_amd", "."]
import oracle, rtsn, bench
p = bench.slab_params(128, "v0", M=4)
p["dt"] = 1e-7
kap = p["group_kappa"].copy(); kap[126] = kap[0]; p["group_kappa"] = kap
q = dict(p, bc_left=0, bc_right=0, dx=p["X"] / p["N"], have_group_bounds=0, have_group_kappa=1, prm_found=1, max_timesteps=12)
o = oracle.OracleSolver(q, g_lo=126, g_hi=128); o.set_threads(2); o.run_substeps(0, 48)
lo, ro = o.group_ends(); e_o = o.ends()
print("oracle ends", lo, ro)
for pipe, tb in ((2, 10), (0, 4), (2, 4), (2, 12), (2, 2)):
    with rtsn.Solver(p, g_lo=126, g_hi=128) as s:
        s.pipeline = pipe; s.time_block = tb
        s.advance(12)
        l, r = s.compute_group_ends()
        e = s.ends()
    d = np.abs(e - e_o)
    print(pipe, tb, "left rel", np.abs(l - lo) / np.abs(lo), "right rel", np.abs(r - ro) / np.abs(ro))
    for g in range(2):
        # worst nodes per group: where, and the value there
        k = np.unravel_index(np.argmax(d[:, g] / np.abs(e_o[:, g]).max()), d[:, g].shape)
        print("   g", g, "max abs err", d[:, g].max(), "at (i,c,node)", k, "val", e_o[:, g][k], "group max", np.abs(e_o[:, g]).max(),
              "cell0 node0 rel", (d[:, g, 0, 0] / np.abs(e_o[:, g, 0, 0])), "cellN-1 node1 rel", d[:, g, -1, 1] / np.abs(e_o[:, g, -1, 1]))
