"""Where the end-to-end time of the reference's own .prm runs goes on the GPU (create +
solve + moments + destroy, as bench.py's reference_config times them): each phase timed
separately, best of 5 after one warm run.  usage: python -u tools/e2e_breakdown.py"""
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import rtsn  # noqa: E402

pdir = REPO / "tests" / "golden" / "prm"
for name in ("llnl_slab_test.prm", "single_group.prm", "multi_group_equilibrium.prm"):
    ph = rtsn.ParameterHandler(pdir / name, table_dir=str(pdir) + "/")
    best = {}
    for rep in range(6):
        t = {}
        t0 = time.perf_counter()
        s = rtsn.Solver(ph)
        t1 = time.perf_counter()
        s.solve()
        t2 = time.perf_counter()
        phi = s.moments()[0]
        t3 = time.perf_counter()
        s.close()
        t4 = time.perf_counter()
        t = {"create": t1 - t0, "solve": t2 - t1, "moments": t3 - t2, "destroy": t4 - t3, "total": t4 - t0}
        if rep:
            for k, v in t.items():
                best[k] = min(best.get(k, 1e9), v)
        else:
            cold = t
    print(json.dumps({"config": name, **{k: round(1e3 * v, 4) for k, v in best.items()},
                      "first_run": {k: round(1e3 * v, 4) for k, v in cold.items()}}), flush=True)
    # host-only parts of rt_create: the Planck group table (rt_planck_groups) for the .prm's groups
    if ph.params.get("group_bounds") is not None:
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            rtsn.planck_groups(ph.params["T"], ph.params["group_bounds"])
            ts.append(time.perf_counter() - t0)
        print(json.dumps({"config": name, "host_planck_ms": round(1e3 * min(ts), 4)}), flush=True)
