"""How long the SL slab's state stays finite under the reference's BDF2 (const_B from the
full dt, solver.cpp:501, grows the state on optically thick, finely resolved lines) per dt:
advance in chunks, rt_state_finite after each.  usage: python -u tools/finite_horizon.py G
dt1,dt2 chunk total"""
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import bench  # noqa: E402
import rtsn  # noqa: E402

G = int(sys.argv[1])
dts = [float(x) for x in sys.argv[2].split(",")]
chunk, total = int(sys.argv[3]), int(sys.argv[4])
for dt in dts:
    with rtsn.Solver(dict(bench.slab_params(G, "v0"), dt=dt)) as s:
        s.time_block = 20
        done, first_bad = 0, None
        while done < total:
            s.advance(chunk)
            done += chunk
            if not s.state_finite():
                first_bad = done
                break
        print(json.dumps({"groups": G, "dt": dt, "finite_through": done if first_bad is None else done - chunk,
                          "first_nonfinite_by": first_bad}), flush=True)
