"""1000 BDF2 steps of llnl_slab_test at T = 40 (the block rt_solve picks), for a kernel trace."""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import rtsn  # noqa: E402

pdir = REPO / "tests" / "golden" / "prm"
ph = rtsn.ParameterHandler(pdir / "llnl_slab_test.prm", table_dir=str(pdir) + "/")
with rtsn.Solver(dict(ph.params, max_timesteps=1000)) as s:
    s.time_block = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    for _ in range(3):
        s.advance(1000)
        s.finish()
        s.synchronize()
    print("dims", s.M, s.G, s.N, "block", s.time_block, "level_waves", s.level_waves, flush=True)
