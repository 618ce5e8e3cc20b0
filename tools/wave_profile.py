"""One reference configuration's 1000-step wavefront advance, for rocprofv3 (kernel trace /
PMC of wavefront_kernel): python tools/wave_profile.py <prm name> [steps]."""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "radiative-transfer_amd")]
import rtsn  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "multi_group_equilibrium.prm"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
pdir = REPO / "tests" / "golden" / "prm"
q = rtsn.ParameterHandler(pdir / name, table_dir=str(pdir) + "/").params
for rep in range(3):
    with rtsn.Solver(q) as s:
        st = s.wavefront_state()
        s.advance(steps)
        s.finish()
        s.synchronize()
print(name, st, flush=True)
