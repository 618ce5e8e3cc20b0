"""GPU parity on seeded random configurations: the grids of test_gpu_parity.py, test_schedule_gpu.py
and test_wavefront_gpu.py cover each axis on its own; here every case draws all of them at once --
M, G, N (1 .. 5000 cells, log-uniform), ts_method, the boundary pair, the v/c correction, dt, the
run length, a random psi_source table, and the schedule the handle is left to choose or is forced
to (time block, pipelined / aligned, wavefront on / off, segmentation) -- and the run is read out
in one piece or advanced in random chunks with read-outs between.  Every field against the oracle
(tests/test_gpu_parity.compare_all, 1e-10 per group).  Work per case is capped so the oracle
finishes in about a second."""
import numpy as np
import pytest

from test_gpu_parity import compare_all, load, to_rt

pytestmark = pytest.mark.gpu

BC_PAIRS = [(0, 0), (1, 1), (2, 1), (2, 0), (1, 2), (0, 1), (2, 2)]


def _case(oracle_mod, seed):
    rng = np.random.default_rng(31000 + seed)
    M = int(rng.choice([2, 4, 6, 8, 12, 16, 32]))
    G = int(rng.integers(1, 13))
    N = int(np.exp(rng.uniform(0.0, np.log(5000.0))))
    steps = int(rng.integers(1, 41))
    while M * G * N * steps > 4e6 and steps > 1:  # the oracle's share: ~1 s
        steps = max(1, steps // 2)
    while M * G * N * steps > 4e6 and N > 1:
        N //= 2
    ts = int(rng.integers(1, 4))
    bc_left, bc_right = BC_PAIRS[int(rng.integers(len(BC_PAIRS)))]
    corr = bool(rng.random() < 0.5)
    p = load(oracle_mod, "template.prm", M=M, G=G, N=N, ts_method=ts, bc_left=bc_left, bc_right=bc_right,
             max_timesteps=steps, V=float(rng.choice([0.0, 1.0, 5.994])) if corr else 0.0,
             use_correction=int(corr), dt=float(10.0 ** rng.uniform(-7, -5)))
    p["dx"] = p["X"] / p["N"]
    p["psi_source"] = rng.uniform(0.2, 3.0, size=(M, G))
    sched = {}
    if rng.random() < 0.5:
        sched["time_block"] = int(rng.choice([1, 2, 3, 4, 8, 10, 16, 20]))
        sched["pipeline"] = int(rng.integers(0, 3))
    if rng.random() < 0.3:
        sched["wavefront"] = 0
    if rng.random() < 0.3:
        sched["segmentation"] = int(rng.choice([1, 4, 16]))
    chunks = None
    if rng.random() < 0.4 and steps > 1:
        cuts = sorted(set(int(c) for c in rng.integers(1, steps, size=int(rng.integers(1, 4)))))
        chunks = [b - a for a, b in zip([0] + cuts, cuts + [steps])]
    return p, sched, chunks


@pytest.mark.parametrize("seed", range(200))
def test_random_configuration(rtsn_mod, oracle_mod, seed):
    p, sched, chunks = _case(oracle_mod, seed)
    with rtsn_mod.Solver(to_rt(p)) as gpu:
        if "time_block" in sched:
            try:
                gpu.time_block = sched["time_block"]
            except rtsn_mod.RtError:
                pytest.skip(f"time block {sched['time_block']} not offered for ts {p['ts_method']}")
            gpu.pipeline = sched["pipeline"]
        if "wavefront" in sched:
            gpu.wavefront = sched["wavefront"]
        if "segmentation" in sched:
            gpu.set_segmentation(sched["segmentation"])
        if chunks is None:
            gpu.solve()
            orc = oracle_mod.OracleSolver(p)
            orc.solve()
            compare_all(gpu, orc)
        else:
            done = 0
            for n in chunks:
                gpu.advance(n)
                done += n
                orc = oracle_mod.OracleSolver(dict(p, max_timesteps=done))
                orc.solve()
                compare_all(gpu, orc)
