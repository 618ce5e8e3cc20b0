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
    shard = (0, 0)
    if G > 1 and rng.random() < 0.3:  # a group shard [g_lo, g_hi) of the configuration
        lo = int(rng.integers(0, G))
        shard = (lo, int(rng.integers(lo + 1, G + 1)))
    return p, sched, chunks, shard


@pytest.mark.parametrize("seed", range(200))
def test_random_configuration(rtsn_mod, oracle_mod, seed):
    p, sched, chunks, (g_lo, g_hi) = _case(oracle_mod, seed)
    with rtsn_mod.Solver(to_rt(p), g_lo=g_lo, g_hi=g_hi) as gpu:
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
            orc = oracle_mod.OracleSolver(p, g_lo=g_lo, g_hi=g_hi)
            orc.solve()
            compare_all(gpu, orc)
        else:
            done = 0
            for n in chunks:
                gpu.advance(n)
                done += n
                orc = oracle_mod.OracleSolver(dict(p, max_timesteps=done), g_lo=g_lo, g_hi=g_hi)
                orc.solve()
                compare_all(gpu, orc)


def _material_case(oracle_mod, seed):
    from test_material import params
    rng = np.random.default_rng(47000 + seed)
    M = int(rng.choice([2, 4, 6, 8, 16]))
    G = int(rng.integers(1, 11))
    N = int(np.exp(rng.uniform(0.0, np.log(2000.0))))
    ts = int(rng.choice([1, 1, 2, 3]))
    bc_left, bc_right = BC_PAIRS[int(rng.integers(len(BC_PAIRS)))]
    dt = float(10.0 ** rng.uniform(-5, -4 if ts == 3 else -3))
    p = params(oracle_mod, ts=ts, dt=dt, M=M, G=G, N=N, bc_left=bc_left, bc_right=bc_right,
               kappa=float(10.0 ** rng.uniform(-1, 3)), T=float(10.0 ** rng.uniform(-0.5, 1.5)),
               efirst=float(10.0 ** rng.uniform(-2, -0.3)), elast=float(10.0 ** rng.uniform(0.7, 2)))
    p["psi_source"] = rng.uniform(0.0, 2.0, size=(M, G))
    T0 = 10.0 ** rng.uniform(-0.5, 1.5, size=N)
    if rng.random() < 0.5:  # a smooth profile instead of cell-to-cell noise
        T0 = np.sort(T0) if rng.random() < 0.5 else np.full(N, float(T0[0]))
    shard = (0, 0)
    if G > 1 and rng.random() < 0.3:  # a group shard: its own q, as the oracle shard does
        lo = int(rng.integers(0, G))
        shard = (lo, int(rng.integers(lo + 1, G + 1)))
    return p, T0, float(10.0 ** rng.uniform(-2, 2)), int(rng.integers(1, 7)), int(rng.choice([0, 0, 1, 4, 16])), shard


@pytest.mark.parametrize("seed", range(60))
def test_random_material_configuration(rtsn_mod, oracle_mod, seed):
    """The material coupling on seeded random configurations: quadrature, groups, cells,
    scheme, boundaries, opacity (0.1 .. 1e3), radiation and cell temperatures (0.3 .. 30 keV,
    noisy, sorted or uniform), rho c_v (0.01 .. 100: stiffness from ~0 to ~1e6), group grid,
    dt, steps and segmentation: T, psi, B, Beff and the owed energy against the oracle
    (test_material_gpu.compare)."""
    from test_material_gpu import compare, run_pair
    p, T0, rho_cv, steps, wgs, (g_lo, g_hi) = _material_case(oracle_mod, seed)
    gpu, orc = run_pair(rtsn_mod, oracle_mod, p, steps, rho_cv=rho_cv, T0=T0, g_lo=g_lo, g_hi=g_hi, wgs_per_cu=wgs)
    with gpu:
        compare(gpu, orc)
        assert np.isfinite(gpu.temperature()).all()
