"""Material-temperature coupling on the GPU (rt_material_*) against the oracle.

The device Planck kernel (planck_cells_kernel) against the oracle's long
double restatement; the coupled sweep (sweep_block_kernel<S,1,0,true>, the
per-cell emission scaling the map constants) + T update against
orc_material_*; energy conservation of the BE coupling on the device; group
shards summing q (two handles on one GPU; two ranks over gloo sharing it,
through rtsn.coupling.coupled_steps).

Tolerances: T(x) relative 1e-12 and the transport fields per group 1e-10
(the north_star's 1e-10 for intensities); the device evaluates the Planck
integrals in double (the oracle in the reference's long double Gauss nodes,
glibc exp per series term; the device one exp and a running product), so B_g
agrees to 1e-12 relative plus 1e-14 a c T^4 absolute -- the series difference
s(z1) - s(z2) of the reference's algorithm cancels in narrow groups, leaving a
few ulps of a c T^4 -- and the last group, a remainder a c T^4 - (rest), to
1e-13 a c T^4.
"""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest

from conftest import PRM_DIR, REPO
from parity import per_group_rel
from test_material import C_LIGHT, params, t_profile

pytestmark = pytest.mark.gpu


def to_rt(p: dict) -> dict:
    q = dict(p)
    q["bc_left_indicator"] = p["bc_left"]
    q["bc_right_indicator"] = p["bc_right"]
    return q


def grey(T):
    """kcon x rad_a_long c T^4 = sum_g B_g(T) (Planck.cpp:79-83)."""
    import oracle
    return oracle.planck_cell(T, np.array([0.0, 1.0]), 0) if T > 0 else 0.0


def check_planck(gpu_B, orc_B, T):
    """gpu_B, orc_B: (G, N) at T (N)."""
    G = gpu_B.shape[0]
    acT4 = np.array([grey(t) for t in T])
    d = np.abs(gpu_B - orc_B)
    # the series difference s(z1) - s(z2) cancels in narrow groups: its rounding is
    # a few ulps of a c T^4, whatever the group's size (hence the absolute term)
    lim = 1e-12 * np.abs(orc_B[:-1]) + 1e-14 * acT4[None, :]
    assert np.all(d[:-1] <= lim), float(np.max(d[:-1] / np.maximum(lim, 1e-300)))
    assert np.all(d[-1] <= 1e-13 * acT4 + 1e-300), float(np.max(d[-1] / np.maximum(acT4, 1e-300)))
    rel = d[:-1] / np.maximum(np.abs(orc_B[:-1]), 1e-300)
    return float(np.max(np.where(np.abs(orc_B[:-1]) > 1e-200, rel, 0.0))), G


@pytest.mark.parametrize("grid", ["log", "llnl"])
def test_device_planck_matches_oracle(rtsn_mod, oracle_mod, grid):
    N = 257
    T = np.geomspace(1e-3, 50.0, N)
    T[:4] = [0.0, -1.0, 1e-8, 1.0]
    if grid == "llnl":
        p = oracle_mod.parse_prm(PRM_DIR / "llnl_slab_test.prm", table_dir=PRM_DIR)
        p.update(N=N, max_timesteps=1)
        p["dx"] = p["X"] / N
    else:
        p = params(oracle_mod, G=64, N=N, efirst=1e-3, elast=30.0)
    orc = oracle_mod.OracleSolver(p)
    orc.material_enable(1.0, T)
    with rtsn_mod.Solver(to_rt(p)) as gpu:
        gpu.material_enable(1.0, T)
        B = gpu.cell_planck()
    ref = orc.cell_planck()
    assert np.all(B[:, :2] == 0.0)  # T = 0 and T < 0 emit nothing
    check_planck(B, ref, T)


def test_device_planck_uniform_matches_host_table(rtsn_mod, oracle_mod):
    p = oracle_mod.parse_prm(PRM_DIR / "llnl_slab_test.prm", table_dir=PRM_DIR)
    with rtsn_mod.Solver(to_rt(p)) as gpu:
        table = gpu.groups()["B"]  # host Planck (long double, rt_planck_groups' algorithm)
        gpu.material_enable(1.0)
        B = gpu.cell_planck()
    assert np.all(B == B[:, :1])
    check_planck(B[:, :1], table[:, None], np.array([1.0]))


def run_pair(rtsn_mod, oracle_mod, p, steps, rho_cv=5.0, T0=None, g_lo=0, g_hi=0, wgs_per_cu=0):
    """wgs_per_cu > 0: the coupled pass's segments sized by rt_set_segmentation."""
    T0 = t_profile(p["N"]) if T0 is None else T0
    orc = oracle_mod.OracleSolver(p, g_lo=g_lo, g_hi=g_hi)
    orc.material_enable(rho_cv, T0)
    orc.material_step(steps)
    gpu = rtsn_mod.Solver(to_rt(p), g_lo=g_lo, g_hi=g_hi)
    if wgs_per_cu:
        gpu.set_segmentation(wgs_per_cu)
    gpu.material_enable(rho_cv, T0)
    for _ in range(steps):  # a shard's own q, as the oracle shard does
        gpu.material_sweep()
        gpu.material_update()
    return gpu, orc


def planck_rel(a, b, T, last):
    """Per group max|a - b| over its max|b| -- with check_planck's absolute floor: groups
    fainter than 1e-4 of the hottest cell's a c T^4 are measured against that (1e-14 a c T^4
    at 1e-10: the series difference of narrow or far-tail groups), the remainder group (last:
    the handle holds group G-1) against 1e-3 of it (1e-13 a c T^4: a c T^4 minus the rest
    cancels where the remainder is a small share)."""
    acT4 = max([grey(t) for t in np.asarray(T)] + [0.0])
    floor = np.full(a.shape[0], 1e-4 * acT4)
    if last:
        floor[-1] = 1e-3 * acT4
    num = np.abs(a - b).max(axis=1)
    den = np.maximum(np.abs(b).max(axis=1), floor)
    return float(np.max(np.where(den > 0, num / np.where(den > 0, den, 1.0), num)))


def compare(gpu, orc, tol=1e-10):
    """T(x) to 1e-12; the fields, B_g(T), the next emission Beff (B plus the owed share: the
    device's dB/dT against the oracle's) and the owed energy per group to tol."""
    err = {"T": float(np.max(np.abs(gpu.temperature() - orc.temperature()) / np.abs(orc.temperature()))),
           "psi": per_group_rel(gpu.psi(), orc.psi(), 1),
           "ends": per_group_rel(gpu.ends(), orc.ends(), 1),
           "phi": per_group_rel(gpu.moments()[0], orc.moments()[0], 0),
           "B": planck_rel(gpu.cell_planck(), orc.cell_planck(), orc.temperature(), orc.g_lo + orc.Gl == orc.G),
           "Beff": planck_rel(gpu.cell_emission(), orc.cell_emission(), orc.temperature(), orc.g_lo + orc.Gl == orc.G)}
    tr_g, tr_o = gpu.material_transit(), orc.material_transit()
    scale = max(float(np.abs(tr_o).max()), 1e-300)
    err["transit"] = float(np.abs(tr_g - tr_o).max() / scale) if np.abs(tr_o).max() > 0 else float(np.abs(tr_g).max())
    assert err["T"] <= 1e-12, err
    for k in ("psi", "ends", "phi", "B", "Beff", "transit"):
        assert err[k] <= tol, err
    return err


@pytest.mark.parametrize("M", [6, 8, 2])
@pytest.mark.parametrize("ts,dt", [(1, 1e-3), (2, 1e-3), (3, 1e-4)])
@pytest.mark.parametrize("bc_left,bc_right", [(2, 0), (1, 1), (0, 0), (2, 1)])
def test_coupled_steps_match_oracle(rtsn_mod, oracle_mod, ts, dt, bc_left, bc_right, M):
    """M = 8, 2: the angular sums fused into the pass (M/2 divides 64) with the
    correction pending; M = 6: finalize + moments_kernel after each pass."""
    p = params(oracle_mod, ts=ts, dt=dt, M=M, G=5, N=150, bc_left=bc_left, bc_right=bc_right)
    p["psi_source"] = np.linspace(0.5, 2.0, p["M"] * p["G"]).reshape(p["M"], p["G"])
    gpu, orc = run_pair(rtsn_mod, oracle_mod, p, 6)
    with gpu:
        compare(gpu, orc)


@pytest.mark.parametrize("kappa", [0.1, 10.0, 1e3])
@pytest.mark.parametrize("T_rad,T_mat", [(50.0, 55.0), (1.0, 50.0)])
def test_stiff_coupling_matches_oracle(rtsn_mod, oracle_mod, kappa, T_rad, T_mat):
    """the coupling at realistic temperatures -- material at ~50 keV, radiation
    in equilibrium with it or at 1 keV, emission stiffness up to ~1e8 (the explicit emission of
    rounds 1-5 diverged above ~2; its stability warning is gone) -- 12 BE steps on the device
    against the oracle (T, psi, B, Beff with the owed emission, the owed energy), and the
    device's total energy (radiation + material + owed) balancing the boundary outflow."""
    from test_material import net_outflow, total_energy
    p = params(oracle_mod, ts=1, G=6, N=200, M=8, bc_left=0, bc_right=0, kappa=kappa, dt=1e-3, T=T_rad,
               efirst=0.1, elast=100.0)
    p["psi_source"] = np.zeros((p["M"], p["G"]))
    T0 = T_mat * (1.0 + 0.1 * np.sin(2 * np.pi * (np.arange(p["N"]) + 0.5) / p["N"]))
    gpu, orc = run_pair(rtsn_mod, oracle_mod, p, 12, rho_cv=1.0, T0=T0)
    with gpu:
        assert gpu.material_stability() > 1.0 or kappa < 1.0
        compare(gpu, orc)
        T = gpu.temperature()
        assert np.isfinite(T).all() and (T > 0).all() and (gpu.cell_emission() >= 0).all()
        e0 = total_energy(gpu, p, 1.0)
        gpu.material_step(1)
        resid = (total_energy(gpu, p, 1.0) - e0) + p["dt"] * net_outflow(GpuView(gpu), p)
        assert abs(resid) <= 1e-12 * abs(e0), (resid, e0)


@pytest.mark.parametrize("rho_cv,kappa", [(0.63, 32.0), (0.04, 5.0), (0.013, 83.0)])
def test_far_from_equilibrium_cells_match_oracle(rtsn_mod, oracle_mod, rho_cv, kappa):
    """Cells at 0.35-28 keV at random, small heat capacity (test_material's
    test_far_from_equilibrium_cells_stay_bounded): the cells whose linearised update would
    heat them by more than a quarter solve the full emission over all groups on the device
    (material_update_kernel's Newton) -- where the linear update diverged to inf within four
    steps -- against the oracle's solve, and the device's energy balance each step."""
    from test_material import net_outflow, total_energy
    p = params(oracle_mod, ts=1, G=10, N=42, M=2, bc_left=2, bc_right=1, kappa=kappa, dt=1.3e-4, T=1.5,
               efirst=0.35, elast=11.5)
    rng = np.random.default_rng(5)
    p["psi_source"] = rng.uniform(0.0, 2.0, size=(p["M"], p["G"]))
    T0 = 10.0 ** rng.uniform(np.log10(0.35), np.log10(28.0), size=p["N"])
    gpu, orc = run_pair(rtsn_mod, oracle_mod, p, 8, rho_cv=rho_cv, T0=T0)
    with gpu:
        compare(gpu, orc)
        T = gpu.temperature()
        assert np.isfinite(T).all() and (T > 0).all() and T.max() <= T0.max()
        e0 = total_energy(gpu, p, rho_cv)
        gpu.material_step(1)
        resid = (total_energy(gpu, p, rho_cv) - e0) + p["dt"] * net_outflow(GpuView(gpu), p)
        assert abs(resid) <= 1e-11 * abs(e0), (resid, e0)


@pytest.mark.parametrize("ts", [1, 2])
def test_coupled_long_lines_llnl_groups(rtsn_mod, oracle_mod, ts):
    """20k-cell lines in many segments (fold + finalize of every coupled pass),
    reflective left boundary, LL opacities (up to 1e6) on groups 10..26.  (The
    reference's BDF2 grows ~30x per step at these opacities, DESIGN.md §4, so
    BE and CN here; BDF2 is covered on the small configurations.)"""
    p = oracle_mod.parse_prm(PRM_DIR / "llnl_slab_test.prm", table_dir=PRM_DIR)
    p.update(N=20000, M=4, bc_left=2, dt=1e-5, max_timesteps=1, ts_method=ts)
    p["dx"] = p["X"] / p["N"]
    p["psi_source"] = np.zeros((p["M"], p["G"]))
    gpu, orc = run_pair(rtsn_mod, oracle_mod, p, 3, rho_cv=0.5, T0=t_profile(p["N"], 0.5, 1.5), g_lo=10, g_hi=26)
    with gpu:
        compare(gpu, orc)


@pytest.mark.parametrize("ts", [1, 2])
@pytest.mark.parametrize("M,bc_left,waves", [(64, 0, 1), (64, 2, 1), (16, 1, 2), (8, 2, 0)])
def test_be_correction_closed_form(rtsn_mod, oracle_mod, M, bc_left, waves, ts):
    """BE and CN: the correction's share in closed form (phi_correction_geo_kernel: lanes over
    cells, the live scalar's propagator by powers) against the oracle and against the
    cell-by-cell walk (rt_set_phi_correction_form 1), on 50k-cell lines in segments longer
    than a workgroup's 2048-cell range (few workgroups per CU, rt_set_segmentation -> few,
    long segments; 0 keeps the default segmentation: short segments)."""
    p = params(oracle_mod, ts=ts, dt=1e-3, M=M, G=6, N=50000, bc_left=bc_left, bc_right=0)
    p["psi_source"] = np.linspace(0.5, 2.0, M * p["G"]).reshape(M, p["G"])
    T0 = t_profile(p["N"], 0.5, 1.5)
    gpu, orc = run_pair(rtsn_mod, oracle_mod, p, 3, T0=T0, wgs_per_cu=waves)
    with gpu:
        compare(gpu, orc)
        T_geo, phi_geo = gpu.temperature(), gpu.moments()[0]
        segs = gpu.sweep_geometry()[1]
    with rtsn_mod.Solver(to_rt(p)) as walk:
        if waves:
            walk.set_segmentation(waves)
        walk.set_phi_correction_form(1)
        walk.material_enable(5.0, T0)
        assert walk.sweep_geometry()[1] == segs
        for _ in range(3):
            walk.material_sweep()
            walk.material_update()
        np.testing.assert_allclose(T_geo, walk.temperature(), rtol=1e-13)
        assert per_group_rel(phi_geo, walk.moments()[0], 0) <= 1e-12


@pytest.mark.parametrize("M,bc_left,waves", [(64, 0, 1), (64, 2, 1), (32, 1, 2), (16, 2, 0), (8, 0, 1)])
def test_bdf2_correction_rows(rtsn_mod, oracle_mod, M, bc_left, waves):
    """BDF2: the correction's share by tabulated rows b A^j (phi_correction_rows_kernel: lanes
    over cells, A^64 per 64-cell chunk) against the oracle and against the cell-by-cell walk
    (rt_set_phi_correction_form 1), on 50k-cell lines: segments longer than a workgroup's
    2048-cell range (few workgroups per CU) and short ones (0); H = 32 (two waves per group),
    16, 8, 4 lines.
    dt = 1e-6 keeps the coupled BDF2 run bounded (at 1e-4 the oracle's T goes negative)."""
    p = params(oracle_mod, ts=3, dt=1e-6, M=M, G=6, N=50000, bc_left=bc_left, bc_right=0)
    p["psi_source"] = np.linspace(0.5, 2.0, M * p["G"]).reshape(M, p["G"])
    T0 = t_profile(p["N"], 0.5, 1.5)
    gpu, orc = run_pair(rtsn_mod, oracle_mod, p, 3, rho_cv=5.0, T0=T0, wgs_per_cu=waves)
    with gpu:
        compare(gpu, orc)
        T_rows, phi_rows = gpu.temperature(), gpu.moments()[0]
        segs = gpu.sweep_geometry()[1]
    with rtsn_mod.Solver(to_rt(p)) as walk:
        if waves:
            walk.set_segmentation(waves)
        walk.set_phi_correction_form(1)
        walk.material_enable(5.0, T0)
        assert walk.sweep_geometry()[1] == segs
        for _ in range(3):
            walk.material_sweep()
            walk.material_update()
        np.testing.assert_allclose(T_rows, walk.temperature(), rtol=1e-13)
        assert per_group_rel(phi_rows, walk.moments()[0], 0) <= 1e-12


def test_backward_euler_energy_on_device(rtsn_mod, oracle_mod):
    from test_material import net_outflow, total_energy
    p = params(oracle_mod, ts=1, M=8, G=6, N=300, bc_left=2, bc_right=0)
    rho_cv = 5.0
    with rtsn_mod.Solver(to_rt(p)) as gpu:
        gpu.material_enable(rho_cv, t_profile(p["N"]))
        for _ in range(10):
            e0 = total_energy(gpu, p, rho_cv)
            gpu.material_step(1)
            e1 = total_energy(gpu, p, rho_cv)
            resid = (e1 - e0) + p["dt"] * net_outflow(GpuView(gpu), p)
            assert abs(resid) <= 1e-12 * e1, (resid, e1)


class GpuView:
    """rtsn.Solver with the oracle-named accessors net_outflow reads."""

    def __init__(self, s):
        self.s = s

    def ends(self):
        return self.s.ends()

    def quad(self):
        return self.s.quad()

    def psi_source(self):
        return self.s.psi_source()


@pytest.mark.parametrize("M", [6, 16])
def test_group_shards_on_one_gpu(rtsn_mod, oracle_mod, M):
    """Two shard handles, q summed on the device, equal one full handle."""
    import torch
    p = to_rt(params(oracle_mod, ts=2, G=7, N=200, M=M, bc_left=2))
    T0 = t_profile(p["N"])
    with rtsn_mod.Solver(p) as full:
        full.material_enable(4.0, T0)
        full.material_step(5)
        T_full, psi_full = full.temperature(), full.psi()
    shards = [rtsn_mod.Solver(p, g_lo=lo, g_hi=hi) for lo, hi in ((0, 3), (3, 7))]
    q = [torch.zeros(2 * p["N"], dtype=torch.float64, device="cuda") for _ in shards]  # [q, b]
    for s in shards:
        s.material_enable(4.0, T0)
    for _ in range(5):
        for s, qq in zip(shards, q):
            s.material_sweep(qq)
        for s in shards:
            s.synchronize()
        tot = q[0] + q[1]
        torch.cuda.synchronize()
        for s in shards:
            s.material_update(tot)
        for s in shards:
            s.synchronize()
    for s in shards:
        np.testing.assert_allclose(s.temperature(), T_full, rtol=1e-13)
    psi = np.concatenate([s.psi() for s in shards], axis=1)
    assert per_group_rel(psi, psi_full, 1) <= 1e-12
    for s in shards:
        s.close()


@pytest.mark.parametrize("pairs", [((0, 4), (4, 8)), ((0, 3), (3, 8))])
def test_direction_shards_on_one_gpu(rtsn_mod, oracle_mod, pairs):
    """Direction-pair shards (rt_create_direction_shard, the fallback for fewer groups than
    GPUs) in the coupled mode: each shard's exchange term q is its directions' share,
    summed on the device; T(x) and every direction's psi equal one full handle's (4 + 4
    pairs: the fused angular sums; 3 + 5: the finalize + moments path)."""
    import torch
    p = to_rt(params(oracle_mod, ts=2, G=7, N=200, M=16, bc_left=2))
    T0 = t_profile(p["N"])
    with rtsn_mod.Solver(p) as full:
        full.material_enable(4.0, T0)
        full.material_step(5)
        T_full, psi_full = full.temperature(), full.psi()
    shards = [rtsn_mod.Solver(p, d_lo=lo, d_hi=hi) for lo, hi in pairs]
    q = [torch.zeros(2 * p["N"], dtype=torch.float64, device="cuda") for _ in shards]  # [q, b]: b from pair 0's
    for s in shards:
        s.material_enable(4.0, T0)
    for _ in range(5):
        for s, qq in zip(shards, q):
            s.material_sweep(qq)
        for s in shards:
            s.synchronize()
        tot = q[0] + q[1]
        torch.cuda.synchronize()
        for s in shards:
            s.material_update(tot)
        for s in shards:
            s.synchronize()
    H = p["M"] // 2
    for s, (lo, hi) in zip(shards, pairs):
        np.testing.assert_allclose(s.temperature(), T_full, rtol=1e-12)
        idx = list(range(H - hi, H - lo)) + list(range(H + lo, H + hi))
        assert per_group_rel(s.psi(), psi_full[idx], 1) <= 1e-12
        s.close()


def test_coupled_steps_driver_single_rank(rtsn_mod, oracle_mod):
    """rtsn.coupling.coupled_steps (the multi-rank driver, here one rank) == rt_material_step."""
    import torch
    from rtsn.coupling import coupled_steps
    p = to_rt(params(oracle_mod, ts=3, dt=1e-4, G=5, N=100))
    out = []
    for use_driver in (False, True):
        with rtsn_mod.Solver(p) as s:
            s.material_enable(4.0, t_profile(p["N"]))
            if use_driver:
                coupled_steps(s, 4, torch.zeros(2 * p["N"], dtype=torch.float64, device="cuda"))
            else:
                s.material_step(4)
            out.append((s.temperature(), s.ends()))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, outdir):
    """One rank of the coupled run: its group shard on the (shared) GPU, q
    all-reduced over gloo on the solver's stream (RCCL needs one GPU per rank;
    the 8-GPU run uses it through the same coupled_steps)."""
    import torch
    import torch.distributed as dist
    sys.path.insert(0, str(REPO / "radiative-transfer_amd"))
    sys.path.insert(0, str(REPO / "oracle"))
    sys.path.insert(0, str(REPO / "tests"))
    import oracle
    import rtsn
    from rtsn.coupling import coupled_steps
    from test_material import params as mparams
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p = to_rt(mparams(oracle, ts=1, G=6, N=120, M=4))
        lo, hi = ((0, 2), (2, 6))[rank]
        with rtsn.Solver(p, g_lo=lo, g_hi=hi) as s:
            s.material_enable(4.0, t_profile(p["N"]))
            q = torch.zeros(2 * p["N"], dtype=torch.float64, device="cuda")
            coupled_steps(s, 5, q, world_size=world)
            np.save(os.path.join(outdir, f"T{rank}.npy"), s.temperature())
            np.save(os.path.join(outdir, f"psi{rank}.npy"), s.psi())
    finally:
        dist.destroy_process_group()


def test_two_ranks_share_gpu_coupled(tmp_path, rtsn_mod, oracle_mod):
    import torch.multiprocessing as mp
    mp.start_processes(_rank, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    T = [np.load(tmp_path / f"T{r}.npy") for r in range(2)]
    np.testing.assert_array_equal(T[0], T[1])
    p = params(oracle_mod, ts=1, G=6, N=120, M=4)
    orc = oracle_mod.OracleSolver(p)
    orc.material_enable(4.0, t_profile(p["N"]))
    orc.material_step(5)
    np.testing.assert_allclose(T[0], orc.temperature(), rtol=1e-12)
    psi = np.concatenate([np.load(tmp_path / f"psi{r}.npy") for r in range(2)], axis=1)
    assert per_group_rel(psi, orc.psi(), 1) <= 1e-10


def test_material_mode_errors(rtsn_mod, oracle_mod):
    p = to_rt(params(oracle_mod, G=4))
    with rtsn_mod.Solver(p) as s:
        for bad in (0.0, -1.0, float("nan")):
            with pytest.raises(rtsn_mod.RtError) as e:
                s.material_enable(bad)
            assert e.value.status == 8
        with pytest.raises(rtsn_mod.RtError) as e:
            s.material_sweep()
        assert e.value.status == 9
        s.material_enable(2.0)
        with pytest.raises(rtsn_mod.RtError) as e:
            s.advance(1)
        assert e.value.status == 9
    with rtsn_mod.Solver(p, g_lo=1, g_hi=3) as s:
        s.material_enable(2.0)
        with pytest.raises(rtsn_mod.RtError) as e:
            s.material_step(1)
        assert e.value.status == 9
    q = dict(p, V=2.0, use_correction=1)
    with rtsn_mod.Solver(q) as s:
        with pytest.raises(rtsn_mod.RtError) as e:
            s.material_enable(2.0)
        assert e.value.status == 3
    with rtsn_mod.Solver(p, d_lo=0, d_hi=1) as s:  # a direction-pair shard holds part of q as well
        s.material_enable(2.0)
        with pytest.raises(rtsn_mod.RtError) as e:
            s.material_step(1)
        assert e.value.status == 9


def test_material_stability_number(rtsn_mod, oracle_mod):
    """rt_material_stability = dt W sum_g rho kappa_g dB_g/dT(T_max) / rho_cv over all groups
    (W = the quadrature's weight sum, the host Planck table at the hottest cell): a shard
    reports the whole configuration's; rt_material_enable no longer warns above 2 (the T
    update is implicit in the emission) and the coupled steps run."""
    import warnings
    p = to_rt(params(oracle_mod, G=4))
    orc = oracle_mod.OracleSolver(params(oracle_mod, G=4))
    e = orc.groups()["e_edge"]
    T = np.linspace(0.5, 1.5, p["N"])
    _, dB = rtsn_mod.planck_groups(1.5, e)
    W = orc.quad()[1].sum()  # the reference's 4 pi (pi = 3.1415926546, GLQuad.cpp)
    want = p["dt"] * W * (p["rho"] * orc.groups()["kappa"] * dB).sum()
    for lo, hi in ((0, 4), (1, 3)):
        with rtsn_mod.Solver(p, g_lo=lo, g_hi=hi) as s:
            with warnings.catch_warnings():
                warnings.simplefilter("error")
                got = s.material_enable(want, T)  # number = 1
            assert got == pytest.approx(1.0, rel=1e-12)
            assert s.material_stability() == pytest.approx(1.0, rel=1e-12)
    with rtsn_mod.Solver(p) as s:
        with warnings.catch_warnings():
            warnings.simplefilter("error")
            got = s.material_enable(want / 3e4, T)
        assert got == pytest.approx(3e4, rel=1e-12)
        s.material_step(3)
        assert np.isfinite(s.temperature()).all() and (s.temperature() > 0).all()


@pytest.mark.parametrize("variant", ["v0", "corr"])
def test_bench_material_leg(rtsn_mod, variant):
    """bench.run_material for either SL variant (the corr variant's V = 5.994
    with the correction on must not reach rt_material_enable): BE steps through the one-rank
    rt_comm communicator, a finite T(x) and a stability number below 2."""
    import torch
    sys.path.insert(0, str(REPO))
    import bench
    p = bench.slab_params(8, variant, N=20000, M=8)
    comm, err = bench.open_comm(1, 0, 0)
    assert comm is not None, err
    out = bench.run_material(p, (8, 0, 8), 1, torch.device("cuda", 0), 0, 2, comm=comm, comm_error=err)
    comm.close()
    assert out["allreduce"].startswith("rt_comm_material_step")
    assert out["state_finite"] and 0.0 < out["stability_number"] < 2.0
    assert out["T_range_keV"][0] > 0.0


def test_bench_rccl_gather_check(rtsn_mod):
    """bench.rccl_gather_check (the N > 1 bench line's `rt_comm_gather`) on a one-rank
    communicator: the rt_comm gathers equal bench.gather_results' arrays bitwise."""
    import torch
    sys.path.insert(0, str(REPO))
    import bench
    p = dict(bench.slab_params(12, "v0", N=3000, M=8), dt=1e-9)
    dev = torch.device("cuda", 0)
    comm, err = bench.open_comm(1, 0, 0)
    assert comm is not None, err
    with rtsn_mod.Solver(p, device=0, g_lo=0, g_hi=12) as s:
        s.advance(7)
        s.finish()
        gathered = bench.gather_results(s, p["N"], 1, (12, 0, 12), None, dev)
        out = bench.rccl_gather_check(comm, s, gathered, None)
    comm.close()
    assert out["ok"] and out["bitwise"], out
