"""Material-temperature coupling (include/rtsn.h rt_material_*), CPU side.

The reference holds T constant (solver.cpp:157); SURVEY §8(f)-4 names the
T(x) update fed by the group-sum all-reduce as the next row.  Its definition
(the emission linearised implicit in T, include/rtsn.h
"material") is restated in the oracle (rt_oracle.c orc_material_*), which
these tests pin by properties the definition guarantees -- there is no
reference output to pin it against ("parity unpinned" beyond these
properties):
  * the per-cell dB_g/dT is the derivative of the per-cell B_g (central
    differences) and, at a uniform T, the reference's dBdT table
    (Planck.cpp:161-229);
  * the coupling stays finite, positive and conservative at emission
    stiffness up to ~1e8 (50 keV, thin and thick cells), where the explicit
    emission of rounds 1-5 diverged;
  * the per-cell Planck emission at a uniform T is the reference's group
    table (Planck.cpp:44-77) -- bitwise for every group but the last, whose
    remainder takes the other groups as one integral;
  * backward Euler conserves sum_x dx (sum_g phi_g / c + rho_cv T) up to the
    boundary outflow, to rounding;
  * a uniform equilibrium (psi = B_g(T), source inflow B_g) stays put;
  * material colder than the radiation heats monotonically toward it;
  * group shards whose q are summed reproduce the one-shard run (gloo,
    world_size 2, through rtsn.coupling.coupled_steps -- the product's
    multi-rank driver).
"""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest

from conftest import REPO

C_LIGHT = 299.792458
A_C = None  # a c of Constants.h:22-23, from the oracle's table below


def params(oracle_mod, ts=1, M=4, G=4, N=40, bc_left=2, bc_right=0, kappa=10.0, dt=1e-3, **over):
    p = oracle_mod.default_params()
    p.update(M=M, G=G, N=N, X=0.4, dx=0.4 / N, efirst=0.1, elast=10.0, bc_left=bc_left, bc_right=bc_right,
             use_mg_equilib=0, rho=1.0, kappa_grey=kappa, T=1.0, V=0.0, use_correction=0, ts_method=ts, dt=dt,
             max_timesteps=1, include_validation=0)
    p["psi_source"] = np.zeros((M, G))
    p.update(over)
    return p


def t_profile(N, lo=0.7, hi=1.3):
    x = (np.arange(N) + 0.5) / N
    return lo + (hi - lo) * 0.5 * (1.0 + np.sin(2.0 * np.pi * x))


def total_energy(s, p, rho_cv):
    """sum_x dx (sum_g phi_g / c + rho_cv T + the emission in transit) over the solver's
    groups and T (the transit: dt W b dT of the last update, owed to the next sweep)."""
    phi, _, _ = s.moments()
    return p["dx"] * float((phi.sum(axis=0) / C_LIGHT + rho_cv * s.temperature() + s.material_transit()).sum())


def net_outflow(s, p):
    """sum_i w_i |mu_i| (outflow node - inflow value) over lines, from the step-end ends."""
    e = s.ends()
    mu, w = s.quad()
    M, N = p["M"], p["N"]
    net = 0.0
    for i in range(M):
        if mu[i] < 0:
            out, inn = e[i, :, 0, 0], (s.psi_source()[i, :] if p["bc_right"] == 1 else 0.0)
        else:
            out = e[i, :, N - 1, 1]
            inn = e[M - 1 - i, :, 0, 0] if p["bc_left"] == 2 else s.psi_source()[i, :]
        net += w[i] * abs(mu[i]) * float(np.sum(out - inn))
    return net


def test_cell_planck_uniform_equals_group_table(oracle_mod):
    p = params(oracle_mod, G=12, efirst=0.01, elast=30.0)
    for T in (0.05, 0.3, 1.0, 4.0):
        p["T"] = T
        s = oracle_mod.OracleSolver(p)
        table = s.groups()
        e = table["e_edge"]
        s.material_enable(1.0)
        B = s.cell_planck()
        assert np.all(B == B[:, :1])  # uniform T: every cell the same
        np.testing.assert_array_equal(B[:-1, 0], table["B"][:-1])
        acT4 = table["B"].sum()
        assert abs(B[-1, 0] - table["B"][-1]) <= 1e-14 * acT4
        for g in (0, 5, 11):
            assert oracle_mod.planck_cell(T, e, g) == B[g, 0]


def test_cell_dbdt_is_derivative_of_cell_planck(oracle_mod):
    """kcon dB_g/dT per cell (orc_planck_cell_dBdT: Planck::integrate_dBdT, the last group the
    remainder 4 a c T^3 - the joint integral) against central differences of planck_cell, on
    every branch of the integral (Gauss z2 <= 0.7, series z1 >= 0.5, split), and at a
    uniform T the reference's dBdT table (Planck.cpp:161-229) bitwise but the last group."""
    e = np.array([0.0, 0.01, 0.1, 0.5, 1.0, 3.0, 10.0, 30.0])
    G = len(e) - 1
    for T in (0.05, 0.4, 1.0, 7.0, 50.0):
        h = T * 1e-5
        for g in range(G):
            d = oracle_mod.planck_cell_dBdT(T, e, g)
            fd = (oracle_mod.planck_cell(T + h, e, g) - oracle_mod.planck_cell(T - h, e, g)) / (2 * h)
            # the last group's remainder cancels against the grey total 4 a c T^3, and so does
            # its difference quotient (rounding of B_total / h): an absolute term of that scale
            grey = oracle_mod.planck_cell_dBdT(T, np.array([0.0, 30.0]), 0)
            assert abs(d - fd) <= 1e-6 * abs(fd) + 1e-9 * grey, (T, g, d, fd, grey)
    p = params(oracle_mod, G=12, efirst=0.01, elast=30.0)
    s = oracle_mod.OracleSolver(p)
    table = s.groups()
    kcon = table["B"][0] / oracle_mod.planck_groups(1.0, table["e_edge"][:-1], table["e_edge"][1:])[0][0]
    for g in range(11):
        assert oracle_mod.planck_cell_dBdT(1.0, table["e_edge"], g) == table["dBdT"][g]
    for T in (0.0, -1.0, float("nan")):
        assert oracle_mod.planck_cell_dBdT(T, e, 3) == 0.0
    assert kcon > 0


@pytest.mark.parametrize("kappa", [0.1, 10.0, 1e3])
@pytest.mark.parametrize("T_rad,T_mat", [(50.0, 55.0), (5.0, 5.5), (1.0, 50.0)])
def test_stiff_emission_stays_stable(oracle_mod, kappa, T_rad, T_mat):
    """Material at T_mat against radiation at B(T_rad), BE, vacuum boundaries, rho_cv = 1,
    dt = 1e-3: emission stiffness dt W sum sigma dB/dT / rho_cv from ~1e-1 to ~1e8 -- the
    explicit emission of rounds 1-5 diverged from ~2 on.  50 steps: T finite and > 0 in
    every cell, the emission Beff >= 0, and radiation + material + owed energy balance the
    boundary outflow to rounding every step."""
    p = params(oracle_mod, ts=1, G=6, N=40, bc_left=0, bc_right=0, kappa=kappa, dt=1e-3, T=T_rad, efirst=0.1,
               elast=100.0)
    p["psi_source"] = np.zeros((p["M"], p["G"]))
    s = oracle_mod.OracleSolver(p)
    rho_cv = 1.0
    s.material_enable(rho_cv, T_mat * (1.0 + 0.1 * np.sin(2 * np.pi * (np.arange(p["N"]) + 0.5) / p["N"])))
    for n in range(50):
        e0 = total_energy(s, p, rho_cv)
        s.material_step(1)
        e1 = total_energy(s, p, rho_cv)
        T = s.temperature()
        assert np.isfinite(T).all() and np.all(T > 0.0), (n, T.min(), T.max())
        assert np.all(s.cell_emission() >= 0.0), n
        resid = (e1 - e0) + p["dt"] * net_outflow(s, p)
        assert abs(resid) <= 1e-12 * max(abs(e0), abs(e1)), (n, resid, e0)


@pytest.mark.parametrize("rho_cv,kappa", [(0.63, 32.0), (0.04, 5.0), (0.013, 83.0)])
def test_far_from_equilibrium_cells_stay_bounded(oracle_mod, rho_cv, kappa):
    """Cells at 0.35-28 keV, cell to cell at random, small heat capacity, BE: a cold cell
    beside hot ones absorbs many times its energy in one step, where the update linearised
    about T^n overshot by 10^3 and diverged within four steps (T -> inf, found by
    tests/test_random_gpu.py).  Those cells solve the full emission (dT > T / 4): T stays
    finite, > 0 and below the hottest initial temperature, the emission >= 0, and radiation +
    material + owed energy balance the boundary outflow to rounding every step."""
    p = params(oracle_mod, ts=1, G=10, N=42, M=2, bc_left=2, bc_right=1, kappa=kappa, dt=1.3e-4, T=1.5,
               efirst=0.35, elast=11.5)
    rng = np.random.default_rng(5)
    p["psi_source"] = rng.uniform(0.0, 2.0, size=(p["M"], p["G"]))
    T0 = 10.0 ** rng.uniform(np.log10(0.35), np.log10(28.0), size=p["N"])
    s = oracle_mod.OracleSolver(p)
    s.material_enable(rho_cv, T0)
    def parts(s):  # the energy's terms by magnitude: the residual's rounding scale
        phi = s.moments()[0]
        return p["dx"] * float((np.abs(phi).sum(axis=0) / C_LIGHT + rho_cv * np.abs(s.temperature())
                                + np.abs(s.material_transit())).sum())

    for n in range(12):
        e0, m0 = total_energy(s, p, rho_cv), parts(s)
        s.material_step(1)
        e1, m1 = total_energy(s, p, rho_cv), parts(s)
        T = s.temperature()
        assert np.isfinite(T).all() and np.all(T > 0.0) and T.max() <= T0.max(), (n, T.min(), T.max())
        assert np.all(s.cell_emission() >= 0.0), n
        resid = (e1 - e0) + p["dt"] * net_outflow(s, p)
        assert abs(resid) <= 1e-12 * (m0 + m1), (n, resid, e0, m0, m1)


def test_cell_planck_edge_temperatures(oracle_mod):
    e = np.array([0.0, 0.1, 1.0, 10.0])
    for T in (0.0, -1.0, float("nan"), float("inf")):
        assert all(oracle_mod.planck_cell(T, e, g) == 0.0 for g in range(3))
    # one group: the grey total a c T^4 (kcon x rad_a_long c T^4)
    b1 = oracle_mod.planck_cell(2.0, np.array([0.0, 5.0]), 0)
    b2 = sum(oracle_mod.planck_cell(2.0, e, g) for g in range(3))
    assert b1 == pytest.approx(b2, rel=1e-14)


@pytest.mark.parametrize("bc_left,bc_right", [(2, 0), (0, 0), (1, 1), (2, 1)])
def test_backward_euler_conserves_energy(oracle_mod, bc_left, bc_right):
    p = params(oracle_mod, ts=1, bc_left=bc_left, bc_right=bc_right)
    p["psi_source"] = np.full((p["M"], p["G"]), 0.3)
    s = oracle_mod.OracleSolver(p)
    rho_cv = 5.0
    s.material_enable(rho_cv, t_profile(p["N"]))
    for _ in range(15):
        e0 = total_energy(s, p, rho_cv)
        s.material_step(1)
        e1 = total_energy(s, p, rho_cv)
        resid = (e1 - e0) + p["dt"] * net_outflow(s, p)
        assert abs(resid) <= 1e-13 * e1, (resid, e1)


@pytest.mark.parametrize("ts,dt", [(1, 1e-3), (2, 1e-3), (3, 1e-4)])
def test_uniform_equilibrium_is_stationary(oracle_mod, ts, dt):
    """psi = B_g(T) everywhere, inflow B_g (use_mg_equilib with V = 0): T and psi stay."""
    p = params(oracle_mod, ts=ts, dt=dt, bc_left=1, bc_right=1, use_mg_equilib=1)
    s = oracle_mod.OracleSolver(p)
    psi0 = s.psi()
    s.material_enable(3.0)
    s.material_step(10)
    np.testing.assert_allclose(s.temperature(), 1.0, rtol=1e-12)
    np.testing.assert_allclose(s.psi(), psi0, rtol=1e-11)


def test_cold_material_heats_toward_radiation(oracle_mod):
    """Radiation at B_g(1 keV) with inflow B_g(1), material at 0.5 keV: T rises
    monotonically and stays below the radiation temperature."""
    p = params(oracle_mod, ts=1, bc_left=1, bc_right=1, use_mg_equilib=1, kappa=20.0)
    s = oracle_mod.OracleSolver(p)
    s.material_enable(2.0, np.full(p["N"], 0.5))
    prev = s.temperature()
    for _ in range(40):
        s.material_step(1)
        T = s.temperature()
        assert np.all(T >= prev - 1e-14) and np.all(T <= 1.0 + 1e-12)
        prev = T
    assert prev.min() > 0.8


def test_material_requires_correction_off(oracle_mod):
    p = params(oracle_mod, V=2.0, use_correction=1)
    s = oracle_mod.OracleSolver(p)
    with pytest.raises(oracle_mod.OracleError):
        s.material_enable(1.0)


def test_group_shards_sum_q(oracle_mod):
    """Two group shards with q summed equal the one-shard run (up to the order of the group sum)."""
    p = params(oracle_mod, ts=1, G=6)
    T0 = t_profile(p["N"])
    full = oracle_mod.OracleSolver(p)
    full.material_enable(4.0, T0)
    parts = [oracle_mod.OracleSolver(p, g_lo=lo, g_hi=hi) for lo, hi in ((0, 2), (2, 6))]
    for s in parts:
        s.material_enable(4.0, T0)
    for _ in range(8):
        full.material_step(1)
        q = sum(s.material_sweep() for s in parts)  # [q, b]: one sum of 2N values
        for s in parts:
            s.material_update(q)
    for s in parts:
        np.testing.assert_allclose(s.temperature(), full.temperature(), rtol=1e-13)
    psi = np.concatenate([s.psi() for s in parts], axis=1)
    np.testing.assert_allclose(psi, full.psi(), rtol=1e-12, atol=1e-14 * np.abs(full.psi()).max())


# ---------------------------------------------------------------------------
# world_size 2 over gloo: rtsn.coupling.coupled_steps with an oracle stand-in
# ---------------------------------------------------------------------------
class OracleMaterialShard:
    """CPU stand-in with the two methods coupled_steps uses (the test's, never the product's)."""

    def __init__(self, orc):
        self.s = orc

    def material_sweep(self, q):
        import torch
        q.copy_(torch.from_numpy(self.s.material_sweep()))

    def material_update(self, q):
        self.s.material_update(q.numpy())


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, outdir):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, str(REPO / "oracle"))
    sys.path.insert(0, str(REPO / "radiative-transfer_amd"))
    import oracle
    from rtsn.coupling import coupled_steps

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p = params(oracle, ts=1, G=6)
        lo, hi = ((0, 3), (3, 6))[rank]
        s = oracle.OracleSolver(p, g_lo=lo, g_hi=hi)
        s.material_enable(4.0, t_profile(p["N"]))
        q = torch.zeros(2 * p["N"], dtype=torch.float64)
        coupled_steps(OracleMaterialShard(s), 6, q, world_size=world)
        np.save(os.path.join(outdir, f"T{rank}.npy"), s.temperature())
        np.save(os.path.join(outdir, f"psi{rank}.npy"), s.psi())
    finally:
        dist.destroy_process_group()


def test_two_rank_coupled_steps(tmp_path, oracle_mod):
    import torch.multiprocessing as mp
    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    T = [np.load(tmp_path / f"T{r}.npy") for r in range(2)]
    np.testing.assert_array_equal(T[0], T[1])  # every rank holds the same T(x)
    p = params(oracle_mod, ts=1, G=6)
    full = oracle_mod.OracleSolver(p)
    full.material_enable(4.0, t_profile(p["N"]))
    full.material_step(6)
    np.testing.assert_allclose(T[0], full.temperature(), rtol=1e-13)
    psi = np.concatenate([np.load(tmp_path / f"psi{r}.npy") for r in range(2)], axis=1)
    np.testing.assert_allclose(psi, full.psi(), rtol=1e-12, atol=1e-14 * np.abs(full.psi()).max())
