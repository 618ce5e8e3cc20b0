"""Pin the CPU oracle (oracle/rt_oracle.c) against every known-answer check
the reference owns, and against an independently derived restatement.

The reference ships no golden vectors and cannot be compiled here (Eigen3 is
absent), so these are the pins:
  * GrayTest        tests/test_gray.cpp:89     |max_c F| < 1e-6 on single_group.prm
  * validators      correction.cpp:39-63,100-122  sum B_g = a c T^4, sum kappa B = kappa_grey a c T^4 (1e-6)
  * GLQuad          GLQuad.cpp:4-44            mu symmetric, weights sum to 4 pi (pi = 3.1415926546)
  * Planck          Planck.cpp:85-229          group integrals vs adaptive quadrature of the Planck function
  * Eigen 2x2 solve (solver.cpp:348-349)       PartialPivLU inverse vs numpy
  * solver.cpp:733  per-cell `half_ends = ends` copy == the single surviving copy (bitwise)
  * oracle/fused_np.py (upwind frame, time-fused) == oracle (1e-13) on every config / scheme / BC
"""
import numpy as np
import pytest
from scipy import integrate

import fused_np
from conftest import PRM_DIR
from parity import per_group_rel

CONFIGS = ["single_group.prm", "multi_group_equilibrium.prm", "llnl_slab_test.prm",
           "llnl_slab_test_uncapped.prm", "default.prm", "template.prm"]
PI = 3.1415926546
A_RAD, C_LIGHT = 1.3653104e-2, 299.79245800


def load(oracle_mod, name, **over):
    p = oracle_mod.parse_prm(PRM_DIR / name, table_dir=PRM_DIR)
    p.update(over)
    return p


def test_gray_test_known_answer(oracle_mod):
    """GrayTest: equilibrium single group, reflective left / source right."""
    s = oracle_mod.OracleSolver(load(oracle_mod, "single_group.prm"))
    s.solve()
    phi, F, _ = s.moments()
    assert abs(F.max()) < 1e-6
    # the gray equilibrium keeps psi at B = a c T^4 (jk/cm^2/sh)
    np.testing.assert_allclose(s.psi(), s.groups()["B"][0], rtol=1e-6)


@pytest.mark.parametrize("name,ok", [("single_group.prm", True), ("multi_group_equilibrium.prm", True),
                                     ("default.prm", True), ("template.prm", True),
                                     ("llnl_slab_test.prm", False)])
def test_validate_correction(oracle_mod, name, ok):
    """Grey opacities satisfy both validators; tabulated opacities fail the
    emission check -- the reason llnl_slab_test.prm:54 turns validation off."""
    s = oracle_mod.OracleSolver(load(oracle_mod, name))
    assert s.validate() == ok
    g = s.groups()
    assert abs(g["B"].sum() - A_RAD * C_LIGHT * s.params["T"] ** 4) < 1e-6


def test_validation_failure_is_reported(oracle_mod):
    p = load(oracle_mod, "llnl_slab_test.prm", include_validation=1)
    s = oracle_mod.OracleSolver(p)
    with pytest.raises(oracle_mod.OracleError, match="validation"):
        s.solve()


@pytest.mark.parametrize("M", [2, 4, 8, 16, 64])
def test_glquad(oracle_mod, M):
    mu, wt = oracle_mod.glquad(M)
    assert np.all(np.diff(mu) > 0)
    np.testing.assert_allclose(mu, -mu[::-1], atol=1e-15)
    # Newton stops at |dz| <= 1e-12 (GLQuad.h:11), so nodes/weights are good to ~1e-11
    assert abs(wt.sum() - 4 * PI) < 1e-10
    x, w = np.polynomial.legendre.leggauss(M)
    np.testing.assert_allclose(mu, x, atol=1e-11)
    np.testing.assert_allclose(wt, w * 2 * PI, rtol=1e-10)
    if M == 2:
        np.testing.assert_allclose(mu, [-1 / np.sqrt(3), 1 / np.sqrt(3)], rtol=1e-15)


def _planck_B(E, T):
    h, c = 4.141895e-10, C_LIGHT
    return 2.0 * E ** 3 / (h ** 3 * c ** 2) / np.expm1(E / T)


def _planck_dBdT(E, T):
    h, c = 4.141895e-10, C_LIGHT
    x = E / T
    return 2.0 * E ** 4 / (h ** 3 * c ** 2 * T ** 2) * np.exp(x) / np.expm1(x) ** 2


@pytest.mark.parametrize("T", [0.5, 1.0, 2.0])
def test_planck_group_integrals(oracle_mod, T):
    """Gauss (z<0.7), series (z>0.5) and split branches against adaptive quadrature."""
    edges = np.array([1e-3, 0.05, 0.3, 0.55, 0.62, 0.8, 1.5, 4.0, 12.0, 30.0]) * T
    B, dB = oracle_mod.planck_groups(T, edges[:-1], edges[1:])
    for g in range(len(edges) - 2):  # the last group is the remainder
        ref = integrate.quad(_planck_B, edges[g], edges[g + 1], args=(T,), epsabs=0, epsrel=1e-13, limit=200)[0]
        refd = integrate.quad(_planck_dBdT, edges[g], edges[g + 1], args=(T,), epsabs=0, epsrel=1e-13, limit=200)[0]
        assert B[g] == pytest.approx(4 * PI * ref, rel=1e-10)
        assert dB[g] == pytest.approx(4 * PI * refd, rel=1e-10)
    # remainder group: grey total minus the others
    a_long = 8.0 * PI ** 5 / (15.0 * 4.141895e-10 ** 3 * C_LIGHT ** 3)
    tail = integrate.quad(_planck_B, edges[-2], np.inf, args=(T,), epsabs=0, epsrel=1e-12)[0] * 4 * PI
    head = integrate.quad(_planck_B, 0, edges[0], args=(T,), epsabs=0, epsrel=1e-12)[0] * 4 * PI
    assert B[-1] == pytest.approx(tail + head, rel=1e-6)
    assert B.sum() == pytest.approx(a_long * C_LIGHT * T ** 4, rel=1e-14)


def test_eigen_inverse2(oracle_mod):
    rng = np.random.default_rng(20261015)
    for _ in range(200):
        m = rng.normal(size=(2, 2)) * rng.choice([1e-6, 1.0, 1e6])
        inv = oracle_mod.eigen_inverse2(m)
        np.testing.assert_allclose(inv, np.linalg.inv(m), rtol=1e-12, atol=1e-12 * np.abs(np.linalg.inv(m)).max())


@pytest.mark.parametrize("name", ["single_group.prm", "llnl_slab_test.prm", "template.prm"])
def test_half_copy_literal_equals_lazy(oracle_mod, name):
    p = load(oracle_mod, name, max_timesteps=2)
    a = oracle_mod.OracleSolver(p, half_copy_literal=True)
    b = oracle_mod.OracleSolver(p, half_copy_literal=False)
    a.solve()
    b.solve()
    assert np.array_equal(a.ends(), b.ends())


@pytest.mark.parametrize("name", CONFIGS)
@pytest.mark.parametrize("ts", [1, 2, 3])
@pytest.mark.parametrize("bc_left", [0, 1, 2])
def test_fused_restatement_matches_oracle(oracle_mod, name, ts, bc_left):
    p = load(oracle_mod, name, ts_method=ts, bc_left=bc_left)
    p["max_timesteps"] = min(p["max_timesteps"], 3)
    s = oracle_mod.OracleSolver(p)
    s.solve()
    g = s.groups()
    cc = s.correction_coeffs()
    mu, _ = s.quad()
    f = fused_np.FusedSolver(p, mu, g["B"], g["kappa"], cc["cor1"], cc["cor2"], cc["cor3"], s.psi_source())
    for _ in range(p["max_timesteps"]):
        f.step()
    assert per_group_rel(f.ends(), s.ends(), 1) < 1e-13


def test_group_subset_is_independent(oracle_mod):
    """Groups never couple (T is constant): a shard equals the full run's slice."""
    p = load(oracle_mod, "llnl_slab_test.prm")
    full = oracle_mod.OracleSolver(p)
    full.solve()
    part = oracle_mod.OracleSolver(p, g_lo=30, g_hi=70)
    part.solve()
    assert np.array_equal(part.ends(), full.ends()[:, 30:70])


def test_threaded_oracle_bitwise(oracle_mod):
    """orc_set_threads (the multi-core CPU baseline, and the one-group oracle runs of the
    full-size GPU check: lines of a run of same-sign directions over the threads) does not
    change any bit, reflective left BC included."""
    p = oracle_mod.parse_prm(PRM_DIR / "llnl_slab_test.prm", table_dir=PRM_DIR)
    p.update(M=8, N=200, V=5.994, bc_left=2, max_timesteps=3)
    p["psi_source"] = np.ones((8, p["G"]))
    p["dx"] = p["X"] / p["N"]
    for g_lo, g_hi in ((0, 0), (63, 64)):
        outs = []
        for threads in (1, 4):
            s = oracle_mod.OracleSolver(p, g_lo=g_lo, g_hi=g_hi)
            s.set_threads(threads)
            s.solve()
            outs.append((s.ends(), s.psi(), s.moments()))
        np.testing.assert_array_equal(outs[0][0], outs[1][0])
        np.testing.assert_array_equal(outs[0][1], outs[1][1])
        for a, b in zip(outs[0][2], outs[1][2]):
            np.testing.assert_array_equal(a, b)


def test_equilibrium_known_answer(oracle_mod):
    """SURVEY §8(c) KAT 3: multi_group_equilibrium.prm (source BCs at the
    equilibrium psi_source = B + mu beta (4B - dEB), 500 BDF2 steps) stays at
    the equilibrium profile: every psi(i, g, c) within 0.5% of psi_source(i, g).
    (compute_balance is not ~0 here: solver.cpp:258-265 takes the mu>0 inflow
    from node 1 of cell 0 and the mu<0 inflow from node 0 of cell N-1 -- we
    reproduce the formula, tests/test_gpu_parity.py compares it.)"""
    p = oracle_mod.parse_prm(PRM_DIR / "multi_group_equilibrium.prm", table_dir=PRM_DIR)
    s = oracle_mod.OracleSolver(p)
    s.solve()
    src = s.psi_source()
    dev = np.abs(s.psi() - src[:, :, None]).max(axis=2) / np.abs(src)
    assert dev.max() < 5e-3, dev


@pytest.mark.parametrize("ts", [1, 2, 3])
@pytest.mark.parametrize("bc", [(0, 0), (1, 1), (0, 2)])
def test_parallel_copies_baseline_mode_is_exact(oracle_mod, ts, bc):
    """The CPU baseline's threaded form (lines of a direction over 4 threads, the
    whole-array prev/half snapshot copies split over them) gives the same bits as the
    serial run."""
    import sys
    from conftest import REPO
    sys.path.insert(0, str(REPO))
    import bench
    oracle = oracle_mod
    p = bench.slab_params(6, "corr", N=300, M=8)
    q = dict(p, bc_left=bc[0], bc_right=bc[1], bc_left_indicator=bc[0], bc_right_indicator=bc[1], dx=p["X"] / 300,
             have_group_bounds=0, have_group_kappa=1, prm_found=1, ts_method=ts, max_timesteps=3,
             psi_source=np.full((8, 6), 0.3))
    a = oracle.OracleSolver(q)
    a.solve()
    b = oracle.OracleSolver(q)
    b.set_threads(4)
    b.set_parallel_copies(True)
    b.solve()
    assert np.array_equal(a.ends(), b.ends())
    assert np.array_equal(a.psi(), b.psi())
