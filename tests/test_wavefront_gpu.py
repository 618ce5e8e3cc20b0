"""The short-line wavefront (kernels_wave.hip wavefront_kernel; include/rtsn.h
rt_set_wavefront): lanes over cells, every step of an advance in one launch.

Same arithmetic per (cell, level) as the pipelined segment pass -- the per-line affine map
with exact carries, the reflective mu > 0 head by its own map (rtsn_lines.hip
cell_map<S, true>, the reference's head algebra probed into the same rows) -- so its node
array must equal the pipelined schedule's BITWISE (the segment kernels are pinned to the
oracle by test_gpu_parity.py), for every scheme, boundary pair and line length around the
lane-count edges (C = 1, 2, 4, 8 cells per lane; a chain of up to 8 waves handing over
through LDS, or one wave with rt_set_wavefront_waves(1)); and through the reference's own
configurations it runs by default (rt_solve with no block or schedule chosen), which
test_gpu_parity.test_reference_configs checks against the oracle.
"""
import numpy as np
import pytest

from conftest import PRM_DIR, SEED
from parity import per_group_rel

pytestmark = pytest.mark.gpu

LENGTHS = [1, 5, 31, 32, 33, 50, 63, 64, 65, 100, 127, 128, 129, 255, 256, 257, 511, 512, 513, 1000, 2049,
           4096]


# kernels_wave.hip's tick costs (ns; profiles/r05d_chain_plan.jsonl), rows C = 1, 2, 4, 8, columns 1..8 waves
TICK_VACUUM = [[79, 141, 166, 185, 225, 248, 259, 272], [126, 194, 217, 238, 306, 343, 356, 368],
               [220, 300, 323, 341, 441, 541, 560, 579], [410, 500, 532, 555, 800, 880, 910, 943]]
TICK_REFLECTIVE = [[83, 156, 173, 191, 230, 255, 266, 278], [131, 203, 222, 244, 321, 349, 363, 388],
                   [227, 307, 330, 351, 515, 551, 570, 587], [421, 529, 559, 579, 927, 977, 1001, 1046]]


def wave_plan(N, reflective, max_waves=8):
    """kernels_wave.hip wavefront_plan: the cells per lane C (1, 2, 4, 8) whose chain of
    ceil(N / C) lanes per line (a reflective pair: both lines') fits max_waves waves with the
    least (1000 + lanes - 1) x measured tick cost at (C, waves) (x 1.3 for a reflective pair
    whose N is not a multiple of C); (0, 0) when none fits."""
    best = None
    for ci, C in enumerate((1, 2, 4, 8)):
        used = -(-N // C) * (2 if reflective else 1)
        w = -(-used // 64)
        if w > max_waves:
            continue
        cost = (1000.0 + used - 1) * (TICK_REFLECTIVE if reflective else TICK_VACUUM)[ci][w - 1]
        if reflective and N % C:
            cost *= 1.3  # the padded kernel
        if best is None or cost < best[0]:
            best = (cost, C, w)
    return (best[1], best[2]) if best else (0, 0)


def _params(oracle_mod, N, ts, bc_left, bc_right, M=6, V=5.994, dt=1e-6):
    p = oracle_mod.parse_prm(PRM_DIR / "llnl_slab_test.prm", table_dir=PRM_DIR)
    p.update(N=N, M=M, ts_method=ts, bc_left=bc_left, bc_right=bc_right, use_correction=1, V=V, dt=dt)
    p["dx"] = p["X"] / p["N"]
    p["psi_source"] = np.linspace(0.5, 2.0, M * p["G"]).reshape(M, p["G"])
    q = dict(p, bc_left_indicator=bc_left, bc_right_indicator=bc_right)
    return p, q


def _random_ends(q, lo, hi, B, seed):
    rng = np.random.default_rng(seed)
    return B[None, :, None, None] * rng.uniform(0.5, 1.5, size=(q["M"], hi - lo, q["N"], 2))


@pytest.mark.parametrize("N", LENGTHS)
@pytest.mark.parametrize("ts", [1, 2, 3])
@pytest.mark.parametrize("bc_left,bc_right", [(0, 0), (1, 1), (2, 1), (2, 0), (0, 2)])
def test_wavefront_bitwise_pipelined(rtsn_mod, oracle_mod, N, ts, bc_left, bc_right):
    """7 steps from a random state on 10 groups x 6 directions: the wavefront's node array
    equals the pipelined segment schedule's (T = 1, every segment exact) bitwise."""
    lo, hi, steps = 40, 50, 7
    p, q = _params(oracle_mod, N, ts, bc_left, bc_right)
    B = oracle_mod.OracleSolver(p, g_lo=lo, g_hi=hi).groups()["B"][lo:hi]
    ends0 = _random_ends(q, lo, hi, B, SEED + N + 7 * ts + 3 * bc_left + bc_right)
    out = {}
    for wave, maxw in ((2, 8), (2, 1), (0, 8)):
        with rtsn_mod.Solver(q, g_lo=lo, g_hi=hi) as s:
            s.wavefront = wave
            s.wavefront_waves = maxw
            if wave == 0:
                s.pipeline = 2
                s.time_block = 1
            st = s.wavefront_state()
            fits = st["cells_per_lane"] > 0
            assert (st["cells_per_lane"], st["waves"]) == wave_plan(N, bc_left == 2, maxw)
            assert st["active"] == (wave == 2 and fits)
            s.set_ends(ends0)
            s.advance(steps)
            out[(wave, maxw)] = (fits, s.ends())
    # one wave: up to 64 lanes x 8 cells (32 per line when reflective); 8 waves: 8 x that
    assert out[(2, 1)][0] == (N <= (256 if bc_left == 2 else 512))
    assert out[(2, 8)][0] == (N <= (2048 if bc_left == 2 else 4096))
    for key in ((2, 8), (2, 1)):  # (too long: the handle ran a segment schedule of its own choosing)
        if out[key][0]:
            assert np.array_equal(out[key][1], out[(0, 8)][1]), key


@pytest.mark.parametrize("N", [1, 33, 64, 100, 129, 255, 256, 512, 1000, 2000])
@pytest.mark.parametrize("ts", [1, 2, 3])
@pytest.mark.parametrize("bc_left,bc_right", [(0, 0), (2, 1), (1, 1)])
def test_wavefront_bitwise_pipelined_long(rtsn_mod, oracle_mod, N, ts, bc_left, bc_right):
    """As above for 150 steps, more than a chain's wave has lanes: the ticks between a wave's
    fill and drain (every lane at a level in [1, n)) run unmasked and take component 0 of
    the carried state from the previous tick instead of a lane shift, and the waves of a
    multi-wave chain run skewed by a block of ticks -- bitwise the pipelined schedule still
    (dt = 1e-9 keeps the reference's BDF2 finite over the run)."""
    lo, hi, steps = 40, 44, 150
    p, q = _params(oracle_mod, N, ts, bc_left, bc_right, dt=1e-9)
    B = oracle_mod.OracleSolver(p, g_lo=lo, g_hi=hi).groups()["B"][lo:hi]
    ends0 = _random_ends(q, lo, hi, B, SEED + 3 * N + 11 * ts + 5 * bc_left + bc_right)
    out = {}
    for wave in (2, 0):
        with rtsn_mod.Solver(q, g_lo=lo, g_hi=hi) as s:
            s.wavefront = wave
            if wave == 0:
                s.pipeline = 2
                s.time_block = 1
            fits = s.wavefront_state()["cells_per_lane"] > 0
            s.set_ends(ends0)
            s.advance(steps)
            out[wave] = s.ends()
    if fits:
        assert np.isfinite(out[0]).all()
        assert np.array_equal(out[2], out[0])


@pytest.mark.parametrize("ts", [1, 3])
def test_wavefront_oracle_and_default(rtsn_mod, oracle_mod, ts):
    """llnl_slab_test's geometry (M = 2, 124 groups, N = 50) but reflective on the left and
    40 steps: the default handle takes the wavefront (nothing chosen), matches the oracle
    to 1e-10 per group; choosing a time block or a schedule turns it off."""
    p, q = _params(oracle_mod, 50, ts, 2, 1, M=2, dt=1e-4)
    p["max_timesteps"] = q["max_timesteps"] = 40
    orc = oracle_mod.OracleSolver(p)
    orc.solve()
    with rtsn_mod.Solver(q) as s:
        C, w = wave_plan(50, True)
        assert s.wavefront_state() == {"mode": 1, "active": True, "cells_per_lane": C, "waves": w}
        s.solve()
        assert per_group_rel(s.psi(), orc.psi(), 1) <= 1e-10
        assert per_group_rel(s.ends(), orc.ends(), 1) <= 1e-10
    with rtsn_mod.Solver(q) as s:
        s.time_block = 4
        assert not s.wavefront_state()["active"]
    with rtsn_mod.Solver(q) as s:
        s.pipeline = 1
        assert not s.wavefront_state()["active"]
        s.wavefront = 2
        assert s.wavefront_state()["active"]


def test_wavefront_long_advance_chunks(rtsn_mod, oracle_mod):
    """An advance longer than one launch's 65536 steps runs in chunks: 70000 BE steps of a
    tiny slab equal 7 x 10000 and the segment schedule's aligned passes (one segment: exact)."""
    p, q = _params(oracle_mod, 8, 1, 2, 1, M=2, V=0.0, dt=1e-6)
    q["G"] = 1
    q["group_bounds"] = None
    q["group_kappa"] = None
    q["psi_source"] = np.full((2, 1), 0.7)
    res = []
    for mode in ("one", "chunks", "segments"):
        with rtsn_mod.Solver(q) as s:
            if mode == "segments":
                s.wavefront = 0
                s.pipeline = 0
                s.time_block = 4
                assert s.sweep_geometry()[1] == 1
            else:
                assert s.wavefront_state()["active"]
            for n in ([70000] if mode != "chunks" else [10000] * 7):
                s.advance(n)
            res.append(s.ends())
    assert np.array_equal(res[0], res[1])
    assert np.array_equal(res[0], res[2])


@pytest.mark.parametrize("N,bc_left", [(50, 0), (300, 2), (1000, 0)])
def test_wavefront_deferred_small_advances(rtsn_mod, oracle_mod, N, bc_left):
    """Advances shorter than 8 x the chain's fill stay queued (pipeline_state's queued steps)
    and run as one launch when they reach it or at a read-out: 2-9-step advances with
    read-outs in between, and a switch to the segment schedule with steps still queued,
    equal one advance of all the steps bitwise (BDF2, 150 steps, random state)."""
    lo, hi, steps = 40, 44, 150
    p, q = _params(oracle_mod, N, 3, bc_left, 1, dt=1e-9)
    B = oracle_mod.OracleSolver(p, g_lo=lo, g_hi=hi).groups()["B"][lo:hi]
    ends0 = _random_ends(q, lo, hi, B, SEED + 17 * N)
    with rtsn_mod.Solver(q, g_lo=lo, g_hi=hi) as s:
        assert s.wavefront_state()["active"]
        s.set_ends(ends0)
        s.advance(steps)
        ref = s.ends()
    chunks = [2, 9, 5, 3, 8, 4, 7, 6] * 4
    with rtsn_mod.Solver(q, g_lo=lo, g_hi=hi) as s:
        s.set_ends(ends0)
        done, mids = 0, 0
        for i, n in enumerate(chunks):
            n = min(n, steps - done)
            if n <= 0:
                break
            s.advance(n)
            done += n
            if i == 0:
                assert s.pipeline_state()["queued_steps"] == n  # deferred
            if i in (5, 13):
                s.ends()  # a read-out runs what is queued
                assert s.pipeline_state()["queued_steps"] == 0
                mids += 1
            if i == 20:  # switch schedules with steps queued: they run first, on the wavefront
                s.wavefront = 0
                s.pipeline = 2
                s.time_block = 1
        if done < steps:
            s.advance(steps - done)
        assert np.array_equal(s.ends(), ref)


@pytest.mark.parametrize("N,bc_left", [(300, 0), (300, 2), (700, 0), (129, 2), (1000, 1)])
@pytest.mark.parametrize("ts", [2, 3])
def test_wavefront_cells_choice_bitwise(rtsn_mod, oracle_mod, N, bc_left, ts):
    """rt_set_wavefront_cells: every cells-per-lane choice (one wave, or chains of 2-8 waves;
    a choice past the wave cap falls back to the plan's) runs the same arithmetic per (cell,
    level): the node arrays after 40 steps from a random state are bitwise equal."""
    p, q = _params(oracle_mod, N, ts, bc_left, 1 if bc_left == 2 else bc_left)
    lo, hi = 20, 26
    B = oracle_mod.OracleSolver(p, g_lo=lo, g_hi=hi).groups()["B"][lo:hi]
    ends0 = _random_ends(q, lo, hi, B, 77 + N + ts)
    out, seen = [], set()
    for C in (0, 1, 2, 4, 8):
        with rtsn_mod.Solver(q, g_lo=lo, g_hi=hi) as s:
            s.wavefront = 2
            s.set_wavefront_cells(C)
            st = s.wavefront_state()
            assert st["active"]
            seen.add((st["cells_per_lane"], st["waves"]))
            s.set_ends(ends0)
            s.advance(40)
            out.append(s.ends())
    assert len(seen) >= 2
    for o in out[1:]:
        assert np.array_equal(out[0], o)
