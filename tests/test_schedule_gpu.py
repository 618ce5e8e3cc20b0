"""GPU parity of the run schedules on few long lines (round 4): chunked rt_advance calls,
the deferred start of the pipeline, the aligned schedule's own segmentation and the fold
with its LDS-resident propagator, the transient planned schedule, and the run's n mod T
remainder riding the pipeline's drain as a tail block.

Geometry: llnl_slab_test's material and tabulated opacities resampled to 4 groups, M = 2
(8 lines), N = 5000 or 50000 cells, dt = 1e-9 -- lines beyond the wavefront chain's 4096
cells, with few lines, where round 3 measured 1000 aligned steps at 1.4-4.5 s against
3.5-17 ms for rt_solve (profiles/archive/r03ao_solve_mid.jsonl).  Every field against the oracle
to 1e-10 per group (tests/test_gpu_parity.compare_all)."""
import numpy as np
import pytest

from conftest import PRM_DIR
from test_gpu_parity import compare_all, to_rt

pytestmark = pytest.mark.gpu


def _params(oracle_mod, N, steps, bc_left=0, bc_right=0, G=4):
    p = oracle_mod.parse_prm(PRM_DIR / "llnl_slab_test.prm", table_dir=PRM_DIR)
    p.update(N=N, G=G, group_bounds=None, group_kappa=None, dt=1e-9, max_timesteps=steps, bc_left=bc_left,
             bc_right=bc_right)
    p["dx"] = p["X"] / p["N"]
    p["psi_source"] = np.full((p["M"], G), 0.5)
    return p


def _oracle(oracle_mod, p):
    orc = oracle_mod.OracleSolver(p)
    orc.solve()
    return orc


@pytest.mark.parametrize("bc_left", [0, 2])
def test_chunked_advances_pipeline_through(rtsn_mod, oracle_mod, bc_left):
    """A run advanced in 7-step chunks with no read-out in between: the first chunks stay
    queued (no pipeline fill for a handful of steps), then the run takes rt_solve's plan for
    the .prm's length and pipelines through the remaining chunks (lag > 0 while running);
    the read-out drains it, and the handle's own schedule (time block 16) is back after."""
    steps = 420
    p = _params(oracle_mod, 5000, steps, bc_left=bc_left)
    orc = _oracle(oracle_mod, p)
    with rtsn_mod.Solver(to_rt(p)) as gpu:
        assert not gpu.wavefront_state()["active"]
        plan = gpu.plan_schedule(steps)
        gpu.advance(7)
        st = gpu.pipeline_state()
        assert st["queued_steps"] == 7 and st["lag_steps"] == 0  # deferred
        done = 7
        lagged = False
        while done < steps:
            n = min(7, steps - done)
            gpu.advance(n)
            done += n
            lagged = lagged or gpu.pipeline_state()["lag_steps"] > 0
        assert lagged, "the chunked run never pipelined"
        assert gpu.time_block == plan["time_block"]
        compare_all(gpu, orc)
        assert gpu.time_block == 16 and gpu.pipeline_state()["lag_steps"] == 0


@pytest.mark.parametrize("N", [5000, 50000])
def test_short_advances_with_readouts(rtsn_mod, oracle_mod, N):
    """Short advances each followed by a read-out run as aligned passes (the deferred steps
    at finalize) on the aligned schedule's own, coarser segmentation -- not the pipeline's
    hundreds of segments -- and the fold walks them from LDS.  The state after every
    read-out equals the oracle's at the same step."""
    chunks = [5, 9, 3, 7]
    p = _params(oracle_mod, N, sum(chunks))
    with rtsn_mod.Solver(to_rt(p)) as gpu:
        done = 0
        for n in chunks:
            gpu.advance(n)
            done += n
            orc = _oracle(oracle_mod, dict(p, max_timesteps=done))
            compare_all(gpu, orc)
        _, segs = gpu.sweep_geometry()
        assert segs <= 400, segs  # aligned_segments: ~100-200 here (the pipeline's would be 312 / 1024+)


def test_aligned_schedule_chunked_long_line(rtsn_mod, oracle_mod):
    """The aligned schedule on request (rt_set_pipeline 0): 50000 cells in chunked advances
    of 1-8 steps with the correction pending across calls, reflective left boundary (the
    mid-pass fold of the mu < 0 outflow): against the oracle."""
    chunks = [3, 8, 1, 4, 6, 2]
    p = _params(oracle_mod, 50000, sum(chunks), bc_left=2, bc_right=1)
    orc = _oracle(oracle_mod, p)
    with rtsn_mod.Solver(to_rt(p)) as gpu:
        gpu.pipeline = 0
        for n in chunks:
            gpu.advance(n)
        compare_all(gpu, orc)


def test_solve_plan_is_transient(rtsn_mod, oracle_mod):
    """rt_solve plans its run (time block, four waves per segment, segmentation) and gives
    the handle back its own schedule afterwards: the reported time block and waves per
    segment are the defaults again, and a following advance + read-out is still exact."""
    p = _params(oracle_mod, 5000, 64)
    with rtsn_mod.Solver(to_rt(p)) as gpu:
        tb0, lw0 = gpu.time_block, gpu.level_waves
        gpu.solve()
        assert (gpu.time_block, gpu.level_waves) == (tb0, lw0)
        gpu.advance(10)
        compare_all(gpu, _oracle(oracle_mod, dict(p, max_timesteps=74)))


@pytest.mark.parametrize("T,waves,steps,bc_right", [(8, 4, 100, 0), (8, 1, 99, 0), (16, 2, 37, 1), (20, 4, 47, 0),
                                                    (12, 4, 30, 1), (32, 4, 119, 0)])
def test_pipelined_tail_bitwise(rtsn_mod, oracle_mod, T, waves, steps, bc_right):
    """The pipelined run's last steps mod T as every position's final block in the drain
    (launch_split_tail: the first active position runs `tail` < T levels while the ones
    behind it run whole blocks): the node array equals the wavefront's -- the exact
    sequential order, bitwise -- from a random state (3000 cells, 4 groups, M = 6).  Tails
    of at least T / 4 steps ride the drain (the launch takes four waves, whatever the run's
    split: T = 8 on one wave here); shorter ones run as aligned passes after it."""
    from test_wavefront_gpu import _params as wparams, _random_ends
    p, q = wparams(oracle_mod, 3000, 3, 0, bc_right, dt=1e-9)
    lo, hi = 40, 44
    B = oracle_mod.OracleSolver(p, g_lo=lo, g_hi=hi).groups()["B"][lo:hi]
    ends0 = _random_ends(q, lo, hi, B, 1234 + T + steps)
    out = {}
    for wave in (2, 0):
        with rtsn_mod.Solver(q, g_lo=lo, g_hi=hi) as s:
            s.wavefront = wave
            if wave == 0:
                s.pipeline = 2
                s.time_block = T
                s.level_waves = waves
            s.set_ends(ends0)
            s.advance(steps)
            if wave == 0:
                st = s.pipeline_state()
                assert st["queued_steps"] == steps % T and st["lag_steps"] > 0  # pipelined, remainder queued
            out[wave] = s.ends()
            if wave == 0:
                assert s.pipeline_state()["queued_steps"] == 0
    assert np.isfinite(out[0]).all()
    assert np.array_equal(out[2], out[0])


def test_solve_remainder_tail(rtsn_mod, oracle_mod):
    """rt_solve of 100 steps on 50000 cells x 4 groups (the plan's block does not divide
    100): the remainder rides the drain; every field against the oracle."""
    p = _params(oracle_mod, 50000, 100)
    orc = _oracle(oracle_mod, p)
    with rtsn_mod.Solver(to_rt(p)) as gpu:
        plan = gpu.plan_schedule(100)
        assert 100 % plan["time_block"], plan
        gpu.solve()
        compare_all(gpu, orc)


@pytest.mark.parametrize("M,G,N", [(64, 128, 300), (64, 100, 257), (32, 70, 129), (16, 64, 64), (16, 3, 50),
                                   (64, 1, 17), (12, 40, 33)])
def test_moments_producer_consumer_bitwise(rtsn_mod, oracle_mod, M, G, N):
    """The moments forms (rt_set_moments_form): the producer/consumer moments_pc_kernel (the
    default) and the one-wave moments_kernel, where H = M/2 is 8, 16 or 32, are bitwise equal
    on a random state -- whole and partial 64-group
    chunks, fewer items than workgroups -- and match the oracle's sums of the same state
    (M = 12 has neither producer/consumer form: every run takes the one-wave kernel)."""
    p = oracle_mod.parse_prm(PRM_DIR / "llnl_slab_test.prm", table_dir=PRM_DIR)
    p.update(M=M, N=N, G=G, group_bounds=None, group_kappa=None, dt=1e-9, max_timesteps=1, bc_left=0, bc_right=0)
    p["dx"] = p["X"] / p["N"]
    p["psi_source"] = np.zeros((M, G))
    rng = np.random.default_rng(M * 1000 + G + N)
    ends = rng.uniform(-1.0, 2.0, size=(M, G, N, 2))
    out = []
    with rtsn_mod.Solver(to_rt(p)) as gpu:
        for form in (0, 1):
            gpu.set_moments_form(form)
            gpu.set_ends(ends)
            out.append(gpu.moments())
        gpu.set_moments_form(0)  # the setter drops the cached moments of the same state
        assert all(np.array_equal(a, b) for a, b in zip(gpu.moments(), out[0]))
        with pytest.raises(rtsn_mod.RtError):
            gpu.set_moments_form(2)
    for o in out[1:]:
        for a, b in zip(out[0], o):
            assert np.array_equal(a, b)
    orc = oracle_mod.OracleSolver(p)
    orc.set_ends(ends)
    for a, b in zip(out[1], orc.moments()):
        scale = np.maximum(np.abs(b).max(axis=1, keepdims=True), 1e-300)
        assert (np.abs(a - b) / scale).max() <= 1e-13


def test_moments_host_copy_follows_state(rtsn_mod, oracle_mod):
    """The pinned host copy of the moments (one transfer per state, every later read-out of
    the same state a host copy): read-outs interleaved with balance and group ends (their
    own small transfers), then an advance, a new ends state and a moments-form switch -- the
    moments always those of the current state (oracle; the device read-out bitwise)."""
    import torch
    p = _params(oracle_mod, 600, 12, G=4)
    with rtsn_mod.Solver(to_rt(p)) as gpu:
        for done, step in ((5, 5), (12, 7)):
            gpu.advance(step)
            orc = _oracle(oracle_mod, dict(p, max_timesteps=done))
            first = gpu.moments()
            gpu.compute_balance()
            gpu.compute_group_ends()
            again = gpu.moments()
            assert all(np.array_equal(a, b) for a, b in zip(first, again))
            for a, b in zip(again, orc.moments()):
                scale = np.maximum(np.abs(b).max(axis=1, keepdims=True), 1e-300)
                assert (np.abs(a - b) / scale).max() <= 1e-10
            dev = [torch.empty(gpu.G * gpu.N, dtype=torch.float64, device="cuda") for _ in range(3)]
            gpu.moments_device(*dev)
            torch.cuda.synchronize()
            for a, d in zip(again, dev):
                assert np.array_equal(a, d.cpu().numpy().reshape(gpu.N, gpu.G).T)
        rng = np.random.default_rng(7)
        ends = rng.uniform(0.0, 1.0, size=(p["M"], 4, 600, 2))
        gpu.set_ends(ends)
        after = gpu.moments()
        orc = oracle_mod.OracleSolver(p)
        orc.set_ends(ends)
        for a, b in zip(after, orc.moments()):
            assert (np.abs(a - b) / np.abs(b).max(axis=1, keepdims=True)).max() <= 1e-13
        gpu.set_moments_form(0)
        assert all(np.array_equal(a, b) for a, b in zip(gpu.moments(), after))


@pytest.mark.parametrize("bc_left", [0, 2])
def test_ramp_launches_cut_into_rounds(rtsn_mod, oracle_mod, bc_left):
    """Ramp launches of more positions than one round of four-wave workgroups holds (128 groups
    x S64: 128 workgroups per position, 4 positions per round on 256 CUs; reflective chains of
    2 Sg positions with 64 workgroups each, 8 per round) run as consecutive launches of at most
    a round's positions (ramp_chunk); positions never exchange data within a launch, so the
    node array equals the one-launch ramps' (level_waves 4, and 2) bitwise, through the fill
    and the drain of 10 passes -- and the default really cut its ramps: more sub-launches
    (profiled event pairs) than the P + C - 1 launches of the one-launch ramps."""
    import sys
    from conftest import REPO
    sys.path.insert(0, str(REPO))
    import bench
    p = dict(bench.slab_params(128, "v0", N=2000, M=64), dt=1e-9, bc_left_indicator=bc_left)
    rng = np.random.default_rng(5 + bc_left)
    out, launches = {}, {}
    for lw in (0, 4, 2):
        with rtsn_mod.Solver(p) as s:
            s.time_block = 20
            s.pipeline = 2
            s.set_segmentation(8)
            s.level_waves = lw
            C = s.sweep_geometry()[1] * (2 if bc_left == 2 else 1)
            assert C >= 10
            if lw == 0:
                ends = rng.uniform(0.5, 1.5, size=(64, 128, 2000, 2)) * 1e-3
            s.set_ends(ends)
            s.set_profiling(True)
            s.advance(200)
            s.finish()
            launches[lw] = s.sweep_time()[1]
            out[lw] = s.ends()
    assert np.isfinite(out[0]).all()
    assert np.array_equal(out[0], out[4]) and np.array_equal(out[0], out[2])
    assert launches[4] == launches[2] == 10 + C - 1, launches
    assert launches[0] > launches[4], launches


@pytest.mark.parametrize("bc_left", [0, 2])
def test_failed_sub_launch_resumes_exactly(rtsn_mod, bc_left):
    """a ramp launch cut into sub-launches commits each sub-launch's
    positions as it enters the stream, so a failure part-way (rt_debug_fail_launch: a
    sub-launch that returns RT_ERR_DEVICE without running) leaves the handle owing exactly the
    positions not yet launched; the next call runs those and the run ends bitwise equal to an
    undisturbed one.  Failures at the first sub-launch, at the second chunk of the first cut
    ramp launch (vacuum: k = 5 of chunks 4 + 1 is sub-launch 5; reflective: k = 9 of 8 + 1 is
    sub-launch 9) and later in the fill and the drain."""
    import sys
    from conftest import REPO
    sys.path.insert(0, str(REPO))
    import bench
    p = dict(bench.slab_params(128, "v0", N=2000, M=64), dt=1e-9, bc_left_indicator=bc_left)
    ends = np.random.default_rng(11 + bc_left).uniform(0.5, 1.5, size=(64, 128, 2000, 2)) * 1e-3

    def run(fail_after):
        with rtsn_mod.Solver(p) as s:
            s.time_block = 20
            s.pipeline = 2
            s.set_segmentation(8)
            s.set_ends(ends)
            s.set_profiling(True)  # counts the sub-launches that ran
            if fail_after is not None:
                s.debug_fail_launch(fail_after)
                with pytest.raises(rtsn_mod.RtError) as e:
                    s.advance(200)
                    s.finish()
                assert e.value.status == 6 and "pipelined launch" in str(e.value)
            else:
                s.advance(200)
            s.finish()  # resumes the interrupted launch, then drains
            assert s.pipeline_state()["lag_steps"] == 0
            return s.ends(), s.sweep_time()[1]

    want, total = run(None)
    first_cut = 5 if bc_left == 0 else 9
    assert total > first_cut + 2
    for after in (0, first_cut, total // 2, total - 1):
        got, n = run(after)
        assert n == total, (after, n, total)  # every sub-launch ran once: none repeated, none lost
        assert np.array_equal(got, want), after


def test_experiment_env_ignored(rtsn_mod, oracle_mod, monkeypatch):
    """the experiment variables of rounds 3-5 no longer change a
    handle's schedule (rt_set_* are the only way): created with RTSN_TIME_BLOCK=4,
    RTSN_WAVEFRONT=0, RTSN_WAVE_WAVES=1, RTSN_LEVEL_WAVES=4, RTSN_WAVES_PER_CU=1,
    RTSN_MOMENTS_FORM=0 and RTSN_PHI_WALK=1 in the environment, a handle reports the same
    time block, wavefront state, waves per segment and segments as one created without them
    (the library's getenv calls are listed in test_host.test_getenv_only_documented)."""
    p = _params(oracle_mod, 5000, 10)
    with rtsn_mod.Solver(to_rt(p)) as s:
        want = (s.time_block, s.level_waves, s.wavefront_state(), s.sweep_geometry())
    q = _params(oracle_mod, 300, 10)
    with rtsn_mod.Solver(to_rt(q)) as s:
        want_w = s.wavefront_state()
    for k, v in (("RTSN_TIME_BLOCK", "4"), ("RTSN_WAVEFRONT", "0"), ("RTSN_WAVE_WAVES", "1"), ("RTSN_LEVEL_WAVES", "4"),
                 ("RTSN_WAVES_PER_CU", "1"), ("RTSN_MOMENTS_FORM", "0"), ("RTSN_PHI_WALK", "1")):
        monkeypatch.setenv(k, v)
    with rtsn_mod.Solver(to_rt(p)) as s:
        assert (s.time_block, s.level_waves, s.wavefront_state(), s.sweep_geometry()) == want
    with rtsn_mod.Solver(to_rt(q)) as s:
        assert s.wavefront_state() == want_w and want_w["active"]


@pytest.mark.parametrize("bc_left", [0, 2])
def test_segmentation_bitwise(rtsn_mod, oracle_mod, bc_left):
    """Results do not depend on the segmentation (rt_set_segmentation: the segments sized for
    1, 2, 4 workgroups per CU, against the default): every segment of the pipelined schedule
    starts from its predecessor's exact exit state, so the node array is bitwise the same for
    every cut of the lines (6000 cells in ~50 to ~375 chain positions), through the fill and
    drain of 2 passes at T = 20 (vacuum and reflective chains) -- and matches the oracle."""
    steps, M, G = 40, 8, 8
    p = _params(oracle_mod, 6000, steps, bc_left=bc_left, G=G)
    p["M"] = M
    p["psi_source"] = np.full((M, G), 0.5)
    orc = _oracle(oracle_mod, p)
    ends, positions = {}, {}
    for w in (0, 1, 2, 4):
        with rtsn_mod.Solver(to_rt(p)) as gpu:
            gpu.time_block = 20
            gpu.pipeline = 2
            if w:
                gpu.set_segmentation(w)
            positions[w] = gpu.sweep_geometry()[1]
            gpu.advance(steps)
            ends[w] = gpu.ends()
            if w == 0:
                compare_all(gpu, orc)
    assert len(set(positions.values())) >= 3, positions  # the cuts really differ
    for w in (1, 2, 4):
        assert np.array_equal(ends[0], ends[w]), (w, positions)
