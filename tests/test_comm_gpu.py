"""RCCL behind the C ABI (include/rtsn.h "multi-GPU", csrc/rtsn_comm.hip) on the GPU box.

The box has one GPU and RCCL refuses two ranks on one device, so the communicator runs
with one rank here: every collective then goes through ncclCommInitRank, ncclAllGather /
ncclAllReduce / ncclSend-Recv on the handle's stream and the gather assembly, and its
result must equal the single handle's own getters bitwise.  The split logic across ranks
(ragged group shards, direction shards) is covered by the world-size-2 gloo tests of the
same layouts (tests/test_distributed.py) and by the driver's multi-GPU runs.
"""
import numpy as np
import pytest

from conftest import PRM_DIR

pytestmark = pytest.mark.gpu


def _params(oracle_mod, name="llnl_slab_test.prm", **over):
    p = oracle_mod.parse_prm(PRM_DIR / name, table_dir=PRM_DIR)
    p.update(over)
    q = dict(p, bc_left_indicator=p["bc_left"], bc_right_indicator=p["bc_right"])
    return q


@pytest.fixture
def comm(rtsn_mod):
    with rtsn_mod.Comm(1, 0, rtsn_mod.Comm.unique_id(), 0) as c:
        yield c


@pytest.mark.parametrize("name", ["llnl_slab_test.prm", "multi_group_equilibrium.prm"])
def test_world_one_gathers_equal_the_handle(rtsn_mod, oracle_mod, comm, name):
    p = _params(oracle_mod, name)
    with rtsn_mod.Solver(p) as s:
        s.solve()
        assert comm.rank == (1, 0)
        for got, want in zip(comm.gather_moments(s), s.moments()):
            assert np.array_equal(got, want)
        for got, want in zip(comm.gather_group_ends(s), s.compute_group_ends()):
            assert np.array_equal(got, want)
        for got, want in zip(comm.gather_balance(s), s.compute_balance_terms()):
            assert np.array_equal(got, want)
        assert np.array_equal(comm.gather_psi(s, root=0), s.psi())


def test_world_one_absorption_allreduce(rtsn_mod, oracle_mod, comm):
    import torch
    p = _params(oracle_mod)
    with rtsn_mod.Solver(p) as s:
        s.solve()
        a = torch.zeros(p["N"], dtype=torch.float64, device="cuda")
        b = torch.zeros_like(a)
        s.group_absorption_device(a.data_ptr())
        comm.allreduce_absorption(s, b)
        s.synchronize()
        assert torch.equal(a, b)


@pytest.mark.parametrize("ts", [1, 3])
def test_world_one_material_step(rtsn_mod, oracle_mod, comm, ts):
    """rt_comm_material_step (sweep, all-reduce of q on the stream, update) equals
    rt_material_step on an identical handle, bitwise."""
    p = _params(oracle_mod, "multi_group_equilibrium.prm", ts_method=ts, V=0.0, N=300)
    out = []
    for use_comm in (False, True):
        with rtsn_mod.Solver(p) as s:
            s.material_enable(0.05, np.linspace(0.6, 1.4, p["N"]))  # out of equilibrium
            if use_comm:
                comm.material_step(s, 5)
            else:
                s.material_step(5)
            out.append(s.temperature())
    assert np.array_equal(out[0], out[1])
    assert not np.array_equal(out[0], np.linspace(0.6, 1.4, p["N"]))


def test_shards_must_tile(rtsn_mod, oracle_mod, comm):
    """One rank holding groups [7, 70) of 124 does not tile the configuration."""
    p = _params(oracle_mod)
    with rtsn_mod.Solver(p, g_lo=7, g_hi=70) as s:
        s.solve()
        with pytest.raises(rtsn_mod.RtError) as e:
            comm.gather_moments(s)
        assert e.value.status == 3


def test_comm_version_is_the_loaded_rccl(rtsn_mod, comm):
    """rt_comm_version names the RCCL the communicator runs on: the librccl.so.1 this
    process resolved (torch imports first, so its bundled RCCL -- the one torch.distributed
    uses -- serves librtsn too), with a 2.x version code."""
    import os
    v = rtsn_mod.comm_version()
    assert v["code"] >= 20000 and v["version"].startswith("2.")
    assert os.path.exists(v["path"]) and "rccl" in os.path.basename(v["path"])
    loaded = [l.split()[-1] for l in open("/proc/self/maps") if "librccl" in l]
    assert os.path.realpath(v["path"]) in {os.path.realpath(x) for x in loaded}


_MISSING_PEER = r"""
import sys, time
sys.path[:0] = [sys.argv[1], sys.argv[1] + "/radiative-transfer_amd"]
import rtsn
uid = rtsn.Comm.unique_id()
t0 = time.perf_counter()
try:
    rtsn.Comm(2, 0, uid, 0)      # rank 0 of two; rank 1 never starts
except rtsn.RtError as e:
    print("STATUS", e.status, round(time.perf_counter() - t0, 2), str(e)[:200], flush=True)
else:
    print("STATUS 0", flush=True)
"""


def test_comm_init_without_peer_times_out(tmp_path):
    """rt_comm_init is non-blocking and bounded: rank 0 of a 2-rank communicator whose
    peer never joins returns RT_ERR_TIMEOUT (7) once RTSN_COMM_TIMEOUT_S passes, instead of
    waiting in ncclCommInitRank for ever (a child process, so a regression cannot hang the
    test session: it is killed at the subprocess limit)."""
    import os
    import subprocess
    import sys
    from conftest import REPO
    env = dict(os.environ, RTSN_COMM_TIMEOUT_S="5")
    r = subprocess.run([sys.executable, "-c", _MISSING_PEER, str(REPO)], env=env, capture_output=True, text=True,
                       timeout=150)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("STATUS")]
    assert line, (r.stdout[-2000:], r.stderr[-2000:])
    parts = line[0].split()
    assert parts[1] == "7", line[0]
    assert 4.5 <= float(parts[2]) <= 60.0, line[0]
    assert "RTSN_COMM_TIMEOUT_S" in line[0]


def test_comm_deadline_ignores_local_work_ahead(rtsn_mod, monkeypatch):
    """the RTSN_COMM_TIMEOUT_S deadline clocks a collective from the moment
    the stream reaches it, not the host wait.  With a 1 s deadline, a one-rank communicator
    runs coupled steps whose sweeps take several seconds of local work (material_step: sweep,
    all-reduce of q, update per step, all stream-ordered) and then a gather whose stream still
    holds a long rt_advance: both succeed, and ncclCommCount reports the one rank."""
    import sys
    import time
    from conftest import REPO
    sys.path.insert(0, str(REPO))
    import bench
    monkeypatch.setenv("RTSN_COMM_TIMEOUT_S", "1")
    with rtsn_mod.Comm(1, 0, rtsn_mod.Comm.unique_id(), 0) as c:
        assert c.count == 1
        p = bench.material_params(bench.slab_params(16, "v0", N=1_000_000, M=64))
        with rtsn_mod.Solver(p, device=0) as s:
            s.material_enable(1.0)
            s.synchronize()
            t0 = time.perf_counter()
            c.material_step(s, 250)      # ~6 ms of sweep per step ahead of each all-reduce
            c.synchronize(s)
            dt = time.perf_counter() - t0
            assert np.isfinite(s.temperature()).all()
        assert dt > 1.2, f"only {dt:.2f} s of local work: the test does not exercise the deadline"
        q = dict(bench.slab_params(16, "v0", N=1_000_000, M=64), dt=1e-9)
        with rtsn_mod.Solver(q, device=0) as s:
            s.pipeline = 2
            s.advance(2000)              # ~2 s of pipelined sweeps, enqueued without a host wait
            t0 = time.perf_counter()
            left, right = c.gather_group_ends(s)
            dt = time.perf_counter() - t0
            l2, r2 = s.compute_group_ends()
            assert np.array_equal(left, l2) and np.array_equal(right, r2)
        assert dt > 1.2, f"the gather waited only {dt:.2f} s: the test does not exercise the deadline"
        assert c.count == 1
