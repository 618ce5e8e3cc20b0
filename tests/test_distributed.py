"""Multi-rank path of bench.py on CPU: world_size 2 over gloo.

bench.py shards energy groups across ranks: no collective in
the data path, barrier + max-over-ranks timing, one all-reduce of the
group-summed absorption A(x) = sum_g rho kappa_g phi_g(x) after timing.  Here
each rank drives bench.run_rank() with a CPU stand-in solver built on the
oracle over its group shard (the stand-in is the test's, never the product's),
and the all-reduced A(x) must equal the single-process oracle over all groups
-- the check that the shard boundaries, the per-rank group tables (the last
Planck group is a remainder of ALL groups) and the reductions are right.
"""
from __future__ import annotations

import json
import os
import socket
import sys
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO

sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "oracle"))

import bench  # noqa: E402
import oracle  # noqa: E402

oracle.build()


def small_params(G_total: int, variant: str = "corr") -> dict:
    p = bench.slab_params(G_total, variant, N=48, M=8)
    return p


def oracle_dict(p: dict) -> dict:
    q = dict(p)
    q.update(bc_left=p["bc_left_indicator"], bc_right=p["bc_right_indicator"], dx=p["X"] / p["N"],
             have_group_bounds=0, have_group_kappa=1, prm_found=1)
    return q


class OracleShard:
    """CPU stand-in with the rtsn.Solver methods run_rank uses."""

    def __init__(self, p: dict, g_lo: int, g_hi: int):
        self.p = p
        self.s = oracle.OracleSolver(oracle_dict(p), g_lo=g_lo, g_hi=g_hi)
        self.g_lo, self.g_hi = g_lo, g_hi
        self.it = 0
        self.prof = False
        self.ms = 0.0
        self.n = 0

    def sweep_traffic(self):
        Gl = self.g_hi - self.g_lo
        return 32.0 * self.p["M"] * Gl * self.p["N"], 4.0 * self.p["M"] * Gl * self.p["N"]

    def sweep_flops(self):
        return 56.0 * self.p["M"] * (self.g_hi - self.g_lo) * self.p["N"]

    def sweep_geometry(self):
        return 1, 1

    def advance(self, n):
        for _ in range(n):
            t0 = time.perf_counter()
            self.s.run_substeps(self.it, 4)
            self.it += 4
            if self.prof:
                self.ms += 1e3 * (time.perf_counter() - t0)
                self.n += 1

    def synchronize(self):
        pass

    def finish(self):
        pass

    def pipeline_state(self):
        return {"lag_steps": 0, "queued_steps": 0, "pending": False}

    def set_profiling(self, on):
        self.prof = bool(on)
        if on:
            self.ms, self.n = 0.0, 0

    def sweep_time(self):
        return self.ms, self.n

    def moments_device(self, phi, F=None, phi_plus=None):
        ph, f, pp = self.s.moments()  # (G_local, N) -> N x G_local, g fastest
        for t, a in ((phi, ph), (F, f), (phi_plus, pp)):
            if t is not None:
                t.copy_(torch.from_numpy(np.ascontiguousarray(a.T).ravel()))

    def compute_group_ends(self):
        return self.s.group_ends()

    def state_finite(self):
        return bool(np.isfinite(self.s.ends()).all())

    def compute_balance(self):
        return self.s.balance()

    def group_absorption(self, out):
        phi, _, _ = self.s.moments()
        kap = self.s.groups()["kappa"][self.g_lo:self.g_hi]
        a = (self.p["rho"] * kap[:, None] * phi).sum(axis=0) if len(kap) else np.zeros(self.p["N"])
        out.copy_(torch.from_numpy(a))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, scaling, groups, steps, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        info = bench.shard(scaling, groups, world, rank)
        p = small_params(info[0])
        solver = OracleShard(p, info[1], info[2])
        shards = [bench.shard(scaling, groups, world, r)[1:] for r in range(world)]
        line, absorb, gathered = bench.run_rank(solver, p, steps, 1, world, torch.device("cpu"), info, scaling,
                                                shards)
        np.save(os.path.join(outdir, f"absorb{rank}.npy"), absorb.numpy())
        np.savez(os.path.join(outdir, f"gathered{rank}.npz"), **{k: v.numpy() for k, v in gathered.items()})
        with open(os.path.join(outdir, f"line{rank}.json"), "w") as f:
            json.dump({"line": line, "info": list(info), "wall_ms": solver.ms}, f)
    finally:
        dist.destroy_process_group()


def _run(tmp_path, scaling, groups, steps=2, world=2):
    mp.start_processes(_worker, args=(world, _free_port(), scaling, groups, steps, str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    lines = [json.load(open(tmp_path / f"line{r}.json")) for r in range(world)]
    absorbs = [np.load(tmp_path / f"absorb{r}.npy") for r in range(world)]
    gathered = [dict(np.load(tmp_path / f"gathered{r}.npz")) for r in range(world)]
    return lines, absorbs, gathered


def full_run(G_total: int, steps: int):
    """Single-process oracle over all groups: absorption and the gathered fields."""
    p = small_params(G_total)
    s = oracle.OracleSolver(oracle_dict(p))
    s.run_substeps(0, 4 * (steps + 1))  # warmup 1 + timed steps
    phi, F, pp = s.moments()
    kap = s.groups()["kappa"]
    left, right = s.group_ends()
    ref = {"phi": phi.T, "F": F.T, "phi_plus": pp.T, "left": left, "right": right, "balance": s.balance()}
    return (p["rho"] * kap[:, None] * phi).sum(axis=0), ref


@pytest.mark.parametrize("scaling,groups", [("weak", 3), ("strong", 5)])
def test_two_rank_group_shards(tmp_path, scaling, groups):
    steps = 2
    lines, absorbs, gathered = _run(tmp_path, scaling, groups, steps)
    G_total = groups * 2 if scaling == "weak" else groups
    # shards tile [0, G_total) without overlap
    spans = sorted(tuple(l["info"][1:]) for l in lines)
    assert spans[0][0] == 0 and spans[-1][1] == G_total and spans[0][1] == spans[1][0]
    # all-reduced absorption == single-process oracle over all groups
    ref, fields = full_run(G_total, steps)
    for a in absorbs:
        np.testing.assert_array_equal(a, absorbs[0])
        np.testing.assert_allclose(a, ref, rtol=1e-13, atol=0)
    # end-of-run all-gather: every rank holds the full (N, G) fields and (G) vectors,
    # equal (bitwise: same per-group arithmetic) to the single-process oracle
    for g in gathered:
        for k, v in fields.items():
            np.testing.assert_array_equal(g[k], v, err_msg=k)
    # the JSON line: whole-job updates over the max-over-ranks wall time
    line = lines[0]["line"]
    for k in ("value", "ms_per_step", "n_gpus", "state_finite"):
        assert line[k] == lines[1]["line"][k]  # reduced over ranks
    assert line["roofline"]["kernel_ms"] == lines[1]["line"]["roofline"]["kernel_ms"]
    total = sum(4.0 * 8 * (l["info"][2] - l["info"][1]) * 48 * steps for l in lines)
    assert line["n_gpus"] == 2 and line["scaling"] == scaling
    assert line["value"] == pytest.approx(total / (line["ms_per_step"] * 1e-3 * steps), rel=1e-12)
    assert line["config"]["groups_total"] == G_total
    assert line["state_finite"] is True
    assert line["roofline"]["kernel_ms"] >= max(l["wall_ms"] for l in lines) / steps * (1 - 1e-9)
    # every rank's own timing beside the max: the same table on both ranks, the max its worst
    pr = line["per_rank"]
    assert pr == lines[1]["line"]["per_rank"] and [r["rank"] for r in pr] == [0, 1]
    assert max(r["wall_ms"] for r in pr) == pytest.approx(line["ms_per_step"] * steps, rel=1e-12)
    assert max(r["kernel_ms"] for r in pr) == line["roofline"]["kernel_ms"]
    for r, l in zip(pr, lines):
        upd = 4.0 * 8 * (l["info"][2] - l["info"][1]) * 48 * steps
        assert r["updates_per_s"] == pytest.approx(upd / (r["wall_ms"] * 1e-3), rel=1e-12)


def test_shard_table():
    assert bench.shard("weak", 128, 8, 3) == (1024, 384, 512)
    assert bench.shard("strong", 128, 3, 2) == (128, 86, 128)
    spans = [bench.shard("strong", 10, 4, r)[1:] for r in range(4)]
    assert spans == [(0, 3), (3, 6), (6, 9), (9, 10)]


def test_warmup_rule():
    """bench.py: the warmup covers the pipeline fill and whole passes, whatever W is asked."""
    import bench
    assert bench.warmup_steps(-1, 128, 16) == 128   # default: the fill
    assert bench.warmup_steps(1, 128, 16) == 128    # BASELINE's W = 1
    assert bench.warmup_steps(200, 128, 16) == 208  # more than the fill: whole passes
    assert bench.warmup_steps(5, 80, 10) == 80
    assert bench.warmup_steps(0, 2, 2) == 2         # aligned schedule: one pass


def test_material_params_valid_for_both_variants():
    """the material leg must not inherit the corr variant's V = 5.994 with the
    correction on, which rt_material_enable refuses (RT_ERR_PARAM)."""
    import bench
    for variant in ("v0", "corr"):
        q = bench.material_params(bench.slab_params(4, variant, N=100, M=4))
        assert q["ts_method"] == 1
        assert q["V"] == 0.0 or not q["use_correction"]


def test_time_block_choice():
    """bench.py: K timed steps run as whole passes of the fastest block dividing K."""
    import bench
    assert bench.choose_time_block(20) == 20        # the driver's window
    assert bench.choose_time_block(32) == 32
    assert bench.choose_time_block(80) == 40
    assert bench.choose_time_block(48) == 16        # 16 before 24 when both divide
    assert bench.choose_time_block(60) == 20
    assert bench.choose_time_block(30) == 10
    assert bench.choose_time_block(2) == 2
    assert bench.choose_time_block(7) == 7
    assert bench.choose_time_block(11) == 1
    assert bench.choose_time_block(20, forced=10) == 10
    assert bench.choose_time_block(64, forced=32) == 32
    with pytest.raises(ValueError):
        bench.choose_time_block(20, forced=16)
    for k in range(1, 200):
        t = bench.choose_time_block(k)
        assert k % t == 0 and t in bench.SUPPORTED_TIME_BLOCKS


class OracleDirShard(OracleShard):
    """CPU stand-in for a direction-pair shard (rt_create_direction_shard): the oracle
    over all directions and groups, reporting the partial sums over its directions --
    what the library's shard handle returns (its psi is bitwise the full handle's rows,
    tests/test_gpu_parity.py::test_direction_shards)."""

    def __init__(self, p: dict, d_lo: int, d_hi: int):
        super().__init__(p, 0, p["G"])
        H = p["M"] // 2
        self.idx = list(range(H - d_hi, H - d_lo)) + list(range(H + d_lo, H + d_hi))
        self.M_l = len(self.idx)

    def sweep_traffic(self):
        return 32.0 * self.M_l * self.p["G"] * self.p["N"], 4.0 * self.M_l * self.p["G"] * self.p["N"]

    def sweep_flops(self):
        return 56.0 * self.M_l * self.p["G"] * self.p["N"]

    def _partial(self):
        mu, wt = self.s.quad()
        psi = self.s.psi()  # (M, G, N)
        phi = F = pp = 0.0
        for i in self.idx:  # ascending i, as the handle sums its own directions
            phi = phi + wt[i] * psi[i]
            F = F + mu[i] * wt[i] * psi[i]
            if mu[i] > 0:
                pp = pp + wt[i] * psi[i]
        return phi, F, pp

    def moments_device(self, phi, F=None, phi_plus=None):
        for t, a in zip((phi, F, phi_plus), self._partial()):
            if t is not None:
                t.copy_(torch.from_numpy(np.ascontiguousarray(np.asarray(a).T).ravel()))

    def compute_group_ends(self):
        mu, _ = self.s.quad()
        ends = self.s.ends()  # (M, G, N, 2)
        de = self.s.groups()["de_ave"] * 299.792458
        left = sum(ends[i, :, 0, 0] for i in self.idx if mu[i] < 0) / de
        right = sum(ends[i, :, -1, 1] for i in self.idx if mu[i] > 0) / de
        return left, right

    def compute_balance(self):
        raise AssertionError("a direction shard has no balance (rt_get_balance* refuses)")

    def group_absorption(self, out):
        phi, _, _ = self._partial()
        kap = self.s.groups()["kappa"]
        out.copy_(torch.from_numpy((self.p["rho"] * kap[:, None] * phi).sum(axis=0)))


def _dir_worker(rank, world, port, groups, steps, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p = small_params(groups)
        dirs = bench.direction_shard("strong", groups, p["M"], world, rank)
        info = (groups, 0, groups)
        solver = OracleDirShard(p, *dirs)
        line, absorb, gathered = bench.run_rank(solver, p, steps, 1, world, torch.device("cpu"), info, "strong",
                                                None, dirs=dirs)
        np.save(os.path.join(outdir, f"absorb{rank}.npy"), absorb.numpy())
        np.savez(os.path.join(outdir, f"gathered{rank}.npz"), **{k: v.numpy() for k, v in gathered.items()})
        with open(os.path.join(outdir, f"line{rank}.json"), "w") as f:
            json.dump({"line": line, "dirs": list(dirs)}, f)
    finally:
        dist.destroy_process_group()


def test_two_rank_direction_shards(tmp_path):
    """Fewer groups than ranks (1 group, 2 ranks): bench shards direction pairs; the
    all-reduced absorption and moments and the summed group ends equal one oracle run
    over all directions to rounding (the reference's sum over i regrouped by rank)."""
    steps, world, groups = 2, 2, 1
    mp.start_processes(_dir_worker, args=(world, _free_port(), groups, steps, str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    lines = [json.load(open(tmp_path / f"line{r}.json")) for r in range(world)]
    assert [l["dirs"] for l in lines] == [[0, 2], [2, 4]]  # M = 8: 4 pairs
    ref_abs, ref = full_run(groups, steps)
    for r in range(world):
        a = np.load(tmp_path / f"absorb{r}.npy")
        np.testing.assert_allclose(a, ref_abs, rtol=1e-13, atol=0)
        g = dict(np.load(tmp_path / f"gathered{r}.npz"))
        for k in ("phi", "F", "phi_plus"):
            scale = np.abs(ref["phi"]).max()
            assert np.abs(g[k] - ref[k]).max() <= 1e-13 * scale, k
        for k in ("left", "right"):
            np.testing.assert_allclose(g[k], ref[k], rtol=1e-13, atol=0)
        assert np.isnan(g["balance"]).all()
    line = lines[0]["line"]
    assert line["config"]["parallelism"].startswith("direction-pair shards x2")
    total = 4.0 * 8 * groups * 48 * steps  # both ranks' lines = all M = 8 directions
    assert line["value"] == pytest.approx(total / (line["ms_per_step"] * 1e-3 * steps), rel=1e-12)


def test_direction_shard_plan():
    assert bench.direction_shard("strong", 128, 64, 8, 3) is None  # groups shard
    assert bench.direction_shard("weak", 1, 64, 8, 3) is None
    assert [bench.direction_shard("strong", 4, 64, 8, r) for r in range(8)] == [(4 * r, 4 * r + 4) for r in range(8)]
    assert [bench.direction_shard("strong", 1, 6, 2, r) for r in range(2)] == [(0, 2), (2, 3)]
    with pytest.raises(ValueError):
        bench.direction_shard("strong", 1, 4, 4, 3)  # 2 pairs, 4 ranks


def test_host_cpus_share(monkeypatch):
    """bench.host_cpus: the CPU baseline's threads are the lease's share -- OMP_NUM_THREADS
    where set, capped by the affinity (and the cgroup quota when there is one)."""
    import bench
    h = bench.host_cpus()
    assert 1 <= h["threads"] <= h["affinity"] <= h["nproc"]
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    assert bench.host_cpus()["threads"] == 1


def test_launch_mode():
    """bench.py --gpus N: a plain run with N > 1 starts the ranks itself; under a
    launcher WORLD_SIZE must equal --gpus."""
    assert bench.launch_mode(1, {}) == "rank"
    assert bench.launch_mode(8, {}) == "spawn"
    assert bench.launch_mode(2, {"WORLD_SIZE": "2"}) == "rank"
    assert bench.launch_mode(1, {"WORLD_SIZE": "1"}) == "rank"
    for n, ws in ((8, "1"), (1, "2"), (4, "8")):
        with pytest.raises(ValueError):
            bench.launch_mode(n, {"WORLD_SIZE": ws})
    with pytest.raises(ValueError):
        bench.launch_mode(0, {})


_RANK_CHILD = r"""
import json, os, sys
import torch.distributed as dist
r, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
assert os.environ["LOCAL_RANK"] == str(r) and os.environ["MASTER_ADDR"] == "127.0.0.1"
fail = sys.argv[1] if len(sys.argv) > 1 else ""
if fail == "rank1" and r == 1:
    sys.exit(3)
dist.init_process_group("gloo")
t = __import__("torch").tensor([float(r)])
dist.all_reduce(t)
if r == 0:
    print("progress line")
    print(json.dumps({"n_gpus": n if fail != "count" else 1, "sum": float(t), "launcher": os.environ["RTSN_BENCH_LAUNCHER"]}))
dist.destroy_process_group()
if fail == "straggle" and r == 1:  # finishes its work, then never exits
    __import__("time").sleep(600)
"""


@pytest.mark.parametrize("n", [2, 3])
def test_spawn_ranks_relays_rank0(tmp_path, capsys, n):
    """spawn_ranks starts n fresh rank processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*), they
    rendezvous (gloo here) and rank 0's JSON line is relayed; status 0."""
    script = tmp_path / "child.py"
    script.write_text(_RANK_CHILD)
    assert bench.spawn_ranks(n, [], script=script) == 0
    out = capsys.readouterr().out
    d = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    assert d["n_gpus"] == n and d["sum"] == n * (n - 1) / 2
    assert d["launcher"] == f"bench.py --gpus {n} (child processes)"


@pytest.mark.parametrize("fail,status", [("rank1", 3), ("count", 1), ("straggle", 1)])
def test_spawn_ranks_fails_loudly(tmp_path, fail, status):
    """A rank that exits non-zero stops the job (the others, blocked in the rendezvous, are
    terminated) with that status; a line whose n_gpus is not N is a failure too, and so is a
    rank still running long after the others finished (straggle_s)."""
    script = tmp_path / "child.py"
    script.write_text(_RANK_CHILD)
    t0 = time.time()
    assert bench.spawn_ranks(2, [fail], script=script, grace_s=5, straggle_s=10) == status
    assert time.time() - t0 < 120


_BENCH_RANK_CHILD = r"""
import json, os, sys
sys.path[:0] = [{repo!r}, {tests!r}, {oracle!r}]
import torch
import torch.distributed as dist
import bench
from test_distributed import OracleShard, small_params
r, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
fail = sys.argv[1] if len(sys.argv) > 1 else ""
dist.init_process_group("gloo")
if fail == "rank5" and r == 5:  # dies after the rendezvous: the others wait in the first barrier
    sys.exit(5)
groups = 128
info = bench.shard("strong", groups, n, r)
p = small_params(info[0])
shards = [bench.shard("strong", groups, n, k)[1:] for k in range(n)]
line, _, gathered = bench.run_rank(OracleShard(p, info[1], info[2]), p, 2, 1, n, torch.device("cpu"), info,
                                   "strong", shards)
line["shards"] = shards
line["gathered_groups"] = int(gathered["phi"].shape[1])
if r == 0:
    print(json.dumps(line), flush=True)
dist.destroy_process_group()
"""


def test_spawn_ranks_eight_rank_rehearsal(tmp_path, capsys):
    """VERDICT r05 #2a: the driver's SCALE shape on CPU -- bench.spawn_ranks(8, ...) starts eight
    rank processes (fresh interpreters, gloo), each runs bench.run_rank on its 16-group shard of
    the 128-group slab (a tiny slab: N = 48, S8, the oracle stand-in), and rank 0's line says
    n_gpus 8 with eight per_rank entries, the shard table [0, 16), [16, 32), ..., [112, 128),
    and the end-of-run gather holding all 128 groups."""
    script = tmp_path / "bench_rank.py"
    script.write_text(_BENCH_RANK_CHILD.format(repo=str(REPO), tests=str(REPO / "tests"), oracle=str(REPO / "oracle")))
    assert bench.spawn_ranks(8, [], script=script) == 0
    out = capsys.readouterr().out
    d = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    assert d["n_gpus"] == 8 and len(d["per_rank"]) == 8
    assert [e["rank"] for e in d["per_rank"]] == list(range(8))
    assert d["shards"] == [[16 * k, 16 * k + 16] for k in range(8)]
    assert d["config"]["groups_per_gpu"] == 16 and d["config"]["groups_total"] == 128
    assert d["gathered_groups"] == 128
    assert d["value"] > 0 and d["state_finite"]


def test_spawn_ranks_eight_ranks_failing_rank_stops_all(tmp_path):
    """... and rank 5 dying after the rendezvous stops the other seven (blocked in the first
    barrier): a non-zero job status -- rank 5's 5, or the status of a peer whose gloo
    connection to it broke in the same poll interval -- well inside the grace period."""
    script = tmp_path / "bench_rank.py"
    script.write_text(_BENCH_RANK_CHILD.format(repo=str(REPO), tests=str(REPO / "tests"), oracle=str(REPO / "oracle")))
    t0 = time.time()
    assert bench.spawn_ranks(8, ["rank5"], script=script, grace_s=5, straggle_s=30) != 0
    assert time.time() - t0 < 120
