#!/usr/bin/env python3
"""Sweep throughput benchmark (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--variant v0|corr]
                    [--scaling weak|strong] [--time-block T] [--no-cpu-baseline]
                    [--material-steps K]

Workload (SURVEY.md §8(d) "SL"): 1D slab X = 0.4 cm, N = 1e6 cells, S64
Gauss-Legendre (M = 64), 128 energy groups per GPU on a log grid 0.001-30 keV
with kappa_g resampled from the LLNL capped table, rho = 1, T = 1 keV, BDF2
(ts_method = 3), vacuum boundaries; V = 0 (variant v0) or V = 5.994 with the
v/c correction (variant corr).  dt = 1e-9 (--dt): at SURVEY's dt = 1e-3 the
reference's BDF2 (const_B from the full dt, solver.cpp:501) overflows the state
to inf within the pipeline fill, and inf arithmetic runs ~4% faster than the
finite state (interleaved A/B, profiles/archive/r03c_ab_finite.jsonl), so the headline
is timed on a finite one and dt = 1e-3 is a side leg (overflow_control).  The
state stays finite for 200-400 steps at dt = 1e-7, 1200-1400 at 1e-8 and more
than 4000 at 1e-9 (profiles/archive/r03j_finite_horizon.jsonl); the fill grows as the
groups per GPU shrink (160 steps at 128 groups, 1280 at the 16 of an 8-GPU
run), so every N runs the same dt = 1e-9, whose timing equals dt = 1e-7's
(profiles/archive/r03k_window_ab.jsonl).  A "step" is one full BDF2
step (4 substeps) of every cell x angle x group of the GPU's groups, i.e.
4 M G N cell-angle-group updates, computed in fp64 by the fused HIP sweep.
State is resident in HBM before timing.

Multi-GPU: one process per GPU, groups sharded across
ranks with no collective in the data path (groups are independent for the
whole run: T is constant).  Launch: under torch.distributed.run (WORLD_SIZE set; it must
equal --gpus), or plain `python bench.py --gpus N`, where this process -- which never
touches the GPU -- starts the N rank processes itself (spawn_ranks: fresh interpreters with
RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*), relays rank 0's JSON line and fails if any rank
fails.  strong scaling (default, the north_star's "same
slab"): the 128 groups are split N ways (16 per GPU at N = 8); weak: every
rank owns 128 groups of a 128*N-group grid.  Timing:
barrier + device synchronise on both sides of the K timed steps, max over
ranks.  After timing, the group-summed absorption rate is all-reduced over
RCCL once (the north_star group-sum hook) and checked.

Time blocking: one sweep launch (a "pass") advances T full steps (default
T = 16, --time-block), reading and writing the state once.

material (--material-steps, default 3; 0 skips): after the sweep measurement
the same shard runs the material-temperature coupling (rt_material_*, beyond
the reference): BE steps with the per-cell Planck emission, the shard's
exchange term q(x), one all-reduce of q over the ranks and the T update.
Reported under "material"; not part of value.

roofline: per pass, the algorithmic HBM bytes (16 B read + 16 B write per
cell x line) and the algorithmic FP64 flops (2 per coefficient of the
per-line affine cell map, 28 FMAs per cell x line x BDF2 step, times T) over
the sweep kernel's mean duration from HIP events recorded around each
launch on the library's stream.  At T = 1 the pass is HBM-bound (peak
8.0 TB/s, MI355X_MICROARCH.md); at T > 1 it is FP64-bound (peak 78.6
TFLOP/s spec).  traffic: per-launch HBM bytes from rocprofv3 PMC passes
recorded in profiles/pmc_<variant>_t<T>.json (FETCH_SIZE x 2 + WRITE_SIZE,
the gfx950 correction), null if absent.
cpu_baseline: the C oracle (a single-threaded port of the reference's
algorithm) on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
T_PROCESS0 = time.perf_counter()  # the process's own clock: process_wall_s in the line
sys.path.insert(0, str(REPO / "radiative-transfer_amd"))

import numpy as np  # noqa: E402

# BASELINE.json's metric, named on the workload the headline value is measured on: the SL
# slab (the north_star's 1e6-cell x S64 x 128-group slab); the metric's named
# config, llnl_slab_test, is timed on the same run under the top-level "llnl_slab_test" key
METRIC = ("cell·angle·group updates/sec (Sn sweep) + BDF2 steps/sec, SL slab (N=1e6 x S64 x 128 groups); "
          "llnl_slab_test rate under 'llnl_slab_test'")
HBM_PEAK = 8.0e12
SUPPORTED_TIME_BLOCKS = (1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 16, 20, 24, 32, 40)  # rt_set_time_block
# the bench's choice for K timed steps: the first of these dividing K, fastest per step first
# (SL pipelined, same box, ms/step: T = 40 7.49-7.53, 32 7.69-7.75, 16 8.13-8.19, 20 8.22,
# 24 8.26-8.29, 12 ~9.0, 10 8.9-9.0, 8 9.5, 4 12.3, 2 21; profiles/archive/r02g_big_time_blocks.jsonl,
# r02a_windows.jsonl)
TIME_BLOCK_PREFERENCE = (40, 32, 16, 20, 24, 12, 10, 8, 7, 6, 5, 4, 3, 2, 1)
DEFAULT_TIME_BLOCK = 40  # the default window: two passes of the fastest block
FP64_PEAK = 78.6e12  # MI355X FP64 vector spec (256 CU x 4 SIMD x 16 FMA lanes x 2 x 2.4 GHz); measured 71 TF: profiles/r01_fp64_peak.txt
KAPPA_TABLE = REPO / "tests" / "golden" / "prm" / "llnl_slab_test_group_kappa_a.txt"


def slab_params(G_total: int, variant: str, N: int = 1_000_000, M: int = 64) -> dict:
    kap = np.loadtxt(KAPPA_TABLE)
    return dict(M=M, G=G_total, N=N, X=0.4, efirst=0.001, elast=30.0,
                bc_left_indicator=0, bc_right_indicator=0, use_mg_equilib=0,
                rho=1.0, kappa_grey=1.0, T=1.0, V=(5.994 if variant == "corr" else 0.0),
                use_correction=1, ts_method=3, dt=1e-3, max_timesteps=1, include_validation=0,
                psi_source=np.zeros((M, G_total)), group_bounds=None,
                group_kappa=kap[(np.arange(G_total) * len(kap)) // G_total])


def host_cpus() -> dict:
    """The host the CPU baseline runs on: model, os.cpu_count(), the process's CPU affinity,
    the cgroup CPU quota (cpu.max) and OMP_NUM_THREADS -- and the threads used: the
    lease's CPU share, i.e. OMP_NUM_THREADS where the pool sets it (16 per GPU on the
    GPU box, whose affinity lists the whole machine), capped by the affinity and quota."""
    info = {"cpu_model": "unknown", "nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
            "cgroup_quota_cpus": None, "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}
    try:  # name the host CPU the baseline ran on
        info["cpu_model"] = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo")
                                 if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            info["cgroup_quota_cpus"] = int(q) / int(per)
    except (OSError, ValueError):
        pass
    threads = info["affinity"]
    if info["omp_num_threads"]:
        threads = min(threads, max(1, int(info["omp_num_threads"])))
    if info["cgroup_quota_cpus"]:
        threads = min(threads, max(1, int(info["cgroup_quota_cpus"])))
    info["threads"] = threads
    return info


def cpu_baseline(variant: str, dt: float = 1e-9) -> dict:
    """The C oracle (the reference's algorithm restated, solver.cpp loop order, gcc -O3) on
    a bounded sample of the SL workload -- all 64 angles, N = 200000 cells, 1 BDF2 step --
    on the lease's CPU share (host_cpus):
      threaded_copies_value: 16 groups (1024 lines), the lines of each direction over the
             OpenMP threads and the whole-array prev/half snapshot copies (solver.cpp:620-625,
             733, its one surviving copy) split over them too (orc_set_parallel_copies: same
             values);
      reference_shaped_value: the same with the copies serial, as the reference makes them;
      value: the faster of the two (identical results);
      single_thread_value: 1 group on 1 thread.
    The state arrays sit on transparent huge pages (the reference layout strides M G
    doubles from cell to cell)."""
    sys.path.insert(0, str(REPO / "oracle"))
    import oracle
    oracle.build()
    host = host_cpus()
    T = host["threads"]
    G, N = 128, 200_000
    p = dict(slab_params(G, variant, N=N), dt=dt)
    q = dict(p)
    q.update(bc_left=p["bc_left_indicator"], bc_right=p["bc_right_indicator"], dx=p["X"] / N,
             have_group_bounds=0, have_group_kappa=1, prm_found=1)

    def timed(g_lo, g_hi, threads, par_copies):
        s = oracle.OracleSolver(q, g_lo=g_lo, g_hi=g_hi)
        s.set_threads(threads)
        s.set_parallel_copies(par_copies)
        t0 = time.perf_counter()
        s.solve()
        return 4.0 * q["M"] * N * (g_hi - g_lo), time.perf_counter() - t0

    u1, t1 = timed(64, 65, 1, False)
    un, tn = timed(56, 72, T, True)
    ur, tr = timed(56, 72, T, False)
    best = "threaded copies" if un / tn >= ur / tr else "serial copies"
    return dict({"value": max(un / tn, ur / tr), "unit": "cell-angle-group updates/s", "cores": T, "kind": "port",
                 "threaded_copies_value": un / tn, "reference_shaped_value": ur / tr, "single_thread_value": u1 / t1,
                 "sample": f"oracle/rt_oracle.c (restatement of solver.cpp, gcc -O3), SL {variant}: M=64, N={N}, "
                           f"1 BDF2 step; 16 groups (1024 lines) on {T} OpenMP threads with the snapshot copies "
                           f"threaded = {un:.3g} updates in {tn:.2f} s; the same with serial copies as in the "
                           f"reference {tr:.2f} s (value: the faster, {best}); 1 group on 1 thread = {u1:.3g} "
                           f"updates in {t1:.2f} s"}, **host)


REFERENCE_CONFIGS = ("single_group.prm", "multi_group_equilibrium.prm", "llnl_slab_test.prm",
                     "llnl_slab_test_uncapped.prm")


RATE_REPS = 5
E2E_REPS = 5  # timed end-to-end runs per reference configuration (median reported)


def gpu_rate(params: dict, ts_method: int, rate_steps: int = 1000) -> dict:
    """rate_steps steps of a configuration on the GPU exactly as rt_solve runs them (the
    handle's max_timesteps = rate_steps): the short-line wavefront (one launch per advance)
    where the lines fit a chain of waves, else the pipelined schedule rt_solve plans for the
    run (rt_plan_schedule: time block, waves per segment, segmentation).  The handle is
    created and warmed outside the timer; rt_solve + rt_finish (the pending correction of an
    aligned remainder, if any) + device sync are timed, RATE_REPS times (a fresh handle from
    the initial state each time): BDF2 steps/s and cell-angle-group updates/s from the median
    run (all runs in ms_runs), with the number of sweep launches (HIP event pairs) of one run."""
    import rtsn
    params = dict(params, max_timesteps=rate_steps)
    upd_step = (4.0 if ts_method == 3 else 1.0) * params["M"] * params["G"] * params["N"]

    with rtsn.Solver(params) as s:  # warm: kernels loaded, equilibrium sources built
        s.solve()
        s.finish()
        s.synchronize()
    reps = []  # RATE_REPS runs, each on a fresh handle from the initial state: the median is reported
    for _ in range(RATE_REPS):
        with rtsn.Solver(params) as s:
            wst = s.wavefront_state()
            path = "wavefront" if wst["active"] else "segments"
            plan = None if wst["active"] else s.plan_schedule(rate_steps)
            s.synchronize()
            t0 = time.perf_counter()
            s.solve()
            s.finish()
            s.synchronize()
            reps.append(time.perf_counter() - t0)
            finite = s.state_finite()
    gpu_s = sorted(reps)[len(reps) // 2]
    with rtsn.Solver(params) as s:  # the launches, counted by HIP event pairs outside the timed run
        s.set_profiling(True)
        s.solve()
        s.finish()
        passes = s.sweep_time()[1]
        s.set_profiling(False)
    return {"steps": rate_steps, "bdf2_steps_per_s": rate_steps / gpu_s, "updates_per_s": upd_step * rate_steps / gpu_s,
            "ms": 1e3 * gpu_s, "ms_runs": [round(1e3 * r, 4) for r in reps], "timing": f"median of {RATE_REPS} runs",
            "sweep_passes": passes, "path": path,
            "time_block": plan["time_block"] if plan else None, "state_finite": finite,
            **({"cells_per_lane": wst["cells_per_lane"], "waves_per_chain": wst["waves"]} if path == "wavefront"
               else {"plan": plan})}


def llnl_slab_test_rate(ref_configs=None, rate_steps: int = 1000) -> dict:
    """BASELINE.json's named config, prm/llnl_slab_test.prm (M = 2, G = 124 tabulated groups,
    N = 50), as a rate over rate_steps BDF2 steps on the GPU -- from reference_config when
    it ran (with the oracle beside it), else measured here (GPU only)."""
    import rtsn
    cfg = "prm/llnl_slab_test.prm (M=2, G=124 tabulated bounds/kappa, N=50, BDF2 dt=1e-3)"
    if ref_configs and "llnl_slab_test.prm" in ref_configs:
        r = ref_configs["llnl_slab_test.prm"]
        rate = r["rate"]
        return {"config": cfg, "steps": rate["steps"], "bdf2_steps_per_s": rate["gpu_bdf2_steps_per_s"],
                "updates_per_s": rate["gpu_updates_per_s"], "ms": rate["gpu_ms"], "path": rate["path"],
                "time_block": rate["time_block"],
                "sweep_passes": rate["gpu_sweep_passes"], "state_finite": rate["state_finite"],
                "cpu_bdf2_steps_per_s": rate["cpu_bdf2_steps_per_s"], "cpu": rate["cpu"],
                "prm_length_end_to_end_ms": r["gpu_end_to_end_ms"], "prm_length_cpu_ms": r["cpu_ms"],
                "phi_max_rel_diff_vs_oracle": r["phi_max_rel_diff"]}
    pdir = REPO / "tests" / "golden" / "prm"
    ph = rtsn.ParameterHandler(pdir / "llnl_slab_test.prm", table_dir=str(pdir) + "/")
    g = gpu_rate(ph.params, 3, rate_steps)
    return dict({"config": cfg}, **g)


def reference_config_timings(rate_steps: int = 1000) -> dict:
    """BASELINE.json's small configs (the reference's own .prm files, SURVEY §8(d) SG, EQ,
    LL, LL-uncapped):
      * end to end at the .prm's own length -- create + solve + moments on the GPU, and
        the oracle (the reference's loop order) on one core -- with the GPU's phi checked
        against the oracle's (max per-group relative difference); for llnl_slab_test also
        the oracle with the reference's literal per-cell half_ends copy (solver.cpp:733,
        quadratic in the state size);
      * as a rate: `rate_steps` BDF2 steps of the same configuration as rt_solve runs them
        (gpu_rate: handle created and warmed outside the timer; rt_solve + finish + device
        sync timed), GPU BDF2 steps/s
        and updates/s beside the oracle's on one core over the same steps, with the
        number of sweep passes (HIP event pairs) the GPU ran -- the metric's named config,
        llnl_slab_test, among them."""
    import rtsn
    sys.path.insert(0, str(REPO / "oracle"))
    import oracle
    oracle.build()
    pdir = REPO / "tests" / "golden" / "prm"
    tdir = str(pdir) + "/"
    out = {}
    for name in REFERENCE_CONFIGS:
        ph = rtsn.ParameterHandler(pdir / name, table_dir=tdir)
        q = oracle.parse_prm(pdir / name, table_dir=tdir)
        r = {"M": q["M"], "G": q["G"], "N": q["N"], "steps": q["max_timesteps"],
             "ts_method": q["ts_method"]}
        runs = []
        for _ in range(1 + E2E_REPS):  # the first untimed (it pays module/kernel loading)
            t0 = time.perf_counter()
            with rtsn.Solver(ph) as s:
                s.solve()
                phi = s.moments()[0]
            runs.append(1e3 * (time.perf_counter() - t0))
        r["gpu_end_to_end_ms"] = sorted(runs[1:])[E2E_REPS // 2]  # median of the timed runs
        r["gpu_end_to_end_ms_runs"] = [round(x, 4) for x in runs[1:]]
        for literal in ((False, True) if name == "llnl_slab_test.prm" else (False,)):
            o = oracle.OracleSolver(q, half_copy_literal=literal)
            t0 = time.perf_counter()
            o.solve()
            phi_o = o.moments()[0]
            r["cpu_literal_half_copy_ms" if literal else "cpu_ms"] = 1e3 * (time.perf_counter() - t0)
        scale = np.maximum(np.abs(phi_o).max(axis=1, keepdims=True), 1e-300)
        r["phi_max_rel_diff"] = float((np.abs(phi - phi_o) / scale).max())

        # the rate over rate_steps BDF2 steps
        params = dict(ph.params, max_timesteps=rate_steps)
        upd_step = (4.0 if q["ts_method"] == 3 else 1.0) * q["M"] * q["G"] * q["N"]
        g = gpu_rate(params, q["ts_method"], rate_steps)
        o = oracle.OracleSolver(dict(q, max_timesteps=rate_steps))
        t0 = time.perf_counter()
        o.solve()
        cpu_s = time.perf_counter() - t0
        r["rate"] = {"steps": rate_steps, "gpu_bdf2_steps_per_s": g["bdf2_steps_per_s"],
                     "cpu_bdf2_steps_per_s": rate_steps / cpu_s, "gpu_updates_per_s": g["updates_per_s"],
                     "cpu_updates_per_s": upd_step * rate_steps / cpu_s, "gpu_ms": g["ms"], "cpu_ms": 1e3 * cpu_s,
                     "gpu_sweep_passes": g["sweep_passes"], "path": g["path"], "time_block": g["time_block"],
                     "state_finite": g["state_finite"], "cpu": "oracle, 1 thread, the reference's loop order"}
        out[name] = r
    return out


def load_traffic(variant: str, tb: int, algorithmic_bytes: float):
    """Measured HBM bytes per sweep launch (rocprofv3 PMC: scripts/gpu.sh TAG pmc) for
    this variant and time block, or None -- also None when the profile was taken on a
    different problem size (its bytes are not within 10% of this launch's)."""
    f = REPO / "profiles" / f"pmc_{variant}_t{tb}.json"
    if not f.exists():
        return None
    try:
        b = json.loads(f.read_text()).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None
    return b if b and abs(b / algorithmic_bytes - 1.0) < 0.1 else None


def choose_time_block(steps: int, forced: int = 0) -> int:
    """Steps per pass for a timed region of exactly `steps` steps: `forced` when given
    (it must divide `steps`), else the first block of TIME_BLOCK_PREFERENCE (measured
    fastest per step first) that divides it."""
    if forced:
        if forced not in SUPPORTED_TIME_BLOCKS or steps % forced:
            raise ValueError(f"--time-block {forced} must be a supported block dividing --steps {steps}")
        return forced
    return next(t for t in TIME_BLOCK_PREFERENCE if steps % t == 0)


def warmup_steps(requested: int, fill: int, tb: int) -> int:
    """Untimed steps before the K timed ones: at least the `requested` W (negative: none
    asked) rounded up to whole passes of tb steps, and at least the pipeline `fill`
    (segments per line x tb), so the timed passes are the schedule's steady state."""
    if requested < 0:
        return fill
    return max(fill, -(-requested // tb) * tb)


def shard(scaling: str, groups: int, world: int, rank: int):
    """(G_total, g_lo, g_hi) of this rank.  weak: every rank owns `groups`
    groups of a groups*world grid; strong: `groups` split into contiguous
    ceil(groups/world) shards (the last may be short, or empty)."""
    if scaling == "weak":
        return groups * world, rank * groups, (rank + 1) * groups
    per = (groups + world - 1) // world
    lo = min(groups, rank * per)
    return groups, lo, min(groups, lo + per)


def direction_shard(scaling: str, groups: int, M: int, world: int, rank: int):
    """(d_lo, d_hi) of this rank when strong scaling has fewer groups than ranks: every rank
    takes all groups and a contiguous block of the M/2 direction pairs (SURVEY §8e fallback,
    rt_create_direction_shard); None when groups shard (the normal case)."""
    if scaling != "strong" or groups >= world:
        return None
    H = M // 2
    per = -(-H // world)
    lo, hi = rank * per, min(H, (rank + 1) * per)
    if lo >= hi:
        raise ValueError(f"{world} ranks but only {groups} groups and {H} direction pairs")
    return lo, hi


def make_solver(p: dict, local: int, info, dirs):
    """The rank's handle: its group shard, or all groups and its direction pairs."""
    import rtsn
    if dirs:
        return rtsn.Solver(p, device=local, d_lo=dirs[0], d_hi=dirs[1])
    return rtsn.Solver(p, device=local, g_lo=info[1], g_hi=info[2])


def gather_results(solver, N: int, world: int, shard_info, shards, device, dirs=None, timings=None):
    """All-gather of the per-rank result blocks (RCCL on the GPU box, gloo in
    the CPU tests): returns {"phi", "F", "phi_plus"} as (N, G_total) tensors and
    {"left", "right", "balance"} as (G_total,) tensors.  timings (a dict) receives the
    wall time of each step in ms, every step synchronised: alloc (the device buffers),
    moments (rt_get_moments_device: the moments kernel and the copy out), group_ends,
    balance (both reuse the moments of the same state), collective (the all-gathers),
    assemble (the per-rank blocks into the (N, G) arrays)."""
    import torch
    import torch.distributed as dist

    t = timings if timings is not None else {}
    clock = [time.perf_counter()]

    def mark(name):
        solver.synchronize()
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        now = time.perf_counter()
        t[name] = t.get(name, 0.0) + 1e3 * (now - clock[0])
        clock[0] = now

    G_total, g_lo, g_hi = shard_info
    if dirs:  # direction shards: every rank holds partial sums over its directions of all groups
        mom = torch.empty(3, N * G_total, dtype=torch.float64, device=device)
        mark("alloc")
        solver.moments_device(mom[0], mom[1], mom[2])
        mark("moments")
        left, right = solver.compute_group_ends()
        ends = torch.as_tensor(np.stack([left, right]), device=device)
        mark("group_ends")
        if world > 1:
            dist.all_reduce(mom)
            dist.all_reduce(ends)
        mark("collective")
        fields = mom.view(3, N, G_total)
        nan = torch.full((G_total,), float("nan"), dtype=torch.float64, device=device)
        return {"phi": fields[0], "F": fields[1], "phi_plus": fields[2],
                "left": ends[0], "right": ends[1], "balance": nan}  # balance needs the total phi
    shards = shards or [(g_lo, g_hi)]
    Gl = g_hi - g_lo
    Gmax = max(hi - lo for lo, hi in shards)
    # the rank's wire block [3][N][Gmax]: the moments land in it directly when this shard
    # is the largest, else in its first Gl columns
    block = (torch.empty if Gl == Gmax else torch.zeros)(3, N, Gmax, dtype=torch.float64, device=device)
    mom = block.view(3, N * Gmax) if Gl == Gmax else torch.empty(3, N * Gl, dtype=torch.float64, device=device)
    mark("alloc")
    solver.moments_device(mom[0], mom[1], mom[2])
    mark("moments")
    left, right = solver.compute_group_ends()
    mark("group_ends")
    bal = solver.compute_balance()
    mark("balance")
    if Gl != Gmax:
        block[:, :, :Gl] = mom.view(3, N, Gl)
    small = torch.zeros(3, Gmax, dtype=torch.float64, device=device)
    small[:, :Gl] = torch.as_tensor(np.stack([left, right, bal]), device=device)
    if world == 1:  # one shard: the block is the result
        mark("assemble")
        return {"phi": block[0], "F": block[1], "phi_plus": block[2],
                "left": small[0], "right": small[1], "balance": small[2]}
    big = [torch.empty_like(block) for _ in range(world)]
    sm = [torch.empty_like(small) for _ in range(world)]
    mark("alloc")
    dist.all_gather(big, block)
    dist.all_gather(sm, small)
    mark("collective")
    fields = torch.cat([big[r][:, :, :hi - lo] for r, (lo, hi) in enumerate(shards)], dim=2)
    scal = torch.cat([sm[r][:, :hi - lo] for r, (lo, hi) in enumerate(shards)], dim=1)
    mark("assemble")
    return {"phi": fields[0], "F": fields[1], "phi_plus": fields[2],
            "left": scal[0], "right": scal[1], "balance": scal[2]}


def run_rank(solver, p: dict, steps: int, warmup: int, world: int, device, shard_info, scaling: str,
             scaling_shards=None, gather: bool = True, dirs=None):
    """Warmup, K timed steps between barrier + device sync, max over ranks,
    then the absorption all-reduce.  Collectives go through torch.distributed
    on whatever backend is initialised (RCCL on the GPU box, gloo in the CPU
    tests).  Returns the JSON line (all ranks compute it; rank 0 prints)."""
    import torch
    import torch.distributed as dist

    G_total, g_lo, g_hi = shard_info
    bytes_launch, upd_step = solver.sweep_traffic()  # per pass (T fused steps), per full step
    flops_launch = solver.sweep_flops()               # algorithmic FP64 flops per pass
    tb = getattr(solver, "time_block", 1)
    wg, tiles = solver.sweep_geometry()

    def barrier():
        if world > 1:
            dist.barrier()
        if device.type == "cuda":
            torch.cuda.synchronize(device)

    t_start = time.perf_counter()
    solver.advance(warmup)
    if solver.pipeline_state()["queued_steps"]:  # W not whole passes: complete them untimed
        solver.finish()
    solver.synchronize()
    barrier()
    before = solver.pipeline_state()
    # the pass the timed region runs, as rocprof names it: pipelined when the pipeline is
    # filled, level-split (two waves per segment) where the handle runs it (default: T = 20)
    if before["lag_steps"] > 0:
        lw = solver.level_waves if p.get("ts_method", 3) == 3 else 1
        kernel_name = f"sweep_split_kernel<3, {tb}, {lw}>" if lw > 1 else f"sweep_block_kernel<3, {tb}, 2, false>"
    else:
        kernel_name = f"sweep_block_kernel<3, {tb}, 0, false>"
    solver.set_profiling(True)
    t0 = time.perf_counter()
    solver.advance(steps)
    # The timed region must hold exactly K steps of work.  It does when the schedule
    # ends as it started (a filled pipeline one pass per segment apart, or an aligned
    # pass's pending correction): every segment advanced K steps.  Otherwise (the
    # pipeline filled inside the region, or K is not whole passes) complete them here.
    steady = solver.pipeline_state() == before
    if not steady:
        solver.finish()
    solver.synchronize()
    barrier()
    wall = time.perf_counter() - t0
    kern_ms, nlaunch = solver.sweep_time()
    solver.set_profiling(False)
    # outside the timed region: finish every queued step (pipeline drain / correction)
    t1 = time.perf_counter()
    solver.finish()
    solver.synchronize()
    barrier()
    t_end = time.perf_counter()
    # device memory in use with the state resident (the handle's hipMallocs are not torch's,
    # so the device's own count: total - free)
    free_b, total_b = torch.cuda.mem_get_info(device) if device.type == "cuda" else (0, 0)

    # group-summed absorption all-reduce, outside the timed region
    absorb = torch.zeros(p["N"], dtype=torch.float64, device=device)
    solver.group_absorption(absorb)
    solver.synchronize()
    if world > 1:
        dist.all_reduce(absorb)
    # NaN/Inf scan of the state (rt_state_finite), every rank; see DESIGN.md §5: the
    # reference's BDF2 grows ~10^3 per step on SL
    fin = torch.tensor([1.0 if solver.state_finite() else 0.0], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(fin, op=dist.ReduceOp.MIN)
    finite = bool(fin.item() == 1.0)

    # end-of-run gather: every rank's phi, F, phi_plus (N x G_local, g
    # fastest) and its group ends and balance, assembled into the reference's (N, G)
    # / (G) arrays on every rank; ragged shards are padded to the largest
    t2 = time.perf_counter()
    gather_steps = {}
    gathered = (gather_results(solver, p["N"], world, shard_info, scaling_shards, device, dirs, gather_steps)
                if gather else None)
    gather_ms = 1e3 * (time.perf_counter() - t2)

    mine = torch.tensor([wall, kern_ms / max(nlaunch, 1), upd_step * steps], dtype=torch.float64, device=device)
    per_rank = None
    if world > 1:  # every rank's own timing (the line reports the max; a slow rank shows here)
        allr = torch.zeros(world * 3, dtype=torch.float64, device=device)
        dist.all_gather_into_tensor(allr, mine)
        allr = allr.view(world, 3).cpu().numpy()
        per_rank = [{"rank": r, "wall_ms": 1e3 * float(a[0]), "kernel_ms": float(a[1]),
                     "updates_per_s": float(a[2] / a[0]) if a[0] > 0 else None} for r, a in enumerate(allr)]
    t = mine[:2].clone()
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall_max, kern_avg_ms = float(t[0]), float(t[1])
    # whole-job updates: every rank's own count (shards may be ragged under strong scaling)
    u = torch.tensor([upd_step * steps], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(u)
    total_updates = float(u[0])

    value = total_updates / wall_max
    ms_per_step = 1e3 * wall_max / steps
    kern_s = kern_avg_ms * 1e-3
    achieved = bytes_launch / kern_s if kern_s > 0 else 0.0
    achieved_fl = flops_launch / kern_s if kern_s > 0 else 0.0
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "cell-angle-group updates/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "bdf2_steps_per_s": 1e3 / ms_per_step,
        "schedule": {"pipeline_mode": int(getattr(solver, "pipeline", 0)), "steps_per_pass": tb,
                     "steady_state_at_start": steady, "lag_steps": before["lag_steps"],
                     "warmup_steps": warmup, "drain_ms": 1e3 * (t_end - t1),
                     "end_to_end_ms": 1e3 * (t_end - t_start),
                     "end_to_end_updates_per_s": upd_step * (warmup + steps) / (t_end - t_start)},
        "config": {
            "workload": f"SL slab: N={p['N']} cells x S{p['M']} x {g_hi - g_lo} groups per GPU "
                        f"({G_total} total), BDF2 dt={p['dt']:g}, V={p['V']}, use_correction=1, vacuum BCs",
            "cells": p["N"], "angles": p["M"], "groups_per_gpu": g_hi - g_lo, "groups_total": G_total,
            "time_scheme": "BDF2 (4 fused substeps per step)",
            "steps_per_pass": tb,
            "parallelism": (f"direction-pair shards x{world} ({dirs[1] - dirs[0]} of {p['M'] // 2} pairs per GPU), "
                            "no data-path collective" if dirs else f"group shards x{world}, no data-path collective"),
            "sweep_workgroups": wg, "tiles_per_step": tiles,
        },
        # One pass moves the state once (HBM-bound at T = 1) and runs T steps of
        # the cell map (FP64-bound at T > 1): the bound is the
        # roofline the pass sits on; both are reported.
        "roofline": {
            "bound": "fp64" if tb > 1 else "hbm",
            "achieved": achieved_fl / 1e12 if tb > 1 else achieved / 1e9,
            "peak": FP64_PEAK / 1e12 if tb > 1 else HBM_PEAK / 1e9,
            "unit": "TFLOP/s" if tb > 1 else "GB/s",
            "frac": achieved_fl / FP64_PEAK if tb > 1 else achieved / HBM_PEAK,
            "traffic": None,
            # the pass the timed region ran: pipelined (MODE 2) when the pipeline was filled
            "kernel": kernel_name,
            "kernel_ms": kern_avg_ms,
            "algorithmic_flops_per_launch": flops_launch,
            "algorithmic_bytes_per_launch": bytes_launch,
            "hbm": {"achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                    "frac": achieved / HBM_PEAK},
            "fp64": {"achieved": achieved_fl / 1e12, "peak": FP64_PEAK / 1e12, "unit": "TFLOP/s",
                     "frac": achieved_fl / FP64_PEAK},
            "note": ("bound 'fp64': the time-blocked pass is FP64 vector-ALU bound (a per-line affine "
                     "recurrence, no dense contraction, so no MFMA); the same pass at one step per "
                     "pass is HBM-bound: see hbm_pass_t1") if tb > 1 else "HBM-bound pass",
        },
        "state_finite": finite,
        "device_memory_gb": {"used": (total_b - free_b) / 1e9, "total": total_b / 1e9},
    }
    if per_rank is not None:
        line["per_rank"] = per_rank
    # BASELINE.md's roofline definition for the north_star target (>= 0.5): updates/s per GPU
    # x the unfused algorithm's minimal state bytes per update (48 B, 52 B with the
    # v/c correction active) / 8.0 TB/s.  Above 1 means the fused pass moves fewer bytes per
    # update than that algorithm could at the HBM peak.
    b_upd = 52.0 if (p.get("use_correction") and p.get("V", 0.0) != 0.0) else 48.0
    line["baseline_roofline"] = {
        "definition": "BASELINE.md: updates/s per GPU x bytes/update / 8.0e12 B/s (unfused algorithm's bytes)",
        "bytes_per_update": b_upd, "frac": value / world * b_upd / HBM_PEAK, "target": 0.5}
    if gather:
        line["gather"] = {"fields": "phi, F, phi_plus (N x G) + left/right ends, balance (G)",
                          "bytes_per_rank": 8 * 3 * p["N"] * (g_hi - g_lo), "ms": gather_ms,
                          "steps_ms": {k: round(v, 3) for k, v in gather_steps.items()}}
    return line, absorb, gathered


def side_leg(p: dict, info, world: int, device, local: int, scaling: str, tb: int, what: str,
             dirs=None) -> dict:
    """A second sweep measurement on the same shard, reported beside `value` (never as
    it): the state is created fresh, the pipeline filled untimed, then two passes timed
    exactly as the headline.  Used for (a) the HBM-bound T = 1 pass (one HBM round trip
    of the state per BDF2 step: the north_star's HBM-roofline view of the sweep), (b)
    the overflow control (dt = 1e-3, SURVEY's step: the reference's BDF2 overflows the
    state to inf, which runs ~4% faster -- not the headline) and (c) the
    other SL variant (v/c correction on / inactive)."""
    import rtsn
    with make_solver(p, local, info, dirs) as s:
        s.time_block = tb
        s.pipeline = 1
        warm = s.sweep_geometry()[1] * tb
        line, _, _ = run_rank(s, p, 2 * tb, warm, world, device, info, scaling, gather=False, dirs=dirs)
    r = line["roofline"]
    out = {"what": what, "dt": p["dt"], "steps_per_pass": tb, "steps": 2 * tb, "warmup": warm,
           "value": line["value"], "ms_per_step": line["ms_per_step"], "kernel_ms": r["kernel_ms"],
           "state_finite": line["state_finite"]}
    if tb == 1:
        out["hbm"] = dict(r["hbm"], traffic=load_traffic(p["variant"], 1, r["algorithmic_bytes_per_launch"]),
                          algorithmic_bytes_per_launch=r["algorithmic_bytes_per_launch"])
    else:
        out["fp64"] = r["fp64"]
    return out


def material_params(p: dict) -> dict:
    """The material leg's configuration from the sweep's: BE, the v/c correction inactive
    (V = 0) as rt_material_enable requires -- for either SL variant -- and SURVEY's dt = 1e-3
    (stiffness number 1.22 at 1 keV and rho_cv = 1; ~1e5 with the material at 50 keV, where the
    explicit emission of rounds 1-5 diverged and the linearised implicit one is stable)."""
    return dict(p, ts_method=1, V=0.0, dt=1e-3)


COMM_TIMEOUT_S = "120"  # the bench's bound on every rt_comm wait (RTSN_COMM_TIMEOUT_S unless set)


def comm_agree(comm, err, world: int, device):
    """Collective: keep the communicator only if every rank still has a live one (a rank
    whose init or gather timed out would otherwise leave the others in a collective it
    never joins).  Returns (comm or None, reason or None)."""
    import torch
    import torch.distributed as dist
    if world > 1:
        ok = torch.tensor([1.0 if comm is not None else 0.0], dtype=torch.float64, device=device)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if float(ok.item()) < 1.0 and comm is not None:
            comm.close()
            return None, err or "another rank's rt_comm failed"
    return comm, err


def open_comm(world: int, rank: int, local: int, device=None):
    """The RCCL communicator behind the C ABI (rt_comm: non-blocking ncclCommInitRankConfig
    over every rank's GPU, bounded by RTSN_COMM_TIMEOUT_S), or (None, reason) where RCCL
    cannot form it -- the one-GPU multi-rank rehearsal (two ranks on one device), or a rank
    that does not join in time (RT_ERR_TIMEOUT: "skipped (timeout)").  Collective over the
    ranks; every rank ends with a communicator or none does."""
    import torch.distributed as dist
    import rtsn
    os.environ.setdefault("RTSN_COMM_TIMEOUT_S", COMM_TIMEOUT_S)
    comm, err = None, None
    try:
        uid = [rtsn.Comm.unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(uid, src=0)
        comm = rtsn.Comm(world, rank, uid[0], local)
    except rtsn.RtError as e:
        err = ("skipped (timeout): " if e.status == 7 else "") + str(e)
    return comm_agree(comm, err, world, device) if device is not None else (comm, err)


def rccl_gather_check(comm, solver, gathered, dirs) -> dict:
    """The end-of-run result arrays gathered a second way, by RCCL behind the C ABI
    (rt_comm_gather_moments / _group_ends / _balance: the shard table all-gathered, one
    all-gather of every rank's padded blocks, assembled by comm_layout.cpp's copy plans --
    the code a C++ host uses without torch), against the torch.distributed gather above:
    bitwise for group shards; direction shards' sums (an all-reduce) within rounding.
    Outside the timed region; runs only where a communicator formed (every rank calls
    the same collectives in the same order, sequenced after torch's)."""
    import numpy as np
    t0 = time.perf_counter()
    phi, F, pp = comm.gather_moments(solver)     # (G, N) each, on the host
    left, right = comm.gather_group_ends(solver)
    bal = None if dirs else comm.gather_balance(solver)[0]
    ms = 1e3 * (time.perf_counter() - t0)
    ours = {"phi": phi.T, "F": F.T, "phi_plus": pp.T, "left": left, "right": right}
    if bal is not None:
        ours["balance"] = bal
    rel = {}
    for k, v in ours.items():
        ref = gathered[k].cpu().numpy()
        scale = max(float(np.abs(ref).max()), 1e-300)
        rel[k] = float(np.abs(v - ref).max() / scale) if v.shape == ref.shape else float("inf")
    bitwise = all(np.array_equal(v, gathered[k].cpu().numpy()) for k, v in ours.items())
    ok = bitwise if not dirs else max(rel.values()) <= 1e-12
    return {"what": "rt_comm gathers (RCCL in librtsn) vs the torch.distributed gather of the same arrays",
            "ok": bool(ok), "bitwise": bool(bitwise), "max_rel_diff": rel, "ms": ms,
            "fields": sorted(ours)}


def run_material(p: dict, info, world: int, device, local: int, steps: int, dirs=None, rank: int = 0,
                 comm=None, comm_error=None, T0_keV=None) -> dict:
    """The material-temperature coupling (rt_material_*, beyond the reference) on
    the same SL shard: BE steps (the reference's BDF2 diverges on SL within a few
    steps, DESIGN.md §4, which would leave T meaningless; the v/c correction off, as
    the coupling requires) from T = 1 keV, each step = coupled sweep + phi + the
    shard's q(x) + ONE all-reduce (sum) of q over the ranks + T update + per-cell
    Planck.  The all-reduce is RCCL behind the C ABI (rt_comm_material_step: enqueued
    on the handle's stream, no host synchronisation); where RCCL cannot form the
    communicator (the one-GPU multi-rank rehearsal: two ranks on one device) the
    same step runs with torch.distributed's all-reduce on the handle's stream
    (rtsn.coupling.coupled_steps).  One warm-up step, then `steps` timed between
    barrier + device sync, max over ranks."""
    import torch
    import torch.distributed as dist
    import rtsn
    from rtsn.coupling import coupled_steps

    G_total, g_lo, g_hi = info
    q = material_params(p)
    path = "rt_comm_material_step (RCCL in librtsn, stream-ordered)"
    if comm is None:
        path = f"torch.distributed all-reduce on the handle's stream (rt_comm unavailable: {comm_error})"
    with make_solver(q, local, info, dirs) as s:  # q(x): each rank's groups or directions, summed
        number = s.material_enable(1.0, None if T0_keV is None else np.full(q["N"], float(T0_keV)))
        buf = torch.zeros(2 * q["N"], dtype=torch.float64, device=device)

        def step(n):
            if comm is not None:
                comm.material_step(s, n)
            else:
                coupled_steps(s, n, buf, world_size=world)

        step(1)

        def barrier():
            if comm is not None:
                comm.synchronize(s)  # bounded by RTSN_COMM_TIMEOUT_S (RCCL all-reduces in the stream)
            else:
                s.synchronize()
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize(device)

        barrier()
        t0 = time.perf_counter()
        step(steps)
        barrier()
        wall = time.perf_counter() - t0
        T = s.temperature()
        M_local = s.M  # the handle's directions (a direction shard holds 2 (d_hi - d_lo))
    t = torch.tensor([wall], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall = float(t[0])
    u = torch.tensor([float(M_local) * (g_hi - g_lo) * q["N"] * steps], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(u)
    upd = float(u[0])
    return {"what": "material-temperature coupling (beyond the reference): BE step with the per-cell Planck "
                    "emission, [q, b] all-reduce over ranks, T update implicit in the material's emission (the implied emission owed to the next sweeps)",
            "T0_keV": float(T0_keV if T0_keV is not None else q["T"]),
            "ts_method": 1, "steps": steps, "warmup": 1, "ms_per_step": 1e3 * wall / steps,
            "updates_per_s": upd / wall, "allreduce_bytes_per_step": 16 * q["N"], "allreduce": path,
            "rccl": rtsn.comm_version(),  # the RCCL rt_comm ran on (the process's librccl.so.1)
            "stability_number": number, "rho_cv": 1.0, "T_range_keV": [float(T.min()), float(T.max())],
            "state_finite": bool(np.isfinite(T).all())}


def launch_mode(gpus: int, env) -> str:
    """How this process runs the job: "rank" (it is one of the ranks: WORLD_SIZE is set by a
    launcher, or a one-GPU run without one) or "spawn" (no launcher and --gpus > 1: start the
    ranks).  A launcher's WORLD_SIZE that differs from --gpus is an error: the line would
    report a GPU count other than the one asked for."""
    if gpus < 1:
        raise ValueError(f"--gpus {gpus}: at least one GPU")
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return "spawn" if gpus > 1 else "rank"
    if int(ws) != gpus:
        raise ValueError(f"WORLD_SIZE={ws} from the launcher but --gpus {gpus}")
    return "rank"


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def spawn_ranks(n: int, argv, script=None, env=None, grace_s: float = 20.0, straggle_s: float = 300.0) -> int:
    """Start n rank processes of `script` (default: this file) with `argv`, one per GPU
    (LOCAL_RANK r -> cuda:r), rendezvous on 127.0.0.1 at a free port.  Each child is a fresh
    interpreter started by fork+exec from this process, which has not initialised the GPU (it
    imports neither torch nor librtsn).  Rank 0's stdout is relayed line by line; the other
    ranks' output and every stderr pass through.  When a rank exits non-zero the others are
    terminated (their own PIDs: SIGTERM, then SIGKILL after grace_s) and that status is
    returned; 0 when all ranks succeed and rank 0 printed a JSON line whose n_gpus is n.  Ranks
    still running straggle_s after the first one finished cleanly are stopped (status 1)."""
    import signal
    import subprocess
    import threading
    script = str(script or Path(__file__).resolve())
    base = dict(os.environ if env is None else env)
    base.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", RTSN_BENCH_LAUNCHER=f"bench.py --gpus {n} (child processes)")
    procs = []
    lines = []

    def relay(stream):
        for ln in stream:
            sys.stdout.write(ln)
            sys.stdout.flush()
            if ln.startswith("{"):
                lines.append(ln)

    def stop_all(*_):
        for q in procs:
            if q.poll() is None:
                q.terminate()
        t_end = time.time() + grace_s
        for q in procs:
            try:
                q.wait(timeout=max(0.1, t_end - time.time()))
            except subprocess.TimeoutExpired:
                q.kill()
                q.wait()

    old_term = signal.signal(signal.SIGTERM, lambda *a: (stop_all(), sys.exit(143)))
    try:
        for r in range(n):
            e = dict(base, RANK=str(r), LOCAL_RANK=str(r))
            procs.append(subprocess.Popen([sys.executable, "-u", script, *argv], env=e,
                                          stdout=subprocess.PIPE if r == 0 else None, text=True))
        reader = threading.Thread(target=relay, args=(procs[0].stdout,), daemon=True)
        reader.start()
        status = 0
        first_done = None  # when the first rank finished cleanly: the rest get straggle_s more
        while [q.poll() for q in procs].count(None):
            bad = [q.returncode for q in procs if q.returncode not in (None, 0)]
            if bad:
                status = bad[0]
                print(f"bench.py: a rank exited with status {status}; stopping the others", file=sys.stderr)
                stop_all()
                break
            if first_done is None and any(q.returncode == 0 for q in procs):
                first_done = time.time()
            if first_done is not None and time.time() - first_done > straggle_s:
                print(f"bench.py: ranks still running {straggle_s:.0f} s after the first finished; stopping them",
                      file=sys.stderr)
                stop_all()
                status = 1
                break
            time.sleep(0.2)
        reader.join(timeout=30)
        if status == 0:
            bad = [q.returncode for q in procs if q.returncode != 0]
            status = bad[0] if bad else 0
        if status == 0:
            try:
                got = json.loads(lines[-1]).get("n_gpus") if lines else None
            except ValueError:
                got = None
            if got != n:
                print(f"bench.py: rank 0 reported n_gpus={got}, expected {n}", file=sys.stderr)
                status = 1
        return status if status > 0 else (128 - status if status < 0 else 0)
    finally:
        stop_all()
        signal.signal(signal.SIGTERM, old_term)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults: the timed region is 2 steady-state passes of the fastest block (T = 40)
    ap.add_argument("--steps", type=int, default=0, help="timed steps (default: two passes of 40)")
    ap.add_argument("--warmup", type=int, default=-1,
                    help="untimed steps before timing, at least the pipeline fill (default: the fill)")
    ap.add_argument("--variant", choices=["v0", "corr"], default="v0")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="strong")
    ap.add_argument("--groups", type=int, default=128, help="groups per GPU (weak) or in total (strong)")
    ap.add_argument("--cells", type=int, default=1_000_000)
    # SURVEY §8(d)'s SL names dt = 1e-3, at which the reference's BDF2 (const_B from the full dt,
    # solver.cpp:501) overflows the slab's state to inf within the pipeline fill; the headline is
    # timed on a finite state, which runs ~4% slower than the overflowed one on the same box
    # (profiles/archive/r03c_ab_finite.jsonl); dt = 1e-3 is the side leg "overflow_control".  1e-9 keeps
    # the state finite through the longest fill (1280 steps for the 16 groups of an 8-GPU run)
    ap.add_argument("--dt", type=float, default=1e-9,
                    help="time step of the SL slab (default 1e-9: finite state at every GPU count)")
    ap.add_argument("--time-block", type=int, default=0,
                    help="full steps fused per HBM pass, dividing --steps (0: the fastest dividing it)")
    ap.add_argument("--schedule", choices=["pipelined", "aligned"], default="pipelined",
                    help="staggered segments (exact starts) or aligned segments with deferred correction")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--side-legs", type=int, default=1,
                    help="1: also time the T=1 (HBM-bound) pass, the overflowing dt = 1e-3 state and the other variant")
    ap.add_argument("--material-steps", type=int, default=3,
                    help="timed steps of the material-coupled run reported under 'material' (0: skip)")
    # rehearsal of the multi-rank path on a one-GPU box: every rank on cuda:0, gloo
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl", help=argparse.SUPPRESS)
    ap.add_argument("--share-device", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    try:
        mode = launch_mode(args.gpus, os.environ)
    except ValueError as e:
        print(f"bench.py: {e}", file=sys.stderr)
        sys.exit(2)
    if mode == "spawn":  # no launcher: this process starts the ranks and touches no GPU
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))

    import torch
    import torch.distributed as dist
    import rtsn

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.share_device else int(os.environ.get("LOCAL_RANK", "0"))
    device = torch.device("cuda", local)
    if world > 1:
        torch.cuda.set_device(local)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")

    info = shard(args.scaling, args.groups, world, rank)
    p = dict(slab_params(info[0], args.variant, N=args.cells), dt=args.dt)
    dirs = direction_shard(args.scaling, args.groups, p["M"], world, rank)
    if dirs:  # fewer groups than ranks: all groups, a block of direction pairs per rank
        info = (args.groups, 0, args.groups)
    solver = make_solver(p, local, info, dirs)
    if args.time_block:
        solver.time_block = args.time_block
    solver.pipeline = 1 if args.schedule == "pipelined" else 0  # 1: pipelined when the run fills it
    # exactly K timed steps: the time block is --time-block, or the fastest supported one
    # dividing K; the handle re-sizes its segments for that block
    steps = args.steps if args.steps > 0 else 2 * (args.time_block or DEFAULT_TIME_BLOCK)
    tb = choose_time_block(steps, args.time_block)
    solver.time_block = tb
    # Warmup: at least W steps, and always whole passes that fill the pipeline (segments
    # per line passes: every segment position running, one pass apart), so that the K timed
    # steps are the schedule's steady state whatever W the caller asks for; the steps run
    # are reported as "warmup" (W as "warmup_requested").
    fill = solver.sweep_geometry()[1] * tb if solver.pipeline else tb
    warmup = warmup_steps(args.warmup, fill, tb)
    shards = [shard(args.scaling, args.groups, world, r)[1:] for r in range(world)]
    solver_tb = solver.time_block
    line, _, gathered = run_rank(solver, p, steps, warmup, world, device, info, args.scaling, shards, dirs=dirs)
    line["warmup_requested"] = args.warmup if args.warmup >= 0 else None
    # one RCCL communicator behind the C ABI for the rest of the run (the gather cross-check
    # on N > 1 GPUs, the material leg's per-step all-reduce)
    comm, comm_error = (open_comm(world, rank, local, device) if (world > 1 or args.material_steps > 0)
                        else (None, None))
    # environment variables the library or this script reads (test and diagnostic hooks):
    # reported so that a run under any of them is visible in its line
    line["rtsn_env"] = {k: v for k, v in sorted(os.environ.items()) if k.startswith("RTSN_")}
    line["launcher"] = os.environ.get("RTSN_BENCH_LAUNCHER", "torch.distributed.run" if world > 1 else "none")
    if comm is not None:
        try:
            line["rccl_nranks"] = comm.count  # ncclCommCount behind the C ABI
        except rtsn.RtError as e:
            line["rccl_nranks"] = f"rt_comm_count failed: {e}"
    if world > 1:
        if comm is not None:
            try:
                line["rt_comm_gather"] = rccl_gather_check(comm, solver, gathered, dirs)
            except rtsn.RtError as e:  # a bounded wait expired: the communicator is aborted
                comm.close()
                comm, comm_error = None, ("skipped (timeout): " if e.status == 7 else "") + str(e)
                line["rt_comm_gather"] = {"ok": None, "skipped": comm_error}
            comm, comm_error = comm_agree(comm, comm_error, world, device)
        else:
            line["rt_comm_gather"] = {"ok": None, "skipped": f"rt_comm unavailable: {comm_error}"}
    del gathered
    line["roofline"]["traffic"] = load_traffic(args.variant, solver.time_block,
                                               line["roofline"]["algorithmic_bytes_per_launch"])
    solver.close()  # frees the sweep's state before the next run allocates its own
    if args.side_legs:
        pv = dict(p, variant=args.variant)
        line["hbm_pass_t1"] = side_leg(pv, info, world, device, local, args.scaling, 1,
                                       "same workload, one full step per pass: HBM-bound sweep", dirs)
        line["overflow_control"] = side_leg(dict(pv, dt=1e-3), info, world, device, local, args.scaling,
                                            solver_tb, "same workload at SURVEY's dt = 1e-3, where the reference's "
                                                       "BDF2 overflows the state to inf within the fill: not the "
                                                       "headline (inf arithmetic runs ~4% faster)", dirs)
        other = "corr" if args.variant == "v0" else "v0"
        # at most 1e-9: with the v/c correction on, the reference's BDF2 overflows the SL state
        # within the fill already at dt = 1e-7 (profiles/archive/r03o_bench.json)
        line[f"variant_{other}"] = side_leg(dict(slab_params(info[0], other, N=args.cells), variant=other,
                                                 dt=min(args.dt, 1e-9)), info,
                                            world, device, local, args.scaling, solver_tb,
                                            f"SURVEY §8(d) SL variant {other} (V = "
                                            f"{5.994 if other == 'corr' else 0.0}, v/c correction "
                                            f"{'on' if other == 'corr' else 'inactive'}), same timing", dirs)
    if args.material_steps > 0:
        try:
            line["material"] = run_material(p, info, world, device, local, args.material_steps, dirs, rank,
                                            comm, comm_error)
            # the same at 50 keV: emission stiffness ~1e5, beyond any explicit step
            line["material_hot"] = run_material(p, info, world, device, local, args.material_steps, dirs, rank,
                                                comm, comm_error, T0_keV=50.0)
        except rtsn.RtError as e:  # an rt_comm wait expired or RCCL failed: the side leg is skipped
            if comm is not None:   # (every rank raises: the collectives are the same on all)
                comm.close()
                comm = None
            line["material"] = {"skipped": ("timeout: " if e.status == 7 else "") + str(e)}
    if comm is not None:
        comm.close()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.variant, args.dt)
        line["reference_config"] = reference_config_timings()
    if rank == 0:
        line["llnl_slab_test"] = llnl_slab_test_rate(line.get("reference_config"))
    if rank == 0:
        line["process_wall_s"] = time.perf_counter() - T_PROCESS0
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
