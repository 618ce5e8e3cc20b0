"""Host-side checks of librtsn.so that need no GPU: the library loads and
exports every entry point of include/rtsn.h, and its host logic (the .prm
reader with the kaityo256/param quirks, GLQuad, Planck) agrees with the
oracle's restatement of the reference -- bitwise, since both run the
reference's arithmetic on the same host."""
import ctypes
import subprocess

import numpy as np
import pytest

from conftest import PRM_DIR, REPO

LIB = REPO / "radiative-transfer_amd" / "lib" / "librtsn.so"


def test_library_exports_every_header_symbol(rtsn_mod):
    assert LIB.exists(), "build librtsn.so first (__graft_entry__.build())"
    out = subprocess.run(["nm", "-D", "--defined-only", str(LIB)], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    declared = rtsn_mod.exported_symbols()
    assert len(declared) >= 25
    missing = [s for s in declared if s not in exported]
    assert not missing, missing
    ctypes.CDLL(str(LIB))  # loads (links against libamdhip64 only)


def test_library_is_gfx950_code(rtsn_mod):
    """The fat binary carries gfx950 code objects (and nothing else to fall back to)."""
    blob = LIB.read_bytes()
    assert b"gfx950" in blob
    for other in (b"gfx942", b"gfx90a", b"sm_"):
        assert other + b"\x00" not in blob or other == b"sm_"


def test_getenv_only_documented():
    """the shipped library and executables read only the environment
    variables include/rtsn.h documents (kernel forms and segmentation are ABI setters), and
    no build-time tuning macro has a branch the tested build does not compile (no
    #ifndef RT_... overrides, no #if on one)."""
    import re
    src = REPO / "radiative-transfer_amd" / "csrc"
    allowed = {"TRANSFER_DIR", "RT_TABLE_DIR", "RTSN_QUIET", "RTSN_COMM_TIMEOUT_S", "RTSN_POOL_MB",
               "RTSN_DEVICE_BASE", "RTSN_FAULT_STALL_RANK", "RTSN_RANKS"}
    read, knobs = set(), []
    for f in sorted(src.iterdir()):
        text = f.read_text()
        read |= set(re.findall(r'getenv\("([A-Z_0-9]+)"\)', text))
        knobs += [f"{f.name}: {m}" for m in re.findall(r"#\s*(?:ifndef|ifdef|if)\s+(RT_\w+)", text)]
    assert read <= allowed, read - allowed
    header = (REPO / "include" / "rtsn.h").read_text()
    for name in read:
        assert name in header, name
    assert not knobs, knobs


def _params_equal(ph, ref):
    for k in ("M", "G", "N", "efirst", "elast", "X", "rho", "kappa_grey", "T", "V", "dt", "max_timesteps"):
        assert ph.params[k] == ref[k], k
    assert ph.params["bc_left_indicator"] == ref["bc_left"]
    assert ph.params["bc_right_indicator"] == ref["bc_right"]
    assert ph.params["use_mg_equilib"] == ref["use_mg_equilib"]
    assert ph.params["use_correction"] == ref["use_correction"]
    assert ph.params["ts_method"] == ref["ts_method"]
    assert ph.params["include_validation"] == ref["include_validation"]
    np.testing.assert_array_equal(ph.params["psi_source"], ref["psi_source"])
    for a, b in (("group_bounds", "group_bounds"), ("group_kappa", "group_kappa")):
        if ref[b] is None:
            assert ph.params[a] is None
        else:
            np.testing.assert_array_equal(ph.params[a], ref[b])


@pytest.mark.parametrize("name", ["single_group.prm", "multi_group_equilibrium.prm", "llnl_slab_test.prm",
                                  "llnl_slab_test_uncapped.prm", "default.prm", "template.prm"])
def test_prm_reader_matches_oracle(rtsn_mod, oracle_mod, name):
    ph = rtsn_mod.ParameterHandler(PRM_DIR / name, table_dir=PRM_DIR)
    ref = oracle_mod.parse_prm(PRM_DIR / name, table_dir=PRM_DIR)
    _params_equal(ph, ref)


def test_prm_quirks(rtsn_mod, tmp_path):
    """param.h:62-75 / param.cpp:4-66 semantics."""
    f = tmp_path / "q.prm"
    f.write_text("\n".join([
        "# comment line",
        " # not a comment: key is ' # not a comment: key is ' -> ignored",
        "M=4                    # trailing comment after a number is fine",
        "M=8",                      # duplicate: first one wins
        "G=2",
        "use_correction=true   # trailing text -> false (exact match only)",
        "include_validation=Yes",
        "use_mg_equilib=TRUE",      # not one of yes/Yes/true/True
        "N = 7",                    # key is 'N ' -> N stays at its default 100
        "psi_source=1.5 2.5 3 4.25 7 8 9 10 # stops at '#'",
        "dt=2.5e-3xyz",
        "bc_left_indicator=1",
    ]) + "\n")
    ph = rtsn_mod.ParameterHandler(f, table_dir=tmp_path)
    assert ph.get_M() == 4
    assert ph.get_G() == 2
    assert ph.get_N() == 100
    assert ph.get_use_correction() == 0
    assert ph.get_validation() == 1
    assert ph.get_use_mg_equilib() == 0
    assert ph.get_dt() == 2.5e-3
    np.testing.assert_array_equal(ph.params["psi_source"], np.array([[1.5, 2.5], [3, 4.25], [7, 8], [9, 10]]))


def test_prm_missing_file_gives_defaults(rtsn_mod, tmp_path):
    ph = rtsn_mod.ParameterHandler(tmp_path / "nope.prm", table_dir=tmp_path)
    assert not ph.prm_found
    assert (ph.get_M(), ph.get_G(), ph.get_N(), ph.get_ts_method(), ph.get_max_timesteps()) == (2, 1, 100, 3, 1000)
    assert ph.get_bc_left_indicator() == 2 and ph.get_bc_right_indicator() == 1


def test_prm_errors(rtsn_mod, tmp_path):
    f = tmp_path / "bad.prm"
    f.write_text("M=abc\n")
    with pytest.raises(rtsn_mod.RtError) as e:
        rtsn_mod.ParameterHandler(f, table_dir=tmp_path)
    assert e.value.status == 2  # RT_ERR_PARSE (std::stoi throws)
    f.write_text("G=3\nhave_group_bounds=true\nfilename_group_bounds=missing.txt\n")
    with pytest.raises(rtsn_mod.RtError) as e:
        rtsn_mod.ParameterHandler(f, table_dir=tmp_path)
    assert e.value.status == 1  # RT_ERR_IO (exit(1) in the reference)
    (tmp_path / "b.txt").write_text("0.1 0.2\n")
    f.write_text("G=3\nhave_group_bounds=true\nfilename_group_bounds=b.txt\n")
    with pytest.raises(rtsn_mod.RtError) as e:
        rtsn_mod.ParameterHandler(f, table_dir=tmp_path)
    assert e.value.status == 3  # count assert


@pytest.mark.parametrize("M", [2, 4, 16, 64, 128])
def test_quadrature_bitwise(rtsn_mod, oracle_mod, M):
    mu, wt = rtsn_mod.quadrature(M)
    mo, wo = oracle_mod.glquad(M)
    assert np.array_equal(mu, mo) and np.array_equal(wt, wo)


@pytest.mark.parametrize("name", ["llnl_slab_test.prm", "multi_group_equilibrium.prm", "single_group.prm"])
def test_planck_bitwise(rtsn_mod, oracle_mod, name):
    p = oracle_mod.parse_prm(PRM_DIR / name, table_dir=PRM_DIR)
    s = oracle_mod.OracleSolver(p)
    g = s.groups()
    B, dB = rtsn_mod.planck_groups(p["T"], g["e_edge"])
    assert np.array_equal(B, g["B"])
    assert np.array_equal(dB, g["dBdT"])


def test_solver_without_gpu_fails_loudly(rtsn_mod):
    from conftest import gpu_available
    if gpu_available():
        pytest.skip("a GPU is present")
    with pytest.raises(rtsn_mod.RtError) as e:
        rtsn_mod.Solver(rtsn_mod.params_default())
    assert e.value.status == 6  # RT_ERR_DEVICE: no CPU fallback


def test_host_code_under_sanitizers(tmp_path):
    """The library's host code (prm reader, Planck/GLQuad/correction tables,
    equilibrium sources) over every golden .prm under ASan + UBSan
    (tools/host_sanitize.cpp; GPU sanitizers are not available)."""
    import shutil
    import subprocess
    if not shutil.which("g++"):
        pytest.skip("no g++")
    exe = tmp_path / "host_sanitize"
    csrc = REPO / "radiative-transfer_amd" / "csrc"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                    "-fno-sanitize-recover=all", f"-I{csrc}", str(REPO / "tools" / "host_sanitize.cpp"),
                    str(csrc / "prm.cpp"), str(csrc / "physics.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), str(PRM_DIR) + "/"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "6 files, 0 bad" in r.stdout and "ERROR" not in r.stderr


def test_cell_maps_and_head_map(tmp_path):
    """The per-line affine maps the kernels run instead of the reference's cell algebra
    (cell.hpp cell_map, tools/cell_map_check.cpp) under ASan + UBSan: for 2000 random lines per
    scheme the probe finds the structural pattern, the reflective head cell's own map equals
    the line's map bitwise in the rows the wavefront lanes share (head_map_first), and both
    maps reproduce cell_step / cell_step_maybe_head to rounding."""
    import shutil
    import subprocess
    if not shutil.which("g++"):
        pytest.skip("no g++")
    exe = tmp_path / "cell_map_check"
    csrc = REPO / "radiative-transfer_amd" / "csrc"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                    "-fno-sanitize-recover=all", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", f"-I{csrc}",
                    str(REPO / "tools" / "cell_map_check.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert ", 0 failures," in r.stdout and "ERROR" not in r.stderr


def test_c_client_links_and_runs(tmp_path):
    """include/rtsn.h compiles as C99 and librtsn.so links from C: host-only entry
    points work, rt_create_from_params reports RT_ERR_DEVICE without a gfx950
    (or succeeds on one)."""
    import shutil
    import subprocess
    if not shutil.which("gcc") or not LIB.exists():
        pytest.skip("no gcc or library")
    exe = tmp_path / "abi_check"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-pedantic", f"-I{REPO / 'include'}",
                    str(REPO / "tests" / "c_abi" / "abi_check.c"), "-o", str(exe), f"-L{LIB.parent}", "-lrtsn",
                    f"-Wl,-rpath,{LIB.parent}", "-lm"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert r.stdout.strip().endswith("ok")


def test_direction_shard_argument_checks(rtsn_mod):
    """rt_create_direction_shard validates the pair range before touching the device
    (RT_ERR_PARAM), and like every constructor fails loudly without a gfx950 device."""
    p = rtsn_mod.params_default()
    p.update(M=8)
    for lo, hi in ((-1, 2), (2, 2), (3, 1), (0, 5)):
        with pytest.raises(rtsn_mod.RtError) as e:
            rtsn_mod.Solver(p, d_lo=lo, d_hi=hi)
        assert e.value.status == 3  # RT_ERR_PARAM
    with pytest.raises(rtsn_mod.RtError) as e:
        rtsn_mod.Solver(p, d_lo=1, d_hi=3)
    assert e.value.status == 6  # RT_ERR_DEVICE


def test_plan_time_block(rtsn_mod):
    """rt_solve's run-length-aware block on the SL slab's geometry (rt_plan_time_block: the
    schedule model of rt_plan_schedule at N = 1e6, S64, 128 groups, 256 CUs) picks the
    measured fastest whole runs of the finite-state grid (profiles/archive/r03l_grid128.jsonl): 300
    steps T = 20 (2659 ms; T = 40 with its 20 aligned remainder steps 2838-2899), 1000 steps
    T = 40 (8139-8188 ms; T = 20 8524-8573); every choice has at least one whole pass."""
    plan = rtsn_mod.plan_time_block
    assert plan(3, 300) == 20
    assert plan(3, 1000) == 40
    assert plan(3, 4000) == 40
    assert plan(3, 96) == 24 and plan(3, 100) in (20, 24)
    assert plan(3, 2) == 16  # no whole pass of any block: the default, run as aligned passes
    for n in range(8, 2000, 7):  # always a pipelined block with at least one whole pass
        T = plan(3, n)
        assert T in (8, 16, 20, 24, 32, 40) and n // T >= 1
    assert plan(1, 1000) == 16 and plan(2, 1000) == 16  # BE / CN keep the default
    with pytest.raises(rtsn_mod.RtError):
        plan(4, 10)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["llnl_slab_test.prm", "single_group.prm", "multi_group_equilibrium.prm"])
def test_c_client_solves_against_oracle(oracle_mod, tmp_path, name):
    """The boundary from C, on the GPU: tests/c_abi/abi_solve.c (C99, links librtsn.so only)
    runs rt_create(.prm) + rt_solve and reads psi, phi, F, phi_plus, the group ends,
    balance and e_ave through the host getters in the reference's ColMajor layouts; every
    array against the oracle (the reference's algorithm) per group to 1e-10, F against its
    summands' scale, e_ave exactly."""
    import subprocess
    from parity import flux_rel, per_group_rel
    exe = tmp_path / "abi_solve"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-pedantic", f"-I{REPO / 'include'}",
                    str(REPO / "tests" / "c_abi" / "abi_solve.c"), "-o", str(exe), f"-L{LIB.parent}", "-lrtsn",
                    f"-Wl,-rpath,{LIB.parent}"], check=True)
    out = tmp_path / "out.bin"
    prm = REPO / "tests" / "golden" / "prm"
    r = subprocess.run([str(exe), str(prm / name), str(prm) + "/", str(out)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    o = oracle_mod.OracleSolver(oracle_mod.parse_prm(prm / name, table_dir=prm))
    o.solve()
    M, G, N = (int(x.split("=")[1]) for x in r.stdout.split())
    a = np.fromfile(out)
    MGN, GN = M * G * N, G * N
    psi = a[:MGN].reshape(N, G, M).transpose(2, 1, 0)  # ColMajor (M, G, N)
    phi, F, pp = (a[MGN + k * GN:MGN + (k + 1) * GN].reshape(N, G).T for k in range(3))
    rest = a[MGN + 3 * GN:]
    left, right, bal, e_ave = (rest[k * G:(k + 1) * G] for k in range(4))
    mu, wt = o.quad()
    phi_o, F_o, pp_o = o.moments()
    assert per_group_rel(psi, o.psi(), 1) <= 1e-10
    assert per_group_rel(phi, phi_o, 0) <= 1e-10 and per_group_rel(pp, pp_o, 0) <= 1e-10
    assert flux_rel(F, F_o, o.psi(), mu, wt) <= 1e-10
    l_o, r_o = o.group_ends()
    assert np.allclose(left, l_o, rtol=1e-10, atol=0) and np.allclose(right, r_o, rtol=1e-10, atol=0)
    assert np.allclose(bal, o.balance(), rtol=1e-9, atol=1e-12)
    assert np.array_equal(e_ave, o.groups()["e_ave"])


def test_host_workers_survive_fork(rtsn_mod):
    """The Planck table runs on persistent host workers (physics.cpp HostPool); a child forked
    after they started has none of their threads and must compute the same table alone,
    not wait for workers that do not exist (a bounded wait here)."""
    import os
    import time
    from conftest import PRM_DIR
    ph = rtsn_mod.ParameterHandler(PRM_DIR / "llnl_slab_test.prm", table_dir=PRM_DIR)
    e = ph.params["group_bounds"]
    B, dB = rtsn_mod.planck_groups(1.0, e)
    pid = os.fork()
    if pid == 0:  # the child: same table, then exit with the verdict
        B2, dB2 = rtsn_mod.planck_groups(1.0, e)
        os._exit(0 if (B2 == B).all() and (dB2 == dB).all() else 3)
    t0 = time.time()
    while time.time() - t0 < 60:
        done, status = os.waitpid(pid, os.WNOHANG)
        if done:
            assert os.waitstatus_to_exitcode(status) == 0
            return
        time.sleep(0.05)
    os.kill(pid, 9)
    os.waitpid(pid, 0)
    raise AssertionError("the forked child hung in the host worker pool")
