"""The reference's executables on the MI355X path: bin/transfer (src/main.cc)
and bin/test_gray (tests/test_gray.cpp).

CSV text: main.cc:37-57 writes `file << mat << endl` with Eigen's default
IOFormat (Eigen/src/Core/IO.h print_matrix, Eigen 3.3/3.4 -- Eigen is absent
from this image, so the format is restated below from its published
algorithm): stream precision 6 (printf "%.6g"), every coefficient
right-aligned to the widest one, " " between coefficients, "\n" between rows;
a rank-3 Tensor prints as its dim0 x (rest) ColMajor matrix (Eigen
TensorIO.h).  `eigen_text` is that restatement; the CPU test pins the C++
writer (csrc/eigen_text.hpp) to it on edge values, the GPU test compares the
eight CSV files of a run with the oracle's numbers byte for byte.
"""
from __future__ import annotations

import os
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

from conftest import REPO, PRM_DIR

PKG = REPO / "radiative-transfer_amd"


def eigen_text(a: np.ndarray, left: bool = False) -> str:
    """`os << m << std::endl` for a 2-D array under Eigen's default IOFormat.
    left: the stream carries std::left (sticky) -- as std::cout does in the
    reference after its first setw/left table -- so the padding goes right."""
    a = np.atleast_2d(np.asarray(a, dtype=np.float64))
    s = [["%.6g" % v for v in row] for row in a]
    w = max(len(x) for row in s for x in row)
    pad = (lambda x: x.ljust(w)) if left else (lambda x: x.rjust(w))
    return "\n".join(" ".join(pad(x) for x in row) for row in s) + "\n"


def tensor_text(psi: np.ndarray, left: bool = False) -> str:
    """Eigen::Tensor<double,3>(M,G,N): dim0 x (G*N) ColMajor view."""
    M, G, N = psi.shape
    return eigen_text(psi.transpose(0, 2, 1).reshape(M, N * G), left)


DRIVER = r"""
#include "eigen_text.hpp"
#include <cstdio>
#include <cstdlib>
#include <vector>
int main(int argc, char **argv) {
  // argv: out rows cols v0 v1 ... (ColMajor)
  const size_t r = std::atol(argv[2]), c = std::atol(argv[3]);
  std::vector<double> v;
  for (int k = 4; k < argc; ++k) v.push_back(std::strtod(argv[k], nullptr));
  return rtamd::write_eigen_text(argv[1], v, r, c) ? 0 : 1;
}
"""


@pytest.fixture(scope="module")
def text_driver(tmp_path_factory):
    d = tmp_path_factory.mktemp("eigen_text")
    src = d / "drv.cpp"
    src.write_text(DRIVER)
    exe = d / "drv"
    subprocess.run(["g++", "-std=c++17", "-O1", f"-I{PKG / 'csrc'}", str(src), "-o", str(exe)], check=True)
    return exe


@pytest.mark.parametrize("rows,cols,vals", [
    (1, 1, [0.5]),
    (2, 3, [1.0, -2.5, 1e-300, 123456789.0, -0.0, 3.14159265358979]),
    (3, 1, [1e20, -1e-5, 7.0]),
    (1, 4, [0.1, 0.25, -1234567.0, 5e-324]),
    (2, 2, [999999.5, 1e6, 0.000123456789, -0.0001]),
])
def test_eigen_text_format(text_driver, tmp_path, rows, cols, vals):
    out = tmp_path / "m.csv"
    subprocess.run([str(text_driver), str(out), str(rows), str(cols)] + [repr(v) for v in vals], check=True)
    a = np.array(vals).reshape(cols, rows).T  # ColMajor input
    assert out.read_text() == eigen_text(a)


DRIVER_BIN = r"""
#include "eigen_text.hpp"
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <vector>
int main(int argc, char **argv) {
  // argv: in.bin out rows cols left -- doubles ColMajor from in.bin; left: std::left on the stream
  const size_t r = std::atol(argv[3]), c = std::atol(argv[4]);
  std::vector<double> v(r * c);
  FILE *f = std::fopen(argv[1], "rb");
  if (!f || std::fread(v.data(), sizeof(double), v.size(), f) != v.size()) return 2;
  std::fclose(f);
  std::ofstream os(argv[2]);
  if (std::atoi(argv[5])) os << std::left;
  rtamd::write_eigen_text(os, v.data(), r, c);
  os << std::endl;
  return os ? 0 : 1;
}
"""


def _c_g6(v: float) -> str:
    """printf("%.6g") as C prints it (Python drops the sign of a negative NaN)."""
    return ("-nan" if np.signbit(v) else "nan") if np.isnan(v) else "%.6g" % v


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("left", [False, True])
def test_eigen_text_random(tmp_path, seed, left):
    """The C++ writer on 4000 random coefficients per case -- random bit patterns (subnormals,
    huge, inf, nan of either sign), values at the 6-digit rounding edges, plain decimals --
    against the restatement: the default stream (the one-pass snprintf path) and a stream
    carrying std::left (the per-coefficient stream path), byte for byte."""
    rng = np.random.default_rng(7000 + seed)
    bits = rng.integers(0, 2**63, size=1500, dtype=np.uint64) | (rng.integers(0, 2, 1500, dtype=np.uint64) << 63)
    edge = np.array([999999.5, 9999995.0, 0.00099999995, 1e-5, 99999.95, 1e16, 1e-7, 123456.5, 5e-324, -0.0])
    vals = np.concatenate([bits.view(np.float64), rng.choice(edge, 500) * rng.choice([1, -1, 10, 0.1], 500),
                           np.round(rng.normal(0, 1e3, 2000), rng.integers(0, 9))])
    rows, cols = 40, 100
    src, exe = tmp_path / "drv.cpp", tmp_path / "drv"
    src.write_text(DRIVER_BIN)
    subprocess.run(["g++", "-std=c++17", "-O1", f"-I{PKG / 'csrc'}", str(src), "-o", str(exe)], check=True)
    (tmp_path / "in.bin").write_bytes(vals.astype("<f8").tobytes())
    out = tmp_path / "m.csv"
    subprocess.run([str(exe), str(tmp_path / "in.bin"), str(out), str(rows), str(cols), str(int(left))], check=True)
    a = vals.reshape(cols, rows).T
    s = [[_c_g6(v) for v in row] for row in a]
    w = max(len(x) for row in s for x in row)
    pad = (lambda x: x.ljust(w)) if left else (lambda x: x.rjust(w))
    assert out.read_text() == "\n".join(" ".join(pad(x) for x in row) for row in s) + "\n"


def test_tensor_text_layout():
    psi = np.arange(2 * 3 * 4, dtype=float).reshape(2, 3, 4)
    lines = tensor_text(psi).splitlines()
    assert len(lines) == 2 and len(lines[0].split()) == 12
    # column j = g + G*c holds psi(i, g, c)
    assert float(lines[1].split()[1 + 3 * 2]) == psi[1, 1, 2]


def _bin(name: str) -> Path:
    exe = PKG / "bin" / name
    if not exe.exists():
        pytest.skip(f"{exe} not built")
    return exe


def _run_tree(tmp_path: Path) -> Path:
    """build/ next to prm/, as the reference is run (tables from ../prm/)."""
    shutil.copytree(PRM_DIR, tmp_path / "prm")
    run = tmp_path / "build"
    run.mkdir()
    return run


@pytest.mark.gpu
@pytest.mark.parametrize("ranks", [None, "1"])
@pytest.mark.parametrize("name", ["llnl_slab_test", "single_group"])
def test_transfer_csv_files(oracle_mod, tmp_path, name, ranks):
    """The eight CSV files byte for byte; ranks "1": RTSN_RANKS=1 runs the multi-GPU path
    (a forked rank, its handle joined by a one-rank RCCL communicator, every result
    gathered through rt_comm_*) -- the one-GPU box's check of the code the N-GPU CLI runs."""
    run = _run_tree(tmp_path)
    prm = f"../prm/{name}.prm"
    env = dict(os.environ)
    if ranks:
        env["RTSN_RANKS"] = ranks
    r = subprocess.run([str(_bin("transfer")), prm], cwd=run, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith(f"filename: {prm}\n")

    q = oracle_mod.parse_prm(str(run / prm), table_dir=str(tmp_path / "prm") + "/")
    s = oracle_mod.OracleSolver(q)
    s.solve()
    phi, F, phi_plus = s.moments()
    left, right = s.group_ends()
    N = q["N"]
    x = (np.arange(N) + 0.5) * q["dx"]
    expect = {
        "phi.csv": eigen_text(phi), "phi_plus.csv": eigen_text(phi_plus), "F.csv": eigen_text(F),
        "psi.csv": tensor_text(s.psi()), "x.csv": eigen_text(x[:, None]),
        "e_ave.csv": eigen_text(s.groups()["e_ave"][:, None]),
        "left_ends.csv": eigen_text(left[:, None]), "right_ends.csv": eigen_text(right[:, None]),
    }
    for fname, text in expect.items():
        got = (run / fname).read_text()
        if fname == "F.csv":
            # F cancels to ~1e-17 in equilibrium: its digits are rounding noise, so
            # compare the layout and the values to the scale of the summands
            g = np.loadtxt(run / fname, ndmin=2)
            assert g.shape == F.shape
            np.testing.assert_allclose(g, F, rtol=1e-5, atol=1e-10 * np.abs(phi).max())
        else:
            assert got == text, fname


def cpp_g(v: float, showpos: bool = False) -> str:
    """`os << double` at the default stream precision (printf %g)."""
    return ("%+g" if showpos else "%g") % v


def expected_solver_log(q: dict, orc) -> str:
    """The reference's solver-side stdout (solver.cpp:55-187, 296-312, 620-625;
    correction.cpp:301), restated from its iostream calls, up to the balance
    lines (:278-282, compared numerically by the caller)."""
    mu, wt = orc.quad()
    gr = orc.groups()
    out = ["Solver constructor."]
    out.append(f"{'Mu':<16}{'Wt':<16}")
    out.append(f"{'--':<16}{'--':<16}")
    out += [f"{cpp_g(m, True):<16}{cpp_g(w, True):<16}" for m, w in zip(mu, wt)]
    out.append("")
    out.append(f"{'Group Index':<13}{'Average Energy':<16}{'Upper Energy':<14}{'Group Width':<13}")
    out.append(f"{'-----------':<13}{'(keV)---------':<16}{'(keV)-------':<14}{'(keV)------':<13}")
    for g in range(q["G"]):
        out.append(f"{g:<13}{cpp_g(gr['e_ave'][g]):<16}{cpp_g(gr['e_edge'][g + 1]):<14}"
                   f"{cpp_g(gr['e_edge'][g + 1] - gr['e_edge'][g]):<13}")
    out += ["", "", "Correction constructor."]
    text = "\n".join(out) + "\n"
    # std::left is still set on cout from the tables above, so Eigen pads on the right
    text += "B: " + eigen_text(gr["B"][:, None], left=True)
    psi0 = np.repeat(np.repeat(gr["B"][None, :, None], q["M"], 0), q["N"], 2)
    text += "psi_mat_ref: " + tensor_text(psi0, left=True)
    text += "end solver constructor\n"
    if q["use_mg_equilib"]:
        src = orc.psi_source()
        for i in range(q["M"]):
            for g in range(q["G"]):
                text += f"source condition for mu: {cpp_g(mu[i])} and group {g}: {cpp_g(src[i, g])}\n"
    its = q["max_timesteps"] * (4 if q["ts_method"] == 3 else 1)
    for it in range(its):
        if q["ts_method"] != 3 or it % 4 == 0:
            text += f"============= Timestep: {it} =============\n"
    return text


@pytest.mark.gpu
@pytest.mark.parametrize("ranks", [None, "1"])
@pytest.mark.parametrize("name", ["llnl_slab_test", "multi_group_equilibrium"])
def test_transfer_stdout(oracle_mod, tmp_path, name, ranks):
    """transfer prints what the reference prints, in its formats (also through the
    multi-GPU path with one rank)."""
    run = _run_tree(tmp_path)
    prm = f"../prm/{name}.prm"
    env = dict(os.environ)
    if ranks:
        env["RTSN_RANKS"] = ranks
    r = subprocess.run([str(_bin("transfer")), prm], cwd=run, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr
    q = oracle_mod.parse_prm(str(run / prm), table_dir=str(tmp_path / "prm") + "/")
    orc = oracle_mod.OracleSolver(q)
    orc.solve()
    start = r.stdout.index("Solver constructor.")
    bal_at = r.stdout.index("sources: ")
    assert r.stdout[:start] == expected_display(q, tmp_path / "prm" / f"{name}.prm")
    assert r.stdout[start:bal_at] == expected_solver_log(q, orc)
    # balance lines: sources / sinks / balance per group; balance = |sinks - sources| /
    # sources cancels, so compare the numbers, not their 6-digit text
    lines = r.stdout[bal_at:].splitlines()
    bal_o = orc.balance()
    for g in range(q["G"]):
        s_line, k_line, b_line = lines[3 * g: 3 * g + 3]
        assert s_line.startswith("sources: ") and k_line.startswith("sinks: ")
        assert b_line.startswith(f"balance at ({g}): ")
        assert float(b_line.split(": ")[1]) == pytest.approx(bal_o[g], rel=1e-4, abs=1e-12)
    assert r.stdout.startswith(f"filename: {prm}\n") and len(lines) == 3 * q["G"]


def prm_text_value(path: Path, key: str) -> str:
    """The raw text of `key=` in a .prm (kaityo256/param: key at column 0, value to the end
    of the line, first occurrence wins), as get<string> returns it."""
    for line in path.read_text().splitlines():
        if line.startswith(key + "="):
            return line[len(key) + 1:]
    return "NA"


def expected_display(q: dict, prm: Path) -> str:
    """What the reference prints from main.cc:78 through display_input_quantities: the
    filename line, get_parameters' own prints while it reads the tables
    (ParameterHandler.cpp:165, 191, 195) and display_input_quantities
    (ParameterHandler.cpp:20-96), restated from its iostream calls.  `cout << double` is
    %g; `cout << psi_source` is an Eigen MatrixXd (M, G) under the default IOFormat."""
    bc = {0: "vacuum", 2: "reflective", 1: "source"}
    out = f"filename: ../prm/{prm.name}\n"
    bounds = "../prm/" + prm_text_value(prm, "filename_group_bounds")
    kappa = "../prm/" + prm_text_value(prm, "filename_group_kappa")
    if q["have_group_bounds"]:
        out += f"specified group bounds: {bounds}\n"
    if q["have_group_kappa"]:
        out += f"group_kappa size: {q['G']}\nspecified group opacities filename: {kappa}\n"
    out += "\n--- Input Parameters ---\n"
    out += f"Angle quadrature order: {q['M']}\nNumber of energy groups: {q['G']}\n"
    if q["have_group_bounds"]:
        out += f"Group bounds (keV) specified in file: {bounds}\n"
    else:
        out += ("Group bounds (keV) will be computed logarithmically, with first group edge at "
                f"{cpp_g(q['efirst'])} and last group edge at {cpp_g(q['elast'])}\n")
    out += f"Slab thickness (cm): {cpp_g(q['X'])}\nNumber of cells: {q['N']}\n"
    out += f"Material density (g/cm^3): {cpp_g(q['rho'])}\n"
    if q["have_group_kappa"]:
        out += f"Group opacities (cm^2/g) specified in file: {kappa}\n"
    else:
        out += f"Group opacities will be set to the constant grey opacity (cm^2/g): {cpp_g(q['kappa_grey'])}\n"
    out += f"Material temperature (keV): {cpp_g(q['T'])}\nMaterial velocity (cm/shake): {cpp_g(q['V'])}\n"
    out += f"Beta: {cpp_g(q['V'] / 299.792458)}\n"
    out += "Right boundary condition: "
    if q["bc_right"] not in bc:
        return out + "Incorrect boundary conditions provided.\n"
    out += bc[q["bc_right"]] + "\n"
    out += "Left boundary condition: "
    if q["bc_left"] not in bc:
        return out + "Incorrect boundary conditions provided.\n\n"
    out += bc[q["bc_left"]] + "\n\n"
    return out + "Psi_source: \n" + eigen_text(q["psi_source"])


DISPLAY_EDITS = {  # edge cases of the display: (golden .prm, {key: new line text})
    "widths": ("template.prm", {"psi_source": "psi_source=1.5 -2 1e-7 100 0.333333333 7"}),
    "bad_right_bc": ("template.prm", {"bc_right_indicator": "bc_right_indicator=7"}),
    "bad_left_bc": ("single_group.prm", {"bc_left_indicator": "bc_left_indicator=-1"}),
    "tables_on": ("template.prm", {"have_group_bounds": "have_group_bounds=true",
                                   "have_group_absorption_opacities": "have_group_absorption_opacities=true"}),
    "beta": ("multi_group_equilibrium.prm", {"V": "V=5.994"}),
}


@pytest.mark.parametrize("case", sorted(p.name for p in PRM_DIR.glob("*.prm")) + sorted(DISPLAY_EDITS))
def test_transfer_display_text(oracle_mod, tmp_path, case):
    """Row f-2: `transfer` prints the reference's input display (ParameterHandler.cpp:20-96,
    with get_parameters' table prints and main.cc's filename line) byte for byte, for
    every golden .prm (table / no-table branches, mg_equilib) and edited copies (psi_source
    of mixed widths, incorrect boundary indicators, both tables on, V != 0).  The display
    precedes any device call, so this runs without a GPU (there the solver then reports
    that no device exists; on the GPU box the stdout continues with the solver's log)."""
    run = _run_tree(tmp_path)
    name = case
    if case in DISPLAY_EDITS:
        base, edits = DISPLAY_EDITS[case]
        lines = (tmp_path / "prm" / base).read_text().splitlines()
        for key, text in edits.items():
            hit = [k for k, l in enumerate(lines) if l.startswith(key + "=")]
            if hit:
                lines[hit[0]] = text
            else:
                lines.append(text)
        name = f"edit_{case}.prm"
        (tmp_path / "prm" / name).write_text("\n".join(lines) + "\n")
    prm = tmp_path / "prm" / name
    r = subprocess.run([str(_bin("transfer")), f"../prm/{name}"], cwd=run, capture_output=True, text=True,
                       timeout=120)
    q = oracle_mod.parse_prm(str(prm), table_dir=str(tmp_path / "prm") + "/")
    got = r.stdout.split("Solver constructor.")[0]
    assert got == expected_display(q, prm)


@pytest.mark.gpu
def test_transfer_validation_assert(tmp_path):
    """include_validation with the LLNL tabulated opacities: the reference prints
    the failed emission check and its assert aborts (llnl_slab_test.prm:54)."""
    run = _run_tree(tmp_path)
    src = (tmp_path / "prm" / "llnl_slab_test.prm").read_text()
    (tmp_path / "prm" / "llnl_validate.prm").write_text(src.replace("include_validation=false",
                                                                    "include_validation=true"))
    r = subprocess.run([str(_bin("transfer")), "../prm/llnl_validate.prm"], cwd=run, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode in (-6, 134), (r.returncode, r.stderr)
    assert "Total Emission = " in r.stdout and "kappa_ref*acT^4 = " in r.stdout
    assert "Assertion" in r.stderr


@pytest.mark.gpu
def test_gray_binary(tmp_path):
    run = _run_tree(tmp_path)
    env = dict(os.environ, TRANSFER_DIR=str(tmp_path) + "/")
    r = subprocess.run([str(_bin("test_gray"))], cwd=run, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr


def test_transfer_ranks_fail_cleanly_without_gpu(tmp_path):
    """RTSN_RANKS=n forks n ranks; when rank 0 cannot make the communicator id (here: no
    GPU, ncclGetUniqueId needs one) it exits non-zero, the other ranks read end-of-file on
    their pipe and exit too, and the parent returns the failure -- no rank is left waiting."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("the failure path needs a host without a GPU")
    run = _run_tree(tmp_path)
    r = subprocess.run([str(_bin("transfer")), "../prm/llnl_slab_test.prm"], cwd=run, capture_output=True, text=True,
                       timeout=60, env=dict(os.environ, RTSN_RANKS="3"))
    assert r.returncode != 0
    assert "rt_comm_unique_id" in r.stderr


def test_transfer_ranks_stop_survivors_on_failure(tmp_path):
    """A rank that fails after the fork must not leave the others blocked (in
    ncclCommInitRank or a collective) with the parent waiting on them: the parent reaps
    whichever rank ends first and stops the rest.  RTSN_FAULT_STALL_RANK=2 makes rank 2
    block right after the fork; rank 0 fails (no GPU here, so no communicator id) and the
    run must still end, non-zero, well within the timeout."""
    import time
    import torch
    if torch.cuda.is_available():
        pytest.skip("the failure path needs a host without a GPU")
    run = _run_tree(tmp_path)
    t0 = time.perf_counter()
    r = subprocess.run([str(_bin("transfer")), "../prm/llnl_slab_test.prm"], cwd=run, capture_output=True, text=True,
                       timeout=60, env=dict(os.environ, RTSN_RANKS="3", RTSN_FAULT_STALL_RANK="2"))
    assert r.returncode != 0
    assert time.perf_counter() - t0 < 30


@pytest.mark.gpu
def test_transfer_ranks_missing_device_fails_cleanly(tmp_path):
    """RTSN_RANKS=2 on a one-GPU box: rank 1's device (RTSN_DEVICE_BASE + 1) does not exist,
    so its rt_create_from_params fails after the id hand-off while rank 0 waits in
    ncclCommInitRank for it.  The parent stops rank 0 and returns the failure instead of
    hanging."""
    import torch
    if torch.cuda.device_count() != 1:
        pytest.skip("needs exactly one visible GPU")
    run = _run_tree(tmp_path)
    r = subprocess.run([str(_bin("transfer")), "../prm/llnl_slab_test.prm"], cwd=run, capture_output=True, text=True,
                       timeout=90, env=dict(os.environ, RTSN_RANKS="2", RTSN_QUIET="1"))
    assert r.returncode != 0
    assert "rt_create_from_params" in r.stderr
