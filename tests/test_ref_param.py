"""The .prm reader pinned against the REFERENCE's own reader (CPU).

oracle/_ref/ref_param is the reference's kaityo256/param library
(src/param.cpp + include/param.h), compiled unmodified from /root/reference by
`make -C oracle ref` (build() does it where the reference exists), driven
through the get<T>(key, default) calls of ParameterHandler::get_parameters
(src/ParameterHandler.cpp:100-212) by oracle/ref_param_driver.cpp.  Every
golden .prm and a set of edge-case files must parse the same through it, the
product's reader (radiative-transfer_amd/csrc/prm.cpp via rt_params_load) and
the oracle's (oracle/rt_oracle.c orc_parse_prm): same values bit for bit, and
an error status exactly where the reference terminates (std::stoi / std::stod
throwing) or would index psi_source out of range (Eigen assert).
"""
import math
import subprocess
from pathlib import Path

import numpy as np
import pytest

from conftest import PRM_DIR, REPO

REF = REPO / "oracle" / "_ref" / "ref_param"

pytestmark = pytest.mark.skipif(not REF.exists(), reason="oracle/_ref/ref_param not built (needs /root/reference)")

INTS = ("M", "G", "N", "bc_left_indicator", "bc_right_indicator", "ts_method", "max_timesteps")
DOUBLES = ("efirst", "elast", "X", "rho", "kappa_grey", "T", "V", "dt")
BOOLS = ("use_mg_equilib", "use_correction", "include_validation")


def ref_parse(path: Path) -> dict:
    r = subprocess.run([str(REF), str(path)], capture_output=True, text=True, timeout=30)
    out = {"psi": []}
    for line in r.stdout.splitlines():
        if not line.startswith("@"):
            continue  # param's own "Found <key> to be true." lines
        k, _, v = line[1:].partition("\t")
        if k.startswith("psi_source["):
            out["psi"].append(float(v))
        else:
            out[k] = v
    if out.get("status") != "ok":
        assert r.returncode != 0 and "terminate called" in r.stderr, (r.returncode, r.stderr)
        out["status"] = "throw"
    return out


def same_double(a: float, b: float) -> bool:
    return (math.isnan(a) and math.isnan(b)) or (a == b and math.copysign(1, a) == math.copysign(1, b))


def check(path: Path, rtsn_mod, oracle_mod):
    ref = ref_parse(path)
    M, G = int(ref.get("M", "2")), int(ref.get("G", "1"))
    over = len(ref["psi"]) > M * G  # psi_source(_m, _g) past the matrix: Eigen's index assert
    expect_error = ref["status"] == "throw" or over
    for name, parse in (("product", lambda: rtsn_mod.ParameterHandler(path, table_dir=PRM_DIR).params),
                        ("oracle", lambda: oracle_mod.parse_prm(path, table_dir=PRM_DIR))):
        if expect_error:
            with pytest.raises((rtsn_mod.RtError, oracle_mod.OracleError)):
                parse()
            continue
        got = parse()
        for k in INTS:
            key = {"bc_left_indicator": "bc_left", "bc_right_indicator": "bc_right"}.get(k, k) \
                if name == "oracle" else k
            assert got[key] == int(ref[k]), (name, k)
        for k in DOUBLES:
            assert same_double(got[k], float(ref[k])), (name, k, got[k], ref[k])
        for k in BOOLS:
            assert bool(got[k]) == (ref[k] == "1"), (name, k)
        assert (got["group_bounds"] is not None) == (ref["have_group_bounds"] == "1"), name
        assert (got["group_kappa"] is not None) == (ref["have_group_absorption_opacities"] == "1"), name
        want = np.zeros(M * G)
        if ref["use_mg_equilib"] != "1":
            want[:len(ref["psi"])] = ref["psi"]
        psi = np.asarray(got["psi_source"], dtype=np.float64).reshape(-1)
        assert psi.shape == want.shape and all(same_double(a, b) for a, b in zip(psi, want)), (name, psi, want)


@pytest.mark.parametrize("name", sorted(p.name for p in PRM_DIR.glob("*.prm")))
def test_golden_prm_files(rtsn_mod, oracle_mod, name):
    check(PRM_DIR / name, rtsn_mod, oracle_mod)


EDGE = {
    "spaces_in_key": "M = 4\nG=3\n",
    "first_duplicate_wins": "M=4\nM=6\nN=7\nN=9\n",
    "comment_column0_only": "#M=8\n M=6\nG=2 # trailing comment\n",
    "numeric_prefix": "N=12abc\nX=0.5cm\nts_method=1.9\nmax_timesteps=0x10\n",
    "no_numeric_prefix_int": "N=abc\n",
    "empty_int": "M=\n",
    "int_overflow": "max_timesteps=99999999999\n",
    "int_limits": "max_timesteps=2147483647\nbc_left_indicator=-2147483648\n",
    "double_overflow": "dt=1e999\n",
    "double_subnormal": "dt=1e-320\n",
    "double_underflow_zero": "V=1e-400\n",
    "double_smallest_normal": "dt=2.2250738585072014e-308\n",
    "double_specials": "V=inf\nT=nan\nrho=0x1p-2\nkappa_grey=-0\n",
    "double_exponent_without_digits": "dt=1e\nX=2.5e+\n",
    "double_no_prefix": "V=abc\n",
    "bools": "use_mg_equilib=Yes\nuse_correction=YES\ninclude_validation=true \n",
    "bools_true": "use_correction=True\ninclude_validation=yes\n",
    "value_with_equals": "N=4=5\nG=2\n",
    "crlf": "M=4\r\nG=3\r\nuse_correction=yes\r\nV=0.5\r\n",
    "psi_source_full": "M=2\nG=2\nbc_left_indicator=1\npsi_source=1 2 3 4\n",
    "psi_source_partial": "M=4\nG=2\npsi_source=1.5 -2 .5 5.\n",
    "psi_source_bad_token": "M=2\nG=2\npsi_source=1 2 abc 4\n",
    "psi_source_exponent_without_digits": "M=2\nG=2\npsi_source=1e 2\n",
    "psi_source_inf_nan": "M=2\nG=2\npsi_source=inf 2\n",
    "psi_source_hex": "M=2\nG=2\npsi_source=0x10 1\n",
    "psi_source_overflow": "M=2\nG=2\npsi_source=1e999 1\n",
    "psi_source_subnormal": "M=2\nG=2\npsi_source=1e-320 1e-400 2.5e-308\n",
    "psi_source_two_points": "M=2\nG=2\npsi_source=1.2.3\n",
    "psi_source_trailing_garbage": "M=2\nG=2\npsi_source=1.5e+2x 3\n",
    "psi_source_comma": "M=2\nG=2\npsi_source=1,2 3\n",
    "psi_source_lone_sign": "M=2\nG=2\npsi_source=- 1\n",
    "psi_source_too_many": "M=2\nG=2\npsi_source=1 2 3 4 5\n",
    "psi_source_ignored_with_equilibrium": "M=2\nG=2\nuse_mg_equilib=true\npsi_source=1 2 3 4 5 6\n",
    "tables": ("G=124\nhave_group_bounds=yes\nfilename_group_bounds=llnl_slab_test_group_bounds.txt\n"
               "have_group_absorption_opacities=True\nfilename_group_kappa=llnl_slab_test_group_kappa_a.txt\n"),
    "empty_file": "",
    "no_newline_at_end": "M=6\nN=33",
}


@pytest.mark.parametrize("case", sorted(EDGE))
def test_edge_cases(rtsn_mod, oracle_mod, tmp_path, case):
    f = tmp_path / f"{case}.prm"
    f.write_bytes(EDGE[case].encode())
    check(f, rtsn_mod, oracle_mod)


def test_missing_file_gives_defaults(rtsn_mod, oracle_mod, tmp_path):
    """param.h:53-57: an unopenable file prints and continues with every default."""
    f = tmp_path / "absent.prm"
    assert ref_parse(f)["found"] == "0"
    check(f, rtsn_mod, oracle_mod)
    assert not rtsn_mod.ParameterHandler(f).prm_found


def test_table_stream_semantics(rtsn_mod, oracle_mod, tmp_path):
    """Tables are read with `fin >> d` (ParameterHandler.cpp:152,184): the same
    extraction rules as psi_source -- a table whose third token is "abc" holds two
    values, so G = 1 bounds (2 expected) parse and G = 2 bounds fail the count assert."""
    (tmp_path / "b.txt").write_text("0.1 1.0 abc 3.0\n")
    for G, ok in ((1, True), (2, False)):
        f = tmp_path / f"t{G}.prm"
        f.write_text(f"G={G}\nhave_group_bounds=yes\nfilename_group_bounds=b.txt\n")
        if ok:
            ph = rtsn_mod.ParameterHandler(f, table_dir=tmp_path)
            assert list(ph.params["group_bounds"]) == [0.1, 1.0]
            assert list(oracle_mod.parse_prm(f, table_dir=tmp_path)["group_bounds"]) == [0.1, 1.0]
        else:
            with pytest.raises(rtsn_mod.RtError):
                rtsn_mod.ParameterHandler(f, table_dir=tmp_path)
            with pytest.raises(oracle_mod.OracleError):
                oracle_mod.parse_prm(f, table_dir=tmp_path)


# Random .prm files from the reader's grammar (seeded): keys the reference reads and junk
# keys, spaces around keys and values, comment and '='-less lines, duplicates, CRLF, and
# numeric strings from a pool of the conversions' edge shapes (signs, hex, exponents with and
# without digits, inf / nan, overflow / subnormal, garbage suffixes).  Tables stay off (their
# files are covered above); M, G and N stay small and positive.
_NUM = ["0", "1", "2", "4", "-1", "+3", "007", " 5", "6 ", "\t8", "1.5", ".5", "5.", "-0", "1e3", "1e", "2.5e+",
        "1e-320", "1e-400", "1e999", "-1e999", "0x10", "0x1p-2", "inf", "-inf", "nan", "NaN", "12abc", "abc", "",
        "2147483647", "2147483648", "-2147483649", "99999999999", "1.2.3", "1,5", "-", "+", "3 4", "0.1e-5x"]
_BOOL = ["yes", "Yes", "YES", "true", "True", "TRUE", "no", "1", "", " yes", "yes "]
# (M, G, N > 0: the product's reader refuses others with RT_ERR_PARAM, where the reference's
# sizes its psi_source matrix and fails later)
_SMALL = ["1", "2", "3", "4", "6", "8", " 2", "2 ", "+3", "007", "abc", "", "2.9", "1e1"]


def _random_prm(rng) -> str:
    lines = []
    for _ in range(int(rng.integers(0, 14))):
        kind = rng.random()
        if kind < 0.1:
            lines.append("#" + str(rng.choice(INTS + DOUBLES)) + "=1")
            continue
        if kind < 0.15:
            lines.append(str(rng.choice(["junk line", "", "   ", "M 4"])))
            continue
        key = str(rng.choice(INTS + DOUBLES + BOOLS + ("psi_source", "unknown_key")))
        if key in ("M", "G", "N"):
            val = str(rng.choice(_SMALL))
        elif key in BOOLS:
            val = str(rng.choice(_BOOL))
        elif key == "psi_source":
            val = " ".join(str(rng.choice(_NUM)) for _ in range(int(rng.integers(0, 7))))
        else:
            val = str(rng.choice(_NUM))
        pad_k = str(rng.choice(["", "", "", " "]))
        lines.append(f"{key}{pad_k}={val}" + str(rng.choice(["", "", "", " # c", "=x"])))
    sep = "\r\n" if rng.random() < 0.2 else "\n"
    return sep.join(lines) + (sep if rng.random() < 0.8 else "")


@pytest.mark.parametrize("seed", range(8))
def test_random_prm_files(rtsn_mod, oracle_mod, tmp_path, seed):
    """40 random files per seed (320 in all) parse the same through the reference's reader,
    the product's and the oracle's, values bit for bit, errors exactly where it throws."""
    rng = np.random.default_rng(20261018 + seed)
    for i in range(40):
        f = tmp_path / f"r{seed}_{i}.prm"
        f.write_bytes(_random_prm(rng).encode())
        check(f, rtsn_mod, oracle_mod)
