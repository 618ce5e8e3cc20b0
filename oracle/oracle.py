"""ctypes front end of the C oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker.  See rt_oracle.h for what the oracle
restates (Helblindi/radiative-transfer src/solver.cpp & friends).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "build" / "librtoracle.so"

ORC_ERRORS = {0: "ok", 1: "io", 2: "parse", 3: "param", 4: "validation", 5: "nomem"}


class orc_params(C.Structure):
    _fields_ = [
        ("M", C.c_int), ("G", C.c_int), ("N", C.c_int),
        ("efirst", C.c_double), ("elast", C.c_double), ("X", C.c_double), ("dx", C.c_double),
        ("bc_left", C.c_int), ("bc_right", C.c_int),
        ("use_mg_equilib", C.c_int),
        ("have_group_bounds", C.c_int), ("have_group_kappa", C.c_int),
        ("rho", C.c_double), ("kappa_grey", C.c_double), ("T", C.c_double), ("V", C.c_double),
        ("use_correction", C.c_int),
        ("ts_method", C.c_int),
        ("dt", C.c_double),
        ("max_timesteps", C.c_int),
        ("include_validation", C.c_int),
        ("prm_found", C.c_int),
        ("psi_source", C.POINTER(C.c_double)),
        ("group_bounds", C.POINTER(C.c_double)),
        ("group_kappa", C.POINTER(C.c_double)),
    ]


def build(force: bool = False) -> Path:
    if force or not LIB_PATH.exists() or LIB_PATH.stat().st_mtime < (HERE / "rt_oracle.c").stat().st_mtime:
        subprocess.run(["make", "-C", str(HERE)], check=True, stdout=subprocess.DEVNULL)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(str(LIB_PATH))
        dp = C.POINTER(C.c_double)
        L.orc_parse_prm.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(orc_params)]
        L.orc_default_params.argtypes = [C.POINTER(orc_params)]
        L.orc_free_params.argtypes = [C.POINTER(orc_params)]
        L.orc_create.argtypes = [C.POINTER(orc_params), C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int)]
        L.orc_create.restype = C.c_void_p
        L.orc_destroy.argtypes = [C.c_void_p]
        L.orc_solve.argtypes = [C.c_void_p]
        L.orc_run_substeps.argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.orc_set_threads.argtypes = [C.c_void_p, C.c_int]
        L.orc_set_threads.restype = None
        L.orc_set_parallel_copies.argtypes = [C.c_void_p, C.c_int]
        L.orc_set_parallel_copies.restype = None
        L.orc_num_groups_local.argtypes = [C.c_void_p]
        for name in ("orc_get_psi", "orc_get_ends", "orc_set_ends", "orc_get_psi_source"):
            getattr(L, name).argtypes = [C.c_void_p, dp]
        L.orc_moments.argtypes = [C.c_void_p, dp, dp, dp]
        L.orc_group_ends.argtypes = [C.c_void_p, dp, dp]
        L.orc_balance.argtypes = [C.c_void_p, dp, dp]
        L.orc_get_quad.argtypes = [C.c_void_p, dp, dp]
        L.orc_get_groups.argtypes = [C.c_void_p, dp, dp, dp, dp, dp, dp]
        L.orc_get_correction_coeffs.argtypes = [C.c_void_p, dp, dp, dp, dp, dp, dp]
        L.orc_validate.argtypes = [C.c_void_p]
        L.orc_glquad.argtypes = [C.c_int, C.c_double, dp, dp]
        L.orc_planck_groups.argtypes = [C.c_double, C.c_int, dp, dp, dp, dp]
        L.orc_eigen_inverse2.argtypes = [dp, dp]
        L.orc_material_enable.argtypes = [C.c_void_p, C.c_double, dp]
        L.orc_material_sweep.argtypes = [C.c_void_p, dp]
        L.orc_material_update.argtypes = [C.c_void_p, dp]
        L.orc_material_update.restype = None
        L.orc_get_material_transit.argtypes = [C.c_void_p, dp]
        L.orc_get_material_transit.restype = None
        L.orc_get_temperature.argtypes = [C.c_void_p, dp]
        L.orc_get_temperature.restype = None
        L.orc_get_cell_planck.argtypes = [C.c_void_p, dp]
        L.orc_get_cell_planck.restype = None
        L.orc_get_cell_emission.argtypes = [C.c_void_p, dp]
        L.orc_get_cell_emission.restype = None
        L.orc_planck_cell.argtypes = [C.c_double, C.c_int, dp, C.c_int]
        L.orc_planck_cell.restype = C.c_double
        L.orc_planck_cell_dBdT.argtypes = [C.c_double, C.c_int, dp, C.c_int]
        L.orc_planck_cell_dBdT.restype = C.c_double
        _lib = L
    return _lib


def _dp(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class OracleError(RuntimeError):
    pass


def parse_prm(path, table_dir=None) -> dict:
    """ParameterHandler::get_parameters restated (dict of every key)."""
    L = lib()
    p = orc_params()
    td = None if table_dir is None else (str(table_dir).rstrip("/") + "/").encode()
    st = L.orc_parse_prm(str(path).encode(), td, C.byref(p))
    if st:
        L.orc_free_params(C.byref(p))
        raise OracleError(f"parse_prm({path}) -> {ORC_ERRORS.get(st, st)}")
    d = {f: getattr(p, f) for f, _ in orc_params._fields_ if f not in ("psi_source", "group_bounds", "group_kappa")}
    d["psi_source"] = np.ctypeslib.as_array(p.psi_source, shape=(p.M * p.G,)).copy().reshape(p.M, p.G)
    d["group_bounds"] = (np.ctypeslib.as_array(p.group_bounds, shape=(p.G + 1,)).copy()
                         if p.have_group_bounds else None)
    d["group_kappa"] = (np.ctypeslib.as_array(p.group_kappa, shape=(p.G,)).copy()
                        if p.have_group_kappa else None)
    L.orc_free_params(C.byref(p))
    return d


def default_params() -> dict:
    L = lib()
    p = orc_params()
    L.orc_default_params(C.byref(p))
    d = {f: getattr(p, f) for f, _ in orc_params._fields_ if f not in ("psi_source", "group_bounds", "group_kappa")}
    d["psi_source"] = np.zeros((p.M, p.G))
    d["group_bounds"] = None
    d["group_kappa"] = None
    L.orc_free_params(C.byref(p))
    return d


class OracleSolver:
    """The reference's Solver (solver.h:18-98) on the CPU restatement."""

    def __init__(self, params: dict, half_copy_literal: bool = False, g_lo: int = 0, g_hi: int = 0):
        L = lib()
        self.params = dict(params)
        p = orc_params()
        keep = []
        for f, _ in orc_params._fields_:
            if f in ("psi_source", "group_bounds", "group_kappa"):
                continue
            setattr(p, f, params[f])
        if "dx" not in params or params.get("dx") is None:
            p.dx = params["X"] / params["N"]
        ps = np.ascontiguousarray(np.asarray(params.get("psi_source") if params.get("psi_source") is not None
                                             else np.zeros((params["M"], params["G"])), dtype=np.float64)
                                  .reshape(params["M"], params["G"]))
        keep.append(ps)
        p.psi_source = _dp(ps)
        if params.get("group_bounds") is not None:
            gb = np.ascontiguousarray(params["group_bounds"], dtype=np.float64)
            keep.append(gb)
            p.group_bounds = _dp(gb)
            p.have_group_bounds = 1
        if params.get("group_kappa") is not None:
            gk = np.ascontiguousarray(params["group_kappa"], dtype=np.float64)
            keep.append(gk)
            p.group_kappa = _dp(gk)
            p.have_group_kappa = 1
        st = C.c_int(0)
        self._h = L.orc_create(C.byref(p), int(half_copy_literal), g_lo, g_hi, C.byref(st))
        if not self._h:
            raise OracleError(f"orc_create -> {ORC_ERRORS.get(st.value, st.value)}")
        self.M, self.G, self.N = p.M, p.G, p.N
        self.Gl = L.orc_num_groups_local(self._h)
        self.g_lo = int(g_lo)  # first group of the handle (its groups: g_lo .. g_lo + Gl - 1)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().orc_destroy(h)
            self._h = None

    def set_parallel_copies(self, on: bool = True):
        """CPU baseline: the whole-array snapshot copies split over the threads."""
        lib().orc_set_parallel_copies(self._h, 1 if on else 0)

    def set_threads(self, n: int):
        """OpenMP threads over the (direction, group) lines of a run of same-sign directions
        (results do not depend on it).."""
        lib().orc_set_threads(self._h, int(n))

    def solve(self):
        st = lib().orc_solve(self._h)
        if st:
            raise OracleError(f"solve -> {ORC_ERRORS.get(st, st)}")

    def run_substeps(self, it0: int, n: int):
        st = lib().orc_run_substeps(self._h, it0, n)
        if st:
            raise OracleError(f"run_substeps -> {ORC_ERRORS.get(st, st)}")

    def psi(self) -> np.ndarray:
        """(M, Gl, N) array (C order view of the ColMajor tensor transposed)."""
        out = np.empty(self.M * self.Gl * self.N)
        lib().orc_get_psi(self._h, _dp(out))
        return out.reshape(self.N, self.Gl, self.M).transpose(2, 1, 0).copy()

    def ends(self) -> np.ndarray:
        """(M, Gl, N, 2)."""
        out = np.empty(2 * self.M * self.Gl * self.N)
        lib().orc_get_ends(self._h, _dp(out))
        return out.reshape(2, self.N, self.Gl, self.M).transpose(3, 2, 1, 0).copy()

    def set_ends(self, ends: np.ndarray):
        flat = np.ascontiguousarray(np.asarray(ends, dtype=np.float64).transpose(3, 2, 1, 0)).ravel()
        lib().orc_set_ends(self._h, _dp(flat))

    def moments(self):
        phi = np.empty(self.Gl * self.N)
        F = np.empty(self.Gl * self.N)
        pp = np.empty(self.Gl * self.N)
        lib().orc_moments(self._h, _dp(phi), _dp(F), _dp(pp))
        f = lambda a: a.reshape(self.N, self.Gl).T.copy()  # noqa: E731  (G, N)
        return f(phi), f(F), f(pp)

    def group_ends(self):
        left = np.empty(self.Gl)
        right = np.empty(self.Gl)
        lib().orc_group_ends(self._h, _dp(left), _dp(right))
        return left, right

    def balance(self):
        phi = np.empty(self.Gl * self.N)
        lib().orc_moments(self._h, _dp(phi), None, None)
        bal = np.empty(self.Gl)
        lib().orc_balance(self._h, _dp(phi), _dp(bal))
        return bal

    def quad(self):
        mu = np.empty(self.M)
        wt = np.empty(self.M)
        lib().orc_get_quad(self._h, _dp(mu), _dp(wt))
        return mu, wt

    def groups(self) -> dict:
        G = self.G
        arrs = {k: np.empty(G + (1 if k == "e_edge" else 0)) for k in
                ("e_edge", "e_ave", "de_ave", "B", "dBdT", "kappa")}
        lib().orc_get_groups(self._h, *(_dp(arrs[k]) for k in ("e_edge", "e_ave", "de_ave", "B", "dBdT", "kappa")))
        return arrs

    def correction_coeffs(self) -> dict:
        G = self.G
        arrs = {k: np.empty(G) for k in ("dEB", "dsigEdE", "dkapEB", "cor1", "cor2", "cor3")}
        lib().orc_get_correction_coeffs(self._h, *(_dp(arrs[k]) for k in ("dEB", "dsigEdE", "dkapEB", "cor1", "cor2", "cor3")))
        return arrs

    def psi_source(self) -> np.ndarray:
        out = np.empty(self.M * self.G)
        lib().orc_get_psi_source(self._h, _dp(out))
        return out.reshape(self.M, self.G)

    def validate(self) -> bool:
        return bool(lib().orc_validate(self._h))

    # ---- material-temperature coupling (beyond the reference; rtsn.h rt_material_*) ----
    def material_enable(self, rho_cv: float, T_cells=None):
        T = None if T_cells is None else np.ascontiguousarray(T_cells, dtype=np.float64)
        st = lib().orc_material_enable(self._h, float(rho_cv), None if T is None else _dp(T))
        if st:
            raise OracleError(f"material_enable -> {ORC_ERRORS.get(st, st)}")

    def material_sweep(self) -> np.ndarray:
        """One coupled full step; returns this solver's [q, b] (2N: q(x), then
        sum over its groups of sigma_g dB_g/dT(x)) -- sum it over group shards."""
        q = np.empty(2 * self.N)
        st = lib().orc_material_sweep(self._h, _dp(q))
        if st:
            raise OracleError(f"material_sweep -> {ORC_ERRORS.get(st, st)}")
        return q

    def material_update(self, q):
        qq = np.ascontiguousarray(q, dtype=np.float64)
        lib().orc_material_update(self._h, _dp(qq))

    def material_step(self, n: int = 1):
        for _ in range(n):
            self.material_update(self.material_sweep())

    def temperature(self) -> np.ndarray:
        out = np.empty(self.N)
        lib().orc_get_temperature(self._h, _dp(out))
        return out

    def material_transit(self) -> np.ndarray:
        """(N) energy per volume the material owes the radiation (this solver's groups)."""
        out = np.empty(self.N)
        lib().orc_get_material_transit(self._h, _dp(out))
        return out

    def cell_planck(self) -> np.ndarray:
        """(G_local, N) B_g(T(x))."""
        out = np.empty(self.N * self.Gl)
        lib().orc_get_cell_planck(self._h, _dp(out))
        return out.reshape(self.N, self.Gl).T.copy()

    def cell_emission(self) -> np.ndarray:
        """(G_local, N) the next step's emission B_g(T) + dB_g/dT(T_prev) dT_prev."""
        out = np.empty(self.N * self.Gl)
        lib().orc_get_cell_emission(self._h, _dp(out))
        return out.reshape(self.N, self.Gl).T.copy()


def glquad(M: int, norm: float = 4.0 * 3.1415926546):
    mu = np.empty(M)
    wt = np.empty(M)
    lib().orc_glquad(M, norm, _dp(mu), _dp(wt))
    return mu, wt


def planck_groups(T: float, e_lo, e_hi):
    e_lo = np.ascontiguousarray(e_lo, dtype=np.float64)
    e_hi = np.ascontiguousarray(e_hi, dtype=np.float64)
    G = len(e_lo)
    B = np.empty(G)
    dB = np.empty(G)
    lib().orc_planck_groups(T, G, _dp(e_lo), _dp(e_hi), _dp(B), _dp(dB))
    return B, dB


def planck_cell(T: float, e_edge, g: int) -> float:
    """kcon x B_g(T) per the material coupling's definition (rt_oracle.c orc_planck_cell)."""
    e = np.ascontiguousarray(e_edge, dtype=np.float64)
    return lib().orc_planck_cell(float(T), len(e) - 1, _dp(e), int(g))


def planck_cell_dBdT(T: float, e_edge, g: int) -> float:
    """kcon x dB_g/dT(T) (rt_oracle.c orc_planck_cell_dBdT)."""
    e = np.ascontiguousarray(e_edge, dtype=np.float64)
    return lib().orc_planck_cell_dBdT(float(T), len(e) - 1, _dp(e), int(g))


def eigen_inverse2(m) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(m, dtype=np.float64).reshape(4))
    out = np.empty(4)
    lib().orc_eigen_inverse2(_dp(a), _dp(out))
    return out.reshape(2, 2)


if __name__ == "__main__":  # pragma: no cover
    build(force=True)
    print("built", LIB_PATH, os.path.getsize(LIB_PATH))
