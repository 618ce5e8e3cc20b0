"""ctypes binding of include/rtsn.h (see package docstring)."""
from __future__ import annotations

import ctypes as C
import os
import re
import subprocess
import sys
from pathlib import Path
from typing import Optional

import numpy as np

PKG_ROOT = Path(__file__).resolve().parent.parent          # radiative-transfer_amd/
REPO_ROOT = PKG_ROOT.parent
LIB_PATH = Path(os.environ.get("RTSN_LIB", PKG_ROOT / "lib" / "librtsn.so"))  # RTSN_LIB: timing experiments
HEADER = REPO_ROOT / "include" / "rtsn.h"

STATUS = {0: "ok", 1: "io error", 2: "parse error", 3: "invalid parameter", 4: "correction validation failed",
          5: "out of memory", 6: "device error", 7: "timeout (communicator aborted)", 8: "bad argument",
          9: "not valid in the handle's mode", 10: "warning (not returned since round 6)"}


class RtError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"{msg}: {STATUS.get(status, status)}")
        self.status = status


class rt_params(C.Structure):
    _fields_ = [
        ("M", C.c_int), ("G", C.c_int), ("N", C.c_int),
        ("efirst", C.c_double), ("elast", C.c_double), ("X", C.c_double),
        ("bc_left_indicator", C.c_int), ("bc_right_indicator", C.c_int),
        ("use_mg_equilib", C.c_int),
        ("rho", C.c_double), ("kappa_grey", C.c_double), ("T", C.c_double), ("V", C.c_double),
        ("use_correction", C.c_int), ("ts_method", C.c_int),
        ("dt", C.c_double),
        ("max_timesteps", C.c_int), ("include_validation", C.c_int),
        ("psi_source", C.POINTER(C.c_double)),
        ("group_bounds", C.POINTER(C.c_double)),
        ("group_kappa", C.POINTER(C.c_double)),
    ]


class rt_shard(C.Structure):
    _fields_ = [(f, C.c_int) for f in ("G", "M", "g_lo", "g_hi", "d_lo", "d_hi", "N", "reserved")]


_SCALARS = [f for f, _ in rt_params._fields_ if f not in ("psi_source", "group_bounds", "group_kappa")]


def build(force: bool = False) -> Path:
    """Compile librtsn.so (hipcc, gfx950) in-tree."""
    if force or not LIB_PATH.exists():
        subprocess.run(["make", "-C", str(PKG_ROOT), "-j8"], check=True)
    return LIB_PATH


_lib = None


def lib():
    """Load librtsn.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        # PyTorch-ROCm bundles its own libamdhip64.so.7; load it first (if
        # torch is installed) so that torch and librtsn share ONE HIP runtime
        # in the process instead of two that race for the device.
        if "torch" not in sys.modules:
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
        if not LIB_PATH.exists():
            raise RtError(6, f"{LIB_PATH} is missing -- run build() / make -C radiative-transfer_amd")
        L = C.CDLL(str(LIB_PATH))
        dp = C.POINTER(C.c_double)
        vp = C.c_void_p
        L.rt_params_load.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(rt_params), C.POINTER(C.c_int)]
        L.rt_params_free.argtypes = [C.POINTER(rt_params)]
        L.rt_params_free.restype = None
        L.rt_params_default.argtypes = [C.POINTER(rt_params)]
        L.rt_params_default.restype = None
        L.rt_quadrature.argtypes = [C.c_int, dp, dp]
        L.rt_planck_groups.argtypes = [C.c_double, C.c_int, dp, dp, dp]
        L.rt_create.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.POINTER(vp)]
        L.rt_create_from_params.argtypes = [C.POINTER(rt_params), C.c_int, C.c_int, C.c_int, C.POINTER(vp)]
        L.rt_create_direction_shard.argtypes = [C.POINTER(rt_params), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                                C.POINTER(vp)]
        L.rt_destroy.argtypes = [vp]
        L.rt_destroy.restype = None
        for name in ("rt_solve", "rt_synchronize", "rt_finish"):
            getattr(L, name).argtypes = [vp]
        L.rt_advance.argtypes = [vp, C.c_int]
        L.rt_stream.argtypes = [vp]
        L.rt_stream.restype = vp
        L.rt_get_dims.argtypes = [vp] + [C.POINTER(C.c_int)] * 5
        for name in ("rt_get_psi", "rt_get_ends", "rt_get_balance", "rt_get_e_ave", "rt_get_psi_source",
                     "rt_group_absorption_device"):
            getattr(L, name).argtypes = [vp, dp]
        L.rt_set_ends.argtypes = [vp, dp]
        L.rt_get_moments.argtypes = [vp, dp, dp, dp]
        L.rt_get_balance_terms.argtypes = [vp, dp, dp, dp]
        L.rt_get_moments_device.argtypes = [vp, vp, vp, vp]
        L.rt_get_group_ends.argtypes = [vp, dp, dp]
        L.rt_get_group_data.argtypes = [vp, dp, dp, dp, dp]
        L.rt_get_quadrature.argtypes = [vp, dp, dp]
        L.rt_set_profiling.argtypes = [vp, C.c_int]
        L.rt_state_finite.argtypes = [vp, C.POINTER(C.c_int)]
        L.rt_get_sweep_time.argtypes = [vp, dp, C.POINTER(C.c_longlong)]
        L.rt_sweep_traffic.argtypes = [vp, dp, dp]
        L.rt_sweep_geometry.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_longlong)]
        L.rt_sweep_flops.argtypes = [vp, dp]
        L.rt_set_time_block.argtypes = [vp, C.c_int]
        L.rt_set_pipeline.argtypes = [vp, C.c_int]
        L.rt_set_level_waves.argtypes = [vp, C.c_int]
        L.rt_get_pipeline.argtypes = [vp, C.POINTER(C.c_int)]
        L.rt_pipeline_state.argtypes = [vp, C.POINTER(C.c_longlong), C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.rt_get_time_block.argtypes = [vp, C.POINTER(C.c_int)]
        L.rt_plan_time_block.argtypes = [C.c_int, C.c_longlong, C.POINTER(C.c_int)]
        L.rt_plan_schedule.argtypes = [vp, C.c_longlong, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int),
                                       dp]
        L.rt_set_segmentation.argtypes = [vp, C.c_int]
        L.rt_set_moments_form.argtypes = [vp, C.c_int]
        L.rt_set_phi_correction_form.argtypes = [vp, C.c_int]
        L.rt_debug_fail_launch.argtypes = [vp, C.c_int]
        L.rt_debug_set_transfer_chunk.argtypes = [vp, C.c_longlong]
        L.rt_get_level_waves.argtypes = [vp, C.POINTER(C.c_int)]
        L.rt_set_wavefront.argtypes = [vp, C.c_int]
        L.rt_get_wavefront.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.rt_set_wavefront_waves.argtypes = [vp, C.c_int]
        L.rt_get_wavefront_waves.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.rt_set_wavefront_cells.argtypes = [vp, C.c_int]
        L.rt_material_enable.argtypes = [vp, C.c_double, dp]
        L.rt_material_sweep.argtypes = [vp, vp]
        L.rt_material_update.argtypes = [vp, vp]
        L.rt_material_step.argtypes = [vp, C.c_int]
        L.rt_material_stability.argtypes = [vp, dp]
        L.rt_get_cell_emission.argtypes = [vp, dp]
        L.rt_get_material_transit.argtypes = [vp, dp]
        L.rt_get_temperature.argtypes = [vp, dp]
        L.rt_get_cell_planck.argtypes = [vp, dp]
        L.rt_get_shard.argtypes = [vp] + [C.POINTER(C.c_int)] * 6
        L.rt_get_balance_partials.argtypes = [vp, dp, dp, dp]
        L.rt_comm_unique_id.argtypes = [C.c_char_p]
        L.rt_comm_init.argtypes = [C.c_int, C.c_int, C.c_char_p, C.c_int, C.POINTER(vp)]
        L.rt_comm_destroy.argtypes = [vp]
        L.rt_comm_destroy.restype = None
        L.rt_comm_rank.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.rt_comm_count.argtypes = [vp, C.POINTER(C.c_int)]
        L.rt_comm_gather_moments.argtypes = [vp, vp, dp, dp, dp]
        L.rt_comm_gather_group_ends.argtypes = [vp, vp, dp, dp]
        L.rt_comm_gather_balance.argtypes = [vp, vp, dp, dp, dp]
        L.rt_comm_gather_psi.argtypes = [vp, vp, C.c_int, dp]
        L.rt_comm_gather_psi_source.argtypes = [vp, vp, dp]
        L.rt_comm_allreduce_absorption.argtypes = [vp, vp, vp]
        L.rt_comm_material_step.argtypes = [vp, vp, C.c_int]
        L.rt_comm_synchronize.argtypes = [vp, vp]
        L.rt_comm_version.argtypes = [C.POINTER(C.c_int), C.c_char_p, C.c_size_t]
        sp = C.POINTER(rt_shard)
        L.rt_layout_mode.argtypes = [sp, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.rt_layout_pack_moments.argtypes = [sp, C.c_int, C.c_int, dp, dp]
        L.rt_layout_unpack_moments.argtypes = [sp, C.c_int, dp, dp, dp, dp]
        L.rt_layout_pack_vectors.argtypes = [sp, C.c_int, C.c_int, C.c_int, C.POINTER(dp), dp]
        L.rt_layout_unpack_vectors.argtypes = [sp, C.c_int, C.c_int, dp, C.POINTER(dp)]
        L.rt_layout_place_psi.argtypes = [sp, dp, dp]
        L.rt_layout_place_psi_source.argtypes = [sp, dp, dp]
        L.rt_comm_last_error.argtypes = [vp]
        L.rt_comm_last_error.restype = C.c_char_p
        L.rt_status_string.argtypes = [C.c_int]
        L.rt_status_string.restype = C.c_char_p
        L.rt_last_error.argtypes = [vp]
        L.rt_last_error.restype = C.c_char_p
        _lib = L
    return _lib


def exported_symbols() -> list[str]:
    """Function names declared in include/rtsn.h."""
    text = HEADER.read_text()
    return sorted(set(re.findall(r"\b(rt_[a-z_0-9]+)\s*\(", text)))


def _dp(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _check(st: int, what: str, handle=None):
    if st != 0:
        msg = lib().rt_last_error(handle).decode(errors="replace")
        raise RtError(st, f"{what} ({msg})")


_DEFAULTS = None


def params_default() -> dict:
    """rt_params_default as a dict (a fresh copy; the library's values are read once)."""
    global _DEFAULTS
    if _DEFAULTS is None:
        p = rt_params()
        lib().rt_params_default(C.byref(p))
        _DEFAULTS = {f: getattr(p, f) for f in _SCALARS}
        _DEFAULTS.update(psi_source=None, group_bounds=None, group_kappa=None)
    return dict(_DEFAULTS)


def quadrature(M: int):
    mu, wt = np.empty(M), np.empty(M)
    _check(lib().rt_quadrature(M, _dp(mu), _dp(wt)), "rt_quadrature")
    return mu, wt


def plan_time_block(ts_method: int, nsteps: int) -> int:
    """The time block rt_solve picks for a run of nsteps (rt_plan_time_block; host only)."""
    t = C.c_int()
    _check(lib().rt_plan_time_block(int(ts_method), int(nsteps), C.byref(t)), "rt_plan_time_block")
    return t.value


def planck_groups(T: float, e_edge):
    e = np.ascontiguousarray(e_edge, dtype=np.float64)
    G = len(e) - 1
    B, dB = np.empty(G), np.empty(G)
    _check(lib().rt_planck_groups(T, G, _dp(e), _dp(B), _dp(dB)), "rt_planck_groups")
    return B, dB


class ParameterHandler:
    """ParameterHandler(filename) (include/ParameterHandler.h:67): the .prm reader."""

    def __init__(self, filename, table_dir: Optional[str] = None):
        p = rt_params()
        found = C.c_int(0)
        td = None if table_dir is None else (str(table_dir).rstrip("/") + "/").encode()
        _check(lib().rt_params_load(str(filename).encode(), td, C.byref(p), C.byref(found)), "rt_params_load")
        self.prm_found = bool(found.value)
        self.params = {f: getattr(p, f) for f in _SCALARS}
        M, G = p.M, p.G
        self.params["psi_source"] = (np.ctypeslib.as_array(p.psi_source, shape=(M * G,)).copy().reshape(M, G)
                                     if p.psi_source else np.zeros((M, G)))
        self.params["group_bounds"] = (np.ctypeslib.as_array(p.group_bounds, shape=(G + 1,)).copy()
                                       if p.group_bounds else None)
        self.params["group_kappa"] = (np.ctypeslib.as_array(p.group_kappa, shape=(G,)).copy()
                                      if p.group_kappa else None)
        lib().rt_params_free(C.byref(p))

    def __getattr__(self, name):
        # get_M(), get_G(), ... get_validation() as in ParameterHandler.h:73-98
        if name.startswith("get_"):
            key = {"get_validation": "include_validation",
                   "get_bc_left_indicator": "bc_left_indicator", "get_bc_right_indicator": "bc_right_indicator",
                   "get_have_group_bounds": "group_bounds",
                   "get_have_group_absorption_opacities": "group_kappa"}.get(name, name[4:])
            if key in ("group_bounds", "group_kappa"):
                return lambda: self.params[key] is not None
            if key == "dx":
                return lambda: self.params["X"] / self.params["N"]
            if key in self.params:
                return lambda: self.params[key]
        raise AttributeError(name)


def _to_struct(params: dict, keep: list) -> rt_params:
    p = rt_params()
    for f in _SCALARS:
        setattr(p, f, params[f])
    M, G = params["M"], params["G"]
    ps = params.get("psi_source")
    if ps is not None:
        a = np.ascontiguousarray(np.asarray(ps, dtype=np.float64).reshape(M * G))
        keep.append(a)
        p.psi_source = _dp(a)
    for key in ("group_bounds", "group_kappa"):
        v = params.get(key)
        if v is not None:
            a = np.ascontiguousarray(v, dtype=np.float64)
            keep.append(a)
            setattr(p, key, _dp(a))
    return p


class Solver:
    """The reference's Solver (include/solver.h:18-98) on librtsn.

    Solver(parameter_handler_or_params, device=0, g_lo=0, g_hi=0).  Results
    are numpy arrays in the reference's index order: psi (M, G, N), phi / F /
    phi_plus (G, N), ends (M, G, N, 2)."""

    def __init__(self, ph, device: int = 0, g_lo: int = 0, g_hi: int = 0, d_lo: int = 0, d_hi: int = 0):
        """d_hi > 0: a direction-pair shard [d_lo, d_hi) of the M/2 pairs (rt_create_direction_shard)."""
        params = ph.params if isinstance(ph, ParameterHandler) else dict(ph)
        for k, v in params_default().items():
            params.setdefault(k, v)
        keep: list = []
        p = _to_struct(params, keep)
        h = C.c_void_p()
        if d_hi > 0:
            _check(lib().rt_create_direction_shard(C.byref(p), g_lo, g_hi, d_lo, d_hi, device, C.byref(h)),
                   "rt_create_direction_shard")
        else:
            _check(lib().rt_create_from_params(C.byref(p), g_lo, g_hi, device, C.byref(h)), "rt_create_from_params")
        self._h = h
        M, Gl, N, lo, hi = (C.c_int() for _ in range(5))
        lib().rt_get_dims(h, C.byref(M), C.byref(Gl), C.byref(N), C.byref(lo), C.byref(hi))
        self.M, self.G, self.N, self.g_lo, self.g_hi = M.value, Gl.value, N.value, lo.value, hi.value
        self.d_lo, self.d_hi = (d_lo, d_hi) if d_hi > 0 else (0, self.M // 2)  # M: this handle's directions
        self.G_total = params["G"]
        self.params = params
        self._phi_plus = None
        self._balance = None
        self._ends = None

    def close(self):
        if getattr(self, "_h", None):
            lib().rt_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---- stepping ----
    def solve(self):
        _check(lib().rt_solve(self._h), "rt_solve", self._h)

    def advance(self, nsteps: int):
        _check(lib().rt_advance(self._h, int(nsteps)), "rt_advance", self._h)

    def finish(self):
        """Enqueue the pipeline drain / remainder / pending correction (rt_finish)."""
        _check(lib().rt_finish(self._h), "rt_finish", self._h)

    def synchronize(self):
        _check(lib().rt_synchronize(self._h), "rt_synchronize", self._h)

    @property
    def stream(self) -> int:
        return lib().rt_stream(self._h) or 0

    # ---- results ----
    def psi(self) -> np.ndarray:
        out = np.empty(self.M * self.G * self.N)
        _check(lib().rt_get_psi(self._h, _dp(out)), "rt_get_psi", self._h)
        return out.reshape(self.N, self.G, self.M).transpose(2, 1, 0).copy()

    def ends(self) -> np.ndarray:
        out = np.empty(2 * self.M * self.G * self.N)
        _check(lib().rt_get_ends(self._h, _dp(out)), "rt_get_ends", self._h)
        return out.reshape(2, self.N, self.G, self.M).transpose(3, 2, 1, 0).copy()

    def set_ends(self, ends: np.ndarray):
        flat = np.ascontiguousarray(np.asarray(ends, dtype=np.float64).transpose(3, 2, 1, 0)).ravel()
        _check(lib().rt_set_ends(self._h, _dp(flat)), "rt_set_ends", self._h)

    def moments(self):
        n = self.G * self.N
        phi, F, pp = np.empty(n), np.empty(n), np.empty(n)
        _check(lib().rt_get_moments(self._h, _dp(phi), _dp(F), _dp(pp)), "rt_get_moments", self._h)
        f = lambda a: a.reshape(self.N, self.G).T.copy()  # noqa: E731
        return f(phi), f(F), f(pp)

    def compute_angle_integrated_intensity(self) -> np.ndarray:
        return self.moments()[0]

    def compute_radiative_flux(self) -> np.ndarray:
        return self.moments()[1]

    def compute_positive_angle_integrated_intensity(self) -> np.ndarray:
        self._phi_plus = self.moments()[2]
        return self._phi_plus

    def get_phi_plus(self) -> np.ndarray:
        return self._phi_plus

    def compute_balance(self) -> np.ndarray:
        out = np.empty(self.G)
        _check(lib().rt_get_balance(self._h, _dp(out)), "rt_get_balance", self._h)
        self._balance = out
        return out

    def compute_balance_terms(self):
        """(balance, sources, sinks) per group (rt_get_balance_terms, solver.cpp:240-284)."""
        b, src, snk = np.empty(self.G), np.empty(self.G), np.empty(self.G)
        _check(lib().rt_get_balance_terms(self._h, _dp(b), _dp(src), _dp(snk)), "rt_get_balance_terms", self._h)
        self._balance = b
        return b, src, snk

    def get_balance(self) -> np.ndarray:
        return self._balance

    def compute_group_ends(self):
        left, right = np.empty(self.G), np.empty(self.G)
        _check(lib().rt_get_group_ends(self._h, _dp(left), _dp(right)), "rt_get_group_ends", self._h)
        self._ends = (left, right)
        return self._ends

    def get_ends(self, side: str) -> np.ndarray:
        assert side in ("left", "right"), "Invalid option for 'side'."
        return self._ends[0] if side == "left" else self._ends[1]

    def get_e_ave(self) -> np.ndarray:
        out = np.empty(self.G_total)
        _check(lib().rt_get_e_ave(self._h, _dp(out)), "rt_get_e_ave", self._h)
        return out

    def groups(self) -> dict:
        G = self.G_total
        d = {"e_edge": np.empty(G + 1), "B": np.empty(G), "dBdT": np.empty(G), "kappa": np.empty(G)}
        _check(lib().rt_get_group_data(self._h, _dp(d["e_edge"]), _dp(d["B"]), _dp(d["dBdT"]), _dp(d["kappa"])),
               "rt_get_group_data", self._h)
        return d

    def quad(self):
        mu, wt = np.empty(self.M), np.empty(self.M)
        _check(lib().rt_get_quadrature(self._h, _dp(mu), _dp(wt)), "rt_get_quadrature", self._h)
        return mu, wt

    def psi_source(self) -> np.ndarray:
        out = np.empty(self.M * self.G_total)
        _check(lib().rt_get_psi_source(self._h, _dp(out)), "rt_get_psi_source", self._h)
        return out.reshape(self.M, self.G_total)

    def group_absorption_device(self, d_out_ptr: int):
        _check(lib().rt_group_absorption_device(self._h, C.cast(C.c_void_p(d_out_ptr), C.POINTER(C.c_double))),
               "rt_group_absorption_device", self._h)

    def moments_device(self, phi, F=None, phi_plus=None):
        """rt_get_moments_device into contiguous float64 CUDA tensors of N*G_local
        elements (layout g + G_local*c), on the solver's stream."""
        import torch
        ptrs = []
        for t in (phi, F, phi_plus):
            if t is None:
                ptrs.append(None)
                continue
            if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float64
                    and t.is_contiguous() and t.numel() == self.N * self.G):
                raise ValueError("moments_device: need contiguous float64 CUDA tensors of N*G_local elements")
            ptrs.append(t.data_ptr())
        _check(lib().rt_get_moments_device(self._h, *ptrs), "rt_get_moments_device", self._h)

    def state_finite(self) -> bool:
        """rt_state_finite: every node of the state finite (NaN/Inf scan on the device)."""
        f = C.c_int(0)
        _check(lib().rt_state_finite(self._h, C.byref(f)), "rt_state_finite", self._h)
        return bool(f.value)

    def group_absorption(self, out):
        """Group-summed absorption into a contiguous float64 torch tensor of N
        elements on this solver's GPU (ordered on the solver's stream)."""
        import torch
        if not (isinstance(out, torch.Tensor) and out.is_cuda and out.dtype == torch.float64
                and out.is_contiguous() and out.numel() == self.N):
            raise ValueError("group_absorption: need a contiguous float64 CUDA tensor of N elements")
        self.group_absorption_device(out.data_ptr())

    # ---- material-temperature coupling (beyond the reference; rtsn.h rt_material_*) ----
    def material_enable(self, rho_cv: float, T_cells=None):
        """T(x) coupling on: rho_cv > 0, T_cells (N) or None for the uniform .prm T."""
        T = None if T_cells is None else np.ascontiguousarray(T_cells, dtype=np.float64)
        if T is not None and T.size != self.N:
            raise ValueError("material_enable: T_cells must hold N values")
        _check(lib().rt_material_enable(self._h, float(rho_cv), None if T is None else _dp(T)),
               "rt_material_enable", self._h)
        return self.material_stability()

    def material_stability(self) -> float:
        """dt W sum_g rho kappa_g dB_g/dT(T_max) / rho_cv: the emission's stiffness at the hottest
        cell (the implicit update scales the explicit change by 1 / (1 + number); < 2 was the
        explicit emission's limit)."""
        v = C.c_double()
        _check(lib().rt_material_stability(self._h, C.byref(v)), "rt_material_stability", self._h)
        return v.value

    @staticmethod
    def _device_vec(t, n: int, what: str):
        if t is None:
            return None
        import torch
        if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float64
                and t.is_contiguous() and t.numel() == n):
            raise ValueError(f"{what}: need a contiguous float64 CUDA tensor of {n} elements")
        return t.data_ptr()

    def material_sweep(self, q=None):
        """One coupled full step; this handle's [q, b] (2N: q(x), then sum_g sigma_g dB_g/dT(x))
        into the CUDA tensor q (None: kept inside the handle), ordered on the handle's stream."""
        _check(lib().rt_material_sweep(self._h, self._device_vec(q, 2 * self.N, "material_sweep")),
               "rt_material_sweep", self._h)

    def material_update(self, q=None):
        """T += dt q / (rho_cv + dt W b), then the owed emission and the next step's emission,
        from the group-summed [q, b] (CUDA tensor of 2N, or None: the handle's own)."""
        _check(lib().rt_material_update(self._h, self._device_vec(q, 2 * self.N, "material_update")),
               "rt_material_update", self._h)

    def material_step(self, nsteps: int = 1):
        _check(lib().rt_material_step(self._h, int(nsteps)), "rt_material_step", self._h)

    def temperature(self) -> np.ndarray:
        out = np.empty(self.N)
        _check(lib().rt_get_temperature(self._h, _dp(out)), "rt_get_temperature", self._h)
        return out

    def cell_planck(self) -> np.ndarray:
        """(G_local, N) per-cell B_g(T(x))."""
        out = np.empty(self.N * self.G)
        _check(lib().rt_get_cell_planck(self._h, _dp(out)), "rt_get_cell_planck", self._h)
        return out.reshape(self.N, self.G).T.copy()

    def cell_emission(self) -> np.ndarray:
        """(G_local, N) the next coupled step's emission B_g + the owed share it pays."""
        out = np.empty(self.N * self.G)
        _check(lib().rt_get_cell_emission(self._h, _dp(out)), "rt_get_cell_emission", self._h)
        return out.reshape(self.N, self.G).T.copy()

    def material_transit(self) -> np.ndarray:
        """(N) energy per volume the material owes the radiation (rt_get_material_transit)."""
        out = np.empty(self.N)
        _check(lib().rt_get_material_transit(self._h, _dp(out)), "rt_get_material_transit", self._h)
        return out

    # ---- measurement ----
    def set_profiling(self, on: bool):
        _check(lib().rt_set_profiling(self._h, int(on)), "rt_set_profiling", self._h)

    def sweep_time(self):
        ms = C.c_double()
        n = C.c_longlong()
        _check(lib().rt_get_sweep_time(self._h, C.byref(ms), C.byref(n)), "rt_get_sweep_time", self._h)
        return ms.value, n.value

    @property
    def time_block(self) -> int:
        """Full steps advanced per pass over HBM (rt_set_time_block)."""
        t = C.c_int()
        _check(lib().rt_get_time_block(self._h, C.byref(t)), "rt_get_time_block", self._h)
        return t.value

    @time_block.setter
    def time_block(self, steps_per_pass: int):
        _check(lib().rt_set_time_block(self._h, int(steps_per_pass)), "rt_set_time_block", self._h)

    @property
    def level_waves(self) -> int:
        """Waves per segment of a pipelined BDF2 pass of 8/10/12/16/20/24/32/40 steps
        (rt_set_level_waves; 0 = auto: one up to T = 16, two at T = 20, four above);
        reads the effective choice."""
        v = C.c_int()
        _check(lib().rt_get_level_waves(self._h, C.byref(v)), "rt_get_level_waves", self._h)
        return v.value

    @level_waves.setter
    def level_waves(self, waves: int):
        _check(lib().rt_set_level_waves(self._h, int(waves)), "rt_set_level_waves", self._h)

    @property
    def pipeline(self) -> int:
        """Pipelined (staggered-segment) schedule: 0 off, 1 auto, 2 always (rt_set_pipeline)."""
        v = C.c_int()
        _check(lib().rt_get_pipeline(self._h, C.byref(v)), "rt_get_pipeline", self._h)
        return v.value

    @pipeline.setter
    def pipeline(self, mode):
        _check(lib().rt_set_pipeline(self._h, int(mode)), "rt_set_pipeline", self._h)

    @property
    def wavefront(self) -> int:
        """Short lines in one launch per advance, lanes over cells (rt_set_wavefront): 0 off,
        1 auto (the line fits and the caller chose neither time block nor schedule), 2 on."""
        v = C.c_int()
        _check(lib().rt_get_wavefront(self._h, C.byref(v), None, None), "rt_get_wavefront", self._h)
        return v.value

    @wavefront.setter
    def wavefront(self, mode):
        _check(lib().rt_set_wavefront(self._h, int(mode)), "rt_set_wavefront", self._h)

    @property
    def wavefront_waves(self) -> int:
        """Waves a wavefront chain may span, 1..8 (rt_set_wavefront_waves; default 8)."""
        v = C.c_int()
        _check(lib().rt_get_wavefront_waves(self._h, C.byref(v), None), "rt_get_wavefront_waves", self._h)
        return v.value

    @wavefront_waves.setter
    def wavefront_waves(self, n):
        _check(lib().rt_set_wavefront_waves(self._h, int(n)), "rt_set_wavefront_waves", self._h)

    def set_wavefront_cells(self, c: int):
        """Cells per lane of the wavefront chain (rt_set_wavefront_cells): 0 the plan's, 1, 2, 4, 8."""
        _check(lib().rt_set_wavefront_cells(self._h, int(c)), "rt_set_wavefront_cells", self._h)

    def wavefront_state(self) -> dict:
        """{"mode", "active" (the next advance takes the wavefront), "cells_per_lane" (0: too
        long), "waves" (per chain; 0: too long)}."""
        m, a, c, w = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        _check(lib().rt_get_wavefront(self._h, C.byref(m), C.byref(a), C.byref(c)), "rt_get_wavefront", self._h)
        _check(lib().rt_get_wavefront_waves(self._h, None, C.byref(w)), "rt_get_wavefront_waves", self._h)
        return {"mode": m.value, "active": bool(a.value), "cells_per_lane": c.value, "waves": w.value}

    def plan_schedule(self, nsteps: int) -> dict:
        """rt_plan_schedule: the pipelined BDF2 schedule rt_solve picks for nsteps on this
        handle -- {"time_block", "level_waves", "wgs_per_cu", "estimated_ms"}."""
        T, lw, w, ms = C.c_int(), C.c_int(), C.c_int(), C.c_double()
        _check(lib().rt_plan_schedule(self._h, int(nsteps), C.byref(T), C.byref(lw), C.byref(w), C.byref(ms)),
               "rt_plan_schedule", self._h)
        return {"time_block": T.value, "level_waves": lw.value, "wgs_per_cu": w.value, "estimated_ms": ms.value}

    def set_segmentation(self, wgs_per_cu: int):
        """rt_set_segmentation: segments sized for wgs_per_cu workgroups per CU (0: occupancy)."""
        _check(lib().rt_set_segmentation(self._h, int(wgs_per_cu)), "rt_set_segmentation", self._h)

    def set_moments_form(self, form: int):
        """rt_set_moments_form: 1 producer/consumer (default), 0 one-wave moments kernel."""
        _check(lib().rt_set_moments_form(self._h, int(form)), "rt_set_moments_form", self._h)

    def set_phi_correction_form(self, form: int):
        """rt_set_phi_correction_form: 0 closed forms (default), 1 the cell-by-cell walk."""
        _check(lib().rt_set_phi_correction_form(self._h, int(form)), "rt_set_phi_correction_form", self._h)

    def debug_fail_launch(self, after: int):
        """rt_debug_fail_launch: the pipelined sub-launch after `after` more fails (-1: off)."""
        _check(lib().rt_debug_fail_launch(self._h, int(after)), "rt_debug_fail_launch", self._h)

    def debug_set_transfer_chunk(self, doubles: int):
        """rt_debug_set_transfer_chunk: host transfers in pieces of at most `doubles` doubles
        (0: the defaults)."""
        _check(lib().rt_debug_set_transfer_chunk(self._h, int(doubles)), "rt_debug_set_transfer_chunk", self._h)

    def pipeline_state(self) -> dict:
        """{"lag_steps", "queued_steps", "pending"} (rt_pipeline_state)."""
        lag, q, pend = C.c_longlong(), C.c_int(), C.c_int()
        _check(lib().rt_pipeline_state(self._h, C.byref(lag), C.byref(q), C.byref(pend)), "rt_pipeline_state", self._h)
        return {"lag_steps": lag.value, "queued_steps": q.value, "pending": bool(pend.value)}

    def sweep_traffic(self):
        b = C.c_double()
        u = C.c_double()
        _check(lib().rt_sweep_traffic(self._h, C.byref(b), C.byref(u)), "rt_sweep_traffic", self._h)
        # (algorithmic bytes per pass = per profiled launch, updates per full step)
        return b.value, u.value

    def sweep_flops(self) -> float:
        """Algorithmic FP64 flops of one pass (rt_sweep_flops)."""
        f = C.c_double()
        _check(lib().rt_sweep_flops(self._h, C.byref(f)), "rt_sweep_flops", self._h)
        return f.value

    def sweep_geometry(self):
        wg = C.c_int()
        t = C.c_longlong()
        _check(lib().rt_sweep_geometry(self._h, C.byref(wg), C.byref(t)), "rt_sweep_geometry", self._h)
        return wg.value, t.value


def _shard(h) -> dict:
    v = [C.c_int() for _ in range(6)]
    _check(lib().rt_get_shard(h, *[C.byref(x) for x in v]), "rt_get_shard", h)
    return dict(zip(("G", "M", "g_lo", "g_hi", "d_lo", "d_hi"), (x.value for x in v)))


class Comm:
    """rt_comm (include/rtsn.h, multi-GPU): an RCCL communicator joining the ranks' shard
    handles, one process per GPU.  Every method is collective over the ranks.

    uid = Comm.unique_id() on one rank, handed to the others (e.g. by torch.distributed's
    broadcast_object_list or a file); Comm(nranks, rank, uid, device).  Every wait on the
    collective is bounded by RTSN_COMM_TIMEOUT_S seconds (default 300) from the moment the
    stream reaches it: a missing or stalled rank gives RtError status 7 (RT_ERR_TIMEOUT)
    instead of a hang; the handle's own queued work is not clocked.  allreduce_absorption and
    material_step leave their all-reduces on the handle's stream: retire them with
    synchronize() before any other host wait on the handle (Solver.temperature(),
    Solver.synchronize(), a read-out), whose waits have no deadline."""

    def __init__(self, nranks: int, rank: int, uid: bytes, device: int = 0):
        assert len(uid) == 128
        h = C.c_void_p()
        st = lib().rt_comm_init(nranks, rank, uid, device, C.byref(h))
        if st:
            raise RtError(st, "rt_comm_init (" + lib().rt_comm_last_error(None).decode(errors="replace") + ")")
        self._h = h

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        st = lib().rt_comm_unique_id(buf)
        if st:
            raise RtError(st, "rt_comm_unique_id (" + lib().rt_comm_last_error(None).decode(errors="replace") + ")")
        return buf.raw

    def _check(self, st, what):
        if st:
            raise RtError(st, f"{what} ({lib().rt_comm_last_error(self._h).decode(errors='replace')})")

    def close(self):
        if getattr(self, "_h", None):
            lib().rt_comm_destroy(self._h)
            self._h = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def rank(self):
        n, r = C.c_int(), C.c_int()
        self._check(lib().rt_comm_rank(self._h, C.byref(n), C.byref(r)), "rt_comm_rank")
        return n.value, r.value

    @property
    def count(self) -> int:
        """ncclCommCount: the ranks RCCL reports for the communicator."""
        n = C.c_int()
        self._check(lib().rt_comm_count(self._h, C.byref(n)), "rt_comm_count")
        return n.value

    def gather_moments(self, solver: "Solver"):
        """phi, F, phi_plus of all groups, (G, N) each, on every rank."""
        sh = _shard(solver._h)
        out = [np.empty((solver.N, sh["G"])) for _ in range(3)]
        self._check(lib().rt_comm_gather_moments(self._h, solver._h, *[_dp(a) for a in out]), "rt_comm_gather_moments")
        return tuple(a.T for a in out)

    def gather_group_ends(self, solver: "Solver"):
        G = _shard(solver._h)["G"]
        left, right = np.empty(G), np.empty(G)
        self._check(lib().rt_comm_gather_group_ends(self._h, solver._h, _dp(left), _dp(right)),
                    "rt_comm_gather_group_ends")
        return left, right

    def gather_balance(self, solver: "Solver"):
        """(balance, sources, sinks) of all groups."""
        G = _shard(solver._h)["G"]
        b, so, si = np.empty(G), np.empty(G), np.empty(G)
        self._check(lib().rt_comm_gather_balance(self._h, solver._h, _dp(b), _dp(so), _dp(si)), "rt_comm_gather_balance")
        return b, so, si

    def gather_psi(self, solver: "Solver", root: int = 0):
        """psi (M, G, N) of the whole configuration on `root` (None elsewhere)."""
        sh = _shard(solver._h)
        mine = self.rank[1] == root
        psi = np.empty((solver.N, sh["G"], sh["M"])) if mine else None
        ptr = _dp(psi) if mine else None
        self._check(lib().rt_comm_gather_psi(self._h, solver._h, root, ptr), "rt_comm_gather_psi")
        return psi.transpose(2, 1, 0) if mine else None

    def allreduce_absorption(self, solver: "Solver", out):
        """A(x) over all groups into the device tensor `out` (N doubles), stream-ordered."""
        self._check(lib().rt_comm_allreduce_absorption(self._h, solver._h, C.c_void_p(out.data_ptr())),
                    "rt_comm_allreduce_absorption")

    def material_step(self, solver: "Solver", nsteps: int = 1):
        """nsteps coupled steps with one all-reduce of q(x) per step on the handle's stream."""
        self._check(lib().rt_comm_material_step(self._h, solver._h, int(nsteps)), "rt_comm_material_step")

    def synchronize(self, solver: "Solver"):
        """Host wait for the handle's stream (its sweeps and this communicator's stream-ordered
        collectives), bounded by RTSN_COMM_TIMEOUT_S (RtError status 7 after an abort)."""
        self._check(lib().rt_comm_synchronize(self._h, solver._h), "rt_comm_synchronize")


def comm_version() -> dict:
    """rt_comm_version: the RCCL the library's collectives run on -- ncclGetVersion's code
    and version string, and the librccl file the process resolved it from."""
    v = C.c_int()
    path = C.create_string_buffer(4096)
    _check(lib().rt_comm_version(C.byref(v), path, len(path)), "rt_comm_version")
    code = v.value
    major, rest = divmod(code, 10000)
    minor, patch = divmod(rest, 100)
    return {"code": code, "version": f"{major}.{minor}.{patch}", "path": path.value.decode(errors="replace")}


class Layout:
    """Host-side layout of the gathered shard blocks (include/rtsn.h rt_layout_*): the copy
    plans the rt_comm gathers run on the device, on numpy arrays.  shards: one dict (or
    tuple) per rank with G, M, g_lo, g_hi, d_lo, d_hi, N."""

    def __init__(self, shards):
        n = len(shards)
        self.n = n
        arr = (rt_shard * n)()
        for r, sh in enumerate(shards):
            if not isinstance(sh, dict):
                sh = dict(zip(("G", "M", "g_lo", "g_hi", "d_lo", "d_hi", "N"), sh))
            for f in ("G", "M", "g_lo", "g_hi", "d_lo", "d_hi", "N"):
                setattr(arr[r], f, int(sh[f]))
            arr[r].reserved = 0
        self._sh = arr
        mode, gm = C.c_int(), C.c_int()
        st = lib().rt_layout_mode(arr, n, C.byref(mode), C.byref(gm))
        self.mode, self.max_groups = mode.value, gm.value
        _check(st, "rt_layout_mode")
        self.G, self.M, self.N = arr[0].G, arr[0].M, arr[0].N

    def shard(self, r: int) -> rt_shard:
        return self._sh[r]

    @staticmethod
    def _need(arr, count: int, what: str, out: bool = False) -> np.ndarray:
        """The C plans read and write through raw pointers: a float64 array of at least count
        elements (an output also C-contiguous, since it is written in place)."""
        if out:
            if not (isinstance(arr, np.ndarray) and arr.dtype == np.float64 and arr.flags["C_CONTIGUOUS"]):
                raise ValueError(f"{what}: the output must be a C-contiguous float64 numpy array")
        else:
            arr = np.ascontiguousarray(arr, dtype=np.float64)
        if arr.size < count:
            raise ValueError(f"{what}: {arr.size} elements, the layout needs at least {count}")
        return arr

    def _shard_dims(self, rank: int):
        if not 0 <= rank < self.n:
            raise ValueError(f"rank {rank} outside [0, {self.n})")
        sh = self._sh[rank]
        return 2 * (sh.d_hi - sh.d_lo), sh.g_hi - sh.g_lo

    def pack_moments(self, rank: int, phi, F, phi_plus) -> np.ndarray:
        """rank's (N, G_local) fields (g fastest) -> its wire block (3, N, Gmax)."""
        local = np.ascontiguousarray(np.stack([phi, F, phi_plus]), dtype=np.float64)
        block = np.empty((3, self.N, self.max_groups))
        _check(lib().rt_layout_pack_moments(self._sh, self.n, rank, _dp(local), _dp(block)), "rt_layout_pack_moments")
        return block

    def unpack_moments(self, gathered: np.ndarray):
        """gathered wire blocks -> phi, F, phi_plus as (N, G) arrays (g fastest)."""
        blocks = 1 if self.mode == 1 else self.n  # direction shards: one summed block
        g = self._need(gathered, blocks * 3 * self.N * self.max_groups, "unpack_moments: gathered")
        out = [np.empty((self.N, self.G)) for _ in range(3)]
        _check(lib().rt_layout_unpack_moments(self._sh, self.n, _dp(g), *[_dp(a) for a in out]),
               "rt_layout_unpack_moments")
        return out

    def pack_vectors(self, rank: int, vecs) -> np.ndarray:
        vecs = [np.ascontiguousarray(v, dtype=np.float64) for v in vecs]
        ptrs = (C.POINTER(C.c_double) * len(vecs))(*[_dp(v) for v in vecs])
        block = np.empty((len(vecs), self.max_groups))
        _check(lib().rt_layout_pack_vectors(self._sh, self.n, rank, len(vecs), ptrs, _dp(block)),
               "rt_layout_pack_vectors")
        return block

    def unpack_vectors(self, k: int, gathered: np.ndarray):
        blocks = 1 if self.mode == 1 else self.n
        g = self._need(gathered, blocks * k * self.max_groups, "unpack_vectors: gathered")
        out = [np.empty(self.G) for _ in range(k)]
        ptrs = (C.POINTER(C.c_double) * k)(*[_dp(v) for v in out])
        _check(lib().rt_layout_unpack_vectors(self._sh, self.n, k, _dp(g), ptrs), "rt_layout_unpack_vectors")
        return out

    def place_psi(self, rank: int, block: np.ndarray, psi_flat: np.ndarray):
        """rank's psi (as rt_get_psi's flat ColMajor (M_l, G_l, N) buffer) into psi_flat
        (the (M, G, N) ColMajor buffer, i + M (g + G c))."""
        Ml, Gl = self._shard_dims(rank)
        b = self._need(block, Ml * Gl * self.N, "place_psi: block")
        self._need(psi_flat, self.M * self.G * self.N, "place_psi: psi_flat", out=True)
        _check(lib().rt_layout_place_psi(C.byref(self._sh[rank]), _dp(b), _dp(psi_flat)), "rt_layout_place_psi")

    def place_psi_source(self, rank: int, rows: np.ndarray, table: np.ndarray):
        Ml, _ = self._shard_dims(rank)
        r = self._need(rows, Ml * self.G, "place_psi_source: rows")
        self._need(table, self.M * self.G, "place_psi_source: table", out=True)
        _check(lib().rt_layout_place_psi_source(C.byref(self._sh[rank]), _dp(r), _dp(table)),
               "rt_layout_place_psi_source")
