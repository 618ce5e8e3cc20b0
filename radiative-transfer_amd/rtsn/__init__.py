"""rtsn -- Python front end of librtsn.so, the MI355X-native S_n solver.

Mirrors the reference's host interface (Helblindi/radiative-transfer
include/ParameterHandler.h, include/solver.h) over the C ABI declared in
include/rtsn.h.  The HIP library is required: importing works anywhere, but
creating a Solver without a gfx950 device raises RtError -- there is no CPU
fallback in this package.
"""
from .api import (  # noqa: F401
    Comm,
    Layout,
    LIB_PATH,
    ParameterHandler,
    RtError,
    Solver,
    build,
    comm_version,
    exported_symbols,
    lib,
    params_default,
    plan_time_block,
    planck_groups,
    quadrature,
)
