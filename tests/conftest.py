"""Shared fixtures.  `-m gpu` tests need an MI355X (gfx950) and librtsn.so;
everything else runs on the CPU (oracle, host logic, C-ABI loading)."""
import os
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "radiative-transfer_amd"))
sys.path.insert(0, str(REPO / "oracle"))
sys.path.insert(0, str(REPO / "tests"))

PRM_DIR = REPO / "tests" / "golden" / "prm"
SEED = 20261015


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built librtsn.so")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def prm_dir():
    return PRM_DIR


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle  # noqa: WPS433
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def rtsn_mod():
    import rtsn
    return rtsn


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
