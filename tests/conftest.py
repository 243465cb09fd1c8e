"""Test configuration: markers, import paths, shared fixtures.

`-m "not gpu"` runs here (no GPU): oracle KATs + golden fixtures, host logic,
ABI/export checks, gloo multi-process tests.  `-m gpu` runs on the MI355X and
compares the HIP path (through the C-ABI) with the CPU oracle.
"""
import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "oracle"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

import vo_amd  # noqa: E402,F401  (registers the package as r7020e_visual_odometry_amd)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device; runs through libvo.so")
    config.addinivalue_line("markers", "slow: longer CPU oracle runs")


@pytest.fixture(scope="session")
def oracle():
    import oracle as o
    o.build()
    return o


@pytest.fixture(scope="session")
def vo():
    from r7020e_visual_odometry_amd import vo as v
    return v


@pytest.fixture(scope="session")
def syn():
    from r7020e_visual_odometry_amd import synthetic as s
    return s
