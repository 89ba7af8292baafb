"""Shared test setup.

`-m "not gpu"` (CPU): oracle KATs, golden fixtures, host logic, ABI exports.
`-m gpu` (MI355X): GPU-vs-oracle parity through the C-ABI (libkfx.so).
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "slam-kinectfusion_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libkfx.so on the device)")


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle
    if not os.path.exists(oracle.LIB_PATH):
        oracle.build()
    return oracle


@pytest.fixture(scope="session")
def kfx_lib():
    import kfx
    if not os.path.exists(kfx.LIB_PATH):
        kfx.build()
    return kfx
