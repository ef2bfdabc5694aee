"""pytest configuration: `gpu` marker, import paths for the package and the oracle."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "lqr.jl_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs on the MI355X box)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as o
    o.load()
    return o


@pytest.fixture(scope="session")
def lqrx():
    import lqrx as L
    L.load()
    return L


@pytest.fixture(scope="session")
def gpu_ok(lqrx):
    if lqrx.load().lqrx_device_available() != 1:
        pytest.fail("gpu-marked test but no gfx950 device visible to liblqrx.so")
    return True
