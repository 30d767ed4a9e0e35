"""Shared fixtures.  `-m gpu` tests need a gfx950 device; everything else
runs on the CPU (the oracle, the host-side code of liblqro.so, gloo)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lqr-obstacles_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
GOLDEN = os.path.join(ROOT, "tests", "golden")
REFERENCE = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    pyoracle.lib()
    return pyoracle


@pytest.fixture(scope="session")
def lqro_mod():
    import lqro
    if os.environ.get("LQRO_LIB"):   # a variant library in lqr-obstacles_amd/ (A/B and regression runs)
        lqro.LIB_PATH = os.path.join(os.path.dirname(lqro.LIB_PATH), os.environ["LQRO_LIB"])
    if not os.path.exists(lqro.LIB_PATH):
        import __graft_entry__ as ge
        ge.build_lib()
    lqro.lib()
    return lqro


@pytest.fixture(scope="session")
def gains(oracle):
    return oracle.synthesize()
