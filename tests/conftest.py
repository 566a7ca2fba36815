import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def spt():
    """The product package (small-pathtracer_amd); libspt.so must have been built."""
    mod = importlib.import_module("small-pathtracer_amd")
    if not os.path.exists(mod.LIB_PATH):
        import __graft_entry__
        __graft_entry__.build()
    mod.load_library()
    return mod


@pytest.fixture(scope="session")
def oracle(spt):
    from oracle import oracle as o
    o.lib()
    return o
