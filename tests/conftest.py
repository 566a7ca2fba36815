import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_sessionfinish(session, exitstatus):
    """SPT_MAPS_OUT=<file>: record which in-tree shared libraries this pytest process had mapped
    (scripts/gpu_record.py puts them in the committed GPU test record as proof that the HIP library
    ran, not a fallback)."""
    out = os.environ.get("SPT_MAPS_OUT")
    if not out:
        return
    with open("/proc/self/maps") as f:
        libs = sorted({ln.split()[-1] for ln in f if ln.rstrip().endswith(".so") and ROOT in ln})
    with open(out, "w") as f:
        f.write("\n".join(libs) + "\n")


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
