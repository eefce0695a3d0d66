import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "multicol-slam-annotation_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) device")


@pytest.fixture(scope="session")
def built():
    """Build (incrementally) the HIP library and the oracle before any test uses them."""
    import __graft_entry__ as g
    g.build_hip()
    g.build_oracle()
    return True


@pytest.fixture(scope="session")
def gpu(built):
    import mcs_amd
    if mcs_amd.device_count() < 1:
        pytest.fail("gpu-marked test but no HIP device visible (no CPU fallback exists)")
    return True
