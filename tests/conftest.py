import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "gym-narde_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def golden(name):
    import numpy as np

    return dict(np.load(os.path.join(GOLDEN, name), allow_pickle=False))


@pytest.fixture(scope="session")
def hostcheck():
    """Test-only host build of the device rules engine (tests/hostcheck)."""
    import ctypes

    path = os.environ.get("NARDE_HOSTCHECK_LIB",  # tools/sanitize.sh: an ASan/UBSan build
                          os.path.join(ROOT, "tests", "hostcheck", "build", "libhostcheck.so"))
    if not os.path.exists(path):
        import __graft_entry__ as g

        g.build()
    return ctypes.CDLL(path)
