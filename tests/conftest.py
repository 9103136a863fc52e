import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def ctx():
    """EXACT-math context on device 0.  Fails (does not skip) without a GPU:
    -m gpu runs only where one exists and must exercise the native path."""
    import jwave_amd as jw
    c = jw.Context(0, "exact")
    yield c
    c.close()


@pytest.fixture(scope="session")
def ctx_fma():
    import jwave_amd as jw
    c = jw.Context(0, "fma")
    yield c
    c.close()
