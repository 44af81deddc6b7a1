import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")


@pytest.fixture(scope="session", autouse=True)
def _built_libraries():
    """Build the engine/oracle libraries once if they are missing."""
    need = [os.path.join(ROOT, "primesim_amd", "libprimeuncore.so"), os.path.join(ROOT, "oracle", "libpu_oracle.so")]
    if not all(os.path.exists(p) for p in need):
        import __graft_entry__
        __graft_entry__.build()
    yield
