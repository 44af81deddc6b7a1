import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")


def _built_hash() -> str:
    """Source hash baked into libprimeuncore.so (pu_version), read in a child
    process so this one never maps a stale library."""
    code = ("import ctypes,sys; L=ctypes.CDLL(sys.argv[1]); L.pu_version.restype=ctypes.c_char_p; "
            "v=L.pu_version().decode(); print(v.rsplit(' src ',1)[1] if ' src ' in v else '')")
    lib = os.path.join(ROOT, "primesim_amd", "libprimeuncore.so")
    r = subprocess.run([sys.executable, "-c", code, lib], capture_output=True, text=True)
    return r.stdout.strip() if r.returncode == 0 else ""


@pytest.fixture(scope="session", autouse=True)
def _built_libraries():
    """The engine under test must be built from the checked-out sources:
    rebuild where the toolchain and the reference live (this container), refuse
    a mismatching binary elsewhere (the GPU box runs what was shipped)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from src_hash import src_hash
    need = [os.path.join(ROOT, "primesim_amd", "libprimeuncore.so"), os.path.join(ROOT, "oracle", "libpu_oracle.so")]
    want = src_hash()
    if not all(os.path.exists(p) for p in need) or _built_hash() != want:
        if os.path.isdir("/root/reference/src") or not os.path.exists(need[0]):
            import __graft_entry__
            __graft_entry__.build()
        got = _built_hash()
        if got != want:
            pytest.exit(f"libprimeuncore.so was built from sources {got!r}, the checkout is {want!r}: "
                        "run __graft_entry__.build() before shipping", returncode=3)
    yield
