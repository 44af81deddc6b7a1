"""Source hash of the HIP engine library: sha256 over primesim_amd/csrc/{*.hip,*.cpp,*.h,Makefile}
and include/*.h (relative path + NUL + bytes, sorted by path), first 16 hex digits.

The Makefile bakes it into pu_version(); tests/conftest.py and smoke() recompute it
from the checkout and refuse a library built from other sources."""
import glob
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def files() -> list[str]:
    pats = ["primesim_amd/csrc/*.hip", "primesim_amd/csrc/*.cpp", "primesim_amd/csrc/*.h",
            "primesim_amd/csrc/Makefile", "include/*.h"]
    out = set()
    for p in pats:
        out.update(os.path.relpath(f, ROOT) for f in glob.glob(os.path.join(ROOT, p)))
    return sorted(out)


def src_hash() -> str:
    h = hashlib.sha256()
    for rel in files():
        h.update(rel.encode() + b"\0")
        with open(os.path.join(ROOT, rel), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    sys.stdout.write(src_hash())
