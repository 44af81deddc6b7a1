"""Register, spill and LDS use of the compiled-configuration kernels of one
preset: the code objects the build-time warm-up (hipcc) produces (pu_config_jit_warm
into a scratch cache), read from its AMDGPU metadata.  No GPU.

    python tools/kernel_resources.py [C4] [--lib primesim_amd/libprimeuncore_X.so]
"""
from __future__ import annotations

import argparse
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
KEYS = (".vgpr_count", ".agpr_count", ".sgpr_count", ".vgpr_spill_count", ".sgpr_spill_count",
        ".group_segment_fixed_size", ".private_segment_fixed_size")


def resources(preset: str, lib: str | None = None) -> dict:
    with tempfile.TemporaryDirectory() as d:
        env = dict(os.environ, PRIMEUNCORE_JIT_CACHE=d, PRIMEUNCORE_JIT_OFFLINE="1")   # hipcc, as shipped
        if lib:
            env["PRIMEUNCORE_LIB"] = os.path.abspath(lib)
        code = ("import ctypes as C, sys; sys.path.insert(0, %r); import primesim_amd as P; "
                "from primesim_amd import config as CF, uncore; cfg = P.config_from_dict(CF.preset(%r)); "
                "rc = uncore.lib().pu_config_jit_warm(C.byref(cfg)); sys.exit(0 if rc >= 0 else 1)") % (ROOT, preset)
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True)
        if r.returncode != 0:
            raise SystemExit(r.stderr[-3000:])
        # two code objects per configuration (jit.cpp: throughput and latency kernels)
        notes = "".join(subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", hsaco],
                                       capture_output=True, text=True).stdout
                        for hsaco in sorted(glob.glob(os.path.join(d, "*.hsaco"))))
    # one map per kernel, keys in alphabetical order (.agpr_count first, .name
    # in the middle): a kernel's entry starts at its .agpr_count line
    out: dict = {}
    entry: dict = {}
    for ln in notes.splitlines():
        s = ln.strip().lstrip("- ")
        if s.startswith(".agpr_count:"):
            entry = {}
        m = re.match(r"\.name:\s+(\S+)", s)
        if m and m.group(1).startswith("pu_jit"):
            out[m.group(1)] = entry
            continue
        m = re.match(r"(\.[a-z_]+):\s+(\d+)$", s)
        if m and m.group(1) in KEYS:
            entry[m.group(1)] = int(m.group(2))
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("preset", nargs="?", default="C4")
    ap.add_argument("--lib", default=None)
    a = ap.parse_args()
    for k, v in sorted(resources(a.preset, a.lib).items()):
        print(k, v)


if __name__ == "__main__":
    main()
