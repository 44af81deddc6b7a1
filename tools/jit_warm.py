"""Warm the compile-time-configuration cache (primesim_amd/jit_cache/) for every
configuration the GPU tests, smoke() and bench.py use: the golden XMLs, the
C1-C5 presets, the DRAM-bank test geometries and tests/extra_configs.py.  Runs on the CPU (hipcc, in a
child process of each worker; no GPU), several compiles at once; a configuration already cached is skipped.
A same-box A/B of compile options (tools/gpu_session.sh V@FLAGS) compiles its variant with hipRTC on the
GPU box unless the variant is warmed here first with the same environment:

    python3 tools/jit_warm.py [-j N] [--only "preset C4"]
    PRIMEUNCORE_JIT_EXTRA="..." python3 tools/jit_warm.py --only "preset C4"
"""
from __future__ import annotations

import argparse
import ctypes as C
import glob
import os
import subprocess
import sys
import time
from concurrent.futures import ProcessPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PRUNE_HOURS = 1   # grace for code objects written by a library being rebuilt
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
# this process and its workers never touch the GPU: the library may start the
# offline compiler (hipcc) here, and only here (jit.cpp offline_allowed)
os.environ["PRIMEUNCORE_JIT_OFFLINE"] = "1"


def configs():
    import primesim_amd as P
    from primesim_amd import config as CF
    out = []
    for x in sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "*.xml"))):
        out.append((os.path.basename(x), P.load_config(x)))
    for name in ("C1", "C2", "C3", "C4", "C5"):
        out.append((f"preset {name}", P.config_from_dict(CF.preset(name))))
    try:
        from dram_cases import dram_configs
        out.extend(dram_configs())
    except ImportError:
        pass
    try:
        from extra_configs import extra_configs
        out.extend(extra_configs())
    except ImportError:
        pass
    return out


def live_source_tags() -> set:
    """Source tags (pu_jit_source_tag) of every engine library in the tree:
    the product library and experiment builds (libprimeuncore_*.so).  Each is
    asked in a child process, so their identical symbol names never meet."""
    tags = set()
    for lib in glob.glob(os.path.join(ROOT, "primesim_amd", "libprimeuncore*.so")):
        r = subprocess.run([sys.executable, "-c", "import ctypes, sys; f = ctypes.CDLL(sys.argv[1]).pu_jit_source_tag; "
                            "f.restype = ctypes.c_char_p; print(f().decode())", lib],
                           capture_output=True, text=True, timeout=60)
        if r.returncode == 0 and r.stdout.strip():
            tags.add(r.stdout.strip())
    return tags


def _warm(item):
    name, cfg_bytes = item
    import primesim_amd as P
    from primesim_amd import _abi as A
    from primesim_amd import uncore
    cfg = A.SimCfg.from_buffer_copy(cfg_bytes)
    t = time.time()
    rc = uncore.lib().pu_config_jit_warm(C.byref(cfg))
    return name, rc, time.time() - t, uncore.last_error() if rc < 0 else ""


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--only", default="", help="warm only the configurations whose name contains this")
    a = ap.parse_args()
    items = [(n, bytes(c)) for n, c in configs() if a.only in n]
    bad = 0
    t0 = time.time()
    with ProcessPoolExecutor(a.j) as ex:
        for name, rc, dt, err in ex.map(_warm, items):
            if rc < 0:
                bad += 1
                print(f"[jit_warm] {name}: FAILED {err[:2000]}", flush=True)
            elif rc == 0:
                print(f"[jit_warm] {name}: compiled in {dt:.1f}s", flush=True)
    # drop code objects of the in-tree cache compiled from sources no library in
    # the tree embeds (their name's prefix is the source tag), after an hour's
    # grace: code objects pu_create compiled on demand for user configurations
    # and those of experiment builds stay; a cache outside the tree
    # (PRIMEUNCORE_JIT_CACHE) is never pruned
    intree = os.path.join(ROOT, "primesim_amd", "jit_cache")
    cache = os.environ.get("PRIMEUNCORE_JIT_CACHE") or intree
    stale = []
    if not bad and not a.only and os.path.realpath(cache) == os.path.realpath(intree):
        live = live_source_tags()
        # the product library's own tag, read in this process: if it is missing
        # from what the children reported (a child load failed, a library
        # lacks the symbol), nothing is pruned
        from primesim_amd import uncore
        own = uncore.lib().pu_jit_source_tag
        own.restype = C.c_char_p
        own_tag = own().decode()
        if own_tag not in live:
            print(f"[jit_warm] the product library's source tag {own_tag} was not among the tags read back "
                  f"({sorted(live)}): nothing pruned", flush=True)
            live = None
        for f in glob.glob(os.path.join(cache, "*.hsaco")) if live else []:
            tag = os.path.basename(f).split("-")[0]
            if tag not in live and os.path.getmtime(f) < t0 - PRUNE_HOURS * 3600:
                stale.append(f)
        for f in stale:
            os.remove(f)
    print(f"[jit_warm] {len(items)} configurations, {bad} failed, {len(stale)} code objects of sources no library "
          f"here compiles removed, {time.time() - t0:.0f}s", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
