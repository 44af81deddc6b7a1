"""Warm the compile-time-configuration cache (primesim_amd/jit_cache/) for every
configuration the GPU tests, smoke() and bench.py use: the golden XMLs, the
C1-C5 presets and the DRAM-bank test geometries.  Runs on the CPU (hipRTC needs
no GPU), several compiles at once; a configuration already cached is skipped.

    python3 tools/jit_warm.py [-j N]
"""
from __future__ import annotations

import argparse
import ctypes as C
import glob
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


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
    return out


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
    a = ap.parse_args()
    items = [(n, bytes(c)) for n, c in configs()]
    bad = 0
    t0 = time.time()
    with ProcessPoolExecutor(a.j) as ex:
        for name, rc, dt, err in ex.map(_warm, items):
            if rc < 0:
                bad += 1
                print(f"[jit_warm] {name}: FAILED {err[:2000]}", flush=True)
            elif rc == 0:
                print(f"[jit_warm] {name}: compiled in {dt:.1f}s", flush=True)
    # drop code objects no current configuration uses (older sources or geometries)
    cache = os.environ.get("PRIMEUNCORE_JIT_CACHE") or os.path.join(ROOT, "primesim_amd", "jit_cache")
    stale = [f for f in glob.glob(os.path.join(cache, "*.hsaco")) if os.path.getmtime(f) < t0 - 1]
    if not bad:
        for f in stale:
            os.remove(f)
    print(f"[jit_warm] {len(items)} configurations, {bad} failed, {len(stale) if not bad else 0} stale code objects "
          f"removed, {time.time() - t0:.0f}s", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
