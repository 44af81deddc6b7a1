"""Where the engine's time goes: region cycle counters of the profiling build.

Runs bench.py's workload against libprimeuncore_prof.so (make -C
primesim_amd/csrc prof: the same engine with s_memtime stamps, -DPU_PROF) and
prints, per region, the summed per-wave cycles and their share of the
per-request loop.  Regions are inclusive (NET contains NSETUP/NHOPS/NWB, NHOPS
contains NTREE, NTREE contains NWAIT, HOME contains the transmits it makes).

    python tools/prof_regions.py -- --steps 3 --warmup 1 --no-cpu
    python tools/prof_regions.py --jit -- --replicas 1 ...   (the shipped
        compiled-configuration kernels, latency mode included: the product
        library with PRIMEUNCORE_JIT_EXTRA=-DPU_PROF, its own cache entry;
        warm it first with the same environment: tools/jit_warm.py)
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF_LIB = os.environ.get("PROF_LIB") or os.path.join(ROOT, "primesim_amd", "libprimeuncore_prof.so")
NAMES = ["LOOP", "REQ", "NET", "NSETUP", "NHOPS", "NTREE", "NWAIT", "NWB", "SETL0", "SETLN", "HOME_LD",
         "HOME", "DOWN", "windows", "tree_hops", "demand_hops", "T_LDS", "T_SEARCH", "T_DECIDE", "T_EDIT",
         "T_STORE", "T_REFILL", "NPRE", "NPOST", "MG1RUN", "mg1_lanes", "mg1_cache_hits", "MAINTAIL",
         "mg1_cache_present", "mg1_helper_stored", "mg1_helper_batches", "T_UPD"]
COUNTS = {"windows", "tree_hops", "demand_hops", "mg1_lanes", "mg1_cache_hits", "mg1_cache_present",
          "mg1_helper_stored", "mg1_helper_batches"}


def main() -> None:
    jit = "--jit" in sys.argv[1:]
    if jit:
        # the compiled-configuration kernels with the counters compiled in
        os.environ["PRIMEUNCORE_JIT_EXTRA"] = "-DPU_PROF"
        os.environ["PU_PROF_JIT"] = "1"
    else:
        if not os.path.exists(PROF_LIB):
            raise SystemExit(f"{PROF_LIB} missing: make -C primesim_amd/csrc prof")
        os.environ["PRIMEUNCORE_LIB"] = PROF_LIB
        # the ahead-of-time kernels of the profiling build
        os.environ["PRIMEUNCORE_JIT"] = "0"
    os.environ["PU_PROF_RESET_AFTER_WARMUP"] = "1"
    sys.path.insert(0, ROOT)
    args = [a for a in sys.argv[1:] if a not in ("--", "--jit")]
    import bench  # noqa: E402
    import primesim_amd.uncore as U  # noqa: E402

    sys.argv = ["bench.py", *args]
    bench.main()
    L = U.lib()
    fn = L.pu_jit_prof_read if jit else L.pu_engine_prof_read
    fn.restype = C.c_int
    fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
    buf = (C.c_ulonglong * len(NAMES))()
    if fn(buf, len(NAMES), 0) <= 0:
        raise SystemExit("no region counters read (a kernel built with -DPU_PROF must have run)")
    vals = dict(zip(NAMES, (int(x) for x in buf)))
    loop = max(vals["LOOP"], 1)
    out = {}
    for k, v in vals.items():
        out[k] = v if k in COUNTS else {"cycles": v, "frac_of_loop": round(v / loop, 4)}
    # per-replica balance: summed per-block durations of the timed launches and
    # the last launch's start/end spread (s_memrealtime ticks, 100 MHz)
    R = min(4096, bench.LAST_REPLICAS or 0)
    if R and not jit:
        import numpy as np
        t0 = (C.c_ulonglong * R)()
        t1 = (C.c_ulonglong * R)()
        du = (C.c_ulonglong * R)()
        fb = L.pu_engine_prof_blocks
        fb.restype = C.c_int
        fb.argtypes = [C.POINTER(C.c_ulonglong)] * 3 + [C.c_int]
        if fb(t0, t1, du, R) == R:
            a0, a1, d = (np.array(list(x), dtype=np.float64) for x in (t0, t1, du))
            span = a1.max() - a0.min()
            if bench.LAST_PER_REPLICA is not None:
                dump = {k: np.array(v) for k, v in bench.LAST_PER_REPLICA.items()}
                dump["timed_dur_ticks"] = d
                np.savez(os.path.join(ROOT, "gpurun_out", "per_replica.npz"), **dump)
            out["blocks"] = {
                "replicas": R,
                "last_launch_span_ms": span / 1e5,
                "last_launch_end_ms_pcts": {p: float(np.percentile(a1 - a0.min(), p) / 1e5) for p in (0, 10, 50, 90, 99, 100)},
                "last_launch_start_ms_max": float((a0.max() - a0.min()) / 1e5),
                "timed_dur_ms_pcts": {p: float(np.percentile(d, p) / 1e5) for p in (0, 10, 50, 90, 99, 100)},
                "busy_fraction_last_launch": float((a1 - a0).sum() / (span * R)),
            }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
