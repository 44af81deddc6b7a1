"""Where the engine's write bytes go per access: the CPU
restatement, built with its CPUREF_TRACE hook (tools/reuse/write_audit.cpp),
on bench.py's C4 replica-0 stream after the bench's warm-up, counting the
stores the engine makes for the same events: a 32-B queue header per link
visit, the free-interval ring slots a tree operation writes back (16 B each),
the L1 line's timestamp (8 B) per access and its 16-B record per miss or
downward state change, a 24-B directory line per home-slice access, the 4-B
delay and the 8-B completion cycle per request.  CPU only.

    python tools/reuse/write_audit.py [--replay open|closed] [--requests N] [--json out.json]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def build() -> str:
    out = os.path.join(ROOT, "build", "libwrite_audit.so")
    src = os.path.join(ROOT, "tools", "reuse", "write_audit.cpp")
    deps = [src, os.path.join(ROOT, "oracle", "cpu_ref.cpp")]
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(d) for d in deps):
        os.makedirs(os.path.dirname(out), exist_ok=True)
        subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-w",
                        "-I" + os.path.join(ROOT, "include"), "-o", out, src], check=True)
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--replay", choices=("closed", "open"), default="open")
    ap.add_argument("--requests", type=int, default=100000)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--chunk", type=int, default=40960)
    ap.add_argument("--json", default="")
    a = ap.parse_args()

    import oracle as O
    O.ORACLE_LIB = build()
    O._olib = None
    L = O.oracle_lib()
    L.audit_enable.argtypes = [C.c_int]
    L.audit_read.argtypes = [C.c_void_p, C.c_int]

    import bench
    import primesim_amd as P
    from primesim_amd import config as CF
    from primesim_amd.dist import replica_seed
    cfg = P.config_from_dict(CF.preset("C4"))
    n_w = a.warmup * a.chunk
    reqs = P.generate_stream(bench.stream_spec(replica_seed(bench.SEED_BASE, 0, 0), n_w + a.requests))
    ref = O.CpuRef(cfg)
    ref.set_mode(O.MODE_CLOSED if a.replay == "closed" else 0)
    for prog, th in P.stream_threads(bench.stream_spec(bench.SEED_BASE)):
        ref.alloc_core(prog, th)
    for s in range(0, n_w, 16384):
        ref.run(reqs[s:min(n_w, s + 16384)])
    before = ref.stats().as_dict()
    L.audit_enable(1)
    for s in range(n_w, n_w + a.requests, 16384):
        d, rc = ref.run(reqs[s:min(n_w + a.requests, s + 16384)])
        if rc != 0:
            break
    L.audit_enable(0)
    st = {k: v - before.get(k, 0) for k, v in ref.stats().as_dict().items() if isinstance(v, int)}
    out = np.zeros(6, dtype=np.uint64)
    L.audit_read(out.ctypes.data, 6)
    visits, tree, slots, splits, removes, shrinks = (int(x) for x in out)
    A = max(1, st["requests"])
    per = {
        "queue headers (32 B per link visit)": 32.0 * visits / A,
        "free-interval ring slots (16 B each)": 16.0 * slots / A,
        "L1 timestamps (8 B per access)": 8.0,
        "L1 line records (16 B per miss)": 16.0 * st["L0_miss"] / A,
        "L1 records changed by invalidations / shares (16 B each)": 16.0 * st["lockdown_calls"] / A,
        "directory lines (24 B per home-slice access)": 24.0 * st["directory_ins"] / A,
        "delay + completion cycle (4 + 8 B)": 12.0,
    }
    res = {"replay": a.replay, "requests": A, "link_visits_per_access": visits / A, "tree_visits_per_access": tree / A,
           "ring_slots_per_tree_visit": slots / max(1, tree),
           "tree_ops": {"splits": splits, "removals": removes, "shrinks": shrinks},
           "engine_store_bytes_per_access": per, "total_store_bytes_per_access": sum(per.values())}
    print(json.dumps(res, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
