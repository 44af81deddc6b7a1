"""Reuse of the link rings the lone wave's tree hops touch.

Runs the CPU restatement, built with its CPUREF_TRACE hook
(tools/reuse/tree_reuse.cpp), on bench.py's C4 replica-0 stream: the same
warmup as the bench (--warmup x --chunk requests, not recorded), then
--requests recorded requests, open or closed loop.  For every link visit that
takes the tree branch of computeQueueDelay (the branch whose free-interval
ring is staged into LDS and written back) it records the LRU stack distance
among tree-visited links, and prints what fraction of tree visits find their
ring among the last K tree-visited rings (the hit rate of an on-chip cache of
K rings), for K = 4 .. 256.  CPU only.

    python tools/reuse/tree_reuse.py [--replay closed|open] [--requests N]
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
KMAX = 512


def build() -> str:
    out = os.path.join(ROOT, "build", "libtree_reuse.so")
    src = os.path.join(ROOT, "tools", "reuse", "tree_reuse.cpp")
    deps = [src, os.path.join(ROOT, "oracle", "cpu_ref.cpp")]
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(d) for d in deps):
        os.makedirs(os.path.dirname(out), exist_ok=True)
        subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-w",
                        "-I" + os.path.join(ROOT, "include"), "-o", out, src], check=True)
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--replay", choices=("closed", "open"), default="closed")
    ap.add_argument("--requests", type=int, default=100000)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--chunk", type=int, default=40960)
    ap.add_argument("--json", default="")
    a = ap.parse_args()

    import oracle as O
    O.ORACLE_LIB = build()
    O._olib = None
    L = O.oracle_lib()
    L.trace_enable.argtypes = [C.c_int]
    L.trace_read.argtypes = [C.c_void_p, C.c_int]
    L.trace_read.restype = C.c_int

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
    L.trace_enable(1)
    done = 0
    for s in range(n_w, n_w + a.requests, 16384):
        d, rc = ref.run(reqs[s:min(n_w + a.requests, s + 16384)])
        done += len(d) if rc == 0 else max(rc, 0)
        if rc != 0:
            break
    L.trace_enable(0)
    buf = np.zeros(3 + 2 * (KMAX + 1) + 128, dtype=np.uint64)
    assert L.trace_read(buf.ctypes.data, len(buf)) == len(buf)
    visits, tree, ksum = int(buf[0]), int(buf[1]), int(buf[2])
    h_tree = buf[3:3 + KMAX + 1].astype(np.float64)
    h_all = buf[3 + KMAX + 1:3 + 2 * (KMAX + 1)].astype(np.float64)
    h_k = buf[3 + 2 * (KMAX + 1):].astype(np.float64)
    ks = (1, 2, 4, 8, 12, 16, 24, 32, 48, 64, 128, 256, 512)
    res = {
        "replay": a.replay, "requests": done, "warmup_requests": n_w,
        "link_visits_per_access": visits / max(1, done),
        "tree_visits_per_access": tree / max(1, done),
        "mean_found_index_at_tree_visit": ksum / max(1, tree),
        "tree_visits_found_below_k": {k: float(h_k[:k].sum() / max(1, tree)) for k in (1, 2, 4, 8, 16, 32, 64, 96, 128)},
        "tree_hit_rate_last_k_tree_rings": {k: float(h_tree[:k].sum() / max(1, tree)) for k in ks},
        "visit_hit_rate_last_k_links": {k: float(h_all[:k].sum() / max(1, visits)) for k in ks},
    }
    print(f"[tree_reuse] C4 replica 0, {a.replay} loop, {done} requests after a {n_w}-request warmup")
    print(f"  link visits/access {res['link_visits_per_access']:.1f}, tree visits/access "
          f"{res['tree_visits_per_access']:.2f}, mean index of the interval a tree search stops at "
          f"{res['mean_found_index_at_tree_visit']:.1f}")
    print("  tree searches stopping below index K: " +
          ", ".join(f"K={k} {v:.3f}" for k, v in res["tree_visits_found_below_k"].items()))
    print("  K    tree visits whose ring is among the last K tree-visited rings | any visit among the last K links")
    for k in ks:
        print(f"  {k:<4d} {res['tree_hit_rate_last_k_tree_rings'][k]:.3f}"
              f"{'':58s}{res['visit_hit_rate_last_k_links'][k]:.3f}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
