"""Quick GPU-vs-oracle check over the C1..C4 shapes (developer tool).

Runs each case through the HIP engine (access_batch, replica 0) and the CPU
restatement; prints the first mismatch if any.  Usage: python tools/gpu_check.py [max_requests]
"""
from __future__ import annotations

import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import primesim_amd as P  # noqa: E402
from primesim_amd import _abi as A  # noqa: E402
from primesim_amd import config as CF  # noqa: E402
import oracle as O  # noqa: E402


def case(name, sim, spec):
    cfg = P.config_from_dict(sim)
    reqs = P.generate_stream(spec)
    um = P.UncoreManager()
    um.init(cfg, replicas=1)
    ref = O.CpuRef(cfg)
    for prog, th in P.stream_threads(spec):
        um.allocCore(prog, th)
        ref.alloc_core(prog, th)
    t0 = time.time()
    got = um.access_batch(reqs)
    t1 = time.time()
    want, _ = ref.run(reqs)
    t2 = time.time()
    ok = np.array_equal(got, want)
    gs, ws = um.stats().as_dict(), ref.stats().as_dict()
    bad = {k: (gs[k], ws[k]) for k in ws if gs.get(k) != ws[k] and k != "requests"}
    print(f"{name}: n={len(reqs)} delays_equal={ok} stats_mismatch={bad} "
          f"gpu {len(reqs) / (t1 - t0):.0f}/s (kernel {um.last_kernel_ms():.1f} ms) cpu {len(reqs) / (t2 - t1):.0f}/s",
          flush=True)
    if not ok:
        i = int(np.nonzero(got != want)[0][0])
        print("  first mismatch", i, got[i], want[i], reqs[i], flush=True)
    um.close()
    return ok and not bad


def main():
    cap = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
    allok = True
    allok &= case("C1", CF.preset("C1"), P.StreamSpec(A.PU_STREAM_PRIVATE_STREAMING, 16, 1, num_quanta=3,
                                                      max_requests=cap))
    allok &= case("C1hot", CF.preset("C1"), P.StreamSpec(A.PU_STREAM_UNIFORM_HOTSPOT, 16, 11, num_quanta=3,
                                                         max_requests=cap))
    allok &= case("C2", CF.preset("C2"), P.StreamSpec(A.PU_STREAM_SHARED_UNIFORM, 64, 2, num_quanta=2,
                                                      max_requests=cap))
    allok &= case("C3", CF.preset("C3"), P.StreamSpec(A.PU_STREAM_MULTIPROGRAM, 256, 3, num_progs=4,
                                                      max_requests=cap))
    allok &= case("C4", CF.preset("C4"), P.StreamSpec(A.PU_STREAM_UNIFORM_HOTSPOT, 1024, 4, max_requests=cap))
    print("ALL OK" if allok else "MISMATCH")
    sys.exit(0 if allok else 1)


if __name__ == "__main__":
    main()
