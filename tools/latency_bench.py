"""Latency of the single-request and per-message paths (run on the GPU box).

uncore_access (pu_access) and access_batch of one 100-request message
(pu_access_batch, prime.cpp's MEM_REQUESTS), on replica 0 of a C4 engine after a
warm-up, wall-clock per call; with the resident kernel (no launch per call) and
with one launch per call (pu_set_resident 0), each on its own slice of the stream.

    python tools/latency_bench.py [--calls 2000] [--out gpurun_out/latency.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=2000)
    ap.add_argument("--out", default="")
    ap.add_argument("--resident", choices=("0", "1", "both"), default="both",
                    help="resident mode (pu_set_resident) on, off, or both in turn (each on a fresh engine over the same slices)")
    a = ap.parse_args()
    import primesim_amd as P
    from primesim_amd import _abi as A
    from primesim_amd import config as CF
    cfg = P.config_from_dict(CF.preset("C4"))
    spec = P.StreamSpec(A.PU_STREAM_UNIFORM_HOTSPOT, 1024, seed=4, num_quanta=2, max_requests=200_000 + 200 * a.calls)
    reqs = P.generate_stream(spec)
    out = {}
    for mode in ((1, 0) if a.resident == "both" else (int(a.resident),)):
        # a fresh engine per mode, the same warm-up and the same stream slices:
        # the per-request work depends on the stream's phase (link histories)
        um = P.UncoreManager()
        um.init(cfg, replicas=1)
        for prog, th in P.stream_threads(spec):
            um.allocCore(prog, th)
        um.set_resident(mode)
        um.access_batch(reqs[:100_000])                # warm caches and link histories (one launch)
        i0 = um.resident_info()
        r = {"call_overhead_us": call_overhead(um, reqs, a.calls)}
        i1 = um.resident_info()
        if i1["commands"] > i0["commands"]:
            # where a resident call's time goes: kernel-side phases, the rest is the
            # mailbox round trip (host write -> kernel poll, kernel write -> host poll)
            nc = i1["commands"] - i0["commands"]
            nfast = i1["fast_answers"] - i0["fast_answers"]
            nfull = nc - nfast
            r["call_overhead_fast_answers"] = nfast
            r["call_overhead_breakdown_us"] = {k: (i1["sums_us"][k] - i0["sums_us"][k]) / (nc if k == "host_call" else
                                                                                          max(1, nfull))
                                               for k in i1["sums_us"]}
        t = time.perf_counter()
        for _ in range(a.calls):
            P.uncore.lib().pu_num_replicas(um._handle())
        r["python_ctypes_call_us"] = (time.perf_counter() - t) / a.calls * 1e6
        r.update(measure(um, reqs, a, 100_000))
        r["resident_info"] = um.resident_info()
        out["resident" if mode else "launch_per_call"] = r
        um.close()
    res = {"library_source_hash": P.uncore.library_source_hash(), "calls": a.calls,
           "lds_headers_env": os.environ.get("PRIMEUNCORE_LDS_HEADERS", ""), **out}
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


def call_overhead(um, reqs, calls: int) -> float:
    """µs per pu_access_status call whose request is an L1 hit (one core
    re-reading one line, timers advancing): the call's own cost, the
    simulation work nearly nil.  The ctypes call is prepared once."""
    import ctypes as C

    import primesim_amd as P
    q = reqs[100_000]
    core, prog, t0 = int(q["core"]), int(q["prog_id"]), int(q["timer"])
    addr = C.c_uint64(int(q["addr"]))
    d = C.c_int32(0)
    f, h = P.uncore.lib().pu_access_status, um._handle()
    for k in range(10):                                # the line into the L1
        addr.value = int(q["addr"])
        f(h, core, prog, 0, C.byref(addr), t0 + k, C.byref(d))
    t = time.perf_counter()
    for k in range(calls):
        addr.value = int(q["addr"])
        f(h, core, prog, 0, C.byref(addr), t0 + 10 + k, C.byref(d))
    return (time.perf_counter() - t) / calls * 1e6


def measure(um, reqs, a, i0: int) -> dict:
    import primesim_amd as P
    t0 = time.perf_counter()
    for q in reqs[i0:i0 + a.calls]:
        ins = P.InsMem(mem_type=int(q["mem_type"]), prog_id=int(q["prog_id"]), addr_dmem=int(q["addr"]))
        um.uncore_access(int(q["core"]), ins, int(q["timer"]))
    single = (time.perf_counter() - t0) / a.calls
    i1 = i0 + a.calls
    bs = np.flatnonzero(reqs["batch_start"][i1:]) + i1
    nmsg = min(max(1, a.calls // 10), len(bs) - 1)
    bounds = [(int(bs[k]), int(bs[k + 1])) for k in range(nmsg)]
    kms = 0.0
    t0 = time.perf_counter()
    for s, e in bounds:
        um.access_batch(reqs[s:e])
        kms += um.last_kernel_ms()
    per_msg = (time.perf_counter() - t0) / nmsg
    n = sum(e - s for s, e in bounds)
    res = {"uncore_access_us": single * 1e6, "message_us": per_msg * 1e6, "requests_per_message": n / nmsg,
           "message_us_per_request": per_msg * 1e6 / (n / nmsg),
           "kernel_us_per_message": kms * 1e3 / nmsg}
    # kernel time per request against the launch size (contiguous slices of the
    # same stream): separates per-launch costs from the per-request chain
    pos = bounds[-1][1]
    sweep = {}
    for size in (100, 1000, 10_000, 40_000):
        e = int(bs[np.searchsorted(bs, pos + size)])
        t0 = time.perf_counter()
        um.access_batch(reqs[pos:e])
        wall = time.perf_counter() - t0
        sweep[str(size)] = {"requests": e - pos, "kernel_us_per_request": um.last_kernel_ms() * 1e3 / (e - pos),
                            "wall_us_per_request": wall * 1e6 / (e - pos)}
        pos = e
    res["size_sweep"] = sweep
    return res


if __name__ == "__main__":
    main()
