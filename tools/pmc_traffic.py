"""Collect the engine kernel's HBM traffic from PMC counters (run on the GPU box).

Follows MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7: FETCH_SIZE and
WRITE_SIZE (KB, derived from the TCC EA request counters) are collected in
SEPARATE rocprofv3 passes (FETCH_SIZE needs 3 TCC slots, WRITE_SIZE 2), each
with nothing but the counter pass; plus one --kernel-trace --stats pass for
durations; plus passes for the read side in 32-B units (TCC_EA0_RDREQ_*_32B:
every read request counted by its size, no FETCH_SIZE per-size assumption),
the read request-size mix and the write side in 32-B units.  The reported
fabric bytes per launch = 32-B-unit reads + WRITE_SIZE; FETCH_SIZE is kept
beside it with their ratio (MI355X_MICROARCH.md: FETCH_SIZE reads 1/2 for
wide streaming reads, uncalibrated for other widths).

    python tools/pmc_traffic.py --out profiles/traffic.json -- --steps 20 --warmup 5 --no-cpu --no-extras

The summary carries the library's source hash (pu_version): bench.py reports
`roofline.traffic` only from a summary measured on the build it runs.

Writes the summary JSON, and copies the rocprofv3 summaries under profiles/.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the timed (time-sliced or replica-pool, headers in HBM) launches of bench.py:
# the compiled configuration's kernel (jit.cpp) or the ahead-of-time one
KERNELS = ("pu_jit_uncore_s1_h0", "pu_jit_uncore_s2_h0", "uncore_kernel<1, 1, false>", "uncore_kernel<1, 2, false>")


def run(cmd, log):
    print("+", " ".join(cmd), flush=True)
    with open(log, "w") as f:
        r = subprocess.run(cmd, cwd=ROOT, stdout=f, stderr=subprocess.STDOUT, timeout=300)
    if r.returncode != 0:
        raise SystemExit(f"{cmd[0]} failed ({r.returncode}); see {log}")


def counter_rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    with open(files[0]) as f:
        return list(csv.DictReader(f))


def per_dispatch(rows, counter):
    vals = {}
    for r in rows:
        if any(k in r.get("Kernel_Name", "") for k in KERNELS) and r.get("Counter_Name") == counter:
            did = int(r["Dispatch_Id"])
            vals[did] = vals.get(did, 0.0) + float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--work", default=os.path.join(ROOT, "gpurun_out", "pmc"))
    ap.add_argument("bench_args", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    bargs = [x for x in a.bench_args if x != "--"]
    os.makedirs(a.work, exist_ok=True)
    os.environ.setdefault("TMPDIR", "/tmp")
    py = sys.executable
    bench = [py, os.path.join(ROOT, "bench.py"), *bargs]
    passes = {}
    for name, extra in (("fetch", ["--pmc", "FETCH_SIZE"]), ("write", ["--pmc", "WRITE_SIZE"]),
                        ("trace", ["--kernel-trace", "--stats"]),
                        # the read side in 32-B units per destination (a 64-B request counts 2, 128-B 4):
                        # bytes without FETCH_SIZE's per-request-size assumptions
                        ("rd32", ["--pmc", "TCC_EA0_RDREQ_DRAM_32B_sum", "TCC_EA0_RDREQ_GMI_32B_sum",
                                  "TCC_EA0_RDREQ_IO_32B_sum"]),
                        # the request-size mix FETCH_SIZE is computed from
                        ("rdmix", ["--pmc", "TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_BUBBLE_sum",
                                   "TCC_EA0_RDREQ_128B_sum"]),
                        ("wr32", ["--pmc", "TCC_EA0_WRREQ_WRITE_DRAM_32B_sum", "TCC_EA0_WRREQ_ATOMIC_DRAM_32B_sum"])):
        d = os.path.join(a.work, name)
        shutil.rmtree(d, ignore_errors=True)
        run(["rocprofv3", *extra, "--output-format", "csv", "-d", d, "-o", "run", "--", *bench],
            os.path.join(a.work, f"{name}.log"))
        passes[name] = d
    with open(os.path.join(a.work, "trace.log")) as f:
        bench_line = json.loads([ln for ln in f if ln.startswith("{")][-1])
    fetch = per_dispatch(counter_rows(passes["fetch"]), "FETCH_SIZE")
    write = per_dispatch(counter_rows(passes["write"]), "WRITE_SIZE")
    steps, warm = bench_line["steps"], bench_line["warmup"]
    n = min(len(fetch), len(write))
    timed = list(range(n - steps, n))             # the timed launches are the last `steps`
    f_kb = sum(fetch[i] for i in timed) / steps
    w_kb = sum(write[i] for i in timed) / steps

    def timed_mean(pass_name, counter):
        v = per_dispatch(counter_rows(passes[pass_name]), counter)
        return sum(v[-steps:]) / steps if len(v) >= steps else float("nan")

    rd32 = {c: timed_mean("rd32", c) for c in ("TCC_EA0_RDREQ_DRAM_32B_sum", "TCC_EA0_RDREQ_GMI_32B_sum",
                                                "TCC_EA0_RDREQ_IO_32B_sum")}
    rdmix = {c: timed_mean("rdmix", c) for c in ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_BUBBLE_sum",
                                                  "TCC_EA0_RDREQ_128B_sum")}
    wr32 = {c: timed_mean("wr32", c) for c in ("TCC_EA0_WRREQ_WRITE_DRAM_32B_sum", "TCC_EA0_WRREQ_ATOMIC_DRAM_32B_sum")}
    read_b32 = 32.0 * sum(rd32.values())          # read bytes counted in 32-B units, every destination
    R = bench_line["config"]["replicas_per_gpu"]
    chunk = bench_line["config"]["mean_requests_per_replica_per_step"]
    accesses = R * chunk
    raw = (f_kb + w_kb) * 1024.0
    upper = (2.0 * f_kb + w_kb) * 1024.0
    calibrated = read_b32 + w_kb * 1024.0         # the one figure bench.py reports
    sys.path.insert(0, ROOT)
    from primesim_amd import uncore
    out = {
        "kernel": bench_line["roofline"]["kernel"],
        "src_hash": uncore.library_source_hash(),
        "launches_measured": steps,
        "warmup": warm,
        "replicas": R,
        "requests_per_replica_per_launch": chunk,
        "fetch_size_kb_per_launch": f_kb,
        "write_size_kb_per_launch": w_kb,
        "fetch_size_plus_write_size_bytes_per_launch": raw,
        "fetch_size_read_x2_bound_bytes_per_launch": upper,
        "read_bytes_per_launch_32b_units": read_b32,
        "read_32b_units_per_launch": rd32,
        "read_request_mix_per_launch": rdmix,
        "write_32b_units_per_launch": wr32,
        "fabric_bytes_per_launch": calibrated,
        "fabric_bytes_per_access": calibrated / accesses,
        "fabric_read_bytes_per_access": read_b32 / accesses,
        "fabric_read_bytes_per_access_fetch_size": f_kb * 1024.0 / accesses,
        "fabric_write_bytes_per_access": w_kb * 1024.0 / accesses,
        "atomic_dram_32b_units_per_access": wr32["TCC_EA0_WRREQ_ATOMIC_DRAM_32B_sum"] / accesses,
        "read_fetch_size_ratio": read_b32 / (f_kb * 1024.0) if f_kb else None,
        "alg_bytes_per_launch": bench_line["roofline"]["alg_bytes_per_launch"],
        "alg_bytes_per_access": bench_line["roofline"]["alg_bytes_per_launch"] / accesses,
        "avg_launch_ms_under_profiler": bench_line["roofline"]["avg_launch_ms"],
        "note": "Per timed launch (the last `steps` dispatches of the bench's own window), separate --pmc passes. "
                "These are the L2's memory-side (fabric) requests: Infinity-Cache hits are counted, so this is "
                "fabric traffic, an upper bound on HBM bytes. Reads: the TCC_EA0_RDREQ_{DRAM,GMI,IO}_32B counters "
                "tally every read in 32-B units whatever the request size (a 64-B request counts 2, a 128-B one "
                "4), so they need none of FETCH_SIZE's per-size assumptions (MI355X_MICROARCH.md notes FETCH_SIZE "
                "reading 1/2 for wide streaming reads); read_fetch_size_ratio compares the two. Writes: "
                "WRITE_SIZE (exact for this kernel's 16-B stores per the guide), cross-checked by "
                "TCC_EA0_WRREQ_WRITE_DRAM_32B. fabric_bytes_* = 32-B-unit reads + WRITE_SIZE",
        "bench_args": bargs,
    }
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    prefix = os.path.splitext(a.out)[0]
    for name in ("fetch", "write", "trace", "rd32", "rdmix", "wr32"):
        for src in glob.glob(os.path.join(passes[name], "**", "*stats.csv"), recursive=True):
            shutil.copy(src, f"{prefix}_{name}_{os.path.basename(src)}")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
