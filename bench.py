"""Benchmark: simulated memory accesses/s through the uncore at 1024 cores.

Workload (BASELINE.json configs[3]): 1024-core 32x32 mesh,
private L1 32 KB/8 W + one 256 KB/8 W shared-LLC slice per tile, directory
MESI (full map), XY links with the Graphite history-tree/M/G/1 model,
DRAM 120 cycles; synthetic stream: 80% uniform over 2^20 lines + 20% over a
64-line hotspot, 25% writes, 1-4-cycle gaps, 1000-cycle barriers,
100-request messages, canonical order.

Every replica on this GPU first runs the first quantum of its own request
stream untimed, in --warmup fixed steps of --chunk (40,960) requests (a C4
quantum is ~409,600 requests: 1024 cores x ~400 requests per 1000-cycle
quantum, so every core is active; cold caches and empty link histories).  The
requests of the next --steps x --chunk are then made resident in HBM and each
timed "step" is one engine launch (the hot path: prime.cpp's message loop over
System::access) in which every replica continues its own stream for a
--slice-ms wall-time slice, stopping only between requests
(pu_run_device_sliced).  Replicas differ several-fold in cost per request (link
histories, tree-vs-M/G/1 mix), so a fixed number of requests per replica per
launch would leave most waves idle behind the slowest (measured 26% busy); the
slice keeps every wave simulating.  A replica is one complete, independent
1024-core uncore (its own seed); the engine runs one replica per wavefront and
many replicas per GPU, because a single uncore is a strictly sequential fold
(DESIGN.md).  `value` = all requests processed by all ranks / max-over-ranks
wall time of the K timed steps.  --slice-ms 0 gives fixed --chunk steps.

Rank 0 also times the reference's own CPU uncore (oracle/_ref, compiled from
/root/reference in the build container) — or, if that library is absent, the
CPU restatement — on replica 0's stream on one host core: an untimed fill over
the warmup requests, then timed over the GPU's timed window; it checks that the
GPU's delays for every request it ran are bit-identical.

Launch: python bench.py [--gpus N --steps K --warmup W]; N>1 under
torch.distributed.run (one process per GPU).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

LAST_REPLICAS = 0       # replicas of the last main() run (tools/prof_regions.py)
LAST_PER_REPLICA = None  # per-replica stat deltas of the timed steps (profiling runs only)
METRIC = "simulated memory accesses/sec (uncore) at 1024 cores; % HBM roofline"
REQ_BYTES = 32          # sizeof(pu_req)
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def alg_bytes(st: dict, cfg) -> float:
    """SURVEY.md §8d algorithmic bytes for the counted events."""
    y = cfg.sys
    b = 28.0 * st["requests"]
    for lvl in range(y.num_levels):
        b += st[f"L{lvl}_ins"] * (16.0 * y.cache[lvl].num_ways + 16.0)
    n_llc = math.ceil(y.num_cores / y.cache[y.num_levels - 1].share)
    b += st["directory_ins"] * (16.0 * y.directory_cache.num_ways + 16.0 + 16.0 * math.ceil(n_llc / 64))
    b += st["net_distance"] * 96.0
    b += st["dram_accesses"] * 8.0
    return b


def sum_stats(um, replicas: int) -> dict:
    tot: dict = {}
    for r in range(replicas):
        d = um.stats(r).as_dict()
        for k, v in d.items():
            if k == "error_flags":
                tot[k] = tot.get(k, 0) | v
            elif k != "num_levels":
                tot[k] = tot.get(k, 0) + v
    return tot


def cpu_baseline(cfg_xml: str, cfg, reqs: np.ndarray, threads, fill: int, budget_s: float):
    """Time the reference CPU uncore (or the restatement) on reqs[fill:], after
    an untimed run over reqs[:fill]; returns every delay it produced."""
    import oracle as O
    kind = "reference" if O.ref_available() else "port"
    eng = O.RefUncore(cfg_xml) if kind == "reference" else O.CpuRef(cfg)
    for prog, th in threads:
        eng.alloc_core(prog, th)
    chunk = 8192
    delays = []
    for a in range(0, fill, chunk):
        d, rc = eng.run(reqs[a:min(fill, a + chunk)])
        delays.append(d)
    done = fill
    t0 = time.perf_counter()
    while done < len(reqs) and time.perf_counter() - t0 < budget_s:
        d, rc = eng.run(reqs[done:done + chunk])
        delays.append(d)
        done += len(d)
    el = time.perf_counter() - t0
    return kind, done - fill, el, np.concatenate(delays) if delays else np.zeros(0, np.int32)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10, help="timed steps (default: the stream's second quantum)")
    ap.add_argument("--warmup", type=int, default=10, help="untimed steps (default: the first quantum)")
    ap.add_argument("--replicas", type=int, default=0, help="replicas per GPU (0 = size to HBM)")
    ap.add_argument("--chunk", type=int, default=40960, help="requests per replica per step")
    ap.add_argument("--slice-ms", type=float, default=400.0,
                    help="timed steps are wall-time slices: every replica continues its own stream for this long "
                         "per launch (stopping only between requests); 0 = fixed --chunk requests per replica per step")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL) normally; gloo for CPU-side rehearsal")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC traffic summary written by tools/pmc_traffic.py for this kernel")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import primesim_amd as P
    from primesim_amd import _abi as A
    from primesim_amd import config as CF
    from primesim_amd.dist import reduce_run, replica_seed

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group(args.dist_backend, init_method="env://")
    # PU_BENCH_DEVICE pins every rank to one card (rehearsing N>1 on a 1-GPU box)
    local = int(os.environ.get("PU_BENCH_DEVICE", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    sim = CF.preset("C4")
    xml_path = os.path.join(tempfile.gettempdir(), f"pu_bench_c4_{os.getpid()}.xml")
    CF.write_xml(sim, xml_path)
    cfg = P.load_config(xml_path)

    # ---- per-replica HBM: engine state + the timed request slabs + one warmup chunk
    um = P.UncoreManager()
    probe = P.UncoreManager()
    probe.init(cfg, replicas=1, device=local)
    rbytes = probe.replica_bytes
    resident = probe.resident_replicas
    probe.close()
    per_bytes = rbytes + (args.steps + 1) * args.chunk * (REQ_BYTES + 4)
    free, total = torch.cuda.mem_get_info(dev)
    # as many replicas as fit in HBM, but no more than the kernel keeps resident
    # (one wave each): a time-sliced launch over more would run in two rounds
    R = args.replicas or max(1, min(resident, int((free * 0.88) // per_bytes)))
    R = max(1, R - R % 8) if R >= 8 else R
    log(f"[bench] rank {rank}: replica {rbytes / 2**20:.0f} MiB + requests {(per_bytes - rbytes) / 2**20:.0f} MiB, "
        f"{R} replicas (resident limit {resident}), free {free / 2**30:.0f} GiB")
    global LAST_REPLICAS
    LAST_REPLICAS = R
    um.init(cfg, replicas=R, device=local)
    threads = P.stream_threads(P.StreamSpec(A.PU_STREAM_UNIFORM_HOTSPOT, 1024))
    for prog, th in threads:
        um.allocCore(prog, th)

    # ---- request streams: one seed per replica (disjoint across ranks), produced
    # chunk by chunk in canonical order by the resumable host generator
    specs = [P.StreamSpec(A.PU_STREAM_UNIFORM_HOTSPOT, 1024, seed=replica_seed(4, rank, r), num_quanta=64)
             for r in range(R)]
    gen = P.StreamSet(specs)
    host = np.zeros((R, args.chunk), dtype=A.REQ_DTYPE)
    offs = torch.from_numpy((np.arange(R + 1, dtype=np.uint64) * np.uint64(args.chunk)).view(np.int64)).to(dev)
    # a dedicated (non-null) stream: the engine launches on it and the HIP
    # events below time exactly those launches
    stream = torch.cuda.Stream(dev)
    sptr = stream.cuda_stream
    assert sptr != 0
    rep0 = []                                       # replica 0's delays, for the parity check

    def next_chunk() -> torch.Tensor:
        got = gen.next_into(host)
        assert got == args.chunk, (got, args.chunk)
        return torch.from_numpy(host.view(np.uint8).reshape(-1)).to(dev)

    # warmup: the first quantum of every replica's stream (all 1024 cores, cold
    # caches, empty link histories); untimed, requests uploaded step by step
    d_warm_delay = torch.zeros(R * args.chunk, dtype=torch.int32, device=dev)
    t_w = time.time()
    for s in range(args.warmup):
        d_req = next_chunk()
        um.run_device(d_req.data_ptr(), offs.data_ptr(), d_warm_delay.data_ptr(), sptr)
        torch.cuda.synchronize(dev)
        rep0.append(d_warm_delay[:args.chunk].cpu().numpy())
        del d_req
        log(f"[bench] warmup step {s} done ({time.time() - t_w:.1f}s)")
    if os.environ.get("PU_PROF_RESET_AFTER_WARMUP"):   # tools/prof_regions.py: count the timed steps only
        P.uncore.lib().pu_engine_prof_read(None, 0, 1)
    # timed window: the next steps x chunk requests of every replica, generated
    # and made resident in HBM first, replica-major ([R][steps*chunk])
    t_gen = time.time()
    W_t = args.steps * args.chunk
    d_win = torch.empty((R, W_t, REQ_BYTES), dtype=torch.uint8, device=dev)
    for k in range(args.steps):
        d_win[:, k * args.chunk:(k + 1) * args.chunk, :] = next_chunk().view(R, args.chunk, REQ_BYTES)
    d_win_delay = torch.zeros(R * W_t, dtype=torch.int32, device=dev)
    win_off = np.arange(R + 1, dtype=np.uint64) * np.uint64(W_t)
    d_win_off = torch.from_numpy(win_off.view(np.int64)).to(dev)
    d_pos = torch.from_numpy(win_off[:-1].copy().view(np.int64)).to(dev)
    # fixed-size steps (--slice-ms 0): launch k covers [k*chunk, (k+1)*chunk) of every replica
    step_offs = [torch.from_numpy(np.concatenate([[0], win_off[:-1] + np.uint64((k + 1) * args.chunk)])
                                  .astype(np.uint64).view(np.int64)).to(dev) for k in range(args.steps)]
    torch.cuda.synchronize(dev)
    log(f"[bench] timed requests resident: {R} x {W_t} in {time.time() - t_gen:.1f}s")
    before = sum_stats(um, R)
    prof_keys = ("requests", "net_accesses", "net_distance", "mg1_calls", "lockdown_calls", "dram_accesses",
                 "total_num_broadcast", "L0_miss", "directory_ins", "directory_miss", "net_total_delay")
    per_before = None
    if os.environ.get("PU_PROF_RESET_AFTER_WARMUP"):
        per_before = [um.stats(r).as_dict() for r in range(R)]

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        if args.slice_ms > 0:
            ev[k][0].record(stream)
            um.run_device_sliced(d_win.data_ptr(), d_win_off.data_ptr(), d_win_delay.data_ptr(), d_pos.data_ptr(),
                                 int(args.slice_ms * 1000), sptr)
            ev[k][1].record(stream)
        else:
            ev[k][0].record(stream)
            um.run_device_sliced(d_win.data_ptr(), step_offs[k].data_ptr(), d_win_delay.data_ptr(), d_pos.data_ptr(),
                                 0, sptr)
            ev[k][1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = [a.elapsed_time(b) for a, b in ev]
    log(f"[bench] timed {args.steps} steps in {elapsed:.3f}s; per-launch ms {['%.1f' % x for x in kern_ms]}")
    pos = d_pos.cpu().numpy().view(np.uint64)
    adv = (pos - win_off[:-1]).astype(np.int64)
    log(f"[bench] requests per replica in the timed window: min {adv.min()} median {int(np.median(adv))} "
        f"max {adv.max()} of {W_t}; {int((adv >= W_t).sum())} at the end (halted replicas skip to it)")
    rep0.append(d_win_delay[:int(adv[0])].cpu().numpy())
    gen.close()

    after = sum_stats(um, R)
    if per_before is not None:
        global LAST_PER_REPLICA
        per_after = [um.stats(r).as_dict() for r in range(R)]
        LAST_PER_REPLICA = {k: [int(per_after[r][k] - per_before[r][k]) for r in range(R)] for k in prof_keys}
    delta = {k: after[k] - before.get(k, 0) for k in after if k != "error_flags"}
    errf = after.get("error_flags", 0)
    # requests that actually reached the uncore: a replica whose message delay
    # went negative stops there, like the reference's handler (prime.cpp:130-134)
    processed = int(delta["requests"])
    halted = sum(1 for r in range(R) if um.stats(r).error_flags & A.PU_ERRF_NEG_DELAY)
    t_max, tot_processed = reduce_run(elapsed, processed, dev if args.dist_backend == "nccl" else None)
    value = tot_processed / t_max

    # ---- roofline of the engine kernel (per launch, this rank)
    avg_ms = float(np.mean(kern_ms))
    bytes_per_launch = alg_bytes(delta, cfg) / args.steps
    achieved = bytes_per_launch / (avg_ms / 1e3) / 1e9

    # HBM traffic from the PMC counters (FETCH_SIZE + WRITE_SIZE, separate rocprofv3
    # passes of this same command, tools/pmc_traffic.py): bytes per access x this
    # launch's accesses
    traffic, traffic_src = None, None
    if os.path.exists(args.traffic_json):
        with open(args.traffic_json) as f:
            tj = json.load(f)
        traffic = tj["hbm_bytes_per_access"] * (processed / args.steps)
        traffic_src = (f"{os.path.relpath(args.traffic_json, ROOT)}: {tj['hbm_bytes_per_access']:.0f} B/access "
                       f"measured at {tj['replicas']} replicas x {tj['requests_per_replica_per_launch']} requests")

    result = None
    if rank == 0:
        cpu = None
        if not args.no_cpu:
            # replica 0's stream: the reference fills the warmup quantum untimed,
            # then is timed on the requests of the GPU's timed window (as many as
            # fit in --cpu-seconds); parity is checked on every request both ran
            w0, n_t = args.warmup * args.chunk, args.steps * args.chunk
            s0 = P.generate_stream(P.StreamSpec(A.PU_STREAM_UNIFORM_HOTSPOT, 1024, seed=replica_seed(4, rank, 0),
                                                num_quanta=64, max_requests=w0 + n_t))
            kind, n_cpu, el, d_cpu = cpu_baseline(xml_path, cfg, s0, threads, w0, args.cpu_seconds)
            gpu_d = np.concatenate(rep0)
            m = min(len(d_cpu), len(gpu_d))
            parity = bool(np.array_equal(gpu_d[:m], d_cpu[:m]))
            cpu = {"value": n_cpu / el, "unit": "accesses/s", "cores": 1, "kind": kind,
                   "sample": f"replica 0's C4 stream: requests {w0}..{w0 + n_cpu} (the GPU's timed window; the GPU "
                             f"ran {int(adv[0])} of them for replica 0), after an untimed fill of the {w0}-request "
                             f"warmup, single-threaded "
                             f"({'reference uncore compiled from /root/reference/src' if kind == 'reference' else 'oracle/cpu_ref restatement'}), "
                             f"{el:.1f} s; GPU delays bit-identical on all {m} requests compared: {parity}"}
            log(f"[bench] cpu baseline ({kind}): {n_cpu / el:.0f} accesses/s; parity on {m} delays: {parity}")
        result = {
            "metric": METRIC,
            "value": value,
            "unit": "accesses/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": t_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic",
            "config": {
                "workload": "C4: 1024-core 32x32 mesh, L1 32KB/8W + 256KB/8W shared-LLC slice per tile, "
                            "directory MESI full-map, uniform 2^20 lines + 64-line hotspot, 25% writes",
                "replicas_per_gpu": R,
                "step": (f"wall-time slice: every replica continues its own stream for {args.slice_ms:g} ms per "
                         f"launch, stopping only between requests" if args.slice_ms > 0 else
                         f"fixed: {args.chunk} requests per replica per launch"),
                "mean_requests_per_replica_per_step": processed / (R * args.steps),
                "warmup_requests_per_replica": args.warmup * args.chunk,
                "parallelism": f"replicas: {R} independent uncores per GPU x {world} GPU(s)",
                "per_replica_accesses_per_s": value / (R * world),
                "halted_replicas": halted,
                "error_flags": errf & ~A.PU_ERRF_NEG_DELAY,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel": "uncore_kernel<1, true>" if args.slice_ms > 0 else "uncore_kernel<1, true> (no budget)",
                "avg_launch_ms": avg_ms,
                "alg_bytes_per_launch": bytes_per_launch,
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(result), flush=True)
    um.close()
    try:
        os.remove(xml_path)
    except OSError:
        pass
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
