"""Benchmark: simulated memory accesses/s through the uncore at 1024 cores.

Workload (BASELINE.json configs[3]): 1024-core 32x32 mesh,
private L1 32 KB/8 W + one 256 KB/8 W shared-LLC slice per tile, directory
MESI (full map), XY links with the Graphite history-tree/M/G/1 model,
DRAM 120 cycles; synthetic stream: 80% uniform over 2^20 lines + 20% over a
64-line hotspot, 25% writes, 1-4-cycle gaps, 1000-cycle barriers,
100-request messages, canonical order.

Headline (`value`): every replica on this GPU first runs --warmup fixed steps
of --chunk (40,960) requests of its own stream untimed (a C4 quantum is
~409,600 requests: 1024 cores x ~400 requests per 1000-cycle quantum, so every
core is active; cold caches and empty link histories are warmed).  The next
--steps x --chunk requests are then made resident in HBM and each timed "step"
is one engine launch (prime.cpp's message loop over System::access) in which
every wavefront continues its replica's stream for a --slice-ms wall-time
slice, stopping only between requests: replicas differ several-fold in cost
per request, and the slice keeps every wave simulating.  A replica is one
complete, independent 1024-core uncore (its own seed), simulated by one
wavefront at a time.  The GPU holds one wavefront per resident slot and
--spare-replicas more replicas (all warmed alike): a wavefront whose replica
stops by prime.cpp's rule (open-loop overload) or finishes its window takes
the next unstarted replica within the slice (the replica pool,
pu_run_device_pool), so no slot idles.  `value` = all requests processed by
all ranks / max-over-ranks wall time of the K timed steps.  Replay is open
loop (recorded timers).

At N=1 (rank 0) the same line also carries:
  * per_simulation_accesses_per_s — value / wavefronts: the rate of ONE of the
    concurrent simulations;
  * replica_parity — the delays of 16 replicas spread over 0..R-1 (warmup and
    timed window) against the reference's, replayed by the ensemble processes;
  * single_instance — ONE simulation alone on the GPU (a 1-replica engine on
    replica 0's stream, same warmup, then --single-requests in one launch);
  * closed_loop — the same workload replayed closed-loop (timer_i += the core's
    earlier batch delays, core_manager.cpp:265): rate, halted replicas, M/G/1
    share, parity vs the reference in closed mode;
  * cpu_baseline — the reference's own uncore (oracle/_ref) on ONE host core
    on replica 0's stream (untimed fill over the warmup, then the GPU's timed
    window), with bit-exact parity of every delay both ran;
  * cpu_baseline_ensemble — the reference on ALL host cores of this box's
    share, one replica per process (forked before any GPU call), each on its
    replica's stream after the same fill: the ensemble comparison.
  * roofline.traffic — fabric bytes (FETCH_SIZE + WRITE_SIZE, separate PMC
    passes; includes Infinity-Cache hits) measured by tools/pmc_traffic.py for
    THIS library build only (refused when its source hash differs).
At N>1 every rank forks --rank-parity-workers reference processes before it
touches its GPU; they replay that rank's replica 0 and its first replica-pool
spare, each rank checks their delays against its own, and rank 0's line
carries `rank_parity` (per rank and overall) and `roofline.job` (algorithmic
bytes summed over ranks / the slowest rank's mean launch / (N x 8 TB/s)).
The run exits non-zero when a parity check fails on any rank.

Launch: python bench.py [--gpus N --steps K --warmup W]; N>1 under
torch.distributed.run (one process per GPU).
"""
from __future__ import annotations

import argparse
import json
import math
import multiprocessing as mp
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

LAUNCH_CMD = None       # rank command for launch_ranks (None: this file; tests point it at a stub)
LAST_REPLICAS = 0       # replicas of the last main() run (tools/prof_regions.py)
LAST_PER_REPLICA = None  # per-replica stat deltas of the timed steps (profiling runs only)
METRIC = "simulated memory accesses/sec (uncore) at 1024 cores; % HBM roofline"
# --config: the SURVEY.md §8d shape and its seeded stream.  C4 is the metric's
# configuration (BASELINE.json configs[3]); C3 and C5 are the deeper and the
# larger shapes, measured the same way (their lines name their own metric).
WORKLOADS = {
    # (C3's replicas run ~2x faster than C4's: 1.5x the chunk, so the timed
    # window outlasts the 20 slices for most replicas and HBM still holds ~10%
    # spare replicas for the pool; at 2x only 8 spares fit: busy 0.93)
    "C3": {"cores": 256, "stream": "PU_STREAM_MULTIPROGRAM", "num_progs": 4, "replay": "open", "chunk": 61440,
           "desc": "C3: 256-core 16x16 mesh, private L1 32KB/8W + private L2 256KB/8W/5cyc + 1MB/16W shared-LLC "
                   "slice per tile, directory MESI full-map; multi-programmed mix, 4 programs x 64 cores, "
                   "per-program footprints 4-64 MB, 20% writes"},
    "C4": {"cores": 1024, "stream": "PU_STREAM_UNIFORM_HOTSPOT", "num_progs": 1, "replay": "open", "chunk": 40960,
           "desc": "C4: 1024-core 32x32 mesh, L1 32KB/8W + 256KB/8W shared-LLC slice per tile, "
                   "directory MESI full-map, uniform 2^20 lines + 64-line hotspot, 25% writes"},
    # open loop, the producer/consumer stream's link delays pass 2^31 within
    # its first quantum (golden big_c5_preset stops at request 165,860 by
    # prime.cpp:130-134): every replica would halt in the warm-up, so C5 is
    # replayed closed loop (core_manager.cpp:265) by default
    "C5": {"cores": 4096, "stream": "PU_STREAM_PRODUCER_CONSUMER", "num_progs": 1, "replay": "closed", "chunk": 40960,
           "desc": "C5: 4096-core 64x64 mesh, L1 32KB/8W + 256KB/8W shared-LLC slice per tile, directory MESI "
                   "full-map; producer/consumer pairs (p, p+2048) sharing 1,024-line buffers, 50% writes"},
}
WORKLOAD = "C4"         # set by main() before the ensemble forks (its workers read it)
LIMITER = ("dependent-load latency and instruction issue (profiles/r6y_sq.json: 25.3% of wave cycles issuing, "
           "39.6% waiting on memory, 35.1% in issue stalls at 7 waves/SIMD, 1,210 VALU + 1,339 SALU per access; "
           "fabric traffic about 43% of 8 TB/s), not HBM bandwidth")
REQ_BYTES = 32          # sizeof(pu_req)
VARIANTS = {0: "ahead-of-time kernels (runtime geometry) for every launch",
            1: "ahead-of-time kernels for the replicas (throughput launches); the configuration compiled into "
               "the kernel (jit.cpp) for one simulation alone (latency launches)",
            2: "configuration compiled into the kernel (jit.cpp) for every launch"}
COMPILERS = {1: "hipRTC at run time", 2: "hipcc at build time",
             3: "throughput and latency code objects from different compilers (hipcc / hipRTC)"}
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
SEED_BASE = 4
STAGE_GROUP = 256       # replicas whose requests the host generates per staging copy
BUSY_MIN = 0.95         # a replica pool busier than this kept every slot resident for the whole slice


def timed_req_bytes(args) -> int:
    """Bytes per request record of the timed window (pu_req16 or pu_req)."""
    return 16 if getattr(args, "req_format", 32) == 16 else REQ_BYTES


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


def busy_guard(pool) -> str | None:
    """Why a replica-pool pass cannot be reported, or None.  While unstarted
    replicas remain, every slot's wavefront is resident for the whole slice
    (busy ~1); a busy fraction under BUSY_MIN means part of the grid was not
    resident and waited for the first waves' slice to end: the launch took
    two slices (round 4's six-wave kernel: exactly half the rate)."""
    if not pool or pool["replicas_started"] >= pool["replicas"]:
        return None          # the pool ran dry: idle slots are expected
    if pool["busy_fraction"] < BUSY_MIN:
        return (f"replica pool busy fraction {pool['busy_fraction']:.3f} < {BUSY_MIN} with "
                f"{pool['replicas'] - pool['replicas_started']} replicas never started: the grid of "
                f"{pool['wavefronts']} wavefronts was not all resident (pu_resident_replicas overstated)")
    return None


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


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_core_share() -> int:
    """Host cores this job may use: the box exports its CPU share in
    OMP_NUM_THREADS (os.cpu_count() shows the whole machine there)."""
    n = os.cpu_count() or 1
    e = os.environ.get("OMP_NUM_THREADS")
    if e and e.isdigit() and int(e) > 0:
        n = min(n, int(e))
    return n


def stream_spec(seed: int, n: int = 0):
    import primesim_amd as P
    from primesim_amd import _abi as A
    w = WORKLOADS[WORKLOAD]
    return P.StreamSpec(getattr(A, w["stream"]), w["cores"], seed=seed, num_quanta=64, num_progs=w["num_progs"],
                        max_requests=n)


def reference_engine(cfg_xml: str, cfg, mode: int = 0):
    """The timed CPU baseline: the reference uncore compiled in place without
    the golden generator's counting wraps (oracle/_ref/libprime_ref_nowrap.so;
    a wrap adds a call per link visit), else the restatement."""
    import oracle as O
    kind = "reference" if O.ref_available(plain=True) else "port"
    eng = O.RefUncore(cfg_xml, plain=True) if kind == "reference" else O.CpuRef(cfg)
    eng.set_mode(mode)
    return kind, eng


def ref_mode(args) -> int:
    """The reference's replay mode for the headline's (oracle MODE_*)."""
    import oracle as O
    return O.MODE_CLOSED if args.replay == "closed" else 0


def simulated(n: int, rc: int) -> int:
    """Requests of one reference run() call that were actually simulated: all
    of them (rc 0), the first rc (the prime.cpp:130-134 stop after request
    rc-1), or none (rc -1: already stopped)."""
    return n if rc == 0 else max(rc, 0)


def cpu_baseline(cfg_xml: str, cfg, reqs: np.ndarray, threads, fill: int, budget_s: float, mode: int = 0):
    """Time the reference CPU uncore (or the restatement) on reqs[fill:], after
    an untimed run over reqs[:fill]; returns every delay it produced."""
    kind, eng = reference_engine(cfg_xml, cfg, mode)
    for prog, th in threads:
        eng.alloc_core(prog, th)
    chunk = 8192
    delays = []
    for a in range(0, fill, chunk):
        d, rc = eng.run(reqs[a:min(fill, a + chunk)])
        delays.append(d)
    done, sim = fill, 0
    t0 = time.perf_counter()
    while done < len(reqs) and time.perf_counter() - t0 < budget_s:
        d, rc = eng.run(reqs[done:done + chunk])
        delays.append(d)
        done += len(d)
        sim += simulated(len(d), rc)
        if rc != 0:                                   # prime.cpp:130-134 stop: nothing more is simulated
            break
    el = time.perf_counter() - t0
    return kind, sim, el, np.concatenate(delays) if delays else np.zeros(0, np.int32)


# ---------------------------------------------------------------- CPU ensemble
def _ensemble_worker(conn, cfg_xml: str, fill: int, n_timed: int, budget_s: float, rank: int = 0,
                     mode: int = 0) -> None:
    """One replica of the ensemble: wait for its replica index (the parent
    knows the replica count only once it has the GPU), fill untimed, wait for
    "go", run for budget_s; send back every delay it produced (parity)."""
    try:
        msg = conn.recv()
        if msg[0] != "replica":
            return
        rep = int(msg[1])
        import primesim_amd as P
        from primesim_amd.dist import replica_seed
        cfg = P.load_config(cfg_xml)
        reqs = P.generate_stream(stream_spec(replica_seed(SEED_BASE, rank, rep), fill + n_timed))
        threads = P.stream_threads(stream_spec(SEED_BASE))
        kind, eng = reference_engine(cfg_xml, cfg, mode)
        for prog, th in threads:
            eng.alloc_core(prog, th)
        delays = []
        for a in range(0, fill, 16384):
            d, _ = eng.run(reqs[a:min(fill, a + 16384)])
            delays.append(d)
        conn.send(("ready", kind))
        conn.recv()                                   # go
        done, sim, t0 = fill, 0, time.perf_counter()
        while done < len(reqs) and time.perf_counter() - t0 < budget_s:
            d, rc = eng.run(reqs[done:done + 2048])
            delays.append(d)
            done += len(d)
            sim += simulated(len(d), rc)
            if rc != 0:                               # halted: the rest would only be skipped
                break
        el = time.perf_counter() - t0
        conn.send(("done", sim, el, rep, np.concatenate(delays).astype(np.int32).tobytes()))
    except Exception as e:  # noqa: BLE001 — reported to the parent
        conn.send(("error", repr(e)))
    finally:
        conn.close()


def parity_replicas(R: int, workers: int, slots: int = 0) -> list:
    """Replicas the ensemble replays: spread over the slot range 0..S-1 (the
    last one S-1), S = slots when the replica pool runs (slots < R), else R.
    With the pool, a quarter of the workers (at least one) take the first
    spare replicas S, S+1, ...: the pool hands out spares in index order as
    slot replicas halt, so those are the spares that start (mid-slice, on a
    wavefront that finished another replica) — R-1 usually never does."""
    if workers <= 1 or R <= 1:
        return [0][:workers]
    S = slots if 0 < slots < R else R
    k_sp = min(max(1, workers // 4), R - S) if S < R else 0
    spread = max(1, workers - k_sp)
    if spread == 1:
        reps = [0]
    else:
        step = max(1, S // spread)
        reps = [min(w * step, S - 1) for w in range(spread - 1)] + [S - 1]
    return sorted(set(reps) | set(range(S, S + k_sp)))


class Ensemble:
    """The reference uncore on every host core of this job's share, one replica
    per process, forked before the parent touches the GPU.  Each process is
    told its replica once the parent knows the replica count (assign), fills
    while the GPU warms up, and returns its delays: the parity check of those
    replicas against the GPU's."""

    def __init__(self, cfg_xml: str, workers: int, fill: int, n_timed: int, budget_s: float, rank: int = 0,
                 mode: int = 0):
        ctx = mp.get_context("fork")
        self.workers, self.budget, self.rank = workers, budget_s, rank
        self.fill = fill
        self.pipes, self.procs = [], []
        self.replicas: list = []
        for w in range(workers):
            a, b = ctx.Pipe()
            p = ctx.Process(target=_ensemble_worker, args=(b, cfg_xml, fill, n_timed, budget_s, rank, mode),
                            daemon=True)
            p.start()
            self.pipes.append(a)
            self.procs.append(p)

    def assign(self, R: int, slots: int = 0) -> list:
        self.replicas = parity_replicas(R, self.workers, slots)
        for k, c in enumerate(self.pipes):
            c.send(("replica", self.replicas[k]) if k < len(self.replicas) else ("stop",))
        self.pipes, dropped = self.pipes[:len(self.replicas)], self.pipes[len(self.replicas):]
        for c in dropped:
            c.close()
        return self.replicas

    def run(self) -> dict:
        kinds = set()
        for c in self.pipes:
            msg = c.recv()
            if msg[0] == "error":
                raise RuntimeError(f"ensemble worker: {msg[1]}")
            kinds.add(msg[1])
        t0 = time.perf_counter()
        for c in self.pipes:
            c.send("go")
        res = [c.recv() for c in self.pipes]
        wall = time.perf_counter() - t0
        for p in self.procs:
            p.join(30)
        bad = [r for r in res if r[0] != "done"]
        if bad:
            raise RuntimeError(f"ensemble worker: {bad[0]}")
        n = sum(r[1] for r in res)
        el = max(r[2] for r in res)
        kind = kinds.pop() if len(kinds) == 1 else "mixed"
        self.delays = {r[3]: np.frombuffer(r[4], dtype=np.int32) for r in res}
        nw = len(self.pipes)
        return {"value": n / el, "unit": "accesses/s", "cores": nw, "kind": kind,
                "cpu_model": cpu_model(),
                "sample": f"{nw} processes, one per host core of this job's share, each the "
                          f"{'reference uncore compiled from /root/reference/src, no counting wraps' if kind == 'reference' else kind} "
                          f"on one GPU replica's {WORKLOAD} stream (replicas {self.replicas[0]}..{self.replicas[-1]}, spread "
                          f"over the GPU's replicas) after an untimed {self.fill}-request fill, run concurrently for "
                          f"{self.budget:g} s: {n} requests in {el:.2f} s (wall {wall:.2f} s)",
                "per_process_accesses_per_s": [r[1] / r[2] for r in res]}


def replica_parity(ens: Ensemble, H, slots: int, kind: str, warm_reqs: int) -> dict:
    """The GPU delays of the ensemble's replicas (warmup, then timed window)
    against the reference's on the same streams, over the requests both ran."""
    per = {}
    for r, d_cpu in ens.delays.items():
        g = H.kept[r]
        m = min(len(g), len(d_cpu))
        per[str(r)] = {"requests_compared": m, "gpu_window_requests": int(H.adv[r]),
                       "spare": bool(r >= slots),
                       "bit_identical": bool(np.array_equal(g[:m], d_cpu[:m]))}
    # spares the pool started mid-slice and that ran requests of the timed window
    spares_run = [int(k) for k, v in per.items() if v["spare"] and v["gpu_window_requests"] > 0]
    return {"replicas": sorted(ens.delays), "count": len(per),
            "requests_compared": sum(v["requests_compared"] for v in per.values()),
            "bit_identical": all(v["bit_identical"] for v in per.values()),
            "spares_started_and_compared": spares_run,
            "covers_pool_handoff": bool(H.pool) and len(spares_run) > 0,
            "per_replica": per,
            "note": f"GPU delays of each replica (its {warm_reqs}-request warmup, then its timed window) against "
                    f"the {kind} uncore's on the same stream, run by the ensemble processes, compared over the "
                    f"requests both ran"}


def job_roofline(infos: list) -> dict:
    """The whole job's roofline: algorithmic bytes per launch summed over the
    ranks / the slowest rank's mean launch time / (ranks x HBM peak)."""
    n = len(infos)
    b = sum(i["bytes_per_launch"] for i in infos)
    ms = max(i["avg_launch_ms"] for i in infos)
    ach = b / (ms / 1e3) / 1e9
    return {"achieved": ach, "peak": n * HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / (n * HBM_PEAK_GBS),
            "alg_bytes_per_launch": b, "avg_launch_ms_max_over_ranks": ms,
            "per_rank_frac": [i["bytes_per_launch"] / (i["avg_launch_ms"] / 1e3) / 1e9 / HBM_PEAK_GBS for i in infos],
            "note": f"algorithmic bytes per launch summed over {n} rank(s) / the max over ranks of the HIP-event mean "
                    f"launch time / ({n} x {HBM_PEAK_GBS:g} GB/s)"}


# ---------------------------------------------------------------- GPU passes
class Pass:
    """One warmup + timed run of every replica on this GPU."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


def run_pass(um, args, R: int, rank: int, world: int, dev, stream, replay: int, steps: int, keep: list,
             slots: int = 0):
    """Warm every replica, then time `steps` launches.  `keep`: replicas whose
    delays (warmup and timed window) are returned for parity checks.  With
    slots < R the timed launches run the replica pool (pu_run_device_pool):
    `slots` wavefronts, each taking the next unstarted replica once its own is
    done or halted."""
    import torch
    import torch.distributed as dist

    import primesim_amd as P
    from primesim_amd import _abi as A
    from primesim_amd.dist import replica_seed

    sptr = stream.cuda_stream
    um.set_replay_mode(replay)
    specs = [stream_spec(replica_seed(SEED_BASE, rank, r)) for r in range(R)]
    # the host generates STAGE_GROUP replicas' chunks at a time into one reused
    # buffer (335 MB at the default chunk), so 8 ranks of 5,120 replicas each
    # hold ~3 GB of host staging in all instead of 6.7 GB per rank
    G = min(R, STAGE_GROUP)
    gens = [P.StreamSet(specs[g:g + G]) for g in range(0, R, G)]
    host = np.zeros((G, args.chunk), dtype=A.REQ_DTYPE)
    offs = torch.from_numpy((np.arange(R + 1, dtype=np.uint64) * np.uint64(args.chunk)).view(np.int64)).to(dev)
    kept = {r: [] for r in keep}

    def next_chunk(rb: int = REQ_BYTES) -> torch.Tensor:
        # rb = 16: the chunk as pu_req16 records (pack_req16 refuses what does not fit)
        out = torch.empty((R, args.chunk * rb), dtype=torch.uint8, device=dev)
        for k, gen in enumerate(gens):
            n = len(gen)
            got = gen.next_into(host[:n])
            assert got == args.chunk, (got, args.chunk)
            rec = host[:n] if rb == REQ_BYTES else P.uncore.pack_req16(host[:n])
            out[k * G:k * G + n].copy_(torch.from_numpy(rec.view(np.uint8).reshape(n, -1)))
        return out.view(-1)

    d_warm_delay = torch.zeros(R * args.chunk, dtype=torch.int32, device=dev)
    t_w = time.time()
    for s in range(args.warmup):
        d_req = next_chunk()
        um.run_device(d_req.data_ptr(), offs.data_ptr(), d_warm_delay.data_ptr(), sptr)
        torch.cuda.synchronize(dev)
        for r in keep:
            kept[r].append(d_warm_delay[r * args.chunk:(r + 1) * args.chunk].cpu().numpy())
        del d_req
        log(f"[bench] {'closed' if replay else 'open'}-loop warmup step {s} done ({time.time() - t_w:.1f}s)")
    if os.environ.get("PU_PROF_RESET_AFTER_WARMUP"):   # tools/prof_regions.py: count the timed steps only
        L = P.uncore.lib()
        (L.pu_jit_prof_read if os.environ.get("PU_PROF_JIT") else L.pu_engine_prof_read)(None, 0, 1)
    t_gen = time.time()
    W_t = steps * args.chunk
    # the timed window as 16-B records (--req-format 16): 20 B a request with
    # its delay instead of 36, so the driver's 20-step window fits a replica
    # pool over every resident wavefront in HBM
    rb = timed_req_bytes(args)
    d_win = torch.empty((R, W_t, rb), dtype=torch.uint8, device=dev)
    for k in range(steps):
        d_win[:, k * args.chunk:(k + 1) * args.chunk, :] = next_chunk(rb).view(R, args.chunk, rb)
    for gen in gens:
        gen.close()
    d_win_delay = torch.zeros(R * W_t, dtype=torch.int32, device=dev)
    win_off = np.arange(R + 1, dtype=np.uint64) * np.uint64(W_t)
    d_win_off = torch.from_numpy(win_off.view(np.int64)).to(dev)
    d_pos = torch.from_numpy(win_off[:-1].copy().view(np.int64)).to(dev)
    step_offs = [torch.from_numpy(np.concatenate([[0], win_off[:-1] + np.uint64((k + 1) * args.chunk)])
                                  .astype(np.uint64).view(np.int64)).to(dev) for k in range(steps)]
    pool = 0 < slots < R and args.slice_ms > 0
    d_sched = torch.zeros(um.pool_words(slots) if pool else 1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)
    log(f"[bench] timed requests resident: {R} x {W_t} in {time.time() - t_gen:.1f}s"
        + (f"; replica pool: {slots} wavefronts over {R} replicas" if pool else ""))
    before = sum_stats(um, R)
    per_before = [um.stats(r).as_dict() for r in range(R)] if os.environ.get("PU_PROF_RESET_AFTER_WARMUP") else None

    # HIP events on the engine's (non-null) stream time exactly its launches
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    um.set_device_req_format(P.uncore.PU_REQ_FMT_16 if rb == 16 else P.uncore.PU_REQ_FMT_32)
    try:
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for k in range(steps):
            ev[k][0].record(stream)
            if pool:
                um.run_device_pool(d_win.data_ptr(), d_win_off.data_ptr(), d_win_delay.data_ptr(), d_pos.data_ptr(),
                                   d_sched.data_ptr(), slots, int(args.slice_ms * 1000), sptr)
            elif args.slice_ms > 0:
                um.run_device_sliced(d_win.data_ptr(), d_win_off.data_ptr(), d_win_delay.data_ptr(),
                                     d_pos.data_ptr(), int(args.slice_ms * 1000), sptr)
            else:
                um.run_device_sliced(d_win.data_ptr(), step_offs[k].data_ptr(), d_win_delay.data_ptr(),
                                     d_pos.data_ptr(), 0, sptr)
            ev[k][1].record(stream)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
    finally:
        # the 32-B records the warm-up chunks (and any later pass) use, even
        # when a launch or the barrier raised
        um.set_device_req_format(P.uncore.PU_REQ_FMT_32)
    kern_ms = [a.elapsed_time(b) for a, b in ev]
    log(f"[bench] timed {steps} steps in {elapsed:.3f}s; per-launch ms {['%.1f' % x for x in kern_ms]}")
    pos = d_pos.cpu().numpy().view(np.uint64)
    adv = (pos - win_off[:-1]).astype(np.int64)
    flags = um.error_flags(R)
    halted_mask = (flags & A.PU_ERRF_NEG_DELAY) != 0
    pool_info = None
    if pool:
        sch = d_sched.cpu().numpy().view(np.uint32)
        b0 = (3 + slots) & ~1                                       # PU_POOL_BUSY0: one uint64 per slot
        busy_s = float(sch[b0:b0 + 2 * slots].view(np.uint64).astype(np.float64).sum()) * 1e-8   # 100-MHz ticks
        started = int(min(int(sch[0]), R))
        pool_info = {"wavefronts": slots, "replicas": R, "replicas_started": started,
                     "busy_fraction": busy_s / (slots * sum(kern_ms) / 1e3),
                     "note": "every wavefront's resident time (s_memrealtime) summed over the timed launches / "
                             "(wavefronts x the launches' HIP-event time)"}
        log(f"[bench] replica pool: {started} of {R} replicas started, busy fraction {pool_info['busy_fraction']:.4f}")
    log(f"[bench] requests per replica in the timed window: min {adv.min()} median {int(np.median(adv))} "
        f"max {adv.max()} of {W_t}; {int(((adv >= W_t) & ~halted_mask).sum())} finished the window, "
        f"{int(halted_mask.sum())} halted (prime.cpp:130-134)")
    for r in keep:
        kept[r].append(d_win_delay[r * W_t:r * W_t + int(adv[r])].cpu().numpy())
    after = sum_stats(um, R)
    per_replica = None
    if per_before is not None:
        per_after = [um.stats(r).as_dict() for r in range(R)]
        keys = ("requests", "net_accesses", "net_distance", "mg1_calls", "lockdown_calls", "dram_accesses",
                "total_num_broadcast", "L0_miss", "directory_ins", "directory_miss", "net_total_delay")
        per_replica = {k: [int(per_after[r][k] - per_before[r][k]) for r in range(R)] for k in keys}
    delta = {k: after[k] - before.get(k, 0) for k in after if k != "error_flags"}
    halted = int(halted_mask.sum())
    del d_win, d_win_delay
    return Pass(elapsed=elapsed, kern_ms=kern_ms, adv=adv, kept={r: np.concatenate(v) for r, v in kept.items()},
                delta=delta, halted=halted, errf=int(np.bitwise_or.reduce(flags)) if len(flags) else 0,
                per_replica=per_replica, steps=steps, processed=int(delta["requests"]), pool=pool_info)


def single_instance(cfg, args, dev, threads, replay: int = 0) -> dict:
    """ONE simulation alone on the GPU: replica 0's stream, the same warmup,
    then --single-requests requests in one launch (HIP events)."""
    import torch

    import primesim_amd as P
    from primesim_amd.dist import replica_seed
    n_w, n_t = args.warmup * args.chunk, args.single_requests
    reqs = P.generate_stream(stream_spec(replica_seed(SEED_BASE, 0, 0), n_w + n_t))
    um = P.UncoreManager()
    um.init(cfg, replicas=1, device=dev.index)
    um.set_replay_mode(replay)
    for prog, th in threads:
        um.allocCore(prog, th)
    stream = torch.cuda.Stream(dev)
    d_req = torch.from_numpy(reqs.view(np.uint8)).to(dev)
    d_delay = torch.zeros(len(reqs), dtype=torch.int32, device=dev)
    off_w = torch.tensor([0, n_w], dtype=torch.int64, device=dev)
    off_t = torch.tensor([0, n_w + n_t], dtype=torch.int64, device=dev)
    pos = torch.tensor([n_w], dtype=torch.int64, device=dev)
    um.run_device(d_req.data_ptr(), off_w.data_ptr(), d_delay.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize(dev)
    before = um.stats(0).as_dict()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    um.run_device_sliced(d_req.data_ptr(), off_t.data_ptr(), d_delay.data_ptr(), pos.data_ptr(), 0, stream.cuda_stream)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    ms = e0.elapsed_time(e1)
    st = um.stats(0).as_dict()
    um.close()
    done = st["requests"] - before["requests"]     # a halted replica stops counting
    mode = "closed-loop" if replay else "open-loop"
    return {"value": done / (ms / 1e3), "unit": "accesses/s", "requests": int(done), "kernel_ms": ms, "wall_s": wall,
            "mg1_share_of_link_visits": (st["mg1_calls"] - before["mg1_calls"]) /
                                        max(1, st["net_distance"] - before["net_distance"]),
            "sample": f"one {WORKLOAD} simulation alone on the GPU (replica 0's stream, {mode}): {n_w} warmup requests, then "
                      f"{n_t} requests in one launch; link visits/access "
                      f"{(st['net_distance'] - before['net_distance']) / max(1, done):.1f}",
            "note": "one uncore is a sequential fold (one wavefront); DESIGN.md §1a measures how little of it a "
                    "relaxation can parallelise"}


# ---------------------------------------------------------------- N > 1 launch
def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv: list, child_cmd: list | None = None, timeout_s: float | None = None) -> int:
    """`bench.py --gpus N` without a launcher: start N rank processes (fresh
    children, one per GPU, LOCAL_RANK = rank; no exec) with the env that
    torch.distributed.run would give them, wait for all, and return the worst
    exit code.  Called before this process touches the GPU.  Rank 0 prints
    the JSON line on the inherited stdout."""
    import subprocess
    port = free_port()
    cmd = child_cmd or LAUNCH_CMD or [sys.executable, os.path.abspath(__file__)]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([*cmd, *argv], env=env))
    rc, t0 = 0, time.time()
    try:
        for p in procs:
            left = None if timeout_s is None else max(1.0, timeout_s - (time.time() - t0))
            c = p.wait(timeout=left)
            if c != 0 and rc == 0:
                rc = c
                log(f"[bench] a rank exited with {c}; stopping the others")
                for q in procs:
                    if q.poll() is None:
                        q.terminate()
    finally:
        for q in procs:                       # the exact children started here
            if q.poll() is None:
                q.kill()
                q.wait()
    return rc


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs of this node; N > 1 without WORLD_SIZE starts N rank processes itself")
    ap.add_argument("--steps", type=int, default=10, help="timed steps")
    ap.add_argument("--warmup", type=int, default=10, help="untimed steps of --chunk requests per replica")
    ap.add_argument("--replicas", type=int, default=0, help="replicas per GPU (0 = size to HBM)")
    ap.add_argument("--req-format", type=int, choices=(16, 32), default=16,
                    help="timed-window request records: 16-B pu_req16 (pu_pack_req16) or 32-B pu_req")
    ap.add_argument("--hbm-fraction", type=float, default=float(os.environ.get("PU_BENCH_HBM_FRACTION", "0.88")),
                    help="share of the free HBM the replicas and their request windows may take")
    ap.add_argument("--slots", type=int, default=int(os.environ.get("PU_BENCH_SLOTS", "0")),
                    help="wavefront slots per GPU (0 = every replica slot the kernel keeps resident)")
    ap.add_argument("--spare-replicas", type=float, default=0.1,
                    help="replicas beyond the resident wavefront slots, as a fraction of them (replica pool)")
    ap.add_argument("--chunk", type=int, default=0,
                    help="requests per replica per step (0 = the configuration's: 40,960 for C4 and C5, 61,440 for C3)")
    ap.add_argument("--slice-ms", type=float, default=400.0,
                    help="timed steps are wall-time slices: every replica continues its own stream for this long "
                         "per launch (stopping only between requests); 0 = fixed --chunk requests per replica per step")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--ensemble-seconds", type=float, default=3.0)
    ap.add_argument("--ensemble-workers", type=int, default=0, help="0 = every host core of this job's share")
    ap.add_argument("--rank-parity-workers", type=int, default=2,
                    help="N > 1: reference processes per rank (forked before the GPU) replaying that rank's replica 0 "
                         "and its first pool spare; their delays are checked against the GPU's and gathered to rank 0 "
                         "(0 = no parity at N > 1)")
    ap.add_argument("--closed-steps", type=int, default=5, help="timed steps of the closed-loop pass (0 = skip)")
    ap.add_argument("--single-requests", type=int, default=40960)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="headline only (profiling runs)")
    ap.add_argument("--config", choices=sorted(WORKLOADS), default="C4",
                    help="SURVEY.md §8d shape: C4 (1024 cores) is the metric's; C3 (256 cores, 3 levels) and C5 "
                         "(4096 cores) are measured the same way")
    ap.add_argument("--replay", choices=("open", "closed"), default=None,
                    help="headline replay mode (open: the metric; closed: profiling / A/B runs of the realistic "
                         "regime); default: the configuration's (open for C3/C4, closed for C5)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL) normally; gloo for CPU-side rehearsal")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC traffic summary written by tools/pmc_traffic.py for this build")
    a = ap.parse_args(argv)
    if a.replay is None:
        a.replay = WORKLOADS[a.config]["replay"]
    if a.chunk <= 0:
        a.chunk = WORKLOADS[a.config]["chunk"]
    return a


class Device:
    """This rank's GPU, engine handle and stream (bench's only device state)."""

    def __init__(self, args, cfg, threads, rank: int, local: int):
        import torch

        import primesim_amd as P
        torch.cuda.set_device(local)
        self.dev = torch.device("cuda", local)
        # ---- per-replica HBM: engine state + the timed request slabs + one warmup chunk
        probe = P.UncoreManager()
        probe.init(cfg, replicas=1, device=local)
        rbytes = probe.replica_bytes
        resident = probe.resident_replicas
        probe.close()
        # ranks rehearsed on one card (PU_BENCH_DEVICE) split its memory and waves
        share = int(os.environ.get("LOCAL_WORLD_SIZE", "1")) if "PU_BENCH_DEVICE" in os.environ else 1
        per_bytes = rbytes + args.steps * args.chunk * (timed_req_bytes(args) + 4) + args.chunk * (REQ_BYTES + 4)
        free, _ = torch.cuda.mem_get_info(self.dev)
        # one wavefront per replica slot the kernel keeps resident, and up to
        # --spare-replicas more replicas (as HBM allows) for the replica pool:
        # a wavefront whose replica halts or finishes its window takes an
        # unstarted one (pu_run_device_pool), so no slot idles
        res = max(1, resident // share)
        if args.slots:
            res = min(res, args.slots)
        fit = int((free * args.hbm_fraction / share) // per_bytes)
        R = args.replicas or max(1, min(int(res * (1.0 + args.spare_replicas)), fit))
        R = max(1, R - R % 8) if R >= 8 else R
        self.slots = min(R, res)
        log(f"[bench] rank {rank}: replica {rbytes / 2**20:.0f} MiB + requests {(per_bytes - rbytes) / 2**20:.0f} MiB, "
            f"{R} replicas on {self.slots} wavefronts (resident limit {resident}), free {free / 2**30:.0f} GiB")
        self.R = R
        self.um = P.UncoreManager()
        self.um.init(cfg, replicas=R, device=local)
        for prog, th in threads:
            self.um.allocCore(prog, th)
        self.stream = torch.cuda.Stream(self.dev)
        assert self.stream.cuda_stream != 0
        self.compiled = P.uncore.lib().pu_compiled_config(self.um._handle())   # 0, 1 or 2 (primeuncore.h)
        self.compiler = P.uncore.lib().pu_compiled_compiler(self.um._handle())   # 0, 1 hipRTC, 2 hipcc

    def headline(self, args, rank: int, world: int, keep: list):
        import primesim_amd as P
        mode = P.uncore.PU_REPLAY_CLOSED if args.replay == "closed" else P.uncore.PU_REPLAY_OPEN
        return run_pass(self.um, args, self.R, rank, world, self.dev, self.stream, mode, args.steps, keep,
                        self.slots)

    def reduce_device(self, args):
        """Where the max/sum reduction's tensors live: the GPU under RCCL."""
        return self.dev if args.dist_backend == "nccl" else None


def main(argv=None) -> None:
    args = parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # before any GPU call: this process only waits for its N ranks
        sys.exit(launch_ranks(args.gpus, sys.argv[1:] if argv is None else list(argv)))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        log(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a {world}-rank run "
            f"as {args.gpus} GPUs")
        sys.exit(2)
    extras = rank == 0 and world == 1 and not args.no_extras

    import primesim_amd as P
    from primesim_amd import _abi as A
    from primesim_amd import config as CF
    from primesim_amd.dist import gather_objects, reduce_run, replica_seed

    global WORKLOAD
    WORKLOAD = args.config
    sim = CF.preset(WORKLOAD)
    xml_path = os.path.join(tempfile.gettempdir(), f"pu_bench_c4_{os.getpid()}.xml")
    CF.write_xml(sim, xml_path)
    cfg = P.load_config(xml_path)
    threads = P.stream_threads(stream_spec(SEED_BASE))

    # ---- the CPU ensemble forks now, before this process touches the GPU: at
    # N=1 one reference process per host core (parity + the ensemble baseline);
    # at N>1 a few per rank, replaying this rank's replica 0 and first pool
    # spare (parity of every rank's line)
    ens = None
    rank_parity = world > 1 and not args.no_cpu and args.rank_parity_workers > 0
    if (extras and not args.no_cpu) or rank_parity:
        nw = (args.ensemble_workers or host_core_share()) if extras else args.rank_parity_workers
        ens = Ensemble(xml_path, nw, args.warmup * args.chunk, args.steps * args.chunk, args.ensemble_seconds, rank,
                       ref_mode(args))

    import torch.distributed as dist
    if world > 1:
        dist.init_process_group(args.dist_backend, init_method="env://")
    # PU_BENCH_DEVICE pins every rank to one card (rehearsing N>1 on a 1-GPU box)
    local = int(os.environ.get("PU_BENCH_DEVICE", local))
    D = Device(args, cfg, threads, rank, local)
    R, um, dev, stream = D.R, D.um, D.dev, D.stream
    global LAST_REPLICAS, LAST_PER_REPLICA
    LAST_REPLICAS = R
    # the ensemble's replicas, spread over 0..R-1: their delays are checked
    # against the reference's bit for bit (replica 0 also by cpu_baseline)
    keep = sorted(set(ens.assign(R, D.slots)) | {0}) if ens is not None else [0]

    # ---- headline: open-loop replay
    H = D.headline(args, rank, world, keep)
    LAST_PER_REPLICA = H.per_replica
    t_max, tot_processed = reduce_run(H.elapsed, H.processed, D.reduce_device(args))
    _, tot_replicas = reduce_run(0.0, R, D.reduce_device(args))
    _, tot_slots = reduce_run(0.0, D.slots, D.reduce_device(args))
    value = tot_processed / t_max
    avg_ms = float(np.mean(H.kern_ms))
    bytes_per_launch = alg_bytes(H.delta, cfg) / args.steps
    achieved = bytes_per_launch / (avg_ms / 1e3) / 1e9

    parity_ok = True
    result = None
    busy_err = busy_guard(H.pool)
    if busy_err:
        log(f"[bench] {busy_err}")
    # every rank: its replicas' parity against the reference, then the gather
    ens_res, rparity = None, None
    if ens is not None:
        ens_res = ens.run()
        log(f"[bench] rank {rank}: cpu ensemble ({ens_res['kind']}, {ens_res['cores']} processes): "
            f"{ens_res['value']:.0f} accesses/s")
        rparity = replica_parity(ens, H, D.slots, ens_res["kind"], args.warmup * args.chunk)
        log(f"[bench] rank {rank}: replica parity: {rparity['count']} replicas "
            f"({rparity['replicas'][0]}..{rparity['replicas'][-1]}), "
            f"{rparity['requests_compared']} delays, bit-identical {rparity['bit_identical']}")
    infos = gather_objects({"rank": rank, "bytes_per_launch": bytes_per_launch, "avg_launch_ms": avg_ms,
                            "replicas": R, "wavefronts": D.slots,
                            "parity": None if rparity is None else
                            {k: rparity[k] for k in ("replicas", "requests_compared", "bit_identical",
                                                     "covers_pool_handoff", "spares_started_and_compared")}})
    ranks_checked = [i for i in infos if i["parity"] is not None]
    ranks_parity = None
    if world > 1 and ranks_checked:
        ranks_parity = {"bit_identical": all(i["parity"]["bit_identical"] for i in ranks_checked),
                        "ranks_checked": len(ranks_checked),
                        "requests_compared": sum(i["parity"]["requests_compared"] for i in ranks_checked),
                        "per_rank": [{"rank": i["rank"], **i["parity"]} for i in infos if i["parity"] is not None],
                        "note": "each rank replays its replica 0 and its first replica-pool spare (or its last replica "
                                "without a pool) on the reference uncore in processes forked before the GPU; their "
                                "delays (warmup and timed window) are compared with that rank's GPU delays over the "
                                "requests both ran, then gathered to rank 0"}
        parity_ok &= ranks_parity["bit_identical"]
    if rparity is not None:
        parity_ok &= rparity["bit_identical"]
    job_rf = job_roofline(infos)
    if rank == 0:
        replica_parity_res = rparity if world == 1 else None
        closed = None
        if extras and args.closed_steps > 0 and args.replay == "open":
            um.reset()
            C = run_pass(um, args, R, rank, world, dev, stream, P.uncore.PU_REPLAY_CLOSED, args.closed_steps,
                         [0], D.slots)
            c_par, c_cpu = None, None
            if not args.no_cpu:
                import oracle as O
                w0, n_t = args.warmup * args.chunk, args.closed_steps * args.chunk
                s0 = P.generate_stream(stream_spec(replica_seed(SEED_BASE, 0, 0), w0 + n_t))
                kind, n_cpu, el, d_cpu = cpu_baseline(xml_path, cfg, s0, threads, w0, 5.0, O.MODE_CLOSED)
                gd = C.kept[0]
                m = min(len(d_cpu), len(gd))
                c_par = {"kind": kind, "requests_compared": m, "bit_identical": bool(np.array_equal(gd[:m], d_cpu[:m]))}
                parity_ok &= c_par["bit_identical"]
                c_cpu = {"value": n_cpu / el, "unit": "accesses/s", "cores": 1, "kind": kind, "cpu_model": cpu_model(),
                         "sample": f"replica 0's {WORKLOAD} stream replayed closed-loop: requests {w0}..{w0 + n_cpu} after an "
                                   f"untimed closed-loop fill of {w0}, single-threaded "
                                   f"({'reference uncore compiled from /root/reference/src, no counting wraps' if kind == 'reference' else 'oracle/cpu_ref restatement'}), "
                                   f"{el:.1f} s"}
                log(f"[bench] closed-loop cpu baseline ({kind}): {n_cpu / el:.0f} accesses/s")
            c_ms = float(np.mean(C.kern_ms))
            c_bytes = alg_bytes(C.delta, cfg) / C.steps
            closed = {"value": C.processed / C.elapsed, "unit": "accesses/s", "steps": C.steps,
                      "roofline": {"bound": "hbm", "achieved": c_bytes / (c_ms / 1e3) / 1e9, "peak": HBM_PEAK_GBS,
                                   "unit": "GB/s", "frac": c_bytes / (c_ms / 1e3) / 1e9 / HBM_PEAK_GBS,
                                   "alg_bytes_per_launch": c_bytes, "avg_launch_ms": c_ms,
                                   "alg_bytes_per_access": alg_bytes(C.delta, cfg) / max(1, C.processed),
                                   "tree_visits_per_access": (C.delta["net_distance"] - C.delta["mg1_calls"]) /
                                                             max(1, C.processed),
                                   "note": "the closed-loop pass's algorithmic bytes per launch / its HIP-event mean "
                                           "launch time (same kernel as the headline)"},
                      "per_simulation_accesses_per_s": C.processed / C.elapsed / D.slots,
                      "replica_pool": C.pool,
                      "halted_replicas": C.halted,
                      "mg1_share_of_link_visits": C.delta["mg1_calls"] / max(1, C.delta["net_distance"]),
                      "mean_delay_cycles": 0.0,
                      "parity": c_par,
                      "cpu_baseline": c_cpu,
                      "single_instance": None}
            gd = C.kept[0]
            closed["mean_delay_cycles"] = float(gd[gd != 0].mean()) if (gd != 0).any() else 0.0
            busy_err = busy_err or busy_guard(C.pool)
            log(f"[bench] closed loop: {closed['value']:.4g} accesses/s, halted {C.halted}, "
                f"M/G/1 share {closed['mg1_share_of_link_visits']:.3f}")
        um.close()
        single = single_instance(cfg, args, dev, threads,
                                 P.uncore.PU_REPLAY_CLOSED if args.replay == "closed" else 0) if extras else None
        if single:
            log(f"[bench] single instance: {single['value']:.0f} accesses/s")
        if closed is not None:
            closed["single_instance"] = single_instance(cfg, args, dev, threads, P.uncore.PU_REPLAY_CLOSED)
            log(f"[bench] closed-loop single instance: {closed['single_instance']['value']:.0f} accesses/s")
        cpu = None
        if not args.no_cpu and world == 1:          # the CPU baseline runs at N=1 only
            # replica 0's stream: the reference fills the warmup untimed, then is
            # timed on the requests of the GPU's timed window (as many as fit in
            # --cpu-seconds); parity is checked on every request both ran
            w0, n_t = args.warmup * args.chunk, args.steps * args.chunk
            s0 = P.generate_stream(stream_spec(replica_seed(SEED_BASE, rank, 0), w0 + n_t))
            kind, n_cpu, el, d_cpu = cpu_baseline(xml_path, cfg, s0, threads, w0, args.cpu_seconds, ref_mode(args))
            gpu_d = H.kept[0]
            m = min(len(d_cpu), len(gpu_d))
            parity = bool(np.array_equal(gpu_d[:m], d_cpu[:m]))
            parity_ok &= parity
            cpu = {"value": n_cpu / el, "unit": "accesses/s", "cores": 1, "kind": kind, "cpu_model": cpu_model(),
                   "sample": f"replica 0's {WORKLOAD} stream ({args.replay} loop): requests {w0}..{w0 + n_cpu} (the GPU's timed window; the GPU "
                             f"ran {int(H.adv[0])} of them for replica 0), after an untimed fill of the {w0}-request "
                             f"warmup, single-threaded "
                             f"({'reference uncore compiled from /root/reference/src, no counting wraps' if kind == 'reference' else 'oracle/cpu_ref restatement'}), "
                             f"{el:.1f} s; GPU delays bit-identical on all {m} requests compared: {parity}",
                   "parity": parity}
            log(f"[bench] cpu baseline ({kind}): {n_cpu / el:.0f} accesses/s; parity on {m} delays: {parity}")

        # fabric traffic measured by tools/pmc_traffic.py for this build only
        traffic, traffic_src = None, None
        if os.path.exists(args.traffic_json):
            with open(args.traffic_json) as f:
                tj = json.load(f)
            built = P.uncore.library_source_hash()
            if tj.get("src_hash") == built:
                traffic = tj["fabric_bytes_per_access"] * (H.processed / args.steps)
                how = ("reads in 32-B units (TCC_EA0_RDREQ_*_32B) + WRITE_SIZE" if "read_bytes_per_launch_32b_units" in tj
                       else "FETCH_SIZE+WRITE_SIZE")
                win = " ".join(tj.get("bench_args", [])[:4])
                traffic_src = (f"{os.path.relpath(args.traffic_json, ROOT)}: {tj['fabric_bytes_per_access']:.0f} B/access "
                               f"({how}, separate PMC passes; fabric bytes incl. MALL hits) measured on build {built} "
                               f"at {tj['replicas']} replicas, bench window {win}; "
                               f"{tj['fabric_bytes_per_access'] / max(1e-9, alg_bytes(H.delta, cfg) / H.processed):.2f}x "
                               f"this run's algorithmic bytes per access")
            else:
                traffic_src = (f"not reported: {os.path.relpath(args.traffic_json, ROOT)} was measured on build "
                               f"{tj.get('src_hash')}, this library is {built}")
        result = {
            "metric": METRIC if WORKLOAD == "C4" else
                      METRIC.replace("at 1024 cores", f"at {WORKLOADS[WORKLOAD]['cores']} cores ({WORKLOAD})"),
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
                "workload": f"{WORKLOADS[WORKLOAD]['desc']}, {args.replay}-loop replay",
                "replicas_per_gpu": R,
                "replicas_total": tot_replicas,
                "wavefronts_per_gpu": D.slots,
                "replica_pool": H.pool,
                "step": (f"wall-time slice: every replica continues its own stream for {args.slice_ms:g} ms per "
                         f"launch, stopping only between requests" if args.slice_ms > 0 else
                         f"fixed: {args.chunk} requests per replica per launch"),
                "mean_requests_per_replica_per_step": H.processed / (R * args.steps),
                "warmup_requests_per_replica": args.warmup * args.chunk,
                "timed_request_record_bytes": timed_req_bytes(args),
                "parallelism": (f"replicas: {R} independent uncores per GPU ({D.slots} simulated at once, one "
                                f"wavefront each) x {world} GPU(s), one process per GPU, no data-path collective "
                                f"({args.dist_backend} for the barrier and the max/sum reduction only)" if world > 1 else
                                f"replicas: {R} independent uncores on 1 GPU, {D.slots} simulated at once (one "
                                f"wavefront each)"),
                "halted_replicas": H.halted,
                "mg1_share_of_link_visits": H.delta["mg1_calls"] / max(1, H.delta["net_distance"]),
                "error_flags": H.errf & ~A.PU_ERRF_NEG_DELAY,
                "engine_build": P.uncore.library_source_hash(),
                "engine_variant": VARIANTS[D.compiled] + (f" ({COMPILERS[D.compiler]})" if D.compiler else ""),
            },
            "per_simulation_accesses_per_s": value / tot_slots,
            "single_instance": single,
            "closed_loop": closed,
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel": (("pu_jit_uncore_s2_h0" if H.pool else "pu_jit_uncore_s1_h0") if D.compiled == 2 else
                           ("uncore_kernel<1, 2, false>" if H.pool else "uncore_kernel<1, 1, false>")),
                "avg_launch_ms": avg_ms,
                "alg_bytes_per_launch": bytes_per_launch,
                "limiter": LIMITER,
                "scope": "rank 0's kernel: its algorithmic bytes per launch / its HIP-event mean launch time",
                "job": job_rf,
            },
            "cpu_baseline": cpu,
            "cpu_baseline_ensemble": ens_res if world == 1 else None,
            "replica_parity": replica_parity_res,
            "rank_parity": ranks_parity,
            "parity": parity_ok if (not args.no_cpu and (world == 1 or ranks_parity is not None)) else None,
            "busy_guard": busy_err or f"ok: replica-pool busy fraction >= {BUSY_MIN} (or the pool ran dry)",
        }
        print(json.dumps(result), flush=True)
    else:
        um.close()
    try:
        os.remove(xml_path)
    except OSError:
        pass
    if world > 1:
        dist.destroy_process_group()
    if not parity_ok:
        log("[bench] PARITY FAILURE: GPU delays differ from the reference")
        sys.exit(1)
    if busy_err:
        log("[bench] RESIDENCY FAILURE: the timed launches were not one slice each; the rate is not valid")
        sys.exit(3)


if __name__ == "__main__":
    main()
