"""Generate tests/golden/* from the REFERENCE's own uncore (oracle/_ref).

Run in the build container only (it needs /root/reference compiled by
`make -C oracle ref`).  Every fixture is data: inputs (config XML, request
stream, queue/network call sequences) and the reference's outputs (per-request
delays, per-core completion cycles, UncoreManager::report text minus the
wall-clock line, -Wl,--wrap counters, the parsed XmlSim).

    python tools/gen_golden.py            # all cases
    python tools/gen_golden.py c1_stream  # one case
"""
from __future__ import annotations

import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import primesim_amd as P  # noqa: E402
from primesim_amd import _abi as A  # noqa: E402
from primesim_amd import config as CF  # noqa: E402
import oracle as O  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")


def _c1_shape(cores: int, **kw) -> dict:
    sim = CF.preset("C1", **kw)
    sim["system"]["num_cores"] = cores
    return sim


def _three_level(cores: int) -> dict:
    sim = CF.preset("C1")
    s = sim["system"]
    s["num_cores"] = cores
    s["num_levels"] = 3
    s["cache"] = [
        {"level": 0, "share": 1, "access_time": 1, "size": 8192, "block_size": 64, "num_ways": 4},
        {"level": 1, "share": 1, "access_time": 5, "size": 32768, "block_size": 64, "num_ways": 8},
        {"level": 2, "share": 4, "access_time": 10, "size": 131072, "block_size": 64, "num_ways": 8},
    ]
    s["directory_cache"] = {"level": 0, "share": 1, "access_time": 10, "size": 262144, "block_size": 64,
                            "num_ways": 8}
    s["bus_latency"] = 2
    return sim


def _l2_shared(cores: int) -> dict:
    sim = CF.preset("C1")
    s = sim["system"]
    s["num_cores"] = cores
    s["num_levels"] = 2
    s["cache"] = [
        {"level": 0, "share": 1, "access_time": 1, "size": 8192, "block_size": 64, "num_ways": 4},
        {"level": 1, "share": 4, "access_time": 6, "size": 65536, "block_size": 64, "num_ways": 8},
    ]
    s["bus_latency"] = 3
    return sim


def cases() -> dict:
    S = P.StreamSpec
    c = {}
    c["c1_stream"] = (CF.preset("C1"), S(A.PU_STREAM_PRIVATE_STREAMING, 16, seed=1, num_quanta=3))
    c["c1_hot"] = (CF.preset("C1"), S(A.PU_STREAM_UNIFORM_HOTSPOT, 16, seed=11, num_quanta=2))
    c["c2_canneal"] = (CF.preset("C2"), S(A.PU_STREAM_SHARED_UNIFORM, 64, seed=2, num_quanta=2,
                                          max_requests=20000))
    c["c3_multiprog"] = (CF.preset("C3"), S(A.PU_STREAM_MULTIPROGRAM, 256, seed=3, num_quanta=1, num_progs=4,
                                            max_requests=20000))
    c["c4_hotspot"] = (CF.preset("C4"), S(A.PU_STREAM_UNIFORM_HOTSPOT, 1024, seed=4, num_quanta=1,
                                          max_requests=15000))
    # every core active: a 20-cycle quantum gives ~8 requests per core
    c["c4_allcores"] = (CF.preset("C4"), S(A.PU_STREAM_UNIFORM_HOTSPOT, 1024, seed=44, quantum=20, num_quanta=2,
                                           max_requests=16000))
    # 8192 cores (a 91x91 mesh, more than 4096 LLC nodes: 16-bit inline sharer
    # ids, sharer bitmaps of 128 words); a 4-cycle quantum puts every core in
    # the stream, the 64-line hotspot gives lines thousands of sharers
    c["mesh_8192"] = (_c1_shape(8192), S(A.PU_STREAM_UNIFORM_HOTSPOT, 8192, seed=81, quantum=4, num_quanta=3,
                                         max_requests=30000))
    c["c5_prodcons"] = (CF.preset("C5", dir_size=16384, dir_ways=4),
                        S(A.PU_STREAM_PRODUCER_CONSUMER, 4096, seed=5, quantum=8, num_quanta=2,
                          max_requests=16000))
    c["c5_prodcons_256"] = (_c1_shape(256), S(A.PU_STREAM_PRODUCER_CONSUMER, 256, seed=55, quantum=100,
                                             num_quanta=2, max_requests=20000))
    c["limited_ptr"] = (_c1_shape(16, protocol_type=1, max_num_sharers=2),
                        S(A.PU_STREAM_UNIFORM_HOTSPOT, 16, seed=6, num_quanta=2))
    c["limited_ptr_dironly"] = (_c1_shape(16, protocol_type=1, max_num_sharers=3, shared_llc=0),
                                S(A.PU_STREAM_UNIFORM_HOTSPOT, 16, seed=66, num_quanta=2))
    c["dir_only"] = (_c1_shape(16, shared_llc=0), S(A.PU_STREAM_UNIFORM_HOTSPOT, 16, seed=7, num_quanta=2))
    c["dir_only_c2"] = (CF.preset("C2", shared_llc=0), S(A.PU_STREAM_SHARED_UNIFORM, 64, seed=77, num_quanta=1,
                                                         max_requests=20000))
    # Q7: non-power-of-two directory sets (192 KB / 64 B / 8 W = 384 sets) with
    # 1,464 directory replacements whose victim addresses are mis-reconstructed,
    # on a seed that stays clear of the WB-miss NULL dereference (Q13)
    c["q7_nonpow2"] = (_c1_shape(16, dir_size=196608, dir_ways=8),
                       S(A.PU_STREAM_SHARED_UNIFORM, 16, seed=12, num_quanta=1))
    # Q7 with the config_prime default 30 MB / 24 W slice (20,480 sets)
    c["q7_default_dir"] = (_c1_shape(4, dir_size=31457280, dir_ways=24),
                           S(A.PU_STREAM_UNIFORM, 4, seed=9, num_quanta=3))
    # sets wider than 64 ways (the engine walks them in 64-way chunks): a
    # 128-way directory slice (8 sets), a 128-way L1 with a 128-entry fully
    # associative TLB, a 192-way L1 on the snoopy bus
    c["dir_128way"] = (_c1_shape(16, dir_size=65536, dir_ways=128),
                       S(A.PU_STREAM_SHARED_UNIFORM, 16, seed=31, num_quanta=2))
    wide = _c1_shape(16, tlb_enable=1, page_size=4096)
    wide["system"]["cache"][0].update(size=16384, num_ways=128)
    wide["system"]["tlb_cache"] = {"level": 0, "share": 1, "access_time": 1, "size": 128, "block_size": 1,
                                   "num_ways": 128}
    c["l1_tlb_128way"] = (wide, S(A.PU_STREAM_MULTIPROGRAM, 16, seed=32, num_quanta=2, num_progs=2))
    bwide = _c1_shape(16, sys_type=1)
    bwide["system"]["cache"][0].update(size=24576, num_ways=192)
    c["bus_192way"] = (bwide, S(A.PU_STREAM_SHARED_UNIFORM, 16, seed=33, num_quanta=2))
    c["l2_shared_bus"] = (_l2_shared(64), S(A.PU_STREAM_MULTIPROGRAM, 64, seed=10, num_quanta=1, num_progs=2,
                                            max_requests=20000))
    c["three_level"] = (_three_level(64), S(A.PU_STREAM_SHARED_UNIFORM, 64, seed=12, num_quanta=1,
                                            max_requests=20000))
    c["mesh3d"] = (CF.preset("C2", net_type=1), S(A.PU_STREAM_SHARED_UNIFORM, 64, seed=13, num_quanta=1,
                                                  max_requests=20000))
    c["net_variant"] = (_c1_shape(16, router_delay=1, inject_delay=2, data_width=16, header_flits=2,
                                  link_delay=2, dram_access_time=80),
                        S(A.PU_STREAM_UNIFORM_HOTSPOT, 16, seed=14, num_quanta=2))
    c["nonsquare_12"] = (_c1_shape(12), S(A.PU_STREAM_UNIFORM_HOTSPOT, 12, seed=15, num_quanta=2))
    c["small_msgs"] = (CF.preset("C1"), S(A.PU_STREAM_SHARED_UNIFORM, 16, seed=16, num_quanta=2, max_msg=7))
    # open-loop replay drives a Graphite queue delay past 2^31: the reference's
    # int arithmetic goes negative at request 34,904 and prime.cpp:130-134 stops
    # the handler there; the replay halts at the same request
    c["c4_overflow_halt"] = (CF.preset("C4"), S(A.PU_STREAM_UNIFORM_HOTSPOT, 1024, seed=162, num_quanta=64,
                                                max_requests=35000))
    c["verbose"] = (_c1_shape(16, verbose_report=1), S(A.PU_STREAM_UNIFORM_HOTSPOT, 16, seed=17, num_quanta=1))
    c["verbose_l2"] = (dict(_l2_shared(16), **{}), S(A.PU_STREAM_UNIFORM_HOTSPOT, 16, seed=18, num_quanta=1))
    c["verbose_l2"][0]["system"]["verbose_report"] = 1
    # TLB + first-touch page table (system.cpp:897-918, page_table.cpp:56-72):
    # config_prime's 64-entry fully associative TLB, 4 KB pages, several programs
    c["tlb_c1"] = (_c1_shape(16, tlb_enable=1), S(A.PU_STREAM_MULTIPROGRAM, 16, seed=21, num_quanta=2, num_progs=2))
    c["tlb_verbose"] = (_c1_shape(16, tlb_enable=1, verbose_report=1),
                        S(A.PU_STREAM_MULTIPROGRAM, 16, seed=22, num_quanta=1, num_progs=4))
    c["tlb_c3"] = (CF.preset("C3", tlb_enable=1), S(A.PU_STREAM_MULTIPROGRAM, 256, seed=23, num_quanta=1,
                                                    num_progs=4, max_requests=20000))
    tlb_sa = _c1_shape(16, tlb_enable=1, page_size=1024, page_miss_delay=150)
    tlb_sa["system"]["tlb_cache"] = {"level": 0, "share": 1, "access_time": 1, "size": 32, "block_size": 1,
                                     "num_ways": 4}
    c["tlb_setassoc"] = (tlb_sa, S(A.PU_STREAM_SHARED_UNIFORM, 16, seed=28, num_quanta=2))
    # snoopy bus MESI (sys_type=1, system.cpp:224-368)
    c["bus_c1"] = (_c1_shape(16, sys_type=1), S(A.PU_STREAM_UNIFORM_HOTSPOT, 16, seed=24, num_quanta=2))
    bl2 = _l2_shared(64)
    bl2["system"]["sys_type"] = 1
    c["bus_l2_shared"] = (bl2, S(A.PU_STREAM_MULTIPROGRAM, 64, seed=25, num_quanta=1, num_progs=2,
                                 max_requests=20000))
    b3 = _three_level(64)
    b3["system"]["sys_type"] = 1
    c["bus_three_level"] = (b3, S(A.PU_STREAM_SHARED_UNIFORM, 64, seed=26, num_quanta=1, max_requests=20000))
    c["bus_tlb_verbose"] = (_c1_shape(16, sys_type=1, tlb_enable=1, verbose_report=1),
                            S(A.PU_STREAM_MULTIPROGRAM, 16, seed=27, num_quanta=1, num_progs=2))
    c["bus_c2"] = (CF.preset("C2", sys_type=1), S(A.PU_STREAM_SHARED_UNIFORM, 64, seed=29, num_quanta=1,
                                                  max_requests=20000))
    # closed-loop replay (timer_i += the core's earlier batch delays, core_manager.cpp:265)
    c["c1_closed"] = (CF.preset("C1"), S(A.PU_STREAM_UNIFORM_HOTSPOT, 16, seed=31, num_quanta=4), {"replay": "closed"})
    c["c3_closed"] = (CF.preset("C3"), S(A.PU_STREAM_MULTIPROGRAM, 256, seed=33, num_quanta=1, num_progs=4,
                                         max_requests=20000), {"replay": "closed"})
    c["c4_closed"] = (CF.preset("C4"), S(A.PU_STREAM_UNIFORM_HOTSPOT, 1024, seed=34, quantum=40, num_quanta=2,
                                         max_requests=30000), {"replay": "closed"})
    # full-size runs at the presets, stored as digests (requests regenerate from
    # the stream spec; delays by sha256, completion cycles and report in full)
    c["big_c4_quantum"] = (CF.preset("C4"), S(A.PU_STREAM_UNIFORM_HOTSPOT, 1024, seed=4, num_quanta=1),
                           {"digest": True})
    c["big_c4_closed"] = (CF.preset("C4"), S(A.PU_STREAM_UNIFORM_HOTSPOT, 1024, seed=404, num_quanta=1),
                          {"digest": True, "replay": "closed"})
    c["big_c3"] = (CF.preset("C3"), S(A.PU_STREAM_MULTIPROGRAM, 256, seed=303, num_quanta=1, num_progs=4),
                   {"digest": True})
    # open loop: a queue delay wraps the reference's int at request 165,860 (halt)
    c["big_c5_preset"] = (CF.preset("C5"), S(A.PU_STREAM_PRODUCER_CONSUMER, 4096, seed=505, num_quanta=1),
                          {"digest": True})
    c["big_c5_closed"] = (CF.preset("C5"), S(A.PU_STREAM_PRODUCER_CONSUMER, 4096, seed=505, num_quanta=1),
                          {"digest": True, "replay": "closed"})
    return c


def cfg_dict(cfg: A.SimCfg) -> dict:
    def conv(o):
        if isinstance(o, (A.CacheCfg, A.NetCfg, A.SysCfg, A.SimCfg)):
            # the reference's XmlSys has no <dram> (an engine-only option): not part of the fixture
            return {k: conv(getattr(o, k)) for k, _ in o._fields_ if not k.startswith("_") and k != "dram"}
        if hasattr(o, "__len__") and not isinstance(o, (str, bytes)):
            return [conv(x) for x in o]
        return o
    return conv(cfg)


def sha256(a: np.ndarray) -> str:
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).view(np.uint8).tobytes()).hexdigest()


def gen_case(name: str, sim: dict, spec: P.StreamSpec, opts: dict | None = None) -> None:
    opts = opts or {}
    mode = O.MODE_CLOSED if opts.get("replay") == "closed" else 0
    xml = CF.to_xml(sim)
    with tempfile.NamedTemporaryFile("w", suffix=".xml", delete=False) as f:
        f.write(xml)
        path = f.name
    reqs = P.generate_stream(spec)
    threads = P.stream_threads(spec)
    # screen with the CPU restatement first: states the reference treats as
    # undefined (e.g. Q13's NULL dereference) would crash the generator
    pre = O.CpuRef(P.load_config(path))
    pre.set_mode(mode)
    for prog, th in threads:
        pre.alloc_core(prog, th)
    pre.run(reqs)
    if pre.stats().error_flags & ~A.PU_ERRF_NEG_DELAY:
        raise SystemExit(f"{name}: stream reaches a reference-undefined state (flags {pre.stats().error_flags})")
    pre.close()
    ref = O.RefUncore(path)
    ref.set_mode(mode)
    for prog, th in threads:
        ref.alloc_core(prog, th)
    delays, rc = ref.run(reqs)
    halt_index = rc - 1 if rc > 0 else None   # prime.cpp:130-134 stopped the handler here
    comp = ref.completion()
    report = ref.report()
    counters = ref.counters()
    parsed = cfg_dict(ref.cfg)
    ref.close()
    os.unlink(path)
    meta = {
        "name": name,
        "stream": {k: getattr(spec, k) for k in ("kind", "num_cores", "seed", "quantum", "num_quanta", "max_msg",
                                                 "num_progs", "max_requests", "write_pct")},
        "threads": threads,
        "counters": counters,
        "halt_index": halt_index,
        "xmlsim": parsed,
        "generator": "tools/gen_golden.py via oracle/_ref/libprime_ref.so (reference src compiled in place)",
        "replay": opts.get("replay", "open"),
        "requests": int(len(reqs)),
    }
    if opts.get("digest"):
        meta["digest"] = {"reqs_sha256": sha256(reqs), "delays_sha256": sha256(delays.astype(np.int32)),
                          "delay_sum": int(delays.astype(np.int64).sum())}
        np.savez_compressed(os.path.join(GOLDEN, f"{name}.npz"), completion=comp, head=delays[:2000],
                            tail=delays[-2000:])
    else:
        np.savez_compressed(os.path.join(GOLDEN, f"{name}.npz"), reqs=reqs.view(np.uint8), delays=delays,
                            completion=comp)
    with open(os.path.join(GOLDEN, f"{name}.xml"), "w") as f:
        f.write(xml)
    with open(os.path.join(GOLDEN, f"{name}.report.txt"), "w") as f:
        f.write(report)
    with open(os.path.join(GOLDEN, f"{name}.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print(f"{name}: {len(reqs)} requests, mean delay {delays.mean():.1f}, counters {counters}", flush=True)


def gen_queue() -> None:
    """Graphite QueueModelHistoryTree call sequences (unit goldens)."""
    rng = np.random.default_rng(2024)
    ts, ps, mins, ds, trial = [], [], [], [], []
    for k in range(16):
        n = 2500
        minp = int([1, 1, 2, 3][k % 4])
        skew = [8, 40, 200, 400][k // 4]
        base = np.cumsum(rng.integers(0, 3, n)).astype(np.uint64)
        t = base + rng.integers(0, skew, n).astype(np.uint64)
        if k % 3 == 2:     # core-major style: time restarts per block, mostly "old" packets
            t = (np.arange(n) % 250 * 4 + rng.integers(0, 3, n)).astype(np.uint64) + np.uint64(1000 * (k // 3))
        p = rng.integers(1, 13, n).astype(np.uint64)
        d = O.ref_queue(minp, t, p)
        ts.append(t); ps.append(p); ds.append(d)
        mins.append(np.full(n, minp, np.uint64)); trial.append(np.full(n, k, np.int32))
    np.savez_compressed(os.path.join(GOLDEN, "queue_model.npz"), t=np.concatenate(ts), p=np.concatenate(ps),
                        min_proc=np.concatenate(mins), delay=np.concatenate(ds), trial=np.concatenate(trial))
    print("queue_model: 16 trials x 2500 calls")


def gen_network() -> None:
    """Network::transmit sequences + Network::report text (unit goldens)."""
    import ctypes as C
    L = O.ref_lib()
    rng = np.random.default_rng(7)
    out = {}
    for name, nodes, net_type, dw, hf, rd, ld, inj in [("mesh4x4", 16, 0, 10, 3, 0, 1, 1),
                                                       ("mesh8x8_r1", 64, 0, 16, 2, 1, 2, 3),
                                                       ("mesh3d_4", 64, 1, 10, 3, 0, 1, 1),
                                                       ("mesh_ns_12", 12, 0, 10, 3, 1, 1, 0)]:
        n = 3000
        src = rng.integers(0, nodes, n).astype(np.int32)
        dst = rng.integers(0, nodes, n).astype(np.int32)
        ln = rng.choice(np.array([0, 64, 8, 100], np.int32), n).astype(np.int32)
        timer = np.cumsum(rng.integers(0, 4, n)).astype(np.uint64) + rng.integers(0, 60, n).astype(np.uint64)
        delay = np.zeros(n, np.uint64)
        fd, tmp = tempfile.mkstemp()
        os.close(fd)
        buf = C.create_string_buffer(4096)
        L.ref_network_run(nodes, net_type, dw, hf, rd, ld, inj, src.ctypes.data, dst.ctypes.data, ln.ctypes.data,
                          timer.ctypes.data, n, delay.ctypes.data, tmp.encode(), buf, 4096)
        out[name] = dict(nodes=nodes, net_type=net_type, data_width=dw, header_flits=hf, router_delay=rd,
                         link_delay=ld, inject_delay=inj, report=buf.value.decode())
        np.savez_compressed(os.path.join(GOLDEN, f"net_{name}.npz"), src=src, dst=dst, len=ln, timer=timer,
                            delay=delay)
    with open(os.path.join(GOLDEN, "network.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("network: 4 meshes x 3000 transmits")


def gen_configs() -> None:
    """Reference XmlParser results for schema fixtures (incl. config_prime's default)."""
    out = {}
    variants = {
        "config_prime_default": CF.default_config(),
        "c3": CF.preset("C3"),
        "no_optional": CF.preset("C1"),
    }
    for k in ("max_num_sharers",):
        del variants["no_optional"]["system"][k]
    for k in ("net_type", "inject_delay"):
        del variants["no_optional"]["system"]["network"][k]
    for name, sim in variants.items():
        xml = CF.to_xml(sim)
        with tempfile.NamedTemporaryFile("w", suffix=".xml", delete=False) as f:
            f.write(xml)
            path = f.name
        r = O.RefUncore(path)
        out[name] = {"xml": xml, "xmlsim": cfg_dict(r.cfg)}
        r.close()
        os.unlink(path)
    with open(os.path.join(GOLDEN, "configs.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("configs:", list(out))


def main() -> None:
    if not O.ref_available():
        sys.exit("oracle/_ref/libprime_ref.so missing: run `make -C oracle ref` (needs /root/reference)")
    os.makedirs(GOLDEN, exist_ok=True)
    only = set(sys.argv[1:])
    for name, case in cases().items():
        big = len(case) > 2 and case[2].get("digest")
        if (not only and not big) or name in only or (big and "big" in only):
            gen_case(name, *case)
    if not only or "queue" in only:
        gen_queue()
    if not only or "network" in only:
        gen_network()
    if not only or "configs" in only:
        gen_configs()


if __name__ == "__main__":
    main()
