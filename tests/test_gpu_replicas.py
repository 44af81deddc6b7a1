"""Replica engine paths at larger sizes, checked against the CPU restatement
(itself pinned to the reference by test_oracle_golden):

* many replicas in one launch from device-resident buffers (the bench path),
  split over several launches (state and the open message carry across);
* the full 1024-core C4 configuration with every core active;
* the single-request uncore_access compatibility path, reset, empty and
  out-of-range requests.
"""
import numpy as np
import pytest
import torch

import oracle as O
import primesim_amd as P
from primesim_amd import _abi as A
from primesim_amd import config as CF

pytestmark = pytest.mark.gpu


def _oracle_run(cfg, spec, reqs):
    ref = O.CpuRef(cfg)
    for prog, th in P.stream_threads(spec):
        ref.alloc_core(prog, th)
    d, rc = ref.run(reqs)
    assert rc == 0
    return d, ref


def _device_run(um, streams, cuts):
    """Run every replica's stream through run_device, split at `cuts`."""
    R = len(streams)
    dev = torch.device("cuda", 0)
    outs = [[] for _ in range(R)]
    s = torch.cuda.Stream(dev)
    for a, b in zip(cuts, cuts[1:]):
        chunk = np.concatenate([st[a:b] for st in streams])
        off = np.array([sum(len(st[a:b]) for st in streams[:r]) for r in range(R + 1)], dtype=np.uint64)
        d_reqs = torch.from_numpy(chunk.view(np.uint8).copy()).to(dev)
        d_off = torch.from_numpy(off.view(np.int64)).to(dev)
        d_del = torch.zeros(len(chunk), dtype=torch.int32, device=dev)
        um.run_device(d_reqs.data_ptr(), d_off.data_ptr(), d_del.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize(dev)
        host = d_del.cpu().numpy()
        for r in range(R):
            outs[r].append(host[int(off[r]):int(off[r + 1])])
    return [np.concatenate(o) for o in outs]


@pytest.mark.parametrize("preset,kind,cores", [("C2", A.PU_STREAM_SHARED_UNIFORM, 64),
                                               ("C3", A.PU_STREAM_MULTIPROGRAM, 256)])
def test_many_replicas_device_path(preset, kind, cores):
    cfg = P.config_from_dict(CF.preset(preset))
    R = 12
    specs = [P.StreamSpec(kind, cores, seed=100 + r, num_progs=4 if preset == "C3" else 1, max_requests=3000)
             for r in range(R)]
    streams = [P.generate_stream(s) for s in specs]
    um = P.UncoreManager()
    um.init(cfg, replicas=R)
    try:
        for prog, th in P.stream_threads(specs[0]):
            um.allocCore(prog, th)
        got = _device_run(um, streams, [0, 777, 1500, 3000])
        for r in (0, 5, R - 1):
            want, ref = _oracle_run(cfg, specs[r], streams[r])
            np.testing.assert_array_equal(got[r], want, err_msg=f"replica {r}")
            gs, ws = um.stats(r).as_dict(), ref.stats().as_dict()
            assert {k: gs[k] for k in ws if k != "requests"} == {k: ws[k] for k in ws if k != "requests"}
            np.testing.assert_array_equal(um.completion(r), ref.completion())
        for r in range(R):
            assert um.stats(r).error_flags == 0
            assert um.stats(r).requests == 3000
    finally:
        um.close()


def test_c4_full_size_all_cores():
    """1024-core 32x32 mesh, 1,984 links, every core issuing (20-cycle quantum)."""
    cfg = P.config_from_dict(CF.preset("C4"))
    R = 4
    specs = [P.StreamSpec(A.PU_STREAM_UNIFORM_HOTSPOT, 1024, seed=40 + r, quantum=20, num_quanta=3,
                          max_requests=24000) for r in range(R)]
    streams = [P.generate_stream(s) for s in specs]
    um = P.UncoreManager()
    um.init(cfg, replicas=R)
    try:
        for prog, th in P.stream_threads(specs[0]):
            um.allocCore(prog, th)
        got = _device_run(um, streams, [0, 8000, 24000])
        for r in range(R):
            want, ref = _oracle_run(cfg, specs[r], streams[r])
            np.testing.assert_array_equal(got[r], want, err_msg=f"replica {r}")
            assert um.stats(r).net_distance == ref.stats().net_distance
    finally:
        um.close()


def test_single_request_path_and_reset():
    cfg = P.config_from_dict(CF.preset("C1"))
    spec = P.StreamSpec(A.PU_STREAM_UNIFORM_HOTSPOT, 16, seed=21, max_requests=150)
    reqs = P.generate_stream(spec).copy()
    reqs["batch_start"] = 1            # uncore_access: each call stands alone
    want, _ = _oracle_run(cfg, spec, reqs)
    um = P.UncoreManager()
    um.init(cfg)
    try:
        for prog, th in P.stream_threads(spec):
            um.allocCore(prog, th)
        got = [um.uncore_access(int(q["core"]), P.InsMem(int(q["mem_type"]), int(q["prog_id"]), int(q["addr"])),
                                int(q["timer"])) for q in reqs]
        np.testing.assert_array_equal(np.array(got, np.int32), want)
        um.reset()
        np.testing.assert_array_equal(um.access_batch(reqs), want)
        assert um.access_batch(reqs[:0]).size == 0
    finally:
        um.close()


def test_core_out_of_range():
    cfg = P.config_from_dict(CF.preset("C1"))
    spec = P.StreamSpec(A.PU_STREAM_UNIFORM_HOTSPOT, 16, seed=22, max_requests=400)
    reqs = P.generate_stream(spec)
    bad = reqs.copy()
    bad["core"][10] = 16                 # System::access returns -1 (system.cpp:147)
    um = P.UncoreManager()
    um.init(cfg)
    try:
        d = um.access_batch(bad)
        want, ref = _oracle_run(cfg, spec, bad)
        assert d[10] == -1
        np.testing.assert_array_equal(d, want)
        assert um.stats().error_flags & A.PU_ERRF_CORE_RANGE
        assert um.uncore_access(99, P.InsMem(0, 1, 0x1000), 5) == -1
    finally:
        um.close()


@pytest.mark.parametrize("ids", ["large", "escape_edges", "negative"])
def test_any_prog_id_runs_exactly(ids):
    """Directory lines keep the whole int prog_id (InsMem::prog_id): ids
    outside the inline 10-bit field [0, 1023) escape to a side array; large,
    negative and mixed ids around the escape edge run exactly (the 0.1 engine
    packed 10 bits and stopped)."""
    cfg = P.config_from_dict(CF.preset("C1"))
    spec = P.StreamSpec(A.PU_STREAM_UNIFORM_HOTSPOT, 16, seed=23, max_requests=600)
    reqs = P.generate_stream(spec)
    hi = reqs.copy()
    k = np.arange(len(hi))
    if ids == "large":
        hi["prog_id"] = np.where(k % 3 == 0, 2**31 - 1, 1024 + (k % 5))
    elif ids == "escape_edges":
        hi["prog_id"] = np.array([510, 511, 1022, 1023, 0, 2**31 - 1])[k % 6]
    else:
        hi["prog_id"] = np.where(k % 2 == 0, -1, -(2**31))
    um = P.UncoreManager()
    um.init(cfg)
    try:
        want, _ = _oracle_run(cfg, spec, hi)
        np.testing.assert_array_equal(um.access_batch(hi), want)
        assert um.stats().error_flags == 0
    finally:
        um.close()


def test_thread_sched_mirror():
    um = P.UncoreManager()
    um.init(P.config_from_dict(CF.preset("C1")))
    try:
        assert [um.allocCore(1, t) for t in range(3)] == [0, 1, 2]
        assert um.getCoreId(1, 2) == 2
        assert um.deallocCore(1, 1) == 1          # frees: core_stat == prog 1
        assert um.allocCore(7, 0) == 1
        assert um.deallocCore(7, 0) == 0          # core_stat == 7 != 1: not freed (thread_sched.cpp:81)
    finally:
        um.close()


def test_time_sliced_runs_continue_streams_exactly():
    """pu_run_device_sliced: replicas stop between requests when their slice
    runs out and continue from d_pos in the next launch; the concatenated
    delays, counters and completion cycles equal the CPU restatement's."""
    cfg = P.config_from_dict(CF.preset("C2"))
    R, n = 10, 4000
    specs = [P.StreamSpec(A.PU_STREAM_SHARED_UNIFORM, 64, seed=300 + r, max_requests=n) for r in range(R)]
    streams = [P.generate_stream(s) for s in specs]
    dev = torch.device("cuda", 0)
    um = P.UncoreManager()
    um.init(cfg, replicas=R)
    try:
        for prog, th in P.stream_threads(specs[0]):
            um.allocCore(prog, th)
        host = np.concatenate(streams)
        off = (np.arange(R + 1, dtype=np.uint64) * np.uint64(n))
        d_reqs = torch.from_numpy(host.view(np.uint8).copy()).to(dev)
        d_off = torch.from_numpy(off.view(np.int64)).to(dev)
        d_pos = torch.from_numpy(off[:-1].copy().view(np.int64)).to(dev)
        d_del = torch.full((R * n,), -7, dtype=torch.int32, device=dev)
        s = torch.cuda.Stream(dev)
        launches = 0
        while True:
            um.run_device_sliced(d_reqs.data_ptr(), d_off.data_ptr(), d_del.data_ptr(), d_pos.data_ptr(), 300,
                                 s.cuda_stream)
            torch.cuda.synchronize(dev)
            launches += 1
            pos = d_pos.cpu().numpy().view(np.uint64)
            assert np.all(pos >= off[:-1]) and np.all(pos <= off[1:])
            if np.array_equal(pos, off[1:]):
                break
            assert launches < 10000
        assert launches > 2, "a 300-us slice should not cover 4000 requests"
        got = d_del.cpu().numpy().reshape(R, n)
        for r in (0, 3, R - 1):
            want, ref = _oracle_run(cfg, specs[r], streams[r])
            np.testing.assert_array_equal(got[r], want, err_msg=f"replica {r}")
            gs, ws = um.stats(r).as_dict(), ref.stats().as_dict()
            assert {k: gs[k] for k in ws if k != "requests"} == {k: ws[k] for k in ws if k != "requests"}
            np.testing.assert_array_equal(um.completion(r), ref.completion())
        for r in range(R):
            assert um.stats(r).requests == n
    finally:
        um.close()


def test_c4_replicas_past_4gib_on_the_bench_kernel():
    """The headline's launch shape: C4 with more replicas than CUs, so the
    launch is a throughput one (time-sliced kernel, headers in HBM) and the
    replica-layout offsets of the last replicas lie past 4 GiB (17 MiB each;
    the compiled configuration passes them as opaque scalars).  Replicas 0,
    R/2, R-1 and a spread between are checked against the CPU restatement:
    every delay, counter and completion cycle."""
    cfg = P.config_from_dict(CF.preset("C4"))
    R, n = 320, 2500
    specs = [P.StreamSpec(A.PU_STREAM_UNIFORM_HOTSPOT, 1024, seed=4 + r, num_quanta=64, max_requests=n)
             for r in range(R)]
    ss = P.StreamSet(specs)
    host = np.zeros((R, n), dtype=A.REQ_DTYPE)
    assert ss.next_into(host) == n
    ss.close()
    dev = torch.device("cuda", 0)
    um = P.UncoreManager()
    um.init(cfg, replicas=R)
    try:
        assert um.replica_bytes * (R - 1) > 4 << 30
        for prog, th in P.stream_threads(specs[0]):
            um.allocCore(prog, th)
        off = np.arange(R + 1, dtype=np.uint64) * np.uint64(n)
        d_reqs = torch.from_numpy(host.reshape(-1).view(np.uint8).copy()).to(dev)
        d_off = torch.from_numpy(off.view(np.int64)).to(dev)
        d_pos = torch.from_numpy(off[:-1].copy().view(np.int64)).to(dev)
        d_del = torch.full((R * n,), -7, dtype=torch.int32, device=dev)
        s = torch.cuda.Stream(dev)
        for launch in range(1000):
            um.run_device_sliced(d_reqs.data_ptr(), d_off.data_ptr(), d_del.data_ptr(), d_pos.data_ptr(), 20000,
                                 s.cuda_stream)
            torch.cuda.synchronize(dev)
            if np.array_equal(d_pos.cpu().numpy().view(np.uint64), off[1:]):
                break
        else:
            raise AssertionError("replicas did not finish in 1000 slices")
        got = d_del.cpu().numpy().reshape(R, n)
        for r in (0, 1, 100, R // 2, 241, 255, 256, 300, R - 2, R - 1):
            want, ref = _oracle_run(cfg, specs[r], host[r])
            np.testing.assert_array_equal(got[r], want, err_msg=f"replica {r}")
            gs, ws = um.stats(r).as_dict(), ref.stats().as_dict()
            assert {k: gs[k] for k in ws if k != "requests"} == {k: ws[k] for k in ws if k != "requests"}, r
            np.testing.assert_array_equal(um.completion(r), ref.completion())
        assert all(um.stats(r).error_flags == 0 for r in range(R))
    finally:
        um.close()


def test_mg1_helper_on_hot_links():
    """Latency mode on a 4-core 2x2 mesh: every transmit crosses one of four
    links, so the M/G/1 helper wave recomputes the same links' waits while the
    simulating wave keeps rewriting their headers (the helper's
    reads race the main wave's writes).  60,000 requests in one latency-mode
    launch, closed-loop replay (the realistic regime; open loop saturates a
    4-core mesh), against the CPU restatement."""
    from extra_configs import hot_link_config
    cfg = hot_link_config()
    spec = P.StreamSpec(A.PU_STREAM_UNIFORM_HOTSPOT, 4, seed=77, num_quanta=100000, max_requests=60000)
    reqs = P.generate_stream(spec)
    assert len(reqs) == 60000
    um = P.UncoreManager()
    um.init(cfg, replicas=1)
    um.set_replay_mode(P.uncore.PU_REPLAY_CLOSED)
    ref = O.CpuRef(cfg)
    ref.set_mode(O.MODE_CLOSED)
    try:
        for prog, th in P.stream_threads(spec):
            assert um.allocCore(prog, th) == ref.alloc_core(prog, th)
        got = um.access_batch(reqs)            # >= 16,384 requests: headers in LDS + the helper wave
        want, rc = ref.run(reqs)
        np.testing.assert_array_equal(got, want)
        gs, ws = um.stats().as_dict(), ref.stats().as_dict()
        assert gs["mg1_calls"] == ws["mg1_calls"] and gs["net_total_delay"] == ws["net_total_delay"]
        assert gs["mg1_calls"] > 100000          # the M/G/1 branch is exercised
    finally:
        um.close()


def _pool_run(um, host, n_each, slots, budget_us, max_launches=20000):
    """Every replica's stream through pu_run_device_pool with `slots` wavefronts
    until each is done; returns (delays [R, n_each], launches, sched)."""
    R = host.shape[0]
    dev = torch.device("cuda", 0)
    off = np.arange(R + 1, dtype=np.uint64) * np.uint64(n_each)
    d_reqs = torch.from_numpy(host.reshape(-1).view(np.uint8).copy()).to(dev)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    d_pos = torch.from_numpy(off[:-1].copy().view(np.int64)).to(dev)
    d_del = torch.full((R * n_each,), -7, dtype=torch.int32, device=dev)
    d_sched = torch.zeros(um.pool_words(slots), dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(dev)
    for launch in range(1, max_launches + 1):
        um.run_device_pool(d_reqs.data_ptr(), d_off.data_ptr(), d_del.data_ptr(), d_pos.data_ptr(),
                           d_sched.data_ptr(), slots, budget_us, s.cuda_stream)
        torch.cuda.synchronize(dev)
        pos = d_pos.cpu().numpy().view(np.uint64)
        assert np.all(pos >= off[:-1]) and np.all(pos <= off[1:])
        if np.array_equal(pos, off[1:]):
            return d_del.cpu().numpy().reshape(R, n_each), launch, d_sched.cpu().numpy().view(np.uint32)
    raise AssertionError("the pool did not finish")


def test_replica_pool_runs_every_replica_exactly():
    """pu_run_device_pool: 12 replicas on 4 wavefronts, short slices: a
    wavefront whose replica is done takes the next unstarted one; every
    replica's delays, counters and completion cycles equal the CPU
    restatement's (each replica is still processed in order by one wavefront
    at a time, across launches and across wavefronts)."""
    cfg = P.config_from_dict(CF.preset("C2"))
    R, n, slots = 12, 3000, 4
    specs = [P.StreamSpec(A.PU_STREAM_SHARED_UNIFORM, 64, seed=500 + r, max_requests=n) for r in range(R)]
    host = np.stack([P.generate_stream(sp) for sp in specs])
    um = P.UncoreManager()
    um.init(cfg, replicas=R)
    try:
        assert um.pool_slots() == R                      # far fewer than resident: all could run at once
        for prog, th in P.stream_threads(specs[0]):
            um.allocCore(prog, th)
        got, launches, sched = _pool_run(um, host, n, slots, 300)
        assert launches > R // slots, "a 300-us slice should not cover a replica's 3000 requests"
        assert sched[0] >= R and np.all(sched[2:2 + slots] == 0)   # every replica taken, every slot idle
        busy = sched[(3 + slots) & ~1:][:2 * slots].view(np.uint64)   # PU_POOL_BUSY0: 64-bit ticks per slot
        assert np.all(busy > 0) and np.all(busy < (1 << 40))                 # every slot ran; no wrap or garbage
        for r in range(R):
            want, ref = _oracle_run(cfg, specs[r], host[r])
            np.testing.assert_array_equal(got[r], want, err_msg=f"replica {r}")
            gs, ws = um.stats(r).as_dict(), ref.stats().as_dict()
            assert {k: gs[k] for k in ws if k != "requests"} == {k: ws[k] for k in ws if k != "requests"}, r
            np.testing.assert_array_equal(um.completion(r), ref.completion())
            assert um.stats(r).requests == n
    finally:
        um.close()


def test_replica_pool_moves_on_from_a_halted_replica():
    """Three copies of the c4_overflow_halt golden on ONE wavefront: each stops
    at the golden's request by the prime.cpp:130-134 rule, the rest of its
    range reads 0, and the wavefront takes the next copy within the slice."""
    from golden_util import Case
    c = Case("c4_overflow_halt")
    halt = c.meta["halt_index"]
    cfg = P.load_config(c.xml_path)
    R, n = 3, len(c.reqs)
    host = np.stack([c.reqs] * R)
    um = P.UncoreManager()
    um.init(cfg, replicas=R)
    try:
        for prog, th in c.threads:
            um.allocCore(prog, th)
        got, launches, sched = _pool_run(um, host, n, 1, 200000)
        for r in range(R):
            np.testing.assert_array_equal(got[r], c.delays, err_msg=f"replica {r}")
            assert um.stats(r).requests == halt + 1
            assert um.error_flags(R)[r] & A.PU_ERRF_NEG_DELAY
        assert sched[0] >= R
    finally:
        um.close()
