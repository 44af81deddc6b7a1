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


def test_any_prog_id_runs_exactly():
    """Directory lines hold the whole int prog_id (InsMem::prog_id): large and
    mixed program ids run exactly (the 0.1 engine packed 10 bits and stopped)."""
    cfg = P.config_from_dict(CF.preset("C1"))
    spec = P.StreamSpec(A.PU_STREAM_UNIFORM_HOTSPOT, 16, seed=23, max_requests=600)
    reqs = P.generate_stream(spec)
    hi = reqs.copy()
    hi["prog_id"] = np.where(np.arange(len(hi)) % 3 == 0, 2**31 - 1, 1024 + (np.arange(len(hi)) % 5))
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
