"""Resident mode (engine.hip resident_body, primeuncore.h pu_set_resident):
uncore_access and short host batches served by one persistent latency-mode
workgroup through a host mailbox, without a launch per call.

* every golden replayed request by request through pu_access (prime.cpp:129's
  call, the running delay and the closed-loop shift applied by the caller as
  prime.cpp / core_manager.cpp do), and message by message through
  pu_access_batch (the engine's own message loop: halts, closed loop): every
  delay, the completion cycles, the counters and the report equal the
  reference's — with the queue headers kept in the kernel's LDS across calls;
* the kernel is really resident (one launch serves many calls), steps aside
  for a long batch and for another replica, leaves when idle and comes back,
  and every result stays the reference's.
"""
import time

import numpy as np
import pytest

import primesim_amd as P
from primesim_amd import _abi as A
from primesim_amd import config as CF
from golden_util import Case, assert_stats_match, case_names

pytestmark = pytest.mark.gpu


def _engine(c: Case) -> P.UncoreManager:
    um = P.UncoreManager()
    um.init(P.load_config(c.xml_path), replicas=1)
    for prog, th in c.threads:
        um.allocCore(prog, th)
    return um


def _check_end_state(um, c: Case, upto: int):
    np.testing.assert_array_equal(um.completion(), c.completion)
    st = um.stats().as_dict()
    assert st["requests"] == upto
    assert_stats_match(st, c)
    assert um.report() == c.report


@pytest.mark.parametrize("name", case_names())
def test_uncore_access_per_request_matches_reference(name):
    """prime.cpp's loop around uncore_access, one call per request."""
    c = Case(name)
    um = _engine(c)
    try:
        info0 = um.resident_info()
        halt = c.meta.get("halt_index")
        n = len(c.reqs) if halt is None else halt + 1
        got = np.zeros(n, np.int32)
        shift = {}                       # closed loop: core_manager.cpp:265, cycle += delay per reply
        D, msg_shift = 0, 0
        for i in range(n):
            q = c.reqs[i]
            core = int(q["core"])
            if q["batch_start"]:
                D = 0
                msg_shift = shift.get(core, 0) if c.closed else 0
            t = int(q["timer"]) + msg_shift + D
            d = um.uncore_access(core, P.InsMem(int(q["mem_type"]), int(q["prog_id"]), int(q["addr"])), t)
            got[i] = d
            D = (D + d - 1 + 2**31) % 2**32 - 2**31          # prime.cpp's int
            if c.closed:
                shift[core] = msg_shift + D
        np.testing.assert_array_equal(got, c.delays[:n])
        info = um.resident_info()
        if info["eligible"]:
            # one kernel served (nearly) every call: launches only at the start and after idle gaps
            assert info["commands"] - info0["commands"] == n
            assert info["launches"] < max(4, n // 100)
        _check_end_state(um, c, n)
    finally:
        um.close()


@pytest.mark.parametrize("name", case_names())
def test_access_batch_per_message_matches_reference(name):
    """prime.cpp's MEM_REQUESTS handling: one short batch per message."""
    c = Case(name)
    um = _engine(c)
    try:
        if c.closed:
            um.set_replay_mode(P.uncore.PU_REPLAY_CLOSED)
        starts = np.flatnonzero(c.reqs["batch_start"]).tolist() + [len(c.reqs)]
        if starts[0] != 0:
            starts = [0] + starts
        d = np.concatenate([um.access_batch(c.reqs[a:b]) for a, b in zip(starts, starts[1:])])
        c.check_delays(d)
        halt = c.meta.get("halt_index")
        _check_end_state(um, c, len(c.reqs) if halt is None else halt + 1)
        st = um.stats().as_dict()
        assert st["error_flags"] == (0 if halt is None else A.PU_ERRF_NEG_DELAY)
    finally:
        um.close()


def _c2(n, seed=41):
    cfg = P.config_from_dict(CF.preset("C2"))
    spec = P.StreamSpec(A.PU_STREAM_SHARED_UNIFORM, 64, seed=seed, num_quanta=4, max_requests=n)
    reqs = P.generate_stream(spec)
    import oracle as O
    ref = O.CpuRef(cfg)
    for prog, th in P.stream_threads(spec):
        ref.alloc_core(prog, th)
    want, rc = ref.run(reqs)
    assert rc == 0
    return cfg, spec, reqs, want


def test_resident_steps_aside_for_launches_and_comes_back(monkeypatch):
    """Short batches (resident), a long batch (a latency launch: the resident
    kernel is joined and its headers go back to HBM first), short batches
    again, and an idle gap long enough for the kernel to leave by itself:
    the delays equal the restatement's throughout."""
    monkeypatch.setenv("PRIMEUNCORE_RESIDENT_IDLE_MS", "5")
    cfg, spec, reqs, want = _c2(60_000)
    um = P.UncoreManager()
    um.init(cfg, replicas=1)
    try:
        for prog, th in P.stream_threads(spec):
            um.allocCore(prog, th)
        if not um.resident_info()["eligible"]:
            pytest.skip("resident mode unavailable for this configuration")
        bs = np.flatnonzero(reqs["batch_start"]).tolist() + [len(reqs)]
        msgs = list(zip(bs, bs[1:]))
        k1 = next(k for k, (a, b) in enumerate(msgs) if a >= 3000)
        k2 = next(k for k, (a, b) in enumerate(msgs) if a >= 40_000)
        got = [um.access_batch(reqs[a:b]) for a, b in msgs[:k1]]
        assert um.resident_info()["running"]
        got.append(um.access_batch(reqs[msgs[k1][0]:msgs[k2][0]]))   # > 16,384 requests: a launch
        assert not um.resident_info()["running"]
        l0 = um.resident_info()["launches"]
        for k, (a, b) in enumerate(msgs[k2:]):
            got.append(um.access_batch(reqs[a:b]))
            if k == 3:
                time.sleep(0.05)                               # 10x the idle time: the kernel leaves
                assert not um.resident_info()["running"]
        np.testing.assert_array_equal(np.concatenate(got), want)
        assert um.resident_info()["launches"] >= l0 + 2       # back after the launch, and after the idle gap
    finally:
        um.close()


def test_resident_follows_the_replica_and_can_be_turned_off():
    """Two replicas alternating message by message: the kernel moves with the
    replica (its headers back to HBM, the other's in); with the mode off every
    call launches.  Each replica's delays equal the restatement's."""
    cfg, spec, reqs, want = _c2(8_000, seed=42)
    um = P.UncoreManager()
    um.init(cfg, replicas=2)
    try:
        for prog, th in P.stream_threads(spec):
            um.allocCore(prog, th)
        bs = np.flatnonzero(reqs["batch_start"]).tolist() + [len(reqs)]
        out = {0: [], 1: []}
        for k, (a, b) in enumerate(zip(bs, bs[1:])):
            if k == len(bs) // 3:
                assert um.set_resident(0) == 1
            if k == 2 * len(bs) // 3:
                assert um.set_resident(1) == 0
            for r in (0, 1):
                d = np.zeros(b - a, np.int32)
                rc = P.uncore.lib().pu_access_batch(um._handle(), r, reqs[a:b].ctypes.data, b - a, d.ctypes.data)
                assert rc == 0, P.uncore.last_error()
                out[r].append(d)
        for r in (0, 1):
            np.testing.assert_array_equal(np.concatenate(out[r]), want, err_msg=f"replica {r}")
            assert um.stats(r).requests == len(reqs)
    finally:
        um.close()


def test_engine_limit_reaches_uncore_access(monkeypatch):
    """A one-request call is answered by the fast word only when it raised no
    error bit: with a sharer pool of 2 entries, the uncore_access that runs
    the pool dry raises (PU_ESTATE through the full answer), and every delay
    before it is the reference's."""
    c = Case("c4_allcores")
    monkeypatch.setenv("PRIMEUNCORE_POOL_ENTRIES", "2")
    um = P.UncoreManager()
    um.init(P.load_config(c.xml_path), replicas=1)
    monkeypatch.delenv("PRIMEUNCORE_POOL_ENTRIES")
    try:
        for prog, th in c.threads:
            um.allocCore(prog, th)
        D, got, failed_at = 0, [], None
        for i, q in enumerate(c.reqs):
            if q["batch_start"]:
                D = 0
            try:
                d = um.uncore_access(int(q["core"]), P.InsMem(int(q["mem_type"]), int(q["prog_id"]), int(q["addr"])),
                                     int(q["timer"]) + D)
            except P.UncoreError as e:
                assert "pool" in str(e)
                failed_at = i
                break
            got.append(d)
            D = (D + d - 1 + 2**31) % 2**32 - 2**31
        assert failed_at is not None
        np.testing.assert_array_equal(np.array(got, np.int32), c.delays[:failed_at])
        info = um.resident_info()
        assert info["fast_answers"] >= failed_at - 1 if info["eligible"] else True
        assert um.error_flags(1)[0] & A.PU_ERRF_POOL
    finally:
        um.close()
