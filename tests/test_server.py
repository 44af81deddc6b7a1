"""Server front-end protocol on the CPU.

The server's handler rules (prime.cpp:55-137), framing, MPI-style tag matching,
sessions, rounds and the negative-delay stop are host logic; here they run
with a host executor in place of the engine (the GPU tests in
test_gpu_server.py drive the same protocol into the HIP engine).  One test uses
the CPU restatement oracle as the executor, as the checker of an end-to-end
replay of a golden case, against the reference's own per-request delays.
"""
from __future__ import annotations

import os
import tempfile
import time

import numpy as np
import pytest

import oracle as O
import primesim_amd as P
from primesim_amd import UncoreError
from primesim_amd import server as S
from primesim_amd.uncore import MSG_BARRIER, MSG_PROCESS_FINISHING, MSG_PROCESS_STARTING
from tests.golden_util import Case


def _sock(tmp_path) -> str:
    # AF_UNIX paths are limited to 107 bytes: keep them short
    d = tempfile.mkdtemp(prefix="pus", dir="/tmp")
    return os.path.join(d, "s")


def _fake_delay(reqs: np.ndarray) -> np.ndarray:
    return (2 + (reqs["addr"] % 13) + reqs["core"] + 3 * reqs["mem_type"]).astype(np.int32)


def _batches(reqs):
    starts = np.nonzero(reqs["batch_start"])[0].tolist() + [len(reqs)]
    return [reqs[a:b] for a, b in zip(starts[:-1], starts[1:])]


def test_replies_follow_prime_handler(tmp_path):
    spec = P.StreamSpec(kind=P._abi.PU_STREAM_UNIFORM_HOTSPOT, num_cores=16, seed=3, num_quanta=1, max_requests=3000)
    reqs = P.generate_stream(spec)
    threads = P.stream_threads(spec)
    seen = []

    def ex(session, r):
        seen.append(r.copy())
        return _fake_delay(r)

    path = _sock(tmp_path)
    srv = S.PrimeServer.with_executor(ex, num_cores=16, socket_path=path)
    srv.start()
    drv = S.CoreManagerDriver(path, 0, threads)
    drv.start()
    # NEW_THREAD replies: core % num_recv_threads (1 thread -> 0), prime.cpp:105
    assert set(drv.tag_of.values()) == {0}
    got = drv.run(reqs)
    left = drv.finish()
    assert srv.join(10) == 0
    drv.close()
    want = [int((_fake_delay(b) - 1).sum()) for b in _batches(reqs)]
    assert got.tolist() == want
    assert left == [0]
    # the executor saw the stream's requests exactly, core ids resolved by getCoreId
    allr = np.concatenate(seen)
    for f in ("addr", "timer", "core", "prog_id", "mem_type", "batch_start"):
        assert np.array_equal(allr[f], reqs[f]), f
    st = srv.stats()
    assert st["sessions_ended"] == 1 and st["requests"] == len(reqs)
    srv.close()


def test_pipelined_messages_share_one_launch(tmp_path):
    spec = P.StreamSpec(kind=P._abi.PU_STREAM_SHARED_UNIFORM, num_cores=8, seed=5, num_quanta=1, max_requests=800)
    reqs = P.generate_stream(spec)
    threads = P.stream_threads(spec)
    path = _sock(tmp_path)
    srv = S.PrimeServer.with_executor(lambda s, r: _fake_delay(r), num_cores=8, socket_path=path)
    c = S.Client(path, 0, threads[0][0])
    c.control(MSG_PROCESS_STARTING)
    for p, t in threads:
        c.control(P.uncore.MSG_NEW_THREAD, mem_size=t)
    bs = _batches(reqs)
    for b in bs:                                 # every message sent before any reply is read
        c.send(S.mem_message(threads[int(b[0]["core"])][1], b))
    total = 1 + len(threads) + len(bs)
    while srv.stats()["messages"] < total:       # manual rounds: each takes all that arrived
        srv.round(200)
    assert srv.stats()["launches"] < len(bs)     # several messages per launch
    srv.start()                                  # serve the receives
    assert [c.recv(t) for _, t in threads] == [0] * len(threads)
    got = [c.recv(threads[int(b[0]["core"])][1]) for b in bs]
    # same-tag replies come back in message order
    assert got == [int((_fake_delay(b) - 1).sum()) for b in bs]
    c.close()
    srv.close()


def _wait_messages(srv, n):
    t0 = time.time()
    while srv.stats()["messages"] < n:
        assert time.time() - t0 < 10
        time.sleep(0.005)


def test_barriers_and_process_list(tmp_path):
    path = _sock(tmp_path)
    srv = S.PrimeServer.with_executor(lambda s, r: _fake_delay(r), num_cores=4, socket_path=path)
    srv.start()
    a, b = S.Client(path, 0, 1), S.Client(path, 0, 2)
    a.control(MSG_PROCESS_STARTING)
    b.control(MSG_PROCESS_STARTING)
    _wait_messages(srv, 2)                        # connections race like MPI sources do
    a.control(MSG_BARRIER)
    b.control(MSG_BARRIER)                        # second arrival releases both (prime.cpp:78-88)
    assert a.recv(0) == 2 and b.recv(0) == 2
    a.control(MSG_PROCESS_FINISHING)              # prime.cpp:63-76: reply = programs left
    assert a.recv(0) == 1
    b.control(MSG_BARRIER)                        # one program left: releases at once
    assert b.recv(0) == 1
    b.control(MSG_PROCESS_FINISHING)
    assert b.recv(0) == 0
    a.close()
    b.close()
    srv.close()


def test_negative_delay_stops_the_session(tmp_path):
    path = _sock(tmp_path)
    # every request costs 0 cycles: D = -1 after the first (prime.cpp:129-134)
    srv = S.PrimeServer.with_executor(lambda s, r: np.zeros(len(r), np.int32), num_cores=4, socket_path=path)
    srv.start()
    c = S.Client(path, 0, 1)
    c.control(MSG_PROCESS_STARTING)
    c.control(P.uncore.MSG_NEW_THREAD, mem_size=0)
    assert c.recv(0) == 0
    r = np.zeros(3, P._abi.REQ_DTYPE)
    r["addr"] = [64, 128, 192]
    r["timer"] = [1, 2, 3]
    c.send(S.mem_message(0, r))
    with pytest.raises(UncoreError):
        c.recv(0)                                 # no reply: the handler stopped
    assert srv.join(10) == 0
    st = srv.stats()
    assert st["sessions_halted"] == 1 and st["sessions_ended"] == 1
    c.close()
    srv.close()


def test_sessions_are_independent(tmp_path):
    path = _sock(tmp_path)
    calls = []

    def ex(session, r):
        calls.append((session, len(r)))
        return np.full(len(r), 10 + session, np.int32)

    srv = S.PrimeServer.with_executor(ex, num_cores=2, socket_path=path, sessions=2)
    srv.start()
    cs = [S.Client(path, s, 1) for s in range(2)]
    for c in cs:
        c.control(MSG_PROCESS_STARTING)
        c.control(P.uncore.MSG_NEW_THREAD, mem_size=0)
        c.control(P.uncore.MSG_NEW_THREAD, mem_size=1)
    # each session has its own ThreadSched: both get cores 0 and 1
    assert [(c.recv(0), c.recv(1)) for c in cs] == [(0, 0), (0, 0)]
    r = np.zeros(4, P._abi.REQ_DTYPE)
    r["timer"] = np.arange(4)
    for c in cs:
        c.send(S.mem_message(1, r))
    assert [c.recv(1) for c in cs] == [4 * 9, 4 * 10]
    for c in cs:
        c.control(MSG_PROCESS_FINISHING)
        assert c.recv(0) == 0
        c.control(P.uncore.MSG_PROGRAM_EXITING)
    assert srv.join(10) == 0
    assert {s for s, _ in calls} == {0, 1}
    for c in cs:
        c.close()
    srv.close()


def test_bad_clients_are_rejected(tmp_path):
    path = _sock(tmp_path)
    srv = S.PrimeServer.with_executor(lambda s, r: _fake_delay(r), num_cores=2, socket_path=path)
    bad = S.Client(path, 5, 1)                    # session out of range: dropped
    srv.start()
    with pytest.raises(UncoreError):
        bad.recv(0)
    bad.close()
    srv.close()
    with pytest.raises(UncoreError):
        S.Client(path, 0, 1)                      # nobody listening


def test_golden_replay_through_server_with_oracle_executor(tmp_path):
    """End-to-end protocol check: the CPU oracle (test infrastructure) as the
    executor reproduces the reference's per-message delays of a golden case."""
    case = Case("c3_multiprog")
    cfg = P.load_config(case.xml_path)
    ref = O.CpuRef(cfg)
    for p, t in case.threads:
        ref.alloc_core(p, t)

    def ex(session, r):
        d, rc = ref.run(r)
        assert rc == 0
        return d

    path = _sock(tmp_path)
    srv = S.PrimeServer.with_executor(ex, num_cores=cfg.sys.num_cores, socket_path=path)
    srv.start()
    drv = S.CoreManagerDriver(path, 0, case.threads)
    drv.start()
    got = drv.run(case.reqs)
    drv.finish()
    assert srv.join(30) == 0
    drv.close()
    srv.close()
    starts = np.nonzero(case.reqs["batch_start"])[0].tolist() + [len(case.reqs)]
    want = [int((case.delays[a:b].astype(np.int64) - 1).sum()) for a, b in zip(starts[:-1], starts[1:])]
    assert got.tolist() == want


def _msg_reqs(core: int, n: int, base: int, timer0: int = 0) -> np.ndarray:
    r = np.zeros(n, P._abi.REQ_DTYPE)
    r["addr"] = base + 64 * np.arange(n)
    r["timer"] = timer0 + np.arange(n)
    r["core"] = core
    r["batch_start"][0] = 1
    return r


def test_negative_delay_stops_only_its_receive_thread(tmp_path):
    """num_recv_threads = 2: a negative batch delay ends handler thread `tag`
    only (prime.cpp:130-134 returns from msgHandler); the other thread keeps
    serving, later messages on the dead tag are never received, and the session
    ends once PROGRAM_EXITING has reached the surviving thread."""
    seen = []
    KILL = 0x7000

    def ex(session, r):
        seen.append(r.copy())
        d = np.full(len(r), 5, np.int32)
        d[r["addr"] == KILL] = -1000          # the running delay goes negative here
        return d

    path = _sock(tmp_path)
    srv = S.PrimeServer.with_executor(ex, num_cores=4, socket_path=path, recv_threads=2)
    srv.start()
    c = S.Client(path, 0, 1)
    c.control(P.uncore.MSG_PROCESS_STARTING)
    tags = {}
    for t in range(2):
        c.control(P.uncore.MSG_NEW_THREAD, mem_size=t, tag=0)
        tags[t] = c.recv(t)
    assert tags == {0: 0, 1: 1}                               # core % num_recv_threads
    # thread 1's message goes negative at its 3rd request: no reply, rest skipped
    bad = _msg_reqs(1, 6, 0x6F80)
    assert (bad["addr"] == KILL).sum() == 1
    c.send(S.mem_message(1, bad), tag=1)
    # thread 0 is still served
    ok = _msg_reqs(0, 4, 0x100000)
    c.send(S.mem_message(0, ok), tag=0)
    assert c.recv(0) == 4 * (5 - 1)
    # a later message on the dead tag is never received by anyone
    late = _msg_reqs(1, 3, 0x200000)
    c.send(S.mem_message(1, late), tag=1)
    ok2 = _msg_reqs(0, 2, 0x300000)
    c.send(S.mem_message(0, ok2), tag=0)
    assert c.recv(0) == 2 * (5 - 1)
    c.control(P.uncore.MSG_PROGRAM_EXITING, tag=0)
    assert srv.join(10) == 0
    st = srv.stats()
    assert st["sessions_halted"] == 1 and st["sessions_ended"] == 1 and st["sessions_failed"] == 0
    executed = np.concatenate(seen)
    assert not np.isin(late["addr"], executed["addr"]).any()
    c.close()
    srv.close()


def test_engine_limit_ends_session_without_reply(tmp_path):
    """An engine-side limit (PU_ERRF_LIMITS, e.g. the sharer pool) means no
    exact reply exists: the session ends with an error instead of replying."""
    def ex(session, r):
        d = np.full(len(r), 3, np.int32)
        return (d, P._abi.PU_ERRF_POOL) if (r["addr"] == 0xBAD0).any() else d

    path = _sock(tmp_path)
    srv = S.PrimeServer.with_executor(ex, num_cores=2, socket_path=path)
    srv.start()
    c = S.Client(path, 0, 1)
    c.control(P.uncore.MSG_PROCESS_STARTING)
    c.control(P.uncore.MSG_NEW_THREAD, mem_size=0, tag=0)
    assert c.recv(0) == 0
    c.send(S.mem_message(0, _msg_reqs(0, 3, 0x1000)), tag=0)
    assert c.recv(0) == 3 * 2
    c.send(S.mem_message(0, _msg_reqs(0, 3, 0xBAD0 - 64)), tag=0)
    with pytest.raises(UncoreError):
        c.recv(0)                                             # EOF: no reply for a wrong delay
    assert srv.join(10) == 0
    st = srv.stats()
    assert st["sessions_failed"] == 1 and st["sessions_ended"] == 1
    c.close()
    srv.close()


def test_out_of_range_tag_is_never_received(tmp_path):
    """prime.cpp:53: handler thread k receives tag k only (k < num_recv_threads).
    A PROGRAM_EXITING (or any message) on another tag is dropped: it does not end
    the session, and the session still serves its real thread afterwards."""
    path = _sock(tmp_path)
    srv = S.PrimeServer.with_executor(lambda s, r: _fake_delay(r), num_cores=2, socket_path=path, recv_threads=1)
    srv.start()
    c = S.Client(path, 0, 1)
    c.control(MSG_PROCESS_STARTING)
    c.control(P.uncore.MSG_NEW_THREAD, mem_size=0)
    assert c.recv(0) == 0
    c.control(P.uncore.MSG_PROGRAM_EXITING, tag=5)          # no receive thread 5
    c.control(P.uncore.MSG_PROGRAM_EXITING, tag=64)         # would alias thread 0 in a 64-bit mask
    r = np.zeros(3, P._abi.REQ_DTYPE)
    r["timer"] = np.arange(3)
    c.send(S.mem_message(0, r), tag=0)
    assert c.recv(0) == int((_fake_delay(r) - 1).sum())    # the session is still live
    assert srv.stats()["sessions_ended"] == 0
    c.control(MSG_PROCESS_FINISHING)
    assert c.recv(0) == 0
    c.control(P.uncore.MSG_PROGRAM_EXITING, tag=0)
    assert srv.join(10) == 0
    assert srv.stats()["sessions_ended"] == 1
    c.close()
    srv.close()
