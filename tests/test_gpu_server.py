"""Server front-end into the HIP engine, bit-exact.

Golden cases replayed as the MPI messages core_manager.cpp would send, through
the Unix-socket server into the engine: every MEM_REQUESTS reply must equal the
reference's batch delay (prime.cpp:129 over the golden per-request delays), and
the report the server writes when the session ends must be the reference's
report byte for byte (minus the wall-clock line).  Also: several sessions in
one launch, the negative-delay stop, and the `prime_server` executable.
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile
import threading
import time

import numpy as np
import pytest

import primesim_amd as P
from primesim_amd import UncoreError
from primesim_amd import server as S
from golden_util import Case

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _sock() -> str:
    return os.path.join(tempfile.mkdtemp(prefix="pug", dir="/tmp"), "s")


def _want(case: Case) -> list[int]:
    starts = np.nonzero(case.reqs["batch_start"])[0].tolist() + [len(case.reqs)]
    return [int((case.delays[a:b].astype(np.int64) - 1).sum()) for a, b in zip(starts[:-1], starts[1:])]


def _strip_time(text: str) -> str:
    return "".join(ln for ln in text.splitlines(keepends=True) if not ln.startswith("Total computation time"))


@pytest.mark.parametrize("name", ["c1_stream", "c3_multiprog", "tlb_c3", "bus_c2", "three_level"])
def test_server_replays_golden(name, tmp_path):
    case = Case(name)
    um = P.UncoreManager()
    um.init(P.load_config(case.xml_path), replicas=1)
    path = _sock()
    prefix = str(tmp_path / "result")
    srv = S.PrimeServer(um, path, sessions=1, report_prefix=prefix)
    try:
        srv.start()
        drv = S.CoreManagerDriver(path, 0, case.threads)
        drv.start()
        got = drv.run(case.reqs)
        drv.finish()
        assert srv.join(60) == 0
        drv.close()
        assert got.tolist() == _want(case)
        with open(prefix + "_0") as f:
            assert _strip_time(f.read()) == case.report
        st = srv.stats()
        assert st["requests"] == len(case.reqs) and st["sessions_ended"] == 1
    finally:
        srv.close()
        um.close()


def test_server_on_a_handle_left_in_closed_mode(tmp_path):
    """A handle switched to closed-loop replay (pu_set_replay_mode) and then
    served: live clients' timers already include their earlier replies'
    delays (core_manager.cpp:265), so the server's launches stay open-loop and
    the replies are the reference's."""
    case = Case("c1_stream")
    um = P.UncoreManager()
    um.init(P.load_config(case.xml_path), replicas=1)
    um.set_replay_mode(P.uncore.PU_REPLAY_CLOSED)
    path = _sock()
    srv = S.PrimeServer(um, path, sessions=1)
    try:
        srv.start()
        drv = S.CoreManagerDriver(path, 0, case.threads)
        drv.start()
        got = drv.run(case.reqs)
        drv.finish()
        assert srv.join(60) == 0
        drv.close()
        assert got.tolist() == _want(case)
    finally:
        srv.close()
        um.close()


def test_sessions_share_launches(tmp_path):
    """Three simulations on three replicas, driven concurrently: each gets the
    reference's replies, and rounds batch them into shared launches."""
    case = Case("c2_canneal")
    um = P.UncoreManager()
    um.init(P.load_config(case.xml_path), replicas=3)
    path = _sock()
    prefix = str(tmp_path / "result")
    srv = S.PrimeServer(um, path, sessions=3, report_prefix=prefix)
    results: dict[int, object] = {}

    def one(s):
        try:
            drv = S.CoreManagerDriver(path, s, case.threads)
            drv.start()
            results[s] = drv.run(case.reqs).tolist()
            drv.finish()
            drv.close()
        except Exception as e:   # noqa: BLE001
            results[s] = e

    try:
        srv.start()
        ts = [threading.Thread(target=one, args=(s,)) for s in range(3)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(120)
        assert srv.join(60) == 0
        want = _want(case)
        for s in range(3):
            assert results[s] == want, s
            with open(f"{prefix}_{s}") as f:
                assert _strip_time(f.read()) == case.report
        st = srv.stats()
        assert st["launches"] < 3 * len(want)
    finally:
        srv.close()
        um.close()


def test_negative_delay_stops_session(tmp_path):
    case = Case("c4_overflow_halt")
    halt = case.meta["halt_index"]
    um = P.UncoreManager()
    um.init(P.load_config(case.xml_path), replicas=1)
    path = _sock()
    srv = S.PrimeServer(um, path, sessions=1, report_prefix=str(tmp_path / "result"))
    try:
        srv.start()
        drv = S.CoreManagerDriver(path, 0, case.threads)
        drv.start()
        starts = np.nonzero(case.reqs["batch_start"])[0]
        k = int(np.searchsorted(starts, halt, side="right"))   # messages up to and including the halting one
        got = drv.run(case.reqs[:starts[k - 1]])
        assert got.tolist() == _want(case)[:k - 1]
        with pytest.raises(UncoreError):
            drv.run(case.reqs[starts[k - 1]:])                  # the halting message gets no reply
        assert srv.join(60) == 0
        assert srv.stats()["sessions_halted"] == 1
        drv.close()
        assert um.stats().as_dict()["requests"] == halt + 1
    finally:
        srv.close()
        um.close()


def test_prime_server_executable(tmp_path):
    """`prime_server config.xml output` in its own process, like `prime`."""
    case = Case("c3_multiprog")
    exe = os.path.join(ROOT, "primesim_amd", "prime_server")
    assert os.path.exists(exe), "build with __graft_entry__.build()"
    path = _sock()
    out = str(tmp_path / "result")
    proc = subprocess.Popen([exe, case.xml_path, out, "--socket", path], stdout=subprocess.PIPE,
                            stderr=subprocess.STDOUT, text=True)
    try:
        for _ in range(600):
            if os.path.exists(path):
                break
            time.sleep(0.1)
        drv = S.CoreManagerDriver(path, 0, case.threads)
        drv.start()
        got = drv.run(case.reqs)
        drv.finish()
        drv.close()
        log, _ = proc.communicate(timeout=60)
        assert proc.returncode == 0, log
        assert got.tolist() == _want(case)
        assert "[PriME] Process 1 begins" in log
        with open(out + "_0") as f:
            assert _strip_time(f.read()) == case.report
    finally:
        if proc.poll() is None:
            proc.kill()
            proc.wait()


def test_engine_limit_mid_round_answers_the_batches_before_it(monkeypatch, tmp_path):
    """A sharer pool of 2 entries runs out inside a round of pipelined messages
    (c4_allcores: hotspot lines gain a fifth sharer).  Every message that ended
    before the request that hit the limit is answered with the reference's
    batch delay (the golden); the message holding it and everything after get
    no reply, and the session ends as failed (limit position in
    RunState)."""
    c = Case("c4_allcores")
    cfg = P.load_config(c.xml_path)
    monkeypatch.setenv("PRIMEUNCORE_POOL_ENTRIES", "2")
    probe = P.UncoreManager()
    probe.init(cfg, replicas=1)
    for prog, th in c.threads:
        probe.allocCore(prog, th)
    with pytest.raises(UncoreError):
        probe.access_batch(c.reqs)
    L = int(probe.limit_positions(1)[0])
    probe.close()
    starts = np.nonzero(c.reqs["batch_start"])[0].tolist() + [len(c.reqs)]
    assert 0 < L < len(c.reqs)
    mL = max(i for i, st in enumerate(starts[:-1]) if st <= L)
    assert mL >= 2
    last = min(mL + 2, len(starts) - 2)
    um = P.UncoreManager()
    um.init(cfg, replicas=1)
    monkeypatch.delenv("PRIMEUNCORE_POOL_ENTRIES")
    path = _sock()
    srv = S.PrimeServer(um, path)
    try:
        srv.start()
        drv = S.CoreManagerDriver(path, 0, c.threads)
        drv.start()
        srv.stop()
        srv.join(30)
        for m in range(last + 1):                                   # one round, one launch
            b = c.reqs[starts[m]:starts[m + 1]]
            p, t = c.threads[int(b[0]["core"])]
            drv.clients[p].send(S.mem_message(t, b), tag=drv.tag_of[(p, t)])
        time.sleep(0.5)
        n0 = srv.stats()["launches"]
        srv.round(2000)
        assert srv.stats()["launches"] == n0 + 1
        srv.start()
        want = _want(c)
        for m in range(mL):
            b = c.reqs[starts[m]]
            p, t = c.threads[int(b["core"])]
            assert drv.clients[p].recv(t) == want[m], m
        b = c.reqs[starts[mL]]
        p, t = c.threads[int(b["core"])]
        with pytest.raises(UncoreError):
            drv.clients[p].recv(t)                                  # EOF: no exact reply exists
        assert srv.join(30) == 0
        st = srv.stats()
        assert st["sessions_failed"] == 1 and st["sessions_ended"] == 1
        drv.close()
    finally:
        srv.close()
        um.close()


def test_served_handle_already_stopped_by_an_engine_limit(monkeypatch, tmp_path):
    """A handle whose replica hit an engine limit before serving started (the
    server never resets it): the replica is halted, so the engine writes 0 for
    every request of every later launch.  The limit bit is sticky but the
    limit position belongs to the earlier launch, so the server sees a limit
    with no position in this launch: it must end the session as failed
    instead of answering those zeros."""
    c = Case("c4_allcores")
    cfg = P.load_config(c.xml_path)
    monkeypatch.setenv("PRIMEUNCORE_POOL_ENTRIES", "2")
    um = P.UncoreManager()
    um.init(cfg, replicas=1)
    monkeypatch.delenv("PRIMEUNCORE_POOL_ENTRIES")
    with pytest.raises(UncoreError):                                # (core ids come resolved in the
        um.access_batch(c.reqs)                                     # requests): the pool runs out
    assert int(um.limit_positions(1)[0]) < len(c.reqs)
    path = _sock()
    srv = S.PrimeServer(um, path)
    try:
        srv.start()
        drv = S.CoreManagerDriver(path, 0, c.threads)
        drv.start()
        starts = np.nonzero(c.reqs["batch_start"])[0].tolist() + [len(c.reqs)]
        b = c.reqs[starts[0]:starts[1]]
        p, t = c.threads[int(b[0]["core"])]
        drv.clients[p].send(S.mem_message(t, b), tag=drv.tag_of[(p, t)])
        with pytest.raises(UncoreError):
            drv.clients[p].recv(t)                                  # EOF: no exact reply exists
        assert srv.join(30) == 0
        st = srv.stats()
        assert st["sessions_failed"] == 1 and st["sessions_ended"] == 1
        drv.close()
    finally:
        srv.close()
        um.close()
