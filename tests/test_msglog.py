"""MsgMem message logs: the uncore's receive stream
recorded in the reference's MsgMem layout (common.h:49-59) and replayed with
prime.cpp:55-137's handler semantics."""
import os

import numpy as np
import pytest

import oracle as O
import primesim_amd as P
from primesim_amd import _abi as A
from primesim_amd import uncore as U
from golden_util import Case

FIELDS = ("addr", "timer", "core", "prog_id", "mem_type", "batch_start")


def _same_requests(a, b):
    assert len(a) == len(b)
    for f in FIELDS:
        np.testing.assert_array_equal(a[f], b[f], err_msg=f)


@pytest.mark.parametrize("name", ["c1_stream", "c2_canneal", "c3_multiprog", "small_msgs", "tlb_c1"])
def test_log_round_trip_of_golden_streams(tmp_path, name):
    """stream -> log (NEW_THREAD per thread, one MEM_REQUESTS message per batch) -> replay == stream."""
    c = Case(name)
    s = c.meta["stream"]
    spec = P.StreamSpec(s["kind"], s["num_cores"], s["seed"], s["quantum"], s["num_quanta"], s["max_msg"],
                        s["num_progs"], s["max_requests"], s["write_pct"])
    path = str(tmp_path / "run.msglog")
    P.msglog_from_stream(path, c.reqs, spec)
    got = P.msglog_read(path, num_cores=s["num_cores"])
    _same_requests(got, c.reqs)
    nmsg = int(c.reqs["batch_start"].sum()) + s["num_cores"]
    assert os.path.getsize(path) == 16 + 8 * nmsg + 24 * (nmsg + len(c.reqs))


def test_replay_through_oracle_matches_reference(tmp_path):
    """A replayed log drives the CPU restatement to the reference's golden delays."""
    c = Case("c2_canneal")
    s = c.meta["stream"]
    spec = P.StreamSpec(s["kind"], s["num_cores"], s["seed"], s["quantum"], s["num_quanta"], s["max_msg"],
                        s["num_progs"], s["max_requests"], s["write_pct"])
    path = str(tmp_path / "c2.msglog")
    P.msglog_from_stream(path, c.reqs, spec)
    reqs = P.msglog_read(path, num_cores=s["num_cores"])
    ref = O.CpuRef(P.load_config(c.xml_path))
    for prog, th in c.threads:
        ref.alloc_core(prog, th)
    d, rc = ref.run(reqs)
    assert rc == 0
    np.testing.assert_array_equal(d, c.delays)


def _rec(n):
    return np.zeros(n, dtype=U.MSGMEM_DTYPE)


def _ctl(kind, thread=0):
    r = _rec(1)
    r["timer"] = kind
    r["mem_size"] = thread
    return r


def _mem(thread, items):
    r = _rec(len(items) + 1)
    r["mem_size"][0] = thread
    r["addr_dmem"][0] = len(items) + 1
    for i, (addr, timer, wr) in enumerate(items, 1):
        r["addr_dmem"][i] = addr
        r["timer"][i] = timer
        r["mem_type"][i] = 1 if wr else 0
    return r


def test_handler_semantics(tmp_path):
    """Control messages: process/barrier messages are no-ops, NEW_THREAD allocates
    the first free core, THREAD_FINISHING frees it only when core_stat == 1
    (thread_sched.cpp:55-91), PROGRAM_EXITING ends the log, addr_dmem of a
    message header bounds its requests (prime.cpp:121-127)."""
    path = str(tmp_path / "ctl.msglog")
    w = P.MsgLogWriter(path)
    w.append(1, _ctl(U.MSG_PROCESS_STARTING))
    w.append(1, _ctl(U.MSG_NEW_THREAD, 0))        # (1,0) -> core 0
    w.append(2, _ctl(U.MSG_NEW_THREAD, 0))        # (2,0) -> core 1
    w.append(1, _ctl(U.MSG_NEW_THREAD, 1))        # (1,1) -> core 2
    w.append(1, _mem(1, [(0x1000, 5, False), (0x2000, 6, True)]))
    w.append(2, _ctl(U.MSG_BARRIER))
    w.append(1, _ctl(U.MSG_THREAD_FINISHING, 0))  # core 0: core_stat == 1 -> freed
    w.append(2, _ctl(U.MSG_THREAD_FINISHING, 0))  # core 1: core_stat == 2 -> stays busy
    w.append(3, _ctl(U.MSG_NEW_THREAD, 7))        # (3,7) -> core 0 (first free)
    w.append(3, _mem(7, [(0x3000, 9, False)]))
    w.append(2, _mem(0, [(0x4000, 11, True)]))    # (2,0) still core 1
    short = _mem(1, [(0x5000, 12, False), (0x6000, 13, False)])
    short["addr_dmem"][0] = 2                      # header says 1 request
    w.append(1, short)
    w.append(1, _ctl(U.MSG_PROCESS_FINISHING))
    w.append(0, _ctl(U.MSG_PROGRAM_EXITING))
    w.append(1, _mem(1, [(0x7000, 20, False)]))   # after PROGRAM_EXITING: not replayed
    w.close()
    got = P.msglog_read(path, num_cores=4)
    assert list(got["addr"]) == [0x1000, 0x2000, 0x3000, 0x4000, 0x5000]
    assert list(got["core"]) == [2, 2, 0, 1, 2]
    assert list(got["prog_id"]) == [1, 1, 3, 2, 1]
    assert list(got["mem_type"]) == [A.PU_RD, A.PU_WR, A.PU_RD, A.PU_WR, A.PU_RD]
    assert list(got["batch_start"]) == [1, 0, 1, 1, 1]
    assert list(got["timer"]) == [5, 6, 9, 11, 12]


def test_out_of_cores_and_bad_files(tmp_path):
    path = str(tmp_path / "full.msglog")
    w = P.MsgLogWriter(path)
    w.append(1, _ctl(U.MSG_NEW_THREAD, 0))
    w.append(1, _ctl(U.MSG_NEW_THREAD, 1))
    w.close()
    with pytest.raises(P.UncoreError, match="Not enough cores"):
        P.msglog_read(path, num_cores=1)
    bad = tmp_path / "bad.msglog"
    bad.write_bytes(b"NOTALOG!" + bytes(8))
    with pytest.raises(P.UncoreError, match="PRIMEMSG"):
        P.msglog_read(str(bad), num_cores=1)
    trunc = tmp_path / "trunc.msglog"
    trunc.write_bytes(open(path, "rb").read()[:-5])
    with pytest.raises(P.UncoreError, match="truncated"):
        P.msglog_read(str(trunc), num_cores=4)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c1_hot", "three_level", "bus_l2_shared"])
def test_engine_replays_log_bit_exactly(tmp_path, name):
    """The engine's ThreadSched resolves the log's threads; delays, completion
    cycles and the report equal the reference's."""
    c = Case(name)
    s = c.meta["stream"]
    spec = P.StreamSpec(s["kind"], s["num_cores"], s["seed"], s["quantum"], s["num_quanta"], s["max_msg"],
                        s["num_progs"], s["max_requests"], s["write_pct"])
    path = str(tmp_path / "g.msglog")
    P.msglog_from_stream(path, c.reqs, spec)
    um = P.UncoreManager()
    um.init(P.load_config(c.xml_path), replicas=1)
    try:
        reqs = P.msglog_read(path, um=um)
        _same_requests(reqs, c.reqs)
        d = um.access_batch(reqs)
        np.testing.assert_array_equal(d, c.delays)
        np.testing.assert_array_equal(um.completion(), c.completion)
        assert um.report() == c.report
    finally:
        um.close()
