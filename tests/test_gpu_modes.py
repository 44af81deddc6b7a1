"""Replay modes, the single-request path and engine-limit errors on the GPU.

* closed-loop replay on the device path (many replicas, time-sliced) against
  the CPU restatement (itself pinned to the reference by the *_closed goldens);
* UncoreManager::uncore_access has no prime.cpp halt: a lone-access replay of
  c4_overflow_halt continues past the request whose delay wraps the int,
  against the CPU restatement in no-halt mode (pinned to the reference in
  test_modes_oracle.py);
* an engine limit (a tiny sharer pool) makes the host batch path fail with
  PU_ESTATE instead of returning delays that are no longer the reference's;
* the server's per-receive-thread stop (PU_KF_MSGHALT) on the engine.
"""
import os
import tempfile
import time

import numpy as np
import pytest

import oracle as O
import primesim_amd as P
from primesim_amd import _abi as A
from primesim_amd import server as S
from golden_util import Case, extended_stream

pytestmark = pytest.mark.gpu


def _alloc(objs, threads):
    for prog, th in threads:
        for o in objs:
            o.allocCore(prog, th) if hasattr(o, "allocCore") else o.alloc_core(prog, th)


def test_closed_loop_device_path_many_replicas():
    import torch
    cfg = P.config_from_dict(P.config.preset("C1"))
    R = 6
    specs = [P.StreamSpec(kind=A.PU_STREAM_UNIFORM_HOTSPOT, num_cores=16, seed=100 + r, num_quanta=3) for r in range(R)]
    streams = [P.generate_stream(s) for s in specs]
    off = np.zeros(R + 1, np.uint64)
    off[1:] = np.cumsum([len(s) for s in streams])
    allr = np.concatenate(streams)
    um = P.UncoreManager()
    um.init(cfg, replicas=R)
    um.set_replay_mode(P.uncore.PU_REPLAY_CLOSED)
    _alloc([um], P.stream_threads(specs[0]))
    dev = torch.device("cuda:0")
    d_reqs = torch.from_numpy(allr.view(np.uint8)).to(dev)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    d_pos = d_off[:-1].clone()
    d_delay = torch.zeros(len(allr), dtype=torch.int32, device=dev)
    for _ in range(200):                       # 2 ms slices: replicas stop and resume mid-message
        um.run_device_sliced(d_reqs.data_ptr(), d_off.data_ptr(), d_delay.data_ptr(), d_pos.data_ptr(), 2000)
        um.synchronize()
        if bool((d_pos == d_off[1:]).all()):
            break
    assert bool((d_pos == d_off[1:]).all())
    got = d_delay.cpu().numpy()
    for r in range(R):
        ref = O.CpuRef(cfg)
        ref.set_mode(O.MODE_CLOSED)
        for prog, th in P.stream_threads(specs[r]):
            ref.alloc_core(prog, th)
        want, rc = ref.run(streams[r])
        assert rc == 0
        np.testing.assert_array_equal(got[off[r]:off[r + 1]], want, err_msg=f"replica {r}")
        np.testing.assert_array_equal(um.completion(r), ref.completion())
    um.close()


def test_uncore_access_does_not_halt():
    """uncore_access is System::access: no halt.  The caller runs prime.cpp's
    loop itself and, instead of exiting at the wrapped delay, abandons that
    message and continues with the next one (CpuRef MODE_MSGSKIP, pinned to the
    reference in test_modes_oracle.py)."""
    c = Case("c4_overflow_halt")
    halt = c.meta["halt_index"]
    cfg = P.load_config(c.xml_path)
    reqs = extended_stream(c, 36_000)
    cpu = O.CpuRef(cfg)
    cpu.set_mode(O.MODE_MSGSKIP)
    um = P.UncoreManager()
    um.init(cfg, replicas=1)
    for prog, th in c.threads:
        cpu.alloc_core(prog, th)
        um.allocCore(prog, th)
    want, rc = cpu.run(reqs)
    assert rc == 0
    starts = np.nonzero(reqs["batch_start"])[0]
    a = int(starts[starts <= halt][-2])                # two messages before the wrap
    np.testing.assert_array_equal(um.access_batch(reqs[:a]), want[:a])
    b = min(len(reqs), int(starts[starts > halt][0]) + 400)
    got = np.zeros(b - a, np.int32)
    D, skip = 0, False
    for i in range(a, b):                              # prime.cpp:120-137 on the host
        q = reqs[i]
        if q["batch_start"]:
            D, skip = 0, False
        if skip:
            continue
        ins = P.InsMem(mem_type=int(q["mem_type"]), prog_id=int(q["prog_id"]), addr_dmem=int(q["addr"]))
        d = um.uncore_access(int(q["core"]), ins, int(q["timer"]) + D)
        got[i - a] = d
        D += d - 1
        skip = D < 0
    np.testing.assert_array_equal(got, want[a:b])
    assert (got < 0).any()
    assert um.stats().error_flags & A.PU_ERRF_LIMITS == 0
    um.close()


def test_engine_limit_is_an_error(monkeypatch):
    """A sharer pool of 2 entries: the 3rd line with more than 4 sharers (the
    hotspot lines of a 1024-core run) stops the replica (PU_ERRF_POOL) and
    access_batch raises instead of returning."""
    c = Case("c4_allcores")
    monkeypatch.setenv("PRIMEUNCORE_POOL_ENTRIES", "2")
    um = P.UncoreManager()
    um.init(P.load_config(c.xml_path), replicas=1)
    monkeypatch.delenv("PRIMEUNCORE_POOL_ENTRIES")
    for prog, th in c.threads:
        um.allocCore(prog, th)
    with pytest.raises(P.UncoreError, match="pool"):
        um.access_batch(c.reqs)
    assert um.error_flags(1)[0] & A.PU_ERRF_POOL
    um.close()


def test_server_stops_one_receive_thread_on_the_engine():
    """Two receive threads on the engine: the message that wraps the int
    (c4_overflow_halt) stops its thread; the other thread's next message is
    answered with the delay of the reference's continued System (the CPU
    restatement: halted prefix, then that message)."""
    c = Case("c4_overflow_halt")
    halt = c.meta["halt_index"]
    sim_cfg = P.load_config(c.xml_path)
    sim_cfg.num_recv_threads = 2
    reqs = extended_stream(c, 36_000)
    reqs["tag"] = reqs["core"] % 2                                       # the oracle's receive threads
    starts = np.nonzero(reqs["batch_start"])[0].tolist() + [len(reqs)]
    k = max(i for i, s in enumerate(starts[:-1]) if s <= halt)          # the overflowing message
    bad_core = int(reqs[starts[k]]["core"])
    # a later message whose core is on the other receive thread
    j = next(i for i in range(k + 1, len(starts) - 1) if int(reqs[starts[i]]["core"]) % 2 != bad_core % 2)
    um = P.UncoreManager()
    um.init(sim_cfg, replicas=1)
    path = os.path.join(tempfile.mkdtemp(prefix="pus", dir="/tmp"), "s")
    srv = S.PrimeServer(um, path)
    srv.start()
    drv = S.CoreManagerDriver(path, 0, c.threads, recv_threads=2)
    drv.start()
    ref = O.CpuRef(sim_cfg)
    ref.set_mode(O.MODE_MSGHALT)
    for prog, th in c.threads:
        ref.alloc_core(prog, th)
    got = drv.run(reqs[:starts[k]])
    want_d, _ = ref.run(reqs[:starts[k]])
    want = [int((want_d[a:b] - 1).sum()) for a, b in zip(starts[:k], starts[1:k + 1])]
    assert got.tolist() == want
    # the overflowing message: no reply ever comes (its thread returned)
    p, t = c.threads[bad_core]
    cl = drv.clients[p]
    cl.send(S.mem_message(t, reqs[starts[k]:starts[k + 1]]), tag=drv.tag_of[(p, t)])
    ref.run(reqs[starts[k]:starts[k + 1]])
    # the other thread's message is served, from the state after the abandoned message
    jc = int(reqs[starts[j]]["core"])
    p2, t2 = c.threads[jc]
    drv.clients[p2].send(S.mem_message(t2, reqs[starts[j]:starts[j + 1]]), tag=drv.tag_of[(p2, t2)])
    got_j = drv.clients[p2].recv(t2)
    dj, _ = ref.run(reqs[starts[j]:starts[j + 1]])
    assert got_j == int((dj - 1).sum())
    cl.control(P.uncore.MSG_PROGRAM_EXITING, tag=(bad_core % 2) ^ 1)   # the surviving thread returns too
    assert srv.join(30) == 0
    st = srv.stats()
    assert st["sessions_halted"] == 1 and st["sessions_failed"] == 0
    drv.close()
    srv.close()
    um.close()


def test_dead_receive_thread_skips_its_later_message_in_the_same_launch():
    """Two receive threads; the overflowing message k, a later message on the
    SAME thread and one on the other thread are pipelined into one server round
    (one engine launch, PU_KF_MSGHALT).  The engine abandons k, never runs the
    dead thread's later message (its handler returned, prime.cpp:133) and answers
    the other thread from the System k left: all as the CPU restatement's
    MSGHALT mode with the per-thread dead mask (pinned to the reference by
    test_modes_oracle.py) replays the same three messages."""
    c = Case("c4_overflow_halt")
    halt = c.meta["halt_index"]
    sim_cfg = P.load_config(c.xml_path)
    sim_cfg.num_recv_threads = 2
    reqs = extended_stream(c, 36_000)
    reqs["tag"] = reqs["core"] % 2
    starts = np.nonzero(reqs["batch_start"])[0].tolist() + [len(reqs)]
    k = max(i for i, st in enumerate(starts[:-1]) if st <= halt)
    bad = int(reqs[starts[k]]["core"]) % 2
    k2 = next(i for i in range(k + 1, len(starts) - 1) if int(reqs[starts[i]]["core"]) % 2 == bad)
    j = next(i for i in range(k + 1, len(starts) - 1) if int(reqs[starts[i]]["core"]) % 2 != bad)
    msgs = [reqs[starts[m]:starts[m + 1]] for m in (k, k2, j)]
    um = P.UncoreManager()
    um.init(sim_cfg, replicas=1)
    path = os.path.join(tempfile.mkdtemp(prefix="pus", dir="/tmp"), "s")
    srv = S.PrimeServer(um, path)
    srv.start()
    drv = S.CoreManagerDriver(path, 0, c.threads, recv_threads=2)
    drv.start()
    ref = O.CpuRef(sim_cfg)
    ref.set_mode(O.MODE_MSGHALT)
    for prog, th in c.threads:
        ref.alloc_core(prog, th)
    got = drv.run(reqs[:starts[k]])
    want_d, _ = ref.run(reqs[:starts[k]])
    assert got.tolist() == [int((want_d[a:b] - 1).sum()) for a, b in zip(starts[:k], starts[1:k + 1])]
    srv.stop()
    srv.join(30)
    # the three messages are all in the server's backlog before its next round
    for m in msgs:
        p, t = c.threads[int(m[0]["core"])]
        drv.clients[p].send(S.mem_message(t, m), tag=drv.tag_of[(p, t)])
    time.sleep(0.5)                                                   # all three have arrived
    n0, m0 = srv.stats()["launches"], srv.stats()["messages"]
    srv.round(2000)
    assert srv.stats()["messages"] == m0 + 3
    assert srv.stats()["launches"] == n0 + 1                          # one launch for all three
    srv.start()
    pj, tj = c.threads[int(msgs[2][0]["core"])]
    got_j = drv.clients[pj].recv(tj)
    d3, _ = ref.run(np.concatenate(msgs))
    na, nb = len(msgs[0]), len(msgs[1])
    assert (d3[halt - starts[k] + 1:na + nb] == 0).all()              # k's rest and k2 never run
    assert got_j == int((d3[na + nb:] - 1).sum())
    pb, tb = c.threads[int(msgs[0][0]["core"])]
    drv.clients[pb].control(P.uncore.MSG_PROGRAM_EXITING, tag=bad ^ 1)
    assert srv.join(30) == 0
    st = srv.stats()
    assert st["sessions_halted"] == 1 and st["sessions_failed"] == 0
    drv.close()
    srv.close()
    um.close()
