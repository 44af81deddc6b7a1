"""Replay modes of the CPU restatement against the reference's own System.

* closed loop (timer_i += the core's earlier batch delays, core_manager.cpp:265)
  is pinned by the c*_closed / big_*_closed goldens (test_oracle_golden.py);
* per-message stop (a caller of uncore_access without prime.cpp's exit, or one
  receive thread of several): c4_overflow_halt continued past the request
  whose delay wraps the reference's int, against the reference compiled in place.
"""
import numpy as np
import pytest

import oracle as O
import primesim_amd as P
from golden_util import Case, extended_stream


@pytest.mark.skipif(not O.ref_available(), reason="reference not built here")
def test_msghalt_matches_reference_past_the_overflow():
    """One receive thread of several (the server's PU_KF_MSGHALT): the message
    whose delay wraps the int is abandoned at that request, its receive thread
    (tag) never receives again, and the other thread's next message starts over
    with D = 0 from the System the abandoned message left."""
    c = Case("c4_overflow_halt")
    halt = c.meta["halt_index"]
    ref = O.RefUncore(c.xml_path)
    ref.set_mode(O.MODE_MSGHALT)
    cpu = O.CpuRef(P.load_config(c.xml_path))
    cpu.set_mode(O.MODE_MSGHALT)
    for prog, th in c.threads:
        ref.alloc_core(prog, th)
        cpu.alloc_core(prog, th)
    reqs = extended_stream(c, 36_000)
    reqs["tag"] = reqs["core"] % 2                     # two receive threads: tag = core % 2 (prime.cpp:105)
    want, rc = ref.run(reqs)
    assert rc == 0
    got, rc2 = cpu.run(reqs)
    assert rc2 == 0
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(want[:halt + 1], c.delays[:halt + 1])
    nxt = int(np.nonzero(reqs["batch_start"][halt + 1:])[0][0]) + halt + 1
    assert (want[halt + 1:nxt] == 0).all()             # the rest of that message is never run
    dead = int(reqs["tag"][halt])
    later = reqs[nxt:]
    assert (want[nxt:][later["tag"] == dead] == 0).all()   # its receive thread never receives again
    assert (want[nxt:][later["tag"] != dead] != 0).all()   # the other thread's messages are run


@pytest.mark.skipif(not O.ref_available(), reason="reference not built here")
def test_msgskip_matches_reference_past_the_overflow():
    """A caller of uncore_access that abandons a message whose running delay
    wraps the int and goes on receiving (MODE_MSGSKIP): the next message starts
    over with D = 0, on every tag."""
    c = Case("c4_overflow_halt")
    halt = c.meta["halt_index"]
    ref = O.RefUncore(c.xml_path)
    ref.set_mode(O.MODE_MSGSKIP)
    cpu = O.CpuRef(P.load_config(c.xml_path))
    cpu.set_mode(O.MODE_MSGSKIP)
    for prog, th in c.threads:
        ref.alloc_core(prog, th)
        cpu.alloc_core(prog, th)
    reqs = extended_stream(c, 36_000)
    want, rc = ref.run(reqs)
    got, rc2 = cpu.run(reqs)
    assert rc == rc2 == 0
    np.testing.assert_array_equal(got, want)
    nxt = int(np.nonzero(reqs["batch_start"][halt + 1:])[0][0]) + halt + 1
    assert (want[halt + 1:nxt] == 0).all()             # the rest of that message is never run
    assert (want[nxt:] != 0).all()                     # later messages are, on the same tag


def test_closed_loop_shifts_later_messages_only():
    """Closed loop leaves each core's first message untouched and shifts the
    later ones by that core's summed batch delays (host logic of the oracle)."""
    c = Case("c1_hot")
    cfg = P.load_config(c.xml_path)
    a, b = O.CpuRef(cfg), O.CpuRef(cfg)
    b.set_mode(O.MODE_CLOSED)
    for prog, th in c.threads:
        a.alloc_core(prog, th)
        b.alloc_core(prog, th)
    reqs = c.reqs
    first_msg_end = np.nonzero(reqs["batch_start"])[0][1]
    da, _ = a.run(reqs[:first_msg_end])
    db, _ = b.run(reqs[:first_msg_end])
    np.testing.assert_array_equal(da, db)
    da2, _ = a.run(reqs[first_msg_end:])
    db2, _ = b.run(reqs[first_msg_end:])
    assert not np.array_equal(da2, db2)


@pytest.mark.skipif(not O.ref_available(), reason="reference not built here")
def test_large_prog_ids_match_reference():
    """InsMem::prog_id is an int: the restatement (and the engine, which holds
    the whole id in its directory lines) follows the reference for ids far
    beyond 10 bits, mixed within one directory set."""
    c = Case("c2_canneal")
    reqs = c.reqs.copy()
    i = np.arange(len(reqs))
    reqs["prog_id"] = np.where(i % 3 == 0, 2**31 - 1, 1024 + (i % 5))
    ref = O.RefUncore(c.xml_path)
    cpu = O.CpuRef(P.load_config(c.xml_path))
    for prog, th in c.threads:
        ref.alloc_core(prog, th)
        cpu.alloc_core(prog, th)
    want, rc = ref.run(reqs)
    got, rc2 = cpu.run(reqs)
    assert rc == rc2 == 0
    np.testing.assert_array_equal(got, want)
    assert not np.array_equal(want, c.delays)          # the ids change hits (cache.cpp:193)
