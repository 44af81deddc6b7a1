"""HIP engine vs the reference's own outputs, bit-exact, through the C ABI.

Every golden case (tests/golden, from the reference compiled in place):
per-request delays, per-core completion cycles, the full UncoreManager::report
text (minus the wall-clock line) byte for byte, every counter, no error flags.
"""
import numpy as np
import pytest

import primesim_amd as P
from primesim_amd import _abi as A
from golden_util import Case, assert_stats_match, big_case_names, case_names

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", case_names() + big_case_names())
def test_engine_reproduces_reference(name):
    c = Case(name)
    um = P.UncoreManager()
    um.init(P.load_config(c.xml_path), replicas=1)
    try:
        if c.closed:
            um.set_replay_mode(P.uncore.PU_REPLAY_CLOSED)
        for prog, th in c.threads:
            um.allocCore(prog, th)
        # large runs go in chunks (the open message's delay carries across calls)
        step = 200_000
        d = np.concatenate([um.access_batch(c.reqs[a:a + step]) for a in range(0, len(c.reqs), step)])
        c.check_delays(d)
        np.testing.assert_array_equal(um.completion(), c.completion)
        st = um.stats().as_dict()
        halt = c.meta.get("halt_index")
        assert st["error_flags"] == (0 if halt is None else A.PU_ERRF_NEG_DELAY)
        assert st["requests"] == (len(c.reqs) if halt is None else halt + 1)
        assert_stats_match(st, c)
        assert um.report() == c.report
    finally:
        um.close()


@pytest.mark.parametrize("name", ["c1_hot", "c4_allcores", "three_level", "l2_shared_bus", "c5_prodcons_256",
                                  "c4_closed"])
@pytest.mark.parametrize("mode", ["0", "2"])
def test_engine_header_modes(name, mode, monkeypatch):
    """The same goldens with each queue-header placement forced: "0" keeps the
    headers in HBM for every launch (the throughput kernel's path, which the
    bench runs); "2" uses the latency mode (headers in LDS, launches of at most
    one replica per CU) for short host batches too, which otherwise run with
    the headers in HBM."""
    monkeypatch.setenv("PRIMEUNCORE_LDS_HEADERS", mode)
    test_engine_reproduces_reference(name)

