"""The CPU restatement (oracle/cpu_ref.cpp) against the reference's own outputs.

Pins the oracle before it is trusted as the GPU checker: every golden case
(tests/golden, made by tools/gen_golden.py from the reference compiled in
place) must be reproduced bit-exactly — per-request delays, per-core
completion cycles, every number System::report prints and the -Wl,--wrap
counters (link visits/flits, M/G/1 calls, share/inval visits, bus, DRAM).
"""
import numpy as np
import pytest

import oracle as O
import primesim_amd as P
from primesim_amd import _abi as A
from golden_util import Case, assert_stats_match, big_case_names, case_names


@pytest.mark.parametrize("name", case_names() + big_case_names())
def test_oracle_reproduces_reference(name):
    c = Case(name)
    cfg = P.load_config(c.xml_path)
    ref = O.CpuRef(cfg)
    ref.set_mode(O.MODE_CLOSED if c.closed else 0)
    for prog, th in c.threads:
        ref.alloc_core(prog, th)
    d, rc = ref.run(c.reqs)
    halt = c.meta.get("halt_index")
    assert rc == (0 if halt is None else halt + 1)
    c.check_delays(d)
    np.testing.assert_array_equal(ref.completion(), c.completion)
    st = ref.stats().as_dict()
    assert st["error_flags"] == (0 if halt is None else A.PU_ERRF_NEG_DELAY)
    assert_stats_match(st, c)


@pytest.mark.parametrize("name", ["c1_hot", "small_msgs", "l2_shared_bus"])
def test_oracle_chunked_equals_single(name):
    """The open message's running delay carries across run() calls."""
    c = Case(name)
    cfg = P.load_config(c.xml_path)
    ref = O.CpuRef(cfg)
    for prog, th in c.threads:
        ref.alloc_core(prog, th)
    cuts = [0, 37, 1001, 1002, 4999, len(c.reqs)]
    parts = [ref.run(c.reqs[a:b])[0] for a, b in zip(cuts, cuts[1:])]
    np.testing.assert_array_equal(np.concatenate(parts), c.delays)
