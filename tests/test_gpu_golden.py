"""HIP engine vs the reference's own outputs, bit-exact, through the C ABI.

Every golden case (tests/golden, from the reference compiled in place):
per-request delays, per-core completion cycles, the full UncoreManager::report
text (minus the wall-clock line) byte for byte, every counter, no error flags.
"""
import numpy as np
import pytest

import primesim_amd as P
from primesim_amd import _abi as A
from golden_util import Case, assert_stats_match, case_names

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", case_names())
def test_engine_reproduces_reference(name):
    c = Case(name)
    um = P.UncoreManager()
    um.init(P.load_config(c.xml_path), replicas=1)
    try:
        for prog, th in c.threads:
            um.allocCore(prog, th)
        d = um.access_batch(c.reqs)
        np.testing.assert_array_equal(d, c.delays)
        np.testing.assert_array_equal(um.completion(), c.completion)
        st = um.stats().as_dict()
        halt = c.meta.get("halt_index")
        assert st["error_flags"] == (0 if halt is None else A.PU_ERRF_NEG_DELAY)
        assert st["requests"] == (len(c.reqs) if halt is None else halt + 1)
        assert_stats_match(st, c)
        assert um.report() == c.report
    finally:
        um.close()
