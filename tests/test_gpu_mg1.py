"""M/G/1 arithmetic fuzz on the GPU (queue_model_m_g_1.cpp:16-42).

The engine's mg1_wait divides with a refined reciprocal (v_rcp_f64 + Newton
steps + one residual correction) and without v_div_scale / v_div_fixup
(engine.hip rcp_nr / div_nr): exact for positive normal operands away from
the range limits.  Here it is evaluated on 10^7 seeded queue states
(tests/mg1_states.py: n up to 2^40, newest up to 2^62, variance exactly 0
and +-1 around it, lambda >= mu, lambda just below mu, states whose exact
wait is an integer) by pu_unit_mg1_run, one state per lane, and compared
with the reference's own QueueModelMG1::computeQueueDelay (oracle/_ref,
compiled from the reference sources) on the same states: bit-exact on all.
"""
import numpy as np
import pytest

import oracle as O
from mg1_states import states
from primesim_amd import uncore

pytestmark = pytest.mark.gpu


def _engine_mg1(n, s, q, w):
    out = np.zeros(len(n), dtype=np.uint64)
    rc = uncore.lib().pu_unit_mg1_run(n.ctypes.data, s.ctypes.data, q.ctypes.data, w.ctypes.data, len(n),
                                      out.ctypes.data, 0)
    assert rc == 0, uncore.last_error()
    return out


def test_mg1_fuzz_bit_exact_vs_reference():
    n, s, q, w = states(10_000_000, seed=23)
    want = O.ref_mg1(n, s, q, w) if O.ref_available() else O.cpuref_mg1(n, s, q, w)
    got = _engine_mg1(n, s, q, w)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, (f"{len(bad)} of {len(n)} states differ; first: n={n[bad[0]]} sum={s[bad[0]]!r} "
                           f"sum_sq={q[bad[0]]!r} newest={w[bad[0]]} engine={got[bad[0]]} reference={want[bad[0]]}")
    # the families reach what they are meant to: clamps, large and integer waits
    assert (want == 1).sum() > 0 and (want > 1_000_000).sum() > 0


def test_mg1_empty_queue_and_first_arrival():
    n = np.array([0, 1, 1, 2], dtype=np.uint64)
    s = np.array([0.0, 3.0, 3.0, 6.0])
    q = np.array([0.0, 9.0, 9.0, 18.0])
    w = np.array([0, 3, 4, 7], dtype=np.uint64)
    want = O.ref_mg1(n, s, q, w) if O.ref_available() else O.cpuref_mg1(n, s, q, w)
    assert np.array_equal(_engine_mg1(n, s, q, w), want)
    assert want[0] == 0
