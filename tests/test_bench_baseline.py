"""bench.py's CPU baseline counts only the requests the reference simulated:
a replica stopped by the prime.cpp:130-134 rule (negative running delay)
simulates nothing after the stopping request, so the skipped requests must not
inflate the baseline's accesses/s (CPU only; the reference compiled in place,
or the restatement where it is absent)."""
from __future__ import annotations

import numpy as np

import bench
import primesim_amd as P
from golden_util import Case


def test_simulated_counts():
    assert bench.simulated(100, 0) == 100        # whole call simulated
    assert bench.simulated(100, 37) == 37        # stopped after request 36
    assert bench.simulated(100, -1) == 0         # already stopped: nothing simulated


def test_cpu_baseline_stops_at_the_halt():
    c = Case("c4_overflow_halt")
    cfg = P.load_config(c.xml_path)
    kind, n_sim, el, d = bench.cpu_baseline(c.xml_path, cfg, c.reqs, c.threads, 0, 60.0)
    nz = np.nonzero(c.delays)[0]
    stop = int(nz[-1]) + 1                       # the golden: delays are 0 after the stopping request
    assert n_sim == stop < len(c.reqs)
    np.testing.assert_array_equal(d[:stop], c.delays[:stop])
