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


def test_parity_replicas_spread_to_the_last():
    reps = bench.parity_replicas(5120, 16)
    assert len(reps) == 16 and reps[0] == 0 and reps[-1] == 5119
    assert reps == sorted(set(reps)) and reps[1] == 320
    assert bench.parity_replicas(10, 16) == list(range(10))
    assert bench.parity_replicas(1, 16) == [0]


def test_ensemble_returns_the_delays_of_its_replicas(tmp_path):
    """The ensemble processes (forked before the GPU is touched) are told their
    replicas afterwards and send back every delay they produced: the same
    delays the CPU restatement gives on those replicas' streams."""
    import oracle as O
    from primesim_amd import config as CF
    from primesim_amd.dist import replica_seed
    xml = CF.write_xml(CF.preset("C4"), str(tmp_path / "c4.xml"))
    ens = bench.Ensemble(xml, 3, 3000, 3000, 0.3)
    assert ens.assign(40) == [0, 13, 39]
    res = ens.run()
    assert res["cores"] == 3 and sorted(ens.delays) == [0, 13, 39]
    cfg = P.load_config(xml)
    for r, got in ens.delays.items():
        assert len(got) >= 3000
        reqs = P.generate_stream(bench.stream_spec(replica_seed(bench.SEED_BASE, 0, r), len(got)))
        ref = O.CpuRef(cfg)
        for prog, th in P.stream_threads(bench.stream_spec(bench.SEED_BASE)):
            ref.alloc_core(prog, th)
        want, _ = ref.run(reqs)
        np.testing.assert_array_equal(got, want[:len(got)])
