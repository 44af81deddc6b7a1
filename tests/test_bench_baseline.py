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


def test_parity_replicas_cover_the_pool_spares():
    """With the replica pool (5,120 slots, 5,520 replicas) a quarter of the
    workers take the first spares, which the pool starts as slot replicas
    halt; the rest spread over the slots up to the last slot."""
    reps = bench.parity_replicas(5520, 16, 5120)
    assert len(reps) == 16 and reps[0] == 0
    assert reps[-4:] == [5120, 5121, 5122, 5123] and reps[-5] == 5119
    assert bench.parity_replicas(5121, 16, 5120)[-2:] == [5119, 5120]   # one spare only
    assert bench.parity_replicas(5520, 2, 5120) == [0, 5120]


def test_busy_guard_refuses_a_grid_that_was_not_resident():
    """A replica pool whose slots were not all resident (busy fraction under
    0.95 while unstarted replicas remained) took two slices per launch: the
    bench must not report that rate.  A pool that ran dry may idle."""
    pool = {"wavefronts": 5632, "replicas": 6192, "replicas_started": 5901, "busy_fraction": 0.5}
    assert "not all resident" in bench.busy_guard(pool)
    assert bench.busy_guard(dict(pool, busy_fraction=0.998)) is None
    assert bench.busy_guard(dict(pool, replicas_started=6192)) is None
    assert bench.busy_guard(None) is None


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
