"""Component goldens: the Graphite history-tree queue model and Network::transmit.

The sorted-array restatement of the AVL interval tree is pinned against the
compiled Graphite QueueModelHistoryTree (16 trials x 2,500 calls covering the
100-interval prune, the M/G/1 fallback and min_processing_time 1-3), and the
mesh network against Network::transmit on 2D/3D/non-square meshes.
"""
import json
import os

import numpy as np
import pytest

import oracle as O
from golden_util import GOLDEN


def test_queue_model_golden():
    z = np.load(os.path.join(GOLDEN, "queue_model.npz"), allow_pickle=False)
    total_mg1 = 0
    for k in np.unique(z["trial"]):
        m = z["trial"] == k
        minp = int(z["min_proc"][m][0])
        got, mg1 = O.cpuref_queue(minp, z["t"][m], z["p"][m])
        np.testing.assert_array_equal(got, z["delay"][m], err_msg=f"trial {k}")
        assert 0 <= mg1 <= m.sum()
        total_mg1 += mg1
    assert total_mg1 > 1000   # the analytical fallback is exercised


def _net_report_numbers(text):
    vals = {}
    for line in text.splitlines():
        if ": " in line:
            k, v = line.rsplit(": ", 1)
            vals[k] = v
    return vals


@pytest.mark.parametrize("name", ["mesh4x4", "mesh8x8_r1", "mesh3d_4", "mesh_ns_12"])
def test_network_golden(name):
    with open(os.path.join(GOLDEN, "network.json")) as f:
        meta = json.load(f)[name]
    z = np.load(os.path.join(GOLDEN, f"net_{name}.npz"), allow_pickle=False)
    got, st = O.cpuref_network(meta["nodes"], meta["net_type"], meta["data_width"], meta["header_flits"],
                               meta["router_delay"], meta["link_delay"], meta["inject_delay"],
                               z["src"], z["dst"], z["len"], z["timer"])
    np.testing.assert_array_equal(got, z["delay"])
    rep = _net_report_numbers(meta["report"])
    assert int(rep["# of accesses"]) == st.net_accesses
    assert int(rep["Total network communication distance"]) == st.net_distance
    assert int(rep["Total network delay"]) == st.net_total_delay
    assert int(rep["Total router delay"]) == st.net_router_delay
    assert int(rep["Total link delay"]) == st.net_link_delay
    assert int(rep["Total inject delay"]) == st.net_inject_delay


@pytest.mark.skipif(not O.ref_available(), reason="reference build (oracle/_ref) not present")
@pytest.mark.parametrize("seed", range(6))
def test_queue_model_fuzz_against_reference(seed):
    """Fresh random sequences, both implementations live (build container only)."""
    rng = np.random.default_rng(100 + seed)
    n = 4000
    minp = 1 + seed % 3
    t = (np.cumsum(rng.integers(0, 4, n)) + rng.integers(0, 50 + 100 * seed, n)).astype(np.uint64)
    p = rng.integers(1, 13, n).astype(np.uint64)
    want = O.ref_queue(minp, t, p)
    got, _ = O.cpuref_queue(minp, t, p)
    np.testing.assert_array_equal(got, want)


@pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref not built")
def test_mg1_restatement_matches_reference_arithmetic():
    """cpu_ref's mg1_wait equals the reference's own QueueModelMG1::computeQueueDelay
    (queue_model_m_g_1.cpp:16-42, compiled in place) on 1.2M seeded states,
    including the λ >= μ clamp and exact-integer waits (tests/mg1_states.py)."""
    from mg1_states import states
    n, s, q, w = states(1_200_000, seed=11)
    want = O.ref_mg1(n, s, q, w)
    got = O.cpuref_mg1(n, s, q, w)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, f"{len(bad)} mismatches, first state {[x[bad[0]] for x in (n, s, q, w)]}"
    assert (want > 0).mean() > 0.5
