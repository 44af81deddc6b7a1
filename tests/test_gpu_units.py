"""Engine components alone on the GPU vs the reference's component goldens:
the ring-buffer history-tree queue model (incl. prune and ring wrap-around)
and Network::transmit on 2D/3D/non-square meshes."""
import json
import os

import numpy as np
import pytest

import oracle as O
from golden_util import GOLDEN
from primesim_amd.uncore import unit_network, unit_queue

pytestmark = pytest.mark.gpu


def test_queue_model_golden_gpu():
    z = np.load(os.path.join(GOLDEN, "queue_model.npz"), allow_pickle=False)
    for k in np.unique(z["trial"]):
        m = z["trial"] == k
        minp = int(z["min_proc"][m][0])
        got, mg1 = unit_queue(minp, z["t"][m], z["p"][m])
        np.testing.assert_array_equal(got, z["delay"][m], err_msg=f"trial {k}")
        _, mg1_ref = O.cpuref_queue(minp, z["t"][m], z["p"][m])
        assert mg1 == mg1_ref


def test_queue_model_long_random_gpu():
    """Tens of thousands of calls: the ring head laps the 128-slot ring many times."""
    rng = np.random.default_rng(9)
    n = 30000
    t = (np.cumsum(rng.integers(0, 3, n)) + rng.integers(0, 300, n)).astype(np.uint64)
    p = rng.integers(1, 13, n).astype(np.uint64)
    got, _ = unit_queue(1, t, p)
    want, _ = O.cpuref_queue(1, t, p)
    np.testing.assert_array_equal(got, want)


def test_queue_model_long_time_span_gpu():
    """Arrivals ~2^25 cycles apart for 20,000 calls (times past 2^39): every
    delay against the CPU restatement (written for a compact-ring experiment
    that re-based 32-bit interval offsets; kept as coverage of
    long time spans)."""
    rng = np.random.default_rng(11)
    n = 20000
    t = np.cumsum(rng.integers(1 << 24, 1 << 26, n)).astype(np.uint64)
    t = t + rng.integers(0, 1 << 20, n).astype(np.uint64)
    p = rng.integers(1, 13, n).astype(np.uint64)
    got, _ = unit_queue(1, t, p)
    want, _ = O.cpuref_queue(1, t, p)
    np.testing.assert_array_equal(got, want)


def test_queue_model_history_spans_2_32_gpu():
    """Bursts separated by jumps of 2^33 cycles, so the live intervals of the
    history span more than 2^32 cycles: every delay against the CPU
    restatement."""
    rng = np.random.default_rng(12)
    n = 20000
    steps = rng.integers(0, 3, n).astype(np.uint64)
    steps[::700] += np.uint64(1 << 33)
    t = (np.cumsum(steps) + rng.integers(0, 300, n)).astype(np.uint64)
    p = rng.integers(1, 13, n).astype(np.uint64)
    got, _ = unit_queue(1, t, p)
    want, _ = O.cpuref_queue(1, t, p)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("name", ["mesh4x4", "mesh8x8_r1", "mesh3d_4", "mesh_ns_12"])
def test_network_golden_gpu(name):
    with open(os.path.join(GOLDEN, "network.json")) as f:
        meta = json.load(f)[name]
    z = np.load(os.path.join(GOLDEN, f"net_{name}.npz"), allow_pickle=False)
    got, st = unit_network(meta["nodes"], meta["net_type"], meta["data_width"], meta["header_flits"],
                           meta["router_delay"], meta["link_delay"], meta["inject_delay"],
                           z["src"], z["dst"], z["len"], z["timer"])
    np.testing.assert_array_equal(got, z["delay"])
    _, ref_st = O.cpuref_network(meta["nodes"], meta["net_type"], meta["data_width"], meta["header_flits"],
                                 meta["router_delay"], meta["link_delay"], meta["inject_delay"],
                                 z["src"], z["dst"], z["len"], z["timer"])
    for k in ("net_accesses", "net_distance", "net_total_delay", "net_router_delay", "net_link_delay",
              "net_inject_delay", "link_flits", "mg1_calls"):
        assert getattr(st, k) == getattr(ref_st, k), k
