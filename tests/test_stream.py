"""Synthetic request streams: determinism and the request-stream semantics of
the core model (core_manager.cpp:104-269) in the canonical order."""
import numpy as np
import pytest

import primesim_amd as P
from primesim_amd import _abi as A
from golden_util import Case, case_names


@pytest.mark.parametrize("name", case_names())
def test_golden_streams_regenerate(name):
    c = Case(name)
    s = c.meta["stream"]
    spec = P.StreamSpec(s["kind"], s["num_cores"], s["seed"], s["quantum"], s["num_quanta"], s["max_msg"],
                        s["num_progs"], s["max_requests"], s["write_pct"])
    np.testing.assert_array_equal(P.generate_stream(spec).view(np.uint8), c.reqs.view(np.uint8))
    assert P.stream_threads(spec) == c.threads


@pytest.mark.parametrize("kind", [A.PU_STREAM_PRIVATE_STREAMING, A.PU_STREAM_SHARED_UNIFORM,
                                  A.PU_STREAM_MULTIPROGRAM, A.PU_STREAM_UNIFORM_HOTSPOT,
                                  A.PU_STREAM_PRODUCER_CONSUMER, A.PU_STREAM_UNIFORM])
def test_stream_semantics(kind):
    spec = P.StreamSpec(kind, 32, seed=3, quantum=300, num_quanta=3, max_msg=17, num_progs=4)
    r = P.generate_stream(spec)
    assert len(r) > 0
    q = r["timer"] // spec.quantum
    key = q * spec.num_cores + r["core"]
    assert np.all(np.diff(key) >= 0), "canonical order: quantum-major, then core"
    starts = np.nonzero(r["batch_start"])[0]
    assert starts[0] == 0
    lens = np.diff(np.append(starts, len(r)))
    assert lens.max() <= spec.max_msg
    for a, b in zip(starts, np.append(starts[1:], len(r))):
        seg = r[a:b]
        assert len(set(seg["core"])) == 1
        assert len(set(seg["timer"] // spec.quantum)) == 1, "a message never spans a barrier"
    for c in range(spec.num_cores):
        t = r["timer"][r["core"] == c]
        gaps = np.diff(t)
        assert gaps.min() >= 1 and gaps.max() <= 4
    assert set(np.unique(r["mem_type"])) <= {A.PU_RD, A.PU_WR}
    assert r["prog_id"].min() >= 1


def test_stream_cap_and_determinism():
    spec = P.StreamSpec(A.PU_STREAM_UNIFORM_HOTSPOT, 1024, seed=4, num_quanta=5, max_requests=12345)
    a = P.generate_stream(spec)
    b = P.generate_stream(spec)
    assert len(a) == 12345
    assert a.tobytes() == b.tobytes()
    spec2 = P.StreamSpec(A.PU_STREAM_UNIFORM_HOTSPOT, 1024, seed=5, num_quanta=5, max_requests=12345)
    assert P.generate_stream(spec2).tobytes() != a.tobytes()


def test_thread_map_programs():
    spec = P.StreamSpec(A.PU_STREAM_MULTIPROGRAM, 256, num_progs=4)
    th = P.stream_threads(spec)
    assert th[0] == (1, 0) and th[63] == (1, 63) and th[64] == (2, 0) and th[255] == (4, 63)


@pytest.mark.parametrize("chunk", [1, 7, 100, 4096])
def test_resumable_streams_concatenate_to_one_shot(chunk):
    """pu_stream_next_many chunks == pu_stream_generate, across quantum and
    message boundaries, for several streams advanced on several threads."""
    specs = [P.StreamSpec(k, 48, seed=s, quantum=200, num_quanta=3, max_msg=9, num_progs=2)
             for s, k in ((1, A.PU_STREAM_UNIFORM_HOTSPOT), (2, A.PU_STREAM_SHARED_UNIFORM),
                          (3, A.PU_STREAM_MULTIPROGRAM))]
    want = [P.generate_stream(sp) for sp in specs]
    ss = P.StreamSet(specs)
    got = [[] for _ in specs]
    while True:
        out = np.zeros((len(specs), chunk), dtype=A.REQ_DTYPE)
        ss.next_into(out, threads=3)
        done = True
        for i in range(len(specs)):
            n_i = min(chunk, len(want[i]) - sum(len(x) for x in got[i]))
            if n_i > 0:
                got[i].append(out[i, :n_i].copy())
                done = False
        if done:
            break
    for i in range(len(specs)):
        g = np.concatenate(got[i])
        np.testing.assert_array_equal(g.view(np.uint8), want[i].view(np.uint8))
        assert ss.position(i) == len(want[i])
    assert len(ss.next(5)[0]) == 0          # exhausted
    ss.close()


def test_resumable_stream_respects_max_requests():
    spec = P.StreamSpec(A.PU_STREAM_UNIFORM_HOTSPOT, 1024, seed=4, num_quanta=64, max_requests=10_000)
    ss = P.StreamSet([spec])
    a = ss.next(6000)[0]
    b = ss.next(6000)[0]
    assert len(a) == 6000 and len(b) == 4000
    np.testing.assert_array_equal(np.concatenate([a, b]).view(np.uint8), P.generate_stream(spec).view(np.uint8))
