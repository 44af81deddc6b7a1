"""Opt-in DRAM bank model (pu_dram_cfg) on the HIP engine, through the C ABI.

No reference counterpart exists (the reference Dram is a fixed latency,
dram.cpp:43-47), so the checker is the CPU restatement (oracle/cpu_ref.cpp),
whose bank model is pinned by hand-computed known answers
(tests/test_dram_banks.py); with no <dram> element every golden still runs the
reference's fixed latency (test_gpu_golden.py).  Bit-exact: delays, per-core
completion cycles, every counter including the bank counters.
"""
import numpy as np
import pytest

import oracle as O
import primesim_amd as P
from dram_cases import STREAM_CASES, bank_config, known_answer_requests, one_core_config

pytestmark = pytest.mark.gpu


def test_engine_bank_known_answers():
    um = P.UncoreManager()
    um.init(one_core_config(), replicas=1)
    try:
        um.allocCore(1, 0)
        reqs, want, counts = known_answer_requests()
        np.testing.assert_array_equal(um.access_batch(reqs), want)
        st = um.stats().as_dict()
        for k, v in counts.items():
            assert st[k] == v, k
        assert "Row buffer conflicts: 1" in um.report()
    finally:
        um.close()


@pytest.mark.parametrize("name,preset,over,kind,cores,progs,n", STREAM_CASES, ids=[c[0] for c in STREAM_CASES])
@pytest.mark.parametrize("banks,row_bytes", [(16, 2048), (1, 64)])
def test_engine_banks_match_oracle(name, preset, over, kind, cores, progs, n, banks, row_bytes):
    cfg = bank_config(preset, banks=banks, row_bytes=row_bytes, **over)
    spec = P.StreamSpec(kind, cores, seed=11, num_progs=progs, max_requests=n)
    reqs = P.generate_stream(spec)
    ref = O.CpuRef(cfg)
    um = P.UncoreManager()
    um.init(cfg, replicas=1)
    try:
        for prog, th in P.stream_threads(spec):
            ref.alloc_core(prog, th)
            um.allocCore(prog, th)
        want, rc = ref.run(reqs)
        got = um.access_batch(reqs)
        np.testing.assert_array_equal(got[:len(want)], want)
        np.testing.assert_array_equal(um.completion(), ref.completion())
        gs, ws = um.stats().as_dict(), ref.stats().as_dict()
        assert {k: gs[k] for k in ws if k != "requests"} == {k: ws[k] for k in ws if k != "requests"}
        assert gs["dram_row_hits"] + gs["dram_row_empty"] + gs["dram_row_conflicts"] == gs["dram_accesses"]
        assert gs["dram_accesses"] > 0
    finally:
        um.close()
        ref.close()


def test_engine_banks_across_replicas_and_launches():
    """Bank state is per replica and carries across launches: two replicas
    with different streams, each fed in three chunks."""
    cfg = bank_config("C2", banks=8, row_bytes=4096)
    specs = [P.StreamSpec(P._abi.PU_STREAM_SHARED_UNIFORM, 64, seed=s, max_requests=4500) for s in (21, 22)]
    um = P.UncoreManager()
    um.init(cfg, replicas=2)
    try:
        for prog, th in P.stream_threads(specs[0]):
            um.allocCore(prog, th)
        for r, spec in enumerate(specs):
            reqs = P.generate_stream(spec)
            ref = O.CpuRef(cfg)
            for prog, th in P.stream_threads(spec):
                ref.alloc_core(prog, th)
            want, _ = ref.run(reqs)
            got = np.concatenate([um.access_batch(reqs[a:a + 1500], replica=r) for a in range(0, len(reqs), 1500)])
            np.testing.assert_array_equal(got, want)
            gs, ws = um.stats(r).as_dict(), ref.stats().as_dict()
            assert {k: gs[k] for k in ws if k != "requests"} == {k: ws[k] for k in ws if k != "requests"}
            ref.close()
    finally:
        um.close()
