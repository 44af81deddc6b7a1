"""Opt-in DRAM bank model on the CPU restatement (the checker the GPU tests
use): hand-computed known answers, and the default (no <dram>) path staying
the reference's fixed latency."""
import numpy as np

import oracle as O
import primesim_amd as P
from primesim_amd import _abi as A
from primesim_amd import config as CF
from dram_cases import known_answer_requests, one_core_config


def test_oracle_bank_known_answers():
    cfg = one_core_config()
    ref = O.CpuRef(cfg)
    ref.alloc_core(1, 0)
    reqs, want, counts = known_answer_requests()
    d, rc = ref.run(reqs)
    assert rc == 0
    np.testing.assert_array_equal(d, want)
    st = ref.stats().as_dict()
    for k, v in counts.items():
        assert st[k] == v, k


def test_banks_zero_is_the_fixed_latency():
    sim = CF.preset("C2")
    spec = P.StreamSpec(A.PU_STREAM_SHARED_UNIFORM, 64, seed=5, max_requests=3000)
    reqs = P.generate_stream(spec)
    outs = []
    for dram in (None, {"banks": 0, "row_bytes": 0, "t_rcd": 0, "t_rp": 0, "t_burst": 0}):
        s = CF.preset("C2")
        if dram is not None:
            s["system"]["dram"] = dram
        ref = O.CpuRef(P.config_from_dict(s))
        for prog, th in P.stream_threads(spec):
            ref.alloc_core(prog, th)
        d, rc = ref.run(reqs)
        st = ref.stats().as_dict()
        assert st["dram_row_hits"] == st["dram_row_empty"] == st["dram_row_conflicts"] == 0
        outs.append(d)
    np.testing.assert_array_equal(outs[0], outs[1])


def test_banks_add_latency_and_keep_counts():
    """Against the fixed-latency run of the same stream: the same number of
    DRAM accesses (the model times them, it does not add or remove any), each
    classified exactly once."""
    spec = P.StreamSpec(A.PU_STREAM_SHARED_UNIFORM, 64, seed=6, max_requests=4000)
    reqs = P.generate_stream(spec)
    res = {}
    for banks in (0, 8):
        s = CF.preset("C2")
        if banks:
            s["system"]["dram"] = {"banks": banks, "row_bytes": 2048, "t_rcd": 14, "t_rp": 14, "t_burst": 4}
        ref = O.CpuRef(P.config_from_dict(s))
        for prog, th in P.stream_threads(spec):
            ref.alloc_core(prog, th)
        d, _ = ref.run(reqs)
        res[banks] = (d, ref.stats().as_dict())
    st0, st8 = res[0][1], res[8][1]
    assert st8["dram_row_hits"] + st8["dram_row_empty"] + st8["dram_row_conflicts"] == st8["dram_accesses"]
    assert st8["dram_row_conflicts"] > 0 and st8["dram_row_empty"] <= 8 * 1000
    assert res[8][0].astype(np.int64).sum() > res[0][0].astype(np.int64).sum()


def test_bad_bank_configs_refused():
    import pytest
    for dram in ({"banks": 3, "row_bytes": 2048, "t_rcd": 1, "t_rp": 1, "t_burst": 1},
                 {"banks": 4, "row_bytes": 1000, "t_rcd": 1, "t_rp": 1, "t_burst": 1},
                 {"banks": 4, "row_bytes": 2048, "t_rcd": -1, "t_rp": 1, "t_burst": 1}):
        s = CF.preset("C1")
        s["system"]["dram"] = dram
        cfg = P.config_from_dict(s)
        um = P.UncoreManager()
        # pu_create validates the configuration before it looks for a device
        with pytest.raises(P.UncoreError, match="dram"):
            um.init(cfg, replicas=1)
