"""The two engine variants agree with the reference: the configuration compiled
into the kernel (jit.cpp, hipRTC; the default) and the ahead-of-time kernels
(PRIMEUNCORE_JIT=0) that read the geometry at run time.

By default (pu_create; the cache is warmed by __graft_entry__.build()) a
handle runs the compiled configuration for every launch: latency launches (at
most one replica per CU, headers in LDS: the long golden batches) and
throughput launches (short batches, many replicas).  Here a spread of goldens
(one and three levels, bus system, TLB, limited pointer, 3-D mesh, closed
loop, a full-size digest) also runs with the ahead-of-time kernels only
(PRIMEUNCORE_JIT=0) and with the ahead-of-time kernels for the throughput
launches (PRIMEUNCORE_JIT_THROUGHPUT=0), and every handle reports its variant.
"""
import pytest

import primesim_amd as P
from primesim_amd import uncore
from golden_util import Case
from test_gpu_golden import test_engine_reproduces_reference

pytestmark = pytest.mark.gpu

CASES = ["c1_hot", "c3_multiprog", "three_level", "bus_c2", "tlb_c3", "limited_ptr", "mesh3d", "c4_closed",
         "big_c4_quantum"]


@pytest.mark.parametrize("name", ["c1_hot", "c3_multiprog", "bus_c2", "tlb_c3", "c4_closed", "big_c4_quantum"])
def test_ahead_of_time_throughput_launches_match_reference(name, monkeypatch):
    """PRIMEUNCORE_JIT_THROUGHPUT=0: throughput launches on the ahead-of-time
    kernels, latency launches on the compiled configuration."""
    monkeypatch.setenv("PRIMEUNCORE_JIT_THROUGHPUT", "0")
    test_engine_reproduces_reference(name)


@pytest.mark.parametrize("name", CASES)
def test_ahead_of_time_kernels_match_reference(name, monkeypatch):
    monkeypatch.setenv("PRIMEUNCORE_JIT", "0")
    test_engine_reproduces_reference(name)


@pytest.mark.parametrize("jit,thr,want", [("1", "0", 1), ("1", "1", 2), ("1", "", 2), ("0", "0", 0)])
def test_handle_reports_its_variant(jit, thr, want, monkeypatch):
    monkeypatch.setenv("PRIMEUNCORE_JIT", jit)
    monkeypatch.setenv("PRIMEUNCORE_JIT_THROUGHPUT", thr)
    um = P.UncoreManager()
    um.init(P.load_config(Case("c1_hot").xml_path), replicas=1)
    try:
        assert uncore.lib().pu_compiled_config(um._handle()) == want
    finally:
        um.close()


@pytest.mark.parametrize("name", ["dir_128way", "l1_tlb_128way", "bus_192way"])
def test_wide_sets_need_the_compiled_configuration(name, monkeypatch):
    """Sets of more than 64 ways are walked in 64-way chunks by the compiled
    configuration only (their goldens run in test_gpu_golden); the
    ahead-of-time kernels refuse them at pu_create instead of diverging."""
    monkeypatch.setenv("PRIMEUNCORE_JIT", "0")
    um = P.UncoreManager()
    with pytest.raises(Exception, match="more than 64 ways"):
        um.init(P.load_config(Case(name).xml_path), replicas=1)


def test_handle_reports_its_compiler(tmp_path, monkeypatch):
    """The in-tree cache holds hipcc's code objects (build-time warm-up): a
    handle over it reports compiler 2.  A cache miss at run time (an empty
    cache directory) is compiled by hipRTC in-process, never by starting a
    compiler from a process that has used the GPU: compiler 1, and the same
    delays as the reference."""
    cfg = P.load_config(Case("c1_hot").xml_path)
    um = P.UncoreManager()
    um.init(cfg, replicas=1)
    try:
        assert uncore.lib().pu_compiled_compiler(um._handle()) == 2
    finally:
        um.close()
    monkeypatch.setenv("PRIMEUNCORE_JIT_CACHE", str(tmp_path))
    um = P.UncoreManager()
    um.init(cfg, replicas=1)
    try:
        assert uncore.lib().pu_compiled_compiler(um._handle()) == 1
    finally:
        um.close()
    assert len(list(tmp_path.glob("*.hsaco"))) == 2        # both parts, hipRTC's keys
    test_engine_reproduces_reference("c1_hot")              # on hipRTC's code objects (the env still points there)
