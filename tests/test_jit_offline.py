"""The compile-time configuration's two compilers (jit.cpp), without a GPU:
pu_config_jit_warm writes two code objects per configuration (throughput and
latency kernels) with hipcc when it is present, with hipRTC when the offline
compiler is turned off (PRIMEUNCORE_JIT_HIPCC=0); the two sets have distinct
keys (so a run prefers hipcc's), each object holds its part's kernels, and a
second warm-up finds them cached."""
import ctypes as C
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = ("import ctypes as C, sys; sys.path.insert(0, %r); import primesim_amd as P; "
        "from primesim_amd import config as CF, uncore; cfg = P.config_from_dict(CF.preset('C1')); "
        "print(uncore.lib().pu_config_jit_warm(C.byref(cfg)))") % ROOT


def _warm(cache, **env):
    e = dict(os.environ, PRIMEUNCORE_JIT_CACHE=str(cache), PRIMEUNCORE_JIT_OFFLINE="1")
    e.update(env)
    r = subprocess.run([sys.executable, "-c", CODE], env=e, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return int(r.stdout.strip().splitlines()[-1])


@pytest.mark.skipif(not os.access("/opt/rocm/bin/hipcc", os.X_OK), reason="no hipcc")
def test_warm_up_compiles_both_parts_with_either_compiler(tmp_path):
    off, rtc = tmp_path / "offline", tmp_path / "rtc"
    off.mkdir()
    rtc.mkdir()
    assert _warm(off) == 0
    assert _warm(rtc, PRIMEUNCORE_JIT_HIPCC="0") == 0
    fo, fr = sorted(p.name for p in off.glob("*.hsaco")), sorted(p.name for p in rtc.glob("*.hsaco"))
    assert len(fo) == 2 and len(fr) == 2 and not set(fo) & set(fr)
    for d in (off, rtc):
        blobs = [p.read_bytes() for p in d.glob("*.hsaco")]
        thr = [b for b in blobs if b"pu_jit_uncore_s2_h0" in b]
        lat = [b for b in blobs if b"pu_jit_uncore_s1_h1" in b]
        assert len(thr) == 1 and len(lat) == 1 and thr[0] is not lat[0]
        assert b"pu_jit_uncore_s1_h1" not in thr[0] and b"pu_jit_uncore_s2_h0" not in lat[0]
    assert _warm(off) == 1                                   # cached
    # without the opt-in the warm-up never starts hipcc: hipRTC's objects
    rtc2 = tmp_path / "no_opt_in"
    rtc2.mkdir()
    assert _warm(rtc2, PRIMEUNCORE_JIT_OFFLINE="0") == 0
    assert sorted(p.name for p in rtc2.glob("*.hsaco")) == fr
