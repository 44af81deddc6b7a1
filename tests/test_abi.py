"""The C-ABI library: loads, exports every symbol include/primeuncore.h declares,
validates configurations before touching a device, and fails loudly (no CPU
fallback) where there is no GPU."""
import ctypes as C
import os
import re

import pytest

import primesim_amd as P
from primesim_amd import config as CF
from primesim_amd.uncore import lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    with open(os.path.join(ROOT, "include", "primeuncore.h")) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^[A-Za-z_][\w \*]*?\b(pu_\w+)\s*\(", text, flags=re.M)))


def test_exports_every_declared_symbol():
    syms = declared_symbols()
    assert len(syms) >= 25
    L = lib()
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing


def test_version_and_error_strings():
    assert b"gfx950" in lib().pu_version()
    assert isinstance(P.uncore.last_error(), str)


def _gpu_present() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.mark.skipif(_gpu_present(), reason="checks the no-GPU path")
def test_no_gpu_fails_loudly():
    um = P.UncoreManager()
    with pytest.raises(P.UncoreError, match="no HIP device"):
        um.init(P.config_from_dict(CF.preset("C1")))


@pytest.mark.parametrize("mutate,msg", [
    (lambda s: s["system"].update(tlb_enable=1, tlb_cache=dict(s["system"]["tlb_cache"], size=0)), "TLB"),
    (lambda s: s["system"].update(sys_type=2), "sys_type"),
    (lambda s: s["system"]["cache"][0].update(share=2), "L1 share"),
    (lambda s: s["system"]["network"].update(link_delay=0), "link_delay"),
    (lambda s: s["system"]["directory_cache"].update(size=0), "directory"),
    (lambda s: s["system"].update(protocol_type=1, num_levels=2,
                                  cache=s["system"]["cache"] + [dict(s["system"]["cache"][0], share=4, level=1)]),
     "limited-pointer"),
    # the engine indexes a level's lines in 32 bits: 16 L1s of 2^36 B / 64 B = 2^34 lines
    (lambda s: s["system"]["cache"][0].update(size=1 << 36), "2^32 lines"),
    # sets are walked in 64-way chunks up to 4,096 ways (compiled configuration)
    (lambda s: s["system"]["cache"][0].update(size=8192 * 64, num_ways=8192), "4096 ways"),
    (lambda s: s["system"]["directory_cache"].update(size=8192 * 64, num_ways=8192), "4096 directory ways"),
])
def test_config_validation_before_device(mutate, msg):
    sim = CF.preset("C1")
    mutate(sim)
    cfg = P.config_from_dict(sim)
    h = lib().pu_create(C.byref(cfg), 1, 0)
    assert not h
    assert msg in P.uncore.last_error()


@pytest.mark.skipif(_gpu_present(), reason="checks the no-GPU path")
@pytest.mark.parametrize("mutate", [lambda s: s["system"].update(tlb_enable=1),
                                    lambda s: s["system"].update(sys_type=1),
                                    lambda s: s["system"].update(sys_type=1, tlb_enable=1),
                                    # wide sets pass validation (the device decides the kernel variant)
                                    lambda s: s["system"]["cache"][0].update(size=128 * 64, num_ways=128),
                                    lambda s: s["system"]["directory_cache"].update(size=4096 * 64,
                                                                                    num_ways=4096)])
def test_bus_and_tlb_configs_are_accepted(mutate):
    """sys_type=1 (mesi_bus) and tlb_enable=1 pass validation: creation only stops at the missing device."""
    sim = CF.preset("C1")
    mutate(sim)
    cfg = P.config_from_dict(sim)
    h = lib().pu_create(C.byref(cfg), 1, 0)
    assert not h
    assert "no HIP device" in P.uncore.last_error()


def test_stream_api_errors():
    from primesim_amd import _abi as A
    p = A.StreamParams(99, 16, 1, 1000, 1, 100, 1, 0, -1, 0)
    assert lib().pu_stream_count(C.byref(p)) < 0


def test_cpp_mirror_header_compiles(tmp_path):
    """include/primeuncore.hpp (the UncoreManager mirror a prime.cpp build would use) compiles and links."""
    import shutil
    import subprocess
    if not shutil.which("g++"):
        pytest.skip("no g++")
    src = tmp_path / "use.cpp"
    src.write_text(
        '#include "primeuncore.hpp"\n'
        '#include <sstream>\n'
        'int main(){ pu::UncoreManager m; pu_sim_cfg c{}; (void)c; std::ostringstream o;\n'
        '  if (0) { m.init(&c); pu::InsMem i{0,1,0,0,64}; m.uncore_access(0,&i,1);\n'
        '    char rec[48] = {0}; m.access_msgmem(0,1,rec,2); m.report(&o); }\n'
        '  return 0; }\n')
    out = tmp_path / "use"
    r = subprocess.run(["g++", "-std=c++17", f"-I{ROOT}/include", str(src), "-o", str(out),
                        f"-L{ROOT}/primesim_amd", "-lprimeuncore", f"-Wl,-rpath,{ROOT}/primesim_amd"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
