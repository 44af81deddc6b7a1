"""The C++ mirror takes the reference's own XmlSim (uncore_manager.h:54).

tests/cpp/xmlsim_check.cpp is compiled against the reference's xml_parser.h and
cache.h (in place, /root/reference/src) plus include/primeuncore.hpp, and
linked with the reference's XmlParser object built by oracle/Makefile `ref`:

* prime.cpp's call sites (`uncore_manager.init(xml_sim)` prime.cpp:198,
  `uncore_access(core_id, &ins_mem, ...)` with the reference InsMem
  prime.cpp:129, allocCore/getCoreId/deallocCore/report) compile unchanged
  against pu::UncoreManager;
* every golden XML parsed by the reference XmlParser and converted by
  pu::UncoreManager::config_from equals pu_config_load_xml's pu_sim_cfg field
  for field.

CPU only; skipped where the reference tree is absent (the GPU box).
"""
import glob
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SRC = "/root/reference/src"
XML_OBJ = os.path.join(ROOT, "oracle", "_ref", "obj", "xml_parser.o")


@pytest.mark.skipif(not os.path.isdir(REF_SRC), reason="reference tree not mounted")
def test_reference_xmlsim_drives_the_mirror(tmp_path):
    if not os.path.exists(XML_OBJ):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True, capture_output=True)
    exe = tmp_path / "xmlsim_check"
    lib_dir = os.path.join(ROOT, "primesim_amd")
    cmd = ["g++", "-O1", "-std=c++17", "-w", f"-I{REF_SRC}", f"-I{REF_SRC}/Graphite", "-I/usr/include/libxml2",
           f"-I{ROOT}/include", "-o", str(exe), os.path.join(ROOT, "tests", "cpp", "xmlsim_check.cpp"), XML_OBJ,
           f"-L{lib_dir}", "-lprimeuncore", f"-Wl,-rpath,{lib_dir}", "-lxml2"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    xmls = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "*.xml")))
    assert len(xmls) >= 30
    r = subprocess.run([str(exe), *xmls], capture_output=True, text=True, timeout=120)
    lines = r.stdout.splitlines()
    assert r.returncode == 0, "\n".join(ln for ln in lines if not ln.startswith("OK"))
    assert sum(ln.startswith("OK ") for ln in lines) == len(xmls)
