"""The relaxation tooling behind DESIGN.md §1a (research code, CPU only):
tools/relax/relax_proto.cpp builds from its own source, its exact
fast-forward reproduces the restatement's delays, a relaxed run converges to
them window by window, and its sweep dump (the input of the GPU measurement,
tools/relax/sweep_bench.hip) is self-consistent."""
import os
import re
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RELAX = os.path.join(ROOT, "tools", "relax")


@pytest.fixture(scope="module")
def proto(tmp_path_factory):
    d = tmp_path_factory.mktemp("relax")
    exe = str(d / "relax_proto")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(RELAX, "relax_proto.cpp")], check=True)
    pre = str(d / "c1")
    r = subprocess.run([sys.executable, os.path.join(RELAX, "dump_stream.py"), "C1", "4", "7", "12000", pre],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return exe, pre, d


def test_relaxed_windows_converge_to_the_sequential_delays(proto):
    exe, pre, _ = proto
    r = subprocess.run([exe, pre, "16", "256", "500"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    m = re.search(r"mismatches (\d+)/(\d+)", r.stdout)
    assert m and m.group(1) == "0" and m.group(2) == "12000", r.stdout


def test_fast_forward_and_sweep_dump(proto):
    exe, pre, d = proto
    out = d / "dump"
    out.mkdir()
    env = dict(os.environ, RELAX_SKIP="6000", RELAX_DUMP=str(out), RELAX_DUMP_SWEEP="2")
    r = subprocess.run([exe, pre, "16", "512"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "exact fast-forward: 6000 requests, 0 mismatches" in r.stdout
    meta = np.fromfile(out / "meta.bin", dtype=np.uint32)
    W, nlinks, nvis, nev, nslots, ways, nwords = (int(x) for x in meta[:7])
    assert W == 512 and nvis > 0 and nev > 0
    assert os.path.getsize(out / "l_links.bin") == 48 * nlinks
    assert os.path.getsize(out / "l_iv.bin") == 8 * 256 * nlinks
    assert os.path.getsize(out / "l_vis.bin") == 16 * nvis and os.path.getsize(out / "l_qd.bin") == 8 * nvis
    assert os.path.getsize(out / "f_ev.bin") == 40 * nev
    assert os.path.getsize(out / "f_lines.bin") == 8 * 3 * ways * nslots
    assert os.path.getsize(out / "f_shr.bin") == 8 * nwords * ways * nslots
    links = np.fromfile(out / "l_links.bin", dtype=np.uint32).reshape(nlinks, 12)
    assert (links[:, 9] < links[:, 10]).all() and links[-1, 10] == nvis     # visit ranges, in order
