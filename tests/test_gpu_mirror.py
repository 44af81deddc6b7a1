"""The C++ UncoreManager mirror (include/primeuncore.hpp) at run time on the GPU.

primesim_amd/mirror_check (tests/cpp/mirror_check.cpp, built with the library)
drives the header the way prime.cpp drives the reference: XML config,
allocCore per thread, one access_msgmem per MEM_REQUESTS message (the 24-B
MsgMem records), getSimStartTime/FinishTime and report.  Per-message delays,
the negative-delay stop (NegativeDelay at the reference's halt request) and
the report text must equal the reference's goldens.
"""
import os
import subprocess

import numpy as np
import pytest

from golden_util import Case

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "primesim_amd", "mirror_check")


def _strip_time(text: str) -> str:
    return "".join(ln for ln in text.splitlines(keepends=True) if not ln.startswith("Total computation time"))


@pytest.mark.parametrize("name", ["c1_hot", "small_msgs", "c3_multiprog", "c4_overflow_halt"])
def test_cpp_mirror_replays_golden(name, tmp_path):
    assert os.path.exists(BIN), "mirror_check not built (make -C primesim_amd/csrc)"
    c = Case(name)
    reqs = tmp_path / "reqs.bin"
    c.reqs.tofile(reqs)
    (tmp_path / "threads.txt").write_text("".join(f"{p} {t}\n" for p, t in c.threads))
    out = tmp_path / "out"
    r = subprocess.run([BIN, c.xml_path, str(reqs), str(tmp_path / "threads.txt"), str(out)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = (tmp_path / "out.delays").read_text().split("\n")
    starts = np.nonzero(c.reqs["batch_start"])[0].tolist() + [len(c.reqs)]
    halt = c.meta.get("halt_index")
    want = []
    for a, b in zip(starts, starts[1:]):
        D = 0
        for i in range(a, b):
            D += int(c.delays[i]) - 1
            if D < 0:
                want.append(f"halt {i} {D}")
                break
        else:
            want.append(str(D))
            continue
        break
    assert [ln for ln in lines if ln] == want
    if halt is not None:
        assert want[-1].startswith(f"halt {halt} ")
    assert _strip_time((tmp_path / "out.report").read_text()) == c.report
