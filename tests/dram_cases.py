"""Shared cases for the opt-in DRAM bank model (include/primeuncore.h
pu_dram_cfg; no reference counterpart — the reference Dram is a fixed latency,
dram.cpp:43-47 — so parity is engine vs the CPU restatement, and the
restatement itself is pinned by the hand-computed known answers below).
"""
import numpy as np

import primesim_amd as P
from primesim_amd import _abi as A
from primesim_amd import config as CF

BANKS = {"banks": 4, "row_bytes": 8192, "t_rcd": 10, "t_rp": 20, "t_burst": 5}
DRAM_TIME = 100


def one_core_config():
    """1 core, 1 LLC node (home = the core: no network hops), L1 + directory."""
    sim = CF.preset("C1", num_cores=1, dram_access_time=DRAM_TIME)
    sim["system"]["dram"] = dict(BANKS)
    return P.config_from_dict(sim)


def known_answer_requests():
    """(addr, timer) of single-request messages and the delay each must get.

    base = L1 access (1) + directory access (10) + dram_access_time (100);
    the DRAM access of a request issued at cycle T happens at T + 11.
      1  t=0     row 0 -> bank 0, closed          base + t_rcd
      2  t=1000  row 0 again (bank 0 page open)   base
      3  t=2000  row 4 -> bank 0, other page open base + t_rp + t_rcd
      4  t=3000  row 1 -> bank 1, closed          base + t_rcd
      5  t=3000  row 1 again, bank 1 busy until 3011+10+5: waits 15, hit
      6  t=3000  row 2 -> bank 2, closed (another bank: no wait)
      7  t=2990  row 4 -> bank 0 page open; free since 2011+30+5: hit
    """
    base = 1 + 10 + DRAM_TIME
    rows = [(0, 0, base + 10), (64, 1000, base), (8192 * 4, 2000, base + 30), (8192, 3000, base + 10),
            (8192 + 64, 3000, base + 15), (8192 * 2, 3000, base + 10), (8192 * 4 + 128, 2990, base)]
    reqs = np.zeros(len(rows), dtype=A.REQ_DTYPE)
    for i, (addr, t, _) in enumerate(rows):
        reqs[i] = (addr, t, 0, 1, A.PU_RD, 1, 0, 0)
    want = np.array([d for _, _, d in rows], dtype=np.int32)
    # hits: 2, 5, 7; empty: 1, 4, 6; conflicts: 3; waits: 15
    return reqs, want, {"dram_row_hits": 3, "dram_row_empty": 3, "dram_row_conflicts": 1, "dram_bank_wait": 15,
                        "dram_accesses": 7}


def bank_config(preset, banks=16, row_bytes=2048, **over):
    sim = CF.preset(preset, **over)
    sim["system"]["dram"] = {"banks": banks, "row_bytes": row_bytes, "t_rcd": 14, "t_rp": 14, "t_burst": 4}
    return P.config_from_dict(sim)


# (name, preset, overrides, stream kind, cores, progs, requests)
STREAM_CASES = [
    ("c1_private", "C1", {}, A.PU_STREAM_PRIVATE_STREAMING, 16, 1, 6000),
    ("c2_shared", "C2", {}, A.PU_STREAM_SHARED_UNIFORM, 64, 1, 6000),
    ("c3_multiprog", "C3", {}, A.PU_STREAM_MULTIPROGRAM, 256, 4, 6000),
    ("c2_private_llc", "C2", {"shared_llc": 0}, A.PU_STREAM_SHARED_UNIFORM, 64, 1, 6000),
    ("c4_hotspot", "C4", {}, A.PU_STREAM_UNIFORM_HOTSPOT, 1024, 1, 20000),
]


def dram_configs():
    """(name, pu_sim_cfg) of every bank-model configuration the GPU tests build
    (tools/jit_warm.py compiles them ahead of the GPU run)."""
    out = [("dram one-core", one_core_config())]
    for name, preset, over, *_ in STREAM_CASES:
        for banks, row in ((16, 2048), (1, 64)):          # test_gpu_dram.py's two geometries
            out.append((f"dram {name} {banks}x{row}", bank_config(preset, banks, row, **over)))
    out.append(("dram C2 8x4096", bank_config("C2", 8, 4096)))
    return out
