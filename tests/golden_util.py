"""Helpers to load tests/golden fixtures (data made by tools/gen_golden.py from
the reference's own uncore) and to read the reference's report text."""
from __future__ import annotations

import hashlib
import json
import os
import re

import numpy as np

from primesim_amd import _abi as A

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _all_names() -> list[str]:
    return sorted(f[:-5] for f in os.listdir(GOLDEN) if f.endswith(".json") and f not in
                  ("network.json", "configs.json"))


def case_names() -> list[str]:
    """Fixtures that hold their requests and every delay."""
    return [n for n in _all_names() if not n.startswith("big_")]


def big_case_names() -> list[str]:
    """Full-size preset runs stored as digests (requests regenerate from the spec)."""
    return [n for n in _all_names() if n.startswith("big_")]


def sha256(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).view(np.uint8).tobytes()).hexdigest()


class Case:
    def __init__(self, name: str):
        self.name = name
        z = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
        with open(os.path.join(GOLDEN, f"{name}.json")) as f:
            self.meta = json.load(f)
        self.digest = self.meta.get("digest")
        if self.digest:
            import primesim_amd as P
            spec = P.StreamSpec(**self.meta["stream"])
            self.reqs = P.generate_stream(spec)
            assert sha256(self.reqs) == self.digest["reqs_sha256"], f"{name}: stream generator drifted"
            self.delays = None
            self.head, self.tail = z["head"], z["tail"]
        else:
            self.reqs = z["reqs"].view(A.REQ_DTYPE)
            self.delays = z["delays"]
        self.completion = z["completion"]
        self.xml_path = os.path.join(GOLDEN, f"{name}.xml")
        with open(os.path.join(GOLDEN, f"{name}.report.txt")) as f:
            self.report = f.read()
        self.threads = [tuple(t) for t in self.meta["threads"]]
        self.counters = self.meta["counters"]
        self.closed = self.meta.get("replay", "open") == "closed"

    def check_delays(self, d: np.ndarray) -> None:
        """Every delay equals the reference's (in full, or by digest)."""
        if self.delays is not None:
            np.testing.assert_array_equal(d, self.delays)
            return
        np.testing.assert_array_equal(d[:len(self.head)], self.head)
        np.testing.assert_array_equal(d[-len(self.tail):], self.tail)
        assert int(d.astype(np.int64).sum()) == self.digest["delay_sum"], f"{self.name}: delay sum differs"
        assert sha256(d.astype(np.int32)) == self.digest["delays_sha256"], f"{self.name}: delay digest differs"


def extended_stream(case: "Case", n: int) -> np.ndarray:
    """The case's stream regenerated with n requests (its fixture holds a prefix)."""
    import primesim_amd as P
    spec = dict(case.meta["stream"])
    spec["max_requests"] = n
    r = P.generate_stream(P.StreamSpec(**spec))
    assert np.array_equal(r[:len(case.reqs)], case.reqs), f"{case.name}: stream generator drifted"
    return r


def report_stats(text: str) -> dict:
    """Aggregate numbers printed by System::report (system.cpp:956-1069)."""
    def num(pat, s=text):
        m = re.search(pat, s)
        assert m, pat
        return int(m.group(1))
    out = {
        "net_accesses": num(r"# of accesses: (\d+)"),
        "net_distance": num(r"Total network communication distance: (\d+)"),
        "net_total_delay": num(r"Total network delay: (\d+)"),
        "net_router_delay": num(r"Total router delay: (\d+)"),
        "net_link_delay": num(r"Total link delay: (\d+)"),
        "net_inject_delay": num(r"Total inject delay: (\d+)"),
        "dram_accesses": num(r"Total # of DRAM accesses: (\d+)"),
        "total_bus_contention": num(r"Total delay caused by bus contention: (\d+)"),
        "total_num_broadcast": num(r"Total # of broadcast: (-?\d+)"),
    }
    for m in re.finditer(r"LEVEL(\d)=+\n.*?\nThe total # of memory instructions: (\d+)\n"
                         r"The # of cache-missed instructions: (\d+)\nThe # of evicted instructions: (\d+)\n"
                         r"The # of writeback instructions: (\d+)", text, re.S):
        l = m.group(1)
        out[f"L{l}_ins"], out[f"L{l}_miss"], out[f"L{l}_evict"], out[f"L{l}_wb"] = map(int, m.groups()[1:])
    m = re.search(r"Directory Cache=+\n.*?\nThe total # of memory instructions: (\d+)\n"
                  r"The # of cache-missed instructions: (\d+)\nThe # of replaced instructions: (\d+)", text, re.S)
    out["directory_ins"], out["directory_miss"], out["directory_evict"] = map(int, m.groups())
    m = re.search(r"TLB Cache=+\n.*?\nThe total # of TLB access instructions: (\d+)\n"
                  r"The # of cache-missed instructions: (\d+)", text, re.S)
    if m:                                   # system.cpp:990-1009 (tlb_enable)
        out["tlb_ins"], out["tlb_miss"] = map(int, m.groups())
    return out


def counter_stats(counters: dict) -> dict:
    """Map the reference's -Wl,--wrap counters onto pu_stats fields."""
    return {"net_distance": counters["link_visits"], "link_flits": counters["link_flits"],
            "mg1_calls": counters["mg1_calls"], "lockdown_calls": counters["lockdown_calls"],
            "bus_accesses": counters["bus_accesses"], "dram_accesses": counters["dram_accesses"]}


def assert_stats_match(got: dict, case: Case) -> None:
    want = report_stats(case.report)
    want.update(counter_stats(case.counters))
    bad = {k: (got.get(k), v) for k, v in want.items() if got.get(k) != v}
    assert not bad, f"{case.name}: stats differ (engine, reference): {bad}"
