"""Configuration in the reference's config_prime schema.

`default_config()` reproduces the dictionaries of reference tools/config_prime
(network :62-75, cache :78-120, directory_cache :124-134, tlb_cache :138-148,
system :151-186, simulator :189-199); `write_xml()` emits the same layout as
its print_dict writer (:39-54).  `preset()` builds the C1-C5 shapes of
SURVEY.md §8d.
"""
from __future__ import annotations

import copy
from typing import Any

# Key order follows the reference dictionaries so the XML reads the same.
NETWORK = {
    "net_type": 0, "data_width": 10, "header_flits": 3,
    "router_delay": 0, "link_delay": 1, "inject_delay": 1,
}

CACHE = [
    {"level": 0, "share": 1, "access_time": 1, "size": 32768, "block_size": 64, "num_ways": 8},
    {"level": 1, "share": 1, "access_time": 5, "size": 262144, "block_size": 64, "num_ways": 8},
    {"level": 2, "share": 64, "access_time": 10, "size": 4194304, "block_size": 64, "num_ways": 16},
]

DIRECTORY_CACHE = {"level": 0, "share": 1, "access_time": 10, "size": 31457280, "block_size": 64, "num_ways": 24}

TLB_CACHE = {"level": 0, "share": 1, "access_time": 0, "size": 64, "block_size": 1, "num_ways": 64}

SYSTEM = {
    "dram_access_time": 120, "num_levels": 3, "cpi_nonmem": 1, "num_cores": 64, "sys_type": 0,
    "protocol_type": 0, "max_num_sharers": 6, "page_size": 4096, "tlb_enable": 1, "shared_llc": 0,
    "verbose_report": 1, "freq": 2.5, "bus_latency": 2, "page_miss_delay": 200,
}

SIMULATOR = {
    "max_msg_size": 100, "thread_sync_interval": 1000, "proc_sync_interval": 10000,
    "syscall_cost": 10000, "num_recv_threads": 1,
}


def default_config() -> dict[str, Any]:
    """The config_prime default configuration as a nested dict."""
    sys_ = dict(SYSTEM)
    sys_["network"] = dict(NETWORK)
    sys_["cache"] = copy.deepcopy(CACHE)
    sys_["directory_cache"] = dict(DIRECTORY_CACHE)
    sys_["tlb_cache"] = dict(TLB_CACHE)
    sim = dict(SIMULATOR)
    sim["system"] = sys_
    return sim


def _print_dict(out: list[str], d: dict, ident: str = "    ") -> None:
    for key, value in d.items():
        if isinstance(value, list):
            for item in value:
                if isinstance(item, dict):
                    out.append(f"{ident}<{key}>\n")
                    _print_dict(out, item, ident + "   ")
                    out.append(f"{ident}</{key}>\n")
        elif isinstance(value, dict):
            out.append(f"{ident}<{key}>\n")
            _print_dict(out, value, ident + "   ")
            out.append(f"{ident}</{key}>\n")
        else:
            out.append(f"{ident}<{key}>{value}</{key}>\n")


def to_xml(sim: dict[str, Any]) -> str:
    out = ['<?xml version = "1.0" encoding = "utf-8" standalone = "yes"?>\n\n', "<simulator>\n"]
    _print_dict(out, sim)
    out.append("</simulator>\n")
    return "".join(out)


def write_xml(sim: dict[str, Any], path: str) -> str:
    with open(path, "w") as f:
        f.write(to_xml(sim))
    return path


def preset(name: str, **overrides: Any) -> dict[str, Any]:
    """SURVEY.md §8d shapes.

    C1  16 cores 4x4,  L1 + shared-LLC slice 256 KB/8 W
    C2  64 cores 8x8,  same shape
    C3  256 cores 16x16, private L1 + private L2 256 KB/8 W/5 cyc, LLC slice 1 MB/16 W
    C4  1024 cores 32x32, C1 shape
    C5  4096 cores 64x64, C1 shape
    Common: directory protocol, full map, TLB off, verbose_report 0.
    `overrides` may set any system key (e.g. protocol_type=1) or
    `dir_size`/`dir_ways`/`dir_access_time`.
    """
    cores = {"C1": 16, "C2": 64, "C3": 256, "C4": 1024, "C5": 4096}[name]
    sim = default_config()
    s = sim["system"]
    s.update({"num_cores": cores, "sys_type": 0, "protocol_type": 0, "max_num_sharers": 6,
              "tlb_enable": 0, "shared_llc": 1, "verbose_report": 0})
    l1 = {"level": 0, "share": 1, "access_time": 1, "size": 32768, "block_size": 64, "num_ways": 8}
    if name == "C3":
        l2 = {"level": 1, "share": 1, "access_time": 5, "size": 262144, "block_size": 64, "num_ways": 8}
        s["cache"] = [l1, l2]
        s["num_levels"] = 2
        s["directory_cache"] = {"level": 0, "share": 1, "access_time": 10, "size": 1 << 20,
                                "block_size": 64, "num_ways": 16}
    else:
        s["cache"] = [l1]
        s["num_levels"] = 1
        s["directory_cache"] = {"level": 0, "share": 1, "access_time": 10, "size": 262144,
                                "block_size": 64, "num_ways": 8}
    dir_keys = {"dir_size": "size", "dir_ways": "num_ways", "dir_access_time": "access_time"}
    for k, v in overrides.items():
        if k in dir_keys:
            s["directory_cache"][dir_keys[k]] = v
        elif k in SIMULATOR:
            sim[k] = v
        elif k in s["network"]:
            s["network"][k] = v
        else:
            s[k] = v
    return sim
