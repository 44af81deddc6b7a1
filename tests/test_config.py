"""config_prime XML schema loader vs the reference's XmlParser (xml_parser.cpp)."""
import ctypes as C
import json
import os

import pytest

import primesim_amd as P
from primesim_amd import _abi as A
from primesim_amd import config as CF
from golden_util import GOLDEN, case_names


def _as_dict(cfg):
    """The XmlSim fields (pu_sys_cfg.dram, the opt-in bank model, has no XmlSys counterpart)."""
    def conv(o):
        if isinstance(o, (A.CacheCfg, A.NetCfg, A.SysCfg, A.SimCfg)):
            return {k: conv(getattr(o, k)) for k, _ in o._fields_ if not k.startswith("_") and k != "dram"}
        if hasattr(o, "__len__") and not isinstance(o, (str, bytes)):
            return [conv(x) for x in o]
        return o
    return conv(cfg)


def _strip_unused_levels(d):
    n = d["sys"]["num_levels"]
    d["sys"]["cache"] = d["sys"]["cache"][:n]
    return d


def test_schema_fixtures_match_reference_parser():
    with open(os.path.join(GOLDEN, "configs.json")) as f:
        fx = json.load(f)
    for name, v in fx.items():
        got = _strip_unused_levels(_as_dict(P.parse_config(v["xml"])))
        want = _strip_unused_levels(v["xmlsim"])
        assert got == want, name


@pytest.mark.parametrize("name", case_names())
def test_golden_case_configs(name):
    with open(os.path.join(GOLDEN, f"{name}.json")) as f:
        want = _strip_unused_levels(json.load(f)["xmlsim"])
    got = _strip_unused_levels(_as_dict(P.load_config(os.path.join(GOLDEN, f"{name}.xml"))))
    assert got == want


def test_config_prime_default_values():
    cfg = P.config_from_dict(CF.default_config())
    assert cfg.max_msg_size == 100 and cfg.thread_sync_interval == 1000 and cfg.num_recv_threads == 1
    assert cfg.sys.num_levels == 3 and cfg.sys.num_cores == 64 and cfg.sys.tlb_enable == 1
    assert cfg.sys.cache[2].share == 64 and cfg.sys.directory_cache.size == 31457280
    assert cfg.sys.network.link_delay == 1 and cfg.sys.freq == 2.5


def test_optional_fields_default_to_zero():
    sim = CF.preset("C1")
    del sim["system"]["max_num_sharers"]
    del sim["system"]["network"]["inject_delay"]
    cfg = P.config_from_dict(sim)
    assert cfg.sys.max_num_sharers == 0 and cfg.sys.network.inject_delay == 0


@pytest.mark.parametrize("mutate", [
    lambda s: s.pop("max_msg_size"),                               # simulator count 4 != 5
    lambda s: s["system"].pop("freq"),                             # system count 12 != 13
    lambda s: s["system"]["network"].pop("data_width"),            # network count 3 != 4
    lambda s: s["system"]["directory_cache"].pop("num_ways"),      # directory 5 != 6
    lambda s: s["system"].pop("tlb_cache"),                        # //tlb_cache missing
    lambda s: s["system"]["cache"].pop(),                          # //cache count != num_levels
])
def test_schema_errors_are_reported(mutate):
    sim = CF.default_config()
    mutate(sim)
    with pytest.raises(P.UncoreError):
        P.config_from_dict(sim)


def test_malformed_xml():
    with pytest.raises(P.UncoreError):
        P.parse_config("<simulator><max_msg_size>1</simulator>")


def test_numeric_parse_semantics():
    """`stringstream >> dec >> v`: leading blanks skipped, numeric prefix taken."""
    xml = CF.to_xml(CF.preset("C1")).replace("<num_cores>16</num_cores>", "<num_cores>\n   16abc </num_cores>")
    assert P.parse_config(xml).sys.num_cores == 16


def test_write_xml_round_trip():
    import ctypes as C
    cfg = P.config_from_dict(CF.preset("C3"))
    n = C.c_size_t(0)
    buf = C.create_string_buffer(1 << 16)
    assert P.uncore.lib().pu_config_write_xml(C.byref(cfg), buf, len(buf), C.byref(n)) == 0
    again = P.parse_config(buf.value.decode())
    assert _as_dict(again) == _as_dict(cfg)


def test_dram_bank_element_round_trip():
    """The optional <dram> element (pu_dram_cfg) parses, is written back only
    when banks > 0, and malformed or partial elements are refused."""
    sim = CF.default_config()
    assert P.config_from_dict(sim).sys.dram.banks == 0
    sim["system"]["dram"] = {"banks": 16, "row_bytes": 8192, "t_rcd": 14, "t_rp": 14, "t_burst": 4}
    cfg = P.config_from_dict(sim)
    d = cfg.sys.dram
    assert (d.banks, d.row_bytes, d.t_rcd, d.t_rp, d.t_burst) == (16, 8192, 14, 14, 4)
    buf, n = C.create_string_buffer(1 << 16), C.c_size_t(0)
    assert P.uncore.lib().pu_config_write_xml(C.byref(cfg), buf, len(buf), C.byref(n)) == 0
    text = buf.value.decode()
    assert "<dram>" in text and P.parse_config(text).sys.dram.row_bytes == 8192
    del sim["system"]["dram"]["t_rp"]
    with pytest.raises(P.UncoreError):
        P.config_from_dict(sim)
