"""Configurations the GPU tests use besides the golden XMLs and the C1-C5
presets (tools/jit_warm.py compiles them ahead of the GPU run)."""
from __future__ import annotations

import primesim_amd as P
from primesim_amd import config as CF


def hot_link_config():
    """4 cores on a 2x2 mesh (4 links): the M/G/1 helper stress of
    test_gpu_replicas.test_mg1_helper_on_hot_links."""
    return P.config_from_dict(CF.preset("C1", num_cores=4))


def extra_configs():
    return [("hot-link 2x2", hot_link_config())]
