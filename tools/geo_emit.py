"""Write one configuration's compile-time geometry (pu_config_geo_source) to a
header, for fixed-geometry tool builds of the engine (profiling, experiments):

    python tools/geo_emit.py C4 build/geo_c4.h
    tools/build_exp.sh c4prof "-DPU_PROF -DPU_FIXED_GEO=\\"$PWD/build/geo_c4.h\\""
"""
from __future__ import annotations

import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    import primesim_amd as P
    from primesim_amd import config as CF
    from primesim_amd import uncore
    preset, out = sys.argv[1], sys.argv[2]
    cfg = P.config_from_dict(CF.preset(preset))
    buf = C.create_string_buffer(1 << 16)
    n = uncore.lib().pu_config_geo_source(C.byref(cfg), buf, len(buf))
    if n <= 0:
        raise SystemExit(f"pu_config_geo_source failed ({n})")
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    with open(out, "w") as f:
        f.write(buf.value.decode())
    print(f"{out}: {n} bytes")


if __name__ == "__main__":
    main()
