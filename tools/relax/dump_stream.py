"""Dump a synthetic stream + the CPU restatement's delays for the relaxation prototype.

usage: python tools/relax/dump_stream.py PRESET KIND SEED NREQ OUT_PREFIX
Writes OUT_PREFIX.req (pu_req records) and OUT_PREFIX.delay (int32).
Research tooling only (uses the oracle as the checker)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import primesim_amd as P  # noqa: E402
from primesim_amd import _abi as A  # noqa: E402
from primesim_amd import config as CF  # noqa: E402
import oracle as O  # noqa: E402

preset, kind, seed, nreq, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
sim = CF.preset(preset)
cfg = P.config_from_dict(sim)
cores = cfg.sys.num_cores
spec = P.StreamSpec(kind=kind, num_cores=cores, seed=seed, num_quanta=max(1, nreq // (cores * 300) + 2),
                    max_requests=nreq)
reqs = P.generate_stream(spec)
ref = O.CpuRef(cfg)
for prog, thread in P.stream_threads(spec):
    ref.alloc_core(prog, thread)
d, rc = ref.run(reqs)
print("requests", len(reqs), "rc", rc, "mean delay", float(d.mean()))
reqs.tofile(out + ".req")
d.astype(np.int32).tofile(out + ".delay")
