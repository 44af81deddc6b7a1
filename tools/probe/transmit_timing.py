"""Developer probe: wall time of one transmit on one wavefront
(pu_unit_network_run), 32x32 mesh, random routes, 0/64-byte messages, timers
advancing ~2 cycles per message.  Includes launch + copies (small next to
thousands of transmits)."""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from primesim_amd import _abi as A  # noqa: E402
from primesim_amd import uncore as U  # noqa: E402

L = U.lib()
for n, skew in ((2000, 0), (20000, 0), (20000, 400)):
    rng = np.random.default_rng(1)
    src = rng.integers(0, 1024, n).astype(np.int32)
    dst = rng.integers(0, 1024, n).astype(np.int32)
    ln = rng.choice(np.array([0, 64], np.int32), n).astype(np.int32)
    timer = (np.cumsum(rng.integers(0, 4, n)) + rng.integers(0, skew + 1, n)).astype(np.uint64)
    out = np.zeros(n, np.uint64)
    st = A.Stats()
    t0 = time.perf_counter()
    rc = L.pu_unit_network_run(1024, 0, 10, 3, 0, 1, 1, src.ctypes.data, dst.ctypes.data, ln.ctypes.data,
                               timer.ctypes.data, n, out.ctypes.data, C.byref(st), 0)
    el = time.perf_counter() - t0
    hops = max(st.net_distance, 1)
    print(f"n={n} skew={skew} rc={rc} total {el * 1e3:.1f} ms -> {el / n * 1e6:.2f} us/transmit, "
          f"{hops / n:.1f} hops/transmit, M/G/1 share of hops {st.mg1_calls / hops:.2f}", flush=True)
