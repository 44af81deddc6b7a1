"""N>1 path on CPU: world_size-2 gloo processes each run their own replicas
(here through the CPU restatement, standing in for one GPU's engine) and
reduce timing/request counts exactly as bench.py does."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    import oracle as O
    import primesim_amd as P
    from primesim_amd import _abi as A
    from primesim_amd import config as CF
    from primesim_amd.dist import reduce_run, replica_seed

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = P.config_from_dict(CF.preset("C1"))
    digests, processed = [], 0
    for r in range(2):
        spec = P.StreamSpec(A.PU_STREAM_UNIFORM_HOTSPOT, 16, seed=replica_seed(4, rank, r), max_requests=500)
        reqs = P.generate_stream(spec)
        eng = O.CpuRef(cfg)
        for prog, th in P.stream_threads(spec):
            eng.alloc_core(prog, th)
        d, rc = eng.run(reqs)
        assert rc == 0
        digests.append(int(d.astype(np.int64).sum()))
        processed += len(reqs)
    elapsed = 1.0 + rank   # rank 1 is the slow one
    t, n = reduce_run(elapsed, processed)
    out[rank] = (t, n, processed, tuple(digests))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_reduction():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    (t0, n0, p0, d0), (t1, n1, p1, d1) = out[0], out[1]
    assert t0 == t1 == 2.0                 # max over ranks
    assert n0 == n1 == p0 + p1             # whole-job request count
    assert d0 != d1                        # ranks simulate disjoint replicas
