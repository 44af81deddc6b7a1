"""TEST ONLY: bench.py's N > 1 path with the GPU engine stubbed out.

Run as `python tests/bench_stub_rank.py --gpus 2 --dist-backend gloo ...`:
bench.main() starts the rank processes itself (launch_ranks, re-running this
file), every rank joins the gloo group, "runs" its replicas on the CPU
restatement of the uncore (oracle.CpuRef, standing in for one GPU's engine:
the same replica seeds, the same C4 stream, a fixed number of requests each),
and bench reduces the timing / request counts and prints the JSON line
exactly as on GPUs.  Rank r reports an elapsed time of 0.5 + r seconds.
PU_STUB_CORRUPT_RANK=k changes one delay of rank k's last kept replica (the
per-rank parity must catch it).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import bench  # noqa: E402

REQS_PER_REPLICA = int(os.environ.get("PU_STUB_REQS", "1500"))
REPLICAS = 2


class StubUM:
    def close(self):
        pass

    def reset(self):
        pass


class StubDevice:
    def __init__(self, args, cfg, threads, rank, local):
        self.cfg, self.threads = cfg, threads
        self.R, self.um, self.dev, self.stream = REPLICAS, StubUM(), None, None
        self.slots = REPLICAS
        self.compiled = 0
        self.compiler = 0

    def headline(self, args, rank, world, keep):
        import oracle as O
        import primesim_amd as P
        from primesim_amd.dist import replica_seed
        delta, rep0, processed, kept = {}, [], 0, {}
        corrupt = os.environ.get("PU_STUB_CORRUPT_RANK")
        for r in range(self.R):
            reqs = P.generate_stream(bench.stream_spec(replica_seed(bench.SEED_BASE, rank, r), REQS_PER_REPLICA))
            eng = O.CpuRef(self.cfg)
            for prog, th in self.threads:
                eng.alloc_core(prog, th)
            d, rc = eng.run(reqs)
            assert rc == 0
            if r == 0:
                rep0.append(d)
            if r in keep:
                kept[r] = d.copy()
                if corrupt is not None and int(corrupt) == rank and r == max(keep):
                    kept[r][len(d) // 2] += 1          # one wrong delay on this rank's last kept replica
            for k, v in eng.stats().as_dict().items():
                if k not in ("error_flags", "num_levels"):
                    delta[k] = delta.get(k, 0) + v
            processed += len(reqs)
        with open(os.path.join(os.environ["PU_STUB_OUT"], f"rank{rank}.txt"), "w") as f:
            f.write(f"{processed} {int(sum(int(x.astype(np.int64).sum()) for x in rep0))}\n")
        return bench.Pass(elapsed=0.5 + rank, kern_ms=[1.0] * args.steps, adv=np.array([REQS_PER_REPLICA] * self.R),
                          kept=kept, delta=delta, halted=0, errf=0, per_replica=None, steps=args.steps,
                          processed=processed, pool=None)

    def reduce_device(self, args):
        return None


bench.Device = StubDevice
bench.LAUNCH_CMD = [sys.executable, os.path.abspath(__file__)]

if __name__ == "__main__":
    bench.main()
