"""Multi-GPU plumbing for the replica engine (one process per GPU).

The uncore of one simulated system is a strictly sequential fold,
so N GPUs run disjoint sets of independent replicas: no collective on the data
path.  The only cross-rank operations are the benchmark's barrier and the
reduction of its timing and request counts (max over ranks of the elapsed
time, sum of requests processed) and the gather of each rank's replica parity
and roofline figures — all here so they can be exercised with the gloo
backend on CPU.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def replica_seed(base: int, rank: int, replica: int) -> int:
    """Seed of replica `replica` on `rank`: disjoint across ranks and replicas
    (a rank holds at most 2^16 replicas)."""
    assert 0 <= replica < (1 << 16)
    return base + (rank << 16) + replica


def reduce_run(elapsed_s: float, processed: int, device: torch.device | None = None) -> tuple[float, int]:
    """(max elapsed over ranks, total requests over ranks); identity when not distributed."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return elapsed_s, processed
    dev = device if device is not None else torch.device("cpu")
    t = torch.tensor([elapsed_s], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    n = torch.tensor([processed], dtype=torch.int64, device=dev)
    dist.all_reduce(n, op=dist.ReduceOp.SUM)
    return float(t.item()), int(n.item())


def gather_objects(obj) -> list:
    """Every rank's `obj` (picklable), in rank order, on every rank; [obj]
    when not distributed (the N>1 bench's per-rank parity and roofline)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out
