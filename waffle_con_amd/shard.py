"""Loci sharding across GPUs (loci-sharded mode).

Consensus problems are independent, so every rank owns a disjoint slice of
the loci. The data path has no collective. torch.distributed is used only
for the start/stop barrier and for the max-over-ranks reduction of the timed
region. On GPUs that runs over RCCL. The CPU tests use gloo with the same code.
"""
import time


def shard_seeds(loci_per_rank, rank):
    """Weak scaling: rank r owns seeds [r*loci, (r+1)*loci) (seed = locus id)."""
    return list(range(rank * loci_per_rank, (rank + 1) * loci_per_rank))


def shard_items(items, rank, world):
    """Strong-scaling split of a fixed item list: contiguous, sizes differ by <= 1."""
    n = len(items)
    lo = rank * n // world
    hi = (rank + 1) * n // world
    return items[lo:hi]


def barrier(dist, sync=None):
    if sync is not None:
        sync()
    if dist is not None:
        dist.barrier()


def reduce_run(dist, elapsed, updates, loci, device=None):
    """Max of the per-rank elapsed times; sums of the work done.

    Returns (elapsed_max, total_updates, total_loci). With dist None this is
    the single-process identity.
    """
    if dist is None:
        return float(elapsed), float(updates), float(loci)
    import torch
    t = torch.tensor([float(elapsed)], dtype=torch.float64, device=device)
    w = torch.tensor([float(updates), float(loci)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(w, op=dist.ReduceOp.SUM)
    return t[0].item(), w[0].item(), w[1].item()


class Timer:
    """Barrier + device sync on both sides of the timed region."""

    def __init__(self, dist, sync=None):
        self.dist, self.sync = dist, sync

    def __enter__(self):
        barrier(self.dist, self.sync)
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        barrier(self.dist, self.sync)
        self.elapsed = time.perf_counter() - self.t0
        return False
