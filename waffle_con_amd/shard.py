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


def locus_cost(reads):
    """Estimated cost of one locus (~ N reads x L length): the
    sum over its reads of the read length (chains: every level), i.e. reads x
    length. Measured on 2,000 cfg5 loci (tools/cfg5_lat.py),
    this ranks a locus's critical-path pops better than the work estimate
    reads^2 x length (Spearman 0.875 vs 0.785), and under strong scaling the
    longest critical paths are what must start first."""
    tot = 0
    for r in reads:
        tot += sum(len(x) for x in r) if isinstance(r, (list, tuple)) else len(r)
    return tot


def cost_sorted_assignment(costs, world):
    """Strong scaling of a fixed item list over `world` ranks without any
    communication: items are taken longest-first (the cost-sorted queue of
    SURVEY §8(e)) and each goes to the rank with the least cost so far (LPT;
    ties to the lowest rank). Every rank computes the same assignment.
    Returns one list of item indices per rank, each in queue order."""
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    load = [0] * world
    out = [[] for _ in range(world)]
    for i in order:
        r = min(range(world), key=lambda k: (load[k], k))
        out[r].append(i)
        load[r] += costs[i]
    return out


def prefix_tail_plan(costs, world, prefix_frac=0.75):
    """Strong scaling of a fixed item list: the cost-sorted order (longest
    first) is cut into a heavy prefix holding `prefix_frac` of the total cost,
    assigned statically by LPT (cost_sorted_assignment; every rank computes the
    same split), and the light tail, which ranks pull in chunks through a
    SharedQueue as they run out of work. Returns (per-rank prefix item lists in
    queue order, the tail item list in queue order)."""
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    target = prefix_frac * sum(costs)
    k, cum = 0, 0
    while k < len(order) and (cum < target or k < world):
        cum += costs[order[k]]
        k += 1
    prefix, tail = order[:k], order[k:]
    static = cost_sorted_assignment([costs[i] for i in prefix], world)
    return [[prefix[j] for j in part] for part in static], tail


class LocalStore:
    """In-process stand-in for the process group's store (world size 1)."""

    def __init__(self):
        self.v = {}

    def add(self, key, n):
        self.v[key] = self.v.get(key, 0) + n
        return self.v[key]


class SharedQueue:
    """Dynamic form of the cost-sorted queue: ranks pull chunks of a fixed,
    cost-sorted item order through an atomic counter in the process group's
    store (TCPStore add = fetch-and-add). No collective touches the data path."""

    def __init__(self, store, n_items, chunk, key="wc_queue"):
        self.store, self.n, self.chunk, self.key = store, n_items, max(1, chunk), key

    def next_chunk(self):
        end = self.store.add(self.key, self.chunk)
        start = end - self.chunk
        if start >= self.n:
            return None
        return start, min(end, self.n)


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
