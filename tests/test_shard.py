"""Multi-GPU path on CPU: the loci sharding and timing reduction bench.py uses
(waffle_con_amd/shard.py) with torch.distributed over gloo, world size 2.
Each rank also runs the CPU oracle on its shard, which stands in for the
per-GPU engine. The union of the rank results must equal the single-process
run over all loci."""
import os
import socket

import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from waffle_con_amd import shard  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, loci_per_rank, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        import oracle_ffi as orc
        import waffle_con_amd as w
        seeds = shard.shard_seeds(loci_per_rank, rank)
        with shard.Timer(dist) as tm:
            res = {}
            upd = 0
            for s in seeds:
                r, c = orc.consensus(w.generate_test(4, 200, 6, 0.02, s)[1], counters=True, min_count=2)
                res[s] = [x["sequence"] for x in r]
                upd += c["updates"]
        el, tot_upd, tot_loci = shard.reduce_run(dist, tm.elapsed + rank, upd, len(seeds))
        gathered = [None] * world
        dist.all_gather_object(gathered, res)
        q.put((rank, el, tm.elapsed, tot_upd, tot_loci, upd, gathered))
    finally:
        dist.destroy_process_group()


def test_shard_helpers():
    assert shard.shard_seeds(3, 0) == [0, 1, 2]
    assert shard.shard_seeds(3, 2) == [6, 7, 8]
    items = list(range(10))
    parts = [shard.shard_items(items, r, 3) for r in range(3)]
    assert sum(parts, []) == items and max(map(len, parts)) - min(map(len, parts)) <= 1
    assert shard.reduce_run(None, 1.5, 10, 2) == (1.5, 10.0, 2.0)


def test_gloo_world2_sharded_loci():
    world, per = 2, 3
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, per, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    # every rank sees the max over ranks of its (elapsed + rank)
    expect = max(o[2] + o[0] for o in out)
    assert all(abs(o[1] - expect) < 1e-9 for o in out)
    total_upd = sum(o[5] for o in out)
    assert all(o[3] == total_upd and o[4] == world * per for o in out)
    # disjoint shards covering seeds 0..world*per-1, equal to a single-process run
    merged = {}
    for d in out[0][6]:
        assert not set(d) & set(merged)
        merged.update(d)
    assert sorted(merged) == list(range(world * per))
    import oracle_ffi as orc
    import waffle_con_amd as w
    for s, seqs in merged.items():
        exp = [x["sequence"] for x in orc.consensus(w.generate_test(4, 200, 6, 0.02, s)[1], min_count=2)]
        assert seqs == exp


def test_cost_sorted_assignment_is_a_partition():
    costs = [5, 1, 9, 9, 3, 7, 2, 8, 4, 6, 10, 1]
    for world in (1, 2, 3, 8):
        parts = shard.cost_sorted_assignment(costs, world)
        flat = sorted(i for p in parts for i in p)
        assert flat == list(range(len(costs)))
        # each rank's list is in queue order (non-increasing cost)
        for p in parts:
            assert all(costs[a] >= costs[b] for a, b in zip(p, p[1:]))
        loads = [sum(costs[i] for i in p) for p in parts]
        # LPT bound: max load <= mean + largest item
        assert max(loads) <= sum(costs) / world + max(costs)


def _queue_worker(rank, world, port, n_items, chunk, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from waffle_con_amd import synth
        costs = [synth.cfg5_cost(s) for s in range(n_items)]
        static = shard.cost_sorted_assignment(costs, world)[rank]
        store = dist.distributed_c10d._get_default_store()
        sq = shard.SharedQueue(store, n_items, chunk)
        got = []
        while True:
            c = sq.next_chunk()
            if c is None:
                break
            got.extend(range(*c))
        dist.barrier()
        q.put((rank, static, got))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_cost_sorted_queue():
    """bench.py --workload cfg5 at world size 2: the static cost-sorted (LPT)
    assignment and the store-backed shared queue both hand every locus to
    exactly one rank, with no collective on the data path."""
    world, n, chunk = 2, 37, 4
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_queue_worker, args=(r, world, port, n, chunk, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    static = [o[1] for o in out]
    dyn = [o[2] for o in out]
    assert sorted(static[0] + static[1]) == list(range(n)) and not set(static[0]) & set(static[1])
    assert sorted(dyn[0] + dyn[1]) == list(range(n)) and not set(dyn[0]) & set(dyn[1])


def _bench_cfg5_worker(rank, world, port, total, q):
    """bench.py's cfg5 code path (Cfg5.pregen, Cfg5.step, Cfg5.rank_report) at
    world size 2 over gloo, with the engine call replaced by a recorder."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        import types
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import bench
        a = types.SimpleNamespace(loci=total)
        pre = bench.Cfg5.pregen(a, rank, world)
        C = bench.Cfg5(a, rank, world, None, pre)
        C.chunk = 7  # many pulls
        ran = []

        def fake_run(ids):
            import time
            ran.extend(ids)
            C.last.update((i, None) for i in ids)
            for i in ids:  # as Cfg5._run records them
                C.lat[i] = 0.001 * (i % 7)
                C.done[i] = time.perf_counter() - C.t0 + C.lat[i]
            return {"kernel_ms": 0.0, "updates": len(ids), "w_out": 0, "compares": 0, "launches": 1, "row_bytes": 0}

        C._run = fake_run
        st, n = C.step()
        rep = C.rank_report(dist, None)
        tail = C.tail_report(dist)
        gathered = [None] * world
        dist.all_gather_object(gathered, ran)
        q.put((rank, sorted(pre["loci"]), list(C.static), list(C.tail), gathered, st["updates"], n, rep, tail))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_bench_cfg5_partition():
    """Done-when of the strong-scaling leg: the loci bench.py's cfg5 leg runs
    over 2 ranks (LPT prefix + shared-queue tail) are a disjoint, complete
    partition of the batch, and every rank generated what it ran."""
    world, total = 2, 120
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bench_cfg5_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ran = out[0][4]
    assert not set(ran[0]) & set(ran[1])
    assert sorted(ran[0] + ran[1]) == list(range(total))
    for rank, generated, static, tail, _, upd, n, rep, tl in out:
        assert set(ran[rank]) <= set(generated) and set(static) <= set(ran[rank])
        assert upd == n == len(ran[rank])
        assert rep["rank_loci"] == [len(ran[0]), len(ran[1])]
        # the completion-time quantiles span both ranks' loci; the heaviest
        # locus (largest cost) was found on the rank that ran it
        assert 0 <= tl["t50_s"] <= tl["t95_s"] <= tl["t100_s"]
        assert tl["heaviest_latency_under_load_s"] == 0.001 * (tl["heaviest_locus"] % 7)
    assert out[0][8] == out[1][8]  # every rank reports the same gathered tail
    assert out[0][3] == out[1][3]  # both ranks see the same tail order
