"""GPU parity of the submission service (wc_service_*, csrc/service.cpp): the
reference's per-locus API (ConsensusDWFA / DualConsensusDWFA.consensus(),
consensus.rs:139, dual_consensus.rs:240) called from many threads at once.
Every result must equal the oracle's, whichever lane or path served it."""
import threading

import pytest

import oracle_ffi as orc

pytestmark = pytest.mark.gpu

w = pytest.importorskip("waffle_con_amd")
hip = pytest.importorskip("hip_runner")


def _gen(L, N, err, seed):
    return w.generate_test(4, L, N, err, seed)[1]


def _run_threads(jobs, nthreads):
    """jobs: list of callables; returns their results in order (exceptions re-raised)."""
    out = [None] * len(jobs)
    err = []
    nxt = [0]
    lock = threading.Lock()

    def worker():
        while True:
            with lock:
                i = nxt[0]
                nxt[0] += 1
            if i >= len(jobs):
                return
            try:
                out[i] = jobs[i]()
            except Exception as e:  # noqa: BLE001
                err.append(e)
                return

    th = [threading.Thread(target=worker) for _ in range(nthreads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if err:
        raise err[0]
    return out


def _stats():
    from waffle_con_amd import _lib
    return _lib.service().stats()


def test_threaded_single_calls_match_oracle():
    loci = [_gen(1200, 16, 0.02, 100 + s) for s in range(48)]
    s0 = _stats()
    got = _run_threads([lambda p=p: hip.consensus(p, counters=True, min_count=4) for p in loci], 24)
    s1 = _stats()
    for p, (g, gc) in zip(loci, got):
        e, ec = orc.consensus(p, counters=True, min_count=4)
        assert g == e
        for k in ("updates", "w_out", "compares", "ed_increases", "finalizes", "pops", "nodes_explored"):
            assert gc[k] == ec[k], k
    from waffle_con_amd import _lib
    print("service stats before", s0, "after", s1, "last error", _lib.service().last_error())
    assert s1["served"] - s0["served"] == len(loci), _lib.service().last_error()


def test_threaded_dual_calls_match_oracle():
    def mix(s):
        a, b = _gen(600, 10, 0.01, 2 * s), _gen(600, 10, 0.01, 2 * s + 1)
        return [x for pair in zip(a, b) for x in pair]
    loci = [mix(200 + s) for s in range(12)]
    got = _run_threads([lambda p=p: hip.dual_consensus(p, min_count=3) for p in loci], 12)
    for p, g in zip(loci, got):
        assert g == orc.dual_consensus(p, min_count=3)


def test_mixed_configs_and_kinds_concurrently():
    """Different CdwfaConfigs and both engines at once: one lane each."""
    single = [_gen(800, 12, 0.03, 300 + s) for s in range(16)]
    jobs, exp = [], []
    for i, p in enumerate(single):
        kw = dict(min_count=3) if i % 2 else dict(min_count=4, consensus_cost=1)
        jobs.append(lambda p=p, kw=kw: hip.consensus(p, **kw))
        exp.append(orc.consensus(p, **kw))
    a, b = _gen(500, 8, 0.01, 41), _gen(500, 8, 0.01, 42)
    mix = [x for pair in zip(a, b) for x in pair]
    jobs.append(lambda: hip.dual_consensus(mix, min_count=2))
    exp.append(orc.dual_consensus(mix, min_count=2))
    assert _run_threads(jobs, 17) == exp


def test_larger_problem_restarts_the_lane():
    """A lane planned for small loci drains and restarts for a larger one."""
    small = [_gen(400, 8, 0.02, 500 + s) for s in range(6)]
    big = _gen(3000, 40, 0.01, 77)
    jobs = [lambda p=p: hip.consensus(p, min_count=2) for p in small] + [lambda: hip.consensus(big, min_count=2)]
    got = _run_threads(jobs, 7)
    assert got == [orc.consensus(p, min_count=2) for p in small + [big]]


def test_offsets_and_deep_problems_take_the_batch_path():
    base = _gen(700, 10, 0.02, 61)
    offs = [None] * 8 + [100, 150]
    s0 = _stats()
    assert hip.consensus(base, offsets=offs, min_count=3) == orc.consensus(base, offsets=offs, min_count=3)
    s1 = _stats()
    assert s1["fallback"] - s0["fallback"] == 1


def test_service_off_uses_per_call_launches(monkeypatch):
    monkeypatch.setenv("WAFFLE_CON_SERVICE", "0")
    p = _gen(600, 10, 0.02, 9)
    s0 = _stats()
    assert hip.consensus(p, min_count=3) == orc.consensus(p, min_count=3)
    assert _stats()["calls"] == s0["calls"]


def test_threaded_priority_calls_match_oracle():
    """PriorityConsensusDWFA.consensus() from many threads at once
    (wc_service_priority_consensus: each caller unwinds its own LIFO stack, the
    dual sub-problems share the service's lanes): results and every counter
    equal the oracle's."""
    from waffle_con_amd import synth
    loci = [synth.cfg5_locus(s) for s in range(10)]
    s0 = _stats()
    got = _run_threads([lambda ch=ch: hip.priority_consensus(ch, counters=True, wildcard=ord("*")) for ch in loci], 10)
    s1 = _stats()
    for ch, (g, gc) in zip(loci, got):
        e, ec = orc.priority_consensus(ch, counters=True, wildcard=ord("*"))
        assert g == e
        for k in ("updates", "w_out", "compares", "ed_increases", "finalizes", "pops", "nodes_explored",
                  "nodes_ignored", "peak_queue_size"):
            assert gc[k] == ec[k], k
    assert s1["served"] > s0["served"]


def test_priority_call_with_offsets_and_seed_groups():
    """Sub-problems with offsets take the batch path on the service thread;
    seed groups fix the root order (priority_consensus.rs:180)."""
    from waffle_con_amd import synth
    chains = synth.cfg5_locus(3)
    offs = [[None, None if i % 3 else 10 + i] for i in range(len(chains))]
    groups = [i % 3 if i % 4 else None for i in range(len(chains))]
    kw = dict(wildcard=ord("*"))
    s0 = _stats()
    got = hip.priority_consensus(chains, offsets=offs, seed_groups=groups, **kw)
    assert got == orc.priority_consensus(chains, offsets=offs, seed_groups=groups, **kw)
    assert _stats()["fallback"] > s0["fallback"]


def test_batch_path_requests_under_lane_traffic():
    """Offsets and > 256-read problems (the batch path, run by the service
    thread while no lane runs) mixed with steady lane traffic from many
    threads: every result equals the oracle's and the batch-path count is
    exactly the number of such calls."""
    plain = [_gen(900, 12, 0.02, 700 + s) for s in range(40)]
    base = _gen(700, 10, 0.02, 61)
    offs = [None] * 8 + [100, 150]
    deep = _gen(300, 300, 0.01, 62)
    jobs, exp = [], []
    for i, p in enumerate(plain):
        jobs.append(lambda p=p: hip.consensus(p, min_count=3))
        exp.append(orc.consensus(p, min_count=3))
        if i % 10 == 5:
            jobs.append(lambda: hip.consensus(base, offsets=offs, min_count=3))
            exp.append(orc.consensus(base, offsets=offs, min_count=3))
        if i % 20 == 9:
            jobs.append(lambda: hip.consensus(deep, min_count=50))
            exp.append(orc.consensus(deep, min_count=50))
    s0 = _stats()
    assert _run_threads(jobs, 16) == exp
    s1 = _stats()
    assert s1["fallback"] - s0["fallback"] == 4 + 2


def test_destroy_during_threaded_priority_calls():
    """wc_service_destroy while PriorityConsensusDWFA calls are inside: the
    calls already in submit further sub-problems (and retries) after stop is
    set; the service thread keeps serving them until the last one leaves, so
    every such call completes with the oracle's result and destroy returns.
    Calls that start after stop are refused (WC_E_HIP)."""
    import time
    from waffle_con_amd import _lib, synth
    from waffle_con_amd.cdwfa_config import CdwfaConfig
    from waffle_con_amd.priority_consensus import priority_service_call
    cfg = CdwfaConfig(wildcard=ord("*"))
    svc = _lib.Service(0)
    loci = [synth.cfg5_locus(s) for s in (20, 21, 22, 23)]
    out, refused, errors = [None] * len(loci), [], []

    def call(i):
        try:
            (r,), _ = priority_service_call(([list(map(bytes, ch)) for ch in loci[i]], None, None), cfg,
                                            svc=svc)
            out[i] = {"consensuses": [[hip._cons(c) for c in chain] for chain in r.consensuses()],
                      "sequence_indices": list(r.sequence_indices())}
        except _lib.WaffleConError as e:
            refused.append((i, e))
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=call, args=(i,)) for i in range(len(loci))]
    for t in th:
        t.start()
    time.sleep(0.5)  # the calls are inside, with sub-problems to go
    t0 = time.time()
    svc.close()
    t_destroy = time.time() - t0
    for t in th:
        t.join(60)
        assert not t.is_alive(), "a priority call hung across wc_service_destroy"
    assert not errors, errors
    done = [i for i in range(len(loci)) if out[i] is not None]
    assert len(done) + len(refused) == len(loci)
    assert done, "no call was inside the service when it was destroyed"
    for i in done:
        assert out[i] == orc.priority_consensus(loci[i], wildcard=ord("*"))
    print("destroy took %.2f s, %d calls completed, %d refused" % (t_destroy, len(done), len(refused)))
