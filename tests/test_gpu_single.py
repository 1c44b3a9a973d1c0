"""GPU parity: ConsensusDWFA on the HIP engine vs the reference's golden
vectors and vs the CPU oracle (bit-exact sequences, scores and work counters)."""
import pytest

import oracle_ffi as orc
import ref_cases as rc

pytestmark = pytest.mark.gpu

hip = pytest.importorskip("hip_runner")

@pytest.mark.parametrize("name", sorted(rc.SINGLE_CASES))
def test_reference_single(name):
    rc.check_single(rc.SINGLE_CASES[name], hip)


COUNTER_KEYS = ("updates", "w_out", "compares", "ed_increases", "finalizes", "pops", "nodes_explored",
                "nodes_ignored", "peak_queue_size", "row_bytes")


def _gen(L, N, err, seed):
    import waffle_con_amd as w
    return w.generate_test(4, L, N, err, seed)[1]


@pytest.mark.parametrize("L,N,err,seed", [(1000, 30, 0.01, 0), (1000, 8, 0.02, 0), (300, 8, 0.05, 1),
                                          (2000, 12, 0.03, 2), (500, 5, 0.08, 3)])
def test_example_gen_vs_oracle(L, N, err, seed):
    seqs = _gen(L, N, err, seed)
    cfg = dict(min_count=max(1, N // 4))
    exp, ec = orc.consensus(seqs, counters=True, **cfg)
    got, gc = hip.consensus(seqs, counters=True, **cfg)
    assert got == exp
    for k in COUNTER_KEYS:
        assert gc[k] == ec[k], (k, gc[k], ec[k])


def test_batch_matches_individual():
    probs = [_gen(400, 10, 0.04, s) for s in range(12)]
    cfg = dict(min_count=2)
    got = hip.consensus_batch(probs, **cfg)
    for p, g in zip(probs, got):
        assert g == orc.consensus(p, **cfg)


@pytest.mark.parametrize("chain", ["0", "2", "5", "16", "31", "40"])
@pytest.mark.parametrize("L,N,err,seed", [(1500, 20, 0.01, 11), (800, 12, 0.04, 12), (600, 9, 0.08, 13)])
def test_chain_length_invariance(chain, L, N, err, seed, monkeypatch):
    """The linear-chain run-ahead (WC_CHAIN = max steps, 0 = off) must not
    change results or work counters: every length is bit-exact vs the oracle."""
    monkeypatch.setenv("WC_CHAIN", chain)
    seqs = _gen(L, N, err, seed)
    cfg = dict(min_count=max(1, N // 4))
    exp, ec = orc.consensus(seqs, counters=True, **cfg)
    got, gc = hip.consensus(seqs, counters=True, **cfg)
    assert got == exp
    for k in COUNTER_KEYS:
        assert gc[k] == ec[k], (k, gc[k], ec[k])


@pytest.mark.parametrize("chain", ["2", "5", "16", "31", "40"])
@pytest.mark.parametrize("L,N,err,seed", [(1500, 20, 0.01, 11), (800, 12, 0.04, 12), (600, 9, 0.08, 13)])
def test_chain_length_invariance_cu(chain, L, N, err, seed, monkeypatch):
    """The same on the 1024-thread single engine (engine_cu.hip, WC_CU=1),
    whose chain walk spreads reads over 16 waves: per-call batch path on the
    default context, whose engine mask must show that build ran."""
    from waffle_con_amd import _lib
    monkeypatch.setenv("WAFFLE_CON_SERVICE", "0")
    monkeypatch.setenv("WC_CU", "1")
    monkeypatch.setenv("WC_CHAIN", chain)
    _lib.default_context().engines_used(reset=True)
    seqs = _gen(L, N, err, seed)
    cfg = dict(min_count=max(1, N // 4))
    exp, ec = orc.consensus(seqs, counters=True, **cfg)
    got, gc = hip.consensus(seqs, counters=True, **cfg)
    assert _lib.default_context().engines_used(reset=True) == ["cu.single"]
    assert got == exp
    for k in COUNTER_KEYS:
        assert gc[k] == ec[k], (k, gc[k], ec[k])


def test_failed_refill_leaves_the_batch_usable():
    """host.cpp upload_batch is transactional: a refill rejected by validation
    changes nothing, so the batch still runs its previous problems."""
    import ctypes
    import waffle_con_amd as w
    from waffle_con_amd import _lib
    probs = [_gen(300, 8, 0.03, s) for s in range(4)]
    b = w.ResidentBatch(probs)
    exp, _ = b.consensus(w.CdwfaConfig(min_count=2))
    exp = [[(c.sequence(), c.scores()) for c in r] for r in exp]
    bad = (_lib.WcProblem * 1)()
    bad[0].n_reads = 1
    ptrs = (_lib._u8p * 1)()  # a null read pointer with a non-zero length
    lens = (ctypes.c_uint64 * 1)(5)
    bad[0].reads = ptrs
    bad[0].lens = lens
    rc = _lib.lib().wc_batch_refill(b.ctx.handle, b.handle, 1, bad)
    assert rc == _lib.WC_E_BAD_INPUT
    got, _ = b.consensus(w.CdwfaConfig(min_count=2))
    assert [[(c.sequence(), c.scores()) for c in r] for r in got] == exp
    b.close()


def test_batch_results_pickle_after_the_batch_is_gone():
    import copy
    import gc
    import pickle
    import waffle_con_amd as w
    probs = [_gen(300, 8, 0.03, s) for s in range(3)]
    res, _ = w.consensus_batch(probs, w.CdwfaConfig(min_count=2))
    blobs = [pickle.dumps(r) for r in res]
    dup = copy.deepcopy(res)
    del res
    gc.collect()
    for p, blob, d in zip(probs, blobs, dup):
        exp = orc.consensus(p, min_count=2)
        assert [{"sequence": c.sequence(), "scores": list(c.scores())} for c in pickle.loads(blob)] == exp
        assert [{"sequence": c.sequence(), "scores": list(c.scores())} for c in d] == exp
