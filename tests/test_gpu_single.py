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
                "nodes_ignored", "peak_queue_size")


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
