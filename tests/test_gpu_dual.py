"""GPU parity: DualConsensusDWFA and PriorityConsensusDWFA on the HIP engine
vs the reference's golden vectors (tests + CSV fixtures) and vs the oracle."""
import pytest

import oracle_ffi as orc
import ref_cases as rc

pytestmark = pytest.mark.gpu
hip = pytest.importorskip("hip_runner")

@pytest.mark.parametrize("name", sorted(rc.DUAL_CASES))
def test_reference_dual(name):
    rc.check_dual(rc.DUAL_CASES[name], hip)


@pytest.mark.parametrize("name", sorted(rc.PRIORITY_CASES))
def test_reference_priority(priority_path, name):
    rc.check_priority(rc.PRIORITY_CASES[name], hip)


@pytest.mark.parametrize("name", sorted(rc.DUAL_CASES))
def test_dual_vs_oracle_full_equality(name):
    """Beyond the reference's PartialEq: scores1/scores2 and work counters too."""
    case = rc.DUAL_CASES[name]
    seqs = [rc.b(s) for s in case["seqs"]]
    offs = case.get("offsets")
    if "error" in case:
        with pytest.raises(Exception) as eo:
            orc.dual_consensus(seqs, offsets=offs, **case["cfg"])
        with pytest.raises(Exception) as eh:
            hip.dual_consensus(seqs, offsets=offs, **case["cfg"])
        assert str(eh.value) == str(eo.value)
        return
    exp, ec = orc.dual_consensus(seqs, offsets=offs, counters=True, **case["cfg"])
    got, gc = hip.dual_consensus(seqs, offsets=offs, counters=True, **case["cfg"])
    assert got == exp
    for k in ("updates", "w_out", "compares", "ed_increases", "finalizes", "pops", "nodes_explored",
              "nodes_ignored", "peak_queue_size", "row_bytes"):
        assert gc[k] == ec[k], (k, gc[k], ec[k])


def _two_haplotypes(L, n_each, err, seed, n_var=3):
    import random
    import waffle_con_amd as w
    rng = random.Random(seed)
    con, _ = w.generate_test(4, L, 1, 0.0, seed)
    a = bytearray(b"ACGT"[x] for x in con)
    bb = bytearray(a)
    for _ in range(n_var):
        p = rng.randrange(5, L - 5)
        bb[p] = b"ACGT"[(b"ACGT".index(bb[p]) + 1) % 4]
    reads = []
    for hap in (bytes(a), bytes(bb)):
        for _ in range(n_each):
            r = bytearray()
            for ch in hap:
                x = rng.random()
                if x < err / 3:
                    continue
                if x < 2 * err / 3:
                    r.append(rng.choice(b"ACGT"))
                r.append(ch if x >= err or x < 2 * err / 3 else rng.choice(b"ACGT"))
            reads.append(bytes(r))
    return reads


@pytest.mark.parametrize("seed", range(6))
def test_dual_synthetic_vs_oracle(seed):
    reads = _two_haplotypes(120, 6, 0.02, seed)
    cfg = dict(min_count=3)
    exp = orc.dual_consensus(reads, **cfg)
    got = hip.dual_consensus(reads, **cfg)
    assert got == exp


@pytest.mark.parametrize("seed", range(3))
def test_dual_weighted_l2_vs_oracle(seed):
    reads = _two_haplotypes(80, 5, 0.03, 100 + seed)
    cfg = dict(min_count=2, weighted_by_ed=True, consensus_cost=1, dual_max_ed_delta=4)
    assert hip.dual_consensus(reads, **cfg) == orc.dual_consensus(reads, **cfg)


@pytest.mark.parametrize("seed", range(3))
def test_priority_synthetic_vs_oracle(priority_path, seed):
    reads = _two_haplotypes(100, 5, 0.01, 200 + seed)
    chains = [[r, r[: len(r) // 2]] for r in reads]
    cfg = dict(min_count=3, wildcard=ord("*"))
    assert hip.priority_consensus(chains, **cfg) == orc.priority_consensus(chains, **cfg)


@pytest.mark.parametrize("seed", range(3))
def test_cfg4_shape_length_gaps_vs_oracle(seed):
    # SURVEY §8(d) cfg4 shape, scaled down (4 haplotypes with inserted
    # segments of different lengths, grouped reads) through the multi-split
    # PriorityConsensusDWFA with the priority tests' wildcard config
    from waffle_con_amd import synth
    reads = synth.cfg4_locus(300 + seed, length=500, reads=5, err=0.01, gaps=(0, 4, 9, 20))
    chains = [[r] for r in reads]
    cfg = dict(min_count=3, wildcard=ord("*"))
    assert hip.priority_consensus(chains, **cfg) == orc.priority_consensus(chains, **cfg)


@pytest.mark.parametrize("seed", range(4))
def test_cfg5_shape_hpc_chains_vs_oracle(seed):
    # SURVEY §8(d) cfg5 shape, scaled down: [HPC(read), read] chains
    from waffle_con_amd import synth
    chains = synth.cfg5_locus(400 + seed, len_range=(200, 500), reads_range=(4, 7), err=0.01, max_variants=6)
    cfg = dict(min_count=3, wildcard=ord("*"))
    assert hip.priority_consensus(chains, **cfg) == orc.priority_consensus(chains, **cfg)


@pytest.mark.parametrize("rmax", ["1", "2"])
def test_result_record_retry(rmax, monkeypatch):
    """More tied results than device result records (WC_RMAX shrinks the first
    attempt) rerun with more records: nothing is dropped (dual_consensus.rs:744-766)."""
    monkeypatch.setenv("WC_RMAX", rmax)
    case = rc.DUAL_CASES["equal_options"]
    seqs = [rc.b(s) for s in case["seqs"]]
    exp = orc.dual_consensus(seqs, **case["cfg"])
    assert len(exp) == 6
    assert hip.dual_consensus(seqs, **case["cfg"]) == exp
    single = rc.SINGLE_CASES["dual_sequence"]
    s = [rc.b(x) for x in single["seqs"]]
    assert hip.consensus(s, **single["cfg"]) == orc.consensus(s, **single["cfg"])


def test_alphabet_limit_is_a_clear_error():
    """The device engine votes at most 14 distinct symbols per node side
    (engine_shared.hpp kKout); a wider alphabet at one node is reported as
    WC_E_LIMIT, never as a wrong answer. The reference accepts any u8 alphabet."""
    import waffle_con_amd as w
    reads = [bytes([65 + i]) * 5 for i in range(20)]  # 20 distinct symbols at the root
    with pytest.raises(w.WaffleConError) as e:
        hip.consensus(reads, min_count=1)
    assert e.value.code == 11 and "limit" in str(e.value)


DUAL_KEYS = ("updates", "w_out", "compares", "ed_increases", "finalizes", "pops", "nodes_explored",
             "nodes_ignored", "peak_queue_size", "row_bytes")


def _dual_inputs(kind, seed):
    import waffle_con_amd as w
    from waffle_con_amd import synth
    if kind == "split":  # two haplotypes: single-consensus chains, then dual nodes
        return synth.cfg3_locus(seed, length=700, reads=12, err=0.01), {}
    if kind == "mono":  # one haplotype: the search stays single-consensus (long chains)
        return w.generate_test(4, 900, 20, 0.01, seed)[1], dict(min_count=4)
    if kind == "queue":  # a small queue limit: the PQueueTracker threshold moves inside chains
        return synth.cfg3_locus(seed, length=500, reads=10, err=0.02), dict(max_queue_size=3)
    raise ValueError(kind)


@pytest.mark.parametrize("chain", ["0", "2", "7", "16", "40"])
@pytest.mark.parametrize("kind,seed", [("split", 1), ("mono", 2), ("queue", 3)])
def test_dual_chain_length_invariance(chain, kind, seed, monkeypatch):
    """The dual engine's linear-chain run-ahead over single-consensus nodes
    (WC_DUAL_CHAIN = max steps, 0 = off) changes neither results nor any work
    counter: every length is bit-exact vs the oracle (per-call launches, so
    each call plans its own chain length)."""
    monkeypatch.setenv("WAFFLE_CON_SERVICE", "0")
    monkeypatch.setenv("WC_DUAL_CHAIN", chain)
    seqs, cfg = _dual_inputs(kind, seed)
    exp, ec = orc.dual_consensus(seqs, counters=True, **cfg)
    got, gc = hip.dual_consensus(seqs, counters=True, **cfg)
    assert got == exp
    for k in DUAL_KEYS:
        assert gc[k] == ec[k], (k, gc[k], ec[k])


@pytest.mark.parametrize("chain", ["0", "16"])
def test_priority_chain_invariance(chain, monkeypatch):
    """PriorityConsensusDWFA sub-problems (stream mode) with and without dual chains."""
    from waffle_con_amd import synth
    monkeypatch.setenv("WAFFLE_CON_SERVICE", "0")
    monkeypatch.setenv("WC_DUAL_CHAIN", chain)
    chains = synth.cfg5_locus(11)
    exp, ec = orc.priority_consensus(chains, counters=True, wildcard=ord("*"))
    got, gc = hip.priority_consensus(chains, counters=True, wildcard=ord("*"))
    assert got == exp
    for k in DUAL_KEYS:
        assert gc[k] == ec[k], (k, gc[k], ec[k])
