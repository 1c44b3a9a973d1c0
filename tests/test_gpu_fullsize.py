"""GPU parity at the BASELINE configs' real sizes: the shapes
where the device capacities (wavefront rows, node pool, consensus length,
LDS per workgroup) actually bind. Everything the reference returns is
compared with the CPU oracle: sequences, scores, scores1/2, is_consensus1,
chains and sequence_indices, plus every work counter.

cfg4's oracle run takes about two minutes, so its expected output is a
committed fixture made by tests/golden/make_cfg4_golden.py (the oracle on the
same synthetic bytes)."""
import hashlib
import json
import os

import pytest

import oracle_ffi as orc

pytestmark = pytest.mark.gpu
hip = pytest.importorskip("hip_runner")

COUNTER_KEYS = ("updates", "w_out", "compares", "ed_increases", "finalizes", "pops", "nodes_explored",
                "nodes_ignored", "peak_queue_size", "row_bytes")
HERE = os.path.dirname(os.path.abspath(__file__))


def _counters_equal(gc, ec):
    for k in COUNTER_KEYS:
        assert gc[k] == ec[k], (k, gc[k], ec[k])


@pytest.mark.parametrize("seed", [0, 1])
def test_cfg2_full_locus_vs_oracle(seed):
    """cfg2: 100 reads x 10 kb @ 0.5%, min_count 25 (consensus_bench convention)."""
    import waffle_con_amd as w
    seqs = w.generate_test(4, 10000, 100, 0.005, seed)[1]
    exp, ec = orc.consensus(seqs, counters=True, min_count=25)
    got, gc = hip.consensus(seqs, counters=True, min_count=25)
    assert got == exp
    _counters_equal(gc, ec)


def test_cfg2_batch_per_problem_counters_vs_oracle():
    """A 16-locus cfg2 batch through the resident-batch path (the bench path):
    per-problem results and counters equal the oracle's."""
    import waffle_con_amd as w
    from waffle_con_amd.cdwfa_config import CdwfaConfig
    loci = [w.generate_test(4, 10000, 100, 0.005, s)[1] for s in range(100, 116)]
    b = w.ResidentBatch(loci)
    res, st = b.consensus(CdwfaConfig(min_count=25), per_problem=True)
    for i, seqs in enumerate(loci):
        exp, ec = orc.consensus(seqs, counters=True, min_count=25)
        assert [(c.sequence(), list(c.scores())) for c in res[i]] == [(r["sequence"], r["scores"]) for r in exp]
        _counters_equal(st["per_problem"][i], ec)


def test_cfg3_full_locus_vs_oracle():
    """cfg3: DualConsensusDWFA, 5 kb haplotypes A/B, 2 x 100 reads, default config."""
    from waffle_con_amd import synth
    reads = synth.cfg3_locus(3)
    exp, ec = orc.dual_consensus(reads, counters=True)
    got, gc = hip.dual_consensus(reads, counters=True)
    assert got == exp
    _counters_equal(gc, ec)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_cfg5_full_locus_vs_oracle(priority_path, seed):
    """cfg5: PGx locus at real size (1-6 kb, 15-40 reads per haplotype, [HPC, full] chains)."""
    from waffle_con_amd import synth
    chains = synth.cfg5_locus(seed)
    exp, ec = orc.priority_consensus(chains, counters=True, wildcard=ord("*"))
    got, gc = hip.priority_consensus(chains, counters=True, wildcard=ord("*"))
    assert got == exp
    _counters_equal(gc, ec)


def _digest(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def test_cfg4_full_locus_vs_oracle_fixture(priority_path):
    """cfg4: 4 haplotypes x 50 reads x 8 kb with inserted segments {0, 25, 60,
    150} bp, chain length 1, wildcard '*' (priority tests' config)."""
    path = os.path.join(HERE, "golden", "cfg4_seed4.json")
    with open(path) as f:
        gold = json.load(f)
    from waffle_con_amd import synth
    reads = synth.cfg4_locus(gold["seed"])
    assert _digest(b"".join(reads)) == gold["input_sha256"]
    got, gc = hip.priority_consensus([[r] for r in reads], counters=True, wildcard=ord("*"))
    assert got["sequence_indices"] == gold["sequence_indices"]
    assert [[(_digest(c["sequence"]), c["scores"]) for c in ch] for ch in got["consensuses"]] == \
        [[(c["sha256"], c["scores"]) for c in ch] for ch in gold["consensuses"]]
    _counters_equal(gc, gold["counters"])


def test_thousand_reads_single_vs_oracle():
    """1,000 reads in one locus (the reference accepts any number, consensus.rs:110-134):
    per-read state beyond the LDS of a 4-workgroup/CU launch; the deep problem
    runs in a launch of its own with up to 160 KiB of LDS."""
    import waffle_con_amd as w
    seqs = w.generate_test(4, 200, 1000, 0.01, 5)[1]
    exp, ec = orc.consensus(seqs, counters=True, min_count=250)
    got, gc = hip.consensus(seqs, counters=True, min_count=250)
    assert got == exp
    _counters_equal(gc, ec)
    # and mixed into a batch of ordinary loci
    small = [w.generate_test(4, 300, 20, 0.02, s)[1] for s in range(6)]
    res = hip.consensus_batch(small + [seqs], min_count=5)
    assert res[-1] == orc.consensus(seqs, min_count=5)
    for p, r in zip(small, res):
        assert r == orc.consensus(p, min_count=5)


def test_thousand_reads_dual_vs_oracle():
    import numpy as np
    from waffle_con_amd import synth
    rng = np.random.default_rng(9)
    a = synth.random_seq(rng, 150).tobytes()
    b = synth._variant(rng, a, 3, 1)
    reads = [synth.mutate(rng, a, 0.01) for _ in range(500)] + [synth.mutate(rng, b, 0.01) for _ in range(500)]
    exp, ec = orc.dual_consensus(reads, counters=True)
    got, gc = hip.dual_consensus(reads, counters=True)
    assert got == exp
    _counters_equal(gc, ec)


@pytest.mark.parametrize("seed", [0, 1])
def test_global_state_engine_vs_oracle(seed, monkeypatch):
    """The global-state build (engine_gstate.hip: heap, slot metadata and
    nominations in HBM instead of LDS), forced with WC_GSTATE=1, is bit-exact
    on the single, dual and priority engines."""
    import waffle_con_amd as w
    from waffle_con_amd import synth
    monkeypatch.setenv("WC_GSTATE", "1")
    seqs = w.generate_test(4, 1500, 20, 0.01, 40 + seed)[1]
    exp, ec = orc.consensus(seqs, counters=True, min_count=5)
    got, gc = hip.consensus(seqs, counters=True, min_count=5)
    assert got == exp
    _counters_equal(gc, ec)
    reads = synth.cfg3_locus(50 + seed, length=400, reads=8, err=0.01)
    exp, ec = orc.dual_consensus(reads, counters=True)
    got, gc = hip.dual_consensus(reads, counters=True)
    assert got == exp
    _counters_equal(gc, ec)
    chains = synth.cfg5_locus(60 + seed, len_range=(300, 600), reads_range=(5, 8), err=0.01)
    assert hip.priority_consensus(chains, wildcard=ord("*")) == orc.priority_consensus(chains, wildcard=ord("*"))
