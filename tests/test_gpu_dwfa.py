"""GPU parity: DWFALite (device kernels via wc_dwfa_batch) vs the reference's
DWFA known-answer tests (dynamic_wfa.rs:271-482) and vs the oracle."""
import random

import pytest

import oracle_ffi as orc
import ref_cases as rc

pytestmark = pytest.mark.gpu
w = pytest.importorskip("waffle_con_amd")


@pytest.mark.parametrize("name", sorted(rc.DWFA_CASES))
def test_reference_dwfa(name):
    case = rc.DWFA_CASES[name]
    base, other = rc.b(case["base"]), rc.b(case["other"])
    d = w.DWFALite.new(case.get("wildcard"), case.get("early", False))
    d.set_offset(case.get("offset", 0))
    eds = [d.update(base, other[:l]) for l in rc.dwfa_update_lens(case)]
    fin = None
    if "finalize_e" in case:
        d.finalize(base, other)
        fin = d.edit_distance()
    rc.check_dwfa_result(case, eds, fin)


def test_dwfa_new():
    d = w.DWFALite.default()
    assert d.edit_distance() == 0 and d.wavefront() == [0]


def test_dwfa_cloning():
    """dynamic_wfa.rs:395-421."""
    seq, alt = b"AAAAAAA", b"AAACAAA"
    d1 = w.DWFALite.default()
    d2 = d1.clone()
    for l in range(len(alt)):
        d1.update(seq, seq[:l + 1])
        d2.update(seq, alt[:l + 1])
        if seq[l] == alt[l]:
            assert d1 == d2
        else:
            assert d1 != d2
            d2 = d1.clone()
    assert d1.edit_distance() == 0 and d2.edit_distance() == 0


def test_dwfa_random_vs_oracle():
    rng = random.Random(11)
    for _ in range(40):
        base = bytes(rng.choice(b"ACGT") for _ in range(rng.randint(1, 60)))
        other = bytearray(base)
        for _ in range(rng.randint(0, 6)):
            p = rng.randrange(len(other) + 1)
            op = rng.randrange(3)
            if op == 0 and p < len(other):
                other[p] = rng.choice(b"ACGT")
            elif op == 1 and p < len(other):
                del other[p]
            else:
                other.insert(p, rng.choice(b"ACGT"))
        other = bytes(other) or b"A"
        early = rng.random() < 0.3
        d = w.DWFALite.new(None, early)
        lens = list(range(1, len(other) + 1))
        eds = [d.update(base, other[:l]) for l in lens]
        ref = orc.dwfa_run(base, other, lens, early=early)
        assert eds == ref["eds"] and d.wavefront() == ref["wavefront"]
        cand = d.get_extension_candidates(base, other)
        assert list(cand.items()) == orc.dwfa_candidates(base, other) if not early else True


def test_dwfa_candidate_insertion_order_vs_oracle():
    """wc_dwfa_job.cand_first (the insertion order the Rust crate replays into
    its FxHashMap) equals the reference's first-appearance order, and replaying
    it through the hashbrown model gives the device's iteration order;
    includes the G-then-C collision case."""
    rng = random.Random(5)
    cases = [(b"CG", b"G"), (b"ACGT", b"AG")]
    for _ in range(60):
        cases.append((bytes(rng.choice(b"ACGT") for _ in range(rng.randint(2, 12))),
                      bytes(rng.choice(b"ACGT") for _ in range(rng.randint(1, 9)))))
    for base, other in cases:
        d = w.DWFALite.default()
        for l in range(1, len(other) + 1):
            d.update(base, other[:l])
        cand = d.get_extension_candidates(base, other)
        first = d.candidate_insertion_order(base, other)
        assert list(cand.items()) == orc.dwfa_candidates(base, other)
        assert first == orc.dwfa_candidate_first(base, other)
        assert orc.fxmap_order(bytes(first)) == list(cand.keys())
