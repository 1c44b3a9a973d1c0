"""The reference's own test cases, restated as data.

Each case cites the reference test it restates (path:line under
/root/reference, read as text only). Inputs and expected outputs are the
reference's golden values; the CSV fixtures are copied verbatim into
tests/golden/reference_csv/ (data files the reference's tests hold).

A runner is any object with .consensus/.dual_consensus/.priority_consensus
taking (sequences, offsets=None, **config) and returning dicts shaped like the
oracle's output (tests/oracle_ffi.py); the same cases drive the oracle (CPU)
and the HIP path (GPU).
"""
import csv
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
CSV_DIR = os.path.join(HERE, "golden", "reference_csv")
L1, L2 = 0, 1
STAR = ord("*")


def b(s):
    return s.encode() if isinstance(s, str) else bytes(s)


# ---------------------------------------------------------------------------
# CSV loaders (restating the reference test harnesses)
# ---------------------------------------------------------------------------
def load_dual_csv(name, include_consensus, cost=L1):
    """dual_consensus.rs:1400-1461 (load_dual_csv_test)."""
    seqs, is_c1, ed1, ed2 = [], [], [], []
    con1 = con2 = None
    with open(os.path.join(CSV_DIR, name)) as fh:
        for row in csv.DictReader(fh):
            c = int(row["consensus"]) == 1
            e = int(row["edits"])
            e = e if cost == L1 else e * e
            s = b(row["sequence"])
            if c:
                if con1 is None and e == 0:
                    con1 = s
                    if not include_consensus:
                        continue
                ed1.append(e)
            else:
                if con2 is None and e == 0:
                    con2 = s
                    if not include_consensus:
                        continue
                ed2.append(e)
            is_c1.append(c)
            seqs.append(s)
    assert con2 is None or con1 < con2
    exp = {"consensus1": {"sequence": con1, "scores": ed1},
           "consensus2": None if con2 is None else {"sequence": con2, "scores": ed2},
           "is_consensus1": is_c1}
    return seqs, exp


def load_priority_csv(name, include_consensus):
    """priority_consensus.rs:382-489 (load_priority_csv_test)."""
    consensuses = []
    chains, indices = [], []
    with open(os.path.join(CSV_DIR, name)) as fh:
        for row in csv.DictReader(fh):
            ci = int(row["consensus"]) - 1
            e = int(row["edits"])
            chain = [b(x) for x in row["sequence"].split(";")]
            while len(consensuses) <= ci:
                consensuses.append(None)
            if e == 0 and consensuses[ci] is None:
                consensuses[ci] = chain
                if not include_consensus:
                    continue
            chains.append(chain)
            indices.append(ci)
    assert all(c is not None for c in consensuses)
    order = sorted(range(len(consensuses)), key=lambda i: consensuses[i])
    rank = {old: new for new, old in enumerate(order)}
    exp = {"consensuses": [consensuses[i] for i in order], "sequence_indices": [rank[i] for i in indices]}
    return chains, exp


# ---------------------------------------------------------------------------
# comparisons (reference PartialEq semantics)
# ---------------------------------------------------------------------------
def cons_eq(got, exp):
    return got["sequence"] == exp["sequence"] and list(got["scores"]) == list(exp["scores"])


def dual_eq(got, exp):
    """DualConsensus PartialEq ignores scores1/scores2 (dual_consensus.rs:66-75)."""
    if not cons_eq(got["consensus1"], exp["consensus1"]):
        return False
    if (got["consensus2"] is None) != (exp["consensus2"] is None):
        return False
    if exp["consensus2"] is not None and not cons_eq(got["consensus2"], exp["consensus2"]):
        return False
    return list(got["is_consensus1"]) == list(exp["is_consensus1"])


def priority_check(got, exp):
    """priority_consensus.rs:519-527: indices, chain count, chain sequences."""
    assert list(got["sequence_indices"]) == list(exp["sequence_indices"])
    assert len(got["consensuses"]) == len(exp["consensuses"])
    for cc, ecc in zip(got["consensuses"], exp["consensuses"]):
        assert len(cc) == len(ecc)
        for c, ec in zip(cc, ecc):
            assert c["sequence"] == ec


def C(seq, scores):
    return {"sequence": b(seq), "scores": list(scores)}


def DC(c1, c2, is_c1):
    return {"consensus1": c1, "consensus2": c2, "is_consensus1": list(is_c1)}


# ---------------------------------------------------------------------------
# single-consensus cases (consensus.rs:578-851 + doc example :6-26, lib.rs:15-35)
# ---------------------------------------------------------------------------
SINGLE_CASES = {
    "doc_example": dict(src="consensus.rs:6-26, lib.rs:15-35", seqs=["ACGT", "ACCGT", "ACCCGT"], cfg={},
                        expect=[C("ACCGT", [1, 0, 1])]),
    "single_sequence": dict(src="consensus.rs:579-594", seqs=["ACGTACGTACGT"], cfg={},
                            expect=[C("ACGTACGTACGT", [0])]),
    "dual_sequence": dict(src="consensus.rs:597-623", seqs=["ACGTACGTACGT", "ACGTACCTACGT"], cfg={},
                          expect=[C("ACGTACCTACGT", [1, 0]), C("ACGTACGTACGT", [0, 1])]),
    "trio_sequence": dict(src="consensus.rs:626-650", seqs=["ACGTACGTACGT", "ACGTACGTACGT", "ACGTACCTACGT"], cfg={},
                          expect=[C("ACGTACGTACGT", [0, 0, 1])]),
    "complicated": dict(src="consensus.rs:653-678", seqs=["ACTACGGTACGT", "ACGTAAGTCCGT", "AAGTACGTACGT"], cfg={},
                        expect_seqs=["ACGTACGTACGT"]),
    "wildcards": dict(src="consensus.rs:681-710", seqs=["ACGTACCGT****", "**GTATGTAC**", "****ACGTACGT"],
                      cfg=dict(wildcard=STAR), expect=[C("ACGTACGTACGT", [1, 1, 0])]),
    "all_wildcards": dict(src="consensus.rs:713-743", seqs=["*CGTAACG*ACG*", "*CGTACG*ACG*", "*CGTACG*ATG*"],
                          cfg=dict(wildcard=STAR), expect=[C("*CGTACG*ACG*", [1, 0, 1])]),
    "early_termination_off": dict(src="consensus.rs:746-763", seqs=["A", "AC", "ACG", "ACGT"],
                                  cfg=dict(wildcard=STAR),
                                  expect=[C("AC", [1, 0, 1, 2]), C("ACG", [2, 1, 0, 1])]),
    "early_termination_on": dict(src="consensus.rs:765-779", seqs=["A", "AC", "ACG", "ACGT"],
                                 cfg=dict(wildcard=STAR, allow_early_termination=True),
                                 expect=[C("ACGT", [0, 0, 0, 0])]),
    "offset_windows": dict(src="consensus.rs:783-817",
                           seqs=["ACGTACGTACGTACGT", "ACGTACGTACGT", "GTACGTACGT"], offsets=[None, 4, 7],
                           cfg=dict(offset_window=1, offset_compare_length=4),
                           expect=[C("ACGTACGTACGTACGT", [0, 0, 0])]),
    "offset_gap_err": dict(src="consensus.rs:820-851", seqs=["ACGTACGTACGTACGT", "ACGTACGTACGTACGT"],
                           offsets=[None, 1000], cfg=dict(offset_window=1, offset_compare_length=4),
                           error="Finalize called on DWFA that was never initialized."),
}


def check_single(case, runner):
    seqs = [b(s) for s in case["seqs"]]
    if "error" in case:
        try:
            runner.consensus(seqs, offsets=case.get("offsets"), **case["cfg"])
        except Exception as e:  # noqa: BLE001
            assert str(e) == case["error"], str(e)
            return
        raise AssertionError("expected error")
    got = runner.consensus(seqs, offsets=case.get("offsets"), **case["cfg"])
    if "expect" in case:
        assert len(got) == len(case["expect"]), got
        for g, e in zip(got, case["expect"]):
            assert cons_eq(g, e), (g, e)
    else:
        assert [g["sequence"] for g in got] == [b(s) for s in case["expect_seqs"]]
    return got


# ---------------------------------------------------------------------------
# dual cases (dual_consensus.rs:1361-2055 + doc :7-35)
# ---------------------------------------------------------------------------
def _dual_cases():
    T, F = True, False
    cases = {
        "doc_example": dict(src="dual_consensus.rs:7-35",
                            seqs=["TCCGT", "ACCGT", "ACCGT", "ACCAT", "CCGTAAT", "CGTAAAT", "CGTAAT", "CGTAAT"],
                            cfg={}, expect=[DC(C("ACCGT", [1, 0, 0, 1]), C("CGTAAT", [1, 1, 0, 0]),
                                               [T, T, T, T, F, F, F, F])]),
        "single_sequence": dict(src="dual_consensus.rs:1491-1515", seqs=["ACGTACGTACGT"], cfg={},
                                expect=[DC(C("ACGTACGTACGT", [0]), None, [T])]),
        "trio_sequence": dict(src="dual_consensus.rs:1517-1547",
                              seqs=["ACGTACGTACGT", "ACGTACGTACGT", "ACGTACCTACGT"], cfg={},
                              expect=[DC(C("ACGTACGTACGT", [0, 0, 1]), None, [T, T, T])]),
        "complicated": dict(src="dual_consensus.rs:1549-1582",
                            seqs=["ACTACGGTACGT", "ACGTAAGTCCGT", "AAGTACGTACGT"], cfg={},
                            expect=[DC(C("ACGTACGTACGT", [2, 2, 1]), None, [T, T, T])]),
        "wildcards": dict(src="dual_consensus.rs:1584-1620",
                          seqs=["ACGTACCGT****", "**GTATGTAC**", "****ACGTACGT"], cfg=dict(wildcard=STAR),
                          expect=[DC(C("ACGTACGTACGT", [1, 1, 0]), None, [T, T, T])]),
        "all_wildcards": dict(src="dual_consensus.rs:1622-1659",
                              seqs=["*CGTAACG*ACG*", "*CGTACG*ACG*", "*CGTACG*ATG*"], cfg=dict(wildcard=STAR),
                              expect=[DC(C("*CGTACG*ACG*", [1, 0, 1]), None, [T, T, T])]),
        "dual_sequence": dict(src="dual_consensus.rs:1661-1686", seqs=["ACGT", "AGGT"], cfg=dict(min_count=1),
                              expect=[DC(C("ACGT", [0]), C("AGGT", [0]), [T, F])]),
        "dual_unequal_001": dict(src="dual_consensus.rs:1688-1713", seqs=["ACGT", "AGGTA"], cfg=dict(min_count=1),
                                 expect=[DC(C("ACGT", [0]), C("AGGTA", [0]), [T, F])]),
        "dual_unequal_002": dict(src="dual_consensus.rs:1715-1740", seqs=["ACGTA", "AGGT"], cfg=dict(min_count=1),
                                 expect=[DC(C("ACGTA", [0]), C("AGGT", [0]), [T, F])]),
        "noise_before_variation": dict(
            src="dual_consensus.rs:1742-1780",
            seqs=["ACGTACGTACGT", "ACCGTACGTACGT", "ACGTACGTACGT", "ACGTACGTCCCT", "ACGTACGTCCCT", "ACCGTACGTCCCT"],
            cfg=dict(min_count=1, max_queue_size=1000),
            expect=[DC(C("ACGTACGTACGT", [0, 1, 0]), C("ACGTACGTCCCT", [0, 0, 1]), [T, T, T, F, F, F])]),
        "multi_extension": dict(
            src="dual_consensus.rs:1782-1822",
            seqs=["ACGTACGTACGT", "ACGTACGTACGT", "ACGTACGTGCGT", "ACGTACGTCCCT", "ACGTACGTCCCT", "ACGTACGTGCCT"],
            cfg=dict(min_count=1, max_queue_size=1000),
            expect=[DC(C("ACGTACGTACGT", [0, 0, 1]), C("ACGTACGTCCCT", [0, 0, 1]), [T, T, T, F, F, F])]),
        "equal_options": dict(src="dual_consensus.rs:1824-1863",
                              seqs=["ACGTACGTACGT", "ACGTCCGTCCGT", "ACGTACGTCCGT", "ACGTCCGTACGT"],
                              cfg=dict(min_count=1, max_queue_size=1000), expect_equal_options=(6, 2)),
        "tail_extension": dict(src="dual_consensus.rs:1865-1909", seqs=["ACGT", "ACGTT"],
                               cfg=dict(min_count=1, max_queue_size=1000),
                               expect=[DC(C("ACGT", [0, 1]), None, [T, T]), DC(C("ACGTT", [1, 0]), None, [T, T])]),
        "offset_windows": dict(src="dual_consensus.rs:1985-2021",
                               seqs=["ACGTACGTACGTACGT", "ACGTACGTACGT", "GTACGTACGT"], offsets=[None, 4, 7],
                               cfg=dict(offset_window=1, offset_compare_length=4),
                               expect=[DC(C("ACGTACGTACGTACGT", [0, 0, 0]), None, [T, T, T])]),
        "offset_gap_err": dict(src="dual_consensus.rs:2023-2055",
                               seqs=["ACGTACGTACGTACGT", "ACGTACGTACGTACGT"], offsets=[None, 1000],
                               cfg=dict(offset_window=1, offset_compare_length=4),
                               error="Finalize called on DWFA that was never initialized."),
    }
    s, e = load_dual_csv("dual_001.csv", True)
    cases["csv_dual_001"] = dict(src="dual_consensus.rs:1911-1914", seqs=s, cfg=dict(wildcard=STAR), expect=[e])
    cases["dual_max_ed_delta"] = dict(
        src="dual_consensus.rs:1916-1960", seqs=s, cfg=dict(wildcard=STAR, dual_max_ed_delta=0),
        expect=[DC(C(e["consensus1"]["sequence"], [0, 4, 4, 2]), C(e["consensus2"]["sequence"], [3, 0, 0, 0, 0, 0]),
                   [T, T, F, T, T, F, F, F, F, F])])
    s, e = load_dual_csv("length_gap_001.csv", False, L2)
    cases["csv_length_gap_001"] = dict(src="dual_consensus.rs:1962-1973", seqs=s,
                                       cfg=dict(wildcard=STAR, min_count=2, dual_max_ed_delta=5,
                                                max_queue_size=1000, consensus_cost=L2), expect=[e])
    s, e = load_dual_csv("dual_early_termination_001.csv", True)
    cases["csv_early_termination_001"] = dict(src="dual_consensus.rs:1975-1983", seqs=s,
                                              cfg=dict(wildcard=STAR, allow_early_termination=True), expect=[e])
    return cases


DUAL_CASES = _dual_cases()


def check_dual(case, runner):
    seqs = [b(s) for s in case["seqs"]]
    if "error" in case:
        try:
            runner.dual_consensus(seqs, offsets=case.get("offsets"), **case["cfg"])
        except Exception as e:  # noqa: BLE001
            assert str(e) == case["error"], str(e)
            return
        raise AssertionError("expected error")
    got = runner.dual_consensus(seqs, offsets=case.get("offsets"), **case["cfg"])
    if "expect_equal_options" in case:
        n, total = case["expect_equal_options"]
        assert len(got) == n
        for dc in got:
            assert dc["consensus2"] is not None
            assert sum(dc["consensus1"]["scores"]) + sum(dc["consensus2"]["scores"]) == total
        return got
    assert len(got) == len(case["expect"]), got
    for g, e in zip(got, case["expect"]):
        assert dual_eq(g, e), (g, e)
    return got


# ---------------------------------------------------------------------------
# priority cases (priority_consensus.rs:531-653 + doc :7-51)
# ---------------------------------------------------------------------------
def _priority_cases():
    cases = {}
    for name, inc, cfg in [("dual_001.csv", True, {}), ("multi_exact_001.csv", True, {}),
                           ("multi_exact_002.csv", True, {}), ("multi_err_001.csv", False, {}),
                           ("multi_err_002.csv", False, {}), ("multi_samesplit_001.csv", True, {}),
                           ("multi_postcon_001.csv", True, dict(min_count=2)),
                           ("priority_001.csv", True, {}), ("priority_002.csv", True, {}),
                           ("priority_003.csv", True, {})]:
        chains, exp = load_priority_csv(name, inc)
        c = dict(wildcard=STAR)
        c.update(cfg)
        cases["csv_" + name[:-4]] = dict(src="priority_consensus.rs:531-653 (%s)" % name, chains=chains, cfg=c,
                                         expect_csv=exp)
    s = b("ACGTACGTACGT")
    cases["single_sequence"] = dict(src="priority_consensus.rs:575-596", chains=[[s, s]], cfg={},
                                    expect_full={"consensuses": [[C(s, [0]), C(s, [0])]], "sequence_indices": [0]})
    doc = [["TCCGT", "TCCGT"]] * 3 + [["TCCGT", "ACGGT"]] * 3 + [["ACGT", "ACCCGGTT"]] * 3
    cases["doc_example"] = dict(
        src="priority_consensus.rs:7-51, :598-639", chains=[[b(x) for x in ch] for ch in doc], cfg={},
        expect_full={"consensuses": [[C("ACGT", [0] * 3), C("ACCCGGTT", [0] * 3)],
                                     [C("TCCGT", [0] * 6), C("ACGGT", [0] * 3)],
                                     [C("TCCGT", [0] * 6), C("TCCGT", [0] * 3)]],
                     "sequence_indices": [2, 2, 2, 1, 1, 1, 0, 0, 0]})
    return cases


PRIORITY_CASES = _priority_cases()


def check_priority(case, runner):
    got = runner.priority_consensus(case["chains"], **case["cfg"])
    if "expect_csv" in case:
        priority_check(got, case["expect_csv"])
    else:
        exp = case["expect_full"]
        assert list(got["sequence_indices"]) == exp["sequence_indices"]
        assert len(got["consensuses"]) == len(exp["consensuses"])
        for gc, ec in zip(got["consensuses"], exp["consensuses"]):
            assert len(gc) == len(ec)
            for g, e in zip(gc, ec):
                assert cons_eq(g, e), (g, e)
    return got


# ---------------------------------------------------------------------------
# DWFA known-answer tests (dynamic_wfa.rs:271-482)
# each: baseline, other, mode ("prefix" = update on every prefix, "full" = one
# update with the whole other), wildcard, early, offset, expected final e,
# optional finalize expectation.
# ---------------------------------------------------------------------------
def _dwfa_cases():
    vec = json.load(open(os.path.join(HERE, "golden", "dwfa_vectors.json")))
    seq = "ACGTACGTACGT"
    return {
        "exact_match": dict(src="dynamic_wfa.rs:278-287", base=seq, other=seq, mode="prefix", e=0, every_e=0),
        "simple_mismatch": dict(src="dynamic_wfa.rs:289-298", base=seq, other="ACGTACCTACGT", mode="prefix", e=1),
        "simple_insertion": dict(src="dynamic_wfa.rs:300-309", base=seq, other="ACGTACIGTACGT", mode="prefix", e=1),
        "simple_deletion": dict(src="dynamic_wfa.rs:311-320", base=seq, other="ACGTACTACGT", mode="prefix", e=1),
        "complex_001": dict(src="dynamic_wfa.rs:322-331", base=seq, other="ACTACGCACGGGT", mode="prefix", e=4),
        "complex_002": dict(src="dynamic_wfa.rs:333-348", base="AACGGATCAAGCTTACCAGTATTTACGT",
                            other="AACGGACAAAAGCTTACCTGTATTACGT", mode="full", e=5),
        "big_insertion": dict(src="dynamic_wfa.rs:350-361", base="AACGGATTTTACGT",
                              other="AACGGATAAAAGCTTACCTGTTTTACGT", mode="prefix", e=28 - 14),
        "big_deletion": dict(src="dynamic_wfa.rs:363-374", base="ATTTTTTTTTTAAAAAAAAAA", other="AAAAAAAAAAA",
                             mode="prefix", e=21 - 11),
        "required_finalize": dict(src="dynamic_wfa.rs:376-393", base="ATTTTTTTTTTA", other="AA", mode="prefix",
                                  e=1, finalize_e=12 - 2),
        "wildcards_001": dict(src="dynamic_wfa.rs:423-432", base="*ACGGATCAA**TTACCA*TATTTACG*",
                              other="AACGGATCAAGCTTACCAGTATTTACGT", mode="full", wildcard=STAR, e=0),
        "wildcards_002": dict(src="dynamic_wfa.rs:434-443", base="*ACGATCAA**TATACCA*TATCTACG*",
                              other="AACGGATCAAGCTTACCAGTATTTACGT", mode="full", wildcard=STAR, e=3),
        "early_termination_001": dict(src="dynamic_wfa.rs:445-452", base="ACGT", other="ACGTACGT", mode="full",
                                      early=True, e=0),
        "big_early_termination": dict(src="dynamic_wfa.rs:454-471", base=vec["seq_23"], other=vec["c1"],
                                      mode="prefix", early=True, e=2, max_e=2, finalize_e=2),
        "offsets": dict(src="dynamic_wfa.rs:473-482", base="GTACGT", other="ACGTACGT", mode="full", early=True,
                        offset=2, e=0),
    }


DWFA_CASES = _dwfa_cases()


def dwfa_update_lens(case):
    n = len(case["other"])
    return list(range(1, n + 1)) if case["mode"] == "prefix" else [n]


def check_dwfa_result(case, eds, final_e_after_finalize=None):
    assert eds[-1] == case["e"], (eds[-1], case["e"])
    if "every_e" in case:
        assert all(x == case["every_e"] for x in eds)
    if "max_e" in case:
        assert max(eds) <= case["max_e"]
    if "finalize_e" in case and final_e_after_finalize is not None:
        assert final_e_after_finalize == case["finalize_e"]
