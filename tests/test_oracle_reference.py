"""Pins the CPU oracle against every golden vector the reference's own tests
hold. If these pass, the oracle reproduces the
reference's asserted behaviour, including heap tie order and hash iteration
order wherever the reference tests observe them."""
import pytest

import oracle_ffi as orc
import ref_cases as rc


class OracleRunner:
    consensus = staticmethod(orc.consensus)
    dual_consensus = staticmethod(orc.dual_consensus)
    priority_consensus = staticmethod(orc.priority_consensus)


@pytest.mark.parametrize("name", sorted(rc.SINGLE_CASES))
def test_single(name):
    rc.check_single(rc.SINGLE_CASES[name], OracleRunner)


@pytest.mark.parametrize("name", sorted(rc.DUAL_CASES))
def test_dual(name):
    rc.check_dual(rc.DUAL_CASES[name], OracleRunner)


@pytest.mark.parametrize("name", sorted(rc.PRIORITY_CASES))
def test_priority(name):
    rc.check_priority(rc.PRIORITY_CASES[name], OracleRunner)


@pytest.mark.parametrize("name", sorted(rc.DWFA_CASES))
def test_dwfa(name):
    case = rc.DWFA_CASES[name]
    r = orc.dwfa_run(rc.b(case["base"]), rc.b(case["other"]), rc.dwfa_update_lens(case),
                     wildcard=case.get("wildcard"), early=case.get("early", False), offset=case.get("offset", 0))
    fin = None
    if "finalize_e" in case:
        fin = orc.dwfa_run(rc.b(case["base"]), rc.b(case["other"]), rc.dwfa_update_lens(case),
                           wildcard=case.get("wildcard"), early=case.get("early", False),
                           offset=case.get("offset", 0), finalize=True)["e"]
    rc.check_dwfa_result(case, r["eds"], fin)


def test_dwfa_new():
    """dynamic_wfa.rs:271-276: a new DWFA has e=0, wavefront [0]."""
    r = orc.dwfa_run(b"ACGT", b"", [])
    assert r["e"] == 0 and r["wavefront"] == [0]


def test_dwfa_cloning():
    """dynamic_wfa.rs:395-421: states compare equal exactly when the consumed
    consensus symbols agree; re-cloning resynchronises."""
    import ctypes
    L = orc.lib()
    seq, alt = b"AAAAAAA", b"AAACAAA"

    def step(state, other):
        e = ctypes.c_uint64(state[0])
        wf = (ctypes.c_uint64 * 64)(*state[1])
        wl = ctypes.c_uint64(len(state[1]))
        assert L.orc_dwfa_step(seq, len(seq), other, len(other), -1, 0, 0, 0, ctypes.byref(e), wf,
                               ctypes.byref(wl), 64) == 0
        return (e.value, list(wf[:wl.value]))

    d1 = d2 = (0, [0])
    for l in range(len(alt)):
        d1 = step(d1, seq[:l + 1])
        d2 = step(d2, alt[:l + 1])
        if seq[l] == alt[l]:
            assert d1 == d2
        else:
            assert d1 != d2
            d2 = d1
    assert d1[0] == 0 and d2[0] == 0


def test_ed_weights():
    """dual_consensus.rs:1361-1382 (test_get_ed_weights)."""
    import ctypes
    L = orc.lib()
    bufs, ptrs, lens = orc._seq_arrays([b"ACGT", b"CGTA"])
    out = (ctypes.c_double * 2)()
    L.orc_test_ed_weights.argtypes = [ctypes.c_uint32, type(ptrs), type(lens), ctypes.c_uint8, ctypes.c_uint8,
                                      ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8, ctypes.POINTER(ctypes.c_double)]
    for side1, by_ed, exp in [(1, 1, [1.0 / 1.5, 0.5 / 1.5]), (0, 1, [0.5 / 1.5, 1.0 / 1.5]),
                              (1, 0, [1.0, 0.0]), (0, 0, [0.0, 1.0])]:
        assert L.orc_test_ed_weights(2, ptrs, lens, ord("A"), ord("C"), 1, side1, by_ed, out) == 0
        assert list(out) == exp


def test_wfa_ed_doc():
    """sequence_alignment.rs:9-17 and :29-35 doc examples."""
    v1, v2, v3 = bytes([0, 1, 2, 4, 5]), bytes([0, 1, 3, 4, 5]), bytes([1, 2, 3, 5])
    assert orc.wfa_ed(v1, v1) == 0
    assert orc.wfa_ed(v1, v2) == 1
    assert orc.wfa_ed(v1, v3) == 2
    w2 = bytes([0, 1, 2, 4])
    assert orc.wfa_ed_config(v1, w2, False, ord("*")) == 0
    assert orc.wfa_ed_config(v1, w2, True, ord("*")) == 1


def test_fxmap_orders_appendix_b():
    """SURVEY Appendix B precomputed orders: >=4 keys among {*,A,C,G,T} iterate
    *,G,T,A,C; raw 0..3 iterate 0,2,1,3."""
    assert orc.fxmap_order(b"ACGT*") == list(b"*GTAC")
    assert orc.fxmap_order(bytes([0, 1, 2, 3])) == [0, 2, 1, 3]
    assert orc.fxmap_order(bytes([3, 2, 1, 0])) == [0, 2, 1, 3]
    # <= 3 keys: insertion order decides collisions (C and G share bucket 3 of 4)
    assert orc.fxmap_order(b"CG") == list(b"GC")  # C at 3, G wraps to 0
    assert orc.fxmap_order(b"GC") == list(b"CG")


def _insertion_cases():
    """(baseline, other) pairs: the reference's DWFA test inputs, a G-then-C
    tip collision, and seeded random pairs."""
    import random
    cases = [(rc.b(c["base"]), rc.b(c["other"])) for c in rc.DWFA_CASES.values()]
    cases.append((b"CG", b"G"))  # tips nominate G (diagonal 0) then C (diagonal 2): C and G share bucket 3 of 4
    rng = random.Random(5)
    for _ in range(400):
        cases.append((bytes(rng.choice(b"ACGT") for _ in range(rng.randint(2, 12))),
                      bytes(rng.choice(b"ACGT") for _ in range(rng.randint(1, 9)))))
    return cases


def test_candidate_insertion_order_rebuilds_the_map():
    """dynamic_wfa.rs:241-255 inserts tip symbols in ascending diagonal order.
    Replaying that insertion order through the hashbrown model (Appendix B)
    gives the map's iteration order on every case; replaying the iteration
    order instead (what a shim that only sees the iteration order would do)
    does not, once keys collide (the Rust crate's get_extension_candidates
    inserts in wc_dwfa_job.cand_first order for this reason)."""
    wrong = 0
    for base, other in _insertion_cases():
        it = [s for s, _ in orc.dwfa_candidates(base, other)]
        ins = orc.dwfa_candidate_first(base, other)
        assert sorted(ins) == sorted(it)
        assert orc.fxmap_order(bytes(ins)) == it, (base, other)
        wrong += orc.fxmap_order(bytes(it)) != it
    assert orc.dwfa_candidate_first(b"CG", b"G") == list(b"GC")
    assert [s for s, _ in orc.dwfa_candidates(b"CG", b"G")] == list(b"CG")
    assert orc.fxmap_order(b"CG") == list(b"GC")  # re-inserting the iteration order flips it
    assert wrong > 0
