"""CPU-side checks of the product library: it loads, exports every symbol the
public header declares, and its host-side pieces (RNG restatement, generator,
wfa_ed, host result types, config builder) match the reference's known
answers. No GPU compute here."""
import ctypes
import os
import re

import pytest

import waffle_con_amd as w
from waffle_con_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_header_symbols_exported():
    L = _lib.lib()
    hdr = open(os.path.join(ROOT, "include", "waffle_con.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    names = set(re.findall(r"\b(wc_[a-z0-9_]+)\s*\(", hdr))
    assert len(names) >= 30
    missing = [n for n in sorted(names) if not hasattr(L, n)]
    assert not missing, missing
    assert set(_lib.EXPORTED) <= names


def _rng_hooks():
    """oracle/librnghooks.so: the product's ChaCha/StdRng source (example_gen.cpp)
    behind test-only known-answer hooks (the product library exports none)."""
    return ctypes.CDLL(os.path.join(ROOT, "oracle", "librnghooks.so"))


def test_rng_hooks_not_in_product_abi():
    L = _lib.lib()
    for name in ("wc_rng_words", "wc_rng_stdrng_chain", "wc_rng_seed_from_u64"):
        assert not hasattr(L, name), name


def test_chacha20_zero_key_vector():
    """Original ChaCha20 (64-bit nonce) keystream, all-zero key/nonce, block 0."""
    out = (ctypes.c_uint32 * 16)()
    _rng_hooks().wc_rng_words(bytes(32), 20, 16, out)
    exp = bytes.fromhex("76b8e0ada0f13d90405d6ae55386bd28bdd219b8a08ded1aa836efcc8b770dc7"
                        "da41597c5157488d7724e03fb8d84a376a43b8f41518a11cc387b669b2ee6586")
    assert bytes(out) == exp


def test_stdrng_construction_vector():
    """rand 0.8 src/rngs/std.rs test_stdrng_construction target values."""
    o = (ctypes.c_uint64 * 2)()
    seed = bytes([1, 0, 0, 0, 23, 0, 0, 0, 200, 1, 0, 0, 210, 30, 0, 0] + [0] * 16)
    _rng_hooks().wc_rng_stdrng_chain(seed, o)
    assert list(o) == [10719222850664546238, 14064965282130556830]


def test_generate_test_shape_and_determinism():
    c1, s1 = w.generate_test(4, 1000, 30, 0.01)
    c2, s2 = w.generate_test(4, 1000, 30, 0.01)
    assert c1 == c2 and s1 == s2
    assert len(c1) == 1000 and len(s1) == 30 and set(c1) <= {0, 1, 2, 3}
    c0, s0 = w.generate_test(4, 200, 5, 0.0)
    assert all(s == c0 for s in s0)
    cs, _ = w.generate_test(4, 200, 5, 0.0, seed=7)
    assert cs != c0


def test_wfa_ed_doc_examples():
    """sequence_alignment.rs:9-17 and :29-35."""
    v1, v2, v3 = bytes([0, 1, 2, 4, 5]), bytes([0, 1, 3, 4, 5]), bytes([1, 2, 3, 5])
    assert w.wfa_ed(v1, v1) == 0 and w.wfa_ed(v1, v2) == 1 and w.wfa_ed(v1, v3) == 2
    w2 = bytes([0, 1, 2, 4])
    assert w.wfa_ed_config(v1, w2, False, ord("*")) == 0
    assert w.wfa_ed_config(v1, w2, True, ord("*")) == 1


def test_wfa_ed_matches_oracle_random():
    import random
    import oracle_ffi as orc
    rng = random.Random(5)
    for _ in range(300):
        a = bytes(rng.choice(b"ACGT*") for _ in range(rng.randint(0, 30)))
        b = bytes(rng.choice(b"ACGT") for _ in range(rng.randint(0, 30)))
        for both in (True, False):
            assert w.wfa_ed_config(a, b, both, ord("*")) == orc.wfa_ed_config(a, b, both, ord("*"))


def test_pqueue_tracker_capacity():
    """pqueue_tracker.rs:150-171 (test_basic_capacity)."""
    t = w.PQueueTracker.with_capacity(0, 2)
    assert not t.at_capacity(1) and t.processed(1) == 0
    t.process(1)
    assert not t.at_capacity(1) and t.processed(1) == 1
    t.process(1)
    assert t.at_capacity(1) and t.processed(1) == 2
    with pytest.raises(w.WaffleConError, match="Capacity is full"):
        t.process(1)
    assert t.processed(1) == 2


def test_multiconsensus_sort():
    """multi_consensus.rs:73-94."""
    L1 = w.ConsensusCost.L1Distance
    cons = [w.Consensus(b"ACGT", L1, [0]), w.Consensus(b"TGCA", L1, [0]), w.Consensus(b"AAAA", L1, [0])]
    m = w.MultiConsensus.new(cons, [2, 0, 1])
    assert m.consensuses() == [w.Consensus(b"AAAA", L1, [0]), w.Consensus(b"ACGT", L1, [0]),
                               w.Consensus(b"TGCA", L1, [0])]
    assert m.sequence_indices() == [0, 1, 2]


def test_config_builder_doc():
    """cdwfa_config.rs:5-12 doc example and defaults (:71-103)."""
    c = w.CdwfaConfigBuilder().consensus_cost(w.ConsensusCost.L2Distance).wildcard(ord("N")).build()
    assert c.consensus_cost == w.ConsensusCost.L2Distance and c.wildcard == ord("N")
    d = w.CdwfaConfig()
    assert (d.max_queue_size, d.max_capacity_per_size, d.max_return_size, d.max_nodes_wo_constraint,
            d.min_count, d.min_af, d.dual_max_ed_delta, d.offset_window, d.offset_compare_length) == \
        (20, 20, 10, 1000, 3, 0.0, 20, 50, 50)
    assert not d.weighted_by_ed and not d.allow_early_termination and d.auto_shift_offsets and d.wildcard is None


def test_priority_chain_validation():
    """priority_consensus.rs:143-149 error messages (host-side checks)."""
    p = w.PriorityConsensusDWFA()
    with pytest.raises(w.WaffleConError, match="non-empty"):
        p.add_sequence_chain([])
    p.add_sequence_chain([b"ACGT", b"ACGT"])
    with pytest.raises(w.WaffleConError, match="Expected sequences Vec of length 2, but got one of length 1"):
        p.add_sequence_chain([b"ACGT"])


def test_no_device_fails_loudly():
    """The product path has no CPU fallback: without a GPU, creating a context raises."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(w.WaffleConError):
        w.Context(0)


def test_hpc_codec_and_synthetic_shapes():
    from waffle_con_amd import synth
    assert synth.hpc_compress(b"AACCCGTT") == b"ACGT"
    assert synth.hpc_compress(b"") == b"" and synth.hpc_compress(b"A") == b"A"
    assert synth.hpc_chains([b"AAC", b"GGT"]) == [[b"AC", b"AAC"], [b"GT", b"GGT"]]
    a = synth.cfg3_locus(1, length=300, reads=4)
    assert len(a) == 8 and a == synth.cfg3_locus(1, length=300, reads=4)  # seeded
    c4 = synth.cfg4_locus(2, length=400, reads=3, gaps=(0, 5, 10, 20))
    assert len(c4) == 12
    c5 = synth.cfg5_locus(3, len_range=(200, 300), reads_range=(3, 5))
    assert all(len(ch) == 2 and ch[0] == synth.hpc_compress(ch[1]) for ch in c5)


def test_consensus_pickle_and_deepcopy_of_a_lazy_result():
    """A batch result that still views the library's arenas (Consensus._packed)
    pickles and deep-copies as its plain values (consensus.rs derives Clone),
    never as the arenas or the owner's ctypes handle."""
    import copy
    import pickle
    import numpy as np
    from waffle_con_amd.consensus import Consensus

    class _Handle:  # stands in for the result-set owner: not picklable
        def __init__(self):
            self.h = ctypes.c_void_p(1)

        def __reduce__(self):
            raise TypeError("the result-set owner must not be serialised")

    seq = np.frombuffer(b"ACGTTTGCA", dtype=np.uint8)
    sc = np.array([3, 1, 4, 1, 5], dtype=np.uint64)
    idx = [0, 4, 0, 2, 4, 5, 2, 3]
    pack = (seq, idx, sc, _Handle())
    c0 = Consensus._packed(pack, 0, w.ConsensusCost.L1Distance)
    c1 = Consensus._packed(pack, 1, w.ConsensusCost.L2Distance)
    r0 = pickle.loads(pickle.dumps(c0))
    assert r0 == Consensus(b"ACGT", w.ConsensusCost.L1Distance, [3, 1])
    r1 = copy.deepcopy(c1)
    assert r1.sequence() == b"TTGCA" and r1.scores() == [4, 1, 5] and r1._src is None
    assert copy.copy(c1) == c1
