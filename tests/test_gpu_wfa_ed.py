"""GPU parity: batched wfa_ed / wfa_ed_config on the device (wc_wfa_ed_batch,
sequence_alignment.rs:18-87) vs the reference's doc vectors
(sequence_alignment.rs:9-16, 30-33) and vs the oracle on seeded pairs: empty
and one-sided inputs, wildcards on either side, both end modes, and pairs whose
wavefront spans several 64-entry chunks (edit distance > 32)."""
import random

import pytest

import oracle_ffi as orc

pytestmark = pytest.mark.gpu
w = pytest.importorskip("waffle_con_amd")

STAR = ord("*")


def test_doc_vectors():
    v1, v2, v3 = [0, 1, 2, 4, 5], [0, 1, 3, 4, 5], [1, 2, 3, 5]
    assert w.wfa_ed_batch([(v1, v1), (v1, v2), (v1, v3)]) == [0, 1, 2]
    w2 = [0, 1, 2, 4]
    assert w.wfa_ed_batch([(v1, w2)], require_both_end=False) == [0]
    assert w.wfa_ed_batch([(v1, w2)], require_both_end=True) == [1]


def test_empty_and_one_sided():
    pairs = [(b"", b""), (b"ACGT", b""), (b"", b"ACGT"), (b"A", b"C"), (b"*", b"G"), (b"AC", b"*")]
    for both in (True, False):
        for wc in (STAR, None):
            got = w.wfa_ed_batch(pairs, require_both_end=both, wildcard=wc)
            exp = [orc.wfa_ed_config(a, b, both, wc) for a, b in pairs]
            assert got == exp, (both, wc)


def _mutate(rng, s, rate, alphabet):
    out = bytearray()
    for c in s:
        r = rng.random()
        if r < rate / 3:
            out.append(rng.choice(alphabet))  # substitution (may be silent)
        elif r < 2 * rate / 3:
            out.append(c)
            out.append(rng.choice(alphabet))  # insertion
        elif r < rate:
            continue  # deletion
        else:
            out.append(c)
    return bytes(out)


def _pairs(seed, n, max_len, alphabet, wc_rate=0.0):
    rng = random.Random(seed)
    pairs = []
    for _ in range(n):
        L = rng.randint(0, max_len)
        a = bytes(rng.choice(alphabet) for _ in range(L))
        b = _mutate(rng, a, rng.choice([0.0, 0.01, 0.05, 0.2, 0.6]), alphabet)
        if rng.random() < 0.3:
            b = b[: rng.randint(0, len(b))]  # prefix (partial-read shape)
        if wc_rate:
            a = bytes(STAR if rng.random() < wc_rate else c for c in a)
            b = bytes(STAR if rng.random() < wc_rate else c for c in b)
        pairs.append((a, b))
    return pairs


@pytest.mark.parametrize("both", [True, False])
@pytest.mark.parametrize("wc", [STAR, None])
def test_random_pairs_match_oracle(both, wc):
    pairs = _pairs(17, 300, 400, b"ACGT", wc_rate=0.02)
    got = w.wfa_ed_batch(pairs, require_both_end=both, wildcard=wc)
    exp = [orc.wfa_ed_config(a, b, both, wc) for a, b in pairs]
    assert got == exp


def test_wide_wavefronts():
    # unrelated sequences: edit distances in the hundreds, 2e+1 >> 64 entries
    rng = random.Random(5)
    pairs = [(bytes(rng.choice(b"ACGT") for _ in range(rng.randint(100, 600))),
              bytes(rng.choice(b"ACGT") for _ in range(rng.randint(100, 600)))) for _ in range(24)]
    got = w.wfa_ed_batch(pairs)
    exp = [orc.wfa_ed(a, b) for a, b in pairs]
    assert got == exp
    assert max(exp) > 200


def test_hifi_reads_10kb():
    # generate_test reads against their consensus (cfg2 shape)
    con, reads = w.generate_test(4, 10000, 8, 0.005, 3)
    pairs = [(con, r) for r in reads] + [(reads[0], r) for r in reads[1:]]
    got = w.wfa_ed_batch(pairs, wildcard=None)
    exp = [orc.wfa_ed_config(a, b, True, None) for a, b in pairs]
    assert got == exp


def test_matches_single_call_api():
    pairs = _pairs(23, 40, 200, b"AC*")
    got = w.wfa_ed_batch(pairs)
    assert got == [w.wfa_ed(a, b) for a, b in pairs]
