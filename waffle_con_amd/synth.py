"""Synthetic workload shapes of SURVEY.md §8(d) and the homopolymer-compressed
(HPC) chain builder of the PriorityConsensusDWFA use case
(priority_consensus.rs:91-92: "first split sequences by homo-polymer
compressed sequences and then the full-length sequences").

cfg1/cfg2 use the reference's own generator (example_gen.rs, `generate_test`).
The multi-haplotype shapes below (cfg3 dual split, cfg4 length gaps, cfg5 PGx
loci) have no generator in the reference; they are seeded numpy constructions
with the example_gen error model (per base: substitution, insertion after it,
or deletion, each with probability rate/3). The CPU oracle and the device
engine consume the same bytes. Everything is vectorised, so a 10,000-locus
cfg5 batch generates in seconds.
"""
import numpy as np

ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)
_IDX = np.zeros(256, dtype=np.int64)
_IDX[ACGT] = np.arange(4)


def _rng(seed, stream=0):
    return np.random.default_rng([int(seed), int(stream)])


def _arr(seq):
    return np.frombuffer(bytes(seq), dtype=np.uint8) if not isinstance(seq, np.ndarray) else seq


def hpc_compress(seq):
    """Collapse every homopolymer run to one symbol: b"AACCCGT" -> b"ACGT"."""
    a = _arr(seq)
    if a.size == 0:
        return b""
    keep = np.empty(a.size, dtype=bool)
    keep[0] = True
    np.not_equal(a[1:], a[:-1], out=keep[1:])
    return a[keep].tobytes()


def hpc_chains(reads):
    """One priority chain per read: [HPC(read), read] (cfg5)."""
    return [[hpc_compress(r), bytes(r)] for r in reads]


def random_seq(rng, n):
    return ACGT[rng.integers(0, 4, n)]


def mutate(rng, seq, rate):
    """example_gen-style read of `seq` (ACGT bytes): each base is substituted
    (by one of the three others), followed by an inserted random base, or
    deleted, with probability rate/3 each. Returns bytes."""
    a = _arr(seq)
    u = rng.random(a.size)
    sub = u < rate / 3
    ins = (u >= rate / 3) & (u < 2 * rate / 3)
    dele = (u >= 2 * rate / 3) & (u < rate)
    b = a.copy()
    ns = int(sub.sum())
    if ns:
        b[sub] = ACGT[(_IDX[a[sub]] + rng.integers(1, 4, ns)) % 4]
    counts = (~dele).astype(np.int64) + ins
    out = np.repeat(b, counts)
    ni = int(ins.sum())
    if ni:
        last = np.cumsum(counts) - 1
        out[last[ins]] = ACGT[rng.integers(0, 4, ni)]
    return out.tobytes()


def _variant(rng, hap, n_snv, n_indel, margin=20):
    h = bytearray(bytes(hap))
    L = len(h)
    if L <= 2 * margin:
        return bytes(h)
    span = L - 2 * margin
    for p in rng.choice(span, min(n_snv, span), replace=False) + margin:
        h[p] = int(ACGT[(_IDX[h[p]] + rng.integers(1, 4)) % 4])
    for p in sorted(rng.choice(span, min(n_indel, span), replace=False) + margin, reverse=True):
        k = int(rng.integers(1, 4))
        if rng.random() < 0.5:
            del h[p:p + k]
        else:
            h[p:p] = random_seq(rng, k).tobytes()
    return bytes(h)


def cfg3_locus(seed, length=5000, reads=100, err=0.005):
    """Dual split: haplotype A, B = A + 12 SNVs + 2 indels (1-3 bp); `reads`
    reads of each, A-block then B-block."""
    rng = _rng(seed, 3)
    a = random_seq(rng, length).tobytes()
    b = _variant(rng, a, 12, 2)
    return [mutate(rng, a, err) for _ in range(reads)] + [mutate(rng, b, err) for _ in range(reads)]


def cfg4_locus(seed, length=8000, reads=50, err=0.005, gaps=(0, 25, 60, 150)):
    """Four haplotypes from one base: an inserted segment of each length in
    `gaps` at distinct positions, plus 3 SNVs each; reads grouped by haplotype."""
    rng = _rng(seed, 4)
    base = random_seq(rng, length).tobytes()
    pos = rng.choice(np.arange(length // 10, length - length // 10), len(gaps), replace=False)
    out = []
    for g, p in zip(gaps, pos):
        h = base[:p] + random_seq(rng, g).tobytes() + base[p:]
        h = _variant(rng, h, 3, 0)
        out += [mutate(rng, h, err) for _ in range(reads)]
    return out


def cfg5_params(seed, len_range=(1000, 6000), reads_range=(15, 40), max_variants=15):
    """(length, variants, reads per haplotype) of cfg5 locus `seed`, drawn from
    their own stream, so a batch can be cost-sorted before it is generated."""
    rng = _rng(seed, 50)
    L = int(rng.integers(len_range[0], len_range[1] + 1))
    nv = int(rng.integers(0, max_variants + 1))
    n = int(rng.integers(reads_range[0], reads_range[1] + 1))
    return L, nv, n


def cfg5_cost(seed, **kw):
    """Estimated cost of cfg5 locus `seed`: reads x length, both levels
    (shard.locus_cost; the better predictor of its critical path)."""
    L, _, n = cfg5_params(seed, **kw)
    return 2 * n * L * 2


def cfg5_locus(seed, len_range=(1000, 6000), reads_range=(15, 40), err=0.005, max_variants=15):
    """PGx-like locus: length U[len_range], two haplotypes differing by
    U{0..max_variants} variants, U[reads_range] reads each; returned as HPC
    chains [HPC(read), read]."""
    L, nv, n = cfg5_params(seed, len_range, reads_range, max_variants)
    rng = _rng(seed, 5)
    a = random_seq(rng, L).tobytes()
    b = _variant(rng, a, nv - nv // 4, nv // 4)
    reads = [mutate(rng, a, err) for _ in range(n)] + [mutate(rng, b, err) for _ in range(n)]
    return hpc_chains(reads)
