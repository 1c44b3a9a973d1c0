"""Synthetic workload shapes of SURVEY.md §8(d) and the homopolymer-compressed
(HPC) chain builder of the PriorityConsensusDWFA use case
(priority_consensus.rs:91-92: "first split sequences by homo-polymer
compressed sequences and then the full-length sequences").

cfg1/cfg2 use the reference's own generator (example_gen.rs, `generate_test`).
The multi-haplotype shapes below (cfg3 dual split, cfg4 length gaps, cfg5 PGx
loci) have no generator in the reference; they are seeded Python
constructions with the example_gen error model (uniform substitution /
insertion / deletion). CPU oracle and device engine consume the same bytes.
"""
import random

ACGT = b"ACGT"


def hpc_compress(seq):
    """Collapse every homopolymer run to one symbol: b"AACCCGT" -> b"ACGT"."""
    seq = bytes(seq)
    out = bytearray()
    for c in seq:
        if not out or out[-1] != c:
            out.append(c)
    return bytes(out)


def hpc_chains(reads):
    """One priority chain per read: [HPC(read), read] (cfg5)."""
    return [[hpc_compress(r), bytes(r)] for r in reads]


def mutate(rng, seq, rate):
    """example_gen-style read: each base is substituted, followed by an
    inserted base, or deleted with probability rate/3 each."""
    out = bytearray()
    for c in seq:
        r = rng.random()
        if r < rate / 3:
            out.append(rng.choice(ACGT.replace(bytes([c]), b"")))
        elif r < 2 * rate / 3:
            out.append(c)
            out.append(rng.choice(ACGT))
        elif r < rate:
            continue
        else:
            out.append(c)
    return bytes(out)


def _variant(rng, hap, n_snv, n_indel, margin=20):
    h = bytearray(hap)
    L = len(h)
    if L <= 2 * margin:
        return bytes(h)
    for p in rng.sample(range(margin, L - margin), min(n_snv, L - 2 * margin)):
        h[p] = rng.choice(ACGT.replace(bytes([h[p]]), b""))
    for p in sorted(rng.sample(range(margin, L - margin), min(n_indel, L - 2 * margin)), reverse=True):
        k = rng.randint(1, 3)
        if rng.random() < 0.5:
            del h[p:p + k]
        else:
            h[p:p] = bytes(rng.choice(ACGT) for _ in range(k))
    return bytes(h)


def cfg3_locus(seed, length=5000, reads=100, err=0.005):
    """Dual split: haplotype A, B = A + 12 SNVs + 2 indels (1-3 bp); `reads`
    reads of each, A-block then B-block."""
    rng = random.Random(seed)
    a = bytes(rng.choice(ACGT) for _ in range(length))
    b = _variant(rng, a, 12, 2)
    return [mutate(rng, a, err) for _ in range(reads)] + [mutate(rng, b, err) for _ in range(reads)]


def cfg4_locus(seed, length=8000, reads=50, err=0.005, gaps=(0, 25, 60, 150)):
    """Four haplotypes from one base: an inserted segment of each length in
    `gaps` at distinct positions, plus 3 SNVs each; reads grouped by haplotype."""
    rng = random.Random(seed)
    base = bytes(rng.choice(ACGT) for _ in range(length))
    pos = rng.sample(range(length // 10, length - length // 10), len(gaps))
    out = []
    for g, p in zip(gaps, pos):
        h = base[:p] + bytes(rng.choice(ACGT) for _ in range(g)) + base[p:]
        h = _variant(rng, h, 3, 0)
        out += [mutate(rng, h, err) for _ in range(reads)]
    return out


def cfg5_locus(seed, len_range=(1000, 6000), reads_range=(15, 40), err=0.005, max_variants=15):
    """PGx-like locus: length U[len_range], two haplotypes differing by
    U{0..max_variants} variants, U[reads_range] reads each; returned as HPC
    chains [HPC(read), read]."""
    rng = random.Random(seed)
    L = rng.randint(*len_range)
    a = bytes(rng.choice(ACGT) for _ in range(L))
    nv = rng.randint(0, max_variants)
    b = _variant(rng, a, nv - nv // 4, nv // 4)
    n = rng.randint(*reads_range)
    reads = [mutate(rng, a, err) for _ in range(n)] + [mutate(rng, b, err) for _ in range(n)]
    return hpc_chains(reads)
