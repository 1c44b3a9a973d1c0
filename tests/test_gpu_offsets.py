"""GPU parity for offset activation (add_sequence_offset):
reads that start part-way through the consensus are activated on the device
when a node reaches offset + offset_compare_length (consensus.rs:327-335,
413-448; dual_consensus.rs:633-639, 866-906; wfa_ed_config
sequence_alignment.rs:36-87). Results and work counters must equal the CPU
oracle's bit for bit."""
import random

import pytest

import oracle_ffi as orc

pytestmark = pytest.mark.gpu
hip = pytest.importorskip("hip_runner")

COUNTER_KEYS = ("updates", "w_out", "compares", "ed_increases", "finalizes", "pops", "nodes_explored",
                "nodes_ignored", "peak_queue_size", "row_bytes")


def _truncated(L, N, err, seed, frac=0.5, jitter=3, min_cut=8):
    """example_gen reads; a fraction of them lose a prefix and carry the cut
    position (+- jitter) as their approximate offset."""
    import waffle_con_amd as w
    _, reads = w.generate_test(4, L, N, err, seed)
    rng = random.Random(seed)
    seqs, offs = [], []
    for i, r in enumerate(reads):
        if i > 0 and rng.random() < frac:
            cut = rng.randint(min_cut, max(min_cut, len(r) // 2))
            seqs.append(r[cut:])
            offs.append(max(0, cut + rng.randint(-jitter, jitter)))
        else:
            seqs.append(r)
            offs.append(None)
    return seqs, offs


@pytest.mark.parametrize("L,N,err,seed,cfg", [
    (300, 10, 0.02, 0, dict(min_count=3)),
    (600, 16, 0.01, 1, dict(min_count=4)),
    (400, 12, 0.03, 2, dict(min_count=3, offset_window=10, offset_compare_length=20)),
    (250, 8, 0.02, 3, dict(min_count=2, consensus_cost=1)),
    (300, 10, 0.02, 4, dict(min_count=3, offset_window=80, offset_compare_length=30)),
    (500, 20, 0.01, 5, dict(min_count=5, allow_early_termination=True)),
])
def test_single_offsets_vs_oracle(L, N, err, seed, cfg):
    seqs, offs = _truncated(L, N, err, seed)
    exp, ec = orc.consensus(seqs, offsets=offs, counters=True, **cfg)
    got, gc = hip.consensus(seqs, offsets=offs, counters=True, **cfg)
    assert got == exp
    for k in COUNTER_KEYS:
        assert gc[k] == ec[k], (k, gc[k], ec[k])


def test_single_offsets_auto_shift():
    """Every read has an offset: auto_shift_offsets makes the smallest the start."""
    seqs, offs = _truncated(300, 8, 0.02, 7, frac=1.0)
    offs[0] = 5
    exp = orc.consensus(seqs, offsets=offs, min_count=2)
    assert hip.consensus(seqs, offsets=offs, min_count=2) == exp


def test_single_coverage_gap_message():
    """consensus.rs:303-305: no candidates before the last activation point (early
    termination keeps the inactive read from triggering a finalize first)."""
    seqs = [b"ACGTACGTAC", b"TTTTTTTTTTTTTTTT"]
    offs = [None, 40]
    with pytest.raises(Exception) as ex_o:
        orc.consensus(seqs, offsets=offs, min_count=1, offset_window=1, offset_compare_length=4,
                      allow_early_termination=True)
    with pytest.raises(Exception) as ex_h:
        hip.consensus(seqs, offsets=offs, min_count=1, offset_window=1, offset_compare_length=4,
                      allow_early_termination=True)
    assert str(ex_h.value) == str(ex_o.value)
    assert str(ex_h.value).startswith("Encountered coverage gap: consensus is length 10")


@pytest.mark.parametrize("seed", range(4))
def test_dual_offsets_vs_oracle(seed):
    from test_gpu_dual import _two_haplotypes
    reads = _two_haplotypes(160, 6, 0.02, 300 + seed)
    rng = random.Random(seed)
    seqs, offs = [], []
    for i, r in enumerate(reads):
        if i % 3 == 2:
            cut = rng.randint(10, 60)
            seqs.append(r[cut:])
            offs.append(cut + rng.randint(-2, 2))
        else:
            seqs.append(r)
            offs.append(None)
    cfg = dict(min_count=3)
    exp, ec = orc.dual_consensus(seqs, offsets=offs, counters=True, **cfg)
    got, gc = hip.dual_consensus(seqs, offsets=offs, counters=True, **cfg)
    assert got == exp
    for k in COUNTER_KEYS:
        assert gc[k] == ec[k], (k, gc[k], ec[k])


@pytest.mark.parametrize("seed", range(3))
def test_priority_seeded_offsets_vs_oracle(priority_path, seed):
    from test_gpu_dual import _two_haplotypes
    reads = _two_haplotypes(120, 5, 0.01, 400 + seed)
    rng = random.Random(seed)
    chains, offsets = [], []
    for i, r in enumerate(reads):
        if i % 4 == 3:
            cut = rng.randint(10, 40)
            chains.append([r[cut:], r[cut:len(r) // 2 + cut]])
            offsets.append([cut, cut])
        else:
            chains.append([r, r[: len(r) // 2]])
            offsets.append([None, None])
    cfg = dict(min_count=3, wildcard=ord("*"), offset_window=10, offset_compare_length=10)
    exp = orc.priority_consensus(chains, offsets=offsets, **cfg)
    assert hip.priority_consensus(chains, offsets=offsets, **cfg) == exp
