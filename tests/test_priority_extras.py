"""PriorityConsensusDWFA beyond the reference's own fixtures
(priority_consensus.rs:141-341): seed-group processing order, per-level
offsets, work counters and errors part-way down the split stack.

The seed-group order comes from an FxHashSet<Option<usize>> built with
`.collect()` (priority_consensus.rs:180). No reference test pins it, so the
CPU test checks the oracle against an independent statement of hashbrown's
placement rules (table pre-sized by the iterator's exact size hint), and the
GPU tests compare the HIP path with the oracle on inputs where the order is
observable (identical chains keep processing order under the final stable
sort, priority_consensus.rs:309-335).
"""
import pytest

import oracle_ffi as orc

M64 = (1 << 64) - 1
FX = 0x517CC1B727220A95


def _fx_opt(v):
    # derive(Hash) for Option<usize>: discriminant (isize) then the payload
    def add(h, w):
        return ((((h << 5) | (h >> 59)) & M64) ^ w) * FX & M64
    return add(0, 0) if v is None else add(add(0, 1), v)


def _buckets(cap):
    if cap < 8:
        return 4 if cap < 4 else 8
    adj = cap * 8 // 7
    p = 1
    while p < adj:
        p <<= 1
    return p


def _hashbrown_collect_order(groups):
    """Iteration order of `groups.iter().cloned().collect::<FxHashSet<_>>()`:
    extend() reserves size_hint (= len) first, so no growth happens; inserts
    probe from h1 = hash & mask (16-wide groups, triangular strides; tables
    under 16 buckets scan [pos, B) then wrap to 0)."""
    B = _buckets(max(len(groups), 1))
    tab = [None] * B
    used = [False] * B
    seen = []
    for g in groups:
        if g in seen:
            continue
        seen.append(g)
        h = _fx_opt(g)
        pos = h & (B - 1)
        if B < 16:
            cand = [i for i in range(pos, B) if not used[i]] + [i for i in range(B) if not used[i]]
            slot = cand[0]
        else:
            stride = 0
            slot = None
            while slot is None:
                for j in range(16):
                    i = (pos + j) & (B - 1)
                    if not used[i]:
                        slot = i
                        break
                stride += 16
                pos = (pos + stride) & (B - 1)
        used[slot] = True
        tab[slot] = g
    return [tab[i] for i in range(B) if used[i]]


@pytest.mark.parametrize("groups", [
    [None] * 5,
    [None, 1, None, 2],
    [3, 7, 3, 12, None, 5, 9, 9, 1, 0, 2, 4, 6, 8, 10, 11, 13, 14, 15, 16],
    [100 + 7 * i for i in range(20)],
    [i % 6 for i in range(40)],
    [None if i % 3 == 0 else i * 31 for i in range(33)],
])
def test_seed_group_order_matches_hashbrown_collect(groups):
    assert orc.seed_group_order(groups) == _hashbrown_collect_order(groups)


def _chains(seed, n_hap=2, per=4, L=120, err=0.01):
    import numpy as np
    from waffle_con_amd import synth
    rng = np.random.default_rng(seed)
    haps = [synth.random_seq(rng, L).tobytes() for _ in range(n_hap)]
    reads = [synth.mutate(rng, h, err) for h in haps for _ in range(per)]
    return [[synth.hpc_compress(r), r] for r in reads]


COUNTER_KEYS = ("updates", "w_out", "compares", "ed_increases", "finalizes", "pops", "nodes_explored",
                "nodes_ignored", "peak_queue_size", "row_bytes")


def _cmp_priority(hip, chains, offsets=None, seed_groups=None, **cfg):
    try:
        exp, ec = orc.priority_consensus(chains, offsets=offsets, seed_groups=seed_groups, counters=True, **cfg)
    except Exception as e:  # noqa: BLE001 - the HIP path must fail the same way
        with pytest.raises(Exception) as eh:
            hip.priority_consensus(chains, offsets=offsets, seed_groups=seed_groups, counters=True, **cfg)
        assert str(eh.value) == str(e)
        return
    got, gc = hip.priority_consensus(chains, offsets=offsets, seed_groups=seed_groups, counters=True, **cfg)
    assert got == exp
    for k in COUNTER_KEYS:
        assert gc[k] == ec[k], (k, gc[k], ec[k])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_gpu_priority_counters_vs_oracle(priority_path, seed):
    hip = pytest.importorskip("hip_runner")
    _cmp_priority(hip, _chains(500 + seed), min_count=2, wildcard=ord("*"))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(2))
def test_gpu_priority_seed_groups_vs_oracle(priority_path, seed):
    """Several seed groups over 20 chains; groups 1 and 3 hold identical reads,
    so their (identical) chains keep the seed-group processing order."""
    hip = pytest.importorskip("hip_runner")
    base = _chains(600 + seed, n_hap=2, per=5)
    chains = base + [list(c) for c in base]
    groups = [None] * 5 + [1] * 5 + [7, 7, 7, 7, 7] + [3] * 5
    _cmp_priority(hip, chains, seed_groups=groups, min_count=2, wildcard=ord("*"))


@pytest.mark.gpu
def test_gpu_priority_per_level_offsets_vs_oracle(priority_path):
    """Offsets on the second chain level only (activation at a consensus length)."""
    hip = pytest.importorskip("hip_runner")
    chains = _chains(700, n_hap=2, per=5, L=200)
    offsets = [[None, None if i % 3 else 10 + i] for i in range(len(chains))]
    _cmp_priority(hip, chains, offsets=offsets, min_count=2, wildcard=ord("*"))


@pytest.mark.gpu
def test_gpu_priority_error_mid_stack_vs_oracle(priority_path):
    """A level-1 sub-problem whose reads all carry offsets fails (no start) after
    the level-0 split succeeded: the error and its precedence match."""
    hip = pytest.importorskip("hip_runner")
    chains = _chains(800, n_hap=2, per=5, L=150)
    offsets = [[None, 5 + (i % 4)] for i in range(len(chains))]
    _cmp_priority(hip, chains, offsets=offsets, min_count=2, wildcard=ord("*"), auto_shift_offsets=False)


@pytest.mark.gpu
def test_gpu_priority_batch_per_problem_start_times():
    """wc_stats.start_ms (per problem of a PriorityConsensusDWFA batch): when
    its first sub-problem was published to the device, from the start of the
    call; never after its result (wall_ms), and the results and counters are
    the oracle's for every locus."""
    import waffle_con_amd as w
    from waffle_con_amd.cdwfa_config import CdwfaConfig
    from waffle_con_amd import synth
    loci = [synth.cfg5_locus(s) for s in range(6)]
    res, st = w.priority_consensus_batch([(ch, None, None) for ch in loci], CdwfaConfig(wildcard=ord("*")),
                                         per_problem=True)
    pp = st["per_problem"]
    assert len(pp) == len(loci)
    for chains, r, p in zip(loci, res, pp):
        assert 0.0 <= p["start_ms"] <= p["wall_ms"]
        exp, ec = orc.priority_consensus(chains, counters=True, wildcard=ord("*"))
        assert [[c.sequence() for c in ch] for ch in r.consensuses()] == \
            [[c["sequence"] for c in ch] for ch in exp["consensuses"]]
        for k in ("pops", "updates", "w_out", "compares", "ed_increases"):
            assert p[k] == ec[k], k
