"""GPU parity of the cooperative wave build (engine_coop.hip: the one-wave
dual engine's search on 4 waves, wave w's lane l holding read 64 w + l) on
problems that spread over 1-4 waves, and on the rare paths it shares with the
block engines (wide frontiers and consensus ends, weighted votes, L2 costs,
early termination, the wildcard). WC_COOP=1 forces the build for every dual
launch without offsets; the default takes it for launches of at most one
problem per CU whose largest problem has 65-256 reads. Sequences, scores and
every work counter must equal the oracle's (DualConsensusDWFA,
dual_consensus.rs:240-787; PriorityConsensusDWFA, priority_consensus.rs:172-341)."""
import pytest

import oracle_ffi as orc

pytestmark = pytest.mark.gpu

hip = pytest.importorskip("hip_runner")

KEYS = ("updates", "w_out", "compares", "ed_increases", "finalizes", "pops", "nodes_explored", "nodes_ignored",
        "peak_queue_size", "row_bytes")


@pytest.fixture
def coop(monkeypatch):
    for k in ("WC_WAVE", "WC_NARROW", "WC_LOWLAT", "WC_CU", "WC_GSTATE", "WC_DUAL_CHAIN", "WC_DUAL_HOT"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("WC_COOP", "1")
    monkeypatch.setenv("WAFFLE_CON_SERVICE", "0")
    from waffle_con_amd import _lib
    _lib.default_context().engines_used(reset=True)
    yield


def _used():
    from waffle_con_amd import _lib
    return _lib.default_context().engines_used(reset=True)


def _mix(L, n_a, n_b, err, seeds):
    import waffle_con_amd as w
    a = w.generate_test(4, L, n_a, err, seeds[0])[1]
    b = w.generate_test(4, L, n_b, err, seeds[1])[1]
    out = []
    for k in range(max(n_a, n_b)):
        if k < n_a:
            out.append(a[k])
        if k < n_b:
            out.append(b[k])
    return out


def _check(seqs, **cfg):
    exp, ec = orc.dual_consensus(seqs, counters=True, **cfg)
    got, gc = hip.dual_consensus(seqs, counters=True, **cfg)
    assert _used() == ["coop.dual"]
    assert got == exp
    for k in KEYS:
        assert gc[k] == ec[k], (k, gc[k], ec[k])


# reads per problem: one wave (40), a partial second wave (66), two full (128),
# a partial fourth (200), four full (256)
@pytest.mark.parametrize("L,n_a,n_b,err,seeds", [(700, 20, 20, 0.01, (8, 9)), (500, 33, 33, 0.01, (20, 21)),
                                                 (500, 64, 64, 0.01, (10, 11)), (400, 100, 100, 0.01, (12, 13)),
                                                 (300, 128, 128, 0.01, (14, 15))])
def test_coop_dual_sizes(coop, L, n_a, n_b, err, seeds):
    _check(_mix(L, n_a, n_b, err, seeds), min_count=max(2, (n_a + n_b) // 8))


def test_coop_unbalanced_split_and_single_haplotype(coop):
    """An 80/20 split (min_af decides the split children) and one haplotype
    only (no split: stay-single children, then the consensus end)."""
    _check(_mix(500, 80, 20, 0.01, (30, 31)), min_count=3, min_af=0.1)
    _check(_mix(500, 90, 0, 0.01, (32, 33)), min_count=3)


def test_coop_rare_paths(coop):
    """Weighted votes (the block engines' f64 votes), L2 costs, early
    termination with ragged read lengths (reads at consensus ends), noisy
    reads (wide frontiers, split ties) and the wildcard."""
    seqs = _mix(300, 50, 50, 0.02, (40, 41))
    _check(seqs, min_count=5, weighted_by_ed=True)
    _check(seqs, min_count=5, consensus_cost=1)
    ragged = [s[:len(s) - (7 * k) % 60] for k, s in enumerate(_mix(300, 45, 45, 0.01, (42, 43)))]
    _check(ragged, min_count=5, allow_early_termination=True)
    _check(_mix(150, 40, 40, 0.12, (44, 45)), min_count=4)
    wc = [bytes(ord("*") if (k * 31 + i) % 97 == 0 else c for i, c in enumerate(s))
          for k, s in enumerate(_mix(200, 40, 40, 0.01, (46, 47)))]
    _check(wc, min_count=4, wildcard=ord("*"))


def test_coop_priority_cfg5_loci(coop):
    """PriorityConsensusDWFA sub-problems of 30-80 reads on the cooperating
    waves (cfg5 loci; the batch path)."""
    from waffle_con_amd import synth
    for seed in (2, 2274, 303):  # (30, 76 and 66 reads)
        chains = synth.cfg5_locus(seed)
        exp, ec = orc.priority_consensus(chains, counters=True, wildcard=ord("*"))
        got, gc = hip.priority_consensus(chains, counters=True, wildcard=ord("*"))
        assert "coop.dual" in _used()
        assert got == exp
        for k in KEYS:
            assert gc[k] == ec[k], (seed, k, gc[k], ec[k])


def test_wave_stream_pool_for_occupancy(monkeypatch, capfd):
    """A PriorityConsensusDWFA stream with more sub-problems than fit on the
    chip at once plans the one-wave engine's node pool for occupancy: the
    smallest pool, down to 256 nodes, that gives another workgroup per CU
    (engine_host.cpp plan_caps; a pool of 512 gives 3 per CU). One CU
    (WC_DEVICE_SHARE on a fresh context) makes six loci such a launch.
    Results and counters must equal the oracle's
    (priority_consensus.rs:172-341)."""
    import waffle_con_amd as w
    from waffle_con_amd import _lib, synth
    from waffle_con_amd.cdwfa_config import CdwfaConfig
    for k in ("WC_WAVE", "WC_COOP", "WC_DUAL_LDS_KB", "WC_NARROW", "WC_LOWLAT", "WC_CU", "WC_GSTATE"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("WC_DEVICE_SHARE", "256")
    monkeypatch.setenv("WC_LAUNCH_LOG", "1")
    monkeypatch.setenv("WAFFLE_CON_SERVICE", "0")
    ctx = _lib.Context(0)
    seeds = (2, 6, 8, 9, 17, 303)
    loci = [synth.cfg5_locus(s) for s in seeds]
    cfg = CdwfaConfig(wildcard=ord("*"))
    res, st = w.priority_consensus_batch([(L, None, None) for L in loci], cfg, context=ctx, per_problem=True)
    log = capfd.readouterr().err
    launches = [ln for ln in log.splitlines() if "stream launch" in ln]
    assert launches and "grid=4 per_cu=4 " in launches[0] and "pcap=256 " in launches[0], launches
    for L, r, pp in zip(loci, res, st["per_problem"]):
        exp, ec = orc.priority_consensus(L, counters=True, wildcard=ord("*"))
        got = {"consensuses": [[hip._cons(c) for c in chain] for chain in r.consensuses()],
               "sequence_indices": list(r.sequence_indices())}
        assert got == exp
        for k in KEYS:
            assert pp[k] == ec[k], (k, pp[k], ec[k])
