"""GPU parity of every engine build on the same problems: the 256-thread
build at 4 waves/SIMD (WC_NARROW=0 WC_LOWLAT=0), the same at 2 waves/SIMD
(engine_lowlat.hip, the default for launches of at most 2 problems per CU),
the 128-thread build (engine_narrow.hip; WC_NARROW bit 0 = single engine,
bit 1 = dual engine, default 2), the global-state build (WC_GSTATE), the
1024-thread single engine (engine_cu.hip, the default for batch launches of
at most one problem per CU; WC_CU=1 forces it, WC_CU=0 keeps it off in the
other variants; dual problems keep their 4-wave build there: the dual engine
has no whole-CU build), each dual build with dual_hot forced on, and the one-wave
dual engine (engine_wave.hip, the default for dual problems without offsets;
WC_WAVE=0 in every other variant) and its search on cooperating waves
(engine_coop.hip, WC_COOP=1; WC_COOP=0 in every other variant). The build is picked per launch from
the environment (engine_host.cpp plan_caps), so one process exercises all of
them. The calls take the per-call batch path (WAFFLE_CON_SERVICE=0) on the
thread's default context, whose wc_engines_used mask must name the build the
variant is meant to run: a variant that silently ran another build would pass
the parity checks without testing anything. Sequences, scores and every work
counter must equal the oracle's."""
import os

import pytest

import oracle_ffi as orc

pytestmark = pytest.mark.gpu

hip = pytest.importorskip("hip_runner")

KEYS = ("updates", "w_out", "compares", "ed_increases", "finalizes", "pops", "nodes_explored", "nodes_ignored",
        "peak_queue_size", "row_bytes")
BUILDS = {"wide": {"WC_NARROW": "0", "WC_LOWLAT": "0"}, "lowlat": {"WC_NARROW": "0"},
          "narrow-single": {"WC_NARROW": "1"}, "narrow-dual": {"WC_NARROW": "2"}, "narrow": {"WC_NARROW": "3"},
          "gstate": {"WC_GSTATE": "1"}, "cu": {"WC_CU": "1"},
          # the dual engine with the popped node's RStates in LDS (dual_hot: an
          # opt-in knob, measured not to pay; forced here in every dual build)
          "wide-hot": {"WC_NARROW": "0", "WC_LOWLAT": "0", "WC_DUAL_HOT": "2"},
          "lowlat-hot": {"WC_NARROW": "0", "WC_DUAL_HOT": "2"}, "narrow-hot": {"WC_NARROW": "2", "WC_DUAL_HOT": "2"},
          "wave": {"WC_WAVE": "1"},
          # the one-wave engine's search on cooperating waves (engine_coop.hip,
          # the default for 65-256-read problems in launches of at most one per
          # CU; WC_COOP=1 forces it, WC_COOP=0 keeps it off in the other variants)
          "coop": {"WC_COOP": "1"}}
# the engine build (wc_engine_name) each variant runs for one problem of at
# most 128 reads: (single, dual)
ENGINES = {"wide": ("lds.single", "lds.dual"), "lowlat": ("lowlat.single", "lowlat.dual"),
           "narrow-single": ("narrow.single", "lowlat.dual"), "narrow-dual": ("lowlat.single", "narrow.dual"),
           "narrow": ("narrow.single", "narrow.dual"), "gstate": ("gstate.single", "gstate.dual"),
           "cu": ("cu.single", "narrow.dual"), "wide-hot": ("lds.single", "lds.dual"),
           "lowlat-hot": ("lowlat.single", "lowlat.dual"), "narrow-hot": ("lowlat.single", "narrow.dual"),
           "wave": ("lowlat.single", "wave.dual"), "coop": ("lowlat.single", "coop.dual")}
KNOBS = ("WC_NARROW", "WC_GSTATE", "WC_LOWLAT", "WC_DUAL_HOT", "WC_CU", "WC_WAVE", "WC_COOP", "WC_CHAIN",
         "WC_DUAL_CHAIN")


@pytest.fixture(params=sorted(BUILDS))
def build(request, monkeypatch):
    for k in KNOBS:
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("WC_CU", "0")
    monkeypatch.setenv("WC_WAVE", "0")  # (the default for dual problems without offsets)
    monkeypatch.setenv("WC_COOP", "0")  # (the default for 65-256-read dual problems, few per launch)
    monkeypatch.setenv("WAFFLE_CON_SERVICE", "0")
    for k, v in BUILDS[request.param].items():
        monkeypatch.setenv(k, v)
    from waffle_con_amd import _lib
    _lib.default_context().engines_used(reset=True)
    yield request.param


def _used():
    from waffle_con_amd import _lib
    return _lib.default_context().engines_used(reset=True)


def _gen(L, N, err, seed):
    import waffle_con_amd as w
    return w.generate_test(4, L, N, err, seed)[1]


@pytest.mark.parametrize("L,N,err,seed", [(1500, 40, 0.01, 5), (800, 128, 0.02, 6), (600, 3, 0.05, 7)])
def test_single_builds(build, L, N, err, seed):
    seqs = _gen(L, N, err, seed)
    cfg = dict(min_count=max(1, N // 4))
    exp, ec = orc.consensus(seqs, counters=True, **cfg)
    got, gc = hip.consensus(seqs, counters=True, **cfg)
    assert _used() == [ENGINES[build][0]]
    assert got == exp
    for k in KEYS:
        assert gc[k] == ec[k], (build, k, gc[k], ec[k])


@pytest.mark.parametrize("L,N,err,seeds", [(700, 20, 0.01, (8, 9)), (500, 64, 0.01, (10, 11))])
def test_dual_builds(build, L, N, err, seeds):
    a = _gen(L, N, err, seeds[0])
    b = _gen(L, N, err, seeds[1])
    mix = [x for pair in zip(a, b) for x in pair]
    exp, ec = orc.dual_consensus(mix, counters=True, min_count=max(2, N // 4))
    got, gc = hip.dual_consensus(mix, counters=True, min_count=max(2, N // 4))
    assert _used() == [ENGINES[build][1]]
    assert got == exp
    for k in KEYS:
        assert gc[k] == ec[k], (build, k, gc[k], ec[k])


def test_priority_builds(build):
    from waffle_con_amd import synth
    for seed in (6, 2):
        chains = synth.cfg5_locus(seed)
        exp, ec = orc.priority_consensus(chains, counters=True, wildcard=ord("*"))
        got, gc = hip.priority_consensus(chains, counters=True, wildcard=ord("*"))
        # a locus runs dual sub-problems (and single ones where a side empties)
        used = _used()
        assert ENGINES[build][1] in used, (build, used)
        assert got == exp
        for k in KEYS:
            assert gc[k] == ec[k], (build, seed, k, gc[k], ec[k])
