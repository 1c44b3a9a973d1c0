"""Adapter: the product API (waffle_con_amd, HIP path) with the same call
shape and result dicts as tests/oracle_ffi.py, so ref_cases drive both."""
import os

import waffle_con_amd as w
from waffle_con_amd.cdwfa_config import CdwfaConfig, ConsensusCost


def make_config(**kw):
    kw = dict(kw)
    if "consensus_cost" in kw:
        kw["consensus_cost"] = ConsensusCost(kw["consensus_cost"])
    return CdwfaConfig(**kw)


def _cons(c):
    return {"sequence": c.sequence(), "scores": list(c.scores())}


def consensus(seqs, offsets=None, counters=False, **cfg):
    d = w.ConsensusDWFA.with_config(make_config(**cfg))
    for i, s in enumerate(seqs):
        d.add_sequence_offset(s, None if offsets is None else offsets[i])
    res = [_cons(c) for c in d.consensus()]
    return (res, d.last_stats) if counters else res


def consensus_batch(problems, counters=False, **cfg):
    res, stats = w.consensus_batch(problems, make_config(**cfg), return_errors=True)
    out = [r if isinstance(r, Exception) else [_cons(c) for c in r] for r in res]
    return (out, stats) if counters else out


def dual_consensus(seqs, offsets=None, counters=False, **cfg):
    d = w.DualConsensusDWFA.with_config(make_config(**cfg))
    for i, s in enumerate(seqs):
        d.add_sequence_offset(s, None if offsets is None else offsets[i])
    res = []
    for dc in d.consensus():
        res.append({"consensus1": _cons(dc.consensus1()),
                    "consensus2": None if dc.consensus2() is None else _cons(dc.consensus2()),
                    "is_consensus1": list(dc.is_consensus1()),
                    "scores1": list(dc.scores1()), "scores2": list(dc.scores2())})
    return (res, d.last_stats) if counters else res


def priority_consensus(chains, offsets=None, seed_groups=None, counters=False, **cfg):
    """PriorityConsensusDWFA.consensus() (the service path), or with
    WC_TEST_PRIORITY_PATH=batch the same problem through
    priority_consensus_batch (the streamed batch launch)."""
    d = w.PriorityConsensusDWFA.with_config(make_config(**cfg))
    for i, ch in enumerate(chains):
        offs = [None] * len(ch) if offsets is None else offsets[i]
        grp = None if seed_groups is None else seed_groups[i]
        d.add_seeded_sequence_chain(list(ch), offs, grp)
    if os.environ.get("WC_TEST_PRIORITY_PATH") == "batch":
        from waffle_con_amd.priority_consensus import priority_consensus_batch
        (r,), stats = priority_consensus_batch([(d._sequences, d._offsets, d._seed_groups)], d._config)
    else:
        r = d.consensus()
        stats = d.last_stats
    res = {"consensuses": [[_cons(c) for c in chain] for chain in r.consensuses()],
           "sequence_indices": list(r.sequence_indices())}
    return (res, stats) if counters else res
