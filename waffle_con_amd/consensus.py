"""Consensus / ConsensusDWFA (consensus.rs:42-365) on the MI355X engine.

`ConsensusDWFA.consensus()` runs the reference search on the GPU through
`wc_consensus_batch`; `consensus_batch()` submits many independent problems
(loci) in one device-resident launch.
"""
import ctypes

from . import _lib
from .cdwfa_config import CdwfaConfig, ConsensusCost


class Consensus:
    """consensus.rs:42-74."""
    __slots__ = ("_sequence", "_consensus_cost", "_scores")

    def __init__(self, sequence, consensus_cost, scores):
        self._sequence = bytes(sequence)
        self._consensus_cost = consensus_cost
        self._scores = list(scores)

    def sequence(self):
        return self._sequence

    def consensus_cost(self):
        return self._consensus_cost

    def scores(self):
        return self._scores

    def __eq__(self, other):
        return (isinstance(other, Consensus) and self._sequence == other._sequence
                and self._consensus_cost == other._consensus_cost and self._scores == other._scores)

    def __repr__(self):
        return "Consensus(sequence=%r, consensus_cost=%s, scores=%r)" % (
            self._sequence, self._consensus_cost.name, self._scores)


def _raise_for(results, p, L):
    st = L.wc_results_status(results, p)
    if st != _lib.WC_OK:
        raise _lib.WaffleConError(L.wc_results_error(results, p).decode(), st)


def _stats(results, L, per_problem=False):
    s = _lib.WcStats()
    L.wc_results_stats(results, ctypes.byref(s))
    out = s.as_dict()
    if per_problem:
        pp = []
        for p in range(L.wc_results_problems(results)):
            q = _lib.WcStats()
            L.wc_results_problem_stats(results, p, ctypes.byref(q))
            pp.append(q.as_dict())
        out["per_problem"] = pp
    return out


def _problems(batch):
    keep = []
    arr = (_lib.WcProblem * max(1, len(batch)))()
    for i, (seqs, offsets) in enumerate(batch):
        pr = _lib.PackedReads(seqs)
        offs = _lib.offsets_array(offsets)
        keep.append((pr, offs))
        arr[i].n_reads = len(seqs)
        arr[i].reads = ctypes.cast(pr.ptrs, ctypes.POINTER(_lib._u8p))
        arr[i].lens = ctypes.cast(pr.lens, ctypes.POINTER(ctypes.c_uint64))
        arr[i].offsets = ctypes.cast(offs, ctypes.POINTER(ctypes.c_int64)) if offs is not None else None
    return arr, keep


def consensus_batch(problems, config=None, context=None, return_errors=False):
    """Run ConsensusDWFA::consensus for many independent problems at once.

    problems: list of read lists, or (reads, offsets) tuples.
    Returns (list of per-problem results, run stats). Each result is a list of
    Consensus, or the WaffleConError for that problem when return_errors.
    """
    config = config or CdwfaConfig()
    ctx = context or _lib.default_context()
    L = _lib.lib()
    batch = [(p, None) if not isinstance(p, tuple) else p for p in problems]
    arr, keep = _problems(batch)
    cfg = _lib.make_config(config)
    res = ctypes.c_void_p()
    rc = L.wc_consensus_batch(ctx.handle, ctypes.byref(cfg), len(batch), arr, ctypes.byref(res))
    if rc != _lib.WC_OK:
        raise _lib.WaffleConError("wc_consensus_batch failed: " + ctx.last_error(), rc)
    try:
        out = []
        for p in range(len(batch)):
            try:
                _raise_for(res, p, L)
            except _lib.WaffleConError as e:
                if not return_errors:
                    raise
                out.append(e)
                continue
            items = []
            for k in range(L.wc_results_count(res, p)):
                sp, sl = _lib._u8p(), ctypes.c_uint64()
                cp, cl = ctypes.POINTER(ctypes.c_uint64)(), ctypes.c_uint64()
                L.wc_results_single(res, p, k, ctypes.byref(sp), ctypes.byref(sl), ctypes.byref(cp), ctypes.byref(cl))
                items.append(Consensus(_lib.u8_bytes(sp, sl.value), config.consensus_cost,
                                       _lib.u64_list(cp, cl.value)))
            out.append(items)
        return out, _stats(res, L)
    finally:
        L.wc_results_free(res)


class ConsensusDWFA:
    """consensus.rs:78-365 — same constructor/add/consensus surface."""

    def __init__(self, config=None):
        self._config = config or CdwfaConfig()
        self._sequences = []
        self._offsets = []
        self._alphabet = set()
        self.last_stats = None

    @classmethod
    def with_config(cls, config):
        return cls(config)

    @classmethod
    def default(cls):
        return cls()

    def add_sequence(self, sequence):
        self.add_sequence_offset(sequence, None)

    def add_sequence_offset(self, sequence, last_offset):
        """consensus.rs:120-134."""
        sequence = bytes(sequence)
        self._alphabet.update(sequence)
        if self._config.wildcard is not None:
            self._alphabet.discard(self._config.wildcard)
        self._sequences.append(sequence)
        self._offsets.append(last_offset)

    def consensus(self):
        """consensus.rs:139-351 (on the GPU)."""
        offs = self._offsets if any(o is not None for o in self._offsets) else None
        (res,), stats = consensus_batch([(self._sequences, offs)], self._config)
        self.last_stats = stats
        return res

    def sequences(self):
        return list(self._sequences)

    def consensus_cost(self):
        return self._config.consensus_cost

    def alphabet(self):
        return set(self._alphabet)


__all__ = ["Consensus", "ConsensusDWFA", "consensus_batch", "ConsensusCost"]
