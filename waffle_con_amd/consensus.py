"""Consensus / ConsensusDWFA (consensus.rs:42-365) on the MI355X engine.

`ConsensusDWFA.consensus()` runs the reference search on the GPU through
`wc_consensus_batch`; `consensus_batch()` submits many independent problems
(loci) in one device-resident launch.
"""
import ctypes

import numpy as np

from . import _lib
from .cdwfa_config import CdwfaConfig, ConsensusCost


class Consensus:
    """consensus.rs:42-74. Results of a batch call share one packed host
    buffer (wc_results_single_pack); each Consensus unpacks its own sequence
    and scores from it into Python objects on first access."""
    __slots__ = ("_sequence", "_consensus_cost", "_scores", "_src")

    def __init__(self, sequence, consensus_cost, scores):
        self._sequence = bytes(sequence)
        self._consensus_cost = consensus_cost
        self._scores = list(scores)
        self._src = None

    @classmethod
    def _packed(cls, pack, j, consensus_cost):
        """Result j of a packed result set pack = (seq u8 array, seq offsets,
        scores u64 array, score offsets)."""
        c = cls.__new__(cls)
        c._sequence = c._scores = None
        c._consensus_cost = consensus_cost
        c._src = (pack, j)
        return c

    def _unpack(self):
        (seq, so, sc, co), j = self._src
        self._sequence = seq[so[j]:so[j + 1]].tobytes()
        self._scores = sc[co[j]:co[j + 1]].tolist()
        self._src = None

    def sequence(self):
        if self._src is not None:
            self._unpack()
        return self._sequence

    def consensus_cost(self):
        return self._consensus_cost

    def scores(self):
        if self._src is not None:
            self._unpack()
        return self._scores

    def __eq__(self, other):
        return (isinstance(other, Consensus) and self.sequence() == other.sequence()
                and self._consensus_cost == other._consensus_cost and self.scores() == other.scores())

    def __repr__(self):
        return "Consensus(sequence=%r, consensus_cost=%s, scores=%r)" % (
            self.sequence(), self._consensus_cost.name, self.scores())


def _raise_for(results, p, L):
    st = L.wc_results_status(results, p)
    if st != _lib.WC_OK:
        raise _lib.WaffleConError(L.wc_results_error(results, p).decode(), st)


def _single_results(res, n, cost, L, return_errors):
    """Per problem: a list of Consensus, or its WaffleConError. Everything
    comes out of the library in one wc_results_single_pack call."""
    u64 = ctypes.c_uint64
    nr, sb, ns = u64(), u64(), u64()
    if L.wc_results_single_sizes(res, ctypes.byref(nr), ctypes.byref(sb), ctypes.byref(ns)) != _lib.WC_OK:
        raise _lib.WaffleConError("wc_results_single_sizes: not a single-consensus result set", _lib.WC_E_BAD_INPUT)
    status = np.zeros(max(n, 1), np.int32)
    count = np.zeros(max(n, 1), np.uint32)
    seq = np.empty(max(sb.value, 1), np.uint8)
    soff = np.empty(nr.value + 1, np.uint64)
    sc = np.empty(max(ns.value, 1), np.uint64)
    coff = np.empty(nr.value + 1, np.uint64)
    L.wc_results_single_pack(res, status.ctypes.data, count.ctypes.data, seq.ctypes.data, soff.ctypes.data,
                             sc.ctypes.data, coff.ctypes.data)
    so, co, cnt, st = soff.tolist(), coff.tolist(), count.tolist(), status.tolist()
    pack = (seq, so, sc, co)
    out, k = [], 0
    mk = Consensus._packed
    for p in range(n):
        if st[p] != _lib.WC_OK:
            e = _lib.WaffleConError(L.wc_results_error(res, p).decode(), st[p])
            if not return_errors:
                raise e
            out.append(e)
            k += cnt[p]
            continue
        out.append([mk(pack, j, cost) for j in range(k, k + cnt[p])])
        k += cnt[p]
    return out


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
        out = _single_results(res, len(batch), config.consensus_cost, L, return_errors)
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
