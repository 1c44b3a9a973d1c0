"""DualConsensus / DualConsensusDWFA (dual_consensus.rs:52-801) on the MI355X
engine (`wc_dual_consensus_batch`)."""
import ctypes

from . import _lib
from .cdwfa_config import CdwfaConfig
from .consensus import Consensus, _problems, _raise_for, _stats


class DualConsensus:
    """dual_consensus.rs:52-177. Equality ignores scores1/scores2 (:66-75)."""

    def __init__(self, consensus1, consensus2, is_consensus1, scores1, scores2):
        if not (len(is_consensus1) == len(scores1) == len(scores2)):
            raise _lib.WaffleConError("is_consensus1, scores1, and scores2 must all be the same length")
        self._c1 = consensus1
        self._c2 = consensus2
        self._is_c1 = list(is_consensus1)
        self._s1 = list(scores1)
        self._s2 = list(scores2)

    @classmethod
    def new(cls, consensus1, consensus2, is_consensus1, scores1, scores2):
        return cls(consensus1, consensus2, is_consensus1, scores1, scores2)

    def is_dual(self):
        return self._c2 is not None

    def consensus1(self):
        return self._c1

    def consensus2(self):
        return self._c2

    def is_consensus1(self):
        return self._is_c1

    def scores1(self):
        return self._s1

    def scores2(self):
        return self._s2

    def __eq__(self, other):
        return (isinstance(other, DualConsensus) and self._c1 == other._c1 and self._c2 == other._c2
                and self._is_c1 == other._is_c1)

    def __repr__(self):
        return "DualConsensus(consensus1=%r, consensus2=%r, is_consensus1=%r)" % (self._c1, self._c2, self._is_c1)


def _dual_results(res, batch, config, L, return_errors):
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
            v = _lib.WcDualView()
            L.wc_results_dual(res, p, k, ctypes.byref(v))
            c1 = Consensus(_lib.u8_bytes(v.seq1, v.len1), config.consensus_cost,
                           _lib.u64_list(v.scores_c1, v.n_scores_c1))
            c2 = None
            if v.has_c2:
                c2 = Consensus(_lib.u8_bytes(v.seq2, v.len2), config.consensus_cost,
                               _lib.u64_list(v.scores_c2, v.n_scores_c2))
            n = v.n_reads
            is_c1 = [bool(v.is_consensus1[i]) for i in range(n)]
            s1 = [None if v.scores1[i] < 0 else v.scores1[i] for i in range(n)]
            s2 = [None if v.scores2[i] < 0 else v.scores2[i] for i in range(n)]
            items.append(DualConsensus(c1, c2, is_c1, s1, s2))
        out.append(items)
    return out


def dual_consensus_batch(problems, config=None, context=None, return_errors=False):
    """Run DualConsensusDWFA::consensus for many independent problems at once."""
    config = config or CdwfaConfig()
    ctx = context or _lib.default_context()
    L = _lib.lib()
    batch = [(p, None) if not isinstance(p, tuple) else p for p in problems]
    arr, keep = _problems(batch)
    cfg = _lib.make_config(config)
    res = ctypes.c_void_p()
    rc = L.wc_dual_consensus_batch(ctx.handle, ctypes.byref(cfg), len(batch), arr, ctypes.byref(res))
    if rc != _lib.WC_OK:
        raise _lib.WaffleConError("wc_dual_consensus_batch failed: " + ctx.last_error(), rc)
    try:
        return _dual_results(res, batch, config, L, return_errors), _stats(res, L)
    finally:
        L.wc_results_free(res)


class DualConsensusDWFA:
    """dual_consensus.rs:181-801 — same constructor/add/consensus surface."""

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
        """dual_consensus.rs:221-235."""
        sequence = bytes(sequence)
        self._alphabet.update(sequence)
        if self._config.wildcard is not None:
            self._alphabet.discard(self._config.wildcard)
        self._sequences.append(sequence)
        self._offsets.append(last_offset)

    def consensus(self):
        """dual_consensus.rs:240-787 (on the GPU)."""
        offs = self._offsets if any(o is not None for o in self._offsets) else None
        out = None
        if _lib.service_enabled():
            from .consensus import _service_call
            out = _service_call("wc_service_dual_consensus", (self._sequences, offs), self._config)
        if out is None:
            out = dual_consensus_batch([(self._sequences, offs)], self._config)
        (res,), stats = out
        self.last_stats = stats
        return res

    def sequences(self):
        return list(self._sequences)

    def consensus_cost(self):
        return self._config.consensus_cost

    def alphabet(self):
        return set(self._alphabet)
