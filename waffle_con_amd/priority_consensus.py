"""PriorityConsensus / PriorityConsensusDWFA (priority_consensus.rs:64-355).

The LIFO split/level orchestration runs in the library's host code
(wc_priority_consensus_batch); every DualConsensusDWFA sub-problem runs on the
device engine, batched across all problems of a call. One
PriorityConsensusDWFA.consensus() goes through the device's submission
service (wc_service_priority_consensus), shared by every calling thread.
"""
import ctypes

from . import _lib
from .cdwfa_config import CdwfaConfig
from .consensus import Consensus, _raise_for, _stats


class PriorityConsensus:
    """priority_consensus.rs:64-88."""

    def __init__(self, consensuses, sequence_indices):
        self._consensuses = consensuses
        self._sequence_indices = list(sequence_indices)

    def consensuses(self):
        return self._consensuses

    def sequence_indices(self):
        return self._sequence_indices

    def __eq__(self, other):
        return (isinstance(other, PriorityConsensus) and self._consensuses == other._consensuses
                and self._sequence_indices == other._sequence_indices)

    def __repr__(self):
        return "PriorityConsensus(consensuses=%r, sequence_indices=%r)" % (self._consensuses, self._sequence_indices)


def _chain_problems(problems):
    """WcChainProblem array (and the buffers it points into) for a list of
    (chains, offsets or None, seed_groups or None); chains[i][level] bytes."""
    keep = []
    arr = (_lib.WcChainProblem * max(1, len(problems)))()
    for i, (chains, offsets, groups) in enumerate(problems):
        levels = len(chains[0]) if chains else 0
        flat = [bytes(s) for ch in chains for s in ch]
        pr = _lib.PackedReads(flat)
        offs = None
        if offsets is not None and any(o is not None for ch in offsets for o in ch):
            offs = (ctypes.c_int64 * max(1, len(flat)))(*[-1 if o is None else int(o) for ch in offsets for o in ch])
        grp = None
        if groups is not None and any(g is not None for g in groups):
            grp = (ctypes.c_int64 * max(1, len(chains)))(*[-1 if g is None else int(g) for g in groups])
        keep.append((pr, offs, grp))
        arr[i].n_chains = len(chains)
        arr[i].levels = levels
        arr[i].reads = ctypes.cast(pr.ptrs, ctypes.POINTER(_lib._u8p))
        arr[i].lens = ctypes.cast(pr.lens, ctypes.POINTER(ctypes.c_uint64))
        arr[i].offsets = ctypes.cast(offs, ctypes.POINTER(ctypes.c_int64)) if offs is not None else None
        arr[i].seed_groups = ctypes.cast(grp, ctypes.POINTER(ctypes.c_int64)) if grp is not None else None
    return arr, keep


def _priority_results(res, n, config, L, return_errors):
    out = []
    for p in range(n):
        try:
            _raise_for(res, p, L)
        except _lib.WaffleConError as e:
            if not return_errors:
                raise
            out.append(e)
            continue
        chains = []
        for k in range(L.wc_results_count(res, p)):
            chain = []
            for lvl in range(L.wc_results_chain_len(res, p, k)):
                sp, sl = _lib._u8p(), ctypes.c_uint64()
                cp, cl = ctypes.POINTER(ctypes.c_uint64)(), ctypes.c_uint64()
                L.wc_results_chain(res, p, k, lvl, ctypes.byref(sp), ctypes.byref(sl), ctypes.byref(cp),
                                   ctypes.byref(cl))
                chain.append(Consensus(_lib.u8_bytes(sp, sl.value), config.consensus_cost,
                                       _lib.u64_list(cp, cl.value)))
            chains.append(chain)
        ip, il = ctypes.POINTER(ctypes.c_uint64)(), ctypes.c_uint64()
        L.wc_results_sequence_indices(res, p, ctypes.byref(ip), ctypes.byref(il))
        out.append(PriorityConsensus(chains, _lib.u64_list(ip, il.value)))
    return out


def priority_consensus_batch(problems, config=None, context=None, return_errors=False, per_problem=False):
    """problems: list of (chains, offsets or None, seed_groups or None); chains[i][level] bytes.
    per_problem: the stats also carry "per_problem" (each problem's counters, and
    wall_ms = time from the start of the call until its result was final)."""
    config = config or CdwfaConfig()
    ctx = context or _lib.default_context()
    L = _lib.lib()
    arr, keep = _chain_problems(problems)
    cfg = _lib.make_config(config)
    res = ctypes.c_void_p()
    rc = L.wc_priority_consensus_batch(ctx.handle, ctypes.byref(cfg), len(problems), arr, ctypes.byref(res))
    if rc != _lib.WC_OK:
        raise _lib.WaffleConError("wc_priority_consensus_batch failed: " + ctx.last_error(), rc)
    try:
        return _priority_results(res, len(problems), config, L, return_errors), _stats(res, L, per_problem)
    finally:
        L.wc_results_free(res)


def priority_service_call(problem, config, svc=None):
    """One PriorityConsensusDWFA::consensus through the device's submission
    service (wc_service_priority_consensus): this thread unwinds the LIFO
    stack, the sub-problems share the service's persistent launches with every
    other caller. None when the device has no service. `svc`: a given
    _lib.Service instead of the process-wide one."""
    if svc is None:
        svc = _lib.service()
    if svc is None:
        return None
    L = _lib.lib()
    arr, keep = _chain_problems([problem])
    cfg = _lib.make_config(config)
    res = ctypes.c_void_p()
    rc = L.wc_service_priority_consensus(svc.handle, ctypes.byref(cfg), arr, ctypes.byref(res))
    if rc != _lib.WC_OK:
        raise _lib.WaffleConError("wc_service_priority_consensus failed: " + svc.last_error(), rc)
    try:
        return _priority_results(res, 1, config, L, False), _stats(res, L)
    finally:
        L.wc_results_free(res)


class PriorityConsensusDWFA:
    """priority_consensus.rs:95-355 — same constructor/add/consensus surface."""

    def __init__(self, config=None):
        self._config = config or CdwfaConfig()
        self._sequences = []
        self._offsets = []
        self._seed_groups = []
        self._alphabet = set()
        self.last_stats = None

    @classmethod
    def with_config(cls, config):
        return cls(config)

    @classmethod
    def default(cls):
        return cls()

    def add_sequence_chain(self, sequences):
        """priority_consensus.rs:129-132."""
        self.add_seeded_sequence_chain(sequences, [None] * len(sequences), None)

    def add_seeded_sequence_chain(self, sequences, offsets, seed_group):
        """priority_consensus.rs:141-167 (same error messages)."""
        if len(sequences) == 0:
            raise _lib.WaffleConError("Must provide a non-empty sequences Vec", 9)
        if self._sequences and len(self._sequences[0]) != len(sequences):
            raise _lib.WaffleConError("Expected sequences Vec of length %d, but got one of length %d" % (
                len(self._sequences[0]), len(sequences)), 9)
        for s in sequences:
            self._alphabet.update(bytes(s))
        if self._config.wildcard is not None:
            self._alphabet.discard(self._config.wildcard)
        self._sequences.append([bytes(s) for s in sequences])
        self._offsets.append(list(offsets))
        self._seed_groups.append(seed_group)

    def consensus(self):
        """priority_consensus.rs:172-341."""
        prob = (self._sequences, self._offsets, self._seed_groups)
        out = priority_service_call(prob, self._config) if _lib.service_enabled() else None
        if out is None:
            out = priority_consensus_batch([prob], self._config)
        (res,), stats = out
        self.last_stats = stats
        return res

    def sequences(self):
        return [list(c) for c in self._sequences]

    def consensus_cost(self):
        return self._config.consensus_cost

    def alphabet(self):
        return set(self._alphabet)
