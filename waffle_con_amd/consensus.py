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
    """consensus.rs:42-74. Results of a batch call stay in the library's
    result arenas (wc_results_single_view); each Consensus unpacks its own
    sequence and scores from them into Python objects on first access."""
    __slots__ = ("_sequence", "_consensus_cost", "_scores", "_src")

    def __init__(self, sequence, consensus_cost, scores):
        self._sequence = bytes(sequence)
        self._consensus_cost = consensus_cost
        self._scores = list(scores)
        self._src = None

    @classmethod
    def _packed(cls, pack, j, consensus_cost):
        """Result j of a result set viewed in place: pack = (sequence arena,
        per-result [seq start, len, scores start, len] list, score arena, owner)."""
        c = cls.__new__(cls)
        c._sequence = c._scores = None
        c._consensus_cost = consensus_cost
        c._src = (pack, j)
        return c

    def _unpack(self):
        (seq, idx, sc, _owner), j = self._src
        a, la, c, lc = idx[4 * j:4 * j + 4]
        self._sequence = seq[a:a + la].tobytes()
        self._scores = sc[c:c + lc].tolist()
        self._src = None

    def __reduce__(self):
        """pickle / copy / deepcopy: the plain values only (never the result
        arenas this object may still view), as the reference's derived Clone."""
        return (Consensus, (self.sequence(), self._consensus_cost, self.scores()))

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


class _Owned:
    """Keeps a result set alive while Consensus objects still view its arenas."""
    __slots__ = ("handle",)

    def __init__(self, handle):
        self.handle = handle

    def __del__(self):
        try:
            _lib.lib().wc_results_free(self.handle)
        except Exception:  # noqa: BLE001 (interpreter shutdown)
            pass


def _single_results(res, n, cost, L, return_errors):
    """Per problem: a list of Consensus, or its WaffleConError. The results
    stay in the library's arenas (wc_results_single_view, no copy); takes
    ownership of `res` (freed when no Consensus refers to it any more).
    Retention: one surviving Consensus that was never read keeps the whole
    result set (every problem's arenas) alive; reading it (sequence(),
    scores(), pickling) unpacks it into plain values and drops the reference.
    A caller that keeps a few results of many batches should read them."""
    owner = _Owned(res)
    u64 = ctypes.c_uint64
    nr, sb, ns = u64(), u64(), u64()
    if L.wc_results_single_sizes(res, ctypes.byref(nr), ctypes.byref(sb), ctypes.byref(ns)) != _lib.WC_OK:
        raise _lib.WaffleConError("wc_results_single_sizes: not a single-consensus result set", _lib.WC_E_BAD_INPUT)
    st_p, cnt_p = ctypes.POINTER(ctypes.c_int32)(), ctypes.POINTER(ctypes.c_uint32)()
    seq_p, sc_p, idx_p = _lib._u8p(), ctypes.POINTER(u64)(), ctypes.POINTER(u64)()
    L.wc_results_single_view(res, ctypes.byref(st_p), ctypes.byref(cnt_p), ctypes.byref(seq_p), ctypes.byref(sc_p),
                             ctypes.byref(idx_p))
    as_np = np.ctypeslib.as_array
    seq = as_np(seq_p, shape=(max(sb.value, 1),))
    sc = as_np(sc_p, shape=(max(ns.value, 1),))
    idx = as_np(idx_p, shape=(max(4 * nr.value, 1),)).tolist()
    st = as_np(st_p, shape=(max(n, 1),)).tolist()
    cnt = as_np(cnt_p, shape=(max(n, 1),)).tolist()
    pack = (seq, idx, sc, owner)
    out, k = [], 0
    new = object.__new__
    ok = _lib.WC_OK
    # (Consensus._packed inlined: one object per result, its arenas viewed in place)
    for p in range(n):
        c_p = cnt[p]
        if st[p] != ok:
            e = _lib.WaffleConError(L.wc_results_error(res, p).decode(), st[p])
            if not return_errors:
                raise e
            out.append(e)
            k += c_p
            continue
        row = []
        for j in range(k, k + c_p):
            c = new(Consensus)
            c._sequence = c._scores = None
            c._consensus_cost = cost
            c._src = (pack, j)
            row.append(c)
        out.append(row)
        k += c_p
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


def _bytes_data_offset():
    probe = b"waffle_con"
    off = ctypes.cast(ctypes.c_char_p(probe), ctypes.c_void_p).value - id(probe)
    if not 0 < off < 256:
        raise RuntimeError("unexpected bytes object layout")
    return off


_BYTES_DATA = _bytes_data_offset()
# _lib.WcProblem's layout (u32 n_reads, 4 bytes padding, three pointers)
_PROBLEM_DT = np.dtype([("n_reads", "<u4"), ("_pad", "<u4"), ("reads", "<u8"), ("lens", "<u8"), ("offsets", "<u8")])
assert _PROBLEM_DT.itemsize == ctypes.sizeof(_lib.WcProblem) and _lib.WcProblem.reads.offset == 8


def _problems(batch):
    """WcProblem array for a list of (reads, offsets). Zero-copy and flat: one
    pointer array and one length array for every read of the batch (the
    bytes objects' own buffers, kept alive in `keep`); each problem points at
    its slice. The library copies the bytes once, into its pinned staging."""
    reads = [s if type(s) is bytes else bytes(s) for seqs, _ in batch for s in seqs]
    n = len(reads)
    # the data address of a bytes object is its id plus a fixed header offset
    # (_BYTES_DATA, measured at import): one vectorised pass instead of a
    # ctypes conversion per read
    ptrs = np.fromiter(map(id, reads), dtype=np.uint64, count=n) + np.uint64(_BYTES_DATA)
    lens = np.fromiter(map(len, reads), dtype=np.uint64, count=n)
    if n == 0:
        ptrs = lens = np.zeros(1, np.uint64)
    base_p, base_l = ptrs.ctypes.data, lens.ctypes.data
    # the WcProblem array as a numpy record array of the same layout
    nb = len(batch)
    counts = np.fromiter((len(seqs) for seqs, _ in batch), dtype=np.uint64, count=nb)
    starts = np.zeros(max(1, nb), np.uint64)
    if nb > 1:
        np.cumsum(counts[:-1], out=starts[1:nb])
    rec = np.zeros(max(1, nb), dtype=_PROBLEM_DT)
    rec["n_reads"][:nb] = counts
    rec["reads"][:nb] = np.uint64(base_p) + np.uint64(8) * starts[:nb]
    rec["lens"][:nb] = np.uint64(base_l) + np.uint64(8) * starts[:nb]
    keep = [reads, ptrs, lens, rec]
    for i, (_, offsets) in enumerate(batch):
        if offsets is not None:
            offs = _lib.offsets_array(offsets)
            if offs is not None:
                keep.append(offs)
                rec["offsets"][i] = ctypes.addressof(offs)
    arr = ctypes.cast(rec.ctypes.data, ctypes.POINTER(_lib.WcProblem))
    return arr, keep


def _service_call(fn, problem, config):
    """One locus through the submission service (wc_service_consensus /
    wc_service_dual_consensus): blocks this thread only (the GIL is released
    while it waits). Returns the one-problem result set and its stats, or
    None when the device has no service (the caller takes the batch path)."""
    svc = _lib.service()
    if svc is None:
        return None
    L = _lib.lib()
    arr, keep = _problems([problem])
    cfg = _lib.make_config(config)
    res = ctypes.c_void_p()
    rc = getattr(L, fn)(svc.handle, ctypes.byref(cfg), arr, ctypes.byref(res))
    if rc != _lib.WC_OK:
        raise _lib.WaffleConError("%s failed: %s" % (fn, svc.last_error()), rc)
    if fn == "wc_service_consensus":
        stats = _stats(res, L)
        return _single_results(res, 1, config.consensus_cost, L, False), stats
    from .dual_consensus import _dual_results
    try:
        return _dual_results(res, [problem], config, L, False), _stats(res, L)
    finally:
        L.wc_results_free(res)


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
    stats = _stats(res, L)
    return _single_results(res, len(batch), config.consensus_cost, L, return_errors), stats


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
        """consensus.rs:139-351 (on the GPU). Through the device's submission
        service (any number of threads share the device; WAFFLE_CON_SERVICE=0:
        one batch call per locus instead)."""
        offs = self._offsets if any(o is not None for o in self._offsets) else None
        out = _service_call("wc_service_consensus", (self._sequences, offs), self._config) \
            if _lib.service_enabled() else None
        if out is None:
            out = consensus_batch([(self._sequences, offs)], self._config)
        (res,), stats = out
        self.last_stats = stats
        return res

    def sequences(self):
        return list(self._sequences)

    def consensus_cost(self):
        return self._config.consensus_cost

    def alphabet(self):
        return set(self._alphabet)


__all__ = ["Consensus", "ConsensusDWFA", "consensus_batch", "ConsensusCost"]
