"""ctypes bindings to the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: the oracle is the checker, never the thing measured
or shipped. Results are decoded from the oracle's JSON into plain Python
objects shaped like the reference's result types.
"""
import ctypes
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
_LIB = None


class OrcConfig(ctypes.Structure):
    _fields_ = [
        ("consensus_cost", ctypes.c_int32),
        ("wildcard", ctypes.c_int32),
        ("max_queue_size", ctypes.c_uint64),
        ("max_capacity_per_size", ctypes.c_uint64),
        ("max_return_size", ctypes.c_uint64),
        ("max_nodes_wo_constraint", ctypes.c_uint64),
        ("min_count", ctypes.c_uint64),
        ("min_af", ctypes.c_double),
        ("dual_max_ed_delta", ctypes.c_uint64),
        ("offset_window", ctypes.c_uint64),
        ("offset_compare_length", ctypes.c_uint64),
        ("weighted_by_ed", ctypes.c_uint8),
        ("allow_early_termination", ctypes.c_uint8),
        ("auto_shift_offsets", ctypes.c_uint8),
        ("_pad", ctypes.c_uint8 * 5),
    ]


class OrcCounters(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in (
        "updates", "w_out", "compares", "ed_increases", "finalizes",
        "nodes_explored", "nodes_ignored", "peak_queue_size", "pops", "row_bytes")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


# cdwfa_config.rs:71-103
DEFAULTS = dict(consensus_cost=0, max_queue_size=20, max_capacity_per_size=20,
                max_return_size=10, max_nodes_wo_constraint=1000, min_count=3,
                min_af=0.0, weighted_by_ed=False, wildcard=None, dual_max_ed_delta=20,
                allow_early_termination=False, auto_shift_offsets=True,
                offset_window=50, offset_compare_length=50)


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(ORACLE_DIR, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        cp = ctypes.POINTER(ctypes.c_uint8)
        for name in ("orc_consensus", "orc_dual_consensus"):
            f = getattr(L, name)
            f.restype = ctypes.c_void_p
            f.argtypes = [ctypes.POINTER(OrcConfig), ctypes.c_uint32, ctypes.POINTER(cp),
                          ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int64),
                          ctypes.POINTER(OrcCounters)]
        L.orc_priority_consensus.restype = ctypes.c_void_p
        L.orc_priority_consensus.argtypes = [ctypes.POINTER(OrcConfig), ctypes.c_uint32, ctypes.c_uint32,
                                             ctypes.POINTER(cp), ctypes.POINTER(ctypes.c_uint64),
                                             ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                             ctypes.POINTER(OrcCounters)]
        L.orc_free.argtypes = [ctypes.c_void_p]
        L.orc_dwfa_run.restype = ctypes.c_int
        L.orc_dwfa_run.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p,
                                   ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32, ctypes.c_int32,
                                   ctypes.c_uint8, ctypes.c_uint64, ctypes.c_uint8,
                                   ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                   ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint64,
                                   ctypes.POINTER(ctypes.c_uint64)]
        L.orc_dwfa_candidates.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_uint64,
                                          ctypes.c_int32, ctypes.POINTER(ctypes.c_uint8),
                                          ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32,
                                          ctypes.POINTER(ctypes.c_uint32)]
        L.orc_dwfa_candidate_first.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_uint64,
                                               ctypes.c_int32, ctypes.POINTER(ctypes.c_uint8), ctypes.c_uint32,
                                               ctypes.POINTER(ctypes.c_uint32)]
        L.orc_dwfa_step.restype = ctypes.c_int
        L.orc_dwfa_step.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_uint64,
                                    ctypes.c_int32, ctypes.c_uint8, ctypes.c_uint64, ctypes.c_int,
                                    ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                    ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint64]
        L.orc_wfa_ed_config.restype = ctypes.c_uint64
        L.orc_wfa_ed_config.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_uint64,
                                        ctypes.c_uint8, ctypes.c_int32]
        L.orc_seed_group_order.restype = ctypes.c_uint32
        L.orc_seed_group_order.argtypes = [ctypes.POINTER(ctypes.c_int64), ctypes.c_uint32,
                                           ctypes.POINTER(ctypes.c_int64)]
        L.orc_fxmap_order.restype = ctypes.c_uint32
        L.orc_fxmap_order.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p]
        _LIB = L
    return _LIB


def make_config(**kw):
    d = dict(DEFAULTS)
    for k, v in kw.items():
        if k not in d:
            raise KeyError(k)
        d[k] = v
    c = OrcConfig()
    for k, v in d.items():
        if k == "wildcard":
            c.wildcard = -1 if v is None else int(v)
        elif k == "consensus_cost":
            c.consensus_cost = int(v)
        else:
            setattr(c, k, v)
    return c


def _seq_arrays(seqs):
    bufs = [ctypes.create_string_buffer(bytes(s), max(1, len(s))) for s in seqs]
    cp = ctypes.POINTER(ctypes.c_uint8)
    ptrs = (cp * max(1, len(seqs)))(*[ctypes.cast(b, cp) for b in bufs])
    lens = (ctypes.c_uint64 * max(1, len(seqs)))(*[len(s) for s in seqs])
    return bufs, ptrs, lens


def _offsets(offsets, n):
    if offsets is None:
        return None
    return (ctypes.c_int64 * max(1, n))(*[-1 if o is None else int(o) for o in offsets])


def _decode(ptr):
    L = lib()
    s = ctypes.string_at(ptr).decode()
    L.orc_free(ptr)
    return json.loads(s)


def _cons(d):
    return {"sequence": bytes.fromhex(d["sequence"]), "scores": d["scores"]}


class OracleError(Exception):
    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code


def consensus(seqs, offsets=None, counters=False, **cfg):
    L = lib()
    bufs, ptrs, lens = _seq_arrays(seqs)
    c = OrcCounters()
    out = _decode(L.orc_consensus(ctypes.byref(make_config(**cfg)), len(seqs), ptrs, lens,
                                  _offsets(offsets, len(seqs)), ctypes.byref(c)))
    if not out["ok"]:
        raise OracleError(out["code"], out["error"])
    res = [_cons(r) for r in out["results"]]
    return (res, c.as_dict()) if counters else res


def dual_consensus(seqs, offsets=None, counters=False, **cfg):
    L = lib()
    bufs, ptrs, lens = _seq_arrays(seqs)
    c = OrcCounters()
    out = _decode(L.orc_dual_consensus(ctypes.byref(make_config(**cfg)), len(seqs), ptrs, lens,
                                       _offsets(offsets, len(seqs)), ctypes.byref(c)))
    if not out["ok"]:
        raise OracleError(out["code"], out["error"])
    res = []
    for r in out["results"]:
        res.append({
            "consensus1": _cons(r["consensus1"]),
            "consensus2": None if r["consensus2"] is None else _cons(r["consensus2"]),
            "is_consensus1": [bool(x) for x in r["is_consensus1"]],
            "scores1": [None if x < 0 else x for x in r["scores1"]],
            "scores2": [None if x < 0 else x for x in r["scores2"]],
        })
    return (res, c.as_dict()) if counters else res


def priority_consensus(chains, offsets=None, seed_groups=None, counters=False, **cfg):
    L = lib()
    levels = len(chains[0]) if chains else 0
    flat = [s for ch in chains for s in ch]
    bufs, ptrs, lens = _seq_arrays(flat)
    offs = None
    if offsets is not None:
        offs = (ctypes.c_int64 * max(1, len(flat)))(*[-1 if o is None else o for ch in offsets for o in ch])
    groups = None
    if seed_groups is not None:
        groups = (ctypes.c_int64 * max(1, len(chains)))(*[-1 if g is None else g for g in seed_groups])
    c = OrcCounters()
    out = _decode(L.orc_priority_consensus(ctypes.byref(make_config(**cfg)), len(chains), levels, ptrs, lens,
                                           offs, groups, ctypes.byref(c)))
    if not out["ok"]:
        raise OracleError(out["code"], out["error"])
    res = {"consensuses": [[_cons(x) for x in ch] for ch in out["consensuses"]],
           "sequence_indices": out["sequence_indices"]}
    return (res, c.as_dict()) if counters else res


def dwfa_run(baseline, other, update_lens, wildcard=None, early=False, offset=0, finalize=False, wf_cap=4096):
    L = lib()
    n = len(update_lens)
    ul = (ctypes.c_uint64 * max(1, n))(*update_lens)
    eds = (ctypes.c_uint64 * max(1, n))()
    fe = ctypes.c_uint64()
    wf = (ctypes.c_uint64 * wf_cap)()
    wl = ctypes.c_uint64()
    rc = L.orc_dwfa_run(bytes(baseline), len(baseline), bytes(other), ul, n,
                        -1 if wildcard is None else wildcard, int(early), offset, int(finalize),
                        eds, ctypes.byref(fe), wf, wf_cap, ctypes.byref(wl))
    if rc != 0:
        raise OracleError(rc, "dwfa error")
    return {"eds": list(eds[:n]), "e": fe.value, "wavefront": list(wf[:min(wl.value, wf_cap)])}


def dwfa_candidates(baseline, other, wildcard=None):
    L = lib()
    syms = (ctypes.c_uint8 * 256)()
    cnts = (ctypes.c_uint64 * 256)()
    n = ctypes.c_uint32()
    L.orc_dwfa_candidates(bytes(baseline), len(baseline), bytes(other), len(other),
                          -1 if wildcard is None else wildcard, syms, cnts, 256, ctypes.byref(n))
    return [(syms[i], cnts[i]) for i in range(n.value)]


def dwfa_candidate_first(baseline, other, wildcard=None):
    """The keys of dwfa_candidates in insertion (first-appearance) order."""
    L = lib()
    syms = (ctypes.c_uint8 * 256)()
    n = ctypes.c_uint32()
    L.orc_dwfa_candidate_first(bytes(baseline), len(baseline), bytes(other), len(other),
                               -1 if wildcard is None else wildcard, syms, 256, ctypes.byref(n))
    return list(syms[:n.value])


def wfa_ed_config(v1, v2, require_both_end, wildcard):
    return lib().orc_wfa_ed_config(bytes(v1), len(v1), bytes(v2), len(v2), int(require_both_end),
                                   -1 if wildcard is None else wildcard)


def wfa_ed(v1, v2):
    """sequence_alignment.rs:18 — full ED with '*' wildcard."""
    return wfa_ed_config(v1, v2, True, ord("*"))


def fxmap_order(keys):
    out = ctypes.create_string_buffer(256)
    n = lib().orc_fxmap_order(bytes(keys), len(keys), out)
    return list(out.raw[:n])


def seed_group_order(groups):
    """Processing order of the seed groups (priority_consensus.rs:180); None = no seed."""
    n = len(groups)
    g = (ctypes.c_int64 * max(1, n))(*[-1 if x is None else x for x in groups])
    out = (ctypes.c_int64 * max(1, n))()
    k = lib().orc_seed_group_order(g, n, out)
    return [None if out[i] < 0 else out[i] for i in range(k)]
