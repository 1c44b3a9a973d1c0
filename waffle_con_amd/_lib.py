"""ctypes binding of the in-tree HIP library (waffle_con_amd/libwaffle_con.so).

The library is the product: there is no CPU fallback. Loading fails loudly
when the shared object is missing, and creating a context fails loudly when
no HIP device is visible.
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# WAFFLE_CON_LIB may name another in-tree build variant (A/B benchmarking)
LIB_PATH = os.environ.get("WAFFLE_CON_LIB") or os.path.join(_HERE, "libwaffle_con.so")

_lib = None
_lock = threading.Lock()
_ctx_local = threading.local()

# error codes (include/waffle_con.h)
WC_OK = 0
WC_E_FINALIZE_UNINIT = 1
WC_E_NO_START = 2
WC_E_COVERAGE_GAP = 3
WC_E_CAPACITY = 4
WC_E_BAD_INPUT = 9
WC_E_INVARIANT = 10
WC_E_LIMIT = 11
WC_E_HIP = 12


class WaffleConError(Exception):
    """Error raised for a failed consensus; str() is the reference's message."""

    def __init__(self, message, code=0):
        super().__init__(message)
        self.code = code


class WcConfig(ctypes.Structure):
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


_u8p = ctypes.POINTER(ctypes.c_uint8)


class WcProblem(ctypes.Structure):
    _fields_ = [("n_reads", ctypes.c_uint32),
                ("reads", ctypes.POINTER(_u8p)),
                ("lens", ctypes.POINTER(ctypes.c_uint64)),
                ("offsets", ctypes.POINTER(ctypes.c_int64))]


class WcChainProblem(ctypes.Structure):
    _fields_ = [("n_chains", ctypes.c_uint32),
                ("levels", ctypes.c_uint32),
                ("reads", ctypes.POINTER(_u8p)),
                ("lens", ctypes.POINTER(ctypes.c_uint64)),
                ("offsets", ctypes.POINTER(ctypes.c_int64)),
                ("seed_groups", ctypes.POINTER(ctypes.c_int64))]


class WcDualView(ctypes.Structure):
    _fields_ = [("seq1", _u8p), ("len1", ctypes.c_uint64),
                ("scores_c1", ctypes.POINTER(ctypes.c_uint64)), ("n_scores_c1", ctypes.c_uint64),
                ("has_c2", ctypes.c_uint8),
                ("seq2", _u8p), ("len2", ctypes.c_uint64),
                ("scores_c2", ctypes.POINTER(ctypes.c_uint64)), ("n_scores_c2", ctypes.c_uint64),
                ("is_consensus1", _u8p),
                ("scores1", ctypes.POINTER(ctypes.c_int64)),
                ("scores2", ctypes.POINTER(ctypes.c_int64)),
                ("n_reads", ctypes.c_uint64)]


class WcStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in (
        "updates", "w_out", "compares", "ed_increases", "finalizes", "pops", "nodes_explored",
        "nodes_ignored", "peak_queue_size", "row_bytes", "launches")] + [("kernel_ms", ctypes.c_double),
                                                            ("wall_ms", ctypes.c_double),
                                                            ("start_ms", ctypes.c_double)]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class WcServiceStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in ("calls", "served", "fallback", "lane_starts", "retried",
                                               "lane_failures")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class WcDwfaJob(ctypes.Structure):
    _fields_ = [("baseline", _u8p), ("baseline_len", ctypes.c_uint64),
                ("other", _u8p), ("other_len", ctypes.c_uint64),
                ("offset", ctypes.c_uint64), ("wildcard", ctypes.c_int32),
                ("early", ctypes.c_uint8), ("op", ctypes.c_uint8), ("_pad", ctypes.c_uint8 * 2),
                ("e", ctypes.c_uint64), ("wavefront", ctypes.POINTER(ctypes.c_uint64)),
                ("wf_len", ctypes.c_uint64), ("wf_cap", ctypes.c_uint64),
                ("cand_syms", ctypes.c_uint8 * 16), ("cand_counts", ctypes.c_uint64 * 16),
                ("n_cand", ctypes.c_uint32), ("status", ctypes.c_int32), ("cand_first", ctypes.c_uint8 * 16)]


# every symbol include/waffle_con.h declares (checked by tests/test_cabi.py)
EXPORTED = (
    "wc_config_default", "wc_ctx_create", "wc_ctx_destroy", "wc_last_error",
    "wc_consensus_batch", "wc_dual_consensus_batch", "wc_priority_consensus_batch",
    "wc_batch_create", "wc_batch_refill", "wc_batch_free", "wc_batch_bytes", "wc_batch_consensus", "wc_batch_dual_consensus",
    "wc_results_free", "wc_results_problems", "wc_results_status", "wc_results_error",
    "wc_results_count", "wc_results_single", "wc_results_single_sizes", "wc_results_single_pack", "wc_results_single_view", "wc_results_dual", "wc_results_chain_len",
    "wc_results_chain", "wc_results_sequence_indices", "wc_results_stats",
    "wc_results_problem_stats", "wc_dwfa_batch", "wc_generate_test", "wc_gen_consensus",
    "wc_gen_sample", "wc_gen_free", "wc_wfa_ed_config", "wc_wfa_ed_batch",
    "wc_service_create", "wc_service_destroy", "wc_service_consensus", "wc_service_dual_consensus",
    "wc_service_priority_consensus", "wc_service_get_stats", "wc_service_last_error",
    "wc_engines_used", "wc_engine_name", "wc_last_upload_packed", "wc_service_engines_used",
)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise WaffleConError(
                "HIP library %s is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(hipcc --offload-arch=gfx950)" % LIB_PATH, WC_E_HIP)
        L = ctypes.CDLL(LIB_PATH)
        vp = ctypes.c_void_p
        L.wc_config_default.argtypes = [ctypes.POINTER(WcConfig)]
        L.wc_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
        L.wc_ctx_destroy.argtypes = [vp]
        L.wc_last_error.argtypes = [vp]
        L.wc_last_error.restype = ctypes.c_char_p
        for f, pt in (("wc_consensus_batch", WcProblem), ("wc_dual_consensus_batch", WcProblem),
                      ("wc_priority_consensus_batch", WcChainProblem)):
            fn = getattr(L, f)
            fn.argtypes = [vp, ctypes.POINTER(WcConfig), ctypes.c_uint32, ctypes.POINTER(pt), ctypes.POINTER(vp)]
        L.wc_batch_create.argtypes = [vp, ctypes.c_uint32, ctypes.POINTER(WcProblem), ctypes.POINTER(vp)]
        L.wc_batch_refill.argtypes = [vp, vp, ctypes.c_uint32, ctypes.POINTER(WcProblem)]
        L.wc_batch_free.argtypes = [vp]
        L.wc_batch_bytes.argtypes = [vp]
        L.wc_batch_bytes.restype = ctypes.c_uint64
        for f in ("wc_batch_consensus", "wc_batch_dual_consensus"):
            getattr(L, f).argtypes = [vp, vp, ctypes.POINTER(WcConfig), ctypes.POINTER(vp)]
        L.wc_results_free.argtypes = [vp]
        L.wc_results_problems.argtypes = [vp]
        L.wc_results_problems.restype = ctypes.c_uint32
        L.wc_results_status.argtypes = [vp, ctypes.c_uint32]
        L.wc_results_error.argtypes = [vp, ctypes.c_uint32]
        L.wc_results_error.restype = ctypes.c_char_p
        L.wc_results_count.argtypes = [vp, ctypes.c_uint32]
        L.wc_results_count.restype = ctypes.c_uint32
        L.wc_results_single.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(_u8p),
                                        ctypes.POINTER(ctypes.c_uint64),
                                        ctypes.POINTER(ctypes.POINTER(ctypes.c_uint64)),
                                        ctypes.POINTER(ctypes.c_uint64)]
        u64p = ctypes.POINTER(ctypes.c_uint64)
        L.wc_results_single_sizes.argtypes = [vp, u64p, u64p, u64p]
        L.wc_results_single_pack.argtypes = [vp, vp, vp, vp, vp, vp, vp]
        L.wc_results_single_view.argtypes = [vp, ctypes.POINTER(ctypes.POINTER(ctypes.c_int32)),
                                             ctypes.POINTER(ctypes.POINTER(ctypes.c_uint32)), ctypes.POINTER(_u8p),
                                             ctypes.POINTER(u64p), ctypes.POINTER(u64p)]
        L.wc_results_dual.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(WcDualView)]
        L.wc_results_chain_len.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32]
        L.wc_results_chain_len.restype = ctypes.c_uint32
        L.wc_results_chain.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.POINTER(_u8p), ctypes.POINTER(ctypes.c_uint64),
                                       ctypes.POINTER(ctypes.POINTER(ctypes.c_uint64)),
                                       ctypes.POINTER(ctypes.c_uint64)]
        L.wc_results_sequence_indices.argtypes = [vp, ctypes.c_uint32,
                                                  ctypes.POINTER(ctypes.POINTER(ctypes.c_uint64)),
                                                  ctypes.POINTER(ctypes.c_uint64)]
        L.wc_results_stats.argtypes = [vp, ctypes.POINTER(WcStats)]
        L.wc_results_problem_stats.argtypes = [vp, ctypes.c_uint32, ctypes.POINTER(WcStats)]
        L.wc_dwfa_batch.argtypes = [vp, ctypes.c_uint32, ctypes.POINTER(WcDwfaJob)]
        L.wc_generate_test.argtypes = [ctypes.c_uint8, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_double,
                                       ctypes.c_uint64, ctypes.POINTER(vp)]
        L.wc_gen_consensus.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64)]
        L.wc_gen_consensus.restype = ctypes.c_void_p
        L.wc_gen_sample.argtypes = [vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
        L.wc_gen_sample.restype = ctypes.c_void_p
        L.wc_gen_free.argtypes = [vp]
        L.wc_wfa_ed_config.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_uint64,
                                       ctypes.c_uint8, ctypes.c_int32]
        L.wc_wfa_ed_config.restype = ctypes.c_uint64
        L.wc_wfa_ed_batch.argtypes = [vp, ctypes.c_uint32, ctypes.POINTER(_u8p), ctypes.POINTER(ctypes.c_uint64),
                                      ctypes.POINTER(_u8p), ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint8,
                                      ctypes.c_int32, ctypes.POINTER(ctypes.c_uint64)]
        L.wc_service_create.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.POINTER(vp)]
        L.wc_service_destroy.argtypes = [vp]
        for f in ("wc_service_consensus", "wc_service_dual_consensus"):
            getattr(L, f).argtypes = [vp, ctypes.POINTER(WcConfig), ctypes.POINTER(WcProblem), ctypes.POINTER(vp)]
        L.wc_service_priority_consensus.argtypes = [vp, ctypes.POINTER(WcConfig), ctypes.POINTER(WcChainProblem),
                                                    ctypes.POINTER(vp)]
        L.wc_service_get_stats.argtypes = [vp, ctypes.POINTER(WcServiceStats)]
        L.wc_service_last_error.argtypes = [vp]
        L.wc_service_last_error.restype = ctypes.c_char_p
        L.wc_engines_used.argtypes = [vp, ctypes.c_int]
        L.wc_engines_used.restype = ctypes.c_uint32
        L.wc_service_engines_used.argtypes = [vp, ctypes.c_int]
        L.wc_service_engines_used.restype = ctypes.c_uint32
        L.wc_engine_name.argtypes = [ctypes.c_uint32]
        L.wc_engine_name.restype = ctypes.c_char_p
        L.wc_last_upload_packed.argtypes = [vp]
        L.wc_last_upload_packed.restype = ctypes.c_uint64
        _lib = L
        return L


class Context:
    """One HIP device context (stream, events, cached HBM arenas)."""

    def __init__(self, device=0):
        L = lib()
        h = ctypes.c_void_p()
        rc = L.wc_ctx_create(int(device), ctypes.byref(h))
        if rc != WC_OK:
            raise WaffleConError("no usable HIP device %d for waffle_con (wc_ctx_create rc=%d)" % (device, rc), rc)
        self.handle = h
        self.device = device

    def last_error(self):
        return lib().wc_last_error(self.handle).decode()

    def engines_used(self, reset=False):
        """Names of the engine builds this context has launched (wc_engines_used)."""
        return engine_names(lib().wc_engines_used(self.handle, int(bool(reset))))

    def last_upload_packed(self):
        """Bytes the last batch upload sent 2-bit packed (0 = byte path)."""
        return int(lib().wc_last_upload_packed(self.handle))

    def close(self):
        if self.handle:
            lib().wc_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


def engine_names(mask):
    """The engine build names (wc_engine_name) of the bits of `mask`."""
    out, k = [], 0
    while True:
        name = lib().wc_engine_name(k)
        if name is None:
            return out
        if mask >> k & 1:
            out.append(name.decode())
        k += 1


def default_context():
    """Per-thread default context: device WAFFLE_CON_DEVICE if set, else
    LOCAL_RANK (one process per GPU under torch.distributed.run), else 0."""
    ctx = getattr(_ctx_local, "ctx", None)
    if ctx is None:
        dev = int(os.environ.get("WAFFLE_CON_DEVICE", os.environ.get("LOCAL_RANK", "0")))
        ctx = Context(dev)
        _ctx_local.ctx = ctx
    return ctx


class Service:
    """The device's submission service (wc_service_*, csrc/service.cpp): the
    per-locus ConsensusDWFA / DualConsensusDWFA.consensus() calls of every
    thread of this process share persistent engine launches on the device."""

    def __init__(self, device=0, arena_bytes=0):
        L = lib()
        h = ctypes.c_void_p()
        rc = L.wc_service_create(int(device), int(arena_bytes), ctypes.byref(h))
        if rc != WC_OK:
            raise WaffleConError("no usable HIP device %d for the waffle_con service (rc=%d)" % (device, rc), rc)
        self.handle = h
        self.device = device

    def stats(self):
        s = WcServiceStats()
        lib().wc_service_get_stats(self.handle, ctypes.byref(s))
        return s.as_dict()

    def last_error(self):
        return lib().wc_service_last_error(self.handle).decode()

    def engines_used(self, reset=False):
        return engine_names(lib().wc_service_engines_used(self.handle, int(bool(reset))))

    def close(self):
        if self.handle:
            lib().wc_service_destroy(self.handle)
            self.handle = None


_services = {}


def service_enabled():
    return os.environ.get("WAFFLE_CON_SERVICE", "1") != "0"


_service_failed = {}  # device -> (time of the last failed creation, message)
_SERVICE_RETRY_S = 30.0


def service(device=None):
    """The process-wide service of `device` (default: the default context's
    device), created on first use and closed at exit. None when it cannot be
    created (e.g. its pinned arena): the callers then take the per-call batch
    path, as with WAFFLE_CON_SERVICE=0."""
    if device is None:
        device = default_context().device
    svc = _services.get(device)
    if svc is None and _service_may_try(device):
        with _lock:
            svc = _services.get(device)
            if svc is None and _service_may_try(device):
                try:
                    svc = Service(device)
                except WaffleConError as e:
                    # a transient failure (the pinned arena under memory
                    # pressure) must not turn the service off for good: say
                    # so once per failure, retry after a back-off
                    import sys
                    import time
                    _service_failed[device] = (time.monotonic(), str(e))
                    print("[waffle_con] submission service unavailable on device %d (%s); per-call launches "
                          "for %.0f s" % (device, e, _SERVICE_RETRY_S), file=sys.stderr)
                    return None
                _service_failed.pop(device, None)
                _services[device] = svc
                if len(_services) == 1:
                    import atexit
                    atexit.register(close_services)
    return svc


def _service_may_try(device):
    f = _service_failed.get(device)
    if f is None:
        return True
    import time
    return time.monotonic() - f[0] >= _SERVICE_RETRY_S


def service_failure(device=0):
    """The last failed service creation on `device` as (monotonic time,
    message), or None."""
    return _service_failed.get(device)


def close_services():
    for svc in list(_services.values()):
        svc.close()
    _services.clear()


def make_config(config):
    c = WcConfig()
    lib().wc_config_default(ctypes.byref(c))
    c.consensus_cost = int(config.consensus_cost.value)
    c.wildcard = -1 if config.wildcard is None else int(config.wildcard)
    c.max_queue_size = int(config.max_queue_size)
    c.max_capacity_per_size = int(config.max_capacity_per_size)
    c.max_return_size = int(config.max_return_size)
    c.max_nodes_wo_constraint = int(config.max_nodes_wo_constraint)
    c.min_count = int(config.min_count)
    c.min_af = float(config.min_af)
    c.dual_max_ed_delta = int(config.dual_max_ed_delta)
    c.offset_window = int(config.offset_window)
    c.offset_compare_length = int(config.offset_compare_length)
    c.weighted_by_ed = int(bool(config.weighted_by_ed))
    c.allow_early_termination = int(bool(config.allow_early_termination))
    c.auto_shift_offsets = int(bool(config.auto_shift_offsets))
    return c


class PackedReads:
    """Read pointer/length arrays for one call. Zero-copy: the pointers address
    the bytes objects' own buffers (kept alive here); the library copies the
    bytes once, into its pinned upload staging."""

    def __init__(self, seqs):
        self.bufs = [s if type(s) is bytes else bytes(s) for s in seqs]
        n = max(1, len(seqs))
        self.ptrs = (ctypes.c_char_p * n)(*self.bufs)
        self.lens = (ctypes.c_uint64 * n)(*map(len, self.bufs))


def offsets_array(offsets):
    if offsets is None or all(o is None for o in offsets):
        return None
    return (ctypes.c_int64 * max(1, len(offsets)))(*[-1 if o is None else int(o) for o in offsets])


def u8_bytes(ptr, n):
    return ctypes.string_at(ptr, n) if n else b""


def u64_list(ptr, n):
    return ptr[:n] if n else []
