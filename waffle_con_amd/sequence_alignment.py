"""wfa_ed / wfa_ed_config (sequence_alignment.rs:18-87) via the library."""
from . import _lib


def wfa_ed_config(v1, v2, require_both_end, wildcard):
    v1, v2 = bytes(v1), bytes(v2)
    return _lib.lib().wc_wfa_ed_config(v1, len(v1), v2, len(v2), int(bool(require_both_end)),
                                       -1 if wildcard is None else int(wildcard))


def wfa_ed(v1, v2):
    """Full end-to-end ED with '*' as wildcard (sequence_alignment.rs:18-20)."""
    return wfa_ed_config(v1, v2, True, ord("*"))


def wfa_ed_batch(pairs, require_both_end=True, wildcard=ord("*"), context=None):
    """wfa_ed_config over many (v1, v2) pairs on the device, one wave64 per pair
    (wc_wfa_ed_batch, sequence_alignment.rs:36-87). The defaults are wfa_ed's
    (sequence_alignment.rs:18-20). Returns a list of edit distances."""
    import ctypes
    pairs = [(bytes(a), bytes(b)) for a, b in pairs]
    n = len(pairs)
    if n == 0:
        return []
    ctx = context or _lib.default_context()
    u8p = ctypes.POINTER(ctypes.c_uint8)
    bufs = [(ctypes.create_string_buffer(a, max(len(a), 1)), ctypes.create_string_buffer(b, max(len(b), 1)))
            for a, b in pairs]
    p1 = (u8p * n)(*[ctypes.cast(x, u8p) for x, _ in bufs])
    p2 = (u8p * n)(*[ctypes.cast(y, u8p) for _, y in bufs])
    l1 = (ctypes.c_uint64 * n)(*[len(a) for a, _ in pairs])
    l2 = (ctypes.c_uint64 * n)(*[len(b) for _, b in pairs])
    out = (ctypes.c_uint64 * n)()
    rc = _lib.lib().wc_wfa_ed_batch(ctx.handle, n, p1, l1, p2, l2, int(bool(require_both_end)),
                                    -1 if wildcard is None else int(wildcard), out)
    if rc != _lib.WC_OK:
        raise _lib.WaffleConError("wc_wfa_ed_batch failed: " + ctx.last_error(), rc)
    return list(out)
