"""wfa_ed / wfa_ed_config (sequence_alignment.rs:18-87) via the library."""
from . import _lib


def wfa_ed_config(v1, v2, require_both_end, wildcard):
    v1, v2 = bytes(v1), bytes(v2)
    return _lib.lib().wc_wfa_ed_config(v1, len(v1), v2, len(v2), int(bool(require_both_end)),
                                       -1 if wildcard is None else int(wildcard))


def wfa_ed(v1, v2):
    """Full end-to-end ED with '*' as wildcard (sequence_alignment.rs:18-20)."""
    return wfa_ed_config(v1, v2, True, ord("*"))
