"""DWFALite (dynamic_wfa.rs:12-265) backed by the device: every update /
finalize / get_extension_candidates call runs the DWFA kernels on the GPU
(wc_dwfa_batch). State (edit distance, wavefront, offset) is held on the host
between calls, so clone() is a plain copy, as in the reference."""
import ctypes

from . import _lib


class DWFALite:
    WF_CAP_MIN = 256

    def __init__(self, wildcard=None, allow_early_termination=False):
        self._e = 0
        self._wf = [0]
        self._wildcard = wildcard
        self._early = bool(allow_early_termination)
        self._offset = 0

    @classmethod
    def new(cls, wildcard, allow_early_termination):
        return cls(wildcard, allow_early_termination)

    @classmethod
    def default(cls):
        return cls()

    def set_offset(self, offset):
        self._offset = int(offset)

    def clone(self):
        d = DWFALite(self._wildcard, self._early)
        d._e, d._wf, d._offset = self._e, list(self._wf), self._offset
        return d

    def __eq__(self, other):
        return (isinstance(other, DWFALite) and self._e == other._e and self._wf == other._wf
                and self._wildcard == other._wildcard and self._early == other._early
                and self._offset == other._offset)

    def _job(self, baseline, other, op):
        baseline, other = bytes(baseline), bytes(other)
        cap = max(self.WF_CAP_MIN, 2 * (len(baseline) + len(other)) + 3, len(self._wf))
        wf = (ctypes.c_uint64 * cap)(*self._wf)
        bb = ctypes.create_string_buffer(baseline, max(1, len(baseline)))
        ob = ctypes.create_string_buffer(other, max(1, len(other)))
        j = _lib.WcDwfaJob()
        j.baseline = ctypes.cast(bb, _lib._u8p)
        j.baseline_len = len(baseline)
        j.other = ctypes.cast(ob, _lib._u8p)
        j.other_len = len(other)
        j.offset = self._offset
        j.wildcard = -1 if self._wildcard is None else int(self._wildcard)
        j.early = int(self._early)
        j.op = op
        j.e = self._e
        j.wavefront = wf
        j.wf_len = len(self._wf)
        j.wf_cap = cap
        ctx = _lib.default_context()
        rc = _lib.lib().wc_dwfa_batch(ctx.handle, 1, ctypes.byref(j))
        if rc != _lib.WC_OK:
            raise _lib.WaffleConError("wc_dwfa_batch failed: " + ctx.last_error(), rc)
        if j.status != 0:
            raise _lib.WaffleConError("DWFA device job failed (status %d)" % j.status, j.status)
        return j, wf

    def update(self, baseline_seq, other_seq):
        """dynamic_wfa.rs:75-99; returns the edit distance."""
        j, wf = self._job(baseline_seq, other_seq, 0)
        self._e = j.e
        self._wf = [wf[i] for i in range(j.wf_len)]
        return self._e

    def finalize(self, baseline_seq, other_seq):
        """dynamic_wfa.rs:201-210 (never marks the DWFA finalized, as in the reference)."""
        j, wf = self._job(baseline_seq, other_seq, 1)
        self._e = j.e
        self._wf = [wf[i] for i in range(j.wf_len)]

    def get_extension_candidates(self, baseline_seq, other_seq):
        """dynamic_wfa.rs:241-255: {symbol: count} in FxHashMap iteration order."""
        j, _ = self._job(baseline_seq, other_seq, 2)
        return {j.cand_syms[k]: j.cand_counts[k] for k in range(j.n_cand)}

    def candidate_insertion_order(self, baseline_seq, other_seq):
        """The symbols of get_extension_candidates in the order the reference
        inserts them into its FxHashMap (first tip in ascending diagonal index,
        dynamic_wfa.rs:244-250; wc_dwfa_job.cand_first): the order a caller
        rebuilding the hashbrown map must insert in."""
        j, _ = self._job(baseline_seq, other_seq, 2)
        return [j.cand_first[k] for k in range(j.n_cand)]

    def maximum_baseline_distance(self):
        return max(d + self._e - i for i, d in enumerate(self._wf))

    def maximum_other_distance(self):
        return self._offset + max(self._wf)

    def reached_baseline_end(self, baseline_seq):
        return self.maximum_baseline_distance() == len(baseline_seq)

    def edit_distance(self):
        return self._e

    def wavefront(self):
        return list(self._wf)
