"""Resident batches (wc_batch_*): upload the reads of many loci to HBM once,
then run the consensus engines over them repeatedly. This is the throughput
path bench.py measures (inputs already resident when the timed region starts)."""
import ctypes

from . import _lib
from .cdwfa_config import CdwfaConfig
from .consensus import _problems, _single_results, _stats
from .dual_consensus import _dual_results


class ResidentBatch:
    def __init__(self, problems, context=None):
        self.ctx = context or _lib.default_context()
        L = _lib.lib()
        self._batch = [(p, None) if not isinstance(p, tuple) else p for p in problems]
        arr, keep = _problems(self._batch)
        h = ctypes.c_void_p()
        rc = L.wc_batch_create(self.ctx.handle, len(self._batch), arr, ctypes.byref(h))
        if rc != _lib.WC_OK:
            raise _lib.WaffleConError("wc_batch_create failed: " + self.ctx.last_error(), rc)
        self.handle = h
        self.bytes = L.wc_batch_bytes(h)

    def refill(self, problems):
        """Upload a new set of problems into this batch's device buffers
        (wc_batch_refill: reused when large enough, so no allocation)."""
        L = _lib.lib()
        batch = [(p, None) if not isinstance(p, tuple) else p for p in problems]
        arr, keep = _problems(batch)
        rc = L.wc_batch_refill(self.ctx.handle, self.handle, len(batch), arr)
        if rc != _lib.WC_OK:
            # the library left the batch as it was (host.cpp upload_batch commits
            # only a complete upload), so this object keeps describing it
            raise _lib.WaffleConError("wc_batch_refill failed: " + self.ctx.last_error(), rc)
        self._batch = batch
        self.bytes = L.wc_batch_bytes(self.handle)

    def __len__(self):
        return len(self._batch)

    def consensus(self, config=None, return_errors=True, per_problem=False, context=None):
        """ConsensusDWFA over every problem of the batch. `context` may name
        another context on the same device (e.g. a compute context while this
        batch's own context uploads the next batch)."""
        config = config or CdwfaConfig()
        ctx = context or self.ctx
        L = _lib.lib()
        cfg = _lib.make_config(config)
        res = ctypes.c_void_p()
        rc = L.wc_batch_consensus(ctx.handle, self.handle, ctypes.byref(cfg), ctypes.byref(res))
        if rc != _lib.WC_OK:
            raise _lib.WaffleConError("wc_batch_consensus failed: " + ctx.last_error(), rc)
        stats = _stats(res, L, per_problem)
        return _single_results(res, len(self._batch), config.consensus_cost, L, return_errors), stats

    def dual_consensus(self, config=None, return_errors=True, context=None, per_problem=False):
        config = config or CdwfaConfig()
        ctx = context or self.ctx
        L = _lib.lib()
        cfg = _lib.make_config(config)
        res = ctypes.c_void_p()
        rc = L.wc_batch_dual_consensus(ctx.handle, self.handle, ctypes.byref(cfg), ctypes.byref(res))
        if rc != _lib.WC_OK:
            raise _lib.WaffleConError("wc_batch_dual_consensus failed: " + ctx.last_error(), rc)
        try:
            return _dual_results(res, self._batch, config, L, return_errors), _stats(res, L, per_problem)
        finally:
            L.wc_results_free(res)

    def close(self):
        if getattr(self, "handle", None):
            _lib.lib().wc_batch_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
