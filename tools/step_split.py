"""Where a cfg2 bench step's time goes outside the library call (GPU box):
the native wc_batch_consensus call, the stats, the result objects, and the
release of the previous step's results, per step."""
import ctypes
import gc
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import waffle_con_amd as w  # noqa: E402
from waffle_con_amd import _lib, synth  # noqa: E402,F401
from waffle_con_amd.cdwfa_config import CdwfaConfig  # noqa: E402
from waffle_con_amd.consensus import _single_results, _stats  # noqa: E402
from concurrent.futures import ThreadPoolExecutor  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
with ThreadPoolExecutor(16) as ex:
    loci = list(ex.map(lambda s: w.generate_test(4, 10000, 100, 0.005, s)[1], range(n)))
batch = w.ResidentBatch(loci)
cfg = CdwfaConfig(min_count=25)
L = _lib.lib()
last = None
for it in range(6):
    t0 = time.perf_counter()
    c = _lib.make_config(cfg)
    res = ctypes.c_void_p()
    rc = L.wc_batch_consensus(batch.ctx.handle, batch.handle, ctypes.byref(c), ctypes.byref(res))
    t1 = time.perf_counter()
    st = _stats(res, L)
    t2 = time.perf_counter()
    out = _single_results(res, n, cfg.consensus_cost, L, True)
    t3 = time.perf_counter()
    bad = [r for r in out if isinstance(r, Exception)]
    t4 = time.perf_counter()
    last = out  # drops the previous step's results
    t5 = time.perf_counter()
    print("step %d: native %.2f ms (wall_ms %.2f, kernel %.2f), stats %.2f, results %.2f, check %.2f, release %.2f, total %.2f"
          % (it, (t1 - t0) * 1e3, st["wall_ms"], st["kernel_ms"], (t2 - t1) * 1e3, (t3 - t2) * 1e3, (t4 - t3) * 1e3,
             (t5 - t4) * 1e3, (t5 - t0) * 1e3), flush=True)
    if it == 2:
        gc.collect()
        gc.freeze()
