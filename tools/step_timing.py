"""Where a bench step's wall time goes: Python step wall vs the library's
wall_ms vs the engine kernel's HIP-event time, with or without torch owning
the HIP runtime (--torch-first). Diagnostic only."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--loci", type=int, default=1000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--torch-first", action="store_true")
    a = ap.parse_args()
    if a.torch_first:
        import torch
        torch.cuda.init()
        torch.cuda.set_device(0)
    import waffle_con_amd as w
    from waffle_con_amd.cdwfa_config import CdwfaConfig
    from bench import gen_loci
    loci = gen_loci(range(a.loci), 10000, 100, 0.005)
    ctx = w.Context(0)
    batch = w.ResidentBatch(loci, context=ctx)
    cfg = CdwfaConfig(min_count=25)
    rows = []
    for s in range(a.steps + 1):
        t0 = time.perf_counter()
        res, st = batch.consensus(cfg, return_errors=True)
        dt = (time.perf_counter() - t0) * 1e3
        rows.append({"step": s, "py_ms": round(dt, 2), "lib_wall_ms": round(st["wall_ms"], 2),
                     "kernel_ms": round(st["kernel_ms"], 2), "launches": st["launches"]})
    print(json.dumps({"torch_first": a.torch_first, "rows": rows}), flush=True)


if __name__ == "__main__":
    main()
