"""DualConsensusDWFA throughput on cfg3-shaped loci (a 5 kb
haplotype A, B = A + 12 SNVs + 2 short indels, 100 reads from each at 0.5%
sub/ins/del, A-block then B-block), GPU engine vs the CPU oracle on the same
loci. Diagnostic (not the headline bench). Usage:
  python tools/dual_bench.py --loci 256 [--cpu-loci 32] [--no-gpu]"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--loci", type=int, default=256)
    ap.add_argument("--cpu-loci", type=int, default=32)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--no-gpu", action="store_true")
    a = ap.parse_args()
    from waffle_con_amd import synth
    loci = [synth.cfg3_locus(s) for s in range(a.loci)]
    rep = {"loci": a.loci, "workload": "cfg3-shaped DualConsensusDWFA: 2 x 100 reads x 5 kb @ 0.5%"}
    gpu = None
    if not a.no_gpu:
        import torch
        torch.cuda.init()
        import waffle_con_amd as w
        from waffle_con_amd.cdwfa_config import CdwfaConfig
        batch = w.ResidentBatch(loci)
        cfg = CdwfaConfig()
        batch.dual_consensus(cfg)
        t0 = time.perf_counter()
        gpu, st = batch.dual_consensus(cfg)
        dt = time.perf_counter() - t0
        rep.update({"gpu_loci_per_s": a.loci / dt, "gpu_kernel_ms": st["kernel_ms"], "gpu_wall_s": dt,
                    "launches": st["launches"],
                    "per_locus": {k: st[k] / a.loci for k in ("pops", "nodes_explored", "nodes_ignored",
                                                              "updates", "ed_increases", "finalizes")},
                    "peak_queue_size": st["peak_queue_size"]})
    import oracle_ffi as orc
    n = min(a.cpu_loci, a.loci)
    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=a.threads) as ex:
        cpu = list(ex.map(lambda p: orc.dual_consensus(p), loci[:n]))
    dt = time.perf_counter() - t0
    rep.update({"cpu_loci": n, "cpu_threads": a.threads, "cpu_loci_per_s": n / dt, "cpu_wall_s": dt})
    if gpu is not None:
        def norm(rs):
            if isinstance(rs, Exception):
                return repr(rs)
            return [(r.consensus1().sequence(), r.consensus2().sequence() if r.consensus2() else None,
                     list(r.is_consensus1())) for r in rs]
        ok = 0
        for i in range(n):
            exp = [(r["consensus1"]["sequence"], r["consensus2"]["sequence"] if r["consensus2"] else None,
                    r["is_consensus1"]) for r in cpu[i]]
            ok += norm(gpu[i]) == exp
        rep["gpu_matches_cpu"] = "%d/%d" % (ok, n)
    print(json.dumps(rep), flush=True)


if __name__ == "__main__":
    main()
