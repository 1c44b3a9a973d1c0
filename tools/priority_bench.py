"""PriorityConsensusDWFA throughput on cfg5-shaped PGx loci (SURVEY §8(d)
cfg5: length U[1000, 6000], two haplotypes differing by U{0..15} variants,
U[15, 40] reads each at 0.5% error, chains [HPC(read), read], wildcard '*'),
GPU (wc_priority_consensus_batch) vs the CPU oracle on a sample of the same
loci. Diagnostic (not the headline bench). Usage:
  python tools/priority_bench.py --loci 1024 [--cpu-loci 64]"""
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
    ap.add_argument("--loci", type=int, default=1024)
    ap.add_argument("--cpu-loci", type=int, default=64)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--no-gpu", action="store_true")
    a = ap.parse_args()
    from waffle_con_amd import synth
    with ThreadPoolExecutor(max_workers=a.threads) as ex:
        loci = list(ex.map(synth.cfg5_locus, range(a.loci)))
    rep = {"loci": a.loci, "workload": "cfg5-shaped PriorityConsensusDWFA: [HPC(read), read] chains, 2 haplotypes, "
                                       "1-6 kb, 15-40 reads each @ 0.5%, wildcard '*'",
           "reads_per_locus": sum(len(c) for c in loci) / a.loci}
    gpu = None
    if not a.no_gpu:
        import torch
        torch.cuda.init()
        import waffle_con_amd as w
        from waffle_con_amd.cdwfa_config import CdwfaConfig
        cfg = CdwfaConfig(wildcard=ord("*"))
        probs = [(c, None, None) for c in loci]
        w.priority_consensus_batch(probs[:8], cfg, return_errors=True)  # warm-up
        t0 = time.perf_counter()
        gpu, st = w.priority_consensus_batch(probs, cfg, return_errors=True)
        dt = time.perf_counter() - t0
        rep.update({"gpu_loci_per_s": a.loci / dt, "gpu_wall_s": dt})
    import oracle_ffi as orc
    n = min(a.cpu_loci, a.loci)
    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=a.threads) as ex:
        cpu = list(ex.map(lambda c: orc.priority_consensus(c, wildcard=ord("*")), loci[:n]))
    dt = time.perf_counter() - t0
    rep.update({"cpu_loci": n, "cpu_threads": a.threads, "cpu_loci_per_s": n / dt, "cpu_wall_s": dt})
    if gpu is not None:
        ok = 0
        for i in range(n):
            g = gpu[i]
            if isinstance(g, Exception):
                continue
            gc = [[c.sequence() for c in chain] for chain in g.consensuses()]
            ec = [[c["sequence"] for c in chain] for chain in cpu[i]["consensuses"]]
            ok += gc == ec and list(g.sequence_indices()) == list(cpu[i]["sequence_indices"])
        rep["gpu_matches_cpu"] = "%d/%d" % (ok, n)
    print(json.dumps(rep), flush=True)


if __name__ == "__main__":
    main()
