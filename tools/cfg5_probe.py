"""Where does cfg5 (PriorityConsensusDWFA on PGx loci) lose time? (GPU box)
Runs a few loci one at a time (per-locus latency, pops) and then a batch
(throughput), so the batch wall can be compared with grid x mean latency.
  python tools/cfg5_probe.py [--loci 1024] [--single 8]"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--loci", type=int, default=1024)
    ap.add_argument("--single", type=int, default=8)
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    import waffle_con_amd as w
    from waffle_con_amd import synth
    from waffle_con_amd.cdwfa_config import CdwfaConfig
    cfg = CdwfaConfig(wildcard=ord("*"))
    with ThreadPoolExecutor(max_workers=16) as ex:
        loci = list(ex.map(synth.cfg5_locus, range(a.loci)))
    w.priority_consensus_batch([(loci[0], None, None)], cfg)  # warm-up
    rep = {"single": []}
    for i in range(a.single):
        t0 = time.perf_counter()
        _, st = w.priority_consensus_batch([(loci[i], None, None)], cfg)
        dt = time.perf_counter() - t0
        rep["single"].append({"seed": i, "reads": sum(len(c) for c in loci[i]), "len": len(loci[i][0][-1]),
                              "wall_ms": dt * 1e3, "kernel_ms": st["kernel_ms"], "pops": st["pops"],
                              "updates": st["updates"], "launches": st["launches"]})
        print(json.dumps(rep["single"][-1]), flush=True)
    t0 = time.perf_counter()
    _, st = w.priority_consensus_batch([(c, None, None) for c in loci], cfg)
    dt = time.perf_counter() - t0
    rep["batch"] = {"loci": a.loci, "wall_s": dt, "loci_per_s": a.loci / dt, "kernel_ms": st["kernel_ms"],
                    "pops": st["pops"], "updates": st["updates"], "launches": st["launches"]}
    print(json.dumps(rep["batch"]), flush=True)


if __name__ == "__main__":
    main()
