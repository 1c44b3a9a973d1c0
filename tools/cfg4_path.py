"""The sub-problems of the cfg4 locus (GPU box): the bench's locus
(synth.cfg4_locus(4), one level, wildcard '*'), every DualConsensusDWFA
sub-problem of its PriorityConsensusDWFA search logged (WC_SUBPROB_LOG:
owner level reads made_ms done_ms pops updates split status), with the
engine time per pop.  python tools/cfg4_path.py [--out gpurun_out/c4p]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/c4p")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    import waffle_con_amd as w
    from waffle_con_amd import synth
    from waffle_con_amd.cdwfa_config import CdwfaConfig
    cfg = CdwfaConfig(wildcard=ord("*"))
    chains = [[r] for r in synth.cfg4_locus(4)]
    log = os.path.join(a.out, "sub.txt")
    if os.path.exists(log):
        os.remove(log)
    os.environ["WC_SUBPROB_LOG"] = log
    t0 = time.perf_counter()
    _, st = w.priority_consensus_batch([(chains, None, None)], cfg)
    wall = time.perf_counter() - t0
    del os.environ["WC_SUBPROB_LOG"]
    print(json.dumps({"wall_s": wall, "kernel_ms": st["kernel_ms"], "pops": st["pops"]}), flush=True)
    with open(log) as f:
        for line in f:
            o, lvl, n, tm, td, pops, upd, split, status = line.split()
            run = float(td) - float(tm)
            print(json.dumps({"owner": int(o), "reads": int(n), "made_ms": float(tm), "done_ms": float(td),
                              "run_ms": round(run, 1), "pops": int(pops),
                              "us_per_pop": round(1000 * run / max(1, int(pops)), 2), "split": int(split)}), flush=True)


if __name__ == "__main__":
    main()
