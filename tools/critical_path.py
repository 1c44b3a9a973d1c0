"""The critical path of single cfg5 loci (GPU box): each locus alone, every
DualConsensusDWFA sub-problem of its PriorityConsensusDWFA search logged
(WC_SUBPROB_LOG: owner level reads made_ms done_ms pops updates split status).
Loci: the --top heaviest by the bench's cost model among --total, plus --seeds.
  python tools/critical_path.py [--total 10000] [--top 3] [--seeds 5949 887] [--out gpurun_out/cp]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--total", type=int, default=10000)
    ap.add_argument("--top", type=int, default=3)
    ap.add_argument("--seeds", type=int, nargs="*", default=[])
    ap.add_argument("--out", default="gpurun_out/critical_path")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    from waffle_con_amd import synth
    costs = [synth.cfg5_cost(s) for s in range(a.total)]
    order = sorted(range(a.total), key=lambda i: (-costs[i], i))
    seeds = order[:a.top] + [s for s in a.seeds if s not in order[:a.top]]
    import torch
    torch.cuda.init()
    import waffle_con_amd as w
    from waffle_con_amd.cdwfa_config import CdwfaConfig
    cfg = CdwfaConfig(wildcard=ord("*"))
    w.priority_consensus_batch([(synth.cfg5_locus(seeds[0]), None, None)], cfg)  # warm-up
    rep = []
    for s in seeds:
        chains = synth.cfg5_locus(s)
        log = os.path.join(a.out, "sub_%d.txt" % s)
        if os.path.exists(log):
            os.remove(log)
        os.environ["WC_SUBPROB_LOG"] = log
        t0 = time.perf_counter()
        _, st = w.priority_consensus_batch([(chains, None, None)], cfg)
        wall = time.perf_counter() - t0
        del os.environ["WC_SUBPROB_LOG"]
        subs = []
        with open(log) as f:
            for line in f:
                o, lvl, n, tm, td, pops, upd, split, status = line.split()
                subs.append({"level": int(lvl), "reads": int(n), "made_ms": float(tm), "done_ms": float(td),
                             "run_ms": float(td) - float(tm), "pops": int(pops), "updates": int(upd),
                             "split": int(split)})
        r = {"seed": s, "cost": costs[s] if s < len(costs) else None, "chains": len(chains),
             "len": len(chains[0][-1]), "wall_s": wall, "kernel_ms": st["kernel_ms"], "pops": st["pops"],
             "sub_problems": subs}
        rep.append(r)
        print(json.dumps({k: v for k, v in r.items() if k != "sub_problems"}), flush=True)
        for x in subs:
            print("   ", json.dumps(x), flush=True)
    with open(os.path.join(a.out, "report.json"), "w") as f:
        json.dump(rep, f, indent=1)


if __name__ == "__main__":
    main()
