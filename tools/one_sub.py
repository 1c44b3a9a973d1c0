"""One DualConsensusDWFA problem alone, twice (warm-up + measured), for PMC
passes and A/B runs: the HPC-level sub-problem of cfg5 locus --seed (the
first level of its chains, all reads), the full-read level of the same chains
(cfg5-full: the level whose sub-problems make most of a deep locus's
critical path), or a cfg3 locus.
  python tools/one_sub.py --seed 48 [--workload cfg5-hpc|cfg3] [--reps 1]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg5-hpc",
                    choices=("cfg5-hpc", "cfg5-full", "cfg3", "cfg4-root", "cfg4-h01", "cfg4-h0"))
    ap.add_argument("--seed", type=int, default=48)
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--phases", default="", help="WC_PHASES file: per-pop phase cycles of the measured runs "
                                                 "(WC_PHASE_PROF library via WAFFLE_CON_LIB)")
    a = ap.parse_args()
    import waffle_con_amd as w
    from waffle_con_amd.cdwfa_config import CdwfaConfig
    from waffle_con_amd import synth
    if a.workload == "cfg3":
        p, cfg = synth.cfg3_locus(a.seed), CdwfaConfig()
    elif a.workload.startswith("cfg4"):
        # the cfg4 locus (synth.cfg4_locus(seed), 4 haplotypes x 50 reads):
        # all 200 reads (the priority search's root), the first two
        # haplotypes' 100, or the first one's 50
        p = synth.cfg4_locus(a.seed)
        p = p[:{"cfg4-root": 200, "cfg4-h01": 100, "cfg4-h0": 50}[a.workload]]
        cfg = CdwfaConfig(wildcard=ord("*"))
    else:
        lvl = 1 if a.workload == "cfg5-full" else 0
        p, cfg = [ch[lvl] for ch in synth.cfg5_locus(a.seed)], CdwfaConfig(wildcard=ord("*"))
    b = w.ResidentBatch([p])
    b.dual_consensus(cfg)
    if a.phases:
        if os.path.exists(a.phases):
            os.remove(a.phases)
        os.environ["WC_PHASES"] = a.phases
    for _ in range(a.reps):
        t0 = time.perf_counter()
        res, st = b.dual_consensus(cfg)
        print(json.dumps({"workload": a.workload, "seed": a.seed, "reads": len(p), "wall_s": time.perf_counter() - t0,
                          "kernel_ms": st["kernel_ms"], "pops": st["pops"], "updates": st["updates"],
                          "ed_increases": st["ed_increases"], "explored": st["nodes_explored"],
                          "ignored": st["nodes_ignored"], "peak_queue": st["peak_queue_size"],
                          "us_per_pop": 1000.0 * st["kernel_ms"] / max(1, st["pops"])}), flush=True)
    if a.phases:
        from phase_run import DUAL_PHASES, WAVE_SUB
        with open(a.phases) as f:
            cyc = [int(x) for x in f.read().strip().splitlines()[-1].split()[2:]]
        np_ = max(1, st["pops"])
        names = dict(DUAL_PHASES)
        names.update(WAVE_SUB)
        print(json.dumps({names.get(k, str(k)): round(v / np_, 1) for k, v in enumerate(cyc) if v}), flush=True)


if __name__ == "__main__":
    main()
