"""Run one locus through an engine twice (warm-up + measured) for PMC passes:
  python tools/one_locus.py --workload cfg3 --seed 265"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg3", choices=("cfg2", "cfg3"))
    ap.add_argument("--seed", type=int, default=265)
    a = ap.parse_args()
    import waffle_con_amd as w
    from waffle_con_amd.cdwfa_config import CdwfaConfig
    from waffle_con_amd import synth
    if a.workload == "cfg2":
        b = w.ResidentBatch([w.generate_test(4, 10000, 100, 0.005, a.seed)[1]])
        run = lambda: b.consensus(CdwfaConfig(min_count=25))
    else:
        b = w.ResidentBatch([synth.cfg3_locus(a.seed)])
        run = lambda: b.dual_consensus(CdwfaConfig())
    run()
    t0 = time.perf_counter()
    _, st = run()
    print({"workload": a.workload, "seed": a.seed, "wall_s": time.perf_counter() - t0, "kernel_ms": st["kernel_ms"],
           "pops": st["pops"], "updates": st["updates"], "ed_increases": st["ed_increases"]})


if __name__ == "__main__":
    main()
