"""Occupancy experiment (GPU box): a PriorityConsensusDWFA batch of cfg5 loci
whose sub-problems all have at most 64 reads (2 x reads per haplotype <= 64),
timed once after a warm-up pass, under the environment given (WC_DUAL_LDS_KB:
the node pool's LDS budget, i.e. workgroups per CU; WC_WAVE_KERNEL=2: the
two-reads-per-lane kernel at 1 wave per SIMD for every problem).
  python tools/cfg5_small.py [--loci 4000]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--loci", type=int, default=4000)
    ap.add_argument("--phases", default="", help="WC_PHASES file: per-pop phase cycles of the measured run "
                                                 "(WC_PHASE_PROF library via WAFFLE_CON_LIB)")
    a = ap.parse_args()
    import waffle_con_amd as w
    from waffle_con_amd import synth
    from waffle_con_amd.cdwfa_config import CdwfaConfig
    ids = []
    s = 0
    while len(ids) < a.loci:
        if 2 * synth.cfg5_params(s)[2] <= 64:
            ids.append(s)
        s += 1
    loci = [synth.cfg5_locus(i) for i in ids]
    cfg = CdwfaConfig(wildcard=ord("*"))
    w.priority_consensus_batch([(L, None, None) for L in loci], cfg)
    if a.phases:
        if os.path.exists(a.phases):
            os.remove(a.phases)
        os.environ["WC_PHASES"] = a.phases
    t0 = time.perf_counter()
    _, st = w.priority_consensus_batch([(L, None, None) for L in loci], cfg)
    dt = time.perf_counter() - t0
    print(json.dumps({"loci": len(ids), "wall_s": dt, "loci_per_s": len(ids) / dt, "stats": {k: v for k, v in st.items() if isinstance(v, (int, float, str))}, "env": {k: v for k, v in os.environ.items() if k.startswith("WC_")}}),
          flush=True)
    if a.phases:
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from phase_run import DUAL_PHASES, WAVE_SUB
        cyc = [0] * 64
        with open(a.phases) as f:
            for ln in f.read().strip().splitlines():
                for k, x in enumerate(ln.split()[2:]):
                    cyc[k] += int(x)
        names = dict(DUAL_PHASES)
        names.update(WAVE_SUB)
        np_ = max(1, st["pops"])
        print(json.dumps({names.get(k, str(k)): round(v / np_, 1) for k, v in enumerate(cyc) if v}), flush=True)


if __name__ == "__main__":
    main()
