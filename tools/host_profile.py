"""Where does the host spend a cfg2 bench step outside the kernel? (GPU box)
  python tools/host_profile.py [--loci 1000]"""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--loci", type=int, default=1000)
    a = ap.parse_args()
    import waffle_con_amd as w
    from waffle_con_amd.cdwfa_config import CdwfaConfig
    loci = [w.generate_test(4, 10000, 100, 0.005, s)[1] for s in range(a.loci)]
    b = w.ResidentBatch(loci)
    cfg = CdwfaConfig(min_count=25)
    for _ in range(2):
        b.consensus(cfg)
    t0 = time.perf_counter()
    _, st = b.consensus(cfg)
    wall = time.perf_counter() - t0
    print({"wall_ms": wall * 1e3, "kernel_ms": st["kernel_ms"]})
    pr = cProfile.Profile()
    pr.enable()
    b.consensus(cfg)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(15)


if __name__ == "__main__":
    main()
