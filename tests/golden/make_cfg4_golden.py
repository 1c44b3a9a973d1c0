"""Writes tests/golden/cfg4_seed4.json: the CPU oracle's PriorityConsensusDWFA
output on the cfg4 locus (waffle_con_amd.synth.cfg4_locus(4): 4 haplotypes x
50 reads x 8 kb, inserted segments {0, 25, 60, 150} bp, wildcard '*'). The
oracle needs about two minutes here, so the GPU parity test
(tests/test_gpu_fullsize.py) compares against this fixture instead.
Sequences are stored as SHA-256 digests with their scores; the counters are
the oracle's work counters.

    python tests/golden/make_cfg4_golden.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import oracle_ffi as orc  # noqa: E402
from waffle_con_amd import synth  # noqa: E402


def main(seed=4):
    reads = synth.cfg4_locus(seed)
    res, c = orc.priority_consensus([[r] for r in reads], counters=True, wildcard=ord("*"))
    out = {
        "seed": seed,
        "input_sha256": hashlib.sha256(b"".join(reads)).hexdigest(),
        "config": {"wildcard": "*"},
        "sequence_indices": res["sequence_indices"],
        "consensuses": [[{"sha256": hashlib.sha256(x["sequence"]).hexdigest(), "len": len(x["sequence"]),
                          "scores": x["scores"]} for x in ch] for ch in res["consensuses"]],
        "counters": c,
    }
    with open(os.path.join(HERE, "cfg4_seed%d.json" % seed), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
