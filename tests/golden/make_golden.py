"""Regenerates tests/golden/dwfa_vectors.json from the reference's own DWFA unit
test literals (src/dynamic_wfa.rs:455-471, test_big_early_termination).

Run HERE only (the reference tree does not exist on the GPU box); the output is
a data fixture: the two input sequences of that test. The expected values
(e <= 2 throughout, e == 2 at the end and after finalize) are asserted in
tests/ref_cases.py, citing the reference lines.
"""
import json
import os
import re

SRC = "/root/reference/src/dynamic_wfa.rs"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dwfa_vectors.json")

text = open(SRC).read()
c1 = re.search(r'let c1 = "([ACGT]+)";', text).group(1)
seq_23 = re.search(r'let seq_23 = "([ACGT]+)";', text).group(1)
json.dump({"source": "src/dynamic_wfa.rs:456-457 (test_big_early_termination)",
           "c1": c1, "seq_23": seq_23}, open(OUT, "w"), indent=1)
print("wrote", OUT, len(c1), len(seq_23))
