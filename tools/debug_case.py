"""Debug helper: run one reference dual case through oracle and HIP, print counters."""
import sys
sys.path.insert(0, "tests")
import oracle_ffi as orc
import ref_cases as rc
import hip_runner as hip

name = sys.argv[1]
case = rc.DUAL_CASES[name]
seqs = [rc.b(s) for s in case["seqs"]]
exp, ec = orc.dual_consensus(seqs, counters=True, **case["cfg"])
got, gc = hip.dual_consensus(seqs, counters=True, **case["cfg"])
print("equal results:", got == exp)
for k in ec:
    print(k, ec[k], gc.get(k))
