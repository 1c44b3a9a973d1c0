"""Diagnostic (GPU box): the builds test's dual problem on several builds and
chain settings, each compared with the oracle (results and counters)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import oracle_ffi as orc  # noqa: E402
import hip_runner as hip  # noqa: E402
import waffle_con_amd as w  # noqa: E402

os.environ["WAFFLE_CON_SERVICE"] = "0"
os.environ["WC_WAVE"] = "0"
cases = []
for (L, N, err, seeds) in [(700, 20, 0.01, (8, 9)), (500, 64, 0.01, (10, 11))]:
    a = w.generate_test(4, L, N, err, seeds[0])[1]
    b = w.generate_test(4, L, N, err, seeds[1])[1]
    cases.append(([x for pair in zip(a, b) for x in pair], max(2, N // 4)))
for env in ({"WC_CU": "0"}, {"WC_CU": "1"}, {"WC_CU": "1", "WC_DUAL_CHAIN": "0"}):
    for k in ("WC_CU", "WC_DUAL_CHAIN", "WC_CHAIN"):
        os.environ.pop(k, None)
    os.environ.update(env)
    for i, (mix, mc) in enumerate(cases):
        exp, ec = orc.dual_consensus(mix, counters=True, min_count=mc)
        try:
            got, gc = hip.dual_consensus(mix, counters=True, min_count=mc)
            bad = {k: (gc[k], ec[k]) for k in ec if k in gc and gc[k] != ec[k]}
            print(env, i, "same" if got == exp else "DIFF", bad, flush=True)
        except Exception as e:  # noqa: BLE001
            print(env, i, "ERR", e, flush=True)
