"""Diagnostic (GPU box): the pop sequences (WC_POP_TRACE) of one dual problem
on two engine builds, and the first pop where they differ.
  python tools/pop_trace_diff.py <outdir> <case> A=1,B=2 C=3
(the environments of the two sides, comma-separated). Each side runs the builds test's dual problem `case` (tools/votes_diag.py's
cases) with its environment; each trace record is (cost, len, flags, extra):
flags = dual | action << 1 | nsome1 << 8 | nsome2 << 20, extra = active_min."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import hip_runner as hip  # noqa: E402
import waffle_con_amd as w  # noqa: E402

os.environ["WAFFLE_CON_SERVICE"] = "0"
os.environ["WC_WAVE"] = "0"


def case(i):
    L, N, err, seeds = [(700, 20, 0.01, (8, 9)), (500, 64, 0.01, (10, 11))][i]
    a = w.generate_test(4, L, N, err, seeds[0])[1]
    b = w.generate_test(4, L, N, err, seeds[1])[1]
    return [x for pair in zip(a, b) for x in pair], max(2, N // 4)


def run(tag, env, i, out):
    path = os.path.join(out, "trace_%s.txt" % tag)
    if os.path.exists(path):
        os.remove(path)
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    os.environ["WC_POP_TRACE"] = path
    mix, mc = case(i)
    try:
        hip.dual_consensus(mix, counters=True, min_count=mc)
        msg = "ok"
    except Exception as e:  # noqa: BLE001
        msg = "ERR %s" % e
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    os.environ.pop("WC_POP_TRACE", None)
    launches, cur = [], None
    with open(path) as f:
        for ln in f:
            if ln.startswith("#"):
                cur = []
                launches.append((ln.strip(), cur))
            else:
                cur.append(tuple(int(x) for x in ln.split()))
    print(tag, env, msg, [(h, len(r)) for h, r in launches], flush=True)
    return launches


def main():
    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    i = int(sys.argv[2])
    envs = [dict(kv.split("=", 1) for kv in arg.split(",") if kv) for arg in sys.argv[3:5]]
    ta = run("a", envs[0], i, out)
    tb = run("b", envs[1], i, out)
    ra, rb = ta[0][1], tb[0][1]
    n = min(len(ra), len(rb))
    first = next((k for k in range(n) if ra[k] != rb[k]), None)
    if first is None:
        print("first launches agree on %d pops (lengths %d, %d)" % (n, len(ra), len(rb)))
        return
    print("first difference at pop %d of %d/%d" % (first, len(ra), len(rb)))
    for k in range(max(0, first - 6), min(n, first + 6)):
        def fmt(r):
            c, ln, fl, ex = r
            return "cost %5d len %4d dual %d act %d some %3d/%3d am %d" % (c, ln, fl & 1, (fl >> 1) & 127, (fl >> 8) & 0xFFF,
                                                                          fl >> 20, ex)
        print("%6d %s | %s%s" % (k, fmt(ra[k]), fmt(rb[k]), "  <<" if ra[k] != rb[k] else ""))


if __name__ == "__main__":
    main()
