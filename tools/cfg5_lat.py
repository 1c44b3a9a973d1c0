"""Per-locus latency of a cfg5 batch (GPU box): one priority_consensus_batch
call over loci 0..N-1 (after a warm-up call), each locus's latency inside the
call, and from the sub-problem log (WC_SUBPROB_LOG) its critical path: the
longest chain of dependent sub-problems (a sub-problem is made when its parent
finishes), in pops and in ms under load. Writes one JSON row per locus with
the generator's parameters beside it, for fitting a latency cost model.
  python tools/cfg5_lat.py [--loci 2000] [--out gpurun_out/c5lat]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def critical(subs):
    """subs: (made_ms, done_ms, pops, reads, level) of one locus; the chain of
    parents (made == parent's done) with the most pops."""
    subs = sorted(subs)
    best = []
    for k, (m, d, p, n, lv) in enumerate(subs):
        par = -1
        for j in range(k):
            if abs(subs[j][1] - m) < 0.05 and subs[j][0] <= m:
                par = j if par < 0 or best[j][0] > best[par][0] else par
        prev = best[par] if par >= 0 else (0, 0.0, 0)
        best.append((prev[0] + p, prev[1] + (d - m), prev[2] + 1))
    return max(best) if best else (0, 0.0, 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--loci", type=int, default=2000)
    ap.add_argument("--out", default="gpurun_out/c5lat")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    from waffle_con_amd import synth
    ids = list(range(a.loci))
    loci = [synth.cfg5_locus(s) for s in ids]
    import waffle_con_amd as w
    from waffle_con_amd.cdwfa_config import CdwfaConfig
    cfg = CdwfaConfig(wildcard=ord("*"))
    w.priority_consensus_batch([(loci[0], None, None)], cfg)
    log = os.path.join(a.out, "sub.txt")
    if os.path.exists(log):
        os.remove(log)
    os.environ["WC_SUBPROB_LOG"] = log
    t0 = time.perf_counter()
    _, st = w.priority_consensus_batch([(x, None, None) for x in loci], cfg, per_problem=True)
    wall = time.perf_counter() - t0
    del os.environ["WC_SUBPROB_LOG"]
    per = st.pop("per_problem")
    subs = {}
    with open(log) as f:
        for line in f:
            o, lvl, n, tm, td, pops, upd, split, status = line.split()
            subs.setdefault(int(o), []).append((float(tm), float(td), int(pops), int(n), int(lvl)))
    rows = []
    for i in ids:
        L, nv, n = synth.cfg5_params(i)
        cp, cms, clen = critical(subs.get(i, []))
        rows.append({"seed": i, "len": L, "variants": nv, "reads_per_hap": n, "cost": synth.cfg5_cost(i),
                     "lat_ms": per[i]["wall_ms"], "pops": per[i]["pops"], "subs": len(subs.get(i, [])),
                     "crit_pops": cp, "crit_ms_under_load": cms, "crit_subs": clen})
    with open(os.path.join(a.out, "loci.json"), "w") as f:
        json.dump({"wall_s": wall, "kernel_ms": st["kernel_ms"], "loci": rows}, f)
    rows.sort(key=lambda r: -r["lat_ms"])
    print(json.dumps({"wall_s": wall, "kernel_ms": st["kernel_ms"]}))
    for r in rows[:15]:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
