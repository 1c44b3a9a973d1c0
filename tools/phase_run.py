"""Where does the single engine spend its time? (run on the GPU box)

Loads a phase-profiling build of the library (WAFFLE_CON_LIB, built with
`make -C waffle_con_amd/csrc EXTRA=-DWC_PHASE_PROF OUT=../libwaffle_con_prof.so`)
and writes, for the bench workload:
  - shader cycles per engine phase summed over workgroups (WC_PHASES file),
  - the per-locus work distribution (pops, updates, ED increases),
  - the latency of the single heaviest locus run alone vs the whole batch.
Usage: python tools/phase_run.py [--loci N] [--out gpurun_out/phases]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = {0: "pop-broadcast", 1: "analyze", 2: "finalize", 3: "votes+select", 4: "clone-copy", 5: "push-thread",
          6: "push-heavy", 7: "heap-insert", 8: "chain-prepare", 9: "chain-walk", 10: "chain-votes",
          11: "chain-accept", 12: "votes-wave", 13: "pop-logic", 14: "chain-total"}
# the one-wave dual engine's own counters (wave_dual.hip.hpp; 32..39 and 53..55)
WAVE_SUB = {32: "hot-load-block", 33: "hot-loads", 34: "analysis-lanes", 35: "general-end-or-wide",
            36: "general-weighted-or-f64-tie", 37: "fast-pushes", 38: "votes", 39: "general-children",
            53: "heavy-calls", 54: "heavy-cycles", 55: "heavy-items",
            45: "pop-to-heap", 46: "pop-heap", 47: "pop-meta-pc",
            48: "push-lanes", 49: "push-prune-cost"}
# the dual engine marks the same ids: 10 = activation, 11 = prune + cost
DUAL_PHASES = dict(PHASES)
DUAL_PHASES.update({10: "activate", 11: "prune+cost"})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--loci", type=int, default=1000)
    ap.add_argument("--len", type=int, default=10000)
    ap.add_argument("--reads", type=int, default=100)
    ap.add_argument("--err", type=float, default=0.005)
    ap.add_argument("--out", default="gpurun_out/phases")
    ap.add_argument("--workload", default="cfg2", choices=("cfg2", "cfg3", "cfg5-hpc"),
                    help="cfg2 single engine; cfg3 dual loci; cfg5-hpc: the first (HPC-level) dual "
                         "sub-problem of cfg5 loci")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    ph_file = os.path.join(a.out, "phases.txt")
    if os.path.exists(ph_file):
        os.remove(ph_file)
    import waffle_con_amd as w
    from waffle_con_amd.cdwfa_config import CdwfaConfig
    from waffle_con_amd import synth
    if a.workload == "cfg2":
        cfg = CdwfaConfig(min_count=a.reads // 4)
        loci = [w.generate_test(4, a.len, a.reads, a.err, s)[1] for s in range(a.loci)]
    elif a.workload == "cfg3":
        cfg = CdwfaConfig()
        loci = [synth.cfg3_locus(s) for s in range(a.loci)]
    else:
        cfg = CdwfaConfig(wildcard=ord("*"))
        loci = [[ch[0] for ch in synth.cfg5_locus(s)] for s in range(a.loci)]
    batch = w.ResidentBatch(loci)
    run = batch.consensus if a.workload == "cfg2" else batch.dual_consensus
    run(cfg)  # warm-up (no phase file yet)
    os.environ["WC_PHASES"] = ph_file
    t0 = time.perf_counter()
    if a.workload == "cfg2":
        res, st = batch.consensus(cfg, per_problem=True)
    else:
        res, st = batch.dual_consensus(cfg, per_problem=True)
    wall = time.perf_counter() - t0
    del os.environ["WC_PHASES"]
    rep = {"loci": a.loci, "kernel_ms": st["kernel_ms"], "wall_s": wall, "updates": st["updates"],
           "pops": st["pops"], "ed_increases": st["ed_increases"]}
    with open(ph_file) as f:
        line = f.read().strip().splitlines()[-1].split()
    cyc = [int(x) for x in line[2:]]
    names = PHASES if a.workload == "cfg2" else DUAL_PHASES
    tot = sum(cyc[k] for k in names if k not in (12, 14)) or 1
    rep["phase_share"] = {names[k]: round(cyc[k] / tot, 4) for k in names}
    rep["workload"] = a.workload
    if a.workload != "cfg2":
        rep["cycles_per_pop_per_wg"] = round(tot / max(1, st["pops"]), 1)
        pp = st.get("per_problem")
        if pp:
            # is the launch bound by its heaviest locus (all loci run at once)?
            pops = sorted(p["pops"] for p in pp)
            rep["pops_min_med_p90_max"] = [pops[0], pops[len(pops) // 2], pops[(9 * len(pops)) // 10], pops[-1]]
            heavy = max(range(len(pp)), key=lambda i: pp[i]["pops"])
            one = w.ResidentBatch([loci[heavy]])
            one.dual_consensus(cfg)
            _, s1 = one.dual_consensus(cfg)
            os.environ["WC_PHASES"] = ph_file
            _, s1 = one.dual_consensus(cfg)
            del os.environ["WC_PHASES"]
            with open(ph_file) as f:
                c1 = [int(x) for x in f.read().strip().splitlines()[-1].split()[2:]]
            t1 = sum(c1[k] for k in names if k not in (12, 14)) or 1
            rep["heaviest_alone_kernel_ms"] = s1["kernel_ms"]
            rep["heaviest_alone_us_per_pop"] = 1000.0 * s1["kernel_ms"] / max(1, pp[heavy]["pops"])
            rep["heaviest_alone_cycles_per_pop"] = round(t1 / max(1, pp[heavy]["pops"]), 1)
            rep["heaviest_alone_phase_cycles_per_pop"] = {names[k]: round(c1[k] / max(1, pp[heavy]["pops"]), 1)
                                                          for k in names if c1[k]}
            rep["heaviest_id"] = heavy
        # dual sub-phase counters (engine.hip dual_build_children; wave 0's view)
        np_ = max(1, st["pops"])
        DSUB = {16: "group_items", 17: "wave_items", 18: "row_resumes(w0)", 19: "group_loop_cycles(w0)",
                20: "wave_loop_cycles(w0)", 21: "children", 28: "votes-insertion-order(w0)", 29: "votes-fx-order(w0)",
                30: "votes-sums(w0)", 31: "active-min-growth(t0)", 22: "prune-setup(t0)", 23: "prune-loop(t0)",
                24: "prune-atomics(t0)", 25: "prune-barrier1(t0)", 26: "prune-tail(t0)"}
        rep["dual_sub_per_pop"] = {DSUB[k]: round(cyc[k] / np_, 2) for k in DSUB if k < len(cyc)}
        # the one-wave dual engine (wave_dual.hip.hpp) uses 32..39 for its own timers
        rep["wave_sub_per_pop"] = {nm: round(cyc[k] / np_, 2) for k, nm in WAVE_SUB.items() if k < len(cyc)}
        if len(cyc) >= 40:  # chain statistics per kind (engine.hip dual chain call site)
            for kind, b in (("single_consensus_chains", 32), ("dual_chains", 35)):
                n = max(1, cyc[b])
                rep[kind] = {"attempts": cyc[b], "accepted_nodes": cyc[b + 1], "nodes_per_attempt": round(cyc[b + 1] / n, 2),
                             "speculative_steps_per_attempt": round(cyc[b + 2] / n, 2),
                             "cycles_per_attempt(t0)": round(cyc[b + 6 - (b - 32) // 3 * 2] / n, 1)}
        print(json.dumps(rep, indent=1))
        with open(os.path.join(a.out, "report.json"), "w") as f:
            json.dump(rep, f, indent=1)
        return
    c15 = cyc[15]
    rep["chains"] = {"count": c15 & 0xFFFFF, "full": (c15 >> 20) & 0xFFFFF, "accepted_steps": c15 >> 40}
    # wave-0 sub-phases (cycles per chain, summed over workgroups / chains)
    # (the run-length walk: 16 = the lanes' own loops, 17 = the wave's edit-distance
    # increases and the steps they end, 18 = the whole walk of wave 0, 26 = rounds of
    # lane loops, 27 = lane-loop iterations, the wave's maximum per round)
    SUB = {16: "walk-lanes", 17: "walk-heavy", 18: "walk-total(w0)", 19: "walk-heavy-count(w0)", 20: "votes-fast",
           21: "votes-exact", 23: "prepare-windows", 24: "prepare-predict", 25: "votes-exact-count(w0)",
           26: "walk-rounds(w0)", 27: "walk-lane-iterations(w0)", 40: "accept-tracker-steps(w0)",
           41: "accept-tracker-loop(w0)", 42: "walk-lane0-iterations", 43: "chain-entry(w0)",
           44: "prepare-predict-only(w0)", 45: "walk-total(sum over waves)", 46: "walk-heavy-count(all waves)",
           48: "heavy-row-load(all waves)", 49: "heavy-increase-loop(all waves)", 50: "heavy-store-rebuild(all waves)",
           51: "heavy-call(w0)", 52: "heavy-tail-nominations(w0)"}
    nch = max(1, rep["chains"]["count"])
    rep["sub_cycles_per_chain"] = {SUB[k]: round(cyc[k] / nch, 1) for k in SUB if k < len(cyc)}
    rep["block_cycles_per_chain"] = {PHASES[k]: round(cyc[k] / nch, 1) for k in (8, 9, 10, 11, 14)}
    pp = st.get("per_problem")
    if pp:
        pops = sorted(p["pops"] for p in pp)
        rep["pops_min_med_max"] = [pops[0], pops[len(pops) // 2], pops[-1]]
        heavy = max(range(len(pp)), key=lambda i: pp[i]["pops"] + pp[i]["ed_increases"])
        one = w.ResidentBatch([loci[heavy]])
        one.consensus(cfg)
        _, s1 = one.consensus(cfg)
        rep["heaviest_alone_kernel_ms"] = s1["kernel_ms"]
        rep["heaviest_id"] = heavy
    print(json.dumps(rep, indent=1))
    with open(os.path.join(a.out, "report.json"), "w") as f:
        json.dump(rep, f, indent=1)


if __name__ == "__main__":
    main()
