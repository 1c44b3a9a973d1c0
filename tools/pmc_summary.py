"""Condense a tools/profile_round.sh run into the committed profiles/ files.

  python tools/pmc_summary.py <tag>
reads gpurun_out/prof_<tag>/{kt,fetch,write,sq1,sq2} and writes
  profiles/<tag>_kernel_stats.csv         rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_kernel_trace_engine.csv  engine dispatch rows of the trace
  profiles/<tag>_pmc_traffic.json         HBM bytes per engine launch (bench.py reads it)
  profiles/<tag>_issue_view.json          what a wave spends its cycles on (bench.py reads it)

FETCH_SIZE / WRITE_SIZE are reported by rocprofv3 in KiB. MI355X_MICROARCH.md
(HBM section) calibrates FETCH_SIZE on gfx950 to half the bytes of WIDE
(16 B/lane) coalesced reads only; the engine's reads are mostly narrow and
scattered, for which the guide gives no calibration. Both readings are kept:
traffic_bytes_per_launch takes FETCH_SIZE as reported (the uncalibrated lower
reading) and traffic_bytes_per_launch_if_wide doubles it (the upper reading).
SQ_* cycle counters count quad-cycles (guide, per-instruction constants).
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENGINES = ("engine_kernel", "dual_wave")  # block engines, wave engine (engine_wave.hip)


def counters(path):
    """{counter: [value per engine dispatch]} of one PMC pass."""
    out = {}
    if not os.path.exists(path):
        return out
    with open(path) as f:
        for row in csv.DictReader(f):
            if any(k in row["Kernel_Name"] for k in ENGINES):
                out.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    return out


def bench_line(path):
    with open(path) as f:
        lines = [l for l in f.read().splitlines() if l.startswith("{")]
    return json.loads(lines[-1])


def mean(v):
    return sum(v) / len(v) if v else None


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
    src = os.path.join(ROOT, "gpurun_out", "prof_" + tag)
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "kt", "run_kernel_stats.csv"), os.path.join(dst, tag + "_kernel_stats.csv"))
    with open(os.path.join(src, "kt", "run_kernel_trace.csv")) as f:
        rows = [r for r in csv.reader(f)]
    hdr, body = rows[0], [r for r in rows[1:] if any(k in c for c in r for k in ENGINES)]
    with open(os.path.join(dst, tag + "_kernel_trace_engine.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(hdr)
        w.writerows(body)
    kt = bench_line(os.path.join(src, "kt_bench.json"))
    fb = bench_line(os.path.join(src, "fetch_bench.json"))
    workload = kt["config"]["workload"]
    fetch = counters(os.path.join(src, "fetch", "run_counter_collection.csv")).get("FETCH_SIZE", [])
    write = counters(os.path.join(src, "write", "run_counter_collection.csv")).get("WRITE_SIZE", [])
    fetch_b = mean(fetch) * 1024.0
    write_b = mean(write) * 1024.0
    rec = {
        "tag": tag,
        "kernel": kt["roofline"]["kernel"],
        "workload": workload,
        "launches_fetch_pass": len(fetch),
        "launches_write_pass": len(write),
        "fetch_size_bytes_per_launch": fetch_b,
        "write_size_bytes_per_launch": write_b,
        "traffic_bytes_per_launch": fetch_b + write_b,
        "traffic_bytes_per_launch_if_wide": 2.0 * fetch_b + write_b,
        "traffic_formula": "FETCH_SIZE + WRITE_SIZE (KiB -> bytes); the gfx950 x2 FETCH correction is calibrated for "
                           "16-B/lane coalesced reads only, so it gives the upper reading (_if_wide)",
        "model_bytes_per_launch": kt["roofline"].get("model_bytes_per_launch"),
        "reference_equiv_bytes_per_step": kt["roofline"]["reference_equiv_bytes_per_step"],
        "kernel_ms_per_launch_bench_events": kt["roofline"]["kernel_ms_per_launch"],
        "kernel_ms_per_launch_pmc_pass": fb["roofline"]["kernel_ms_per_launch"],
    }
    with open(os.path.join(dst, tag + "_pmc_traffic.json"), "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec, indent=1))

    sq = {}
    for p in ("sq1", "sq2", "tcc"):
        for k, v in counters(os.path.join(src, p, "run_counter_collection.csv")).items():
            sq[k] = mean(v)
    if sq:
        iv = {"tag": tag, "kernel": kt["roofline"]["kernel"], "workload": workload, "counters_per_launch": sq}
        wc = sq.get("SQ_WAVE_CYCLES")
        if wc:
            iv["wave_cycle_split"] = {k: sq[k] / wc for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                             "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU") if k in sq}
        if sq.get("SQ_WAVES"):
            iv["per_wave"] = {k: sq[k] / sq["SQ_WAVES"] for k in sq if k.startswith("SQ_INSTS")}
        if sq.get("TCC_HIT_sum") is not None and sq.get("TCC_MISS_sum") is not None:
            iv["l2_hit_rate"] = sq["TCC_HIT_sum"] / max(1.0, sq["TCC_HIT_sum"] + sq["TCC_MISS_sum"])
        if sq.get("TCC_EA0_RDREQ_DRAM_sum") is not None:
            iv["dram_requests_per_launch"] = {"read": sq["TCC_EA0_RDREQ_DRAM_sum"],
                                              "write": sq.get("TCC_EA0_WRREQ_DRAM_sum")}
        if sq.get("SQ_INSTS_LDS") and "SQ_LDS_BANK_CONFLICT" in sq and sq.get("SQ_LDS_IDX_ACTIVE"):
            iv["lds_bank_conflict_share"] = sq["SQ_LDS_BANK_CONFLICT"] / sq["SQ_LDS_IDX_ACTIVE"]
        iv["note"] = ("SQ cycle counters are quad-cycles summed over waves; WAIT_ANY (parked on s_waitcnt / barrier) "
                      "+ WAIT_INST_ANY (issue stalls) + ACTIVE_INST_ANY ~= WAVE_CYCLES")
        with open(os.path.join(dst, tag + "_issue_view.json"), "w") as f:
            json.dump(iv, f, indent=1)
        print(json.dumps(iv, indent=1))


if __name__ == "__main__":
    main()
