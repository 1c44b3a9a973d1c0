"""Condense a tools/profile_round.sh run into the committed profiles/ files.

  python tools/pmc_summary.py r01
reads gpurun_out/prof_<tag>/{kt,fetch,write} and writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_kernel_trace_engine.csv   engine dispatch rows of the trace
  profiles/<tag>_pmc_traffic.json   HBM bytes per engine launch

FETCH_SIZE / WRITE_SIZE are reported by rocprofv3 in KiB. Per
MI355X_MICROARCH.md (HBM section) FETCH_SIZE on gfx950 reports half the bytes
of wide (16 B/lane) coalesced reads, so it is doubled; WRITE_SIZE is taken as
is. The engine's loads are a mix of 16-B RState loads and narrower accesses,
which the guide calls uncalibrated: the figure is an estimate of the order of
magnitude of HBM traffic, not an exact byte count.
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENGINE = "engine_kernel"


def counter_rows(path, name):
    out = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if ENGINE in row["Kernel_Name"] and row["Counter_Name"] == name:
                out.append(float(row["Counter_Value"]))
    return out


def bench_line(path):
    with open(path) as f:
        lines = [l for l in f.read().splitlines() if l.startswith("{")]
    return json.loads(lines[-1])


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    src = os.path.join(ROOT, "gpurun_out", "prof_" + tag)
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "kt", "run_kernel_stats.csv"), os.path.join(dst, tag + "_kernel_stats.csv"))
    with open(os.path.join(src, "kt", "run_kernel_trace.csv")) as f:
        rows = [r for r in csv.reader(f)]
    hdr, body = rows[0], [r for r in rows[1:] if any(ENGINE in c for c in r)]
    with open(os.path.join(dst, tag + "_kernel_trace_engine.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(hdr)
        w.writerows(body)
    fetch = counter_rows(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = counter_rows(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    kt = bench_line(os.path.join(src, "kt_bench.json"))
    fb = bench_line(os.path.join(src, "fetch_bench.json"))
    fetch_b = sum(fetch) / len(fetch) * 1024.0
    write_b = sum(write) / len(write) * 1024.0
    traffic = 2.0 * fetch_b + write_b
    cfg = kt["config"]
    rec = {
        "tag": tag,
        "kernel": "wc::single_engine_kernel",
        "workload": {k: cfg[k] for k in ("loci_per_gpu", "reads", "len", "error_rate")},
        "launches_fetch_pass": len(fetch),
        "launches_write_pass": len(write),
        "fetch_size_bytes_per_launch_raw": fetch_b,
        "write_size_bytes_per_launch": write_b,
        "traffic_bytes_per_launch": traffic,
        "traffic_formula": "2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes); gfx950 FETCH_SIZE halving correction",
        "algorithmic_bytes_per_launch": kt["roofline"]["algorithmic_bytes_per_launch"],
        "traffic_over_algorithmic": traffic / kt["roofline"]["algorithmic_bytes_per_launch"],
        "kernel_ms_per_launch_bench_events": kt["kernel_ms_per_step"],
        "kernel_ms_per_launch_pmc_pass": fb["kernel_ms_per_step"],
    }
    with open(os.path.join(dst, tag + "_pmc_traffic.json"), "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
