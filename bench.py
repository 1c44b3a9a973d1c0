"""Benchmark: read-DWFA extension updates/sec + consensus loci/sec on MI355X.

Workload (BASELINE.json configs[1], north-star throughput form): ConsensusDWFA
over synthetic HiFi-like loci — generate_test(alphabet 4, 10 kb, 100 reads,
0.5% error) with seed = locus id, min_count = 100/4 (consensus_bench.rs
convention). One "step" = the whole batch of loci through the device-resident
engine: one engine launch over reads already resident in HBM (ResidentBatch,
uploaded before the timed region), plus the read-back of the consensus
records. The engine kernel time is measured separately with HIP events on the
library's stream (kernel_ms_per_step) and drives the roofline figure.

roofline.traffic is the HBM byte count per launch measured by the rocprofv3
PMC passes committed under profiles/ (FETCH_SIZE and WRITE_SIZE in separate
passes, FETCH_SIZE doubled per MI355X_MICROARCH.md's gfx950 note); it is
reported only when the recorded workload equals this run's.

Multi-GPU: one process per GPU (torch.distributed.run); loci are sharded
(weak scaling: every rank owns --loci loci), no collective on the data path.
Rank 0 prints one JSON line.
"""
import argparse
import gc
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--loci", type=int, default=1000, help="loci per GPU")
    ap.add_argument("--len", type=int, default=10000)
    ap.add_argument("--reads", type=int, default=100)
    ap.add_argument("--err", type=float, default=0.005)
    ap.add_argument("--cpu-sample", type=int, default=1000, help="loci timed on the CPU oracle (rank 0, N=1)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    return ap.parse_args()


def gen_loci(seeds, L, N, err, threads=16):
    import waffle_con_amd as w
    with ThreadPoolExecutor(max_workers=threads) as ex:
        return list(ex.map(lambda s: w.generate_test(4, L, N, err, s)[1], seeds))


def cpu_baseline(loci, min_count, threads):
    """CPU oracle (C++ restatement of the reference search) on a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as orc
    orc.lib()
    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=threads) as ex:
        outs = list(ex.map(lambda p: orc.consensus(p, counters=True, min_count=min_count), loci))
    dt = time.perf_counter() - t0
    updates = sum(c["updates"] for _, c in outs)
    return dt, updates, outs


def pmc_traffic(loci, reads, length, err):
    """HBM bytes per engine launch from the committed rocprofv3 PMC summary."""
    path = os.path.join(ROOT, "profiles", "r01_pmc_traffic.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        rec = json.load(f)
    w = rec.get("workload", {})
    if (w.get("loci_per_gpu"), w.get("reads"), w.get("len"), w.get("error_rate")) != (loci, reads, length, err):
        return None
    return rec.get("traffic_bytes_per_launch")


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # torch ships its own HIP runtime next to the one the library links: torch
    # must initialise the device first, or its later init finds no GPU
    import torch
    torch.cuda.init()
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    import waffle_con_amd as w
    from waffle_con_amd.cdwfa_config import CdwfaConfig

    ctx = w.Context(local_rank)
    cfg = CdwfaConfig(min_count=a.reads // 4)
    from waffle_con_amd.shard import shard_seeds
    seeds = shard_seeds(a.loci, rank)
    t0 = time.perf_counter()
    loci = gen_loci(seeds, a.len, a.reads, a.err)
    gen_s = time.perf_counter() - t0

    t0 = time.perf_counter()
    batch = w.ResidentBatch(loci, context=ctx)  # reads resident in HBM before timing
    upload_s = time.perf_counter() - t0

    def step():
        res, stats = batch.consensus(cfg, return_errors=True)
        bad = [r for r in res if isinstance(r, Exception)]
        if bad:
            raise RuntimeError("engine error: %s" % bad[0])
        return res, stats

    from waffle_con_amd import shard

    def sync():
        torch.cuda.synchronize()

    for _ in range(a.warmup):
        step()
    # the setup (torch, 1000 loci of reads) leaves a large Python heap: move it
    # to the permanent generation so a full collection inside the timed region
    # does not traverse it
    gc.collect()
    gc.freeze()
    kernel_ms, upd, wout, cmp = 0.0, 0, 0, 0
    last = None
    with shard.Timer(dist, sync) as tm:
        for _ in range(a.steps):
            last, st = step()
            kernel_ms += st["kernel_ms"]
            upd += st["updates"]
            wout += st["w_out"]
            cmp += st["compares"]
    elapsed, total_upd, total_loci = shard.reduce_run(
        dist, tm.elapsed, upd, a.loci * a.steps, device="cuda" if dist is not None else None)

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    # roofline of the engine kernel: algorithmic bytes per launch / kernel time
    per_launch_bytes = (8.0 * wout + 2.0 * cmp) / a.steps
    avg_kernel_s = kernel_ms / a.steps / 1e3
    achieved = per_launch_bytes / avg_kernel_s / 1e9
    correct = sum(1 for r in last if r and r[0].sequence() is not None)
    traffic = pmc_traffic(a.loci, a.reads, a.len, a.err)
    roofline = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                "kernel": "wc::single_engine_kernel",
                "algorithmic_bytes_per_launch": per_launch_bytes,
                # `achieved` counts the reference's bytes (every wavefront entry
                # read and written per update, every byte compare); the engine
                # skips the stuck diagonals, so it can exceed the HBM peak. The
                # bytes it really moves are the PMC traffic:
                "measured_gbs": (traffic / avg_kernel_s / 1e9) if traffic else None,
                "measured_frac": (traffic / avg_kernel_s / 1e9 / HBM_PEAK_GBS) if traffic else None}

    line = {
        "metric": "read-DWFA extension updates/sec + consensus loci/sec at 1/2/4/8 MI355X",
        "value": total_upd / elapsed,
        "unit": "updates/s",
        "loci_per_s": total_loci / elapsed,
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "kernel_ms_per_step": kernel_ms / a.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8/u32 (integer DWFA) + f64 votes",
        "data": "synthetic: generate_test(4, %d, %d, %g) seeds 0..%d (reference RNG restated)" % (
            a.len, a.reads, a.err, a.loci * world - 1),
        "config": {"workload": "ConsensusDWFA cfg2 throughput: %d loci/GPU x %d reads x %d bp @ %g error, "
                               "min_count %d" % (a.loci, a.reads, a.len, a.err, a.reads // 4),
                   "loci_per_gpu": a.loci, "reads": a.reads, "len": a.len, "error_rate": a.err,
                   "parallelism": "loci-sharded x%d (no collective)" % world},
        "roofline": roofline,
        "gen_s": gen_s,
        "upload_s": upload_s,
        "upload_bytes": batch.bytes,
        "results_ok": correct,
    }
    if world == 1 and not a.no_cpu:
        n = min(a.cpu_sample, len(loci))
        dt, cu, outs = cpu_baseline(loci[:n], a.reads // 4, a.cpu_threads)
        # parity spot check on the sample: GPU result == oracle result
        match = all([c.sequence() for c in last[i]] == [r["sequence"] for r in outs[i][0]] for i in range(n))
        line["cpu_baseline"] = {"value": cu / dt, "unit": "updates/s", "loci_per_s": n / dt, "cores": a.cpu_threads,
                                "kind": "port", "sample": "%d loci of the same workload (seeds 0..%d), "
                                                          "C++ oracle, %d threads, %.1f s wall" % (n, n - 1, a.cpu_threads, dt),
                                "gpu_matches_cpu_on_sample": match}
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
