"""Benchmark: read-DWFA extension updates/sec + consensus loci/sec on MI355X.

Workloads (--workload, default cfg2):
  cfg2          BASELINE configs[1] throughput form: ConsensusDWFA over
                generate_test(4, 10 kb, 100 reads, 0.5%) loci, seed = locus id,
                min_count 25; --loci per GPU (weak scaling, loci sharded).
  cfg2-latency  one cfg2 locus at a time (single-locus latency); CPU = 1 thread.
  cfg3          DualConsensusDWFA on cfg3 loci (5 kb, 2 x 100 reads); --loci per GPU.
  cfg4          PriorityConsensusDWFA on one cfg4 locus (4 x 50 reads x 8 kb, length gaps).
  cfg5          PriorityConsensusDWFA over a FIXED batch of --loci cfg5 PGx loci
                (default 10,000) split over the ranks by a cost-sorted queue
                (strong scaling, no collective on the data path).
  cfg2-api      cfg2 loci through the per-locus API (ConsensusDWFA.consensus)
                from --api-threads native threads (the submission service).
  cfg5-api      cfg5 loci through PriorityConsensusDWFA.consensus from
                --api-threads native threads (the submission service).

One step = one pass of the engine over the rank's batch, reads resident in HBM
(ResidentBatch uploaded before timing; priority workloads upload per call and
that is inside the step). W untimed warmup steps, then exactly K timed steps
between barrier + device sync; value = work of all ranks / max-over-ranks time.

Reported beside `value`:
  * e2e_loci_per_s (cfg2): fresh batches every step, i.e. Python marshalling +
    pinned staging + H2D of the reads, double-buffered against the compute of
    the previous batch (two contexts on the device).
  * roofline: HBM bytes the dominant kernel actually moves (rocprofv3 PMC
    passes committed under profiles/, same workload) / its HIP-event time, with
    the reference-equivalent algorithmic bytes kept separately.
  * cpu_baseline: the C++ oracle on every CPU this process may use
    (affinity and cgroup quota), timed on the same host on a bounded sample.

--gpus N without torch.distributed.run env: N worker processes are started
(before anything touches the GPU) under torch.distributed.run.
"""
import argparse
import gc
import json
import os
import platform
import statistics
import subprocess
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "read-DWFA extension updates/sec + consensus loci/sec at 1/2/4/8 MI355X"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="cfg2", choices=sorted(WORKLOADS))
    ap.add_argument("--loci", type=int, default=None, help="loci per GPU (cfg2/cfg3) or in total (cfg5)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-oracle sample time")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every usable CPU")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--api-threads", type=int, default=64, help="cfg2-api: native caller threads")
    ap.add_argument("--cfg5-loci", type=int, default=10000,
                    help="cfg2 (default line): also run the fixed cfg5 batch of this many loci, strong-scaled "
                         "over the ranks (0 = skip)")
    return ap.parse_args()


# ---------------------------------------------------------------------------
# host facts
# ---------------------------------------------------------------------------
def usable_cpus():
    """CPUs this process may run on: the affinity set, capped by a cgroup v2
    cpu.max quota when one is set."""
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()
        if q != "max":
            quota = max(1, int(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    return (min(n, quota) if quota else n), n, quota


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def spawn_workers(a):
    """--gpus N without a launcher: start N ranks under torch.distributed.run
    (this process never initialises the GPU) and exit with their status."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(a.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


# ---------------------------------------------------------------------------
# workloads
# ---------------------------------------------------------------------------
def _threads():
    return max(1, min(16, usable_cpus()[0]))


def gen_cfg2(seeds, L=10000, N=100, err=0.005):
    import waffle_con_amd as w
    with ThreadPoolExecutor(max_workers=_threads()) as ex:
        return list(ex.map(lambda s: w.generate_test(4, L, N, err, s)[1], seeds))


def pool_map(fn, items):
    """fn over items in worker processes forked before this process touches
    the GPU (input generation of the large workloads; threads are GIL-bound)."""
    n = max(1, min(16, usable_cpus()[0]))
    if n == 1 or len(items) < 64:
        return [fn(x) for x in items]
    import multiprocessing as mp
    import torch
    assert not torch.cuda.is_initialized(), "pool_map must run before the GPU is initialised"
    with mp.get_context("fork").Pool(n) as p:
        return p.map(fn, items, chunksize=max(1, len(items) // (8 * n)))


def orc():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi
    oracle_ffi.lib()
    return oracle_ffi


def cpu_pool_run(fn, items, threads):
    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=threads) as ex:
        outs = list(ex.map(fn, items))
    return time.perf_counter() - t0, outs


def sample_size(per_item_s, threads, target_s, cap):
    return int(max(1, min(cap, round(target_s * threads / max(per_item_s, 1e-6)))))


class Cfg2:
    """ConsensusDWFA throughput (BASELINE configs[1], north-star 1,000-locus form)."""
    name = "cfg2"
    scaling = "weak"
    kernel = "wc::single_engine_kernel"

    def __init__(self, a, rank, world, ctx, pre=None):
        import waffle_con_amd as w
        from waffle_con_amd.cdwfa_config import CdwfaConfig
        self.a, self.ctx, self.rank, self.world = a, ctx, rank, world
        self.n = a.loci or 1000
        self.L, self.N, self.err = 10000, 100, 0.005
        self.cfg = CdwfaConfig(min_count=self.N // 4)
        from waffle_con_amd.shard import shard_seeds
        self.seeds = shard_seeds(self.n, rank)
        t0 = time.perf_counter()
        self.loci = gen_cfg2(self.seeds, self.L, self.N, self.err)
        self.gen_s = time.perf_counter() - t0
        t0 = time.perf_counter()
        self.batch = w.ResidentBatch(self.loci, context=ctx)
        self.upload_s = time.perf_counter() - t0
        self.last = None
        self._readb = sum(len(r) for p in self.loci for r in p)

    def read_bytes(self):
        """bytes of every read one step runs (each fetched from HBM at least once)"""
        return self._readb

    def step(self):
        res, st = self.batch.consensus(self.cfg, return_errors=True)
        bad = [r for r in res if isinstance(r, Exception)]
        if bad:
            raise RuntimeError("engine error: %s" % bad[0])
        self.last = res
        self.last_st = st
        return st, len(res)

    COUNTERS = ("updates", "w_out", "compares", "ed_increases", "finalizes", "pops", "nodes_explored")

    def extra(self):
        """One more (untimed) pass of the same launch with per-locus counters and
        completion times: where the launch's time goes (verdict r4 item 6) and
        the per-locus counters the CPU check compares (item 2)."""
        if self.name != "cfg2":
            return {}
        res, st = self.batch.consensus(self.cfg, return_errors=True, per_problem=True)
        pp = st["per_problem"]
        self._pp = pp
        self._pp_same = all([(c.sequence(), list(c.scores())) for c in res[i]] ==
                            [(c.sequence(), list(c.scores())) for c in self.last[i]] for i in range(len(res)))
        wall = sorted(p["wall_ms"] for p in pp)
        t100 = wall[-1]

        def q(f):
            return wall[min(len(wall) - 1, int(f * len(wall)))]
        # every locus of a cfg2 launch has its own workgroup from t = 0 (1,000 loci
        # <= 4 workgroups x 256 CUs), so a workgroup slot is busy until its
        # locus's completion: busy fraction = sum(wall) / (loci x t100)
        return {"cfg2_launch_profile": {
            "what": "per-locus completion times inside one 1,000-locus launch (wc_results_problem_stats wall_ms, "
                    "untimed pass after the timed steps)",
            "kernel_ms": st["kernel_ms"], "t50_ms": q(0.5), "t90_ms": q(0.9), "t95_ms": q(0.95), "t100_ms": t100,
            "workgroup_busy_frac": sum(wall) / (len(wall) * t100) if t100 > 0 else None,
            "slowest_loci": sorted(range(len(pp)), key=lambda i: -pp[i]["wall_ms"])[:5],
            "results_equal_timed_pass": self._pp_same}}

    def config(self):
        return {"workload": "ConsensusDWFA cfg2 throughput: %d loci/GPU x %d reads x %d bp @ %g error, min_count %d"
                            % (self.n, self.N, self.L, self.err, self.N // 4),
                "loci_per_gpu": self.n, "reads": self.N, "len": self.L, "error_rate": self.err,
                "parallelism": "loci-sharded x%d (no collective)" % self.world}

    def data(self):
        return "synthetic: generate_test(4, %d, %d, %g) seeds 0..%d (reference RNG restated)" % (
            self.L, self.N, self.err, self.n * self.world - 1)

    def e2e(self, steps):
        """Fresh batches every step: marshalling + pinned staging + H2D of batch
        k+1 (upload context, own thread) overlap the compute of batch k (compute
        context). Returns (loci/s, serial ms of one upload, serial ms of one compute)."""
        import waffle_con_amd as w
        up = self.ctx
        run = w.Context(self.ctx.device)
        bufs = [w.ResidentBatch(self.loci, context=up), w.ResidentBatch(self.loci, context=up)]
        t0 = time.perf_counter()
        bufs[0].refill(self.loci)
        up_ms = (time.perf_counter() - t0) * 1e3
        t0 = time.perf_counter()
        bufs[0].consensus(self.cfg, context=run)
        run_ms = (time.perf_counter() - t0) * 1e3
        ready = [threading.Event() for _ in range(steps)]
        free = [threading.Semaphore(1), threading.Semaphore(1)]
        err = []

        def uploader():
            try:
                for k in range(steps):
                    free[k % 2].acquire()
                    bufs[k % 2].refill(self.loci)
                    ready[k].set()
            except Exception as e:  # noqa: BLE001
                err.append(e)
                for ev in ready:
                    ev.set()

        t0 = time.perf_counter()
        th = threading.Thread(target=uploader)
        th.start()
        for k in range(steps):
            ready[k].wait()
            if err:
                break
            bufs[k % 2].consensus(self.cfg, context=run)
            free[k % 2].release()
        th.join()
        dt = time.perf_counter() - t0
        self.e2e_packed = up.last_upload_packed()
        if err:
            raise err[0]
        for b in bufs:
            b.close()
        run.close()
        return steps * self.n / dt, up_ms, run_ms

    def cpu(self, threads, target_s):
        o = orc()
        t0 = time.perf_counter()
        o.consensus(self.loci[0], min_count=self.N // 4)
        one = time.perf_counter() - t0
        n = sample_size(one, threads, target_s, len(self.loci))
        dt, outs = cpu_pool_run(lambda p: o.consensus(p, counters=True, min_count=self.N // 4), self.loci[:n], threads)
        upd = sum(c["updates"] for _, c in outs)
        ok = all([(c.sequence(), list(c.scores())) for c in self.last[i]] ==
                 [(r["sequence"], r["scores"]) for r in outs[i][0]] for i in range(n))
        out = {"value": upd / dt, "unit": "updates/s", "loci_per_s": n / dt,
               "sample": "%d loci of the same workload (seeds %d..%d), C++ oracle, one locus per thread, %.1f s wall"
                         % (n, self.seeds[0], self.seeds[0] + n - 1, dt),
               "gpu_matches_cpu_on_sample": ok, "checked": "sequences + per-read scores of every result"}
        # the search path, not only its answer: every work counter of every
        # sampled locus (a race that changes the path but not the result shows
        # here), from the per-locus pass; and the timed steps' totals when the
        # sample is the whole batch
        pp = getattr(self, "_pp", None)
        if pp is not None and self.name == "cfg2":
            bad = [i for i in range(n) if any(pp[i][k] != outs[i][1][k] for k in self.COUNTERS)]
            out["counters_match_on_sample"] = not bad and self._pp_same
            out["counters_checked"] = "%s of each of %d loci (per-locus pass), results of that pass = the timed " \
                                      "pass's" % ("/".join(self.COUNTERS), n)
            if bad:
                out["counter_mismatch_loci"] = bad[:10]
            if n == len(self.loci):
                out["timed_step_totals_match"] = all(
                    self.last_st[k] == sum(c[k] for _, c in outs) for k in self.COUNTERS)
        return out


class Cfg2Api(Cfg2):
    """The reference's per-locus API (SURVEY §8(b) "Threading": consensus(&self)
    is re-entrant, one instance per thread) from T native host threads, each
    calling ConsensusDWFA::consensus on its own cfg2 loci one at a time, as a
    Rust caller binding the C ABI would (tools/api_bench.cpp). The calls go
    through the device's submission service (wc_service_consensus: persistent
    launches shared by all callers). One step = every locus once. Reported
    beside the value: a thread sweep, the per-call-launch path (one
    wc_consensus_batch per call) at the same thread counts, and the batch path
    (wc_batch_consensus over all loci at once) on the same loci."""
    name = "cfg2-api"
    scaling = "weak"

    def __init__(self, a, rank, world, ctx, pre=None):
        import ctypes
        from waffle_con_amd import _lib
        from waffle_con_amd.consensus import _problems
        a.loci = a.loci or 1024
        super().__init__(a, rank, world, ctx, pre)
        self.threads = a.api_threads
        path = os.path.join(ROOT, "tools", "libapibench.so")
        if not os.path.exists(path):
            raise RuntimeError("tools/libapibench.so is missing: build it with `make -C tools`")
        self.H = ctypes.CDLL(path)
        self.H.api_bench_run.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
                                         ctypes.c_uint32, ctypes.POINTER(_lib.WcProblem),
                                         ctypes.POINTER(_lib.WcConfig), ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_lib.WcServiceStats)]
        self.arr, self.keep = _problems([(p, None) for p in self.loci])
        self.ccfg = _lib.make_config(self.cfg)
        self.lat = []

    def run(self, mode, threads, n=None):
        """n loci on `threads` native threads; returns (wall s, latencies ms, results, stats, service stats)."""
        import ctypes
        from waffle_con_amd import _lib
        from waffle_con_amd.consensus import _single_results, _stats
        n = n or self.n
        res = (ctypes.c_void_p * n)()
        lat = (ctypes.c_double * n)()
        wall = ctypes.c_double()
        sst = _lib.WcServiceStats()
        L = _lib.lib()
        rc = self.H.api_bench_run(_lib.LIB_PATH.encode(), self.ctx.device, mode, threads, 1, n, self.arr,
                                  ctypes.byref(self.ccfg), res, lat, ctypes.byref(wall), ctypes.byref(sst))
        if rc != 0:
            raise RuntimeError("api_bench_run failed (rc %d)" % rc)
        tot = {"kernel_ms": 0.0, "updates": 0, "w_out": 0, "compares": 0, "launches": 0, "row_bytes": 0}
        out = []
        for i in range(n):
            st = _stats(res[i], L)
            for k in ("updates", "w_out", "compares", "launches", "row_bytes"):
                tot[k] += st[k]
            tot["kernel_ms"] += st["kernel_ms"]
            out.append(_single_results(res[i], 1, self.cfg.consensus_cost, L, True)[0])
        return wall.value, list(lat), out, tot, sst.as_dict()

    def step(self):
        wall, lat, res, tot, sst = self.run(0, self.threads)
        bad = [r for r in res if isinstance(r, Exception)]
        if bad:
            raise RuntimeError("engine error: %s" % bad[0])
        self.last = res
        self.lat = lat
        self.svc = sst
        return tot, len(res)

    def extra(self):
        """Thread sweep (service and per-call launches) and the batch path on the
        same loci; every service result is checked against the batch path's."""
        def key(rs):
            return [[(c.sequence(), list(c.scores())) for c in r] for r in rs]
        batch_t0 = time.perf_counter()
        bres, _ = self.batch.consensus(self.cfg)
        batch_s = time.perf_counter() - batch_t0
        same = key(self.last) == key(bres)
        out = {"api_threads": self.threads, "api_matches_batch_path": same,
               "api_latency_ms_median": statistics.median(self.lat),
               "api_latency_ms_p90": sorted(self.lat)[int(0.9 * (len(self.lat) - 1))],
               "api_service_stats": self.svc,
               "batch_path_loci_per_s": self.n / batch_s}
        sweep = {}
        for t in sorted({16, 64, 256, self.threads}):
            w, _, r, _, _ = self.run(0, t)
            sweep[str(t)] = self.n / w
            out["api_matches_batch_path"] &= key(r) == key(bres)
        out["api_service_loci_per_s_by_threads"] = sweep
        per_call = {}
        for t in (16, 64):
            n = min(self.n, 256)
            w, _, r, _, _ = self.run(1, t, n)
            per_call[str(t)] = n / w
        out["api_per_call_launch_loci_per_s_by_threads"] = per_call
        return out

    def config(self):
        c = super().config()
        c["workload"] = ("ConsensusDWFA cfg2 through the reference's per-locus API: %d loci/GPU x %d reads x %d bp "
                         "@ %g error, min_count %d, %d native caller threads, one locus per call"
                         % (self.n, self.N, self.L, self.err, self.N // 4, self.threads))
        c["api_threads"] = self.threads
        return c

    def e2e(self, steps):
        return None


class Cfg2Latency(Cfg2):
    """One cfg2 locus per launch (single-locus configs, 1 CPU thread)."""
    name = "cfg2-latency"
    scaling = "weak"

    def __init__(self, a, rank, world, ctx, pre=None):
        a.loci = 1
        super().__init__(a, rank, world, ctx, pre)

    def config(self):
        c = super().config()
        c["workload"] = "ConsensusDWFA cfg2 single locus: %d reads x %d bp @ %g error, min_count %d (latency)" % (
            self.N, self.L, self.err, self.N // 4)
        return c

    def e2e(self, steps):
        return None

    def cpu(self, threads, target_s):
        r = super().cpu(1, target_s)
        r["cores"] = 1
        return r


class Cfg3(Cfg2):
    """DualConsensusDWFA on cfg3 loci (BASELINE configs[2])."""
    name = "cfg3"
    kernel = "wc::dual_engine_kernel"

    def __init__(self, a, rank, world, ctx, pre=None):
        import waffle_con_amd as w
        from waffle_con_amd import synth
        from waffle_con_amd.cdwfa_config import CdwfaConfig
        self.a, self.ctx, self.rank, self.world = a, ctx, rank, world
        self.n = a.loci or 768
        self.cfg = CdwfaConfig()
        self.seeds = list(range(rank * self.n, (rank + 1) * self.n))
        t0 = time.perf_counter()
        with ThreadPoolExecutor(max_workers=_threads()) as ex:
            self.loci = list(ex.map(synth.cfg3_locus, self.seeds))
        self.gen_s = time.perf_counter() - t0
        t0 = time.perf_counter()
        self.batch = w.ResidentBatch(self.loci, context=ctx)
        self.upload_s = time.perf_counter() - t0
        self._readb = sum(len(r) for p in self.loci for r in p)

    def step(self):
        res, st = self.batch.dual_consensus(self.cfg, return_errors=True)
        bad = [r for r in res if isinstance(r, Exception)]
        if bad:
            raise RuntimeError("engine error: %s" % bad[0])
        self.last = res
        return st, len(res)

    def config(self):
        return {"workload": "DualConsensusDWFA cfg3: %d loci/GPU, 5 kb haplotypes A/B (12 SNVs + 2 indels), "
                            "2 x 100 reads @ 0.5%%, default config" % self.n,
                "loci_per_gpu": self.n, "parallelism": "loci-sharded x%d (no collective)" % self.world}

    def data(self):
        return "synthetic: synth.cfg3_locus(seed) seeds %d..%d" % (0, self.n * self.world - 1)

    def e2e(self, steps):
        return None

    def cpu(self, threads, target_s):
        o = orc()
        t0 = time.perf_counter()
        o.dual_consensus(self.loci[0])
        one = time.perf_counter() - t0
        n = sample_size(one, threads, target_s, len(self.loci))
        dt, outs = cpu_pool_run(lambda p: o.dual_consensus(p, counters=True), self.loci[:n], threads)
        upd = sum(c["updates"] for _, c in outs)

        def norm(rs):
            return [(r.consensus1().sequence(), r.consensus2().sequence() if r.consensus2() else None,
                     list(r.is_consensus1()), list(r.scores1()), list(r.scores2())) for r in rs]
        ok = all(norm(self.last[i]) == [(r["consensus1"]["sequence"],
                                         r["consensus2"]["sequence"] if r["consensus2"] else None,
                                         r["is_consensus1"], r["scores1"], r["scores2"]) for r in outs[i][0]]
                 for i in range(n))
        return {"value": upd / dt, "unit": "updates/s", "loci_per_s": n / dt,
                "sample": "%d cfg3 loci, C++ oracle, one locus per thread, %.1f s wall" % (n, dt),
                "gpu_matches_cpu_on_sample": ok}


CFG5_FAMILY = "PriorityConsensusDWFA cfg5: fixed batch of "


class Cfg5:
    """PriorityConsensusDWFA over a fixed batch of cfg5 loci, strong-scaled:
    the heavy prefix of the cost-sorted order (75% of the estimated cost) is
    split statically by LPT, the light tail is pulled in chunks through a
    store-backed shared queue by whichever rank runs out of work first
    (shard.prefix_tail_plan / SharedQueue; no collective on the data path)."""
    name = "cfg5"
    scaling = "strong"
    kernel = "wcw::dual_wave2_kernel"

    @staticmethod
    def pregen(a, rank, world, total=None):
        """Plan and loci of this rank (its static prefix and every tail locus it
        may pull), generated before the GPU is touched (forked workers)."""
        from waffle_con_amd import shard, synth
        total = total or a.loci or 10000
        t0 = time.perf_counter()
        costs = [synth.cfg5_cost(s) for s in range(total)]
        # one GPU runs everything in one call (the scheduler publishes largest
        # first); several split the heavy 85% of the cost statically and share
        # the light tail
        static, tail = shard.prefix_tail_plan(costs, world, 1.0 if world == 1 else 0.85)
        ids = static[rank] + tail
        loci = dict(zip(ids, pool_map(synth.cfg5_locus, ids)))
        return {"total": total, "static": static[rank], "tail": tail, "loci": loci, "costs": costs,
                "gen_s": time.perf_counter() - t0}

    def __init__(self, a, rank, world, ctx, pre=None):
        from waffle_con_amd import shard
        from waffle_con_amd.cdwfa_config import CdwfaConfig
        self.a, self.ctx, self.rank, self.world = a, ctx, rank, world
        pre = pre or self.pregen(a, rank, world)
        self.total = pre["total"]
        self.static, self.tail, self.L = pre["static"], pre["tail"], pre["loci"]
        # tail chunks large enough to fill the GPU, about four per rank
        self.chunk = max(256, -(-len(self.tail) // (4 * world)))
        self.costs = pre["costs"]
        self.cfg = CdwfaConfig(wildcard=ord("*"))
        self.gen_s = pre["gen_s"]
        self.upload_s = 0.0
        self.n = self.total
        self.k = 0
        if world > 1:
            import torch.distributed as dist
            self.store = dist.distributed_c10d._get_default_store()
        else:
            self.store = shard.LocalStore()
        self.last, self.mine, self.busy_s, self.static_s = {}, [], 0.0, 0.0
        self.t0, self.done, self.lat, self.dlat = 0.0, {}, {}, {}

    def _run(self, ids):
        """One priority_consensus_batch call over loci `ids`; records each
        locus's completion time (from the step's start: done) and its latency
        inside the call (from the call's start: lat)."""
        import waffle_con_amd as w
        t_call = time.perf_counter()
        res, st = w.priority_consensus_batch([(self.L[i], None, None) for i in ids], self.cfg, context=self.ctx,
                                             return_errors=True, per_problem=True)
        bad = [r for r in res if isinstance(r, Exception)]
        if bad:
            raise RuntimeError("engine error: %s" % bad[0])
        self.last.update(zip(ids, res))
        for i, pp in zip(ids, st.pop("per_problem")):
            self.lat[i] = pp["wall_ms"] / 1e3
            # on the device: from its first sub-problem's publication (a
            # locus that waited to be published is not slow for that)
            self.dlat[i] = (pp["wall_ms"] - pp.get("start_ms", 0.0)) / 1e3
            self.done[i] = t_call - self.t0 + self.lat[i]
        return st

    def read_bytes(self):
        return sum(len(x) for i in self.mine for ch in self.L[i] for x in ch)

    def step(self):
        from waffle_con_amd import shard
        self.k += 1
        q = shard.SharedQueue(self.store, len(self.tail), self.chunk, key="wc_cfg5_%d" % self.k)
        self.last, self.mine, self.done, self.lat, self.dlat = {}, list(self.static), {}, {}, {}
        t0 = self.t0 = time.perf_counter()
        tot = self._run(self.static)
        self.static_s = time.perf_counter() - t0
        keys = ("kernel_ms", "updates", "w_out", "compares", "launches", "row_bytes")
        while True:
            c = q.next_chunk()
            if c is None:
                break
            ids = self.tail[c[0]:c[1]]
            st = self._run(ids)
            for k in keys:
                tot[k] += st[k]
            self.mine += ids
        self.busy_s = time.perf_counter() - t0
        return tot, len(self.mine)

    def config(self):
        return {"workload": "PriorityConsensusDWFA cfg5: fixed batch of %d PGx loci (1-6 kb, 2 haplotypes, 15-40 reads "
                            "each @ 0.5%%, [HPC(read), read] chains, wildcard '*'), LPT prefix + shared-queue tail "
                            "over %d GPU(s)" % (self.total, self.world),
                "loci_total": self.total, "loci_this_rank": len(self.mine),
                "parallelism": "loci-sharded x%d, cost-sorted LPT prefix + store-backed shared queue (no collective)"
                               % self.world}

    def data(self):
        return "synthetic: synth.cfg5_locus(seed) seeds 0..%d" % (self.total - 1)

    def e2e(self, steps):
        return None

    def rank_report(self, dist, device):
        """Per-rank busy time, static-prefix time and loci of the last step (every rank calls this)."""
        vals = [self.busy_s, self.static_s, float(len(self.mine)), float(sum(self.costs[i] for i in self.mine))]
        if dist is None:
            rows = [vals]
        else:
            import torch
            t = torch.zeros(self.world, len(vals), dtype=torch.float64, device=device)
            t[self.rank] = torch.tensor(vals, dtype=torch.float64, device=device)
            dist.all_reduce(t)
            rows = t.tolist()
        busy = [r[0] for r in rows]
        return {"rank_busy_s": busy, "rank_static_s": [r[1] for r in rows], "rank_loci": [int(r[2]) for r in rows],
                "rank_cost_share": [r[3] / max(1.0, float(sum(self.costs))) for r in rows],
                "busy_max_s": max(busy), "busy_min_s": min(busy), "tail_s": max(busy) - min(busy),
                "prefix_loci": None if dist is not None else len(self.static), "tail_loci": len(self.tail),
                "chunk": self.chunk}

    def tail_report(self, dist):
        """Completion-time quantiles over every locus of the batch (all ranks;
        seconds from the leg's start) and the heaviest locus (largest cost)
        under load: its latency inside its call and when it finished."""
        import math
        h = max(range(self.total), key=lambda i: (self.costs[i], -i))
        mine = {"done": [self.done[i] for i in self.mine],
                "slowest": max(((self.dlat.get(i, self.lat[i]), i) for i in self.mine), default=(0.0, -1)),
                "slow2": sorted(((self.dlat.get(i, self.lat[i]), i) for i in self.mine), reverse=True)[:2],
                "slowest_call": max(((self.lat[i], i) for i in self.mine), default=(0.0, -1)),
                "heaviest": (self.lat[h], self.done[h]) if h in self.lat else None}
        if dist is None:
            rows = [mine]
        else:
            rows = [None] * self.world
            dist.all_gather_object(rows, mine)
        done = sorted(d for r in rows for d in r["done"])

        def q(f):
            return done[min(len(done) - 1, max(0, int(math.ceil(f * len(done))) - 1))] if done else None
        hv = next((r["heaviest"] for r in rows if r["heaviest"] is not None), (None, None))
        slow = max(r["slowest"] for r in rows)
        slow_call = max(r["slowest_call"] for r in rows)
        slow2 = sorted((x for r in rows for x in r["slow2"]), reverse=True)[:2]
        return {"t50_s": q(0.50), "t95_s": q(0.95), "t100_s": q(1.0),
                "heaviest_locus": h, "heaviest_cost": self.costs[h],
                "heaviest_latency_under_load_s": hv[0], "heaviest_done_s": hv[1],
                "slowest_device_latency_s": slow[0], "slowest_locus": slow[1],
                "slowest_two_loci": [x[1] for x in slow2],
                "slowest_note": "slowest_device_latency_s / slowest_locus: latency on the device, from the first "
                                "publication of the locus's first sub-problem to its result (wc_stats start_ms / "
                                "wall_ms); slowest_latency_under_load_s: the largest latency inside the call (from "
                                "the call's start, queueing included: the meaning this key had before round 5)",
                "slowest_latency_under_load_s": slow_call[0], "slowest_call_locus": slow_call[1]}

    def heaviest_alone(self, h):
        """The heaviest locus alone on the GPU (one call, nothing else queued): s."""
        t0 = time.perf_counter()
        self._run([h])
        return time.perf_counter() - t0

    def cpu(self, threads, target_s):
        o = orc()
        mine = self.mine
        # this rank's loci in queue order (heaviest first): estimate the mean
        # per-locus time from a few loci spread over that order, sample evenly
        probe = [mine[int(k * len(mine) / 4)] for k in range(4)]
        t0 = time.perf_counter()
        cpu_pool_run(lambda i: o.priority_consensus(self.L[i], wildcard=ord("*")), probe, min(4, threads))
        one = (time.perf_counter() - t0) * min(4, threads) / len(probe)
        n = sample_size(one, threads, target_s, len(mine))
        idx = [mine[int(k * len(mine) / n)] for k in range(n)]
        dt, outs = cpu_pool_run(lambda i: o.priority_consensus(self.L[i], counters=True, wildcard=ord("*")), idx,
                                threads)
        upd = sum(c["updates"] for _, c in outs)
        ok = all([[c.sequence() for c in ch] for ch in self.last[i].consensuses()] ==
                 [[c["sequence"] for c in ch] for ch in outs[k][0]["consensuses"]] and
                 list(self.last[i].sequence_indices()) == list(outs[k][0]["sequence_indices"])
                 for k, i in enumerate(idx))
        return {"value": upd / dt, "unit": "updates/s", "loci_per_s": n / dt,
                "sample": "%d of the rank's cfg5 loci spread over the cost order, C++ oracle, %.1f s wall" % (n, dt),
                "gpu_matches_cpu_on_sample": ok}


class Cfg4(Cfg5):
    """PriorityConsensusDWFA on one cfg4 locus (BASELINE configs[3])."""
    name = "cfg4"
    scaling = "weak"

    @staticmethod
    def pregen(a, rank, world, total=None):
        return None

    def __init__(self, a, rank, world, ctx, pre=None):
        from waffle_con_amd import synth
        from waffle_con_amd.cdwfa_config import CdwfaConfig
        self.a, self.ctx, self.rank, self.world = a, ctx, rank, world
        self.total = self.n = 1
        self.cfg = CdwfaConfig(wildcard=ord("*"))
        t0 = time.perf_counter()
        self.L = {0: [[r] for r in synth.cfg4_locus(4 + rank)]}
        self.static, self.tail, self.costs = [0], [], [1]
        self.chunk = 0  # (rank_report: no shared queue for one locus)
        self.gen_s = time.perf_counter() - t0
        self.upload_s = 0.0
        self.last, self.mine, self.busy_s, self.static_s = {}, [], 0.0, 0.0
        self.t0, self.done, self.lat, self.dlat = 0.0, {}, {}, {}

    def step(self):
        self.last, self.mine, self.done, self.lat, self.dlat = {}, [0], {}, {}, {}
        t0 = self.t0 = time.perf_counter()
        st = self._run([0])
        self.busy_s = self.static_s = time.perf_counter() - t0
        return st, 1

    def cpu(self, threads, target_s):
        """The C++ oracle on the same locus, one thread (about two minutes),
        checked against the GPU's result."""
        o = orc()
        t0 = time.perf_counter()
        res, c = o.priority_consensus(self.L[0], counters=True, wildcard=ord("*"))
        dt = time.perf_counter() - t0
        g = self.last[0]
        ok = ([[x.sequence() for x in ch] for ch in g.consensuses()] ==
              [[x["sequence"] for x in ch] for ch in res["consensuses"]] and
              list(g.sequence_indices()) == list(res["sequence_indices"]))
        return {"value": c["updates"] / dt, "unit": "updates/s", "loci_per_s": 1.0 / dt, "seconds": dt, "cores": 1,
                "sample": "the whole cfg4 locus, C++ oracle, one thread, %.1f s" % dt,
                "gpu_matches_cpu_on_sample": ok}

    def config(self):
        return {"workload": "PriorityConsensusDWFA cfg4: one locus, 4 haplotypes x 50 reads x 8 kb, inserted "
                            "segments {0, 25, 60, 150} bp + 3 SNVs each, 0.5% error, wildcard '*'",
                "loci_per_gpu": 1, "parallelism": "replicas x%d" % self.world}

    def data(self):
        return "synthetic: synth.cfg4_locus(4 + rank)"


class Cfg5Api:
    """PriorityConsensusDWFA::consensus through the reference's per-locus API
    (priority_consensus.rs:172, `&self`, one instance per thread: the PGx
    caller pattern behind cfg5) from T native host threads, each calling it on
    its own cfg5 loci one at a time (tools/api_bench.cpp api_bench_priority_run
    -> wc_service_priority_consensus: every caller unwinds its own LIFO stack,
    all sub-problems share the service's persistent launches). One step =
    every locus once. Reported beside the value: a thread sweep, per-call
    launches (one wc_priority_consensus_batch per call) at 16 and 64 threads,
    and the batch path (wc_priority_consensus_batch over all loci at once) on
    the same loci; every API result is checked against the batch path's."""
    name = "cfg5-api"
    scaling = "weak"
    kernel = "wcw::dual_wave2_kernel"

    @staticmethod
    def pregen(a, rank, world, total=None):
        from waffle_con_amd import synth
        n = a.loci or 512
        ids = list(range(rank * n, (rank + 1) * n))
        t0 = time.perf_counter()
        loci = pool_map(synth.cfg5_locus, ids)
        return {"ids": ids, "loci": loci, "gen_s": time.perf_counter() - t0}

    def __init__(self, a, rank, world, ctx, pre=None):
        import ctypes
        from waffle_con_amd import _lib
        from waffle_con_amd.cdwfa_config import CdwfaConfig
        from waffle_con_amd.priority_consensus import _chain_problems
        self.a, self.ctx, self.rank, self.world = a, ctx, rank, world
        pre = pre or self.pregen(a, rank, world)
        self.ids, self.L, self.gen_s = pre["ids"], pre["loci"], pre["gen_s"]
        self.n = len(self.L)
        self.upload_s = 0.0
        self.threads = a.api_threads
        self.cfg = CdwfaConfig(wildcard=ord("*"))
        path = os.path.join(ROOT, "tools", "libapibench.so")
        if not os.path.exists(path):
            raise RuntimeError("tools/libapibench.so is missing: build it with `make -C tools`")
        self.H = ctypes.CDLL(path)
        self.H.api_bench_priority_run.argtypes = [
            ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
            ctypes.POINTER(_lib.WcChainProblem), ctypes.POINTER(_lib.WcConfig), ctypes.c_void_p, ctypes.c_void_p,
            ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_lib.WcServiceStats)]
        self.arr, self.keep = _chain_problems([(ch, None, None) for ch in self.L])
        self.ccfg = _lib.make_config(self.cfg)
        self.last, self.lat, self.svc = None, [], {}
        self._readb = sum(len(x) for ch in self.L for c in ch for x in c)

    def read_bytes(self):
        return self._readb

    def run(self, mode, threads, n=None):
        """n loci on `threads` native threads: (wall s, latencies ms, results, summed stats, service stats)."""
        import ctypes
        from waffle_con_amd import _lib
        from waffle_con_amd.consensus import _stats
        from waffle_con_amd.priority_consensus import _priority_results
        n = n or self.n
        res = (ctypes.c_void_p * n)()
        lat = (ctypes.c_double * n)()
        wall = ctypes.c_double()
        sst = _lib.WcServiceStats()
        L = _lib.lib()
        rc = self.H.api_bench_priority_run(_lib.LIB_PATH.encode(), self.ctx.device, mode, threads, n, self.arr,
                                           ctypes.byref(self.ccfg), res, lat, ctypes.byref(wall), ctypes.byref(sst))
        if rc != 0:
            raise RuntimeError("api_bench_priority_run failed (rc %d)" % rc)
        tot = {"kernel_ms": 0.0, "updates": 0, "w_out": 0, "compares": 0, "launches": 0, "row_bytes": 0}
        out = []
        try:
            for i in range(n):
                st = _stats(res[i], L)
                for k in ("updates", "w_out", "compares", "launches", "row_bytes"):
                    tot[k] += st[k]
                tot["kernel_ms"] += st["kernel_ms"]
                out.append(_priority_results(res[i], 1, self.cfg, L, True)[0])
        finally:
            for i in range(n):
                if res[i]:
                    L.wc_results_free(res[i])
        return wall.value, list(lat), out, tot, sst.as_dict()

    def step(self):
        wall, lat, res, tot, sst = self.run(0, self.threads)
        bad = [r for r in res if isinstance(r, Exception)]
        if bad:
            raise RuntimeError("engine error: %s" % bad[0])
        self.last, self.lat, self.svc = res, lat, sst
        return tot, len(res)

    def extra(self):
        """The batch path on the same loci, a thread sweep of the service path
        (16 threads on the first 128 loci: a caller with T threads is bound by
        T / latency) and per-call launches (first 64 loci)."""
        import waffle_con_amd as w

        def note(msg):
            print("[bench cfg5-api] %s" % msg, file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        bres, _ = w.priority_consensus_batch([(ch, None, None) for ch in self.L], self.cfg, context=self.ctx)
        batch_s = time.perf_counter() - t0
        note("batch path: %.1f s" % batch_s)
        out = {"api_threads": self.threads, "api_matches_batch_path": self.last == bres,
               "api_latency_ms_median": statistics.median(self.lat),
               "api_latency_ms_p90": sorted(self.lat)[int(0.9 * (len(self.lat) - 1))],
               "api_latency_ms_max": max(self.lat),
               "api_service_stats": self.svc, "batch_path_loci_per_s": self.n / batch_s}
        sweep = {}
        for t in sorted({16, 64, 256, self.threads}):
            n = min(self.n, 128) if t <= 16 else self.n
            wt, _, r, _, _ = self.run(0, t, n)
            sweep[str(t)] = n / wt
            out["api_matches_batch_path"] &= r == bres[:n]
            note("service path, %d threads: %.1f loci/s" % (t, n / wt))
        out["api_service_loci_per_s_by_threads"] = sweep
        per_call = {}
        for t in (16, 64):
            n = min(self.n, 64)
            wt, _, r, _, _ = self.run(1, t, n)
            per_call[str(t)] = n / wt
            out["api_matches_batch_path"] &= r == bres[:n]
            note("per-call launches, %d threads: %.1f loci/s" % (t, n / wt))
        out["api_per_call_launch_loci_per_s_by_threads"] = per_call
        return out

    def config(self):
        return {"workload": "PriorityConsensusDWFA cfg5 through the reference's per-locus API: %d PGx loci/GPU "
                            "(1-6 kb, 2 haplotypes, 15-40 reads each @ 0.5%%, [HPC(read), read] chains, wildcard "
                            "'*'), %d native caller threads, one locus per call" % (self.n, self.threads),
                "loci_per_gpu": self.n, "api_threads": self.threads,
                "parallelism": "loci-sharded x%d (no collective)" % self.world}

    def data(self):
        return "synthetic: synth.cfg5_locus(seed) seeds %d..%d" % (self.ids[0], self.ids[-1])

    def e2e(self, steps):
        return None

    def cpu(self, threads, target_s):
        return None  # the cfg5 CPU baseline is in the default line's cfg5_strong leg (same loci generator)


WORKLOADS = {"cfg2": Cfg2, "cfg2-api": Cfg2Api, "cfg2-latency": Cfg2Latency, "cfg3": Cfg3, "cfg4": Cfg4,
             "cfg5": Cfg5, "cfg5-api": Cfg5Api}


# ---------------------------------------------------------------------------
# roofline / profile records committed under profiles/
# ---------------------------------------------------------------------------
def profile_record(kind, workload_cfg, kernel, family=None):
    """Latest committed PMC summary (profiles/r*_<kind>.json) recorded on this
    kernel (exact name: a record of another build's kernel, or one that does
    not name its kernel, does not describe this one) and on this workload, or,
    with `family`, on any workload whose description starts with it (the same
    generator at another batch size: only the record's size-independent
    ratios apply then)."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_%s.json" % kind)), reverse=True):
        with open(path) as f:
            rec = json.load(f)
        wl = rec.get("workload") or ""
        if rec.get("kernel") != kernel:
            continue
        if wl == workload_cfg or (family is not None and wl.startswith(family)):
            rec["_file"] = os.path.relpath(path, ROOT)
            return rec
    return None


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_workers(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world:
        print("bench.py: --gpus %d but WORLD_SIZE %d" % (a.gpus, world), file=sys.stderr)
        sys.exit(2)
    # large inputs are generated by forked workers before anything touches the GPU
    cls = WORKLOADS[a.workload]
    pre = cls.pregen(a, rank, world) if hasattr(cls, "pregen") else None
    leg_pre = Cfg5.pregen(a, rank, world, total=a.cfg5_loci) if (a.workload == "cfg2" and a.cfg5_loci) else None
    # torch ships its own HIP runtime next to the one the library links: torch
    # must initialise the device first, or its later init finds no GPU
    import torch
    # WC_BENCH_SHARE_GPU=1: a rehearsal of the N-rank path on a box with fewer
    # GPUs (ranks share devices round-robin, gloo for the barrier and the
    # reductions); the line says so and is not a scaling measurement
    share = world > 1 and os.environ.get("WC_BENCH_SHARE_GPU") == "1"
    device_index = local_rank % max(1, torch.cuda.device_count()) if share else local_rank
    if share:
        # co-tenants: every rank's launches are planned for its share of the
        # device's CUs and HBM (the library reads this when its context is made)
        per_dev = -(-world // max(1, torch.cuda.device_count()))
        os.environ.setdefault("WC_DEVICE_SHARE", str(per_dev))
    torch.cuda.init()
    torch.cuda.set_device(device_index)
    dist = None
    rdev = None  # device of the reduction tensors
    if world > 1:
        import torch.distributed as dist
        if share:
            dist.init_process_group("gloo")
            rdev = "cpu"
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
            rdev = "cuda"

    import waffle_con_amd as w
    from waffle_con_amd import shard

    ctx = w.Context(device_index)

    def note(msg):  # progress on stderr (long workloads must not look hung)
        print("[bench rank %d] %s" % (rank, msg), file=sys.stderr, flush=True)

    note("generating %s" % a.workload)
    W = cls(a, rank, world, ctx, pre)
    note("generated in %.1f s; warmup" % W.gen_s)

    def sync():
        torch.cuda.synchronize()

    for _ in range(a.warmup):
        W.step()
    # the setup leaves a large Python heap: move it to the permanent generation
    # so a full collection inside the timed region does not traverse it
    gc.collect()
    gc.freeze()
    note("timed steps")
    kernel_ms, upd, wout, cmp, loci, launches, rowb, readb = 0.0, 0, 0, 0, 0, 0, 0, 0
    step_ms = []
    with shard.Timer(dist, sync) as tm:
        for _ in range(a.steps):
            t0 = time.perf_counter()
            st, nl = W.step()
            step_ms.append((time.perf_counter() - t0) * 1e3)
            kernel_ms += st["kernel_ms"]
            upd += st["updates"]
            wout += st["w_out"]
            cmp += st["compares"]
            launches += st["launches"]
            rowb += st["row_bytes"]
            readb += W.read_bytes()
            loci += nl
    elapsed, total_upd, total_loci = shard.reduce_run(
        dist, tm.elapsed, upd, loci, device=rdev)

    note("timed region done: %.2f s" % tm.elapsed)
    e2e = None
    if world == 1 and not a.no_e2e:
        # (8 batches at least: the first upload is not overlapped, and a
        # shorter pipeline measures its fill more than its steady state)
        e2e_steps = max(8, a.steps)
        e2e = W.e2e(e2e_steps)
    # cfg5 strong-scaling leg of the default line (the fixed
    # 10,000-locus PriorityConsensusDWFA batch the 8-GPU target is quoted on):
    # one pass, barrier + device sync on both sides, max over ranks
    cfg5_leg = None
    if leg_pre is not None:
        note("cfg5 strong-scaling leg: %d loci (untimed warm-up pass)" % a.cfg5_loci)
        C5 = Cfg5(a, rank, world, ctx, leg_pre)
        C5.step()  # warm-up: first-pass allocations and planning stay out of the timed pass
        note("cfg5 leg: timed pass")
        with shard.Timer(dist, sync) as tm5:
            st5, n5 = C5.step()
        el5, upd5, loci5 = shard.reduce_run(dist, tm5.elapsed, st5["updates"], n5,
                                            device=rdev)
        rep = C5.rank_report(dist, rdev)
        tail = C5.tail_report(dist)
        cfg5_leg = {"workload": C5.config()["workload"], "loci": int(loci5), "elapsed_s": el5,
                    "cfg5_loci_per_s": loci5 / el5, "cfg5_updates_per_s": upd5 / el5, "gen_s": C5.gen_s,
                    "scaling": "strong", "n_gpus": world, "warmup": "one untimed pass of the same batch",
                    "tail": tail}
        cfg5_leg.update(rep)
        # roofline of this rank's engine launches (the dual engine): the
        # compulsory-byte model (read bytes once + row bytes) over their kernel
        # time, with the committed PMC profile of the same workload beside it
        kms5 = st5["kernel_ms"]
        model5 = C5.read_bytes() + st5["row_bytes"]
        rl5 = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "kernel": Cfg5.kernel,
               "achieved": model5 / (kms5 / 1e3) / 1e9 if kms5 > 0 else None, "frac": None,
               "model": "compulsory bytes: read bytes (each once) + wavefront-row bytes (engine row_bytes)",
               "model_bytes": model5, "kernel_ms": kms5, "launches": st5["launches"],
               "note": "rank 0's launches; kernel_ms sums the stream epochs' HIP-event times"}
        if rl5["achieved"] is not None:
            rl5["frac"] = rl5["achieved"] / HBM_PEAK_GBS
        # the PMC passes cannot run the whole 10,000-locus batch within the
        # profiler's limits: the record is of a smaller batch of the same
        # generator (its workload names the count), so only its intensive
        # figures (HBM rate, traffic over the compulsory model) are carried
        pmc5 = profile_record("pmc_traffic", C5.config()["workload"], Cfg5.kernel, family=CFG5_FAMILY)
        if pmc5:
            rl5["pmc_workload"] = pmc5["workload"]
            rl5["pmc_traffic_bytes_per_launch"] = pmc5["traffic_bytes_per_launch"]
            rl5["pmc_kernel_ms_per_launch"] = pmc5.get("kernel_ms_per_launch_bench_events")
            if rl5["pmc_kernel_ms_per_launch"]:
                rl5["pmc_achieved"] = pmc5["traffic_bytes_per_launch"] / (rl5["pmc_kernel_ms_per_launch"] / 1e3) / 1e9
                rl5["pmc_frac"] = rl5["pmc_achieved"] / HBM_PEAK_GBS
            if pmc5.get("model_bytes_per_launch"):
                rl5["traffic_over_model"] = pmc5["traffic_bytes_per_launch"] / pmc5["model_bytes_per_launch"]
            rl5["pmc_source"] = pmc5["_file"]
        iv5 = profile_record("issue_view", C5.config()["workload"], Cfg5.kernel, family=CFG5_FAMILY)
        if iv5:
            rl5["issue_view"] = {k: v for k, v in iv5.items() if not k.startswith("_")}
            rl5["issue_view"]["source"] = iv5["_file"]
        cfg5_leg["roofline"] = rl5
        if rank == 0 and tail["heaviest_latency_under_load_s"] is not None:
            cfg5_leg["tail"]["heaviest_latency_alone_s"] = C5.heaviest_alone(tail["heaviest_locus"])
        if rank == 0 and world == 1 and tail["slowest_locus"] is not None and tail["slowest_locus"] >= 0:
            # the critical path a larger GPU count cannot shorten: the slowest
            # locus of the batch, alone; 8 GPUs cannot finish the batch before
            # it, so t_1gpu / (8 x that) bounds the 8-GPU efficiency
            # (the two slowest on the device, each alone: the slowest under
            # load need not be the slowest alone)
            alones = {i: C5.heaviest_alone(i) for i in tail.get("slowest_two_loci") or [tail["slowest_locus"]]}
            alone = alones.get(tail["slowest_locus"], max(alones.values()))
            cfg5_leg["tail"]["slowest_latency_alone_s"] = alone
            cfg5_leg["tail"]["slowest_two_alone_s"] = {str(k): v for k, v in alones.items()}
            crit = max(max(alones.values()), cfg5_leg["tail"].get("heaviest_latency_alone_s") or 0.0)
            cfg5_leg["tail"]["projected_8gpu_eff"] = min(1.0, el5 / (8.0 * crit)) if crit > 0 else None
        if rank == 0 and not a.no_cpu:
            # bounded oracle check of sampled loci (and, at N=1, the CPU baseline)
            cores, aff, quota = usable_cpus()
            threads = a.cpu_threads or cores
            cb = C5.cpu(threads, a.cpu_seconds if world == 1 else 3.0)
            cfg5_leg["gpu_matches_cpu_on_sample"] = cb["gpu_matches_cpu_on_sample"]
            cfg5_leg["check_sample"] = cb["sample"]
            if world == 1:
                cb.update({"cores": threads, "kind": "port", "cpu_model": cpu_model(), "affinity_cpus": aff,
                           "cgroup_quota_cpus": quota})
                cfg5_leg["cpu_baseline"] = cb
                cfg5_leg["gpu_vs_cpu_loci"] = cfg5_leg["cfg5_loci_per_s"] / cb["loci_per_s"]
        note("cfg5 leg done: %.2f s" % el5)

    w_ranks = W.rank_report(dist, rdev) if hasattr(W, "rank_report") else None

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    cfgd = W.config()
    avg_kernel_s = kernel_ms / a.steps / 1e3
    ref_bytes = (8.0 * wout + 2.0 * cmp) / a.steps  # SURVEY §8(d) B_upd summed, per step
    fam = CFG5_FAMILY if W.name in ("cfg5",) else None
    pmc = profile_record("pmc_traffic", cfgd["workload"], W.kernel, family=fam)
    pmc_same = pmc is not None and pmc.get("workload") == cfgd["workload"]
    # (per-launch bytes only from a record of this very workload)
    traffic = pmc.get("traffic_bytes_per_launch") if pmc_same else None
    launches_per_step = launches / a.steps
    per_launch_s = avg_kernel_s / max(launches_per_step, 1)
    # The roofline model: the HBM bytes this search cannot avoid
    # moving in one launch, counted by the engine: every read byte once (the
    # reads are in HBM when the launch starts) plus the wavefront rows that an
    # update growing an edit distance reads and writes whole (row_bytes,
    # u32 entries; rows live in HBM), a finalize reads. Any launch of this
    # algorithm moves at least these bytes, so achieved <= peak by construction.
    model_bytes = (readb + rowb) / a.steps / max(launches_per_step, 1)
    roofline = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "kernel": W.kernel,
                "achieved": model_bytes / per_launch_s / 1e9 if per_launch_s > 0 else None,
                "frac": None, "traffic": traffic,
                "model": "compulsory bytes per launch: read bytes (each once) + wavefront-row bytes of the "
                         "updates/finalizes that grow an edit distance (engine row_bytes counter)",
                "model_bytes_per_launch": model_bytes,
                "read_bytes_per_launch": readb / a.steps / max(launches_per_step, 1),
                "row_bytes_per_launch": rowb / a.steps / max(launches_per_step, 1),
                "kernel_ms_per_launch": per_launch_s * 1e3,
                "reference_equiv_bytes_per_step": ref_bytes,
                "reference_equiv_gbs": ref_bytes / avg_kernel_s / 1e9 if avg_kernel_s > 0 else None,
                "note": "achieved/frac: the compulsory-byte model over the HIP-event kernel time (a lower bound "
                        "on the kernel's HBM traffic). pmc_achieved/pmc_frac: the bytes the kernel actually moves "
                        "(rocprofv3 FETCH_SIZE + WRITE_SIZE, committed under profiles/, same workload). "
                        "reference_equiv: SURVEY 8(d)'s B_upd, which counts the reference's wavefront re-reads "
                        "that the frontier cache skips; not a byte count."}
    if roofline["achieved"] is not None:
        roofline["frac"] = roofline["achieved"] / HBM_PEAK_GBS
    if traffic:
        roofline["pmc_achieved"] = traffic / per_launch_s / 1e9
        roofline["pmc_frac"] = roofline["pmc_achieved"] / HBM_PEAK_GBS
        roofline["pmc_source"] = pmc["_file"]
        roofline["traffic_over_model"] = traffic / model_bytes if model_bytes else None
    elif pmc and pmc.get("kernel_ms_per_launch_bench_events"):
        # a smaller batch of the same generator: its own rate and ratio
        roofline["pmc_workload"] = pmc["workload"]
        roofline["pmc_achieved"] = pmc["traffic_bytes_per_launch"] / (pmc["kernel_ms_per_launch_bench_events"] / 1e3) / 1e9
        roofline["pmc_frac"] = roofline["pmc_achieved"] / HBM_PEAK_GBS
        roofline["pmc_source"] = pmc["_file"]
        if pmc.get("model_bytes_per_launch"):
            roofline["traffic_over_model"] = pmc["traffic_bytes_per_launch"] / pmc["model_bytes_per_launch"]
    issue = profile_record("issue_view", cfgd["workload"], W.kernel, family=fam)
    if issue:
        roofline["issue_view"] = {k: v for k, v in issue.items() if not k.startswith("_") and k != "workload"}
        roofline["issue_view"]["source"] = issue["_file"]

    line = {
        "metric": METRIC,
        "value": total_upd / elapsed,
        "unit": "updates/s",
        "loci_per_s": total_loci / elapsed,
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": statistics.median(step_ms),
        "ms_per_step_mean": elapsed / a.steps * 1e3,
        "kernel_ms_per_step": kernel_ms / a.steps,
        "higher_is_better": True,
        "scaling": W.scaling,
        "vs_baseline": None,
        "dtype": "u8/u32 (integer DWFA) + f64 votes",
        "data": W.data(),
        "config": cfgd,
        "roofline": roofline,
        "gen_s": W.gen_s,
        "upload_s": W.upload_s,
    }
    if hasattr(W, "extra"):
        note("extra legs")
        line.update(W.extra())
    if share:
        line["rehearsal"] = "%d ranks sharing %d GPU(s) (WC_BENCH_SHARE_GPU, gloo): exercises the N-rank path, " \
                            "not a scaling measurement" % (world, max(1, torch.cuda.device_count()))
    if cfg5_leg:
        line["cfg5_strong"] = cfg5_leg
    if w_ranks:
        line["ranks"] = w_ranks
    if e2e:
        line["e2e_loci_per_s"], line["e2e_upload_ms"], line["e2e_compute_ms"] = e2e
        if getattr(W, "e2e_packed", None) is not None:  # bytes of the last refill sent 2-bit packed (0 = byte path)
            line["e2e_upload_packed_bytes"] = W.e2e_packed
        line["e2e_steps"] = e2e_steps
        line["e2e_note"] = ("fresh batch every step: Python marshalling + pinned staging + H2D of the reads, "
                            "double-buffered against the previous batch's compute; e2e_steps batches timed from "
                            "the first upload (not overlapped) to the last result. e2e_upload_ms / e2e_compute_ms: "
                            "one serial upload, and one cold compute call on a fresh context")
    if world == 1 and not a.no_cpu:
        note("CPU baseline")
        cores, aff, quota = usable_cpus()
        threads = a.cpu_threads or cores
        cb = W.cpu(threads, a.cpu_seconds)
        if cb:
            cb.setdefault("cores", threads)
            cb.update({"kind": "port", "cpu_model": cpu_model(), "affinity_cpus": aff, "cgroup_quota_cpus": quota})
            line["cpu_baseline"] = cb
            line["gpu_vs_cpu_loci"] = line["loci_per_s"] / cb["loci_per_s"]
            if e2e:
                line["e2e_vs_cpu_loci"] = line["e2e_loci_per_s"] / cb["loci_per_s"]
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
