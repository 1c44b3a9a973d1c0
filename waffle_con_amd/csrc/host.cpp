// Host orchestration and C ABI of the waffle_con MI355X library.
//
// A batch uploads every problem's reads once into an HBM arena (wc_batch);
// each run launches the device-resident engine once for the whole batch (one
// workgroup per problem, persistent grid pulling problems from an atomic
// counter, longest problems first) and turns the device result records into
// the reference's result types (Consensus, DualConsensus, PriorityConsensus).
// Problems that outgrow a device capacity (wavefront length, node pool,
// consensus length) are re-run on the device with doubled capacities; no
// consensus work is ever done on the CPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "../../include/waffle_con.h"
#include "engine_shared.hpp"
#include "waffle_con_internal.hpp"

namespace wc {
void launch_single_engine(const EngineArgs& a, uint32_t grid, size_t lds, hipStream_t s);
void launch_dual_engine(const EngineArgs& a, uint32_t grid, size_t lds, hipStream_t s);
int engine_blocks_per_cu(uint32_t sides, size_t lds);
void launch_dwfa_jobs(DwfaDevJob* jobs, uint32_t n, hipStream_t s);
void launch_wfa_ed_batch(const EdDevJob* jobs, uint32_t n, const uint8_t* seqs, uint64_t* scratch, int wc,
                         uint32_t both, uint64_t* out, hipStream_t s);
}  // namespace wc

using namespace wc;

// ------------------------------------------------------------------------
// context and device buffers
// ------------------------------------------------------------------------
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  bool ensure(size_t bytes) {
    if (bytes <= cap) return true;
    release();
    size_t want = std::max<size_t>(bytes + bytes / 8, 1 << 20);
    if (hipMalloc(&p, want) != hipSuccess) {
      p = nullptr;
      return false;
    }
    cap = want;
    return true;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// pinned host staging for the per-launch read-back (status, counters, first records)
struct HostBuf {
  void* p = nullptr;
  size_t cap = 0;
  bool ensure(size_t bytes) {
    if (bytes <= cap) return true;
    release();
    size_t want = std::max<size_t>(bytes + bytes / 8, 1 << 20);
    if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) {
      p = nullptr;
      return false;
    }
    cap = want;
    return true;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct wc_ctx {
  int device = 0;
  int n_cu = 256;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::string err;
  DevBuf ract, probs, ws, out, status, stats, counter, jobs, act;
  HostBuf stage;
  HostBuf upstage;  // pinned staging of batch uploads (reused across batches)
};

namespace {
std::string err_msg(int code) {
  switch (code) {
    case WC_E_FINALIZE_UNINIT: return "Finalize called on DWFA that was never initialized.";
    case WC_E_NO_START: return "Must have at least one initial offset of None to see the consensus.";
    case WC_E_COVERAGE_GAP: return "Encountered coverage gap";
    case WC_E_CAPACITY: return "Capacity is full";
    case WC_E_LOCKED: return "Consensus is locked, cannot modify";
    case WC_E_DUAL_TWICE: return "Cannot activate dual on a dual node";
    case WC_E_SAME_SYMBOL: return "Cannot activate dual mode with the same extension symbols";
    case WC_E_ROOT_INACTIVE: return "Root consensus node has no initially active sequences.";
    case WC_E_BAD_INPUT: return "invalid input";
    case WC_E_INVARIANT: return "internal invariant violated";
    case WC_E_LIMIT:
      return "device capacity limit exceeded (alphabet: more than 8 distinct symbols at one read's wavefront tips "
             "or 14 voted at one node side; or more than 64 children of one node)";
    case WC_E_HIP: return "HIP runtime failure";
    default: return "ok";
  }
}

// HBM the node pools of one launch may take: half of what is free plus the
// context's cached workspace (reused by the launch)
inline uint64_t pool_hbm(wc_ctx* ctx) {
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) fr = 32ull << 30;
  return ((uint64_t)fr + (uint64_t)ctx->ws.cap) / 2;
}
inline int set_err(wc_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

#define HIPCHK(call)                                                                                       \
  do {                                                                                                     \
    hipError_t _e = (call);                                                                                \
    if (_e != hipSuccess) return set_err(ctx, WC_E_HIP, std::string(#call) + ": " + hipGetErrorString(_e)); \
  } while (0)

DevConfig to_dev(const wc_config& c) {
  DevConfig d;
  d.max_queue_size = c.max_queue_size;
  d.max_capacity_per_size = c.max_capacity_per_size;
  d.max_return_size = c.max_return_size;
  d.max_nodes_wo_constraint = c.max_nodes_wo_constraint;
  d.min_count = c.min_count;
  d.dual_max_ed_delta = c.dual_max_ed_delta;
  d.offset_window = c.offset_window;
  d.offset_compare_length = c.offset_compare_length;
  d.min_af = c.min_af;
  d.cost_mode = c.consensus_cost;
  d.wildcard = c.wildcard;
  d.weighted = c.weighted_by_ed;
  d.early = c.allow_early_termination;
  return d;
}

inline uint64_t cost_of_h(uint32_t e, int mode) { return mode == 0 ? (uint64_t)e : (uint64_t)e * (uint64_t)e; }
}  // namespace

// ------------------------------------------------------------------------
// resident batch: reads of many problems in one HBM arena
// ------------------------------------------------------------------------
struct BatchProblem {
  uint32_t read_begin = 0;
  uint32_t n_reads = 0;
  uint32_t max_len = 0;
  uint64_t work = 0;             // sum of read lengths (scheduling order)
  std::vector<int64_t> offsets;  // raw add_sequence_offset values (-1 = None)
};

struct wc_batch {
  wc_ctx* ctx = nullptr;
  std::vector<BatchProblem> probs;
  std::vector<uint32_t> rlen_h;
  DevBuf reads, roff, rlen;
  uint64_t bytes = 0;
  ~wc_batch() {
    reads.release();
    roff.release();
    rlen.release();
  }
};

// ------------------------------------------------------------------------
// results
// ------------------------------------------------------------------------
struct ConsRec {
  std::vector<uint8_t> seq;
  std::vector<uint64_t> scores;
};
struct DualRec {
  ConsRec c1, c2;
  bool has_c2 = false;
  std::vector<uint8_t> is_c1;
  std::vector<int64_t> s1, s2;
};
struct ProbRes {
  int status = WC_OK;
  std::string error;
  std::vector<ConsRec> single;
  std::vector<DualRec> dual;
  std::vector<std::vector<ConsRec>> chains;
  std::vector<uint64_t> indices;
  uint64_t stats[S_NSTAT] = {0};
};
struct wc_results {
  int kind = 0;  // 0 single, 1 dual, 2 priority
  std::vector<ProbRes> probs;
  wc_stats stats;
};

struct RawRecord {
  uint32_t len[2] = {0, 0};
  bool dual = false;
  std::vector<uint8_t> con[2];
  std::vector<uint32_t> fe[2];
};

namespace {
// Copies every read of `problems` into one 16-byte-aligned arena and uploads it.
// The host side is one pass of memcpy into pinned staging (split over threads
// by bytes), then a single DMA; the device buffer of `b` is reused when it is
// large enough (wc_batch_refill), so a refill needs no allocation.
int upload_batch(wc_ctx* ctx, uint32_t n, const wc_problem* problems, wc_batch* b) {
  b->ctx = ctx;
  b->probs.assign(n, BatchProblem());
  b->rlen_h.clear();
  uint64_t nr = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (problems[i].n_reads && (!problems[i].reads || !problems[i].lens))
      return set_err(ctx, WC_E_BAD_INPUT, "problem with reads but no read/length arrays");
    nr += problems[i].n_reads;
  }
  std::vector<uint64_t> roff(nr);
  b->rlen_h.resize(nr);
  std::vector<const uint8_t*> src(nr);
  uint64_t pos = 0, k = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const wc_problem& p = problems[i];
    BatchProblem& q = b->probs[i];
    q.read_begin = (uint32_t)k;
    q.n_reads = p.n_reads;
    q.offsets.assign(p.n_reads, -1);
    for (uint32_t r = 0; r < p.n_reads; ++r, ++k) {
      if (p.offsets) q.offsets[r] = p.offsets[r] < 0 ? -1 : p.offsets[r];
      if (p.lens[r] >= (1ull << 31)) return set_err(ctx, WC_E_BAD_INPUT, "read longer than 2^31 bytes");
      roff[k] = pos;
      src[k] = p.reads[r];
      b->rlen_h[k] = (uint32_t)p.lens[r];
      pos += (p.lens[r] + 15) & ~15ull;
      q.max_len = std::max<uint32_t>(q.max_len, (uint32_t)p.lens[r]);
      q.work += p.lens[r];
    }
  }
  // reads start 16-byte aligned; 64 bytes of tail padding let the engine load
  // 64-byte windows with 16-byte accesses anywhere inside a read
  const uint64_t total = pos + 64;
  b->bytes = total;
  std::vector<uint8_t> fallback;
  uint8_t* h = nullptr;
  if (ctx->upstage.ensure(total)) {
    h = (uint8_t*)ctx->upstage.p;
  } else {
    fallback.resize(total);
    h = fallback.data();
  }
  auto fill = [&](uint64_t r0, uint64_t r1) {
    for (uint64_t r = r0; r < r1; ++r) {
      const uint64_t len = b->rlen_h[r], pad = ((len + 15) & ~15ull) - len;
      if (len) memcpy(h + roff[r], src[r], len);
      if (pad) memset(h + roff[r] + len, 0, pad);
    }
  };
  // split the reads into contiguous ranges of about equal bytes
  const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const unsigned nt = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(hw, total >> 23));  // >= 8 MiB per thread
  if (nt <= 1 || nr < 2) {
    fill(0, nr);
  } else {
    std::vector<std::thread> th;
    uint64_t r0 = 0;
    for (unsigned t = 0; t < nt; ++t) {
      const uint64_t want = pos * (t + 1) / nt;
      uint64_t r1 = r0;
      while (r1 < nr && (t + 1 == nt || roff[r1] < want)) ++r1;
      th.emplace_back(fill, r0, r1);
      r0 = r1;
    }
    for (auto& x : th) x.join();
  }
  memset(h + pos, 0, 64);
  if (!b->reads.ensure(total) || !b->roff.ensure(std::max<size_t>(roff.size(), 1) * 8) ||
      !b->rlen.ensure(std::max<size_t>(b->rlen_h.size(), 1) * 4))
    return set_err(ctx, WC_E_HIP, "device allocation failed (reads)");
  HIPCHK(hipMemcpyAsync(b->reads.p, h, total, hipMemcpyHostToDevice, ctx->stream));
  if (!roff.empty()) HIPCHK(hipMemcpyAsync(b->roff.p, roff.data(), roff.size() * 8, hipMemcpyHostToDevice, ctx->stream));
  if (!b->rlen_h.empty())
    HIPCHK(hipMemcpyAsync(b->rlen.p, b->rlen_h.data(), b->rlen_h.size() * 4, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return WC_OK;
}

// auto_shift_offsets + activation points (consensus.rs:151-202); returns a
// per-read activation length (-1 = active at the root) or an error code.
int activation_plan(const wc_config& cfg, const BatchProblem& q, std::vector<int64_t>& act, uint32_t& n_active,
                    std::string& err) {
  if (q.n_reads == 0) {
    err = "No sequences provided";
    return WC_E_BAD_INPUT;
  }
  std::vector<int64_t> offs = q.offsets;
  if (cfg.auto_shift_offsets) {
    int64_t mn = INT64_MAX;
    bool start = false;
    for (auto o : offs) {
      if (o < 0) start = true;
      else mn = std::min(mn, o);
    }
    if (!start)
      for (auto& o : offs) o = (o == mn) ? -1 : o - mn;
  }
  act.assign(q.n_reads, -1);
  n_active = 0;
  for (uint32_t i = 0; i < q.n_reads; ++i) {
    if (offs[i] >= 0) act[i] = offs[i] + (int64_t)cfg.offset_compare_length;
    else n_active++;
  }
  if (n_active == 0) {
    err = err_msg(WC_E_NO_START);
    return WC_E_NO_START;
  }
  return WC_OK;
}

struct EngineRun {
  std::vector<std::vector<RawRecord>> recs;
  std::vector<int> status;
  std::vector<std::string> error;
  std::vector<std::array<uint64_t, S_NSTAT>> stats;
  double kernel_ms = 0;
  uint64_t launches = 0;
};

// Runs the problems `ids` (indices into b->probs) through the engine.
int run_engine(wc_ctx* ctx, wc_batch* b, const wc_config& cfg, uint32_t sides, std::vector<uint32_t> ids,
               EngineRun& R) {
  const uint32_t NP = (uint32_t)b->probs.size();
  R.recs.assign(NP, {});
  R.status.assign(NP, WC_OK);
  R.error.assign(NP, "");
  R.stats.assign(NP, {});
  for (auto& s : R.stats) s.fill(0);

  // per-read activation lengths for the whole batch (indexed by global read)
  std::vector<int64_t> ract(std::max<size_t>(b->rlen_h.size(), 1), -1);
  std::vector<uint32_t> n_active(NP, 0), max_act(NP, 0);
  std::vector<uint32_t> runnable;
  bool any_act = false;
  for (uint32_t id : ids) {
    std::vector<int64_t> act;
    int rc = activation_plan(cfg, b->probs[id], act, n_active[id], R.error[id]);
    if (rc != WC_OK) {
      R.status[id] = rc;
      continue;
    }
    std::copy(act.begin(), act.end(), ract.begin() + b->probs[id].read_begin);
    for (auto a : act)
      if (a >= 0) {
        if (a > (int64_t)UINT32_MAX - 2) {
          R.status[id] = WC_E_LIMIT;
          R.error[id] = "activation offset beyond the device engine's u32 lengths";
        }
        max_act[id] = std::max<uint32_t>(max_act[id], (uint32_t)std::min<int64_t>(a, UINT32_MAX - 2));
        any_act = true;
      }
    if (R.status[id] != WC_OK) continue;
    runnable.push_back(id);
  }
  ids = runnable;
  if (ids.empty()) return WC_OK;
  if (!ctx->ract.ensure(ract.size() * 8)) return set_err(ctx, WC_E_HIP, "device allocation failed");
  HIPCHK(hipMemcpyAsync(ctx->ract.p, ract.data(), ract.size() * 8, hipMemcpyHostToDevice, ctx->stream));

  uint32_t nmax = 1, maxlen = 1;
  for (uint32_t id : ids) {
    nmax = std::max<uint32_t>(nmax, b->probs[id].n_reads);
    maxlen = std::max<uint32_t>(maxlen, b->probs[id].max_len);
  }
  uint32_t ecap = std::max<uint32_t>(31, maxlen / 64);
  uint32_t wcap = ((2 * ecap + 1 + 63) / 64) * 64;
  uint32_t lcap = ((maxlen + maxlen / 8 + 64 + 15) / 16) * 16;
  // node pool: as many slots as ~16 MiB of workspace per workgroup allows
  // (16..256), bounded by the LDS the heap/metadata need
  // single engine: linear-chain run-ahead length (WC_CHAIN=<k> overrides, 0 = off)
  uint32_t chain = (sides == 1 && nmax <= (uint32_t)kBlock) ? kChainDefault : 0;
  const char* chain_env = getenv("WC_CHAIN");
  if (chain_env) chain = std::min<uint32_t>((uint32_t)atoi(chain_env), kChainMax);
  if (sides != 1 || nmax > (uint32_t)kBlock) chain = 0;
  uint32_t pcap = 16;
  {
    // A dual search keeps far more nodes queued than a single one (children
    // of both consensuses, both sides' DWFAs per node: cfg3 loci peak at ~480
    // queued nodes). An exhausted pool restarts the search with a bigger one,
    // so the dual pool gets up to half of the free HBM over the workgroups
    // that can run at once (<= 256 MiB each).
    const uint64_t sb = slot_bytes(sides, nmax, wcap, lcap);
    uint64_t dual_budget = 16ull << 20;
    if (sides == 2) {
      const uint64_t conc = std::max<uint64_t>(1, std::min<uint64_t>(ids.size(), 4ull * (uint64_t)ctx->n_cu));
      dual_budget = std::max<uint64_t>(16ull << 20, std::min<uint64_t>(256ull << 20, pool_hbm(ctx) / conc));
    }
    const uint64_t budget = sides == 1 ? (16ull << 20) : dual_budget;
    const uint32_t pmax = sides == 1 ? 256u : 1024u;
    const uint64_t lmax = sides == 1 ? 40 * 1024 : 48 * 1024;
    while (pcap < pmax && (uint64_t)(pcap * 2) * sb <= budget && lds_bytes(sides, pcap * 2, nmax, chain) <= lmax)
      pcap *= 2;
  }
  // longer chains amortise the per-chain work (prediction, acceptance, the
  // literal pop between chains); take the longest one whose LDS still gives
  // the workgroups per CU of the default length (results do not depend on it)
  if (!chain_env && chain > 0) {
    const int occ = engine_blocks_per_cu(sides, (size_t)lds_bytes(sides, pcap, nmax, chain));
    for (uint32_t k = chain + 1; k <= kChainMax; ++k) {
      const uint64_t l = lds_bytes(sides, pcap, nmax, k);
      if (l > 60 * 1024 || engine_blocks_per_cu(sides, (size_t)l) < occ) break;
      chain = k;
    }
  }
  // result records per problem: up to 256 at first; a problem with more tied
  // results than records reruns with more (ST_RETRY_RMAX), up to max_return_size
  uint32_t rmax = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(cfg.max_return_size, 1), 256);
  if (const char* r0 = getenv("WC_RMAX"))  // test hook: a smaller first record count exercises the retry
    rmax = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(rmax, (uint64_t)atoi(r0)));

  for (int attempt = 0; attempt < 8 && !ids.empty(); ++attempt) {
    std::stable_sort(ids.begin(), ids.end(),
                     [&](uint32_t x, uint32_t y) { return b->probs[x].work > b->probs[y].work; });
    const uint32_t P = (uint32_t)ids.size();
    std::vector<DevProblem> dp(P);
    for (uint32_t i = 0; i < P; ++i) {
      const BatchProblem& q = b->probs[ids[i]];
      dp[i].read_begin = q.read_begin;
      dp[i].n_reads = q.n_reads;
      dp[i].max_read_len = q.max_len;
      dp[i].n_active = n_active[ids[i]];
      dp[i].max_act = max_act[ids[i]];
    }
    size_t lds = (size_t)lds_bytes(sides, pcap, nmax, chain);
    if (lds > 60 * 1024) {
      for (uint32_t id : ids) {
        R.status[id] = WC_E_LIMIT;
        R.error[id] = "problem needs more LDS than the engine allows (reads x node pool)";
      }
      return WC_OK;
    }
    int per_cu = engine_blocks_per_cu(sides, lds);
    uint32_t grid = std::min<uint32_t>(P, (uint32_t)std::max(1, per_cu) * (uint32_t)ctx->n_cu);
    uint64_t wsb = ws_bytes(sides, pcap, nmax, wcap, lcap);
    uint64_t ob = out_bytes(sides, rmax, nmax, lcap);
    // offset activation scratch (wfa_ed_config pair arrays): edits <= |v1| + |v2|
    // with |v1| <= window + ocl and |v2| <= ocl (engine_common wave_pick_offset)
    uint32_t act_m = 0;
    if (any_act) {
      const uint64_t ocl = std::min<uint64_t>(cfg.offset_compare_length, maxlen);
      const uint64_t m = 3 + 2 * (cfg.offset_window + 2 * ocl) + 8;
      if (m > 8192) {
        for (uint32_t id : ids) {
          R.status[id] = WC_E_LIMIT;
          R.error[id] = "offset_window/offset_compare_length too large for the device activation scratch";
        }
        return WC_OK;
      }
      act_m = (uint32_t)m;
    }
    if (act_m && !ctx->act.ensure(act_scr_u64(act_m) * 8 * grid))
      return set_err(ctx, WC_E_HIP, "device allocation failed (activation scratch)");
    if (!ctx->probs.ensure(P * sizeof(DevProblem)) || !ctx->ws.ensure(wsb * grid) || !ctx->out.ensure(ob * P) ||
        !ctx->status.ensure(P * 4) || !ctx->stats.ensure((size_t)P * S_NSTAT * 8) || !ctx->counter.ensure(4))
      return set_err(ctx, WC_E_HIP, "device allocation failed (workspace)");
    HIPCHK(hipMemcpyAsync(ctx->probs.p, dp.data(), P * sizeof(DevProblem), hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemsetAsync(ctx->counter.p, 0, 4, ctx->stream));

    EngineArgs a;
    memset(&a, 0, sizeof(a));
    a.cfg = to_dev(cfg);
    a.problems = (const DevProblem*)ctx->probs.p;
    a.n_problems = P;
    a.sides = sides;
    a.rbytes = (const uint8_t*)b->reads.p;
    a.roff = (const uint64_t*)b->roff.p;
    a.rlen = (const uint32_t*)b->rlen.p;
    a.ractivate = (const int64_t*)ctx->ract.p;
    a.ws = (uint8_t*)ctx->ws.p;
    a.ws_stride = wsb;
    a.pcap = pcap;
    a.wcap = wcap;
    a.lcap = lcap;
    a.nmax = nmax;
    a.rmax = rmax;
    a.chain = chain;
    a.out = (uint8_t*)ctx->out.p;
    a.out_stride = ob;
    a.status = (uint32_t*)ctx->status.p;
    a.stats = (uint64_t*)ctx->stats.p;
    a.work_counter = (uint32_t*)ctx->counter.p;
    a.act_m = act_m;
    a.act_scr = act_m ? (uint64_t*)ctx->act.p : nullptr;
    a.act_stride = act_m ? act_scr_u64(act_m) : 0;
    // debug trace of problem 0's pops (WC_TRACE=<file>); off by default
    const char* trace_path = getenv("WC_TRACE");
    DevBuf tbuf;
    const uint32_t tcap = 1u << 20;
    if (trace_path && tbuf.ensure((size_t)(4 + 4 * tcap) * 4)) {
      a.trace = (uint32_t*)tbuf.p;
      a.trace_cap = tcap;
      HIPCHK(hipMemsetAsync(tbuf.p, 0, 16, ctx->stream));
    }

    // debug phase cycle counters (WC_PHASES=<file>, WC_PHASE_PROF builds only)
    const char* phase_path = getenv("WC_PHASES");
    DevBuf pbuf;
    if (phase_path && pbuf.ensure(kPhases * 8)) {
      a.phases = (unsigned long long*)pbuf.p;
      HIPCHK(hipMemsetAsync(pbuf.p, 0, kPhases * 8, ctx->stream));
    }

    HIPCHK(hipEventRecord(ctx->ev0, ctx->stream));
    if (sides == 1) launch_single_engine(a, grid, lds, ctx->stream);
    else launch_dual_engine(a, grid, lds, ctx->stream);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(ctx->ev1, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    R.kernel_ms += ms;
    R.launches++;
    if (a.phases) {
      unsigned long long ph[kPhases];
      HIPCHK(hipMemcpy(ph, pbuf.p, sizeof(ph), hipMemcpyDeviceToHost));
      if (FILE* f = fopen(phase_path, "a")) {
        fprintf(f, "sides=%u kernel_ms=%.3f", sides, ms);
        for (int k = 0; k < kPhases; ++k) fprintf(f, " %llu", ph[k]);
        fprintf(f, "\n");
        fclose(f);
      }
      pbuf.release();
    }
    if (a.trace) {
      uint32_t cnt = 0;
      HIPCHK(hipMemcpy(&cnt, tbuf.p, 4, hipMemcpyDeviceToHost));
      std::vector<uint32_t> t((size_t)4 * std::min(cnt, tcap));
      if (!t.empty()) HIPCHK(hipMemcpy(t.data(), (uint32_t*)tbuf.p + 4, t.size() * 4, hipMemcpyDeviceToHost));
      if (FILE* f = fopen(trace_path, "w")) {
        for (size_t k = 0; k < t.size(); k += 4) fprintf(f, "%u %u %u %u\n", t[k], t[k + 1], t[k + 2], t[k + 3]);
        fclose(f);
      }
      tbuf.release();
    }

    // read back: status, stats, and the first record of every problem in one
    // strided copy; further records only for problems that returned ties
    const uint64_t rb = result_bytes(sides, nmax, lcap);
    const uint64_t first = 16 + rb;
    const size_t st_off = 0, stats_off = align16((uint64_t)P * 4),
                 out_off = stats_off + align16((uint64_t)P * S_NSTAT * 8);
    if (!ctx->stage.ensure(out_off + (size_t)first * P))
      return set_err(ctx, WC_E_HIP, "pinned host allocation failed");
    uint8_t* stg = (uint8_t*)ctx->stage.p;
    HIPCHK(hipMemcpyAsync(stg + st_off, ctx->status.p, P * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipMemcpyAsync(stg + stats_off, ctx->stats.p, (size_t)P * S_NSTAT * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipMemcpy2DAsync(stg + out_off, first, ctx->out.p, ob, first, P, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    const uint32_t* hst = (const uint32_t*)(stg + st_off);
    const uint64_t* hstats = (const uint64_t*)(stg + stats_off);
    const uint8_t* hout = stg + out_off;

    std::vector<uint32_t> retry;
    uint32_t rflags = 0;
    std::vector<uint8_t> extra;
    for (uint32_t i = 0; i < P; ++i) {
      const uint32_t id = ids[i];
      const uint32_t st = hst[i];
      // counters of the attempt that completed (a capacity retry restarts the search)
      for (int s = 0; s < S_NSTAT; ++s) R.stats[id][s] = hstats[(size_t)i * S_NSTAT + s];
      if (st & ST_RETRY) {
        retry.push_back(id);
        rflags |= st;
        continue;
      }
      R.status[id] = (int)st;
      if (st != ST_OK) {
        R.error[id] = err_msg((int)st);
        if (st == WC_E_COVERAGE_GAP)  // consensus.rs:305 / dual_consensus.rs message
          R.error[id] = "Encountered coverage gap: consensus is length " +
                        std::to_string(((const uint32_t*)(hout + (size_t)i * first))[1]) +
                        " with no candidates, but sequences activate at " + std::to_string(max_act[id]);
        continue;
      }
      const uint8_t* base = hout + (size_t)i * first;
      const uint32_t nres = ((const uint32_t*)base)[0];
      if (nres > 1) {
        extra.resize((size_t)nres * rb);
        HIPCHK(hipMemcpy(extra.data(), (uint8_t*)ctx->out.p + (size_t)i * ob + 16, extra.size(),
                         hipMemcpyDeviceToHost));
      }
      const uint32_t n = b->probs[id].n_reads;
      for (uint32_t k = 0; k < nres; ++k) {
        const uint8_t* rec = k == 0 ? base + 16 : extra.data() + (size_t)k * rb;
        const uint32_t* h = (const uint32_t*)rec;
        RawRecord rr;
        rr.len[0] = h[0];
        rr.len[1] = h[1];
        rr.dual = h[2] != 0;
        for (uint32_t s = 0; s < sides; ++s) {
          const uint8_t* con = rec + 16 + s * align16(lcap);
          rr.con[s].assign(con, con + rr.len[s]);
          const uint32_t* fe = (const uint32_t*)(rec + 16 + sides * align16(lcap) + s * align16((uint64_t)nmax * 4));
          rr.fe[s].assign(fe, fe + n);
        }
        R.recs[id].push_back(std::move(rr));
      }
    }
    // debug: one line per launch on stderr (WC_LAUNCH_LOG=1); off by default
    if (getenv("WC_LAUNCH_LOG"))
      fprintf(stderr, "[wc] sides=%u problems=%u grid=%u per_cu=%d lds=%zu pcap=%u wcap=%u lcap=%u chain=%u ms=%.3f retry=%zu flags=0x%x\n",
              sides, P, grid, per_cu, lds, pcap, wcap, lcap, chain, ms, retry.size(), rflags);
    ids = retry;
    if (rflags & ST_RETRY_WCAP) wcap = wcap * 2;
    if (rflags & (ST_RETRY_PCAP | ST_RETRY_HEAP)) {
      // a failed attempt costs nearly a full search: grow 4x when the HBM
      // share allows it
      const uint64_t conc = std::min<uint64_t>(ids.size(), 4ull * (uint64_t)ctx->n_cu);
      const bool big = ws_bytes(sides, pcap * 4, nmax, wcap, lcap) * conc <= pool_hbm(ctx) &&
                       lds_bytes(sides, pcap * 4, nmax, chain) <= 60 * 1024;
      pcap = pcap * (big ? 4 : 2);
    }
    if (rflags & ST_RETRY_LCAP) lcap = lcap * 2;
    if (rflags & ST_RETRY_RMAX) {
      const uint64_t want = std::min<uint64_t>(cfg.max_return_size, (uint64_t)rmax * 8);
      const uint64_t bytes = out_bytes(sides, (uint32_t)std::min<uint64_t>(want, UINT32_MAX), nmax, lcap) * ids.size();
      if (want > UINT32_MAX || bytes > pool_hbm(ctx)) {
        for (uint32_t id : ids) {
          R.status[id] = WC_E_LIMIT;
          R.error[id] = "more tied results than the device result buffer holds (max_return_size)";
        }
        return WC_OK;
      }
      rmax = (uint32_t)want;
    }
  }
  for (uint32_t id : ids) {
    R.status[id] = WC_E_LIMIT;
    R.error[id] = err_msg(WC_E_LIMIT);
  }
  return WC_OK;
}

void fill_stats(wc_results* R, double kernel_ms, uint64_t launches, double wall_ms) {
  memset(&R->stats, 0, sizeof(R->stats));
  for (auto& p : R->probs) {
    R->stats.updates += p.stats[S_UPDATES];
    R->stats.w_out += p.stats[S_WOUT];
    R->stats.compares += p.stats[S_COMPARES];
    R->stats.ed_increases += p.stats[S_EDINC];
    R->stats.finalizes += p.stats[S_FINALIZES];
    R->stats.pops += p.stats[S_POPS];
    R->stats.nodes_explored += p.stats[S_EXPLORED];
    R->stats.nodes_ignored += p.stats[S_IGNORED];
    R->stats.peak_queue_size = std::max(R->stats.peak_queue_size, p.stats[S_PEAKQ]);
  }
  R->stats.kernel_ms = kernel_ms;
  R->stats.launches = launches;
  R->stats.wall_ms = wall_ms;
}

// consensus.rs:345 — single results sorted by sequence
void build_single(const EngineRun& E, uint32_t id, int mode, ProbRes& pr) {
  for (int s = 0; s < S_NSTAT; ++s) pr.stats[s] = E.stats[id][s];
  pr.status = E.status[id];
  pr.error = E.error[id];
  if (pr.status != WC_OK) return;
  for (const RawRecord& rr : E.recs[id]) {
    ConsRec c;
    c.seq = rr.con[0];
    for (auto e : rr.fe[0]) c.scores.push_back(cost_of_h(e, mode));
    pr.single.push_back(std::move(c));
  }
  std::stable_sort(pr.single.begin(), pr.single.end(), [](const ConsRec& a, const ConsRec& b) { return a.seq < b.seq; });
}

// DualConsensus::from_node (dual_consensus.rs:102-150) on a finalized record
bool dual_from_record(const RawRecord& rr, uint32_t n, int mode, DualRec& d) {
  std::vector<uint64_t> sc[2];
  const bool swap = rr.dual && (rr.con[1] < rr.con[0]);
  d.is_c1.clear();
  for (uint32_t r = 0; r < n; ++r) {
    const uint32_t e1 = rr.fe[0][r], e2 = rr.dual ? rr.fe[1][r] : kInactive;
    int idx = -1;
    uint64_t best = UINT64_MAX;
    if (e1 != kInactive) {
      best = cost_of_h(e1, mode);
      idx = 0;
    }
    if (e2 != kInactive && cost_of_h(e2, mode) < best) {
      best = cost_of_h(e2, mode);
      idx = 1;
    }
    if (idx < 0) return false;  // assert!(best_con_index <= 1)
    d.is_c1.push_back((uint8_t)((idx == 0) ^ swap));
    sc[idx].push_back(best);
  }
  ConsRec c1{rr.con[0], sc[0]}, c2{rr.dual ? rr.con[1] : std::vector<uint8_t>(), sc[1]};
  std::vector<int64_t> s1(n), s2(n);
  for (uint32_t r = 0; r < n; ++r) {
    s1[r] = rr.fe[0][r] == kInactive ? -1 : (int64_t)cost_of_h(rr.fe[0][r], mode);
    uint32_t e2 = rr.dual ? rr.fe[1][r] : kInactive;
    s2[r] = e2 == kInactive ? -1 : (int64_t)cost_of_h(e2, mode);
  }
  if (swap) {
    d.c1 = c2;
    d.c2 = c1;
    d.has_c2 = true;
    d.s1 = s2;
    d.s2 = s1;
  } else {
    d.c1 = c1;
    d.has_c2 = rr.dual;
    if (rr.dual) d.c2 = c2;
    d.s1 = s1;
    d.s2 = s2;
  }
  return true;
}

void build_dual(const EngineRun& E, uint32_t id, uint32_t n, int mode, ProbRes& pr) {
  for (int s = 0; s < S_NSTAT; ++s) pr.stats[s] = E.stats[id][s];
  pr.status = E.status[id];
  pr.error = E.error[id];
  if (pr.status != WC_OK) return;
  for (const RawRecord& rr : E.recs[id]) {
    DualRec d;
    if (!dual_from_record(rr, n, mode, d)) {
      pr.status = WC_E_INVARIANT;
      pr.error = "read without a tracked consensus in a result";
      return;
    }
    pr.dual.push_back(std::move(d));
  }
  if (pr.dual.size() > 1) {
    // dual_consensus.rs:744-766
    std::stable_sort(pr.dual.begin(), pr.dual.end(), [](const DualRec& a, const DualRec& b) {
      static const std::vector<uint8_t> empty;
      const auto& a2 = a.has_c2 ? a.c2.seq : empty;
      const auto& b2 = b.has_c2 ? b.c2.seq : empty;
      if (a.c1.seq != b.c1.seq) return a.c1.seq < b.c1.seq;
      return a2 < b2;
    });
  }
  if (pr.dual.empty()) {
    // dual_consensus.rs:772-779: fallback to the root (every read active, empty consensus)
    RawRecord root;
    root.fe[0].assign(n, 0);
    DualRec d;
    dual_from_record(root, n, mode, d);
    pr.dual.push_back(std::move(d));
  }
}

template <class F>
int with_batch(wc_ctx* ctx, uint32_t n, const wc_problem* problems, F&& fn) {
  std::unique_ptr<wc_batch> b(new wc_batch());
  int rc = upload_batch(ctx, n, problems, b.get());
  if (rc != WC_OK) return rc;
  return fn(b.get());
}

// ---- PriorityConsensusDWFA helpers ----
uint64_t fx_add(uint64_t h, uint64_t w) { return (((h << 5) | (h >> 59)) ^ w) * 0x517cc1b727220a95ULL; }
uint64_t fx_hash_opt(int64_t v) { return v < 0 ? fx_add(0, 0) : fx_add(fx_add(0, 1), (uint64_t)v); }
size_t fx_cap_h(size_t b) { return b == 0 ? 0 : (b < 8 ? b - 1 : b / 8 * 7); }
size_t fx_buckets_h(size_t cap) {
  if (cap < 8) return cap < 4 ? 4 : 8;
  size_t adj = cap * 8 / 7, p = 1;
  while (p < adj) p <<= 1;
  return p;
}
// FxHashSet<Option<usize>> iteration order of the seed groups (priority_consensus.rs:180).
// The set is built by `.collect()`: hashbrown's extend first reserves the
// iterator's exact size hint (one entry per chain), so the table starts with
// capacity_to_buckets(n_chains) buckets and never grows while the (at most
// n_chains) distinct keys are inserted.
std::vector<int64_t> seed_order(const std::vector<int64_t>& groups) {
  std::vector<int64_t> keys;
  std::vector<uint64_t> hashes;
  std::vector<int64_t> tab(fx_buckets_h(std::max<size_t>(groups.size(), 1)), -1);
  size_t items = 0, growth = fx_cap_h(tab.size());
  auto slot = [&](uint64_t h) -> size_t {
    size_t B = tab.size(), mask = B - 1, pos = (size_t)h & mask;
    if (B < 16) {
      for (size_t i = pos; i < B; ++i)
        if (tab[i] < 0) return i;
      for (size_t i = 0; i < B; ++i)
        if (tab[i] < 0) return i;
      return 0;
    }
    size_t stride = 0;
    for (;;) {
      for (size_t j = 0; j < 16; ++j)
        if (tab[(pos + j) & mask] < 0) return (pos + j) & mask;
      stride += 16;
      pos = (pos + stride) & mask;
    }
  };
  for (int64_t g : groups) {
    if (std::find(keys.begin(), keys.end(), g) != keys.end()) continue;
    if (growth == 0) {
      size_t nb = fx_buckets_h(std::max(items + 1, fx_cap_h(tab.size()) + 1));
      std::vector<int64_t> old = tab;
      tab.assign(nb, -1);
      for (auto o : old)
        if (o >= 0) tab[slot(hashes[o])] = o;
      growth = fx_cap_h(nb) - items;
    }
    keys.push_back(g);
    hashes.push_back(fx_hash_opt(g));
    tab[slot(hashes.back())] = (int64_t)keys.size() - 1;
    items++;
    growth--;
  }
  std::vector<int64_t> out;
  for (auto t : tab)
    if (t >= 0) out.push_back(keys[t]);
  return out;
}

struct PWork {
  std::vector<uint8_t> inc;
  uint32_t level;
  std::vector<ConsRec> chain;
  // the sub-problem's DualConsensusDWFA result, computed ahead of its turn
  bool done = false;
  std::unique_ptr<ProbRes> res;
};
}  // namespace

// ------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------
extern "C" {

void wc_config_default(wc_config* c) {
  memset(c, 0, sizeof(*c));
  c->consensus_cost = 0;
  c->wildcard = -1;
  c->max_queue_size = 20;
  c->max_capacity_per_size = 20;
  c->max_return_size = 10;
  c->max_nodes_wo_constraint = 1000;
  c->min_count = 3;
  c->min_af = 0.0;
  c->dual_max_ed_delta = 20;
  c->offset_window = 50;
  c->offset_compare_length = 50;
  c->weighted_by_ed = 0;
  c->allow_early_termination = 0;
  c->auto_shift_offsets = 1;
}

int wc_ctx_create(int device, wc_ctx** out) {
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return WC_E_HIP;
  if (device < 0 || device >= ndev) return WC_E_HIP;
  if (hipSetDevice(device) != hipSuccess) return WC_E_HIP;
  wc_ctx* ctx = new wc_ctx();
  ctx->device = device;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) ctx->n_cu = prop.multiProcessorCount;
  if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&ctx->ev0) != hipSuccess || hipEventCreate(&ctx->ev1) != hipSuccess) {
    delete ctx;
    return WC_E_HIP;
  }
  *out = ctx;
  return WC_OK;
}

void wc_ctx_destroy(wc_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  for (DevBuf* b : {&ctx->ract, &ctx->probs, &ctx->ws, &ctx->out, &ctx->status, &ctx->stats, &ctx->counter, &ctx->jobs, &ctx->act})
    b->release();
  ctx->stage.release();
  ctx->upstage.release();
  if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
  if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

const char* wc_last_error(const wc_ctx* ctx) { return ctx ? ctx->err.c_str() : "no context"; }

int wc_batch_create(wc_ctx* ctx, uint32_t n, const wc_problem* problems, wc_batch** out) {
  *out = nullptr;
  if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, WC_E_HIP, "hipSetDevice failed");
  std::unique_ptr<wc_batch> b(new wc_batch());
  int rc = upload_batch(ctx, n, problems, b.get());
  if (rc != WC_OK) return rc;
  *out = b.release();
  return WC_OK;
}

int wc_batch_refill(wc_ctx* ctx, wc_batch* b, uint32_t n, const wc_problem* problems) {
  if (!b) return set_err(ctx, WC_E_BAD_INPUT, "null batch");
  if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, WC_E_HIP, "hipSetDevice failed");
  return upload_batch(ctx, n, problems, b);
}

void wc_batch_free(wc_batch* b) { delete b; }

uint64_t wc_batch_bytes(const wc_batch* b) { return b ? b->bytes : 0; }

int wc_batch_consensus(wc_ctx* ctx, wc_batch* b, const wc_config* cfg, wc_results** out) {
  auto t0 = std::chrono::steady_clock::now();
  *out = nullptr;
  if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, WC_E_HIP, "hipSetDevice failed");
  const uint32_t n = (uint32_t)b->probs.size();
  std::unique_ptr<wc_results> R(new wc_results());
  R->kind = 0;
  R->probs.resize(n);
  std::vector<uint32_t> ids(n);
  std::iota(ids.begin(), ids.end(), 0u);
  EngineRun E;
  int rc = run_engine(ctx, b, *cfg, 1, ids, E);
  if (rc != WC_OK) return rc;
  for (uint32_t id = 0; id < n; ++id) build_single(E, id, cfg->consensus_cost, R->probs[id]);
  double wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  fill_stats(R.get(), E.kernel_ms, E.launches, wall);
  *out = R.release();
  return WC_OK;
}

int wc_batch_dual_consensus(wc_ctx* ctx, wc_batch* b, const wc_config* cfg, wc_results** out) {
  auto t0 = std::chrono::steady_clock::now();
  *out = nullptr;
  if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, WC_E_HIP, "hipSetDevice failed");
  const uint32_t n = (uint32_t)b->probs.size();
  std::unique_ptr<wc_results> R(new wc_results());
  R->kind = 1;
  R->probs.resize(n);
  std::vector<uint32_t> ids(n);
  std::iota(ids.begin(), ids.end(), 0u);
  EngineRun E;
  int rc = run_engine(ctx, b, *cfg, 2, ids, E);
  if (rc != WC_OK) return rc;
  for (uint32_t id = 0; id < n; ++id) build_dual(E, id, b->probs[id].n_reads, cfg->consensus_cost, R->probs[id]);
  double wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  fill_stats(R.get(), E.kernel_ms, E.launches, wall);
  *out = R.release();
  return WC_OK;
}

int wc_consensus_batch(wc_ctx* ctx, const wc_config* cfg, uint32_t n, const wc_problem* problems, wc_results** out) {
  *out = nullptr;
  if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, WC_E_HIP, "hipSetDevice failed");
  return with_batch(ctx, n, problems, [&](wc_batch* b) { return wc_batch_consensus(ctx, b, cfg, out); });
}

int wc_dual_consensus_batch(wc_ctx* ctx, const wc_config* cfg, uint32_t n, const wc_problem* problems,
                            wc_results** out) {
  *out = nullptr;
  if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, WC_E_HIP, "hipSetDevice failed");
  return with_batch(ctx, n, problems, [&](wc_batch* b) { return wc_batch_dual_consensus(ctx, b, cfg, out); });
}

// ---- PriorityConsensusDWFA (priority_consensus.rs:172-341) ----
// Each problem keeps the reference's LIFO work stack; every round takes the
// top item of every problem and runs all of them as one dual-engine batch.
// Within a problem the processing order is exactly the reference's.
int wc_priority_consensus_batch(wc_ctx* ctx, const wc_config* cfg, uint32_t n, const wc_chain_problem* problems,
                                wc_results** out) {
  auto t0 = std::chrono::steady_clock::now();
  *out = nullptr;
  if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, WC_E_HIP, "hipSetDevice failed");
  std::unique_ptr<wc_results> R(new wc_results());
  R->kind = 2;
  R->probs.resize(n);
  std::vector<std::vector<PWork>> stacks(n);
  std::vector<std::vector<std::vector<ConsRec>>> cons(n);
  std::vector<std::vector<std::vector<uint8_t>>> assigns(n);
  std::vector<bool> alive(n, true);
  for (uint32_t i = 0; i < n; ++i) {
    const wc_chain_problem& q = problems[i];
    if (q.n_chains == 0 || q.levels == 0) {
      R->probs[i].status = WC_E_BAD_INPUT;
      R->probs[i].error = "Must provide a non-empty sequences Vec";
      alive[i] = false;
      continue;
    }
    std::vector<int64_t> groups(q.n_chains, -1);
    if (q.seed_groups)
      for (uint32_t c = 0; c < q.n_chains; ++c) groups[c] = q.seed_groups[c] < 0 ? -1 : q.seed_groups[c];
    for (int64_t g : seed_order(groups)) {
      PWork w;
      w.inc.resize(q.n_chains);
      for (uint32_t c = 0; c < q.n_chains; ++c) w.inc[c] = groups[c] == g;
      w.level = 0;
      stacks[i].push_back(std::move(w));
    }
  }
  // Every stacked sub-problem is an independent DualConsensusDWFA over its
  // own reads, so all of them are evaluated in one launch per round, ahead of
  // their turn. The stacks are then unwound in the reference's LIFO order
  // (priority_consensus.rs:195-307) as far as evaluated results reach: the
  // pop order, the chains, their order and the work counters (added when an
  // item is popped) are those of the one-at-a-time loop; the number of rounds
  // drops from the number of sub-problems to the depth of the split tree.
  double kms = 0;
  uint64_t launches = 0;
  for (;;) {
    // unwind: pop evaluated tops in LIFO order
    for (uint32_t i = 0; i < n; ++i) {
      const wc_chain_problem& q = problems[i];
      ProbRes& pr = R->probs[i];
      while (alive[i] && !stacks[i].empty() && stacks[i].back().done) {
        PWork w = std::move(stacks[i].back());
        stacks[i].pop_back();
        const ProbRes& d = *w.res;
        for (int s = 0; s < S_NSTAT; ++s)
          pr.stats[s] = s == S_PEAKQ ? std::max(pr.stats[s], d.stats[s]) : pr.stats[s] + d.stats[s];
        if (d.status != WC_OK) {
          pr.status = d.status;
          pr.error = d.error;
          alive[i] = false;
          break;
        }
        const DualRec& ch = d.dual[0];
        if (ch.has_c2) {
          std::vector<uint8_t> a1(q.n_chains, 0), a2(q.n_chains, 0);
          size_t idx = 0;
          for (uint32_t c = 0; c < q.n_chains; ++c) {
            if (!w.inc[c]) continue;
            if (ch.is_c1[idx]) a1[c] = 1;
            else a2[c] = 1;
            idx++;
          }
          stacks[i].push_back(PWork{a1, w.level, w.chain});
          stacks[i].push_back(PWork{a2, w.level, w.chain});
        } else {
          w.chain.push_back(ch.c1);
          if (w.level + 1 == q.levels) {
            cons[i].push_back(w.chain);
            assigns[i].push_back(w.inc);
          } else {
            stacks[i].push_back(PWork{w.inc, w.level + 1, w.chain});
          }
        }
      }
    }
    // evaluate every stacked, not yet evaluated sub-problem of the live problems
    std::vector<PWork*> items;
    std::vector<uint32_t> owner;
    for (uint32_t i = 0; i < n; ++i) {
      if (!alive[i]) continue;
      for (PWork& w : stacks[i])
        if (!w.done) {
          items.push_back(&w);
          owner.push_back(i);
        }
    }
    if (items.empty()) break;
    std::vector<std::vector<const uint8_t*>> rp(items.size());
    std::vector<std::vector<uint64_t>> rl(items.size());
    std::vector<std::vector<int64_t>> ro(items.size());
    std::vector<wc_problem> sub(items.size());
    for (size_t k = 0; k < items.size(); ++k) {
      const wc_chain_problem& q = problems[owner[k]];
      const PWork& w = *items[k];
      for (uint32_t c = 0; c < q.n_chains; ++c) {
        if (!w.inc[c]) continue;
        rp[k].push_back(q.reads[c * q.levels + w.level]);
        rl[k].push_back(q.lens[c * q.levels + w.level]);
        ro[k].push_back(q.offsets ? q.offsets[c * q.levels + w.level] : -1);
      }
      sub[k].n_reads = (uint32_t)rp[k].size();
      sub[k].reads = rp[k].data();
      sub[k].lens = rl[k].data();
      sub[k].offsets = ro[k].data();
    }
    wc_results* dr = nullptr;
    int rc = wc_dual_consensus_batch(ctx, cfg, (uint32_t)sub.size(), sub.data(), &dr);
    if (rc != WC_OK) return rc;
    std::unique_ptr<wc_results> D(dr);
    kms += D->stats.kernel_ms;
    launches += D->stats.launches;
    for (size_t k = 0; k < items.size(); ++k) {
      items[k]->res.reset(new ProbRes(std::move(D->probs[k])));
      items[k]->done = true;
    }
  }
  for (uint32_t i = 0; i < n; ++i) {
    ProbRes& pr = R->probs[i];
    if (pr.status != WC_OK) continue;
    const uint32_t M = problems[i].n_chains;
    auto& C = cons[i];
    if (C.size() > 1) {
      std::vector<size_t> ord(C.size());
      std::iota(ord.begin(), ord.end(), 0);
      std::stable_sort(ord.begin(), ord.end(), [&](size_t a, size_t b) {
        size_t m = std::min(C[a].size(), C[b].size());
        for (size_t l = 0; l < m; ++l)
          if (C[a][l].seq != C[b][l].seq) return C[a][l].seq < C[b][l].seq;
        return C[a].size() < C[b].size();
      });
      pr.indices.assign(M, UINT64_MAX);
      for (size_t ci = 0; ci < ord.size(); ++ci) {
        for (uint32_t c = 0; c < M; ++c)
          if (assigns[i][ord[ci]][c]) pr.indices[c] = ci;
        pr.chains.push_back(C[ord[ci]]);
      }
    } else {
      pr.chains = C;
      pr.indices.assign(M, 0);
    }
  }
  double wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  fill_stats(R.get(), kms, launches, wall);
  *out = R.release();
  return WC_OK;
}

void wc_results_free(wc_results* r) { delete r; }
uint32_t wc_results_problems(const wc_results* r) { return (uint32_t)r->probs.size(); }
int wc_results_status(const wc_results* r, uint32_t p) { return p < r->probs.size() ? r->probs[p].status : WC_E_BAD_INPUT; }
const char* wc_results_error(const wc_results* r, uint32_t p) {
  return p < r->probs.size() ? r->probs[p].error.c_str() : "no such problem";
}
uint32_t wc_results_count(const wc_results* r, uint32_t p) {
  if (p >= r->probs.size()) return 0;
  const ProbRes& q = r->probs[p];
  if (r->kind == 0) return (uint32_t)q.single.size();
  if (r->kind == 1) return (uint32_t)q.dual.size();
  return (uint32_t)q.chains.size();
}

int wc_results_single(const wc_results* r, uint32_t p, uint32_t k, const uint8_t** seq, uint64_t* seq_len,
                      const uint64_t** scores, uint64_t* n_scores) {
  if (r->kind != 0 || p >= r->probs.size() || k >= r->probs[p].single.size()) return WC_E_BAD_INPUT;
  const ConsRec& c = r->probs[p].single[k];
  *seq = c.seq.data();
  *seq_len = c.seq.size();
  *scores = c.scores.data();
  *n_scores = c.scores.size();
  return WC_OK;
}

int wc_results_dual(const wc_results* r, uint32_t p, uint32_t k, wc_dual_view* o) {
  if (r->kind != 1 || p >= r->probs.size() || k >= r->probs[p].dual.size()) return WC_E_BAD_INPUT;
  const DualRec& d = r->probs[p].dual[k];
  o->seq1 = d.c1.seq.data();
  o->len1 = d.c1.seq.size();
  o->scores_c1 = d.c1.scores.data();
  o->n_scores_c1 = d.c1.scores.size();
  o->has_c2 = d.has_c2;
  o->seq2 = d.c2.seq.data();
  o->len2 = d.c2.seq.size();
  o->scores_c2 = d.c2.scores.data();
  o->n_scores_c2 = d.c2.scores.size();
  o->is_consensus1 = d.is_c1.data();
  o->scores1 = d.s1.data();
  o->scores2 = d.s2.data();
  o->n_reads = d.is_c1.size();
  return WC_OK;
}

uint32_t wc_results_chain_len(const wc_results* r, uint32_t p, uint32_t k) {
  if (r->kind != 2 || p >= r->probs.size() || k >= r->probs[p].chains.size()) return 0;
  return (uint32_t)r->probs[p].chains[k].size();
}

int wc_results_chain(const wc_results* r, uint32_t p, uint32_t k, uint32_t level, const uint8_t** seq,
                     uint64_t* seq_len, const uint64_t** scores, uint64_t* n_scores) {
  if (r->kind != 2 || p >= r->probs.size() || k >= r->probs[p].chains.size() ||
      level >= r->probs[p].chains[k].size())
    return WC_E_BAD_INPUT;
  const ConsRec& c = r->probs[p].chains[k][level];
  *seq = c.seq.data();
  *seq_len = c.seq.size();
  *scores = c.scores.data();
  *n_scores = c.scores.size();
  return WC_OK;
}

int wc_results_sequence_indices(const wc_results* r, uint32_t p, const uint64_t** idx, uint64_t* n) {
  if (r->kind != 2 || p >= r->probs.size()) return WC_E_BAD_INPUT;
  *idx = r->probs[p].indices.data();
  *n = r->probs[p].indices.size();
  return WC_OK;
}

int wc_results_stats(const wc_results* r, wc_stats* out) {
  *out = r->stats;
  return WC_OK;
}

int wc_results_problem_stats(const wc_results* r, uint32_t p, wc_stats* o) {
  if (p >= r->probs.size()) return WC_E_BAD_INPUT;
  memset(o, 0, sizeof(*o));
  const uint64_t* s = r->probs[p].stats;
  o->updates = s[S_UPDATES];
  o->w_out = s[S_WOUT];
  o->compares = s[S_COMPARES];
  o->ed_increases = s[S_EDINC];
  o->finalizes = s[S_FINALIZES];
  o->pops = s[S_POPS];
  o->nodes_explored = s[S_EXPLORED];
  o->nodes_ignored = s[S_IGNORED];
  o->peak_queue_size = s[S_PEAKQ];
  return WC_OK;
}

// ---- standalone DWFALite batch (dynamic_wfa.rs:48-265) ----
int wc_dwfa_batch(wc_ctx* ctx, uint32_t n, wc_dwfa_job* jobs) {
  if (n == 0) return WC_OK;
  if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, WC_E_HIP, "hipSetDevice failed");
  // one arena: per job baseline | other | wavefront (u32, cap)
  std::vector<uint64_t> boff(n), ooff(n), woff(n);
  uint64_t total = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (jobs[i].wf_cap < jobs[i].wf_len || jobs[i].wf_len != 2 * jobs[i].e + 1)
      return set_err(ctx, WC_E_BAD_INPUT, "wavefront length must be 2e+1 and fit wf_cap");
    boff[i] = total;
    total += (jobs[i].baseline_len + 15) & ~15ull;
    ooff[i] = total;
    total += (jobs[i].other_len + 15) & ~15ull;
    woff[i] = total;
    total += (jobs[i].wf_cap * 4 + 15) & ~15ull;
  }
  // reads start 16-byte aligned; 64 bytes of tail padding let the engine load
  // 64-byte windows with 16-byte accesses anywhere inside a read
  std::vector<uint8_t> h(total + 64);
  std::vector<DwfaDevJob> dj(n);
  for (uint32_t i = 0; i < n; ++i) {
    const wc_dwfa_job& j = jobs[i];
    if (j.baseline_len) memcpy(h.data() + boff[i], j.baseline, j.baseline_len);
    if (j.other_len) memcpy(h.data() + ooff[i], j.other, j.other_len);
    uint32_t* wf = (uint32_t*)(h.data() + woff[i]);
    for (uint64_t k = 0; k < j.wf_len; ++k) wf[k] = (uint32_t)j.wavefront[k];
  }
  DevBuf arena;
  if (!arena.ensure(h.size()) || !ctx->jobs.ensure(n * sizeof(DwfaDevJob)))
    return set_err(ctx, WC_E_HIP, "device allocation failed (dwfa)");
  uint8_t* base = (uint8_t*)arena.p;
  for (uint32_t i = 0; i < n; ++i) {
    const wc_dwfa_job& j = jobs[i];
    DwfaDevJob& d = dj[i];
    memset(&d, 0, sizeof(d));
    d.baseline = base + boff[i];
    d.blen = (uint32_t)j.baseline_len;
    d.other = base + ooff[i];
    d.olen = (uint32_t)j.other_len;
    d.offset = (uint32_t)j.offset;
    d.wildcard = j.wildcard;
    d.early = j.early;
    d.op = j.op;
    d.e = (uint32_t)j.e;
    d.wf = (uint32_t*)(base + woff[i]);
    d.wf_cap = (uint32_t)j.wf_cap;
  }
  int rc = WC_OK;
  do {
    if (hipMemcpyAsync(arena.p, h.data(), h.size(), hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
        hipMemcpyAsync(ctx->jobs.p, dj.data(), n * sizeof(DwfaDevJob), hipMemcpyHostToDevice, ctx->stream) !=
            hipSuccess) {
      rc = set_err(ctx, WC_E_HIP, "copy to device failed (dwfa)");
      break;
    }
    launch_dwfa_jobs((DwfaDevJob*)ctx->jobs.p, n, ctx->stream);
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(ctx->stream) != hipSuccess ||
        hipMemcpy(dj.data(), ctx->jobs.p, n * sizeof(DwfaDevJob), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(h.data(), arena.p, h.size(), hipMemcpyDeviceToHost) != hipSuccess) {
      rc = set_err(ctx, WC_E_HIP, "dwfa kernel failed");
      break;
    }
    for (uint32_t i = 0; i < n; ++i) {
      wc_dwfa_job& j = jobs[i];
      const DwfaDevJob& d = dj[i];
      j.status = (int32_t)d.status;
      if (d.status != 0) continue;
      j.e = d.e;
      const uint32_t W = 2 * d.e + 1;
      j.wf_len = W;
      const uint32_t* wf = (const uint32_t*)(h.data() + woff[i]);
      for (uint32_t k = 0; k < W && k < j.wf_cap; ++k) j.wavefront[k] = wf[k];
      j.n_cand = d.n_cand;
      for (uint32_t k = 0; k < d.n_cand && k < 16; ++k) {
        j.cand_syms[k] = d.cand_syms[k];
        j.cand_counts[k] = d.cand_counts[k];
      }
    }
  } while (0);
  arena.release();
  return rc;
}

// ---- batched wfa_ed_config (sequence_alignment.rs:18-87) ----
// Pairs go to the device in launches whose sequence arena + scratch rows stay
// under kEdLaunchBytes (a single larger pair gets a launch of its own).
int wc_wfa_ed_batch(wc_ctx* ctx, uint32_t n, const uint8_t* const* v1, const uint64_t* l1, const uint8_t* const* v2,
                    const uint64_t* l2, uint8_t require_both_end, int32_t wildcard, uint64_t* out_ed) {
  if (n == 0) return WC_OK;
  if (!v1 || !l1 || !v2 || !l2 || !out_ed) return set_err(ctx, WC_E_BAD_INPUT, "wc_wfa_ed_batch: null argument");
  for (uint32_t i = 0; i < n; ++i) {
    if (l1[i] >= (1ull << 31) || l2[i] >= (1ull << 31))
      return set_err(ctx, WC_E_BAD_INPUT, "wc_wfa_ed_batch: sequence length must be < 2^31");
    if ((l1[i] && !v1[i]) || (l2[i] && !v2[i])) return set_err(ctx, WC_E_BAD_INPUT, "wc_wfa_ed_batch: null sequence");
  }
  if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, WC_E_HIP, "hipSetDevice failed");
  constexpr uint64_t kEdLaunchBytes = 1ull << 30;
  auto a16 = [](uint64_t x) { return (x + 15) & ~15ull; };
  auto cap_of = [&](uint32_t i) { return 2 * (l1[i] + l2[i]) + 3; };
  DevBuf arena, scratch, jobs, out;
  int rc = WC_OK;
  for (uint32_t b = 0; b < n && rc == WC_OK;) {
    // [b, e): pairs of this launch
    uint32_t e = b;
    uint64_t sbytes = 0, sents = 0;
    while (e < n) {
      const uint64_t add = a16(l1[e]) + a16(l2[e]), ents = 2 * cap_of(e);
      if (e > b && sbytes + add + 8 * (sents + ents) > kEdLaunchBytes) break;
      sbytes += add;
      sents += ents;
      ++e;
    }
    const uint32_t m = e - b;
    std::vector<uint8_t> h(sbytes + 16);
    std::vector<EdDevJob> dj(m);
    uint64_t so = 0, eo = 0;
    for (uint32_t k = 0; k < m; ++k) {
      const uint32_t i = b + k;
      EdDevJob& d = dj[k];
      d.v1_off = so;
      if (l1[i]) memcpy(h.data() + so, v1[i], l1[i]);
      so += a16(l1[i]);
      d.v2_off = so;
      if (l2[i]) memcpy(h.data() + so, v2[i], l2[i]);
      so += a16(l2[i]);
      d.l1 = (uint32_t)l1[i];
      d.l2 = (uint32_t)l2[i];
      d.cap = cap_of(i);
      d.scr_off = eo;
      eo += 2 * d.cap;
    }
    if (!arena.ensure(h.size()) || !scratch.ensure(8 * eo) || !jobs.ensure(m * sizeof(EdDevJob)) ||
        !out.ensure(8ull * m)) {
      rc = set_err(ctx, WC_E_HIP, "device allocation failed (wfa_ed batch)");
      break;
    }
    if (hipMemcpyAsync(arena.p, h.data(), h.size(), hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
        hipMemcpyAsync(jobs.p, dj.data(), m * sizeof(EdDevJob), hipMemcpyHostToDevice, ctx->stream) != hipSuccess) {
      rc = set_err(ctx, WC_E_HIP, "copy to device failed (wfa_ed batch)");
      break;
    }
    launch_wfa_ed_batch((const EdDevJob*)jobs.p, m, (const uint8_t*)arena.p, (uint64_t*)scratch.p, (int)wildcard,
                        require_both_end ? 1u : 0u, (uint64_t*)out.p, ctx->stream);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(out_ed + b, out.p, 8ull * m, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
        hipStreamSynchronize(ctx->stream) != hipSuccess) {
      rc = set_err(ctx, WC_E_HIP, "wfa_ed kernel failed");
      break;
    }
    for (uint32_t k = 0; k < m; ++k)
      if (out_ed[b + k] == ~0ull) {
        rc = set_err(ctx, WC_E_LIMIT, "wfa_ed scratch row too short");
        break;
      }
    b = e;
  }
  arena.release();
  scratch.release();
  jobs.release();
  out.release();
  return rc;
}

// ---- generator ----
struct wc_gen {
  std::vector<uint8_t> consensus;
  std::vector<std::vector<uint8_t>> samples;
};

int wc_generate_test(uint8_t alphabet, uint64_t seq_len, uint64_t num_samples, double error_rate, uint64_t seed,
                     wc_gen** handle) {
  if (alphabet < 2 || !(error_rate >= 0.0 && error_rate <= 1.0)) return WC_E_BAD_INPUT;
  wc_gen* g = new wc_gen();
  wc::generate_test(alphabet, seq_len, num_samples, error_rate, seed, g->consensus, g->samples);
  *handle = g;
  return WC_OK;
}
const uint8_t* wc_gen_consensus(const wc_gen* g, uint64_t* len) {
  *len = g->consensus.size();
  return g->consensus.data();
}
const uint8_t* wc_gen_sample(const wc_gen* g, uint64_t i, uint64_t* len) {
  if (i >= g->samples.size()) {
    *len = 0;
    return nullptr;
  }
  *len = g->samples[i].size();
  return g->samples[i].data();
}
void wc_gen_free(wc_gen* g) { delete g; }

}  // extern "C"
