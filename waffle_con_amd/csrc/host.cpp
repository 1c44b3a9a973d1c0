// Host orchestration and C ABI of the waffle_con MI355X library.
//
// A batch call packs every problem's reads into one HBM arena, launches the
// device-resident engine once for the whole batch (one workgroup per problem,
// persistent grid pulling problems from an atomic counter, longest problems
// first), and turns the device result records into the reference's result
// types (Consensus, DualConsensus, PriorityConsensus). Problems that outgrow
// a device capacity (wavefront length, node pool, consensus length) are
// re-run with doubled capacities; no work is ever done on the CPU instead.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstring>
#include <memory>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/waffle_con.h"
#include "engine_shared.hpp"
#include "waffle_con_internal.hpp"

namespace wc {
void launch_single_engine(const EngineArgs& a, uint32_t grid, size_t lds, hipStream_t s);
void launch_dual_engine(const EngineArgs& a, uint32_t grid, size_t lds, hipStream_t s);
int engine_blocks_per_cu(uint32_t sides, size_t lds);
}  // namespace wc

using namespace wc;

// ------------------------------------------------------------------------
// context
// ------------------------------------------------------------------------
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  bool ensure(size_t bytes) {
    if (bytes <= cap) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes, 1 << 20);
    if (hipMalloc(&p, want) != hipSuccess) return false;
    cap = want;
    return true;
  }
  void release() {
    if (p) (void)hipFree(p);
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
  DevBuf reads, roff, rlen, ract, probs, ws, out, status, stats, counter;
};

namespace {
const char* err_msg(int code) {
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
    case WC_E_LIMIT: return "device capacity limit exceeded";
    case WC_E_HIP: return "HIP runtime failure";
    default: return "ok";
  }
}

inline int set_err(wc_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

#define HIPCHK(call)                                                                             \
  do {                                                                                           \
    hipError_t _e = (call);                                                                      \
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

// ------------------------------------------------------------------------
// engine batch runner (shared by single and dual)
// ------------------------------------------------------------------------
namespace {
struct PackedProblem {
  std::vector<const uint8_t*> reads;
  std::vector<uint64_t> lens;
  std::vector<int64_t> activate;  // activation length or -1
  uint32_t n_active = 0;
};

// auto_shift_offsets + activation points (consensus.rs:151-202)
int prepare_problem(const wc_config& cfg, const wc_problem& p, PackedProblem& out, std::string& err) {
  if (p.n_reads == 0) {
    err = "No sequences provided";
    return WC_E_BAD_INPUT;
  }
  out.reads.assign(p.reads, p.reads + p.n_reads);
  out.lens.assign(p.lens, p.lens + p.n_reads);
  std::vector<int64_t> offs(p.n_reads, -1);
  if (p.offsets)
    for (uint32_t i = 0; i < p.n_reads; ++i) offs[i] = p.offsets[i];
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
  out.activate.assign(p.n_reads, -1);
  out.n_active = 0;
  for (uint32_t i = 0; i < p.n_reads; ++i) {
    if (offs[i] >= 0) out.activate[i] = offs[i] + (int64_t)cfg.offset_compare_length;
    else out.n_active++;
  }
  if (out.n_active == 0) {
    err = err_msg(WC_E_NO_START);
    return WC_E_NO_START;
  }
  for (uint32_t i = 0; i < p.n_reads; ++i) {
    if (out.activate[i] >= 0) {
      err = "activation offsets (add_sequence_offset) are not supported by this build's device engine yet";
      return WC_E_LIMIT;
    }
  }
  return WC_OK;
}

struct RawRecord {
  uint32_t len[2];
  bool dual;
  std::vector<uint8_t> con[2];
  std::vector<uint32_t> fe[2];
};

// Runs problems `ids` of `pp` through the engine; fills raw records/status/stats.
int run_engine(wc_ctx* ctx, const wc_config& cfg, uint32_t sides, const std::vector<PackedProblem>& pp,
               std::vector<uint32_t> ids, std::vector<std::vector<RawRecord>>& recs, std::vector<int>& status,
               std::vector<std::array<uint64_t, S_NSTAT>>& stats, double& kernel_ms, uint64_t& launches) {
  // capacities
  uint32_t nmax = 1, maxlen = 1;
  for (uint32_t id : ids) {
    nmax = std::max<uint32_t>(nmax, (uint32_t)pp[id].reads.size());
    for (auto l : pp[id].lens) maxlen = std::max<uint32_t>(maxlen, (uint32_t)l);
  }
  uint32_t ecap = std::max<uint32_t>(31, maxlen / 64);
  uint32_t wcap = ((2 * ecap + 1 + 63) / 64) * 64;
  uint32_t lcap = ((maxlen + maxlen / 8 + 64 + 15) / 16) * 16;
  uint32_t pcap = sides == 1 ? 16 : 64;
  const uint32_t rmax = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(cfg.max_return_size, 1), 256);

  for (int attempt = 0; attempt < 8 && !ids.empty(); ++attempt) {
    // longest problems first (cost ~ n_reads * len)
    std::sort(ids.begin(), ids.end(), [&](uint32_t a, uint32_t b) {
      uint64_t ca = 0, cb = 0;
      for (auto l : pp[a].lens) ca += l;
      for (auto l : pp[b].lens) cb += l;
      return ca > cb;
    });
    const uint32_t P = (uint32_t)ids.size();
    // pack reads
    std::vector<DevProblem> dp(P);
    std::vector<uint64_t> roff;
    std::vector<uint32_t> rlen;
    std::vector<int64_t> ract;
    uint64_t total = 0;
    for (uint32_t i = 0; i < P; ++i)
      for (auto l : pp[ids[i]].lens) total += (l + 15) & ~15ull;
    std::vector<uint8_t> hreads(std::max<uint64_t>(total, 16));
    uint64_t pos = 0;
    for (uint32_t i = 0; i < P; ++i) {
      const PackedProblem& q = pp[ids[i]];
      dp[i].read_begin = (uint32_t)roff.size();
      dp[i].n_reads = (uint32_t)q.reads.size();
      dp[i].n_active = q.n_active;
      uint32_t ml = 0;
      for (size_t r = 0; r < q.reads.size(); ++r) {
        roff.push_back(pos);
        rlen.push_back((uint32_t)q.lens[r]);
        ract.push_back(q.activate[r]);
        if (q.lens[r]) memcpy(hreads.data() + pos, q.reads[r], q.lens[r]);
        pos += (q.lens[r] + 15) & ~15ull;
        ml = std::max<uint32_t>(ml, (uint32_t)q.lens[r]);
      }
      dp[i].max_read_len = ml;
    }
    size_t lds = (size_t)lds_bytes(sides, pcap, nmax);
    if (lds > 160 * 1024 - 4096) return set_err(ctx, WC_E_LIMIT, "problem needs more LDS than a CU has");
    int per_cu = engine_blocks_per_cu(sides, lds);
    uint32_t grid = std::min<uint32_t>(P, (uint32_t)std::max(1, per_cu) * (uint32_t)ctx->n_cu);
    uint64_t wsb = ws_bytes(sides, pcap, nmax, wcap, lcap);
    uint64_t ob = out_bytes(sides, rmax, nmax, lcap);
    if (!ctx->reads.ensure(hreads.size()) || !ctx->roff.ensure(roff.size() * 8) || !ctx->rlen.ensure(rlen.size() * 4) ||
        !ctx->ract.ensure(ract.size() * 8) || !ctx->probs.ensure(P * sizeof(DevProblem)) ||
        !ctx->ws.ensure(wsb * grid) || !ctx->out.ensure(ob * P) || !ctx->status.ensure(P * 4) ||
        !ctx->stats.ensure((size_t)P * S_NSTAT * 8) || !ctx->counter.ensure(4))
      return set_err(ctx, WC_E_HIP, "device allocation failed");
    HIPCHK(hipMemcpyAsync(ctx->reads.p, hreads.data(), hreads.size(), hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(ctx->roff.p, roff.data(), roff.size() * 8, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(ctx->rlen.p, rlen.data(), rlen.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(ctx->ract.p, ract.data(), ract.size() * 8, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(ctx->probs.p, dp.data(), P * sizeof(DevProblem), hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemsetAsync(ctx->counter.p, 0, 4, ctx->stream));
    HIPCHK(hipMemsetAsync(ctx->out.p, 0, 16, ctx->stream));

    EngineArgs a;
    memset(&a, 0, sizeof(a));
    a.cfg = to_dev(cfg);
    a.problems = (const DevProblem*)ctx->probs.p;
    a.n_problems = P;
    a.sides = sides;
    a.rbytes = (const uint8_t*)ctx->reads.p;
    a.roff = (const uint64_t*)ctx->roff.p;
    a.rlen = (const uint32_t*)ctx->rlen.p;
    a.ractivate = (const int64_t*)ctx->ract.p;
    a.ws = (uint8_t*)ctx->ws.p;
    a.ws_stride = wsb;
    a.pcap = pcap;
    a.wcap = wcap;
    a.lcap = lcap;
    a.nmax = nmax;
    a.rmax = rmax;
    a.out = (uint8_t*)ctx->out.p;
    a.out_stride = ob;
    a.status = (uint32_t*)ctx->status.p;
    a.stats = (uint64_t*)ctx->stats.p;
    a.work_counter = (uint32_t*)ctx->counter.p;

    HIPCHK(hipEventRecord(ctx->ev0, ctx->stream));
    if (sides == 1) launch_single_engine(a, grid, lds, ctx->stream);
    else launch_dual_engine(a, grid, lds, ctx->stream);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(ctx->ev1, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    kernel_ms += ms;
    launches++;

    std::vector<uint32_t> hst(P);
    std::vector<uint64_t> hstats((size_t)P * S_NSTAT);
    std::vector<uint8_t> hout(ob * P);
    HIPCHK(hipMemcpy(hst.data(), ctx->status.p, P * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(hstats.data(), ctx->stats.p, hstats.size() * 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(hout.data(), ctx->out.p, hout.size(), hipMemcpyDeviceToHost));

    std::vector<uint32_t> retry;
    uint32_t rflags = 0;
    const uint64_t rb = result_bytes(sides, nmax, lcap);
    for (uint32_t i = 0; i < P; ++i) {
      const uint32_t id = ids[i];
      const uint32_t st = hst[i];
      for (int s = 0; s < S_NSTAT; ++s) stats[id][s] = hstats[(size_t)i * S_NSTAT + s];
      if (st & ST_RETRY) {
        retry.push_back(id);
        rflags |= st;
        continue;
      }
      status[id] = (int)st;
      if (st != ST_OK) continue;
      const uint8_t* base = hout.data() + (size_t)i * ob;
      uint32_t nres = ((const uint32_t*)base)[0];
      const uint32_t n = (uint32_t)pp[id].reads.size();
      recs[id].clear();
      for (uint32_t k = 0; k < nres; ++k) {
        const uint8_t* rec = base + 16 + k * rb;
        const uint32_t* h = (const uint32_t*)rec;
        RawRecord R;
        R.len[0] = h[0];
        R.len[1] = h[1];
        R.dual = h[2] != 0;
        for (uint32_t s = 0; s < sides; ++s) {
          const uint8_t* con = rec + 16 + s * align16(lcap);
          R.con[s].assign(con, con + R.len[s]);
          const uint32_t* fe = (const uint32_t*)(rec + 16 + sides * align16(lcap) + s * align16((uint64_t)nmax * 4));
          R.fe[s].assign(fe, fe + n);
        }
        recs[id].push_back(std::move(R));
      }
    }
    ids = retry;
    if (rflags & ST_RETRY_WCAP) wcap = wcap * 2;
    if (rflags & (ST_RETRY_PCAP | ST_RETRY_HEAP)) pcap = pcap * 4;
    if (rflags & ST_RETRY_LCAP) lcap = lcap * 2;
  }
  for (uint32_t id : ids) status[id] = WC_E_LIMIT;
  return WC_OK;
}

std::vector<PackedProblem> prepare_all(const wc_config& cfg, uint32_t n, const wc_problem* problems,
                                       std::vector<ProbRes>& res, std::vector<uint32_t>& runnable) {
  std::vector<PackedProblem> pp(n);
  for (uint32_t i = 0; i < n; ++i) {
    std::string err;
    int rc = prepare_problem(cfg, problems[i], pp[i], err);
    if (rc != WC_OK) {
      res[i].status = rc;
      res[i].error = err;
    } else {
      runnable.push_back(i);
    }
  }
  return pp;
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
  wc_ctx* ctx = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return WC_E_HIP;
  if (device < 0 || device >= ndev) return WC_E_HIP;
  if (hipSetDevice(device) != hipSuccess) return WC_E_HIP;
  ctx = new wc_ctx();
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
  for (DevBuf* b : {&ctx->reads, &ctx->roff, &ctx->rlen, &ctx->ract, &ctx->probs, &ctx->ws, &ctx->out, &ctx->status,
                    &ctx->stats, &ctx->counter})
    b->release();
  if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
  if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

const char* wc_last_error(const wc_ctx* ctx) { return ctx ? ctx->err.c_str() : "no context"; }

int wc_consensus_batch(wc_ctx* ctx, const wc_config* cfg, uint32_t n, const wc_problem* problems, wc_results** out) {
  auto t0 = std::chrono::steady_clock::now();
  *out = nullptr;
  if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, WC_E_HIP, "hipSetDevice failed");
  std::unique_ptr<wc_results> R(new wc_results());
  R->kind = 0;
  R->probs.resize(n);
  std::vector<uint32_t> runnable;
  std::vector<PackedProblem> pp = prepare_all(*cfg, n, problems, R->probs, runnable);
  std::vector<std::vector<RawRecord>> recs(n);
  std::vector<int> status(n, WC_OK);
  std::vector<std::array<uint64_t, S_NSTAT>> stats(n);
  for (auto& s : stats) s.fill(0);
  double kms = 0;
  uint64_t launches = 0;
  if (!runnable.empty()) {
    int rc = run_engine(ctx, *cfg, 1, pp, runnable, recs, status, stats, kms, launches);
    if (rc != WC_OK) return rc;
  }
  for (uint32_t id : runnable) {
    ProbRes& pr = R->probs[id];
    for (int s = 0; s < S_NSTAT; ++s) pr.stats[s] = stats[id][s];
    pr.status = status[id];
    if (pr.status != WC_OK) {
      pr.error = err_msg(pr.status);
      continue;
    }
    for (auto& rr : recs[id]) {
      ConsRec c;
      c.seq = rr.con[0];
      for (auto e : rr.fe[0]) c.scores.push_back(cost_of_h(e, cfg->consensus_cost));
      pr.single.push_back(std::move(c));
    }
    // consensus.rs:345 — sort by sequence
    std::stable_sort(pr.single.begin(), pr.single.end(),
                     [](const ConsRec& a, const ConsRec& b) { return a.seq < b.seq; });
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

// ---- temporary entry points (implemented in the next milestone) ----
extern "C" {
int wc_dual_consensus_batch(wc_ctx* ctx, const wc_config*, uint32_t, const wc_problem*, wc_results** out) {
  *out = nullptr;
  return set_err(ctx, WC_E_LIMIT, "dual engine not built yet");
}
int wc_priority_consensus_batch(wc_ctx* ctx, const wc_config*, uint32_t, const wc_chain_problem*, wc_results** out) {
  *out = nullptr;
  return set_err(ctx, WC_E_LIMIT, "priority engine not built yet");
}
int wc_dwfa_batch(wc_ctx* ctx, uint32_t, wc_dwfa_job*) { return set_err(ctx, WC_E_LIMIT, "dwfa batch not built yet"); }
}
