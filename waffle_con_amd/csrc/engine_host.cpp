// Host side of the device engines: capacity planning, engine launches (each
// with its own stream, buffers and host-mapped result area), the synchronous
// batch runner, and the streamed PriorityConsensusDWFA scheduler.
//
// Results, status and work counters of every problem are written by the
// engine straight into fine-grained host memory, followed by a system-scope
// completion flag (engine.hip finish_problem). The host can therefore consume
// a problem the moment it finishes, while the rest of its launch still runs.
// The priority scheduler uses that to keep the GPU busy: the children of a
// finished DualConsensusDWFA sub-problem go into the next launch right away
// (up to kSlots launches in flight), instead of waiting for the slowest
// sub-problem of a round. The LIFO stack discipline of the reference
// (priority_consensus.rs:195-307) is preserved by unwinding each problem's
// stack only through finished tops.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <deque>
#include <memory>
#include <numeric>
#include <queue>
#include <thread>

#include <mutex>

#include <hsa/hsa_ext_amd.h>

#include "sched.hpp"

using namespace wc;

namespace {
std::mutex g_persist_mu;
int g_persist_running = 0;
std::vector<std::pair<void*, bool>> g_parked;  // buffers freed while a persistent launch ran
}  // namespace

void persistent_begin() {
  std::lock_guard<std::mutex> g(g_persist_mu);
  g_persist_running++;
}
// The parked buffers are freed under the lock: a persistent_begin on another
// thread (and the launch that follows it) waits for these frees, which would
// otherwise wait for that new persistent kernel (the deadlock the deferral
// exists to prevent).
void persistent_end() {
  std::lock_guard<std::mutex> g(g_persist_mu);
  if (--g_persist_running > 0) return;
  for (auto& b : g_parked) (void)(b.second ? hipHostFree(b.first) : hipFree(b.first));
  g_parked.clear();
}
// Every free of a device or pinned buffer goes through here: parked while a
// persistent launch runs, else freed at once, under the same lock, so that no
// persistent_begin (and the launch after it) can start while a free is in
// flight. Always takes ownership (returns true).
bool free_deferred(void* p, bool host) {
  std::lock_guard<std::mutex> g(g_persist_mu);
  if (g_persist_running > 0) g_parked.emplace_back(p, host);
  else (void)(host ? hipHostFree(p) : hipFree(p));
  return true;
}

namespace wch {

constexpr uint32_t kLdsMax = 160 * 1024;  // one workgroup may take the whole CU's LDS

// HBM the node pools of one launch may take: `frac` of what is free plus the
// launch's own cached workspace (reused by the launch), and never more than
// `frac` of this context's share of the device (WC_DEVICE_SHARE processes on
// one GPU each plan for 1/share of its HBM, not for whatever is free when they
// happen to look)
uint64_t hbm_share(const wc_ctx* ctx, uint64_t cached, double frac) {
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) fr = tot = 32ull << 30;
  const double avail = std::min((double)fr + (double)cached, (double)tot / std::max(1, ctx->share));
  return (uint64_t)(avail * frac);
}

// Capacities of one launch over items[ids] (SURVEY §8(a) sizes): wavefront row
// capacity from the longest read, consensus capacity from the longest read,
// node-pool slots from the HBM share, linear-chain length from the LDS left at
// the same occupancy. Retry outcomes raise them per item (log2 multipliers).
int plan_caps(wc_ctx* ctx, const wc_config& cfg, uint32_t sides, const std::vector<SubProb>& items,
                     const std::vector<uint32_t>& ids, uint64_t hbm_budget, Caps& c, std::string& err,
                     uint32_t max_per_cu, bool cu_ok) {
  uint32_t nmax = 1, maxlen = 1, wx = 0, px = 0, lx = 0, rx = 0;
  bool any_act = false;
  for (uint32_t id : ids) {
    const SubProb& s = items[id];
    nmax = std::max<uint32_t>(nmax, (uint32_t)s.gid.size());
    maxlen = std::max(maxlen, s.max_len);
    wx = std::max<uint32_t>(wx, s.wcap_x);
    px = std::max<uint32_t>(px, s.pcap_x);
    lx = std::max<uint32_t>(lx, s.lcap_x);
    rx = std::max<uint32_t>(rx, s.rmax_x);
    any_act |= s.max_act > 0;
  }
  c.sides = sides;
  c.nmax = nmax;
  const uint32_t ecap = std::max<uint32_t>(31, maxlen / 64);
  c.wcap = (((2 * ecap + 1 + 63) / 64) * 64) << wx;
  c.lcap = (((maxlen + maxlen / 8 + 64 + 15) / 16) * 16) << lx;
  // linear-chain run-ahead length (WC_CHAIN=<k> overrides, 0 = off). The dual
  // engine runs chains from single-consensus nodes (WC_DUAL_CHAIN=<k>, 0 =
  // off) when min_af is 0: its child threshold is then the single engine's
  // (dual_consensus.rs:655-679 with min_count = cfg.min_count)
  uint32_t chain = 0;
  const char* chain_env = getenv(sides == 1 ? "WC_CHAIN" : "WC_DUAL_CHAIN");
  if (nmax <= (uint32_t)kBlock && (sides == 1 || cfg.min_af == 0.0)) {
    chain = sides == 1 ? kChainDefault : kDualChainDefault;
    if (chain_env) chain = std::min<uint32_t>((uint32_t)atoi(chain_env), kChainMax);
    if (chain == 1) chain = 0;  // a chain takes at least 2 steps
  }
  // node pool. A dual search keeps far more nodes queued than a single one
  // (children of both consensuses, both sides' DWFAs per node: cfg3 loci peak
  // at ~480 queued nodes), so the dual pool gets the launch's HBM share over
  // the workgroups that can run at once (16..256 MiB each).
  const uint64_t sb = slot_bytes(sides, nmax, c.wcap, c.lcap);
  const uint64_t conc = std::max<uint64_t>(1, std::min<uint64_t>(ids.size(), (uint64_t)max_per_cu * ctx->n_cu));
  const uint64_t per_wg = std::max<uint64_t>(16ull << 20, hbm_budget / conc);
  const uint64_t budget = sides == 1 ? (16ull << 20) : std::min<uint64_t>(256ull << 20, per_wg);
  uint32_t pmax = sides == 1 ? 256u : 1024u;
  if (const char* e = getenv("WC_SINGLE_PMAX"))  // experiment hook: the single engine's first pool size cap
    if (sides == 1) pmax = std::max<uint32_t>(16u, (uint32_t)atoi(e));
  uint64_t lmax = sides == 1 ? 40 * 1024 : 52 * 1024;  // dual: still 3 workgroups per CU
  if (const char* e = getenv("WC_DUAL_LDS_KB"))  // experiment hook: LDS budget of the dual node pool
    if (sides == 2) lmax = (uint64_t)atoi(e) * 1024;
  // WC_GSTATE=1 (test hook) forces the global-state build for every launch
  bool gstate = getenv("WC_GSTATE") != nullptr;
  auto base_pool = [&]() {
    uint32_t p = 16;
    while (p < pmax && (uint64_t)(p * 2) * sb <= budget && (gstate || lds_bytes(sides, p * 2, nmax, chain) <= lmax))
      p *= 2;
    return p;
  };
  // the dual engine's chain area (both sides' windows, nominations and hot
  // RStates) comes out of the node pool's LDS: a launch with chains gets its
  // own LDS budget (WC_DUAL_CHAIN_LDS_KB) and keeps them while the pool
  // still has 128 slots (a pool that outgrows it retries larger, as always)
  const uint64_t lmax0 = lmax;
  if (sides == 2 && chain > 0 && !gstate)
    if (const char* e = getenv("WC_DUAL_CHAIN_LDS_KB")) lmax = (uint64_t)atoi(e) * 1024;
  uint32_t pcap = base_pool();
  if (sides == 2 && chain > 0 && !gstate && pcap < 128) {
    chain = 0;
    lmax = lmax0;
    pcap = base_pool();
  }
  // a retried (pool-exhausted) item gets 4x per retry, as HBM allows; past
  // what LDS holds, the search state moves to HBM
  c.pool_short = false;
  for (uint32_t k = 0; k < px; ++k) {
    const uint32_t np = pcap * 2;
    if ((uint64_t)np * sb > std::max<uint64_t>(budget, per_wg)) {
      c.pool_short = true;
      break;
    }
    pcap = np;
  }
  if (lds_bytes(sides, pcap, nmax, chain) > kLdsMax) gstate = true;
  if (gstate && sides == 2) chain = 0;  // the global-state dual build runs no chains
  // 128-thread workgroups for problems of <= 128 reads (engine_narrow.hip):
  // for the dual engine (WC_NARROW: bit 0 single engine, bit 1 dual engine;
  // default 2). The single engine's chain walk is faster with 4 waves of
  // fewer reads each: its quiet-step runs are longer (cfg2 34.4 vs 37.1 ms)
  const char* nenv = getenv("WC_NARROW");
  const int nmode = nenv ? atoi(nenv) : 2;
  c.narrow = !gstate && nmax <= 128 && (nmode & (sides == 1 ? 1 : 2)) != 0;
  // a launch of at most 2 problems per CU gets the 2-wave register budget
  // (no spills: each workgroup's latency is what counts); WC_LOWLAT=0 disables
  const char* lenv = getenv("WC_LOWLAT");
  c.lowlat = !gstate && !c.narrow && ids.size() <= 2ull * (uint64_t)ctx->n_cu && !(lenv && atoi(lenv) == 0);
  if (sides == 2 && chain > 0 && !gstate) c.narrow = c.lowlat = false;  // the chain build (wcd)
  // a batch launch of at most one problem per CU runs the 1024-thread single
  // engine (engine_cu.hip): one workgroup of 16 waves per problem, so a
  // chain walk's reads and their edit-distance increases spread over 16 waves
  // instead of 4. WC_CU=0 disables it, WC_CU=1 forces it (test hook)
  const char* wenv = getenv("WC_CU");
  const int wmode = wenv ? atoi(wenv) : 2;
  // (The dual engine has no whole-CU build since round 5: measured slower on
  // one deep locus, cfg4 24.6 vs 22.8 s, and at 16 waves of 128 VGPRs with
  // 110 spilled it diverged under unrelated changes of shared code)
  const bool cu_fit = !gstate && wmode != 0 && (wmode == 1 || ids.size() <= (uint64_t)ctx->n_cu);
  c.cu = cu_ok && cu_fit && sides == 1 && chain > 0;
  if (c.cu) c.narrow = c.lowlat = false;
  // The dual engine on one wave per problem (engine_wave.hip): dual searches
  // without offsets of at most 128 reads, whose popped node stays in LDS with
  // its tip bytes in registers. The default for them: cfg5
  // locus 5949's critical path 17.2 -> 12.7 s, cfg3 210 -> 212 loci/s.
  // WC_WAVE=0 keeps them on the block engines.
  const char* wvenv = getenv("WC_WAVE");
  c.wave = sides == 2 && chain == 0 && !gstate && !any_act && nmax <= 128 && !(wvenv && atoi(wvenv) == 0) &&
           lds_bytes(sides, pcap, nmax, 0, 1) <= kLdsMax;
  if (c.wave) c.narrow = c.lowlat = c.cu = false;
  // The same search on cooperating waves (engine_coop.hip): one read per lane
  // over wcc::engine_waves() waves, for dual searches without offsets of
  // 65-256 reads in a launch whose latency is what counts (at most one
  // problem per CU: a PriorityConsensusDWFA call on one locus, a deep locus
  // alone). WC_COOP=0 disables it, WC_COOP=1 takes it for every dual launch
  // without offsets of at most 256 reads (a test hook: 64 reads or fewer run
  // on wave 0 alone).
  const char* cenv = getenv("WC_COOP");
  const int cmode = cenv ? atoi(cenv) : 2;
  c.coop = sides == 2 && chain == 0 && !gstate && !any_act && (nmax > 64 || cmode == 1) &&
           nmax <= 64u * (uint32_t)wcc::engine_waves() && cmode != 0 &&
           (cmode == 1 || ids.size() <= (uint64_t)ctx->n_cu) && lds_bytes(sides, pcap, nmax, 0, 1) <= kLdsMax;
  if (c.coop) c.wave = c.narrow = c.lowlat = c.cu = false;
  c.waves = c.cu ? (uint32_t)std::max(wcu::engine_waves(), kWaves) : (uint32_t)kWaves;
  c.dual_hot = false;
  auto occupancy = [&](size_t l) {
    if (c.coop) return nmax <= 64u * (uint32_t)wcc2::engine_waves() ? wcc2::coop_blocks_per_cu(l) : wcc::coop_blocks_per_cu(l);
    if (c.wave) return wcw::wave_blocks_per_cu(nmax, l);
    if (c.cu) return wcu::engine_blocks_per_cu(sides, l);
    if (sides == 2 && chain > 0 && !gstate) return wcd::engine_blocks_per_cu(sides, l);
    return c.narrow ? wcn::engine_blocks_per_cu(sides, l, c.dual_hot)
                    : (c.lowlat ? wcl::engine_blocks_per_cu(sides, l, c.dual_hot)
                                : engine_blocks_per_cu(sides, l, c.dual_hot));
  };
  // dual_hot: the dual engine keeps the popped node's RStates (2 x nmax x 64 B)
  // in LDS, where its in-place child is pushed and, most of the time, popped
  // next (no RState round trip to HBM). Measured not to pay (the
  // heaviest cfg5 sub-problem alone, 37.9k vs 36.8k cycles per pop; the
  // RState loads hit L2 and are not the per-pop critical path), so it is off
  // by default: WC_DUAL_HOT=1 turns it on where it costs the launch no
  // workgroups (same occupancy, or room for every problem anyway),
  // WC_DUAL_HOT=2 wherever the LDS allows.
  if (c.wave || c.coop) c.dual_hot = true;  // (the LDS carve of its hot node)
  if (sides == 2 && chain == 0 && !gstate && !c.wave && !c.coop) {
    const char* henv = getenv("WC_DUAL_HOT");
    const int hmode = henv ? atoi(henv) : 0;
    const uint64_t lhot = lds_bytes(sides, pcap, nmax, 0, 1);
    if (hmode != 0 && lhot <= kLdsMax) {
      const int occ0 = occupancy((size_t)lds_bytes(sides, pcap, nmax, 0, 0));
      c.dual_hot = true;
      const int occ1 = occupancy((size_t)lhot);
      c.dual_hot = hmode == 2 || occ1 >= occ0 || ids.size() <= (uint64_t)occ1 * ctx->n_cu;
    }
  }
  // longer chains amortise the per-chain work (prediction, acceptance, the
  // literal pop between chains); take the longest one whose LDS still gives
  // the workgroups per CU of the default length (results do not depend on it)
  if (sides == 1 && !chain_env && chain > 0 && !gstate) {
    const int occ = occupancy((size_t)lds_bytes(sides, pcap, nmax, chain, 0, c.waves));
    for (uint32_t k = chain + 1; k <= kChainMax; ++k) {
      const uint64_t l = lds_bytes(sides, pcap, nmax, k, 0, c.waves);
      if (l > 60 * 1024 || occupancy((size_t)l) < occ) break;
      chain = k;
    }
  }
  // A one-wave launch with more problems than fit at once (a cfg5 stream) is
  // bound by how many run together: its node pool gets the smallest size, down
  // to 256 nodes, that still gives another workgroup per CU (the kernels' 256
  // VGPRs allow 4, one per SIMD; a pool of 512 holds the LDS to 3). A problem
  // that outgrows the pool retries larger, as always. cfg5 10,000 loci: 768 ->
  // 1,024 workgroups, 19.8 -> 16.3 s, no retries (gpurun_out/occ3).
  // WC_DUAL_LDS_KB (experiment hook) keeps the pool it plans.
  if (c.wave && px == 0 && !getenv("WC_DUAL_LDS_KB")) {
    while (pcap > 256) {
      const int occ_now = occupancy((size_t)lds_bytes(sides, pcap, nmax, 0, 1));
      if (ids.size() <= (uint64_t)occ_now * ctx->n_cu) break;
      if (occupancy((size_t)lds_bytes(sides, pcap / 2, nmax, 0, 1)) <= occ_now) break;
      pcap /= 2;
    }
  }
  c.pcap = pcap;
  c.chain = chain;
  // result records per problem: up to 256 at first; a problem with more tied
  // results than records reruns with more (ST_RETRY_RMAX), up to max_return_size
  uint64_t rmax = std::min<uint64_t>(std::max<uint64_t>(cfg.max_return_size, 1), 256);
  if (const char* r0 = getenv("WC_RMAX"))  // test hook: a smaller first record count exercises the retry
    rmax = std::max<uint64_t>(1, std::min<uint64_t>(rmax, (uint64_t)atoi(r0)));
  for (uint32_t k = 0; k < rx; ++k) rmax = std::min<uint64_t>(std::max<uint64_t>(cfg.max_return_size, 1), rmax * 8);
  if (rmax > (1u << 20)) {
    err = "more tied results than the device result buffer holds (max_return_size)";
    return WC_E_LIMIT;
  }
  c.rmax = (uint32_t)rmax;
  // offset activation scratch (wfa_ed_config pair arrays): edits <= |v1| + |v2|
  // with |v1| <= window + ocl and |v2| <= ocl (engine_common wave_pick_offset)
  c.act_m = 0;
  if (any_act) {
    const uint64_t ocl = std::min<uint64_t>(cfg.offset_compare_length, maxlen);
    const uint64_t m = 3 + 2 * (cfg.offset_window + 2 * ocl) + 8;
    if (m > 8192) {
      err = "offset_window/offset_compare_length too large for the device activation scratch";
      return WC_E_LIMIT;
    }
    c.act_m = (uint32_t)m;
  }
  c.conc = (uint32_t)conc;
  c.gstate = gstate;
  c.gsb = align16(lds_bytes(sides, pcap, nmax, chain, c.dual_hot, c.waves));
  c.lds = gstate ? 0 : (size_t)c.gsb;
  c.per_cu = gstate ? wcg::engine_blocks_per_cu(sides, 0) : occupancy(c.lds);
  c.wsb = ws_bytes(sides, pcap, nmax, c.wcap, c.lcap);
  c.ob = out_bytes(sides, c.rmax, nmax, c.lcap);
  return WC_OK;
}

void destroy_launches(wc_ctx* ctx) {
  for (Launch* L : ctx->launches) delete L;
  ctx->launches.clear();
}

// WC_FAULT_LOG=1 (diagnostics): on a GPU memory fault, print the faulting
// address against the buffers of the launches started last (which buffer,
// which workgroup's workspace, the offset inside it). WC_FAULT_SENTINELS=1
// also gives every pointer argument a batch launch does not use a distinct
// unmapped address (kSentinel + field << 32) instead of null, so that a
// fault through one of them names the field (the device code is unchanged:
// these fields are only read behind A.stream or in other builds).
namespace {
struct FaultRange {
  const char* name;
  uint64_t base, bytes, stride;
};
constexpr uint64_t kSentinel = 0x1e0000000000ull;
const char* const kSentinelNames[] = {"sctl", "qhead", "exited", "act_scr", "gstate", "hreads"};
std::mutex g_fault_mu;
std::vector<FaultRange> g_fault_ranges;
hsa_status_t fault_event(const hsa_amd_event_t* ev, void*) {
  if (ev->event_type != HSA_AMD_GPU_MEMORY_FAULT_EVENT) return HSA_STATUS_SUCCESS;
  const uint64_t va = ev->memory_fault.virtual_address;
  fprintf(stderr, "[wc] GPU memory fault at 0x%llx (reason mask 0x%x)\n", (unsigned long long)va,
          ev->memory_fault.fault_reason_mask);
  if (va >= kSentinel && va < kSentinel + (6ull << 32))
    fprintf(stderr, "[wc]   sentinel of EngineArgs::%s + %llu\n", kSentinelNames[(va - kSentinel) >> 32],
            (unsigned long long)((va - kSentinel) & 0xFFFFFFFFull));
  std::lock_guard<std::mutex> g(g_fault_mu);
  for (const FaultRange& r : g_fault_ranges) {
    const int64_t d = (int64_t)(va - r.base);
    fprintf(stderr, "[wc]   %-8s base 0x%llx bytes %llu stride %llu: offset %lld", r.name, (unsigned long long)r.base,
            (unsigned long long)r.bytes, (unsigned long long)r.stride, (long long)d);
    if (r.stride && d >= 0) fprintf(stderr, " (workgroup %lld + %lld)", (long long)(d / (int64_t)r.stride), (long long)(d % (int64_t)r.stride));
    if (d >= 0 && (uint64_t)d < r.bytes) fprintf(stderr, "  <== inside");
    fprintf(stderr, "\n");
  }
  return HSA_STATUS_SUCCESS;
}
void fault_log_record(const Launch& L, const EngineArgs& a, const Caps& caps) {
  static std::once_flag once;
  std::call_once(once, [] { (void)hsa_amd_register_system_event_handler(fault_event, nullptr); });
  std::lock_guard<std::mutex> g(g_fault_mu);
  if (g_fault_ranges.size() > 96) g_fault_ranges.erase(g_fault_ranges.begin(), g_fault_ranges.begin() + 48);
  g_fault_ranges.push_back({"ws", (uint64_t)a.ws, (uint64_t)L.ws.cap, a.ws_stride});
  if (caps.gstate) g_fault_ranges.push_back({"gstate", (uint64_t)a.gstate, (uint64_t)L.gst.cap, a.gstate_stride});
  g_fault_ranges.push_back({"reads", (uint64_t)a.rbytes, L.reads_bytes, 0});
  g_fault_ranges.push_back({"problems", (uint64_t)a.problems, (uint64_t)L.probs.cap, sizeof(DevProblem)});
  g_fault_ranges.push_back({"roff", (uint64_t)a.roff, (uint64_t)L.sroff.cap, 8});
  g_fault_ranges.push_back({"rlen", (uint64_t)a.rlen, (uint64_t)L.srlen.cap, 4});
  g_fault_ranges.push_back({"ract", (uint64_t)a.ractivate, (uint64_t)L.ract.cap, 8});
  g_fault_ranges.push_back({"counter", (uint64_t)a.work_counter, (uint64_t)L.counter.cap, 0});
  g_fault_ranges.push_back({"done", (uint64_t)a.done, (uint64_t)L.host.cap, 0});
  g_fault_ranges.push_back({"out", (uint64_t)a.out, (uint64_t)a.out_stride * L.P, a.out_stride});
  if (a.act_scr) g_fault_ranges.push_back({"act", (uint64_t)a.act_scr, (uint64_t)L.act.cap, a.act_stride * 8});
}
// WC_FAULT_SENTINELS: the unused pointer arguments of a batch launch
void fault_sentinels(EngineArgs& a, const Caps& caps) {
  if (!getenv("WC_FAULT_SENTINELS") || a.stream) return;
  a.sctl = (StreamCtl*)(kSentinel + (0ull << 32));
  a.qhead = (uint32_t*)(kSentinel + (1ull << 32));
  a.exited = (uint32_t*)(kSentinel + (2ull << 32));
  if (!a.act_scr) a.act_scr = (uint64_t*)(kSentinel + (3ull << 32));  // read only by offset activation
  if (!caps.gstate) a.gstate = (uint8_t*)(kSentinel + (4ull << 32));
}
}  // namespace

// engine builds (wc_engine_name): bit = 2 * build + sides - 1
// ("cu.dual": the whole-CU dual build, removed in round 5; the bit stays unused)
const char* const kEngineNames[] = {"lds.single",    "lds.dual",    "narrow.single", "narrow.dual",
                                    "lowlat.single", "lowlat.dual", "cu.single",     "cu.dual",
                                    "chain.single",  "chain.dual",  "wave.single",   "wave.dual",
                                    "gstate.single", "gstate.dual",  "coop.single", "coop.dual"};
const uint32_t kNumEngineNames = sizeof(kEngineNames) / sizeof(kEngineNames[0]);
static uint32_t engine_build(const Caps& caps) {
  if (caps.gstate) return 6;
  if (caps.coop) return 7;
  if (caps.sides == 2 && caps.chain > 0) return 4;
  if (caps.wave) return 5;
  if (caps.cu) return 3;
  if (caps.narrow) return 1;
  if (caps.lowlat) return 2;
  return 0;
}

// launches the engine of `caps` (LDS or global-state build) on L's stream
int launch_kernel(wc_ctx* ctx, Launch& L, EngineArgs& a, const Caps& caps) {
  ctx->engines_used.fetch_or(1u << (2 * engine_build(caps) + (caps.sides == 2 ? 1 : 0)), std::memory_order_relaxed);
  if (caps.gstate) {
    if (!L.gst.ensure((caps.gsb + kGuard) * L.grid)) return set_err(ctx, WC_E_HIP, "device allocation failed (search state)");
    a.gstate = (uint8_t*)L.gst.p;
    a.gstate_stride = caps.gsb + kGuard;
  }
#ifdef WC_CHECK
  L.ws_stride = a.ws_stride;
  HIPCHK(hipMemsetAsync(L.ws.p, kGuardByte, a.ws_stride * L.grid, L.stream));
  if (caps.gstate) HIPCHK(hipMemsetAsync(L.gst.p, kGuardByte, a.gstate_stride * L.grid, L.stream));
#endif
  fault_sentinels(a, caps);
  if (getenv("WC_FAULT_LOG")) fault_log_record(L, a, caps);
  HIPCHK(hipEventRecord(L.ev0, L.stream));
  if (caps.gstate) {
    if (caps.sides == 1) wcg::launch_single_engine(a, L.grid, 0, L.stream);
    else wcg::launch_dual_engine(a, L.grid, 0, L.stream);
  } else if (caps.sides == 2 && caps.chain > 0) {
    wcd::launch_dual_engine(a, L.grid, caps.lds, L.stream);
  } else if (caps.coop) {
    // (2 waves for problems of at most 128 reads, else 4)
    if (caps.nmax <= 64u * (uint32_t)wcc2::engine_waves()) wcc2::launch_dual_engine(a, L.grid, caps.lds, L.stream);
    else wcc::launch_dual_engine(a, L.grid, caps.lds, L.stream);
  } else if (caps.wave) {
    wcw::launch_dual_engine(a, L.grid, caps.lds, L.stream);
  } else if (caps.cu) {
    wcu::launch_single_engine(a, L.grid, caps.lds, L.stream);  // (single engine only)
  } else if (caps.narrow) {
    if (caps.sides == 1) wcn::launch_single_engine(a, L.grid, caps.lds, L.stream);
    else wcn::launch_dual_engine(a, L.grid, caps.lds, L.stream);
  } else if (caps.lowlat) {
    if (caps.sides == 1) wcl::launch_single_engine(a, L.grid, caps.lds, L.stream);
    else wcl::launch_dual_engine(a, L.grid, caps.lds, L.stream);
  } else {
    if (caps.sides == 1) launch_single_engine(a, L.grid, caps.lds, L.stream);
    else launch_dual_engine(a, L.grid, caps.lds, L.stream);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(L.ev1, L.stream));
  return WC_OK;
}

Launch* launch_slot(wc_ctx* ctx, size_t k) {
  while (ctx->launches.size() <= k) {
    Launch* L = new Launch();
    if (hipStreamCreateWithFlags(&L->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&L->ev0) != hipSuccess || hipEventCreate(&L->ev1) != hipSuccess) {
      delete L;
      return nullptr;
    }
    ctx->launches.push_back(L);
  }
  return ctx->launches[k];
}

// Starts one engine launch over items[ids] (already in scheduling order).
int launch_start(wc_ctx* ctx, Launch& L, const wc_batch* b, const wc_config& cfg, const std::vector<SubProb>& items,
                        const std::vector<uint32_t>& ids, const Caps& caps) {
  L.caps = caps;
  L.ids = ids;
  L.P = (uint32_t)ids.size();
  L.taken.assign(L.P, 0);
  L.n_taken = 0;
  L.kernel_ms = 0;
  const uint32_t P = L.P;
  uint64_t nslots = 0;
  for (uint32_t id : ids) nslots += items[id].gid.size();
  L.dp.assign(P, DevProblem());
  L.h_sroff.resize(std::max<uint64_t>(nslots, 1));
  L.h_srlen.resize(std::max<uint64_t>(nslots, 1));
  L.h_ract.resize(std::max<uint64_t>(nslots, 1));
  uint64_t slot = 0;
  for (uint32_t k = 0; k < P; ++k) {
    const SubProb& s = items[ids[k]];
    DevProblem& d = L.dp[k];
    memset(&d, 0, sizeof(d));
    d.read_begin = (uint32_t)slot;
    d.n_reads = (uint32_t)s.gid.size();
    d.max_read_len = s.max_len;
    d.n_active = s.n_active;
    d.max_act = s.max_act;
    for (size_t r = 0; r < s.gid.size(); ++r, ++slot) {
      L.h_sroff[slot] = b->roff_h[s.gid[r]];
      L.h_srlen[slot] = b->rlen_h[s.gid[r]];
      L.h_ract[slot] = s.act[r];
    }
  }
  L.grid = std::min<uint32_t>(P, (uint32_t)std::max(1, caps.per_cu) * (uint32_t)ctx->n_cu);
  L.off_status = align16((uint64_t)P * 4);
  L.off_stats = L.off_status + align16((uint64_t)P * 4);
  L.off_out = L.off_stats + align16((uint64_t)P * S_NSTAT * 8);
  const uint64_t hbytes = L.off_out + (uint64_t)P * caps.ob;
  if (!L.host.ensure(hbytes, true)) return set_err(ctx, WC_E_HIP, "pinned host allocation failed (results)");
  memset(L.host.p, 0, L.off_out);  // done flags, status, counters
  if (caps.act_m && !L.act.ensure(act_scr_u64(caps.act_m, caps.waves) * 8 * L.grid))
    return set_err(ctx, WC_E_HIP, "device allocation failed (activation scratch)");
  if (!L.probs.ensure(P * sizeof(DevProblem)) || !L.sroff.ensure(L.h_sroff.size() * 8) ||
      !L.srlen.ensure(L.h_srlen.size() * 4) || !L.ract.ensure(L.h_ract.size() * 8) ||
      !L.ws.ensure((caps.wsb + kGuard) * L.grid) || !L.counter.ensure(4))
    return set_err(ctx, WC_E_HIP, "device allocation failed (workspace)");
  HIPCHK(hipMemcpyAsync(L.probs.p, L.dp.data(), P * sizeof(DevProblem), hipMemcpyHostToDevice, L.stream));
  HIPCHK(hipMemcpyAsync(L.sroff.p, L.h_sroff.data(), L.h_sroff.size() * 8, hipMemcpyHostToDevice, L.stream));
  HIPCHK(hipMemcpyAsync(L.srlen.p, L.h_srlen.data(), L.h_srlen.size() * 4, hipMemcpyHostToDevice, L.stream));
  HIPCHK(hipMemcpyAsync(L.ract.p, L.h_ract.data(), L.h_ract.size() * 8, hipMemcpyHostToDevice, L.stream));
  HIPCHK(hipMemsetAsync(L.counter.p, 0, 4, L.stream));

  void* dhost = nullptr;
  HIPCHK(hipHostGetDevicePointer(&dhost, L.host.p, 0));
  uint8_t* dh = (uint8_t*)dhost;
  EngineArgs a;
  memset(&a, 0, sizeof(a));
  a.cfg = to_dev(cfg);
  a.problems = (const DevProblem*)L.probs.p;
  a.n_problems = P;
  a.sides = caps.sides;
  a.rbytes = (const uint8_t*)b->reads.p;
  L.reads_bytes = b->reads.cap;
  a.roff = (const uint64_t*)L.sroff.p;
  a.rlen = (const uint32_t*)L.srlen.p;
  a.ractivate = (const int64_t*)L.ract.p;
  a.ws = (uint8_t*)L.ws.p;
  a.ws_stride = caps.wsb + kGuard;
  a.pcap = caps.pcap;
  a.wcap = caps.wcap;
  a.lcap = caps.lcap;
  a.nmax = caps.nmax;
  a.rmax = caps.rmax;
  a.chain = caps.chain;
  a.chain_kinds = env_chain_kinds();
  a.dual_hot = caps.dual_hot ? 1u : 0u;
  a.out = dh + L.off_out;
  a.out_stride = caps.ob;
  a.status = (uint32_t*)(dh + L.off_status);
  a.stats = (uint64_t*)(dh + L.off_stats);
  a.done = (uint32_t*)dh;
  a.work_counter = (uint32_t*)L.counter.p;
  a.act_m = caps.act_m;
  a.act_scr = caps.act_m ? (uint64_t*)L.act.p : nullptr;
  a.act_stride = caps.act_m ? act_scr_u64(caps.act_m, caps.waves) : 0;
  // debug phase cycle counters (WC_PHASES=<file>, WC_PHASE_PROF builds only)
  if (getenv("WC_PHASES") && L.phases.ensure(kPhases * 8)) {
    a.phases = (unsigned long long*)L.phases.p;
    HIPCHK(hipMemsetAsync(L.phases.p, 0, kPhases * 8, L.stream));
  }
  // pop trace of the launch's problem 0 (WC_POP_TRACE=<file>, diagnostics;
  // the device code is the same with or without it): per pop (cost, len,
  // flags, extra), engine.hip trace_pop
  constexpr uint32_t kTraceCap = 1u << 20;
  if (getenv("WC_POP_TRACE") && L.trace.ensure((4ull + 4ull * kTraceCap) * 4)) {
    a.trace = (uint32_t*)L.trace.p;
    a.trace_cap = kTraceCap;
    HIPCHK(hipMemsetAsync(L.trace.p, 0, 16, L.stream));
  }
  const int krc = launch_kernel(ctx, L, a, caps);
  if (krc != WC_OK) return krc;
  L.busy = true;
  L.traced = a.trace != nullptr;
  if (getenv("WC_LAUNCH_LOG"))
    fprintf(stderr, "[wc] launch sides=%u problems=%u grid=%u per_cu=%d lds=%zu gstate=%d narrow=%d lowlat=%d cu=%d wave=%d coop=%d dual_hot=%d pcap=%u wcap=%u lcap=%u chain=%u rmax=%u\n",
            caps.sides, P, L.grid, caps.per_cu, caps.lds, (int)caps.gstate, (int)caps.narrow, (int)caps.lowlat, (int)caps.cu, (int)caps.wave, (int)caps.coop, (int)caps.dual_hot, caps.pcap, caps.wcap, caps.lcap, caps.chain, caps.rmax);
  return WC_OK;
}

// The outcome of launch problem k (its completion flag is set). Returns the
// raw device status (ST_RETRY flags included); `o` gets records and counters.
uint32_t harvest(const Launch& L, uint32_t k, const SubProb& s, EngineOut& o) {
  const uint32_t st = L.status()[k];
  for (int q = 0; q < S_NSTAT; ++q) o.stats[q] = L.stats()[(uint64_t)k * S_NSTAT + q];
  o.recs.clear();
  o.status = (int)st;
  o.error.clear();
  if (st & ST_RETRY) return st;
  const uint8_t* base = L.out(k);
  if ((st & 0xFFFFu) == WC_E_LIMIT) {
    o.status = WC_E_LIMIT;
    o.error = limit_msg(st >> 16);
    return WC_E_LIMIT;
  }
  if (st != ST_OK) {
    o.error = err_msg((int)st);
    if (st == WC_E_COVERAGE_GAP)  // consensus.rs:305 / dual_consensus.rs message
      o.error = "Encountered coverage gap: consensus is length " + std::to_string(((const uint32_t*)base)[1]) +
                " with no candidates, but sequences activate at " + std::to_string(s.max_act);
    return st;
  }
  const Caps& c = L.caps;
  const uint64_t rb = result_bytes(c.sides, c.nmax, c.lcap);
  const uint32_t nres = ((const uint32_t*)base)[0];
  const uint32_t n = (uint32_t)s.gid.size();
  for (uint32_t r = 0; r < nres; ++r) {
    const uint8_t* rec = base + 16 + (uint64_t)r * rb;
    const uint32_t* h = (const uint32_t*)rec;
    RawRecord rr;
    rr.len[0] = h[0];
    rr.len[1] = h[1];
    rr.dual = h[2] != 0;
    for (uint32_t sd = 0; sd < c.sides; ++sd) {
      const uint8_t* con = rec + 16 + sd * align16(c.lcap);
      rr.con[sd].assign(con, con + rr.len[sd]);
      const uint32_t* fe = (const uint32_t*)(rec + 16 + c.sides * align16(c.lcap) + sd * align16((uint64_t)c.nmax * 4));
      rr.fe[sd].assign(fe, fe + n);
    }
    o.recs.push_back(std::move(rr));
  }
  return st;
}

// capacity growth for a retried item
void bump(SubProb& s, uint32_t st) {
  if (st & ST_RETRY_WCAP) s.wcap_x++;
  if (st & (ST_RETRY_PCAP | ST_RETRY_HEAP)) s.pcap_x += 2;
  if (st & ST_RETRY_LCAP) s.lcap_x++;
  if (st & ST_RETRY_RMAX) s.rmax_x++;
  s.attempts++;
}

#ifdef WC_CHECK
// every workgroup's guard zones must still hold kGuardByte
int check_guards(wc_ctx* ctx, const Launch& L) {
  std::vector<uint8_t> g(kGuard);
  auto scan = [&](const DevBuf& b, uint64_t stride, const char* what) -> int {
    for (uint32_t w = 0; w < L.grid; ++w) {
      HIPCHK(hipMemcpy(g.data(), (const uint8_t*)b.p + (uint64_t)w * stride + stride - kGuard, kGuard,
                       hipMemcpyDeviceToHost));
      for (uint64_t i = 0; i < kGuard; ++i)
        if (g[i] != kGuardByte) {
          fprintf(stderr, "[wc-check] %s guard of workgroup %u overwritten at +%llu (byte 0x%02x)\n", what, w,
                  (unsigned long long)i, g[i]);
          return set_err(ctx, WC_E_INVARIANT, std::string("bounds check: ") + what + " guard overwritten");
        }
    }
    return WC_OK;
  };
  int rc = scan(L.ws, L.ws_stride, "workspace");
  if (rc == WC_OK && L.caps.gstate) rc = scan(L.gst, L.caps.gsb + kGuard, "search-state");
  return rc;
}
#endif

int launch_finish(wc_ctx* ctx, Launch& L) {
  HIPCHK(hipStreamSynchronize(L.stream));
#ifdef WC_CHECK
  if (const int grc = check_guards(ctx, L)) return grc;
#endif
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, L.ev0, L.ev1));
  L.kernel_ms = ms;
  L.busy = false;
  if (const char* path = getenv("WC_PHASES")) {
    unsigned long long ph[kPhases];
    HIPCHK(hipMemcpy(ph, L.phases.p, sizeof(ph), hipMemcpyDeviceToHost));
    if (FILE* f = fopen(path, "a")) {
      fprintf(f, "sides=%u kernel_ms=%.3f", L.caps.sides, ms);
      for (int k = 0; k < kPhases; ++k) fprintf(f, " %llu", ph[k]);
      fprintf(f, "\n");
      fclose(f);
    }
  }
  if (getenv("WC_LAUNCH_LOG")) fprintf(stderr, "[wc] done problems=%u ms=%.3f\n", L.P, ms);
  if (const char* path = getenv("WC_POP_TRACE")) {
    if (L.traced) {
      uint32_t k = 0;
      HIPCHK(hipMemcpy(&k, L.trace.p, 4, hipMemcpyDeviceToHost));
      std::vector<uint32_t> rec(4ull * k);
      if (k) HIPCHK(hipMemcpy(rec.data(), (const uint32_t*)L.trace.p + 4, rec.size() * 4, hipMemcpyDeviceToHost));
      if (FILE* f = fopen(path, "a")) {
        fprintf(f, "# launch sides=%u problems=%u pops=%u\n", L.caps.sides, L.P, k);
        for (uint32_t i = 0; i < k; ++i)
          fprintf(f, "%u %u %u %u\n", rec[4 * i], rec[4 * i + 1], rec[4 * i + 2], rec[4 * i + 3]);
        fclose(f);
      }
    }
    L.traced = false;
  }
  return WC_OK;
}


int run_engine(wc_ctx* ctx, wc_batch* b, const wc_config& cfg, uint32_t sides, std::vector<SubProb>& items,
               std::vector<EngineOut>& out, double& kernel_ms, uint64_t& launches,
               const std::function<void(uint32_t)>* on_final) {
  out.resize(items.size());
  std::vector<uint32_t> pending;
  for (uint32_t i = 0; i < items.size(); ++i)
    if (out[i].status == WC_OK) pending.push_back(i);
  Launch* L = launch_slot(ctx, 0);
  if (!L) return set_err(ctx, WC_E_HIP, "stream creation failed");
  while (!pending.empty()) {
    std::stable_sort(pending.begin(), pending.end(),
                     [&](uint32_t x, uint32_t y) { return items[x].work > items[y].work; });
    // capacities are planned per launch from its largest problem, so a few
    // deep problems (many reads: LDS per read, no linear-chain area above
    // kBlock reads) run in a launch of their own instead of shrinking the node
    // pool and occupancy of every other problem
    std::vector<uint32_t> run, later;
    for (uint32_t id : pending) (items[id].gid.size() > (size_t)kBlock ? later : run).push_back(id);
    if (run.empty()) run.swap(later);
    Caps caps;
    std::string err;
    int rc = plan_caps(ctx, cfg, sides, items, run, hbm_share(ctx, L->ws.cap, 0.5), caps, err, 4, true);
    if (rc != WC_OK) {
      for (uint32_t id : run) {
        out[id].status = rc;
        out[id].error = err;
      }
      pending.swap(later);
      continue;
    }
    const auto t0 = std::chrono::steady_clock::now();
    rc = launch_start(ctx, *L, b, cfg, items, run, caps);
    if (rc != WC_OK) return rc;
    const auto t1 = std::chrono::steady_clock::now();
    // consume problems as their completion flags appear, while the launch
    // runs: the result copies and on_final (the caller's result building)
    // overlap the kernel instead of following it
    std::vector<uint32_t> retry;
    std::vector<uint8_t> got(L->P, 0);
    uint32_t ngot = 0;
    auto take = [&](uint32_t k) {
      const uint32_t id = L->ids[k];
      const uint32_t st = harvest(*L, k, items[id], out[id]);
      if (st & ST_RETRY) {
        bump(items[id], st);
        if (items[id].attempts < kMaxAttempts) {
          retry.push_back(id);
          return;
        }
        out[id].status = WC_E_LIMIT;
        out[id].error = retry_msg(st, items[id].attempts);
      }
      if (on_final) (*on_final)(id);
    };
    volatile uint32_t* done = L->done();
    while (ngot < L->P) {
      bool any = false;
      for (uint32_t k = 0; k < L->P; ++k) {
        if (got[k] || !__atomic_load_n(&done[k], __ATOMIC_ACQUIRE)) continue;
        got[k] = 1;
        ngot++;
        any = true;
        take(k);
      }
      if (any) continue;
      if (hipStreamQuery(L->stream) != hipErrorNotReady) break;  // ended (or failed: launch_finish reports it)
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    rc = launch_finish(ctx, *L);
    if (rc != WC_OK) return rc;
    const auto t2 = std::chrono::steady_clock::now();
    kernel_ms += L->kernel_ms;
    launches++;
    for (uint32_t k = 0; k < L->P; ++k)
      if (!got[k]) take(k);
    if (getenv("WC_HOST_TIMING"))
      fprintf(stderr, "[wc] launch: start %.3f ms, to completion %.3f ms (kernel %.3f), harvest after %.3f ms\n",
              std::chrono::duration<double, std::milli>(t1 - t0).count(),
              std::chrono::duration<double, std::milli>(t2 - t1).count(), L->kernel_ms,
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t2).count());
    retry.insert(retry.end(), later.begin(), later.end());
    pending.swap(retry);
  }
  return WC_OK;
}

// One persistent engine launch fed from `ready` (and from whatever `on_done`
// appends to it) until nothing is left to run. on_done(item, raw status) is
// called for every finished item; live(item) = false drops an item unrun.
template <class OnDone, class Live>
static int stream_epoch(wc_ctx* ctx, Launch& L, const wc_batch* b, const wc_config& cfg, const Caps& caps,
                        std::vector<SubProb>& items, std::deque<uint32_t>& ready, OnDone on_done, Live live,
                        std::vector<EngineOut>& outs) {
  L.caps = caps;
  L.grid = std::min<uint32_t>((uint32_t)std::max(1, caps.per_cu) * (uint32_t)ctx->n_cu, std::max(1u, caps.conc));
  // the ring (pinned host memory) holds the published problems and their
  // read tables, from the oldest unfinished one to the newest: at most a grid
  // and a quarter of them are unfinished at once (the backlog below), but a
  // long sub-problem keeps its entry while the sub-problems published after
  // it come and go, so the span grows with the call's work. Sized for the
  // call (16 sub-problems per problem it was given, up to 65,536 entries and
  // 8M read-table slots): a 10,000-locus cfg5 call with a ring of 4,096
  // entries stalled publication behind its slowest sub-problems (49 vs 30 s),
  // while one locus per call from many threads keeps a small ring each.
  auto pow2 = [](uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
  };
  const uint32_t kQcap = (uint32_t)std::min<uint64_t>(
      1u << 16, std::max<uint64_t>({1024, pow2(2ull * L.grid + 64), pow2(16ull * items.size())}));
  const uint32_t kQslots =
      (uint32_t)std::min<uint64_t>(1u << 23, std::max<uint64_t>(1u << 16, pow2((uint64_t)kQcap * caps.nmax)));
  L.P = 2 * L.grid;  // two output slots per workgroup
  L.kernel_ms = 0;
  const uint32_t P = L.P;
  L.stream_layout();
  if (!L.host.ensure(L.off_out + (uint64_t)P * caps.ob, true))
    return set_err(ctx, WC_E_HIP, "pinned host allocation failed (results)");
  memset(L.host.p, 0, L.off_out);
  const uint64_t off_q = align16(sizeof(StreamCtl));
  const uint64_t off_roff = off_q + align16((uint64_t)kQcap * sizeof(DevProblem));
  const uint64_t off_ract = off_roff + (uint64_t)kQslots * 8;
  const uint64_t off_rlen = off_ract + (uint64_t)kQslots * 8;
  if (!L.ring.ensure(off_rlen + (uint64_t)kQslots * 4, true))
    return set_err(ctx, WC_E_HIP, "pinned host allocation failed (problem ring)");
  uint8_t* rh = (uint8_t*)L.ring.p;
  volatile StreamCtl* sc = (volatile StreamCtl*)rh;
  sc->tail = 0;
  sc->stop = 0;
  sc->abort = 0;
  sc->heartbeat = 0;
  DevProblem* qp = (DevProblem*)(rh + off_q);
  uint64_t* qroff = (uint64_t*)(rh + off_roff);
  int64_t* qract = (int64_t*)(rh + off_ract);
  uint32_t* qrlen = (uint32_t*)(rh + off_rlen);
  const uint64_t wsb = caps.wsb + rtab_bytes(caps.nmax) + kGuard;
  if (caps.act_m && !L.act.ensure(act_scr_u64(caps.act_m, caps.waves) * 8 * L.grid))
    return set_err(ctx, WC_E_HIP, "device allocation failed (activation scratch)");
  if (!L.ws.ensure(wsb * L.grid + 64) || !L.counter.ensure(4))
    return set_err(ctx, WC_E_HIP, "device allocation failed (workspace)");
  HIPCHK(hipMemsetAsync(L.counter.p, 0, 4, L.stream));
  void *dhost = nullptr, *dring = nullptr;
  HIPCHK(hipHostGetDevicePointer(&dhost, L.host.p, 0));
  HIPCHK(hipHostGetDevicePointer(&dring, L.ring.p, 0));
  uint8_t* dh = (uint8_t*)dhost;
  uint8_t* dr = (uint8_t*)dring;
  int clk = 0;
  if (hipDeviceGetAttribute(&clk, hipDeviceAttributeWallClockRate, ctx->device) != hipSuccess || clk <= 0) clk = 100000;
  EngineArgs a;
  memset(&a, 0, sizeof(a));
  a.cfg = to_dev(cfg);
  a.problems = (const DevProblem*)(dr + off_q);
  a.sides = 2;
  a.rbytes = (const uint8_t*)b->reads.p;
  a.roff = (const uint64_t*)(dr + off_roff);
  a.rlen = (const uint32_t*)(dr + off_rlen);
  a.ractivate = (const int64_t*)(dr + off_ract);
  a.ws = (uint8_t*)L.ws.p;
  a.ws_stride = wsb;
  a.pcap = caps.pcap;
  a.wcap = caps.wcap;
  a.lcap = caps.lcap;
  a.nmax = caps.nmax;
  a.rmax = caps.rmax;
  a.chain = caps.chain;  // the device carves LDS from it: must match caps.lds
  a.chain_kinds = env_chain_kinds();
  a.dual_hot = caps.dual_hot ? 1u : 0u;
  a.out = dh + L.off_out;
  a.out_stride = caps.ob;
  a.status = (uint32_t*)(dh + L.off_status);
  a.stats = (uint64_t*)(dh + L.off_stats);
  a.done = (uint32_t*)dh;
  a.act_m = caps.act_m;
  a.act_scr = caps.act_m ? (uint64_t*)L.act.p : nullptr;
  a.act_stride = caps.act_m ? act_scr_u64(caps.act_m, caps.waves) : 0;
  if (getenv("WC_PHASES") && L.phases.ensure(kPhases * 8)) {  // (WC_PHASE_PROF builds only)
    a.phases = (unsigned long long*)L.phases.p;
    HIPCHK(hipMemsetAsync(L.phases.p, 0, kPhases * 8, L.stream));
  }
  a.stream = 1;
  a.qcap = kQcap;
  a.qslots = kQslots;
  a.sctl = (StreamCtl*)dr;
  a.qhead = (uint32_t*)L.counter.p;
  a.idle_ticks = (uint64_t)clk * 1000ull * 30ull;  // 30 s without a host heartbeat: the host is gone
  a.exited = (uint32_t*)(dh + L.off_exit);
  persistent_begin();
  const int krc = launch_kernel(ctx, L, a, caps);
  if (krc != WC_OK) {
    persistent_end();
    return krc;
  }
  L.busy = true;
  if (getenv("WC_LAUNCH_LOG"))
    fprintf(stderr, "[wc] stream launch grid=%u per_cu=%d lds=%zu pcap=%u wcap=%u lcap=%u nmax=%u rmax=%u narrow=%d lowlat=%d wave=%d coop=%d dual_hot=%d\n",
            L.grid, caps.per_cu, caps.lds, caps.pcap, caps.wcap, caps.lcap, caps.nmax, caps.rmax, (int)caps.narrow,
            (int)caps.lowlat, (int)caps.wave, (int)caps.coop, (int)caps.dual_hot);

  // publication state: seq -> item, read-ring position; incomplete seqs in order
  std::vector<uint32_t> seq_item;
  std::vector<uint64_t> seq_rw;
  std::vector<uint8_t> seq_done;
  uint64_t rw = 0;
  uint32_t oldest = 0, outstanding = 0;
  volatile uint32_t* done = L.done();
  int rc = WC_OK;
  auto t_idle = std::chrono::steady_clock::now();
  uint32_t beat = 0, finished = 0;
  const bool log = getenv("WC_LAUNCH_LOG") != nullptr;
  auto t_log = std::chrono::steady_clock::now();
  // a launch that stops finishing sub-problems says so (always, not only with
  // WC_LAUNCH_LOG): how far it got and how many workgroups are still in
  auto t_fin = t_log, t_warn = t_log;
  // what is ready but not yet published, in publication order: continuations
  // first (those of the problems that have taken the most pops so far first),
  // then the largest (reads x bases)
  // (WC_PUB_ORDER=bases: new problems by their bases alone, reads x length,
  // the better predictor of a locus's critical path; default reads x bases)
  const char* poe = getenv("WC_PUB_ORDER");
  const bool by_bases = poe && strcmp(poe, "bases") == 0;
  auto later = [&](uint32_t x, uint32_t y) {
    if (items[x].cont != items[y].cont) return items[y].cont;
    if (items[x].crit != items[y].crit) return items[x].crit < items[y].crit;
    const double kx = (double)items[x].work * (by_bases ? 1.0 : (double)items[x].gid.size());
    const double ky = (double)items[y].work * (by_bases ? 1.0 : (double)items[y].gid.size());
    return kx != ky ? kx < ky : x > y;
  };
  std::priority_queue<uint32_t, std::vector<uint32_t>, decltype(later)> waiting(later);
  // an epoch planned for more reads than the one-wave dual engine takes ends
  // as soon as no live sub-problem has more (the rest wait for the next
  // epoch, planned for them): cfg4's 200-read root, then 50-read groups
  // (an epoch on the cooperative build ends once no live sub-problem has
  // more than 64 reads: the one-wave kernel runs the rest)
  const size_t kWaveReads = caps.coop ? 64 : 128;
  const bool can_shrink = !caps.wave && caps.nmax > kWaveReads && !caps.gstate;
  uint32_t big_live = 0;  // outstanding or waiting sub-problems of more than kWaveReads reads
  bool shrink = false;
  for (;;) {
    bool progress = false;
    if (log && std::chrono::duration<double>(std::chrono::steady_clock::now() - t_log).count() > 10.0) {
      t_log = std::chrono::steady_clock::now();
      fprintf(stderr, "[wc] stream: %u published, %u finished, %u outstanding, %zu waiting\n",
              (uint32_t)seq_item.size(), finished, outstanding, ready.size() + waiting.size());
    }
    __atomic_store_n(&sc->heartbeat, ++beat, __ATOMIC_RELAXED);
    // publish. Workgroups claim in publication order, so the host keeps the
    // order: at most a grid and a quarter of problems are published and
    // unfinished at once; the rest wait here, continuations of started
    // problems first (they are on those problems' critical paths), then the
    // largest (reads x bases) first
    const uint32_t backlog = L.grid + L.grid / 4;
    while (!ready.empty()) {  // new arrivals into the host-side order
      big_live += items[ready.front()].gid.size() > kWaveReads;
      waiting.push(ready.front());
      ready.pop_front();
    }
    if (can_shrink && big_live == 0 && !waiting.empty()) shrink = true;
    bool published = false;
    while (!shrink && !waiting.empty() && outstanding < backlog) {
      const uint32_t id = waiting.top();
      if (!live(id)) {
        waiting.pop();
        big_live -= items[id].gid.size() > kWaveReads;
        on_done(id, ~0u);  // dropped: its problem already failed
        continue;
      }
      const SubProb& s = items[id];
      const uint32_t seq = (uint32_t)seq_item.size();
      const uint64_t ow = oldest < seq ? seq_rw[oldest] : rw;
      if (seq - oldest >= kQcap || rw + s.gid.size() - ow > kQslots) break;  // ring full: later
      waiting.pop();
      DevProblem d;
      memset(&d, 0, sizeof(d));
      d.read_begin = (uint32_t)(rw % kQslots);
      d.n_reads = (uint32_t)s.gid.size();
      d.max_read_len = s.max_len;
      d.n_active = s.n_active;
      d.max_act = s.max_act;
        qp[seq % kQcap] = d;
      for (size_t r = 0; r < s.gid.size(); ++r) {
        const uint64_t q = (rw + r) % kQslots;
        qroff[q] = b->roff_h[s.gid[r]];
        qract[q] = s.act[r];
        qrlen[q] = b->rlen_h[s.gid[r]];
      }
      seq_item.push_back(id);
      // first publication only: a retried sub-problem keeps its first start
      if (items[id].t_pub < 0)
        items[id].t_pub = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
      seq_rw.push_back(rw);
      seq_done.push_back(0);
      rw += s.gid.size();
      outstanding++;
      published = true;
    }
    if (published) {
      std::atomic_thread_fence(std::memory_order_release);
      __atomic_store_n(&sc->tail, (uint32_t)seq_item.size(), __ATOMIC_RELEASE);
      progress = true;
    }
    // consume finished problems
    for (uint32_t slot = 0; slot < P; ++slot) {
      const uint32_t v = __atomic_load_n(&done[slot], __ATOMIC_ACQUIRE);
      if (!v) continue;
      const uint32_t seq = v - 1;
      const uint32_t id = seq_item[seq];
      const uint32_t st = harvest(L, slot, items[id], outs[id]);
      __atomic_store_n(&done[slot], 0u, __ATOMIC_RELEASE);  // the slot may be reused
      seq_done[seq] = 1;
      outstanding--;
      big_live -= items[id].gid.size() > kWaveReads;
      finished++;
      while (oldest < seq_item.size() && seq_done[oldest]) oldest++;
      on_done(id, st);
      progress = true;
      t_fin = std::chrono::steady_clock::now();
    }
    if (outstanding == 0 && ready.empty() && (waiting.empty() || shrink)) break;
    {
      const auto now = std::chrono::steady_clock::now();
      const double quiet = std::chrono::duration<double>(now - t_fin).count();
      if (quiet > 20.0 && std::chrono::duration<double>(now - t_warn).count() > 20.0) {
        t_warn = now;
        fprintf(stderr,
                "[wc] stream launch: no sub-problem finished for %.0f s (%u published, %u finished, %u outstanding, "
                "%zu waiting; %u of %u workgroups exited; abort %u; grid planned for %d CUs)\n",
                quiet, (uint32_t)seq_item.size(), finished, outstanding, ready.size() + waiting.size(), L.n_exited(),
                L.grid, (uint32_t)sc->abort, ctx->n_cu);
      }
    }
    if (progress) {
      t_idle = std::chrono::steady_clock::now();
      continue;
    }
    // watchdog: the launch must not end (or give up) while problems are out
    // (exit flags, no HIP call; a stream query only after seconds without
    // progress, to notice a launch that faulted)
    const double idle = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_idle).count();
    if (sc->abort || L.all_exited() || (idle > 5.0 && hipStreamQuery(L.stream) != hipErrorNotReady)) {
      rc = set_err(ctx, WC_E_HIP, "stream launch ended with problems outstanding (abort=" +
                                      std::to_string(sc->abort) + ")");
      break;
    }
    if (idle > 300.0) {
      rc = set_err(ctx, WC_E_HIP, "stream launch made no progress for 300 s");
      break;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  while (!waiting.empty()) {  // not published (an error ended the epoch)
    ready.push_back(waiting.top());
    waiting.pop();
  }
  __atomic_store_n(&sc->stop, 1u, __ATOMIC_RELEASE);
  const int frc = launch_finish(ctx, L);
  persistent_end();
  return rc != WC_OK ? rc : frc;
}

// ---------------------------------------------------------------------------
// PriorityConsensusDWFA (priority_consensus.rs:172-341), streamed
// ---------------------------------------------------------------------------
namespace {
uint64_t fx_add(uint64_t h, uint64_t w) { return (((h << 5) | (h >> 59)) ^ w) * 0x517cc1b727220a95ULL; }
uint64_t fx_hash_opt(int64_t v) { return v < 0 ? fx_add(0, 0) : fx_add(fx_add(0, 1), (uint64_t)v); }
size_t fx_cap_h(size_t b) { return b == 0 ? 0 : (b < 8 ? b - 1 : b / 8 * 7); }
size_t fx_buckets_h(size_t cap) {
  if (cap < 8) return cap < 4 ? 4 : 8;
  size_t adj = cap * 8 / 7, p = 1;
  while (p < adj) p <<= 1;
  return p;
}
}  // namespace
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

// priority_consensus.rs:309-335: the finished chains of one problem (and
// which input chains each covers) into its result: chains stable-sorted by
// their consensus sequences, sequence_indices per input chain
void priority_assemble(uint32_t M, std::vector<std::vector<ConsRec>>& C, std::vector<std::vector<uint8_t>>& assigns,
                       ProbRes& pr) {
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
        if (assigns[ord[ci]][c]) pr.indices[c] = ci;
      pr.chains.push_back(C[ord[ci]]);
    }
  } else {
    pr.chains = C;
    pr.indices.assign(M, 0);
  }
}

namespace {
// one stacked sub-problem: a read subset at a chain level
struct PWork {
  uint32_t owner = 0;
  std::vector<uint8_t> inc;
  uint32_t level = 0;
  std::vector<ConsRec> chain;
  int state = 0;  // 0 waiting to launch, 1 launched, 2 done (result known, successors made)
  std::unique_ptr<ProbRes> res;
  double t_make = 0;  // ms from the call's start (WC_SUBPROB_LOG)
  // the sub-problems this one's result makes (a split's two groups, or the
  // next level), made as soon as the result is known; they go on the stack
  // when this one is popped (the reference's LIFO order)
  std::vector<uint32_t> kids;
  bool final_chain = false;  // no successor: `chain` is finished (the last level)
};
}  // namespace

int priority_stream(wc_ctx* ctx, const wc_config& cfg, uint32_t n, const wc_chain_problem* problems, wc_results* R) {
  const auto t_call = std::chrono::steady_clock::now();
  R->probs.resize(n);
  // WC_SUBPROB_LOG=<file> (diagnostics): owner level reads made_ms done_ms pops updates split status
  FILE* sublog = getenv("WC_SUBPROB_LOG") ? fopen(getenv("WC_SUBPROB_LOG"), "a") : nullptr;
  struct CloseLog {
    FILE* f;
    ~CloseLog() {
      if (f) fclose(f);
    }
  } close_log{sublog};
  // 1. every read of every problem (all chain levels) resident in one arena:
  //    read (problem i, chain c, level l) = arena read base[i] + c * levels + l
  std::vector<wc_problem> flat(n);
  for (uint32_t i = 0; i < n; ++i) {
    flat[i].n_reads = problems[i].n_chains * problems[i].levels;
    flat[i].reads = problems[i].reads;
    flat[i].lens = problems[i].lens;
    flat[i].offsets = nullptr;
  }
  wc_batch all;
  int rc = upload_batch(ctx, n, flat.data(), &all);
  if (rc != WC_OK) return rc;

  // 2. the reference's LIFO stacks, one per problem (pool indices)
  std::vector<std::unique_ptr<PWork>> pool;
  std::vector<SubProb> subs;  // parallel to pool
  std::vector<EngineOut> outs;
  std::vector<std::vector<uint32_t>> stacks(n);
  std::vector<std::vector<std::vector<ConsRec>>> cons(n);
  std::vector<std::vector<std::vector<uint8_t>>> assigns(n);
  std::vector<bool> alive(n, true);
  std::vector<uint64_t> owner_pops(n, 0);  // pops of each problem's finished sub-problems (SubProb::crit)
  // when each problem's first sub-problem was published (ProbRes::start_ms)
  std::vector<double> owner_start(n, -1.0);
  const double t_call_ms = std::chrono::duration<double, std::milli>(t_call.time_since_epoch()).count();
  std::deque<uint32_t> ready, retry_ready;

  bool roots_made = false;  // sub-problems made after the roots are continuations
  auto make = [&](uint32_t i, std::vector<uint8_t> inc, uint32_t level, std::vector<ConsRec> chain) {
    const wc_chain_problem& q = problems[i];
    const uint32_t id = (uint32_t)pool.size();
    pool.emplace_back(new PWork());
    PWork& w = *pool.back();
    w.owner = i;
    w.t_make = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_call).count();
    w.inc = std::move(inc);
    w.level = level;
    w.chain = std::move(chain);
    subs.emplace_back();
    outs.emplace_back();
    SubProb& s = subs.back();
    s.cont = roots_made;
    s.crit = owner_pops[i];
    std::vector<int64_t> offs;
    for (uint32_t c = 0; c < q.n_chains; ++c) {
      if (!w.inc[c]) continue;
      const uint32_t g = all.probs[i].read_begin + c * q.levels + level;
      s.gid.push_back(g);
      const int64_t o = q.offsets ? q.offsets[c * q.levels + level] : -1;
      offs.push_back(o < 0 ? -1 : o);
      s.max_len = std::max(s.max_len, all.rlen_h[g]);
      s.work += all.rlen_h[g];
    }
    std::string err;
    const int arc = activation_plan(cfg, offs, s, err);
    if (arc != WC_OK) {  // reported like an engine failure of this sub-problem
      w.res.reset(new ProbRes());
      w.res->status = arc;
      w.res->error = err;
      w.state = 2;
    } else {
      ready.push_back(id);
    }
    return id;
  };
  // A finished sub-problem's successors (priority_consensus.rs:254-305): a
  // split makes one sub-problem per consensus group at the same level, no
  // split extends the chain to the next level (or finishes it). They depend
  // on this result alone, so they are made and published at once, even when
  // this sub-problem is still deep in the stack: a group whose sibling is
  // still splitting does not wait for the sibling's whole subtree to start
  // its next level. What enters the stack, the counters and the result order
  // still follow the reference's LIFO unwinding (unwind below).
  auto expand = [&](uint32_t id) {
    PWork& w = *pool[id];
    const uint32_t i = w.owner;
    const wc_chain_problem& q = problems[i];
    const ProbRes& d = *w.res;
    if (!alive[i] || d.status != WC_OK) return;
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
      const uint32_t k1 = make(i, std::move(a1), w.level, w.chain);
      const uint32_t k2 = make(i, std::move(a2), w.level, w.chain);
      pool[id]->kids = {k1, k2};
    } else {
      w.chain.push_back(ch.c1);
      if (w.level + 1 == q.levels) {
        w.final_chain = true;
      } else {
        const uint32_t k = make(i, w.inc, w.level + 1, w.chain);
        pool[id]->kids = {k};
      }
    }
  };

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
      std::vector<uint8_t> inc(q.n_chains);
      for (uint32_t c = 0; c < q.n_chains; ++c) inc[c] = groups[c] == g;
      stacks[i].push_back(make(i, std::move(inc), 0, {}));
    }
  }
  roots_made = true;

  // pop finished tops in LIFO order (priority_consensus.rs:195-307); the
  // counters of a sub-problem are added when it is popped, its successors
  // (made when its result came, expand) go on the stack then
  auto unwind = [&](uint32_t i) {
    ProbRes& pr = R->probs[i];
    while (alive[i] && !stacks[i].empty() && pool[stacks[i].back()]->state == 2) {
      const uint32_t id = stacks[i].back();
      stacks[i].pop_back();
      PWork& w = *pool[id];
      const ProbRes& d = *w.res;
      for (int s = 0; s < S_NSTAT; ++s)
        pr.stats[s] = s == S_PEAKQ ? std::max(pr.stats[s], d.stats[s]) : pr.stats[s] + d.stats[s];
      if (d.status != WC_OK) {
        pr.status = d.status;
        pr.error = d.error;
        alive[i] = false;
        break;
      }
      if (w.final_chain) {
        cons[i].push_back(std::move(w.chain));
        assigns[i].push_back(w.inc);
      } else {
        for (uint32_t k : w.kids) stacks[i].push_back(k);
      }
      w.res.reset();
    }
    // the problem's result is final: record when (tail latency in the bench)
    if (!alive[i] || stacks[i].empty())
      if (R->probs[i].done_ms == 0)
        R->probs[i].done_ms =
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_call).count();
  };

  // 3. epochs of one persistent engine launch each (engine.hip stream mode):
  //    sub-problems are published into a host-mapped ring as soon as they
  //    exist, workgroups claim them in publication order, and every finished
  //    one is consumed (and its children published) while the launch goes on.
  //    Sub-problems that outgrow the epoch's capacities (ST_RETRY) run in a
  //    later epoch with larger ones.
  uint32_t max_chains = 1, max_len = 1;
  bool any_offsets = false;
  for (uint32_t i = 0; i < n; ++i) {
    max_chains = std::max(max_chains, problems[i].n_chains);
    for (uint32_t k = 0; k < problems[i].n_chains * problems[i].levels; ++k) {
      max_len = std::max(max_len, all.rlen_h[all.probs[i].read_begin + k]);
      if (problems[i].offsets && problems[i].offsets[k] >= 0) any_offsets = true;
    }
  }
  double kms = 0;
  uint64_t nl = 0;
  for (uint32_t i = 0; i < n; ++i) unwind(i);
  std::vector<uint32_t> retry;
  while (!ready.empty()) {
    // capacities for anything this epoch may see: every read of every problem,
    // plus the growth earned by the items carried over from the last epoch
    std::vector<SubProb> env(1);
    // (a sub-problem's successors never have more reads than it: the ready
    // ones bound the epoch)
    size_t max_ready = 1;
    for (uint32_t id : ready) max_ready = std::max(max_ready, subs[id].gid.size());
    env[0].gid.assign(std::min<size_t>(max_chains, max_ready), 0);
    env[0].max_len = max_len;
    env[0].max_act = any_offsets ? 1 : 0;
    for (uint32_t id : ready) {
      env[0].wcap_x = std::max(env[0].wcap_x, subs[id].wcap_x);
      env[0].pcap_x = std::max(env[0].pcap_x, subs[id].pcap_x);
      env[0].lcap_x = std::max(env[0].lcap_x, subs[id].lcap_x);
      env[0].rmax_x = std::max(env[0].rmax_x, subs[id].rmax_x);
    }
    Launch* L = launch_slot(ctx, 0);
    if (!L) return set_err(ctx, WC_E_HIP, "stream creation failed");
    // the pool share is planned for a full chip of workgroups; when a retried
    // item's node pool outgrows that share, the epoch runs fewer workgroups
    // (halving, down to one per retried item) so that each gets more HBM
    const size_t nretry = std::count_if(ready.begin(), ready.end(), [&](uint32_t id) { return subs[id].attempts > 0; });
    // a problem rarely has more than a few sub-problems runnable at once (the
    // groups of one split level): a few loci get a few workgroups with large
    // node pools, not a full chip of small ones (cfg4: one locus; allocating
    // pools for 768 workgroups cost seconds per epoch)
    size_t live = 0;
    for (uint32_t i = 0; i < n; ++i) live += alive[i] && !stacks[i].empty();
    const size_t conc_cap = std::max<size_t>(std::max<size_t>(1, nretry), 8 * live);
    size_t conc = std::min<size_t>(4 * ctx->n_cu, conc_cap);
    Caps caps;
    std::string err;
    int prc = WC_OK;
    bool widened = false;
    for (;;) {
      std::vector<uint32_t> ids(conc, 0);
      // (few workgroups, e.g. one deep locus: the 1024-thread dual build)
      prc = plan_caps(ctx, cfg, 2, env, ids, hbm_share(ctx, L->ws.cap, 0.8), caps, err, 8, true);
      // a first epoch whose workgroups fit more than 4 per CU plans for all of them
      if (prc == WC_OK && !widened && nretry == 0 && !caps.pool_short &&
          std::min<size_t>((size_t)caps.per_cu * ctx->n_cu, conc_cap) > conc) {
        widened = true;
        conc = std::min<size_t>((size_t)caps.per_cu * ctx->n_cu, conc_cap);
        continue;
      }
      if (prc != WC_OK || !caps.pool_short || conc <= std::max<size_t>(1, nretry)) break;
      conc = std::max<size_t>(std::max<size_t>(1, nretry), conc / 2);
    }
    if (prc != WC_OK) {
      for (uint32_t id : ready) {
        pool[id]->res.reset(new ProbRes());
        pool[id]->res->status = prc;
        pool[id]->res->error = err;
        pool[id]->state = 2;
      }
      ready.clear();
      for (uint32_t i = 0; i < n; ++i) unwind(i);
      continue;
    }
    int rc2 = stream_epoch(ctx, *L, &all, cfg, caps, subs, ready, [&](uint32_t id, uint32_t st) {
      PWork& w = *pool[id];
      EngineOut& o = outs[id];
      if (st == ~0u) {  // dropped unrun: its problem already failed
        w.res.reset(new ProbRes());
        w.state = 2;
        return;
      }
      if (st & ST_RETRY) {
        bump(subs[id], st);
        if (subs[id].attempts < kMaxAttempts) {
          retry.push_back(id);
          return;
        }
        o.status = WC_E_LIMIT;
        o.error = retry_msg(st, subs[id].attempts);
      }
      w.res.reset(new ProbRes());
      build_dual(o, (uint32_t)subs[id].gid.size(), cfg.consensus_cost, *w.res);
      w.state = 2;
      o.recs.clear();
      owner_pops[w.owner] += w.res->stats[S_POPS];
      if (subs[id].t_pub >= 0) {
        const double st0 = subs[id].t_pub - t_call_ms;
        if (owner_start[w.owner] < 0 || st0 < owner_start[w.owner]) owner_start[w.owner] = st0;
      }
      expand(id);
      if (sublog) {
        // diagnostics: one line per finished sub-problem (the critical path of a locus)
        const double t = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_call).count();
        fprintf(sublog, "%u %u %zu %.3f %.3f %llu %llu %d %d\n", w.owner, w.level, subs[id].gid.size(), w.t_make, t,
                (unsigned long long)w.res->stats[S_POPS], (unsigned long long)w.res->stats[S_UPDATES],
                w.res->status == WC_OK && !w.res->dual.empty() && w.res->dual[0].has_c2 ? 1 : 0, w.res->status);
      }
      unwind(w.owner);
    }, [&](uint32_t id) { return (bool)alive[pool[id]->owner]; }, outs);
    if (rc2 != WC_OK) return rc2;
    kms += L->kernel_ms;
    nl++;
    for (uint32_t id : retry) ready.push_back(id);
    retry.clear();
  }
  for (uint32_t i = 0; i < n; ++i) unwind(i);

  for (uint32_t i = 0; i < n; ++i) {
    ProbRes& pr = R->probs[i];
    pr.start_ms = std::max(0.0, owner_start[i]);
    if (pr.status != WC_OK) continue;
    priority_assemble(problems[i].n_chains, cons[i], assigns[i], pr);
  }
  R->stats.kernel_ms = kms;
  R->stats.launches = nl;
  return WC_OK;
}

// ---------------------------------------------------------------------------
// result types
// ---------------------------------------------------------------------------
int activation_plan(const wc_config& cfg, const std::vector<int64_t>& offsets, SubProb& sp, std::string& err) {
  const size_t n = offsets.size();
  if (n == 0) {
    err = "No sequences provided";
    return WC_E_BAD_INPUT;
  }
  std::vector<int64_t> offs = offsets;
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
  sp.act.assign(n, -1);
  sp.n_active = 0;
  sp.max_act = 0;
  for (size_t i = 0; i < n; ++i) {
    if (offs[i] >= 0) {
      const int64_t a = offs[i] + (int64_t)cfg.offset_compare_length;
      if (a > (int64_t)UINT32_MAX - 2) {
        err = "activation offset beyond the device engine's u32 lengths";
        return WC_E_LIMIT;
      }
      sp.act[i] = a;
      sp.max_act = std::max<uint32_t>(sp.max_act, (uint32_t)a);
    } else {
      sp.n_active++;
    }
  }
  if (sp.n_active == 0) {
    err = err_msg(WC_E_NO_START);
    return WC_E_NO_START;
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
    R->stats.row_bytes += p.stats[S_ROWB];
  }
  R->stats.kernel_ms = kernel_ms;
  R->stats.launches = launches;
  R->stats.wall_ms = wall_ms;
}

// consensus.rs:345 — single results sorted by sequence
void pack_single(wc_results* R, uint32_t p) {
  const ProbRes& pr = R->probs[p];
  R->p_seq0[p] = R->a_seq.size();
  R->p_sc0[p] = R->a_sc.size();
  for (const ConsRec& c : pr.single) {
    R->a_seq.insert(R->a_seq.end(), c.seq.begin(), c.seq.end());
    R->a_sc.insert(R->a_sc.end(), c.scores.begin(), c.scores.end());
  }
}

void build_single(const EngineOut& E, int mode, ProbRes& pr) {
  for (int s = 0; s < S_NSTAT; ++s) pr.stats[s] = E.stats[s];
  pr.status = E.status;
  pr.error = E.error;
  if (pr.status != WC_OK) return;
  for (const RawRecord& rr : E.recs) {
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

void build_dual(const EngineOut& E, uint32_t n, int mode, ProbRes& pr) {
  for (int s = 0; s < S_NSTAT; ++s) pr.stats[s] = E.stats[s];
  pr.status = E.status;
  pr.error = E.error;
  if (pr.status != WC_OK) return;
  for (const RawRecord& rr : E.recs) {
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

}  // namespace wch
