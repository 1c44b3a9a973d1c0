// Per-device submission service (wc_service_*): the reference's one-locus-per-
// call API — ConsensusDWFA::consensus (consensus.rs:139) and
// DualConsensusDWFA::consensus (dual_consensus.rs:240), `consensus(&self)`,
// re-entrant, one instance per host thread (SURVEY §8(b) "Threading") — served
// by persistent stream-mode engine launches instead of one small launch per
// call.
//
// A caller writes its reads into a reservation of the service's pinned,
// host-mapped arena and queues the request — no HIP call on the caller's
// side; the service thread publishes it into the host-mapped ring of a
// running launch ("lane": one persistent launch of the single or dual engine
// for one CdwfaConfig; engine.hip stream mode, the same machinery
// PriorityConsensusDWFA uses). The workgroup that claims it pulls the reads
// into its HBM workspace (engine.hip stage_reads) and runs the search. The
// result comes back through the launch's host-mapped result slots; the
// service builds the reference's result types and wakes that caller. So any
// number of threads calling consensus() share the whole GPU, one workgroup
// per in-flight locus, and a call costs one locus's search latency plus a few
// tens of microseconds.
//
// While a lane runs, the service thread makes no HIP call either: the lane's
// end is read from its workgroups' host-mapped exit flags. A persistent
// kernel shares the process's few hardware queues with every other stream,
// so other threads' work can queue behind it, and a HIP call that waits on
// the runtime lock such a thread holds would stall the heartbeat the lane's
// workgroups watch (they give up after 30 s without one).
//
// One lane runs at a time: it starts on demand and stops after kIdleMs
// without work (its idle workgroups would otherwise hold CUs). A request it
// cannot take — another kind or config, or read counts or lengths beyond its
// planned capacities — makes it drain and restart for that request, in arrival
// order. (Two concurrent lanes would each want the whole chip, and resizing
// one lane's buffers while another runs deadlocks: hipFree waits for every
// kernel on the device, and a lane's kernel only ends when the service thread
// says so.) Offsets (add_sequence_offset), problems that still ask for more
// capacity (ST_RETRY) and any service failure take the batch path
// (wc_consensus_batch with one problem, which plans and retries capacities as
// usual: results never depend on the path). The service thread runs it, on
// its own context, while no lane runs: a batch kernel next to a running lane
// would find the CUs held by the lane's waiting workgroups, and a buffer
// resize (hipFree) would wait for the lane itself. A lane that cannot start
// (HBM) sends its requests there too, after one retry with the lane's cached
// buffers released.
//
// PriorityConsensusDWFA::consensus (priority_consensus.rs:172-341) is served
// the same way (wc_service_priority_consensus): the caller's thread keeps the
// reference's LIFO work stack and submits every DualConsensusDWFA sub-problem
// to the dual lane as soon as it exists (a split's two groups run at once),
// unwinding the stack in the reference's order as the tops finish.
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <thread>

#include "sched.hpp"

using namespace wc;
using namespace wch;

namespace {

constexpr uint32_t kQcap = 1u << 14;      // published, unfinished problems per lane
constexpr uint32_t kQslots = 1u << 21;    // their read-table entries
constexpr double kIdleMs = 2.0;           // a lane with nothing to do stops after this
constexpr uint64_t kArenaDefault = 256ull << 20;  // pinned host memory for in-flight callers' reads

using Clock = std::chrono::steady_clock;

struct Req {
  uint32_t sides = 1;
  wc_config cfg;
  SubProb sp;                  // gid = 0..n-1 (read k of this request); activation plan
  std::vector<uint64_t> roff;  // arena offsets of the reads
  std::vector<uint32_t> rlen;
  uint64_t aoff = 0;           // arena reservation
  bool in_arena = false;       // holds it
  bool done = false;
  uint32_t st = 0;             // raw device status (ST_RETRY flags included; ~0u = service failure)
  EngineOut out;
  std::condition_variable cv;
  // the batch path, run by the service thread: the caller's problem (valid
  // until the request completes) and the outcome
  const wc_problem* fb_p = nullptr;
  bool fb = false;
  wc_results* fb_res = nullptr;
  int fb_rc = WC_OK;
  std::condition_variable* notify = nullptr;  // also woken on completion (a priority call's requests)
  bool counted = false;                       // counted as served (poll_req)
};

bool same_cfg(const wc_config& a, const wc_config& b) { return memcmp(&a, &b, sizeof(wc_config)) == 0; }

struct Lane {
  bool running = false;
  bool draining = false;  // a queued request needs larger capacities: finish, then restart
  uint32_t sides = 1;
  wc_config cfg;
  uint32_t nmax = 0, maxlen = 0;  // capacity envelope the launch was planned for
  Launch* L = nullptr;
  volatile StreamCtl* sc = nullptr;
  DevProblem* qp = nullptr;
  uint64_t* qroff = nullptr;
  int64_t* qract = nullptr;
  uint32_t* qrlen = nullptr;
  std::vector<Req*> seq_req;
  std::vector<uint64_t> seq_rw;
  std::vector<uint8_t> seq_done;
  uint32_t oldest = 0, outstanding = 0, published_tail = 0, beat = 0;
  uint32_t grid_full = 0;  // workgroups a full-chip launch of this lane would ask for
  bool can_grow = false;   // a restart with more requests waiting would get more workgroups
  uint64_t rw = 0;
  Clock::time_point idle_since, started, last_result, last_query, last_warn;
};

}  // namespace

struct wc_service {
  int device = 0;
  wc_ctx* ctx = nullptr;
  std::mutex mu;
  std::condition_variable cv_svc;    // requests arrived
  std::condition_variable cv_arena;  // arena space was released
  std::deque<Req*> ready;            // copied to the arena, not yet published (FIFO)
  std::deque<Req*> fbq;              // batch-path requests (run by the service thread, no lane running)
  uint32_t inflight = 0;             // calls inside the service (destroy waits for them)
  std::condition_variable cv_idle;   // inflight reached 0
  HostBuf arena;                     // pinned, host-mapped: callers' reads (the lanes pull them)
  const uint8_t* arena_dev = nullptr;  // its device address
  std::map<uint64_t, uint64_t> live;  // arena reservations: offset -> bytes
  uint64_t cursor = 0;
  Lane lane;  // at most one running launch (see service_loop)
  std::thread th;
  bool stop = false;
  std::string err;
  wc_service_stats stats{};
};

namespace {

// ---- arena reservations (caller threads, under mu) ----
bool arena_fits(const wc_service* S, uint64_t p, uint64_t b) {
  if (p + b > S->arena.cap) return false;
  auto it = S->live.upper_bound(p);
  if (it != S->live.end() && it->first < p + b) return false;
  if (it != S->live.begin()) {
    const auto pr = std::prev(it);
    if (pr->first + pr->second > p) return false;
  }
  return true;
}
bool arena_alloc(wc_service* S, uint64_t b, uint64_t& off) {
  uint64_t p = S->cursor;
  bool ok = arena_fits(S, p, b);
  if (!ok && arena_fits(S, 0, b)) {
    p = 0;
    ok = true;
  }
  if (!ok)
    for (const auto& kv : S->live)
      if (arena_fits(S, kv.first + kv.second, b)) {
        p = kv.first + kv.second;
        ok = true;
        break;
      }
  if (!ok) return false;
  S->live[p] = b;
  S->cursor = p + b;
  off = p;
  return true;
}

void complete(wc_service* S, Req* q, uint32_t st) {
  q->st = st;
  q->done = true;
  if (q->in_arena) {
    S->live.erase(q->aoff);
    q->in_arena = false;
    S->cv_arena.notify_all();
  }
  q->cv.notify_one();
  if (q->notify) q->notify->notify_all();
}

// ---- lanes (service thread, under mu) ----
bool lane_fits(const Lane& ln, const Req* q) {
  return ln.running && !ln.draining && ln.sides == q->sides && same_cfg(ln.cfg, q->cfg) &&
         q->sp.gid.size() <= ln.nmax && q->sp.max_len <= ln.maxlen;
}

// starts the lane for the requests waiting with q's kind and config
int lane_start(wc_service* S, const Req* q) {
  Lane& ln = S->lane;
  Launch* const prev = ln.L;
  ln = Lane();
  ln.L = prev;
  ln.sides = q->sides;
  ln.cfg = q->cfg;
  // capacity envelope: every waiting request of this kind and config, rounded up
  uint32_t nmax = 1, maxlen = 1;
  for (const Req* r : S->ready)
    if (r->sides == q->sides && same_cfg(r->cfg, q->cfg)) {
      nmax = std::max<uint32_t>(nmax, (uint32_t)r->sp.gid.size());
      maxlen = std::max(maxlen, r->sp.max_len);
    }
  ln.nmax = std::min<uint32_t>((nmax + 7) / 8 * 8, (uint32_t)kBlock);
  ln.maxlen = (maxlen + 1023) / 1024 * 1024;
  std::vector<SubProb> env(1);
  env[0].gid.assign(ln.nmax, 0);
  env[0].max_len = ln.maxlen;
  wc_ctx* ctx = S->ctx;
  Launch* L = launch_slot(ctx, 0);
  if (!L) return set_err(ctx, WC_E_HIP, "stream creation failed");
  ln.L = L;
  // workgroups: twice the requests waiting for this lane (callers block on
  // their result, so that bounds what it will see), 64 at least; the lane
  // restarts larger if its callers outgrow it. Planned like a batch launch of
  // that many problems (a small one gets the 2-wave build), with a quarter of
  // the free HBM for the node pools.
  uint32_t waiting = 0;
  for (const Req* r : S->ready) waiting += r->sides == q->sides && same_cfg(r->cfg, q->cfg);
  ln.grid_full = 4 * (uint32_t)ctx->n_cu;
  const uint32_t want = std::min(ln.grid_full, std::max(64u, (2 * waiting + 63) / 64 * 64));
  std::vector<uint32_t> ids(want, 0);
  Caps caps;
  std::string err;
  int rc = plan_caps(ctx, ln.cfg, ln.sides, env, ids, hbm_share(ctx, L->ws.cap, 0.25), caps, err);
  if (rc != WC_OK) return set_err(ctx, rc, err);
  L->caps = caps;
  L->grid = std::min<uint32_t>((uint32_t)std::max(1, caps.per_cu) * (uint32_t)ctx->n_cu, std::max(1u, caps.conc));
  // a larger launch would have more workgroups only if this one got all it asked for
  ln.can_grow = L->grid >= want && want < ln.grid_full;
  L->P = 2 * L->grid;  // two output slots per workgroup
  L->kernel_ms = 0;
  const uint32_t P = L->P;
  L->stream_layout();
  if (!L->host.ensure(L->off_out + (uint64_t)P * caps.ob, true))
    return set_err(ctx, WC_E_HIP, "pinned host allocation failed (service results)");
  memset(L->host.p, 0, L->off_out);
  const uint64_t off_q = align16(sizeof(StreamCtl));
  const uint64_t off_roff = off_q + align16((uint64_t)kQcap * sizeof(DevProblem));
  const uint64_t off_ract = off_roff + (uint64_t)kQslots * 8;
  const uint64_t off_rlen = off_ract + (uint64_t)kQslots * 8;
  if (!L->ring.ensure(off_rlen + (uint64_t)kQslots * 4, true))
    return set_err(ctx, WC_E_HIP, "pinned host allocation failed (service ring)");
  uint8_t* rh = (uint8_t*)L->ring.p;
  ln.sc = (volatile StreamCtl*)rh;
  ln.sc->tail = 0;
  ln.sc->stop = 0;
  ln.sc->abort = 0;
  ln.sc->heartbeat = 0;
  ln.qp = (DevProblem*)(rh + off_q);
  ln.qroff = (uint64_t*)(rh + off_roff);
  ln.qract = (int64_t*)(rh + off_ract);
  ln.qrlen = (uint32_t*)(rh + off_rlen);
  // workspace per workgroup: engine | read table | staged reads | guard
  const uint64_t rstride = rstage_stride(ln.maxlen);
  const uint64_t wsb = caps.wsb + rtab_bytes(caps.nmax) + (uint64_t)caps.nmax * rstride + kGuard;
  if (!L->ws.ensure(wsb * L->grid + 64) || !L->counter.ensure(4))
    return set_err(ctx, WC_E_HIP, "device allocation failed (service workspace)");
  HIPCHK(hipMemsetAsync(L->counter.p, 0, 4, L->stream));
  void *dhost = nullptr, *dring = nullptr;
  HIPCHK(hipHostGetDevicePointer(&dhost, L->host.p, 0));
  HIPCHK(hipHostGetDevicePointer(&dring, L->ring.p, 0));
  uint8_t* dh = (uint8_t*)dhost;
  uint8_t* dr = (uint8_t*)dring;
  int clk = 0;
  if (hipDeviceGetAttribute(&clk, hipDeviceAttributeWallClockRate, S->device) != hipSuccess || clk <= 0) clk = 100000;
  EngineArgs a;
  memset(&a, 0, sizeof(a));
  a.cfg = to_dev(ln.cfg);
  a.problems = (const DevProblem*)(dr + off_q);
  a.sides = ln.sides;
  a.rbytes = (const uint8_t*)L->ws.p;  // staged reads are addressed from the workspace base
  a.hreads = S->arena_dev;
  a.rstage_stride = rstride;
  a.roff = (const uint64_t*)(dr + off_roff);
  a.rlen = (const uint32_t*)(dr + off_rlen);
  a.ractivate = (const int64_t*)(dr + off_ract);
  a.ws = (uint8_t*)L->ws.p;
  a.ws_stride = wsb;
  a.pcap = caps.pcap;
  a.wcap = caps.wcap;
  a.lcap = caps.lcap;
  a.nmax = caps.nmax;
  a.rmax = caps.rmax;
  a.chain = caps.chain;
  a.chain_kinds = env_chain_kinds();
  a.dual_hot = caps.dual_hot ? 1u : 0u;
  a.out = dh + L->off_out;
  a.out_stride = caps.ob;
  a.status = (uint32_t*)(dh + L->off_status);
  a.stats = (uint64_t*)(dh + L->off_stats);
  a.done = (uint32_t*)dh;
  a.stream = 1;
  a.qcap = kQcap;
  a.qslots = kQslots;
  a.sctl = (StreamCtl*)dr;
  a.qhead = (uint32_t*)L->counter.p;
  a.idle_ticks = (uint64_t)clk * 1000ull * 30ull;  // 30 s without a heartbeat: the host is gone
  a.exited = (uint32_t*)(dh + L->off_exit);
  persistent_begin();
  rc = launch_kernel(ctx, *L, a, caps);
  if (rc != WC_OK) {
    persistent_end();
    return rc;
  }
  L->busy = true;
  ln.running = true;
  ln.idle_since = ln.started = ln.last_result = Clock::now();
  S->stats.lane_starts++;
  if (getenv("WC_LAUNCH_LOG"))
    fprintf(stderr, "[wc] service lane: sides=%u grid=%u per_cu=%d nmax=%u maxlen=%u pcap=%u wcap=%u lcap=%u chain=%u\n",
            ln.sides, L->grid, caps.per_cu, caps.nmax, ln.maxlen, caps.pcap, caps.wcap, caps.lcap, caps.chain);
  return WC_OK;
}

// publishes q into lane ln's ring; false when the ring is full
bool lane_publish(Lane& ln, Req* q) {
  const uint32_t seq = (uint32_t)ln.seq_req.size();
  const uint32_t n = (uint32_t)q->sp.gid.size();
  const uint64_t ow = ln.oldest < seq ? ln.seq_rw[ln.oldest] : ln.rw;
  if (seq - ln.oldest >= kQcap || ln.rw + n - ow > kQslots) return false;
  DevProblem d;
  memset(&d, 0, sizeof(d));
  d.read_begin = (uint32_t)(ln.rw % kQslots);
  d.n_reads = n;
  d.max_read_len = q->sp.max_len;
  d.n_active = q->sp.n_active;
  d.max_act = q->sp.max_act;
  ln.qp[seq % kQcap] = d;
  for (uint32_t r = 0; r < n; ++r) {
    const uint64_t k = (ln.rw + r) % kQslots;
    ln.qroff[k] = q->roff[r];
    ln.qract[k] = q->sp.act[r];
    ln.qrlen[k] = q->rlen[r];
  }
  ln.seq_req.push_back(q);
  ln.seq_rw.push_back(ln.rw);
  ln.seq_done.push_back(0);
  ln.rw += n;
  ln.outstanding++;
  return true;
}

// harvests every finished problem of the lane; returns how many
uint32_t lane_poll(wc_service* S, Lane& ln) {
  Launch& L = *ln.L;
  volatile uint32_t* done = L.done();
  uint32_t got = 0;
  for (uint32_t slot = 0; slot < L.P; ++slot) {
    const uint32_t v = __atomic_load_n(&done[slot], __ATOMIC_ACQUIRE);
    if (!v) continue;
    const uint32_t seq = v - 1;
    Req* q = ln.seq_req[seq];
    const uint32_t st = harvest(L, slot, q->sp, q->out);
    __atomic_store_n(&done[slot], 0u, __ATOMIC_RELEASE);  // the slot may be reused
    ln.seq_done[seq] = 1;
    ln.outstanding--;
    while (ln.oldest < ln.seq_req.size() && ln.seq_done[ln.oldest]) ln.oldest++;
    complete(S, q, st);
    got++;
  }
  return got;
}

// ends the lane's launch (nothing may be outstanding unless it failed): every
// workgroup leaves its claim loop (exit flags, heartbeat kept up) before the
// one HIP call that retires the launch
void lane_stop(wc_service* S, Lane& ln, bool failed) {
  __atomic_store_n(&ln.sc->stop, 1u, __ATOMIC_RELEASE);
  const auto t0 = Clock::now();
  while (!ln.L->all_exited() && !ln.sc->abort &&
         std::chrono::duration<double>(Clock::now() - t0).count() < 60.0) {
    __atomic_store_n(&ln.sc->heartbeat, ++ln.beat, __ATOMIC_RELAXED);
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
  (void)launch_finish(S->ctx, *ln.L);
  persistent_end();
  if (failed)
    for (uint32_t s = ln.oldest; s < ln.seq_req.size(); ++s)
      if (!ln.seq_done[s]) complete(S, ln.seq_req[s], ~0u);
  ln.running = false;
  ln.draining = false;
  ln.seq_req.clear();
  ln.seq_rw.clear();
  ln.seq_done.clear();
}

void service_loop(wc_service* S) {
  (void)hipSetDevice(S->device);
  std::unique_lock<std::mutex> lk(S->mu);
  Lane& ln = S->lane;
  const bool trace = getenv("WC_SVC_TRACE") != nullptr;  // diagnostics: report stalls of this loop
  Clock::time_point last_beat = Clock::now();
  for (;;) {
    bool progress = false;
    // 0. batch-path requests, one at a time, with no lane running
    if (!S->fbq.empty() && !ln.running) {
      Req* f = S->fbq.front();
      S->fbq.pop_front();
      S->stats.fallback++;
      lk.unlock();
      wc_results* r = nullptr;
      const int rc = f->sides == 1 ? wc_consensus_batch(S->ctx, &f->cfg, 1, f->fb_p, &r)
                                   : wc_dual_consensus_batch(S->ctx, &f->cfg, 1, f->fb_p, &r);
      const std::string e = rc != WC_OK ? std::string(wc_last_error(S->ctx)) : std::string();
      lk.lock();
      if (rc != WC_OK) S->err = e;
      f->fb_rc = rc;
      f->fb_res = r;
      f->done = true;
      f->cv.notify_one();
      if (f->notify) f->notify->notify_all();
      continue;
    }
    if (ln.running) {
      // a batch-path request needs the device to itself: the lane drains
      if (!S->fbq.empty()) ln.draining = true;
      // 1. publish in arrival order; the first request the lane cannot take
      //    (another kind or config, or larger capacities) makes it drain, and
      //    nothing behind that request is published before the restart
      while (!ln.draining && !S->ready.empty()) {
        Req* q = S->ready.front();
        if (!lane_fits(ln, q)) {
          ln.draining = true;
          break;
        }
        if (!lane_publish(ln, q)) break;  // ring full
        S->ready.pop_front();
        progress = true;
      }
    } else if (!S->ready.empty()) {
      // a lane for the oldest request's kind and config. Buffers are only
      // resized here, with no lane running: hipFree waits for every kernel on
      // the device, the lane's own included, and that one only ends when this
      // thread tells it to.
      const Req* q = S->ready.front();
      int rc = lane_start(S, q);
      if (rc != WC_OK && ln.L) {  // most often HBM: drop the cached buffers and try once more
        launch_release_buffers(*ln.L);
        rc = lane_start(S, q);
      }
      if (rc != WC_OK) {
        // this request and the others of its kind and config take the batch path
        S->stats.lane_failures++;
        S->err = S->ctx->err;
        if (getenv("WC_LAUNCH_LOG")) fprintf(stderr, "[wc] service lane start failed: %s\n", S->err.c_str());
        const uint32_t sides = q->sides;
        const wc_config cfg = q->cfg;
        for (auto jt = S->ready.begin(); jt != S->ready.end();) {
          if ((*jt)->sides == sides && same_cfg((*jt)->cfg, cfg)) {
            complete(S, *jt, ~0u);
            jt = S->ready.erase(jt);
          } else {
            ++jt;
          }
        }
      }
      progress = true;
      continue;  // publish on the next pass
    }
    // 2. heartbeat, tail, harvest; 3. stop the lane when it is done (idle,
    //    draining and empty, or failed)
    if (ln.running) {
      __atomic_store_n(&ln.sc->heartbeat, ++ln.beat, __ATOMIC_RELAXED);
      if (trace) {
        const auto now = Clock::now();
        const double gap = std::chrono::duration<double, std::milli>(now - last_beat).count();
        if (ln.beat > 1 && gap > 20.0) fprintf(stderr, "[wc] service loop: %.1f ms between heartbeats\n", gap);
        last_beat = now;
      }
      const uint32_t ntail = (uint32_t)ln.seq_req.size();
      if (ntail != ln.published_tail) {
        std::atomic_thread_fence(std::memory_order_release);
        __atomic_store_n(&ln.sc->tail, ntail, __ATOMIC_RELEASE);
        ln.published_tail = ntail;
      }
      if (lane_poll(S, ln)) {
        progress = true;
        ln.last_result = Clock::now();
      }
      // a lane planned for fewer workgroups than its callers keep busy drains
      // and restarts with a larger grid
      if (!ln.draining && ln.can_grow) {
        uint32_t waiting = 0;
        for (const Req* r : S->ready) waiting += r->sides == ln.sides && same_cfg(r->cfg, ln.cfg);
        if (2 * (ln.outstanding + waiting) > 3 * ln.L->grid) ln.draining = true;
      }
      if (ln.outstanding > 0) {
        ln.idle_since = Clock::now();
        // ended (gave up, or every workgroup left) with problems out. No HIP
        // call while the lane runs (see Launch::all_exited); a stream query
        // only after seconds without a result, to notice a faulted launch
        const uint32_t ab = ln.sc->abort;
        bool ended = ab || ln.L->all_exited();
        const auto now = Clock::now();
        const double quiet = std::chrono::duration<double>(now - ln.last_result).count();
        if (quiet > 20.0 && std::chrono::duration<double>(now - ln.last_warn).count() > 20.0) {
          ln.last_warn = now;  // a lane that stops finishing says so (always)
          fprintf(stderr, "[wc] service lane: no locus finished for %.0f s (%u outstanding, %u of %u workgroups "
                          "exited, abort %u)\n", quiet, ln.outstanding, ln.L->n_exited(), ln.L->grid, ab);
        }
        if (!ended && quiet > 5.0 &&
            std::chrono::duration<double>(now - ln.last_query).count() > 1.0) {
          ln.last_query = now;
          ended = hipStreamQuery(ln.L->stream) != hipErrorNotReady;
        }
        if (ended) {  // ended with problems out: fail them over
          char buf[160];
          snprintf(buf, sizeof(buf), "service lane ended with %u problems outstanding (abort %u, %.1f ms after its start)",
                   ln.outstanding, ab, std::chrono::duration<double, std::milli>(Clock::now() - ln.started).count());
          S->err = buf;
          if (getenv("WC_LAUNCH_LOG")) fprintf(stderr, "[wc] %s\n", buf);
          lane_stop(S, ln, true);
          S->stats.lane_failures++;
          progress = true;
        }
      } else {
        const double idle = std::chrono::duration<double, std::milli>(Clock::now() - ln.idle_since).count();
        if (ln.draining || S->stop || idle > kIdleMs) {
          lane_stop(S, ln, false);
          progress = true;
        }
      }
    }
    // A stopping service still serves the calls already inside: a priority
    // call submits its next sub-problem, and a retried or failed-lane request
    // comes back through fbq, after stop is set. It ends with the last of them
    // (~InFlight wakes it).
    if (S->stop && S->inflight == 0 && S->ready.empty() && S->fbq.empty() && !ln.running) break;
    if (!progress) {
      if (!ln.running && S->ready.empty() && S->fbq.empty())
        S->cv_svc.wait(lk, [&] { return (S->stop && S->inflight == 0) || !S->ready.empty() || !S->fbq.empty(); });
      else S->cv_svc.wait_for(lk, std::chrono::microseconds(20));
    }
  }
}

// ---- requests (caller threads) ----
// An RAII count of the calls inside the service: wc_service_destroy waits
// until none is left. A call that finds the service stopping fails.
struct InFlight {
  wc_service* S;
  bool ok;
  explicit InFlight(wc_service* s) : S(s) {
    std::lock_guard<std::mutex> g(S->mu);
    ok = !S->stop;
    if (ok) S->inflight++;
  }
  ~InFlight() {
    if (!ok) return;
    std::lock_guard<std::mutex> g(S->mu);
    if (--S->inflight == 0) {
      S->cv_idle.notify_all();
      S->cv_svc.notify_all();  // a stopping service thread waits for the last call
    }
  }
};

// queues q for the batch path (the service thread runs it with no lane running)
void queue_fallback(wc_service* S, Req* q, const wc_problem* p) {
  std::lock_guard<std::mutex> g(S->mu);
  q->fb = true;
  q->fb_p = p;
  q->done = false;
  S->fbq.push_back(q);
  S->cv_svc.notify_one();
}

// Submits one problem (no waiting): into a lane through the arena, or to the
// batch path (offsets, > 256 reads, reads too large for the arena). `p` must
// stay valid until the request completes.
std::unique_ptr<Req> submit(wc_service* S, uint32_t sides, const wc_config* cfg, const wc_problem* p,
                            std::condition_variable* notify = nullptr) {
  std::unique_ptr<Req> q(new Req());
  q->notify = notify;
  q->sides = sides;
  q->cfg = *cfg;
  const uint32_t n = p->n_reads;
  std::vector<int64_t> offs(n, -1);
  if (p->offsets)
    for (uint32_t r = 0; r < n; ++r) offs[r] = p->offsets[r] < 0 ? -1 : p->offsets[r];
  std::string aerr;
  const int arc = activation_plan(*cfg, offs, q->sp, aerr);
  {
    std::lock_guard<std::mutex> g(S->mu);
    S->stats.calls++;
  }
  // offsets (activation scratch) and deep problems (> 256 reads: the batch
  // path gives them a launch of their own) take the batch path
  if (arc != WC_OK || q->sp.max_act > 0 || n > (uint32_t)kBlock) {
    queue_fallback(S, q.get(), p);
    return q;
  }
  // reads back to back (16-byte aligned) in a reservation of the pinned
  // arena, written straight from the caller's buffers: the lane's workgroups
  // pull them into HBM when they claim the locus, so a call makes no HIP
  // call at all (a copy on a stream could queue behind the running lane)
  std::vector<uint64_t> rel(n);
  uint64_t total = 0;
  for (uint32_t r = 0; r < n; ++r) {
    rel[r] = total;
    total += (p->lens[r] + 15) & ~15ull;
  }
  total = std::max<uint64_t>(total, 16);
  {
    std::unique_lock<std::mutex> lk(S->mu);
    if (total > S->arena.cap / 4) {
      lk.unlock();
      queue_fallback(S, q.get(), p);
      return q;
    }
    S->cv_arena.wait(lk, [&] { return S->stop || arena_alloc(S, total, q->aoff); });
    if (S->stop) {  // (the service thread runs until inflight is 0: the request still completes)
      lk.unlock();
      queue_fallback(S, q.get(), p);
      return q;
    }
    q->in_arena = true;
  }
  uint8_t* h = (uint8_t*)S->arena.p + q->aoff;
  q->sp.gid.resize(n);
  q->rlen.resize(n);
  q->roff.resize(n);
  for (uint32_t r = 0; r < n; ++r) {
    const uint64_t len = p->lens[r], pad = ((len + 15) & ~15ull) - len;
    if (len) memcpy(h + rel[r], p->reads[r], len);
    if (pad) memset(h + rel[r] + len, 0, pad);
    q->sp.gid[r] = r;
    q->rlen[r] = (uint32_t)len;
    q->roff[r] = q->aoff + rel[r];
    q->sp.max_len = std::max(q->sp.max_len, q->rlen[r]);
    q->sp.work += len;
  }
  q->fb_p = p;
  std::lock_guard<std::mutex> g(S->mu);
  S->ready.push_back(q.get());
  S->cv_svc.notify_one();
  return q;
}

// Waits for q. A lane outcome that asks for more capacity (ST_RETRY) or a
// failed lane sends the problem to the batch path and waits again. Returns
// WC_OK with either q->out (lane) or q->fb_res (batch path) filled, or the
// batch path's error code.
int wait_req(wc_service* S, Req* q) {
  {
    std::unique_lock<std::mutex> lk(S->mu);
    q->cv.wait(lk, [&] { return q->done; });
    if (q->fb) return q->fb_rc;
    if (q->st != ~0u && !(q->st & ST_RETRY)) {
      S->stats.served++;
      return WC_OK;
    }
    if (q->st != ~0u) S->stats.retried++;
  }
  queue_fallback(S, q, q->fb_p);
  std::unique_lock<std::mutex> lk(S->mu);
  q->cv.wait(lk, [&] { return q->done; });
  return q->fb_rc;
}

int service_call(wc_service* S, uint32_t sides, const wc_config* cfg, const wc_problem* p, wc_results** out) {
  *out = nullptr;
  if (!S || !cfg || !p) return WC_E_BAD_INPUT;
  const auto t0 = Clock::now();
  const uint32_t n = p->n_reads;
  if (n && (!p->reads || !p->lens)) return WC_E_BAD_INPUT;
  for (uint32_t r = 0; r < n; ++r)
    if (p->lens[r] >= (1ull << 31) || (p->lens[r] && !p->reads[r])) return WC_E_BAD_INPUT;
  InFlight in(S);
  if (!in.ok) return WC_E_HIP;  // the service is shutting down
  std::unique_ptr<Req> q = submit(S, sides, cfg, p);
  const int rc = wait_req(S, q.get());
  if (q->fb) {
    *out = q->fb_res;
    return rc;
  }
  std::unique_ptr<wc_results> R(new wc_results());
  R->kind = sides == 1 ? 0 : 1;
  R->probs.resize(1);
  if (sides == 1) build_single(q->out, cfg->consensus_cost, R->probs[0]);
  else build_dual(q->out, n, cfg->consensus_cost, R->probs[0]);
  fill_stats(R.get(), 0.0, 0, std::chrono::duration<double, std::milli>(Clock::now() - t0).count());
  *out = R.release();
  return WC_OK;
}

// ---- PriorityConsensusDWFA::consensus (priority_consensus.rs:172-341) ----
// one sub-problem of a call: a read subset at a chain level
struct PSub {
  std::vector<uint8_t> inc;
  uint32_t level = 0;
  std::vector<ConsRec> chain;
  std::vector<const uint8_t*> rp;
  std::vector<uint64_t> rl;
  std::vector<int64_t> ro;
  wc_problem wp{};
  std::unique_ptr<Req> rq;
  bool done = false;         // result known (and successors made)
  ProbRes res;
  std::vector<size_t> kids;  // successors, made when the result came; stacked when this one is popped
  bool final_chain = false;
};

// The outcome of a finished request: 0 = pending (still running, or just
// sent to the batch path), 1 = done (lane or batch result in q), -1 = the
// batch path failed (q->fb_rc). Caller holds S->mu.
int poll_req(wc_service* S, Req* q) {
  if (!q->done) return 0;
  if (q->fb) return q->fb_rc == WC_OK ? 1 : -1;
  if (q->st != ~0u && !(q->st & ST_RETRY)) {
    if (!q->counted) {
      q->counted = true;
      S->stats.served++;
    }
    return 1;
  }
  if (q->st != ~0u) S->stats.retried++;
  q->fb = true;  // capacity retry or a failed lane: the batch path (queue_fallback without re-locking)
  q->done = false;
  S->fbq.push_back(q);
  S->cv_svc.notify_one();
  return 0;
}

int service_priority(wc_service* S, const wc_config* cfg, const wc_chain_problem* q, wc_results** out) {
  *out = nullptr;
  if (!S || !cfg || !q) return WC_E_BAD_INPUT;
  const auto t0 = Clock::now();
  const uint64_t nr = (uint64_t)q->n_chains * q->levels;
  if (nr && (!q->reads || !q->lens)) return WC_E_BAD_INPUT;
  for (uint64_t k = 0; k < nr; ++k)
    if (q->lens[k] >= (1ull << 31) || (q->lens[k] && !q->reads[k])) return WC_E_BAD_INPUT;
  InFlight in(S);
  if (!in.ok) return WC_E_HIP;
  std::unique_ptr<wc_results> R(new wc_results());
  R->kind = 2;
  R->probs.resize(1);
  ProbRes& pr = R->probs[0];
  if (q->n_chains == 0 || q->levels == 0) {
    pr.status = WC_E_BAD_INPUT;
    pr.error = "Must provide a non-empty sequences Vec";
    fill_stats(R.get(), 0.0, 0, std::chrono::duration<double, std::milli>(Clock::now() - t0).count());
    *out = R.release();
    return WC_OK;
  }
  std::condition_variable call_cv;  // any of this call's requests completed
  std::vector<std::unique_ptr<PSub>> subs;
  std::vector<size_t> stack;  // the reference's LIFO work stack (indices into subs)
  std::vector<std::vector<ConsRec>> cons;
  std::vector<std::vector<uint8_t>> assigns;
  // a new sub-problem, submitted at once
  auto make = [&](std::vector<uint8_t> inc, uint32_t level, std::vector<ConsRec> chain) -> size_t {
    std::unique_ptr<PSub> w(new PSub());
    w->inc = std::move(inc);
    w->level = level;
    w->chain = std::move(chain);
    for (uint32_t c = 0; c < q->n_chains; ++c) {
      if (!w->inc[c]) continue;
      const uint64_t k = (uint64_t)c * q->levels + level;
      w->rp.push_back(q->reads[k]);
      w->rl.push_back(q->lens[k]);
      w->ro.push_back(q->offsets && q->offsets[k] >= 0 ? q->offsets[k] : -1);
    }
    w->wp.n_reads = (uint32_t)w->rp.size();
    w->wp.reads = w->rp.data();
    w->wp.lens = w->rp.empty() ? nullptr : w->rl.data();
    w->wp.offsets = w->ro.data();
    w->rq = submit(S, 2, cfg, &w->wp, &call_cv);
    subs.push_back(std::move(w));
    return subs.size() - 1;
  };
  // a finished sub-problem: its result and its successors (made at once, as
  // in priority_stream's expand: they depend on this result alone)
  auto finish = [&](size_t id) {
    PSub& w = *subs[id];
    if (w.rq->fb) {
      w.res = std::move(w.rq->fb_res->probs[0]);
      wc_results_free(w.rq->fb_res);
      w.rq->fb_res = nullptr;
    } else {
      build_dual(w.rq->out, w.wp.n_reads, cfg->consensus_cost, w.res);
    }
    w.done = true;
    if (w.res.status != WC_OK) return;
    const DualRec& ch = w.res.dual[0];
    if (ch.has_c2) {
      std::vector<uint8_t> a1(q->n_chains, 0), a2(q->n_chains, 0);
      size_t idx = 0;
      for (uint32_t c = 0; c < q->n_chains; ++c) {
        if (!w.inc[c]) continue;
        (ch.is_c1[idx] ? a1 : a2)[c] = 1;
        idx++;
      }
      const std::vector<ConsRec> chain = w.chain;
      const uint32_t level = w.level;
      const size_t k1 = make(std::move(a1), level, chain);
      const size_t k2 = make(std::move(a2), level, chain);
      subs[id]->kids = {k1, k2};
    } else {
      subs[id]->chain.push_back(ch.c1);
      if (subs[id]->level + 1 == q->levels) {
        subs[id]->final_chain = true;
      } else {
        const size_t k = make(subs[id]->inc, subs[id]->level + 1, subs[id]->chain);
        subs[id]->kids = {k};
      }
    }
  };
  {
    std::vector<int64_t> groups(q->n_chains, -1);
    if (q->seed_groups)
      for (uint32_t c = 0; c < q->n_chains; ++c) groups[c] = q->seed_groups[c] < 0 ? -1 : q->seed_groups[c];
    for (int64_t g : seed_order(groups)) {
      std::vector<uint8_t> inc(q->n_chains);
      for (uint32_t c = 0; c < q->n_chains; ++c) inc[c] = groups[c] == g;
      stack.push_back(make(std::move(inc), 0, {}));
    }
  }
  int rc = WC_OK;
  bool stop = false;
  while (!stack.empty() && !stop) {
    // results that came in (any sub-problem, not only the stack's top)
    std::vector<size_t> fin;
    {
      std::unique_lock<std::mutex> lk(S->mu);
      for (;;) {
        for (size_t id = 0; id < subs.size(); ++id) {
          if (subs[id]->done) continue;
          const int pst = poll_req(S, subs[id]->rq.get());
          if (pst < 0) {
            rc = subs[id]->rq->fb_rc;
            stop = true;
          } else if (pst > 0) {
            fin.push_back(id);
          }
        }
        if (stop || !fin.empty()) break;
        call_cv.wait(lk);
      }
    }
    if (stop) break;
    for (size_t id : fin) finish(id);
    // pop finished tops in the reference's order; counters are added then
    while (!stack.empty() && subs[stack.back()]->done) {
      const size_t id = stack.back();
      stack.pop_back();
      PSub& w = *subs[id];
      for (int s = 0; s < S_NSTAT; ++s)
        pr.stats[s] = s == S_PEAKQ ? std::max(pr.stats[s], w.res.stats[s]) : pr.stats[s] + w.res.stats[s];
      if (w.res.status != WC_OK) {
        pr.status = w.res.status;
        pr.error = w.res.error;
        stop = true;
        break;
      }
      if (w.final_chain) {
        cons.push_back(std::move(w.chain));
        assigns.push_back(w.inc);
      } else {
        for (size_t k : w.kids) stack.push_back(k);
      }
    }
  }
  // the search is over (or failed): every request still out finishes first
  // (they read this call's request records and the caller's buffers)
  {
    std::unique_lock<std::mutex> lk(S->mu);
    for (;;) {
      bool pending = false;
      for (auto& w : subs)
        if (!w->done && poll_req(S, w->rq.get()) == 0) pending = true;
      if (!pending) break;
      call_cv.wait(lk);
    }
  }
  for (auto& w : subs)
    if (w->rq->fb_res) wc_results_free(w->rq->fb_res);
  if (rc != WC_OK) return rc;
  if (pr.status == WC_OK) priority_assemble(q->n_chains, cons, assigns, pr);
  fill_stats(R.get(), 0.0, 0, std::chrono::duration<double, std::milli>(Clock::now() - t0).count());
  *out = R.release();
  return WC_OK;
}

}  // namespace

extern "C" {

int wc_service_create(int device, uint64_t arena_bytes, wc_service** out) {
  *out = nullptr;
  std::unique_ptr<wc_service> S(new wc_service());
  S->device = device;
  int rc = wc_ctx_create(device, &S->ctx);
  if (rc != WC_OK) return rc;
  void* dev = nullptr;
  if (!S->arena.ensure(arena_bytes ? arena_bytes : kArenaDefault, true) ||
      hipHostGetDevicePointer(&dev, S->arena.p, 0) != hipSuccess) {
    S->arena.release();
    wc_ctx_destroy(S->ctx);
    return WC_E_HIP;
  }
  S->arena_dev = (const uint8_t*)dev;
  S->th = std::thread(service_loop, S.get());
  *out = S.release();
  return WC_OK;
}

void wc_service_destroy(wc_service* S) {
  if (!S) return;
  {
    std::lock_guard<std::mutex> g(S->mu);
    S->stop = true;
  }
  S->cv_svc.notify_all();
  S->cv_arena.notify_all();
  {
    // calls already inside finish first (the service thread serves them);
    // new ones are refused
    std::unique_lock<std::mutex> lk(S->mu);
    S->cv_idle.wait(lk, [&] { return S->inflight == 0; });
  }
  S->cv_svc.notify_all();
  S->th.join();
  (void)hipSetDevice(S->device);
  S->arena.release();
  wc_ctx_destroy(S->ctx);
  delete S;
}

int wc_service_consensus(wc_service* s, const wc_config* cfg, const wc_problem* problem, wc_results** out) {
  return service_call(s, 1, cfg, problem, out);
}

int wc_service_dual_consensus(wc_service* s, const wc_config* cfg, const wc_problem* problem, wc_results** out) {
  return service_call(s, 2, cfg, problem, out);
}

int wc_service_priority_consensus(wc_service* s, const wc_config* cfg, const wc_chain_problem* problem,
                                  wc_results** out) {
  return service_priority(s, cfg, problem, out);
}

uint32_t wc_service_engines_used(wc_service* s, int reset) { return s ? wc_engines_used(s->ctx, reset) : 0; }

int wc_service_get_stats(wc_service* s, wc_service_stats* out) {
  if (!s || !out) return WC_E_BAD_INPUT;
  std::lock_guard<std::mutex> g(s->mu);
  *out = s->stats;
  return WC_OK;
}

const char* wc_service_last_error(wc_service* s) { return s ? s->err.c_str() : "no service"; }

}  // extern "C"
