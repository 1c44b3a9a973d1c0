// Engine launches and their capacity planning (engine_host.cpp), shared by
// the batch runner, the PriorityConsensusDWFA stream scheduler and the
// per-device submission service (service.cpp). Internal.
#pragma once
#include <string>
#include <vector>

#include "host_internal.hpp"

namespace wch {
using namespace wc;

// Bounds-checked builds (WC_CHECK): every workgroup's HBM regions (workspace,
// global search state) are followed by a guard zone filled with kGuardByte
// before the launch and verified after it (check_guards)
#ifdef WC_CHECK
inline constexpr uint64_t kGuard = 4096;
inline constexpr uint8_t kGuardByte = 0xA5;
#else
inline constexpr uint64_t kGuard = 0;
#endif

inline constexpr uint32_t kMaxAttempts = 8;  // capacity retries of one problem

struct Caps {
  uint32_t sides = 1, pcap = 16, wcap = 64, lcap = 64, nmax = 1, chain = 0, rmax = 1, act_m = 0;
  size_t lds = 0;   // dynamic LDS per workgroup (0 in the global-state build)
  int per_cu = 1;
  uint64_t wsb = 0, ob = 0;
  bool gstate = false;  // search state in HBM (engine_gstate.hip): it does not fit LDS
  bool narrow = false;  // 128-thread build (engine_narrow.hip)
  bool lowlat = false;  // 256-thread build at 2 waves/SIMD (engine_lowlat.hip)
  bool cu = false;      // 1024-thread single engine, one workgroup per CU (engine_cu.hip)
  bool wave = false;    // the dual engine on one wave per problem (engine_wave.hip)
  bool coop = false;    // the same search on cooperating waves, one read per lane (engine_coop.hip)
  uint32_t waves = wc::kWaves;  // waves per workgroup the per-wave layouts are sized for
  bool dual_hot = false;  // dual engine: the popped node's RStates in LDS (EngineArgs::dual_hot)
  uint64_t gsb = 0;     // its bytes per workgroup
  uint32_t conc = 0;    // workgroups the HBM share was planned for
  bool pool_short = false;  // a retried item's node pool did not get its full growth
};

// One engine launch and everything it owns.
struct Launch {
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  DevBuf probs, sroff, srlen, ract, ws, counter, act, phases, gst, trace;
  HostBuf host;  // mapped: done[P] | status[P] | stats[P][S_NSTAT] | out[P]
  HostBuf ring;  // mapped (stream launches): StreamCtl | problem ring | read-table rings
  Caps caps;
  uint32_t P = 0, grid = 0;
  uint64_t off_status = 0, off_stats = 0, off_out = 0;
  uint64_t off_exit = 0;  // stream launches: exited[grid] (between stats and out)
  std::vector<uint32_t> ids;  // launch problem k -> caller item id
  std::vector<uint8_t> taken;
  uint32_t n_taken = 0;
  bool busy = false;
  bool traced = false;  // this launch writes a pop trace (WC_POP_TRACE)
  double kernel_ms = 0;
  uint64_t reads_bytes = 0;  // WC_FAULT_LOG: bytes of the read arena the launch reads
  uint64_t ws_stride = 0;  // WC_CHECK: workspace bytes per workgroup (guard zone at the end)
  std::vector<DevProblem> dp;
  std::vector<uint64_t> h_sroff;
  std::vector<uint32_t> h_srlen;
  std::vector<int64_t> h_ract;

  volatile uint32_t* done() const { return (volatile uint32_t*)host.p; }
  const uint32_t* status() const { return (const uint32_t*)((const uint8_t*)host.p + off_status); }
  const uint64_t* stats() const { return (const uint64_t*)((const uint8_t*)host.p + off_stats); }
  const uint8_t* out(uint32_t k) const { return (const uint8_t*)host.p + off_out + (uint64_t)k * caps.ob; }
  // stream launches: the host-buffer layout (P output slots, grid exit flags)
  void stream_layout() {
    off_status = align16((uint64_t)P * 4);
    off_stats = off_status + align16((uint64_t)P * 4);
    off_exit = off_stats + align16((uint64_t)P * S_NSTAT * 8);
    off_out = off_exit + align16((uint64_t)grid * 4);
  }
  // stream launches: every workgroup has left its claim loop. Read from the
  // host-mapped flags, never through a HIP call: a stream query can wait on a
  // runtime lock that another thread holds while its own work queues behind
  // this (persistent) launch
  bool all_exited() const {
    const uint32_t* e = (const uint32_t*)((const uint8_t*)host.p + off_exit);
    for (uint32_t k = 0; k < grid; ++k)
      if (!__atomic_load_n(&e[k], __ATOMIC_ACQUIRE)) return false;
    return true;
  }
  uint32_t n_exited() const {
    const uint32_t* e = (const uint32_t*)((const uint8_t*)host.p + off_exit);
    uint32_t n = 0;
    for (uint32_t k = 0; k < grid; ++k) n += __atomic_load_n(&e[k], __ATOMIC_ACQUIRE) != 0;
    return n;
  }
  ~Launch() {
    for (DevBuf* b : {&probs, &sroff, &srlen, &ract, &ws, &counter, &act, &phases, &gst, &trace}) b->release();
    host.release();
    ring.release();
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

// HBM the node pools of one launch may take (engine_host.cpp)
uint64_t hbm_share(const wc_ctx* ctx, uint64_t cached, double frac);
// Capacities of one launch over items[ids]; see engine_host.cpp
int plan_caps(wc_ctx* ctx, const wc_config& cfg, uint32_t sides, const std::vector<SubProb>& items,
              const std::vector<uint32_t>& ids, uint64_t hbm_budget, Caps& c, std::string& err,
              uint32_t max_per_cu = 4, bool cu_ok = false);
// launches the engine of `caps` (LDS or global-state build) on L's stream
int launch_kernel(wc_ctx* ctx, Launch& L, wc::EngineArgs& a, const Caps& caps);
// launch slot k of the context (created on first use)
Launch* launch_slot(wc_ctx* ctx, size_t k);
// the outcome of launch output slot k (its completion flag is set): raw device
// status (ST_RETRY flags included); `o` gets records and counters
uint32_t harvest(const Launch& L, uint32_t k, const SubProb& s, EngineOut& o);
// capacity growth for a retried item
void bump(SubProb& s, uint32_t st);
// waits for the launch, records its kernel time (and, WC_CHECK, verifies guards)
int launch_finish(wc_ctx* ctx, Launch& L);
// frees the device and pinned buffers a (finished) launch keeps cached
inline void launch_release_buffers(Launch& L) {
  for (DevBuf* b : {&L.probs, &L.sroff, &L.srlen, &L.ract, &L.ws, &L.counter, &L.act, &L.phases, &L.gst, &L.trace}) b->release();
  L.host.release();
  L.ring.release();
}

}  // namespace wch
