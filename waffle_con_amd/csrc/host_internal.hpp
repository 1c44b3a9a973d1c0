// Host-side types shared by the C ABI (host.cpp) and the engine scheduler
// (engine_host.cpp). Not part of the public interface.
#pragma once
#include <atomic>
#include <hip/hip_runtime.h>

#include <array>
#include <cstdint>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../../include/waffle_con.h"
#include "engine_shared.hpp"

namespace wc {
void launch_unpack2(const uint32_t* packed, const uint64_t* roff, const uint32_t* rlen, uint32_t nreads, uint32_t lut,
                    uint8_t* out, uint64_t pos, hipStream_t s);
void launch_single_engine(const EngineArgs& a, uint32_t grid, size_t lds, hipStream_t s);
void launch_dual_engine(const EngineArgs& a, uint32_t grid, size_t lds, hipStream_t s);
int engine_blocks_per_cu(uint32_t sides, size_t lds, bool dual_hot = false);
void launch_dwfa_jobs(DwfaDevJob* jobs, uint32_t n, hipStream_t s);
void launch_wfa_ed_batch(const EdDevJob* jobs, uint32_t n, const uint8_t* seqs, uint64_t* scratch, int wc,
                         uint32_t both, uint64_t* out, hipStream_t s);
}  // namespace wc
namespace wcg {  // engine_gstate.hip: search state in HBM
void launch_single_engine(const wc::EngineArgs& a, uint32_t grid, size_t lds, hipStream_t s);
void launch_dual_engine(const wc::EngineArgs& a, uint32_t grid, size_t lds, hipStream_t s);
int engine_blocks_per_cu(uint32_t sides, size_t lds, bool dual_hot = false);
}  // namespace wcg
namespace wcn {  // engine_narrow.hip: 128-thread workgroups (problems of <= 128 reads)
void launch_single_engine(const wc::EngineArgs& a, uint32_t grid, size_t lds, hipStream_t s);
void launch_dual_engine(const wc::EngineArgs& a, uint32_t grid, size_t lds, hipStream_t s);
int engine_blocks_per_cu(uint32_t sides, size_t lds, bool dual_hot = false);
}  // namespace wcn
namespace wcl {  // engine_lowlat.hip: 256-thread workgroups at 2 waves/SIMD (launches with few problems)
void launch_single_engine(const wc::EngineArgs& a, uint32_t grid, size_t lds, hipStream_t s);
void launch_dual_engine(const wc::EngineArgs& a, uint32_t grid, size_t lds, hipStream_t s);
int engine_blocks_per_cu(uint32_t sides, size_t lds, bool dual_hot = false);
}  // namespace wcl
namespace wcu {  // engine_cu.hip: the 1024-thread single engine (launches of <= one problem per CU)
void launch_single_engine(const wc::EngineArgs& a, uint32_t grid, size_t lds, hipStream_t s);
int engine_blocks_per_cu(uint32_t sides, size_t lds, bool dual_hot = false);
int engine_waves();
}  // namespace wcu
namespace wcc {  // engine_coop.hip: the one-wave dual engine on cooperating waves (65-256 reads, few problems)
void launch_dual_engine(const wc::EngineArgs& a, uint32_t grid, size_t lds, hipStream_t s);
int coop_blocks_per_cu(size_t lds);
int engine_waves();
}  // namespace wcc
namespace wcc2 {  // engine_coop2.hip: the same on 2 waves (65-128 reads)
void launch_dual_engine(const wc::EngineArgs& a, uint32_t grid, size_t lds, hipStream_t s);
int coop_blocks_per_cu(size_t lds);
int engine_waves();
}  // namespace wcc2
namespace wcw {  // engine_wave.hip: the dual engine on one wave per problem (no offsets, <= 128 reads)
void launch_dual_engine(const wc::EngineArgs& a, uint32_t grid, size_t lds, hipStream_t s);
int wave_blocks_per_cu(uint32_t nmax, size_t lds);
}  // namespace wcw
namespace wcd {  // engine_dchain.hip: the dual engine with chains (launches with caps.chain > 0)
void launch_single_engine(const wc::EngineArgs& a, uint32_t grid, size_t lds, hipStream_t s);
void launch_dual_engine(const wc::EngineArgs& a, uint32_t grid, size_t lds, hipStream_t s);
int engine_blocks_per_cu(uint32_t sides, size_t lds, bool dual_hot = false);
}  // namespace wcd

// Persistent (stream-mode) launches of this process and deferred frees.
// hipFree / hipHostFree wait for every kernel on the device, a persistent
// launch included, and that one only ends when its host thread says so. If
// that thread is meanwhile blocked on the runtime inside another HIP call,
// neither moves (its workgroups give up after 30 s without a heartbeat:
// "stream launch ended with problems outstanding (abort=1)", seen with 16
// threads each running wc_priority_consensus_batch on its own context). So
// while any persistent launch of the process runs, buffers are not freed but
// parked, and released by the thread that ends the last persistent launch.
void persistent_begin();
void persistent_end();
bool free_deferred(void* p, bool host);  // parks (a persistent launch runs) or frees now, under the lock; always true

// device buffer, grown on demand (never shrinks)
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
    if (p && !free_deferred(p, false)) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// pinned host buffer. `mapped`: fine-grained, coherent and device-visible (the
// engine writes results and completion flags straight into it)
struct HostBuf {
  void* p = nullptr;
  size_t cap = 0;
  bool ensure(size_t bytes, bool mapped = false) {
    if (bytes <= cap) return true;
    release();
    size_t want = std::max<size_t>(bytes + bytes / 8, 1 << 20);
    const unsigned flags = mapped ? (hipHostMallocMapped | hipHostMallocCoherent) : hipHostMallocDefault;
    if (hipHostMalloc(&p, want, flags) != hipSuccess) {
      p = nullptr;
      return false;
    }
    cap = want;
    return true;
  }
  void release() {
    if (p && !free_deferred(p, true)) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

namespace wch {
struct Launch;
}

struct wc_ctx {
  int device = 0;
  int n_cu = 256;  // CUs this context plans its launches for: the device's / share
  int share = 1;   // WC_DEVICE_SHARE: processes sharing the device (each plans for 1/share of CUs and HBM)
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::string err;
  DevBuf jobs;
  HostBuf upstage;  // pinned staging of batch uploads (reused across batches)
  DevBuf upk;       // 2-bit packed batch uploads before the device expands them (host.cpp pack_reads)
  uint64_t last_upload_packed = 0;  // bytes the last batch upload sent packed (0 = byte path)
  std::atomic<uint32_t> engines_used{0};  // wc_engines_used: bit per engine build launched (engine_host.cpp)
  // engine launch slots (engine_host.cpp): each has its own stream and buffers
  std::vector<wch::Launch*> launches;
};

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
  std::vector<uint64_t> roff_h;
  DevBuf reads, roff, rlen;
  uint64_t bytes = 0;
  bool valid = false;  // every read is on the device (upload_batch completed)
  ~wc_batch() {
    reads.release();
    roff.release();
    rlen.release();
  }
};

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
  uint64_t stats[wc::S_NSTAT] = {0};
  double done_ms = 0;  // from the start of the call until this problem's result was final
  double start_ms = 0;  // from the start of the call until its first engine work was published (priority stream)
};
struct wc_results {
  int kind = 0;  // 0 single, 1 dual, 2 priority
  std::vector<ProbRes> probs;
  wc_stats stats;
  // single-consensus results in two arenas (wc_results_single_view): the
  // batch path fills them as problems finish (while the kernel runs), in
  // finishing order; the per-result index below is in problem order
  std::vector<uint8_t> a_seq;
  std::vector<uint64_t> a_sc;
  std::vector<uint64_t> p_seq0, p_sc0;  // per problem: arena start of its first result (~0 = not packed)
  std::vector<int32_t> v_status;
  std::vector<uint32_t> v_count;
  std::vector<uint64_t> v_idx;  // per result: seq start, seq len, scores start, scores len
  bool view_ready = false;
};


struct RawRecord {
  uint32_t len[2] = {0, 0};
  bool dual = false;
  std::vector<uint8_t> con[2];
  std::vector<uint32_t> fe[2];
};

namespace wch {
std::string err_msg(int code);
std::string limit_msg(uint32_t why);
std::string retry_msg(uint32_t st, uint32_t attempts);
int set_err(wc_ctx* ctx, int code, const std::string& msg);
wc::DevConfig to_dev(const wc_config& c);
inline uint64_t cost_of_h(uint32_t e, int mode) { return mode == 0 ? (uint64_t)e : (uint64_t)e * (uint64_t)e; }
int upload_batch(wc_ctx* ctx, uint32_t n, const wc_problem* problems, wc_batch* b);
extern const char* const kEngineNames[];
extern const uint32_t kNumEngineNames;

// One engine problem as the host schedules it: global read ids into a batch
// arena and each read's activation length (-1 = active at the root).
struct SubProb {
  std::vector<uint32_t> gid;
  std::vector<int64_t> act;
  uint32_t n_active = 0, max_act = 0, max_len = 0;
  uint64_t work = 0;
  bool cont = false;  // PriorityConsensusDWFA: a later sub-problem of an already started problem
  // capacity growth earned by ST_RETRY outcomes (log2 multipliers)
  uint8_t wcap_x = 0, pcap_x = 0, lcap_x = 0, rmax_x = 0;
  uint32_t attempts = 0;
  // PriorityConsensusDWFA: pops its problem's finished sub-problems took before
  // this one was made (the stream publishes the continuations of the loci that
  // have run longest first: a deep locus's next sub-problem is on its critical path)
  uint64_t crit = 0;
  double t_pub = -1;  // steady-clock ms when the stream published it (-1: not yet)
};
// auto_shift_offsets + activation points (consensus.rs:151-202) of one
// problem; fills sp.act / n_active / max_act or returns an error code.
int activation_plan(const wc_config& cfg, const std::vector<int64_t>& offsets, SubProb& sp, std::string& err);

// Outcome of one engine problem.
struct EngineOut {
  int status = WC_OK;
  std::string error;
  std::vector<RawRecord> recs;
  std::array<uint64_t, wc::S_NSTAT> stats{};
};

// Runs `items` (all reads in batch `b`) to completion on the device, with
// capacity retries; out[i] is item i's outcome. on_final(i), if given, is
// called once per item as soon as out[i] is final (possibly while the launch
// still runs); items that fail before any launch are not reported to it.
int run_engine(wc_ctx* ctx, wc_batch* b, const wc_config& cfg, uint32_t sides, std::vector<SubProb>& items,
               std::vector<EngineOut>& out, double& kernel_ms, uint64_t& launches,
               const std::function<void(uint32_t)>* on_final = nullptr);

// PriorityConsensusDWFA over many problems, streamed (engine_host.cpp).
int priority_stream(wc_ctx* ctx, const wc_config& cfg, uint32_t n, const wc_chain_problem* problems,
                    wc_results* R);

void destroy_launches(wc_ctx* ctx);
// FxHashSet<Option<usize>> iteration order of seed groups (priority_consensus.rs:180)
std::vector<int64_t> seed_order(const std::vector<int64_t>& groups);
// priority_consensus.rs:309-335: finished chains -> sorted chains + sequence_indices
void priority_assemble(uint32_t n_chains, std::vector<std::vector<ConsRec>>& chains,
                       std::vector<std::vector<uint8_t>>& assigns, ProbRes& pr);
bool dual_from_record(const RawRecord& rr, uint32_t n, int mode, DualRec& d);
void build_single(const EngineOut& E, int mode, ProbRes& pr);
// appends problem p's single results to the arenas (wc_results::a_seq/a_sc)
void pack_single(wc_results* R, uint32_t p);
void build_dual(const EngineOut& E, uint32_t n, int mode, ProbRes& pr);
void fill_stats(wc_results* R, double kernel_ms, uint64_t launches, double wall_ms);
}  // namespace wch

#define HIPCHK(call)                                                                                      \
  do {                                                                                                    \
    hipError_t _e = (call);                                                                               \
    if (_e != hipSuccess)                                                                                 \
      return wch::set_err(ctx, WC_E_HIP, std::string(#call) + ": " + hipGetErrorString(_e));              \
  } while (0)
