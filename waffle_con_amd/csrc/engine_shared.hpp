// Structures shared by the host orchestration (host.cpp) and the device
// engines (engine.hip). Plain data only.
#pragma once
#include <stdint.h>
#include <stdlib.h>

namespace wc {

constexpr int kBlock = 256;       // threads per engine workgroup (4 waves)
constexpr int kWaves = kBlock / 64;
// the widest single-engine build (engine_cu.hip: 1024 threads for launches of
// at most one problem per CU); problems still have at most kBlock reads
constexpr int kMaxWaves = 16;
constexpr int kKmax = 8;          // distinct symbols at one read's tips
constexpr int kKout = 14;         // distinct symbols voted across a node side (16-bucket table)
constexpr uint32_t kInactive = 0xFFFFFFFFu;  // Option<DWFALite>::None

// per-problem status (device → host)
enum : uint32_t {
  ST_OK = 0,
  // 1..12 = WC_E_* error codes (include/waffle_con.h)
  ST_RETRY = 0x100,          // capacity retry flags below (OR-ed)
  ST_RETRY_WCAP = 0x1,       // a wavefront outgrew wcap
  ST_RETRY_PCAP = 0x2,       // node pool exhausted
  ST_RETRY_LCAP = 0x4,       // consensus outgrew lcap
  ST_RETRY_HEAP = 0x8,       // priority queue outgrew pcap
  ST_RETRY_RMAX = 0x10,      // more tied results than result records
  // WC_E_LIMIT from the engines carries what overflowed in bits 16+:
  LIM_TIPS = 0x1,       // more than 8 distinct symbols at one read's wavefront tips
  LIM_OFFSET = 0x2,     // offset activation scratch
  LIM_VOTES = 0x8,      // more than 14 voted symbols at one node side
  LIM_CHILDREN = 0x20,  // more than 64 children of one node
};

enum StatIdx : int {
  S_UPDATES = 0,
  S_WOUT,
  S_COMPARES,
  S_EDINC,
  S_FINALIZES,
  S_POPS,
  S_EXPLORED,
  S_IGNORED,
  S_PEAKQ,
  S_ROWB,  // wavefront-row bytes of updates/finalizes that grow e (roofline model)
  S_NSTAT
};

struct DevConfig {
  uint64_t max_queue_size;
  uint64_t max_capacity_per_size;
  uint64_t max_return_size;
  uint64_t max_nodes_wo_constraint;
  uint64_t min_count;
  uint64_t dual_max_ed_delta;
  uint64_t offset_window;
  uint64_t offset_compare_length;
  double min_af;
  int32_t cost_mode;
  int32_t wildcard;
  uint32_t weighted;
  uint32_t early;
};

struct DevProblem {
  uint32_t read_begin;  // first read index in the batch read tables
  uint32_t n_reads;
  uint32_t max_read_len;
  uint32_t n_active;    // reads with offset None (after auto-shift)
  uint32_t max_act;     // largest activation length (add_sequence_offset), 0 = none
  uint32_t _pad[3];
};
static_assert(sizeof(DevProblem) == 32, "DevProblem layout");

// Device result record (one per returned consensus); the host turns these into
// Consensus / DualConsensus values. Layout inside the per-problem output area:
//   u32 n_results, u32 pad, then R records of
//   [u32 len1, u32 len2, u32 is_dual, u32 pad][con1: lcap][con2: lcap (dual)]
//   [fe1: nmax u32][fe2: nmax u32 (dual)]  — finalized edit distances, kInactive = None
struct EngineArgs {
  DevConfig cfg;
  const DevProblem* problems;
  uint32_t n_problems;
  uint32_t sides;        // 1 = ConsensusDWFA, 2 = DualConsensusDWFA
  const uint8_t* rbytes;
  const uint64_t* roff;
  const uint32_t* rlen;
  const int64_t* ractivate;  // per read activation length (-1 = active at root)
  uint8_t* ws;           // per-workgroup workspace
  uint64_t ws_stride;
  uint32_t pcap;         // node slots per workgroup (also heap capacity)
  uint32_t wcap;         // wavefront entries per read per slot
  uint32_t lcap;         // consensus capacity per side
  uint32_t nmax;         // max reads per problem in this batch
  uint32_t rmax;         // result records per problem
  uint32_t chain;        // max linear-chain run-ahead steps (0 = off); sizes the LDS chain area
  uint32_t chain_kinds;  // dual engine: bit 0 chains over single-consensus nodes, bit 1 over dual nodes
  uint32_t dual_hot;     // dual engine (chain == 0): the popped node's RStates live in LDS (hot_sides)
  uint8_t* out;
  uint64_t out_stride;
  uint32_t* status;      // per problem
  uint64_t* stats;       // per problem x S_NSTAT
  uint32_t* done;        // per problem completion flag (host-mapped; set after status, stats, out)
  uint32_t* work_counter;
  uint32_t* trace;       // debug: per-pop records of problem 0 (nullptr = off)
  uint32_t trace_cap;    // records (4 u32 each); trace[0] = count
  uint32_t act_m;        // offset activation: pair entries per lane per array (0 = no scratch)
  uint64_t* act_scr;     // offset activation scratch: per workgroup act_stride u64
  uint64_t act_stride;
  unsigned long long* phases;  // debug (WC_PHASE_PROF builds): shader cycles per phase, kPhases
  // stream mode (1): one persistent launch fed by the host (engine_host.cpp
  // priority_stream). `problems` and roff/rlen/ractivate are host-mapped
  // rings (qcap problems, qslots read entries) published up to sctl->tail;
  // workgroups claim sequence numbers from *qhead, copy the claimed problem's
  // read table into their workspace, and write results to one of their two
  // output slots (blockIdx * 2 + b), flagged done[slot] = seq + 1.
  uint32_t stream;
  uint32_t qcap, qslots;
  struct StreamCtl* sctl;
  uint32_t* qhead;
  uint64_t idle_ticks;   // wall-clock ticks without a host heartbeat before a waiting workgroup gives up
  uint32_t* exited;      // stream mode: per-workgroup exit flags (host-mapped), set as a workgroup leaves
  // stream mode with host-resident reads (service lanes): the claimed
  // problem's reads are copied from `hreads` (host-mapped; roff/rlen index
  // it) into the workgroup's staging area (rstage_stride bytes per read,
  // after its read table), and read from there; rbytes is then the
  // workspace base the staged offsets are relative to
  const uint8_t* hreads;
  uint64_t rstage_stride;
  // global-state build (engine_gstate.hip): per-workgroup HBM region holding
  // what lds_bytes() describes
  uint8_t* gstate;
  uint64_t gstate_stride;
};
// host-mapped control words of a stream launch (16-byte aligned)
struct alignas(16) StreamCtl {  // tail and stop form one 8-byte word (read together by the device)
  uint32_t tail;   // problems published (host)
  uint32_t stop;   // host: nothing more will be published (set after the final tail)
  uint32_t abort;  // device: a workgroup gave up waiting (no heartbeat for idle_ticks)
  uint32_t heartbeat;  // host: bumped on every pass of its event loop (liveness)
};
// per-workgroup copy of the claimed problem's read table (stream mode): roff | ract | rlen
__host__ __device__ inline uint64_t rtab_bytes(uint32_t nmax) {
  return ((uint64_t)nmax * 8 + 15) / 16 * 16 * 2 + ((uint64_t)nmax * 4 + 15) / 16 * 16;
}
// staging stride of one read pulled from host memory (EngineArgs::hreads): its
// bytes rounded up to 16, then 64 zero bytes (the engine's over-read margin)
__host__ __device__ inline uint64_t rstage_stride(uint32_t maxlen) { return ((uint64_t)maxlen + 15) / 16 * 16 + 64; }
constexpr int kPhases = 56;  // 32..39: chain statistics of the dual engine (engine.hip, dual chain call site); 40..: single-engine chain counters
// offset-activation scratch per workgroup (u64): per wave two lane-interleaved pair arrays of m entries
__host__ __device__ inline uint64_t act_scr_u64(uint32_t m, uint32_t waves = kWaves) { return (uint64_t)waves * 2 * m * 64; }  // 0..15 block phases, 16..31 wave-0 sub-phases

// ---- byte layouts (host and device compute them identically) ----
__host__ __device__ inline uint64_t align16(uint64_t x) { return (x + 15) & ~uint64_t(15); }

// Per-read DWFA state of one node side. The full wavefront (wf row, u32 per
// diagonal) stays authoritative in HBM; RState caches what a push needs:
// the frontier F = diagonals with d + off >= |consensus| (the only ones that
// can move when a symbol is appended), plus summaries of the stuck rest.
constexpr int kF = 8;
constexpr uint8_t kWide = 1;  // frontier larger than kF: use the full-scan path
struct RState {
  uint32_t e;       // edit distance, kInactive = None
  uint32_t off;     // DWFALite offset (activation)
  uint32_t maxb;    // max baseline offset d+e-i over stuck diagonals
  uint16_t nscmp;   // stuck diagonals with baseline offset < |read| (each push compares them once)
  uint8_t nf;       // frontier size
  uint8_t flags;    // kWide
  uint16_t fi[kF];  // frontier diagonal indices, ascending
  uint32_t fd[kF];  // frontier d values
};
static_assert(sizeof(RState) == 64, "RState must stay 64 bytes");

// one node slot: per side: RState[nmax], wf[nmax*wcap] u32, con[lcap]
__host__ __device__ inline uint64_t side_bytes(uint32_t nmax, uint32_t wcap, uint32_t lcap) {
  return align16((uint64_t)nmax * sizeof(RState) + (uint64_t)nmax * wcap * 4) + align16(lcap);
}
__host__ __device__ inline uint64_t slot_bytes(uint32_t sides, uint32_t nmax, uint32_t wcap, uint32_t lcap) {
  return sides * side_bytes(nmax, wcap, lcap);
}
// workspace: slots | trackers (2 x 2 arrays of lcap+2 u32) | active arrays (2 x lcap+2 u32) | finalize scratch
__host__ __device__ inline uint64_t ws_bytes(uint32_t sides, uint32_t pcap, uint32_t nmax, uint32_t wcap,
                                             uint32_t lcap) {
  uint64_t t = (uint64_t)pcap * slot_bytes(sides, nmax, wcap, lcap);
  t += align16((uint64_t)4 * (lcap + 2) * 4);
  t += align16((uint64_t)2 * (lcap + 2) * 4);
  t += align16((uint64_t)kMaxWaves * (wcap + 2) * 4);  // per wave of the widest build
  return align16(t);
}
__host__ __device__ inline uint64_t result_bytes(uint32_t sides, uint32_t nmax, uint32_t lcap) {
  return 16 + sides * align16(lcap) + sides * align16((uint64_t)nmax * 4);
}
__host__ __device__ inline uint64_t out_bytes(uint32_t sides, uint32_t rmax, uint32_t nmax, uint32_t lcap) {
  return align16(16 + (uint64_t)rmax * result_bytes(sides, nmax, lcap));
}

// LDS carve (dynamic shared memory)
struct HeapEntry {
  uint64_t cost;
  uint32_t len;
  uint32_t slot;
};
struct SlotMeta {
  uint32_t len[2];
  uint32_t nsome[2];
  uint32_t flags;  // bit0 dual, bit1 lock1, bit2 lock2
  uint32_t pad[3];
};
struct RInfo {
  uint8_t n;      // distinct tip symbols (iteration order below)
  uint8_t end;    // reached_baseline_end
  uint16_t split; // sum of occurrences
  uint8_t sym[kKmax];
  uint16_t occ[kKmax];
  uint32_t e;     // current edit distance (kInactive = None)
};
// ---- linear-chain run-ahead (single engine, engine.hip run_chain) ----
constexpr uint32_t kChainMax = 40;      // steps per chain (upper bound; WC_CHAIN); longer chains outrun the 64-B read windows
constexpr uint32_t kChainDefault = 16;  // steps per chain by default
// dual engine: chains off by default (WC_DUAL_CHAIN=<k> enables them, up to k
// steps): its searches' chains are short (cfg5 median 4 pops), and the
// speculation costs more than it saves on cfg3/cfg4/cfg5
constexpr uint32_t kDualChainDefault = 0;
constexpr uint32_t kChainOvf = 192;  // multi-symbol nominations stored per chain
static_assert(kChainOvf <= 256, "ChainOvf index is the low byte of a u16 nomination code");
struct ChainStep {  // aggregates of one speculative step (node N_j), LDS atomics (one per wave)
  uint64_t cost;    // sum of the reads' costs
  uint64_t po;      // votes in 1/840ths: for the predicted next symbol [0,32), for other symbols [32,64)
  uint64_t ef;      // reads at their end [0,16) | multi-symbol reads [16,32) | fractional pred votes [32,48)
  uint32_t ok, pad;
};
static_assert(sizeof(ChainStep) == 32, "ChainStep layout");
__host__ __device__ inline uint32_t step_nend(uint64_t ef) { return (uint32_t)(ef & 0xFFFFu); }
__host__ __device__ inline uint32_t step_nmulti(uint64_t ef) { return (uint32_t)((ef >> 16) & 0xFFFFu); }
__host__ __device__ inline uint32_t step_nfrac(uint64_t ef) { return (uint32_t)((ef >> 32) & 0xFFFFu); }
struct ChainOvf {  // nominations of a read with >= 2 distinct tip symbols
  uint64_t sym;  // bytes in iteration order
  uint32_t occ;  // nibble k: occurrences of symbol k (<= kF = 8 tips)
  uint32_t sn;   // split | n << 8
  __host__ __device__ void set(uint64_t s, uint64_t occ_bytes, uint32_t split, uint32_t n) {
    sym = s;
    uint32_t o = 0;
    for (uint32_t k = 0; k < 8; ++k) o |= (uint32_t)((occ_bytes >> (8 * k)) & 15u) << (4 * k);
    occ = o;
    sn = split | n << 8;
  }
  __host__ __device__ uint32_t occ_at(uint32_t k) const { return (occ >> (4 * k)) & 15u; }
  __host__ __device__ uint32_t split() const { return sn & 0xFFu; }
  __host__ __device__ uint32_t n() const { return sn >> 8; }
};
static_assert(sizeof(ChainOvf) == 16, "ChainOvf layout");
// Read windows of the chain walk: 64 bytes of each read in LDS. The walk reads
// them per step, one read per lane (read r = 4 * lane + wave), so they are laid
// out for the LDS banks: read r's window is slot (r & 3) * m4 + (r >> 2)
// (m4 = ceil(nmax / 4)) of kWinStride bytes (17 dwords, odd), which puts the 32
// lanes of a wave's half on 32 different banks when they read the same offset.
constexpr uint32_t kWinStride = 68;
__host__ __device__ inline uint32_t win_m4(uint32_t nmax) { return (nmax + 3) / 4; }
__host__ __device__ inline uint32_t win_slot(uint32_t r, uint32_t m4) { return (r & 3u) * m4 + (r >> 2); }
// window slots one side's carve holds for a build of `waves` waves (the single
// engine deals read r to wave r % waves: waves * ceil(n / waves) slots)
__host__ __device__ inline uint32_t win_slots(uint32_t nmax, uint32_t waves) {
  const uint32_t m = waves * ((nmax + waves - 1) / waves);
  return m > 4 * win_m4(nmax) ? m : 4 * win_m4(nmax);
}
// the chain area's per-wave parts are carved for at least kWaves waves
__host__ __device__ constexpr uint32_t chain_waves(uint32_t waves) { return waves > (uint32_t)kWaves ? waves : (uint32_t)kWaves; }
// aggregates of one speculative step of the dual-node chain (dual_chain.hip.hpp)
struct DualStep {
  uint64_t cost;   // sum over reads of the cheaper side's cost
  uint64_t po[2];  // per side: ChainStep::po
  uint64_t ef[2];  // per side: ChainStep::ef
  uint32_t some;   // Some(dwfa) side 1 [0,10) | side 2 [10,20) | reads at the end of either side [20,30)
  uint32_t ok;
};
static_assert(sizeof(DualStep) == 48, "DualStep layout");
__host__ __device__ inline uint32_t chain_sides(uint32_t sides) { return sides == 2 ? 2u : 1u; }
// dual engine chain kinds (EngineArgs::chain_kinds; WC_DUAL_CHAIN_KINDS overrides, default both)
inline uint32_t env_chain_kinds() {
  const char* e = getenv("WC_DUAL_CHAIN_KINDS");
  return e ? (uint32_t)atoi(e) & 3u : 3u;
}
// chain LDS (per side S = chain_sides: the dual engine's chains walk both):
//   steps[K+1] | ovf[kChainOvf] | tmp RState[kWaves][4] | nom[S][K+1][nmax] u16 |
//   win[S][4*m4][68 B] (read windows) | wb[S][nmax] u32 | pc[K+1] u32 | pred[S][K+2] u8 | perm[nmax] u8 | m0[nmax] u8
__host__ __device__ inline uint64_t chain_lds_bytes(uint32_t nmax, uint32_t K, uint32_t sides = 1,
                                                    uint32_t waves = kWaves) {
  if (K == 0) return 0;
  const uint64_t S = chain_sides(sides);
  waves = chain_waves(waves);
  uint64_t t = align16((uint64_t)(K + 1) * (S == 2 ? sizeof(DualStep) : sizeof(ChainStep)));
  t += align16((uint64_t)kChainOvf * sizeof(ChainOvf));
  t += (uint64_t)waves * 4 * 64;  // per wave, one RState per 16-lane group
  t += align16(S * (K + 1) * nmax * 2);
  t += align16(S * win_slots(nmax, waves) * kWinStride);
  t += align16(S * nmax * 4);
  t += align16((uint64_t)(K + 1) * 4);
  t += align16(S * (K + 2));
  t += align16(nmax);  // the walk's read order
  t += align16(nmax);  // each read's first quiet run
  return t;
}

// the dual engine builds up to this many children of a node in one pass (engine.hip kNCB)
constexpr uint32_t kDualChildBatch = 4;
// work list entries (u32): heavy (side, read) items; the dual engine builds up
// to 4 children at once (engine.hip kNCB), so 2 sides x 4 children x nmax
__host__ __device__ inline uint64_t list_entries(uint32_t sides, uint32_t nmax) {
  return (uint64_t)(sides == 2 ? 8 : 2) * nmax;
}
// sides whose expanded node's RStates are held in LDS: the single engine's
// popped node; in the dual engine side 1 of a single-consensus node for its
// chain walk (chain > 0; the two-sided walk reads the slot), or, with
// `dual_hot` (EngineArgs::dual_hot, no chains), both sides of the popped node
// (its in-place child is pushed there and usually popped next)
__host__ __device__ inline uint32_t hot_sides(uint32_t sides, uint32_t chain, uint32_t dual_hot = 0) {
  if (sides == 1 || chain > 0) return 1u;
  return dual_hot ? 2u : 0u;
}
// LDS: hot RStates[hot_sides][nmax] | chain area | heap | freestack | meta | rinfo[sides][nmax] | fe[sides][nmax] |
//      heavy list[list_entries] u32 | (dual) child e[kDualChildBatch][2][nmax] u16 | read table [nmax] u32x2
__host__ __device__ inline uint64_t lds_bytes(uint32_t sides, uint32_t pcap, uint32_t nmax, uint32_t chain,
                                              uint32_t dual_hot = 0, uint32_t waves = kWaves) {
  uint64_t t = (uint64_t)hot_sides(sides, chain, dual_hot) * nmax * sizeof(RState);
  t += chain_lds_bytes(nmax, chain, sides, waves);
  t += (uint64_t)pcap * sizeof(HeapEntry);
  t += align16((uint64_t)pcap * 4);
  t += (uint64_t)pcap * sizeof(SlotMeta);
  t += (uint64_t)sides * nmax * sizeof(RInfo);
  t += align16((uint64_t)sides * nmax * 4);
  t += align16((uint64_t)list_entries(sides, nmax) * 4);
  // dual engine: the children's edit distances per (child, side, read) of one build pass (prune + cost), u16
  if (sides == 2) t += align16((uint64_t)kDualChildBatch * 2 * nmax * 2);
  // the single engine's read table of the claimed problem (offset / 16, length) per read
  if (sides == 1) t += align16((uint64_t)nmax * 8);
  return align16(t);
}

}  // namespace wc

namespace wc {
// one standalone DWFALite job (wc_dwfa_batch); device pointers
struct DwfaDevJob {
  const uint8_t* baseline;
  const uint8_t* other;
  uint32_t* wf;
  uint32_t blen, olen, offset, wf_cap;
  int32_t wildcard;
  uint32_t early, op, e;
  uint32_t status, n_cand;
  uint8_t cand_syms[16];
  uint32_t cand_counts[16];
  uint8_t cand_first[16];  // the same symbols in insertion (first-appearance) order
};
// one standalone wfa_ed_config pair (wc_wfa_ed_batch); offsets into the
// batch's sequence arena and scratch rows (two rows of `cap` u64 entries)
struct EdDevJob {
  uint64_t v1_off, v2_off, scr_off;
  uint32_t l1, l2;
  uint64_t cap;
};
}  // namespace wc
