// Device-resident consensus engines for MI355X (gfx950).
//
// ConsensusDWFA::consensus (consensus.rs:139-351) and
// DualConsensusDWFA::consensus (dual_consensus.rs:240-787) run entirely on the
// GPU: one workgroup (4 x wave64) per consensus problem pulls problems from a
// global work counter and executes the reference's least-cost-first search
// with the reference's exact pop order (priority-queue 1.x heap, SURVEY
// Appendix A), candidate order (hashbrown/FxHash iteration, Appendix B) and
// f64 vote summation order.
//
// Node state lives in a per-workgroup node pool in HBM: per read a 64-byte
// frontier cache (RState) plus the authoritative wavefront row. A push is one
// thread per read on its RState (O(frontier) work, no full scan); only reads
// whose edit distance must grow (or whose frontier is wide) take the
// wave-cooperative path over the full wavefront. The heap, node metadata,
// per-read nominations and the pushed child's analysis live in LDS, so the
// common linear search step (one child, popped next) never re-reads node state.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "engine_common.hip.hpp"

namespace WC_ENGINE_NS {

// WC_SPLIT builds (A/B experiments): the per-pop block phases are separate
// functions with their own register allocation instead of being inlined
#ifdef WC_SPLIT
#define WC_PHASE_FN __device__ __noinline__
#else
#define WC_PHASE_FN __device__ inline
#endif
// The single engine's push and analysis are separate functions: in the
// kernel body they raise register pressure past the 128-VGPR budget of 4
// workgroups/CU (spills), out of line they don't (cfg2 -3% kernel time; the
// dual engine keeps them inline, where the call overhead costs more)
#ifndef WC_SINGLE_FN
#define WC_SINGLE_FN __device__ __noinline__
#endif

// minimum waves per SIMD the engine kernels are register-allocated for
// (4 = 4 workgroups of 4 waves per CU, 128 VGPRs)
#ifndef WC_WAVES_PER_EU
#define WC_WAVES_PER_EU 4
#endif
// the single engine's register budget (default: WC_WAVES_PER_EU)
#ifndef WC_SINGLE_WAVES_PER_EU
#define WC_SINGLE_WAVES_PER_EU WC_WAVES_PER_EU
#endif
// The dual engine's register budget. Not 3 waves per SIMD (168 VGPRs): that
// budget measured cfg3 +9% in round 2, but both 256-thread dual builds
// compiled for it have faulted on addresses outside every buffer (a pointer
// with a wrong high dword; WC_FAULT_LOG) on inputs the 2- and 4-wave builds of
// the same source and the bounds-checked 3-wave build run bit-exact (DESIGN.md
// "3-wave dual builds")
#if !defined(WC_DUAL_WAVES_PER_EU) && defined(WC_WIDE_DUAL_WPE) && !defined(WC_NARROW) && \
    !defined(WC_GLOBAL_STATE) && !defined(WC_LOWLAT)
#define WC_DUAL_WAVES_PER_EU WC_WIDE_DUAL_WPE  // variant builds (tools/gpu.sh w3)
#endif
#ifndef WC_DUAL_WAVES_PER_EU
#define WC_DUAL_WAVES_PER_EU WC_WAVES_PER_EU
#endif

constexpr int kMaxChild = 64;
constexpr uint32_t kNCB = kDualChildBatch;  // dual engine: children built together (engine_shared list_entries)
// children's edit distances (Lds::ce) as u16; e < wcap / 2, and the prune pass
// reads the slots instead when wcap could exceed 2 * kCeNone
constexpr uint32_t kCeNone = 0xFFFFu;
__device__ __forceinline__ uint16_t ce16(uint32_t e) { return e == kInactive ? (uint16_t)kCeNone : (uint16_t)e; }
__device__ __forceinline__ uint32_t ce32(uint32_t c) { return c == kCeNone ? kInactive : c; }
constexpr uint32_t WC_E_COVERAGE_GAP_CODE = 3;  // include/waffle_con.h
constexpr uint32_t WC_E_INVARIANT_CODE = 10;  // include/waffle_con.h
constexpr uint32_t WC_E_LIMIT_CODE = 11;
// WC_E_LIMIT with the overflow reasons (engine_shared LIM_*) in bits 16+
__device__ inline uint32_t limit_status(uint32_t why) { return WC_E_LIMIT_CODE | (why << 16); }
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;

// Cache of hashbrown iteration orders (votes): insertion-ordered keys (lo, hi |
// nk << 56) -> order. Consecutive pops of a dual search rotate among a few
// lineages whose votes see a few distinct key sequences; 16 entries per side
// keep almost all of them (one LDS round trip instead of the table rebuild).
constexpr int kFxCache = 16;
struct FxCache {
  uint64_t k0[kFxCache], k1[kFxCache], ord[kFxCache];
  uint32_t next;
};

struct Ctl {
  uint32_t prob;
  uint32_t oslot, obuf;  // stream mode: output slot of the claimed problem, slot parity
  uint32_t heap_n, nfree;
  uint32_t status;
  uint32_t action;  // 0 expand, 1 ignore, 2 done
  uint32_t top_slot, top_len;
  uint32_t top_dual;
  uint64_t top_cost;
  uint32_t n_end[2];
  uint32_t multi[2];
  uint32_t n_either;
  uint32_t ovf;
  uint32_t reached;
  uint32_t fin[2];
  uint32_t nheavy, nwide;
  uint64_t cost_acc;
  uint64_t max_err;
  uint64_t farthest[2], last_constraint[2];
  uint64_t trk_total[2], trk_thr[2];
  uint32_t am_len;
  uint32_t act_cnt;  // reads activating at the popped length (dual active_min growth)
  uint32_t n_ret;
  int32_t store_idx;
  uint32_t cache_slot, cache_hit, cache_nend, cache_multi;
  uint32_t hot_slot;  // slot whose RStates are held in Lds::hot (authoritative), kNoSlot = none
  uint32_t hot_prev, hot_load, hot_prev_dual;
  // linear-chain run-ahead (run_chain)
  uint32_t chain_k, chain_slot, chain_stop, chain_novf, chain_nochain, chain_len, chain_nbak;
  uint32_t chain_kcur;  // dual engine: the next chain's length (doubles after a fully accepted chain)
  uint32_t chain_pk;    // chain_prepare predicted N_K's next symbol (cpred[K + 1])
  uint32_t chain_next;  // the chain ended with N_K popped virtually: its one child (chain_sym) starts the next
  uint32_t chain_sym;
#ifdef WC_PHASE_PROF
  uint64_t chain_tot[8];  // (+ wave_heavy's timers, WaveCounters::tq)
#else
  uint64_t chain_tot[5];  // updates, w_out, compares, ed increases, row bytes of one chain pass
#endif
  uint32_t deal_cnt[kEW];  // chain_prepare: reads per wave expected to need an ED increase
  // the chain walk's grouped ED increases (chain_group_heavy): the chain's
  // uniform arguments, in LDS rather than in call registers
  Gm<uint32_t>* gh_nwf;  // the node's wavefront rows
  Gm<uint32_t>* gh_swf;  // slot S's rows (first-rewrite copies)
  const Gm<uint8_t>* gh_rbytes;
  const Gm<uint8_t>* gh_con;
  Sh<uint2>* gh_rt;  // (null in the dual engine: the HBM tables below)
  const Gm<uint64_t>* gh_roff;
  const Gm<uint32_t>* gh_rlenp;
  uint32_t gh_rbegin;
  Sh<RState>* gh_tmp;
  Sh<ChainStep>* gh_cstep;
  Sh<uint32_t>* gh_list;
  Sh<uint8_t>* gh_perm;  // the walk's read order
  uint32_t gh_L0, gh_wcap, gh_list_n, gh_flags;  // flags: early | cost_mode << 1
  int32_t gh_wc;
  uint32_t nkeys[2];
  uint8_t keys[2][kKout];
  double vals[2][kKout];
  FxCache fxc[2];  // per side
  // thread-0 scratch for child enumeration (kept in LDS, not private memory)
  int16_t opt[2][kKout + 1];
  double srt_v[kKout];
  uint8_t srt_s[kKout];
  uint32_t nchild;
  int16_t ch_s[kMaxChild][2];  // symbol per side, -1 = none (lock for dual children)
  uint8_t ch_kind[kMaxChild];  // 0 dual child, 1 stay-single, 2 split (activate_dual)
  uint32_t ch_slot[kMaxChild];
  uint64_t ch_cost[kMaxChild];
  uint32_t ch_len[kMaxChild];
  uint32_t ch_some[kNCB][2];  // Some(dwfa) counts per side of the children being built
  uint32_t cur_slot;
  uint64_t cnt[S_NSTAT];
#ifdef WC_PHASE_PROF
  uint64_t ph[kPhases];
  uint64_t ph_t;
#endif
};

// Phase timing (debug builds with -DWC_PHASE_PROF, read out via WC_PHASES):
// thread 0 charges the shader cycles since the previous mark to phase k.
#ifdef WC_PHASE_PROF
#define PH_MARK(k)                                             \
  do {                                                         \
    if (threadIdx.x == 0) {                                    \
      const uint64_t _t = __builtin_amdgcn_s_memtime();        \
      ctl.ph[(k)] += _t - ctl.ph_t;                            \
      ctl.ph_t = _t;                                           \
    }                                                          \
  } while (0)
// wave-0 sub-phase timers (thread 0 charges the cycles of a code span to k)
#define SUB_T0(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define SUB_T1(k, v)                                                          \
  do {                                                                        \
    if (threadIdx.x == 0) ctl.ph[(k)] += __builtin_amdgcn_s_memtime() - (v);  \
  } while (0)
#define SUB_CNT(k, n)                     \
  do {                                    \
    if (threadIdx.x == 0) ctl.ph[(k)] += (n); \
  } while (0)
// every wave's lane 0 adds a count to k (sums over the waves)
#define SUB_WADD(k, n)                                                                    \
  do {                                                                                    \
    if (lane_id() == 0) atomicAdd((unsigned long long*)&ctl.ph[(k)], (unsigned long long)(n)); \
  } while (0)
#else
#define PH_MARK(k) \
  do {             \
  } while (0)
#define SUB_T0(v) \
  do {            \
  } while (0)
#define SUB_T1(k, v) \
  do {               \
  } while (0)
#define SUB_CNT(k, n) \
  do {                \
  } while (0)
#define SUB_WADD(k, n) \
  do {                 \
  } while (0)
#endif

struct Lds {
  Sh<RState>* hot;       // [hot_sides][nmax] RStates of the node being expanded (single engine; dual_hot)
  Sh<ChainStep>* cstep;  // chain area (single engine with A.chain > 0)
  Sh<ChainOvf>* covf;
  Sh<RState>* ctmp;      // [kEW]
  Sh<uint16_t>* cnom;    // [K+1][nmax]
  Sh<uint8_t>* cwin;     // read windows, slot win_slot(r) of kWinStride bytes
  Sh<uint32_t>* cwb;     // [nmax]
  Sh<uint32_t>* cpc;     // [K+1]
  Sh<uint8_t>* cpred;    // [K+2]
  Sh<uint8_t>* cperm;    // [nmax] the chain walk's read at position p (wave p % kEW, lane p / kEW)
  Sh<uint8_t>* cm0;      // [nmax] each read's first quiet run (chain_prepare)
  Sh<HeapEntry>* heap;
  Sh<uint32_t>* freestack;
  Sh<SlotMeta>* meta;
  Sh<RInfo>* rinfo;    // [sides][nmax]
  Sh<uint32_t>* fe;    // [sides][nmax]
  Sh<uint32_t>* list;  // [list_entries] work list (heavy reads / wide analyses)
  Sh<uint16_t>* ce;    // dual: [kNCB * 2][nmax] edit distances of the children being built (prune + cost; kCeNone = None)
  Sh<uint2>* rt;       // [nmax] the claimed problem's reads: byte offset / 16 from rbytes, length (init_problem)
};

__device__ inline Lds carve(Sh<uint8_t>* smem, uint32_t sides, uint32_t pcap, uint32_t nmax, uint32_t K,
                            uint32_t dual_hot) {
  Lds l;
  Sh<uint8_t>* p = smem;
  l.hot = (Sh<RState>*)p;
  p += (uint64_t)hot_sides(sides, K, dual_hot) * nmax * sizeof(RState);
  l.cstep = (Sh<ChainStep>*)p;
  l.covf = nullptr;
  l.ctmp = nullptr;
  l.cnom = nullptr;
  l.cwin = nullptr;
  l.cwb = nullptr;
  l.cpc = nullptr;
  l.cpred = nullptr;
  l.cperm = nullptr;
  l.cm0 = nullptr;
  if (K) {
    // (engine_shared chain_lds_bytes; side s of a per-side array at s * its
    // one-side size, the dual chain's steps are DualSteps)
    const uint64_t S = chain_sides(sides);
    p += align16((uint64_t)(K + 1) * (S == 2 ? sizeof(DualStep) : sizeof(ChainStep)));
    l.covf = (Sh<ChainOvf>*)p;
    p += align16((uint64_t)kChainOvf * sizeof(ChainOvf));
    l.ctmp = (Sh<RState>*)p;
    p += (uint64_t)chain_waves(kEW) * 4 * 64;
    l.cnom = (Sh<uint16_t>*)p;
    p += align16(S * (K + 1) * nmax * 2);
    l.cwin = p;
    p += align16(S * win_slots(nmax, chain_waves(kEW)) * kWinStride);
    l.cwb = (Sh<uint32_t>*)p;
    p += align16(S * nmax * 4);
    l.cpc = (Sh<uint32_t>*)p;
    p += align16((uint64_t)(K + 1) * 4);
    l.cpred = p;
    p += align16(S * (K + 2));
    l.cperm = p;
    p += align16(nmax);
    l.cm0 = p;
    p += align16(nmax);
  }
  l.heap = (Sh<HeapEntry>*)p;
  p += (uint64_t)pcap * sizeof(HeapEntry);
  l.freestack = (Sh<uint32_t>*)p;
  p += align16((uint64_t)pcap * 4);
  l.meta = (Sh<SlotMeta>*)p;
  p += (uint64_t)pcap * sizeof(SlotMeta);
  l.rinfo = (Sh<RInfo>*)p;
  p += (uint64_t)sides * nmax * sizeof(RInfo);
  l.fe = (Sh<uint32_t>*)p;
  p += align16((uint64_t)sides * nmax * 4);
  l.list = (Sh<uint32_t>*)p;
  p += align16((uint64_t)list_entries(sides, nmax) * 4);
  l.ce = sides == 2 ? (Sh<uint16_t>*)p : nullptr;
  if (sides == 2) p += align16((uint64_t)kDualChildBatch * 2 * nmax * 2);
  // the single engine's read table (the dual engine reads the HBM tables: at
  // 200 reads the 1.6 KB cost cfg3 its third workgroup per CU)
  l.rt = sides == 1 ? (Sh<uint2>*)p : nullptr;
  return l;
}

// slot metadata field by field (a struct copy would move the padding through
// private memory)
__device__ __forceinline__ void meta_put(Sh<SlotMeta>& d, const SlotMeta& m) {
  d.len[0] = m.len[0];
  d.len[1] = m.len[1];
  d.nsome[0] = m.nsome[0];
  d.nsome[1] = m.nsome[1];
  d.flags = m.flags;
}
__device__ __forceinline__ SlotMeta meta_get(const Sh<SlotMeta>& d) {
  SlotMeta m;
  m.len[0] = d.len[0];
  m.len[1] = d.len[1];
  m.nsome[0] = d.nsome[0];
  m.nsome[1] = d.nsome[1];
  m.flags = d.flags;
  m.pad[0] = m.pad[1] = m.pad[2] = 0;
  return m;
}

// ---- priority-queue 1.x emulation (thread 0 only) ----
template <class A, class B>
__device__ __forceinline__ bool prio_less(const A& a, const B& b) {
  if (a.cost != b.cost) return a.cost > b.cost;  // Reverse(cost)
  return a.len < b.len;
}
__device__ __forceinline__ void heap_push(Sh<HeapEntry>* h, Lo<uint32_t>& n, uint32_t cap, HeapEntry e) {
  uint32_t pos = WC_IX(n++, cap);
  (void)cap;
  while (pos > 0) {
    uint32_t parent = (pos - 1) / 2;
    if (!prio_less(h[parent], e)) break;
    h[pos] = h[parent];
    pos = parent;
  }
  h[pos] = e;
}
// push(e) then pop() on a heap of n entries returns e and leaves every entry
// where it was (thread 0's form of wave_dual.hip.hpp wheap_push_pop_noop):
// e beats the root strictly, and at each ancestor of position n the pop's
// sift-down picks the path child (the larger, the left one on ties) and moves
// x, the old parent of n, past it (x strictly lower)
__device__ __forceinline__ bool heap_push_pop_noop(const Sh<HeapEntry>* h, uint32_t n, const HeapEntry& e) {
  if (n == 0) return true;
  if (!prio_less(h[0], e)) return false;
  const uint32_t depth = 31u - (uint32_t)__builtin_clz(n + 1);
  const HeapEntry x = h[((n + 1) >> 1) - 1];
  for (uint32_t k = 1; k < depth; ++k) {
    const uint32_t anc = ((n + 1) >> (k + 1)) - 1, pc = ((n + 1) >> k) - 1;
    const uint32_t sib = (pc & 1u) ? pc + 1 : pc - 1;
    const HeapEntry a = h[anc];
    if (sib < n) {
      const HeapEntry b = h[sib];
      if ((pc & 1u) ? prio_less(a, b) : !prio_less(b, a)) return false;
    }
    if (!prio_less(x, a)) return false;
  }
  return true;
}
// Ctl::top_dual of a pending in-place child (dual_main): its push and the
// next pop were skipped, Ctl::top_* hold it
constexpr uint32_t kTopStashed = 0x80000000u;
#ifdef WC_NO_REPOP
constexpr bool kRepopBlock = false;
#else
constexpr bool kRepopBlock = true;
#endif
__device__ __forceinline__ HeapEntry heap_pop(Sh<HeapEntry>* h, Lo<uint32_t>& n, uint32_t cap) {
  HeapEntry top = h[0];
  top.slot = WC_IX(top.slot, cap);
  (void)cap;
  n--;
  // sift the last entry down from the root: the swap-per-level loop of the
  // reference, with the moving entry kept in registers (same final layout)
  const HeapEntry x = h[n];
  uint32_t i = 0;
  if (n > 1) {
    for (;;) {
      const uint32_t l = 2 * i + 1, r = 2 * i + 2;
      uint32_t largest = i;
      HeapEntry best = x;
      if (l < n) {
        const HeapEntry hl = h[l];
        if (prio_less(best, hl)) {
          largest = l;
          best = hl;
        }
        if (r < n) {
          const HeapEntry hr = h[r];
          if (prio_less(best, hr)) {
            largest = r;
            best = hr;
          }
        }
      }
      if (largest == i) break;
      h[i] = best;
      i = largest;
    }
  }
  h[i] = x;
  return top;
}

// ---- PQueueTracker (pqueue_tracker.rs:10-144), thread 0 only ----
// The count arrays live in HBM (lcap + 2 entries each). The updates are
// no-return atomics, so thread 0 never waits on a read-modify-write; the few
// reads bypass the per-CU L1 (which an atomic does not update).
__device__ __forceinline__ uint32_t trk_load(const Gm<uint32_t>* p) {
  return __hip_atomic_load((const uint32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
struct TrackerRef {
  Gm<uint32_t>* lc;
  Gm<uint32_t>* pc;
  Lo<uint64_t>* total;
  Lo<uint64_t>* thr;
  uint64_t cap;
  uint32_t lim;  // entries of lc / pc (lcap + 2)
  __device__ __forceinline__ void insert(uint32_t v) {
    atomicAdd((uint32_t*)&lc[WC_IX(v, lim)], 1u);
    if (v >= *thr) (*total)++;
  }
  __device__ __forceinline__ void remove(uint32_t v) {
    atomicSub((uint32_t*)&lc[WC_IX(v, lim)], 1u);
    if (v >= *thr) (*total)--;
  }
  __device__ __forceinline__ void increment_threshold() {
    *total -= trk_load(&lc[WC_IX(*thr, lim)]);
    (*thr)++;
  }
  __device__ __forceinline__ uint32_t processed(uint32_t v) const { return trk_load(&pc[WC_IX(v, lim)]); }
  // process() of a length whose processed() count is below capacity (the pop
  // just checked it; only this workgroup's thread 0 touches the tracker)
  __device__ __forceinline__ void process_unchecked(uint32_t v) { atomicAdd((uint32_t*)&pc[WC_IX(v, lim)], 1u); }
};

__device__ inline uint64_t ceil_u64(double x) {
  double c = ceil(x);
  if (!(c > 0.0)) return 0;  // Rust `as u64` saturates negatives / NaN to 0
  if (c >= 18446744073709551615.0) return ~0ull;
  return (uint64_t)c;
}

template <int kCtrl>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
  const uint32_t lo = dpp_u32<kCtrl>((uint32_t)v), hi = dpp_u32<kCtrl>((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}
// (uniform) wave sum of u64 values: DPP row sums, four scalar reads
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
  WC_FULL_EXEC();
  v += dpp_u64<0xb1>(v);
  v += dpp_u64<0x4e>(v);
  v += dpp_u64<0x141>(v);
  v += dpp_u64<0x140>(v);
  uint64_t t = 0;
#pragma unroll
  for (int l = 0; l < 64; l += 16)
    t += ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  return t;
}

// ---- wave-aggregated LDS updates (call with the whole wave converged) ----
// Same-address LDS atomics from many lanes serialize lane by lane; here one
// lane adds the wave's total.
__device__ __forceinline__ void agg_add(Lo<uint32_t>* p, uint32_t v) {
  const uint32_t t = wave_sum_u32(v);
  if (lane_id() == 0 && t) atomicAdd((uint32_t*)p, t);
}
__device__ __forceinline__ void agg_add64(Lo<uint64_t>* p, uint64_t v) {
  const uint64_t t = wave_sum_u64(v);
  if (lane_id() == 0 && t) atomicAdd((unsigned long long*)p, (unsigned long long)t);
}
__device__ __forceinline__ void agg_or(Lo<uint32_t>* p, bool cond, uint32_t bits) {
  if (ballot(cond) && lane_id() == 0) atomicOr((uint32_t*)p, bits);
}
// a slot of the list counted by `counter` for every lane with `take`
__device__ __forceinline__ uint32_t agg_append(Lo<uint32_t>* counter, bool take) {
  WC_FULL_EXEC();
  const uint64_t m = ballot(take);
  if (!m) return 0;
  uint32_t base = 0;
  if (lane_id() == 0) base = atomicAdd((uint32_t*)counter, (uint32_t)__popcll((unsigned long long)m));
  base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
  return base + (uint32_t)__popcll((unsigned long long)(m & ((1ull << lane_id()) - 1ull)));
}

// wave-uniform counters (lane 0 holds them)
__device__ inline void flush_counters(Lo<Ctl>& ctl, const WaveCounters& wc) {
  if (lane_id() == 0) {
    if (wc.updates) atomicAdd((unsigned long long*)&ctl.cnt[S_UPDATES], (unsigned long long)wc.updates);
    if (wc.w_out) atomicAdd((unsigned long long*)&ctl.cnt[S_WOUT], (unsigned long long)wc.w_out);
    if (wc.compares) atomicAdd((unsigned long long*)&ctl.cnt[S_COMPARES], (unsigned long long)wc.compares);
    if (wc.edinc) atomicAdd((unsigned long long*)&ctl.cnt[S_EDINC], (unsigned long long)wc.edinc);
    if (wc.finalizes) atomicAdd((unsigned long long*)&ctl.cnt[S_FINALIZES], (unsigned long long)wc.finalizes);
    if (wc.rowb) atomicAdd((unsigned long long*)&ctl.cnt[S_ROWB], (unsigned long long)wc.rowb);
  }
}
// per-thread counters (every lane its own): wave-reduce, then lane 0 adds
__device__ inline void flush_thread_counters(Lo<Ctl>& ctl, WaveCounters c) {
  c.updates = wave_sum_u32(c.updates);
  c.w_out = wave_sum_u32(c.w_out);
  c.compares = wave_sum_u32(c.compares);
  flush_counters(ctl, c);
}

// A value read from LDS that is the same for the whole workgroup: moving it
// to a scalar register lets loops, branches and addresses stay scalar.
__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ int32_t uni(int32_t x) { return __builtin_amdgcn_readfirstlane(x); }

// per-workgroup engine context (registers)
struct Eng {
  DevConfig cfg;  // by value: uniform registers, not loads through A
  uint32_t chain;
  Gm<uint8_t>* ws;
  const Gm<uint8_t>* rbytes;
  const Gm<uint64_t>* roff;
  const Gm<uint32_t>* rlenp;
  const Gm<int64_t>* ract;  // activation length per read (-1 = active at the root)
  uint64_t sbytes;
  uint32_t nmax, wcap, lcap, pcap, sides, n;
  Gm<uint32_t>* trk;  // [lc0 | pc0 | lc1 | pc1], each lcap+2 u32
  Gm<uint32_t>* total_active;
  Gm<uint32_t>* active_min;
  Gm<uint32_t>* scratch;
  Gm<uint64_t>* act_scr;  // this wave's offset-activation scratch (nullptr = none)
  uint32_t act_m;
  DevProblem P;
  Lds L;
  __device__ SideView sv(uint32_t slot, uint32_t side) const {
    return side_view(ws + (uint64_t)WC_IX(slot, pcap) * sbytes, WC_IX(side, sides), nmax, wcap, lcap);
  }
  // a read's bytes and length from the LDS read table (init_problem fills it
  // from the HBM tables: one dependent HBM round trip less wherever a phase
  // loads read bytes)
  __device__ const Gm<uint8_t>* read(uint32_t r) const {
    return L.rt ? rbytes + (uint64_t)L.rt[WC_IX(r, nmax)].x * 16 : rbytes + roff[P.read_begin + WC_IX(r, nmax)];
  }
  __device__ uint32_t rlen(uint32_t r) const {
    return L.rt ? L.rt[WC_IX(r, nmax)].y : rlenp[P.read_begin + WC_IX(r, nmax)];
  }
  __device__ __forceinline__ TrackerRef tracker(Lo<Ctl>& ctl, int k) const {
    const uint64_t L2 = lcap + 2;
    return TrackerRef{trk + 2 * k * L2, trk + (2 * k + 1) * L2, &ctl.trk_total[k], &ctl.trk_thr[k],
                      cfg.max_capacity_per_size, (uint32_t)L2};
  }
};

// Copy of an engine context into scalar registers: every field is
// workgroup-uniform, so each 32-bit word goes through readfirstlane.
__device__ inline Eng eng_uniform(const Eng& s) {
  static_assert(sizeof(Eng) % 4 == 0, "Eng is copied as words");
  // words through memcpy (no type-punned access to the pointer fields); the
  // context is the same in every lane, so lane 0 alone reads it (a context in
  // scratch is per lane: 64 lanes' reads of it per chain call)
  uint32_t w[sizeof(Eng) / 4] = {};
  if (lane_id() == 0) __builtin_memcpy(w, &s, sizeof(Eng));
#pragma unroll
  for (int i = 0; i < (int)(sizeof(Eng) / 4); ++i) w[i] = (uint32_t)__builtin_amdgcn_readfirstlane((int)w[i]);
  Eng d;
  __builtin_memcpy(&d, w, sizeof(Eng));
  return d;
}

__device__ inline Eng make_eng(const EngineArgs& A, Sh<uint8_t>* smem) {
  Eng E;
  E.cfg = A.cfg;
  E.chain = A.chain;
  E.rbytes = (const Gm<uint8_t>*)A.rbytes;
  E.roff = (const Gm<uint64_t>*)A.roff;
  E.rlenp = (const Gm<uint32_t>*)A.rlen;
  E.ract = (const Gm<int64_t>*)A.ractivate;
  E.nmax = A.nmax;
  E.wcap = A.wcap;
  E.lcap = A.lcap;
  E.pcap = A.pcap;
  E.sides = A.sides;
  E.ws = (Gm<uint8_t>*)A.ws + (uint64_t)blockIdx.x * A.ws_stride;
  E.sbytes = slot_bytes(A.sides, A.nmax, A.wcap, A.lcap);
  Gm<uint32_t>* t = (Gm<uint32_t>*)(E.ws + (uint64_t)A.pcap * E.sbytes);
  const uint32_t L2 = A.lcap + 2;
  E.trk = t;
  Gm<uint8_t>* q = E.ws + (uint64_t)A.pcap * E.sbytes + align16((uint64_t)4 * L2 * 4);
  E.total_active = (Gm<uint32_t>*)q;
  E.active_min = E.total_active + L2;
  q += align16((uint64_t)2 * L2 * 4);
  E.scratch = (Gm<uint32_t>*)q + (uint64_t)wave_id() * (A.wcap + 2);
  E.act_m = A.act_m;
  E.act_scr = A.act_scr ? (Gm<uint64_t>*)A.act_scr + (uint64_t)blockIdx.x * A.act_stride +
                              (uint64_t)wave_id() * 2 * A.act_m * 64
                        : nullptr;
  E.L = carve(smem, A.sides, A.pcap, A.nmax, A.chain, A.dual_hot);
  if (A.stream) {
    // the claimed problem's read table is copied here (stream_claim)
    Gm<uint8_t>* t = E.ws + ws_bytes(A.sides, A.pcap, A.nmax, A.wcap, A.lcap);
    E.roff = (const Gm<uint64_t>*)t;
    E.ract = (const Gm<int64_t>*)(t + align16((uint64_t)A.nmax * 8));
    E.rlenp = (const Gm<uint32_t>*)(t + 2 * align16((uint64_t)A.nmax * 8));
  }
  return E;
}

// The engine context inside an out-of-line phase (the chain walks): rebuilt
// from the kernel arguments (kernarg segment) and the claimed problem, so the
// kernel's own context never has its address taken (that would move it, with
// every pointer in it, to scratch memory for the whole kernel).
// (The kernel passes its kernarg segment pointer: a callee's own
// __builtin_amdgcn_kernarg_segment_ptr() is null.)
#if defined(__HIP_DEVICE_COMPILE__)
using KArgs = const __attribute__((address_space(4))) EngineArgs*;
__device__ __forceinline__ KArgs kernel_args() { return (KArgs)__builtin_amdgcn_kernarg_segment_ptr(); }
#else
using KArgs = const EngineArgs*;
__device__ __forceinline__ KArgs kernel_args() { return nullptr; }
#endif
__device__ inline Eng callee_eng(KArgs kp, const DevProblem& P, Sh<uint8_t>* sbase) {
  // the pointer arrives in vector registers (call ABI): made uniform, the
  // argument loads are scalar loads
  const uint64_t kv = (uint64_t)kp;
  const uint64_t ku = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)kv) |
                      (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(kv >> 32)) << 32;
  const EngineArgs A = *(KArgs)ku;  // the copy is split into registers
  Eng E = make_eng(A, sbase);
  E.P = P;
  E.n = P.n_reads;
  return eng_uniform(E);
}

// ---- host-resident reads (service lanes, EngineArgs::hreads) ----
// Copies the claimed problem's reads from host memory into this workgroup's
// staging area (one rstage_stride slot per read: the bytes, zeros after) and
// repoints the read table at the copies (offsets from A.rbytes = the
// workspace base). Every chunk is a 16-byte load; each thread keeps four in
// flight, so a locus costs a few PCIe round trips rather than one per chunk.
// Out of line and with scalar arguments only: a reference to the engine
// context or the kernel arguments would escape and move them to scratch.
__device__ __noinline__ void stage_reads(const uint8_t* hreads, Gm<uint64_t>* lroff, const Gm<uint32_t>* lrlen,
                                         Gm<uint8_t>* stage, uint64_t stride, uint64_t rel, uint32_t n) {
  const int tid = threadIdx.x;
  const uint32_t cps = (uint32_t)(stride / 16);
  const uint32_t total = n * cps;
  constexpr uint32_t kU = 4;
  for (uint32_t g0 = tid; g0 < total; g0 += kEB * kU) {
    uint4 v[kU];
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) {
      const uint32_t g = g0 + u * kEB;
      v[u] = make_uint4(0, 0, 0, 0);
      if (g < total) {
        const uint32_t r = g / cps, c = g - r * cps;
        if (c * 16 < lrlen[r]) v[u] = *(const Gm<uint4>*)((const Gm<uint8_t>*)hreads + lroff[r] + (uint64_t)c * 16);
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) {
      const uint32_t g = g0 + u * kEB;
      if (g < total) {
        const uint32_t r = g / cps, c = g - r * cps;
        *(Gm<uint4>*)(stage + (uint64_t)r * stride + (uint64_t)c * 16) = v[u];
      }
    }
  }
  __syncthreads();
  for (uint32_t r = tid; r < n; r += kEB) lroff[r] = rel + (uint64_t)r * stride;
  __syncthreads();
}

// stream mode: this workgroup has left its claim loop (the host's signal that
// the launch is draining or done, read without any HIP call)
__device__ inline void stream_exit(const EngineArgs& A) {
  if (A.stream && A.exited && threadIdx.x == 0)
    __hip_atomic_store(&A.exited[blockIdx.x], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---- work claiming ----
// Static mode: the next problem of the launch's list. Stream mode: the next
// sequence number of the host-fed ring; wait (bounded by idle_ticks) until the
// host has published it or has said nothing more will come, and until this
// workgroup's next output slot has been consumed; then copy the problem's
// descriptor and read table into the workgroup's workspace. Returns the
// problem (sequence number), or ~0u to exit; `oslot` = output slot index.
__device__ inline uint32_t claim_problem(const EngineArgs& A, Lo<Ctl>& ctl, Eng& E, uint32_t& oslot) {
  const int tid = threadIdx.x;
  if (!A.stream) {
    if (tid == 0) ctl.prob = atomicAdd(A.work_counter, 1u);
    __syncthreads();
    const uint32_t prob = uni(ctl.prob);
    if (prob >= A.n_problems) return ~0u;
    E.P = A.problems[prob];
    oslot = prob;
    return prob;
  }
  if (tid == 0) {
    const uint32_t seq = atomicAdd(A.qhead, 1u);
    uint32_t got = seq;
    uint64_t t0 = wall_clock64();
    // tail and stop in one 8-byte read of host memory; an idle workgroup
    // backs off exponentially (up to ~1 ms between reads) so waiting
    // workgroups put almost no load on the host link
    uint32_t nap = 1, hb_seen = ~0u;
    for (;;) {
      const uint64_t ts = __hip_atomic_load(reinterpret_cast<uint64_t*>(A.sctl), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      if (seq < (uint32_t)ts) break;
      if (ts >> 32) {  // stop: nothing more will be published
        got = ~0u;
        break;
      }
      // give up only when the host itself has stopped (no heartbeat), never
      // because work is slow to come: a claimed sequence number must be served
      const uint32_t hb = __hip_atomic_load(&A.sctl->heartbeat, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (hb != hb_seen) {
        hb_seen = hb;
        t0 = wall_clock64();
      } else if (wall_clock64() - t0 > A.idle_ticks) {
        __hip_atomic_store(&A.sctl->abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        got = ~0u;
        break;
      }
      for (uint32_t k = 0; k < nap; ++k) __builtin_amdgcn_s_sleep(127);
      nap = min(nap * 2, 256u);
    }
    if (got != ~0u) {
      // two output slots per workgroup, used alternately; the host clears a
      // slot's flag when it has consumed the result
      ctl.obuf ^= 1u;
      const uint32_t os = blockIdx.x * 2 + ctl.obuf;
      t0 = wall_clock64();
      nap = 1;
      while (__hip_atomic_load(&A.done[os], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
        const uint32_t hb = __hip_atomic_load(&A.sctl->heartbeat, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (hb != hb_seen) {
          hb_seen = hb;
          t0 = wall_clock64();
        } else if (wall_clock64() - t0 > A.idle_ticks) {
          __hip_atomic_store(&A.sctl->abort, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          got = ~0u;
          break;
        }
        for (uint32_t k = 0; k < nap; ++k) __builtin_amdgcn_s_sleep(127);
        nap = min(nap * 2, 64u);
      }
      ctl.oslot = os;
    }
    ctl.prob = got;
  }
  __syncthreads();
  const uint32_t seq = uni(ctl.prob);
  if (seq == ~0u) return ~0u;
  oslot = uni(ctl.oslot);
  DevProblem P = A.problems[seq % A.qcap];
  const uint32_t base = P.read_begin;
  Gm<uint64_t>* lroff = (Gm<uint64_t>*)E.roff;
  Gm<int64_t>* lract = (Gm<int64_t>*)E.ract;
  Gm<uint32_t>* lrlen = (Gm<uint32_t>*)E.rlenp;
  for (uint32_t r = tid; r < P.n_reads; r += kEB) {
    const uint32_t q = (base + r) % A.qslots;
    lroff[r] = A.roff[q];
    lract[r] = A.ractivate[q];
    lrlen[r] = A.rlen[q];
  }
  P.read_begin = 0;
  E.P = P;
  __syncthreads();
  if (A.hreads) {
    Gm<uint8_t>* stage = (Gm<uint8_t>*)lroff + rtab_bytes(A.nmax);
    stage_reads((const uint8_t*)A.hreads, lroff, lrlen, stage, A.rstage_stride,
                (uint64_t)(stage - (const Gm<uint8_t>*)A.rbytes), P.n_reads);
  }
  return seq;
}

// Where a workgroup's search state (heap, slot metadata, nominations, chain
// area) lives: dynamic LDS, or its own HBM region in the global-state build.
__device__ inline Sh<uint8_t>* state_base(const EngineArgs& A, uint8_t* smem) {
#ifdef WC_GLOBAL_STATE
  return (Sh<uint8_t>*)(A.gstate + (uint64_t)blockIdx.x * A.gstate_stride);
#else
  return (Sh<uint8_t>*)smem;
#endif
}

// ---- per-problem init: free stack, trackers, root node (consensus.rs:384-403) ----
__device__ inline void init_problem(Eng& E, Lo<Ctl>& ctl) {
  const int tid = threadIdx.x;
  const DevConfig& cfg = E.cfg;
  if (tid == 0) {
    ctl.heap_n = 0;
    ctl.nfree = E.pcap - 1;  // slot 0 (the stack top) becomes the root
    ctl.status = ST_OK;
    ctl.max_err = ~0ull;
    for (int k = 0; k < 2; ++k) {
      ctl.farthest[k] = 0;
      ctl.last_constraint[k] = 0;
      ctl.trk_total[k] = 0;
      ctl.trk_thr[k] = 0;
    }
    ctl.n_ret = 0;
    ctl.am_len = 1;
    ctl.cache_slot = kNoSlot;
    ctl.hot_slot = kNoSlot;
    ctl.hot_load = 0;
    ctl.chain_kcur = 4;
    for (int sd = 0; sd < 2; ++sd) {  // no cached fx orders (nk <= 14, so k1 = ~0 never matches)
      for (int k = 0; k < kFxCache; ++k) ctl.fxc[sd].k1[k] = ~0ull;
      ctl.fxc[sd].next = 0;
    }
    for (int s = 0; s < S_NSTAT; ++s) ctl.cnt[s] = 0;
#ifdef WC_PHASE_PROF
    for (int k = 0; k < kPhases; ++k) ctl.ph[k] = 0;
    ctl.ph_t = __builtin_amdgcn_s_memtime();
#endif
  }
  for (uint32_t i = tid; i < E.pcap; i += kEB) E.L.freestack[i] = E.pcap - 1 - i;
  for (uint32_t i = tid; i < 4 * (E.lcap + 2); i += kEB) E.trk[i] = 0;
  // the read table in LDS (reads start 16-byte aligned in every arena)
  for (uint32_t r = tid; E.L.rt && r < E.n; r += kEB)
    E.L.rt[r] = make_uint2((uint32_t)(E.roff[E.P.read_begin + r] >> 4), E.rlenp[E.P.read_begin + r]);
  __syncthreads();
  SideView v = E.sv(0, 0);
  for (uint32_t r = tid; r < E.n; r += kEB) {
    // e = 0 (or None), off = 0, maxb = 0, nscmp = 0, nf = 1: the single
    // diagonal d=0 sits at the (empty) consensus end
    const uint32_t e = E.ract[E.P.read_begin + r] < 0 ? 0u : kInactive;
    const uint4 z = make_uint4(0, 0, 0, 0);
    rstate_store(&v.rs[r], RRaw{make_uint4(e, 0, 0, 1u << 16), z, z, z});
    v.wf[(uint64_t)r * E.wcap] = 0;
  }
  __syncthreads();
  if (tid == 0) {
    auto& m = E.L.meta[0];
    m.len[0] = m.len[1] = 0;
    m.nsome[0] = E.P.n_active;
    m.nsome[1] = 0;
    m.flags = 0;
    E.total_active[0] = E.P.n_active;
    E.active_min[0] = (uint32_t)max(cfg.min_count, ceil_u64(cfg.min_af * (double)E.P.n_active));
    E.tracker(ctl, 0).insert(0);
    heap_push(E.L.heap, ctl.heap_n, E.pcap, HeapEntry{0, 0, 0});
  }
  __syncthreads();
}

// ---- ANALYZE one node side (block-level, contains barriers) ----
// Thread per read from the RState; reads with a wide frontier are nominated by
// a wave over their full wavefront. Counts n_end / multi of the side.
// Where a node's per-read RStates live: in its HBM slot, or (kHot) in the
// LDS copy of the node being expanded (single engine: the popped node).
template <bool kHot>
__device__ __forceinline__ auto node_rs(Eng& E, uint32_t slot, uint32_t side) {
  if constexpr (kHot) return E.L.hot + side * E.nmax;
  else return E.sv(slot, side).rs;
}

// ---- ANALYZE the nominations of every read on up to two sides of one node ----
// Work items are (side, read): thread step from the RState frontier, the
// wave path for wide frontiers. ctl.nheavy must be 0 on entry.
template <bool kHot>
WC_PHASE_FN void analyze_sides(Eng& E, Lo<Ctl>& ctl, uint32_t slot, uint32_t nsides, uint32_t len0, uint32_t len1,
                               Sh<RInfo>* out0, Sh<RInfo>* out1) {
  const int tid = threadIdx.x, lane = lane_id();
  const uint32_t n = E.n, items = nsides * n;
  uint32_t ends0 = 0, ends1 = 0;
  bool multi0 = false, multi1 = false;
  for (uint32_t base = 0; base < items; base += kEB) {
    const uint32_t it = base + tid;
    bool wide = false;
    if (it < items) {
      const uint32_t side = it >= n ? 1u : 0u, r = it - side * n;
      Sh<RInfo>* out = (side ? out1 : out0) + r;
      const RRaw s = rstate_load(&node_rs<kHot>(E, slot, side)[r]);
      if (rraw_e(s) == kInactive) {
        out->e = kInactive;
        out->n = 0;
        out->end = 0;
      } else if (rraw_flags(s) & kWide) {
        wide = true;
      } else {
        Front f;
        front_load(s, f);
        bool m;
        thread_analyze(f, E.read(r), E.rlen(r), side ? len1 : len0, out, m);
        if (side) {
          ends1 += out->end;
          multi1 |= m;
        } else {
          ends0 += out->end;
          multi0 |= m;
        }
      }
    }
    const uint32_t k = agg_append(&ctl.nheavy, wide);
    if (wide) E.L.list[WC_IX(k, list_entries(E.sides, E.nmax))] = it;
  }
  agg_add(&ctl.n_end[0], ends0);
  agg_add(&ctl.n_end[1], ends1);
  agg_or(&ctl.multi[0], multi0, 1u);
  agg_or(&ctl.multi[1], multi1, 1u);
  __syncthreads();
  const uint32_t nh = uni(ctl.nheavy);
  for (uint32_t k = wave_id(); k < nh; k += kEW) {
    const uint32_t it = uni(E.L.list[WC_IX(k, list_entries(E.sides, E.nmax))]);
    const uint32_t side = it >= n ? 1u : 0u, r = it - side * n;
    Sh<RInfo>* out = (side ? out1 : out0) + r;
    const auto rs = node_rs<kHot>(E, slot, side);
    const uint32_t e = rs[r].e, off = rs[r].off;
    const bool ok = wave_analyze_read(E.sv(slot, side).wf + (uint64_t)r * E.wcap, e, off, E.read(r), E.rlen(r),
                                      side ? len1 : len0, out);
    if (lane == 0) {
      if (!ok) atomicOr(&ctl.ovf, 1u);
      if (out->end) atomicAdd(&ctl.n_end[side], 1u);
      if (out->n > 1) atomicOr(&ctl.multi[side], 1u);
    }
  }
  __syncthreads();
}
// side 0 only (the single engine)
template <bool kHot>
WC_SINGLE_FN void analyze_side0(Eng& E, Lo<Ctl>& ctl, uint32_t slot, uint32_t len, Sh<RInfo>* out) {
  if (threadIdx.x == 0) ctl.nheavy = 0;
  __syncthreads();
  analyze_sides<kHot>(E, ctl, slot, 1, len, 0, out, out);
}

// ---- FINALIZE one side on scratch (the node is not modified) ----
template <bool kHot>
WC_PHASE_FN void finalize_side(Eng& E, Lo<Ctl>& ctl, uint32_t slot, uint32_t side, uint32_t len, uint32_t* fe,
                                     WaveCounters& cnt) {
  const int lane = lane_id();
  SideView v = E.sv(slot, side);
  const auto rs = node_rs<kHot>(E, slot, side);
  for (uint32_t r = wave_id(); r < E.n; r += kEW) {
    const uint32_t e = rs[r].e;
    if (e == kInactive) {
      if (lane == 0) fe[r] = kInactive;
      continue;
    }
    uint32_t f = 0;
    const bool ok = wave_finalize_read(v.wf + (uint64_t)r * E.wcap, e, rs[r].off, E.read(r), E.rlen(r), v.con,
                                       len, E.cfg.wildcard, E.scratch, E.wcap, f, cnt);
    if (lane == 0) {
      if (!ok) atomicOr(&ctl.ovf, 4u);
      fe[r] = ok ? f : kInactive;
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// ---- PUSH symbols onto up to two sides of one node (block-level, barriers) ----
// The new symbol is already written at con[len-1] of each pushed side.
// Work items are (side, read) pairs: thread step on the RState, then the wave
// path for reads that must grow their edit distance. When `info` is set, the
// pushed side-0 child's nominations are written there (the next pop's
// analysis). When `want_cost`, accumulates the single-side priority cost.
// kSrcHot: the parent's RStates are the LDS copy (else the slot's own);
// kDstHot: the child's RStates go to the LDS copy (else to the slot).
template <bool kSrcHot, bool kDstHot>
WC_SINGLE_FN void push_sides(Eng& E, Lo<Ctl>& ctl, uint32_t slot, int s0, int s1, uint32_t len0, uint32_t len1,
                                  bool want_cost, Sh<RInfo>* info) {
  const int tid = threadIdx.x, lane = lane_id();
  const DevConfig& cfg = E.cfg;
  const bool early = cfg.early != 0;
  if (tid == 0) ctl.nheavy = 0;
  __syncthreads();
  WaveCounters tc = {0, 0, 0, 0, 0, 0};
  uint64_t cost = 0;
  uint32_t ends = 0, multi = 0;
  // work items over the pushed sides only: (side, read) with side >= first
  const uint32_t first = s0 >= 0 ? 0u : 1u;
  const uint32_t items = ((s0 >= 0 ? 1u : 0u) + (s1 >= 0 ? 1u : 0u)) * E.n;
  for (uint32_t base = 0; base < items; base += kEB) {
    const uint32_t it = base + tid;
    const uint32_t hi = it >= E.n ? 1u : 0u, r = it - hi * E.n, side = first + hi;
    bool heavy_item = false;
    do {
    if (it >= items) break;
    const int sym = side == 0 ? s0 : s1;
    SideView v = E.sv(slot, side);
    const auto dst = node_rs<kDstHot>(E, slot, side);
    const RRaw s = rstate_load(&node_rs<kSrcHot>(E, slot, side)[r]);
    Sh<RInfo>* out = (info && side == 0) ? &info[r] : nullptr;
    if (rraw_e(s) == kInactive) {
      if (kSrcHot != kDstHot) rstate_store(&dst[r], s);
      if (out) {
        out->e = kInactive;
        out->n = 0;
        out->end = 0;
      }
      break;
    }
    const uint32_t olen = side == 0 ? len0 : len1;
    const Gm<uint8_t>* rd = E.read(r);
    const uint32_t blen = E.rlen(r);
    if (rraw_flags(s) & kWide) {  // frontier too wide for the register path
      if (kSrcHot != kDstHot) rstate_store(&dst[r], s);
      heavy_item = true;
      break;
    }
    Front f;
    front_load(s, f);
    uint32_t cmp = 0;
    const bool heavy =
        thread_push(f, GlobalBytes{rd}, blen, olen - 1, (uint8_t)sym, cfg.wildcard, early, v.wf + (uint64_t)r * E.wcap, cmp);
    tc.compares += cmp;
    front_store(&dst[r], f);
    if (heavy) {
      heavy_item = true;
      break;
    }
    tc.updates++;
    tc.w_out += 2 * f.e + 1;
    cost += cost_of(f.e, cfg.cost_mode);
    if (out) {
      bool m;
      thread_analyze(f, rd, blen, olen, out, m);
      ends += out->end;
      multi |= m;
    }
    } while (0);
    const uint32_t k = agg_append(&ctl.nheavy, heavy_item);
    if (heavy_item) E.L.list[WC_IX(k, list_entries(E.sides, E.nmax))] = side * E.n + r;
  }

  flush_thread_counters(ctl, tc);

  agg_add(&ctl.n_end[0], ends);
  agg_or(&ctl.multi[0], multi != 0, 1u);
  if (want_cost) agg_add64(&ctl.cost_acc, cost);
  __syncthreads();
  PH_MARK(5);
  const uint32_t nh = uni(ctl.nheavy);
  WaveCounters cnt = {0, 0, 0, 0, 0, 0};
  for (uint32_t k = wave_id(); k < nh; k += kEW) {
    const uint32_t it = E.L.list[WC_IX(k, list_entries(E.sides, E.nmax))];
    const uint32_t side = it >= E.n ? 1u : 0u, r = it - side * E.n;
    SideView v = E.sv(slot, side);
    const uint32_t olen = side == 0 ? len0 : len1;
    const int sym = side == 0 ? s0 : s1;
    uint32_t e = 0;
    Gm<uint32_t>* wf = v.wf + (uint64_t)r * E.wcap;
    const auto dst = node_rs<kDstHot>(E, slot, side);
    if (!wave_heavy(&dst[r], wf, E.read(r), E.rlen(r), v.con, olen, (uint8_t)sym, cfg.wildcard, early, E.wcap, cnt,
                    e)) {
      if (lane == 0) atomicOr(&ctl.ovf, 4u);
      continue;
    }
    if (info && side == 0) {
      const bool ok = wave_analyze_read(wf, e, dst[r].off, E.read(r), E.rlen(r), olen, &info[r]);
      if (lane == 0) {
        if (!ok) atomicOr(&ctl.ovf, 1u);
        if (info[r].end) atomicAdd(&ctl.n_end[0], 1u);
        if (info[r].n > 1) atomicOr(&ctl.multi[0], 1u);
      }
    }
    if (want_cost && lane == 0) atomicAdd((unsigned long long*)&ctl.cost_acc, (unsigned long long)cost_of(e, cfg.cost_mode));
  }
  flush_counters(ctl, cnt);
  __syncthreads();
  PH_MARK(6);
}

__device__ inline void copy_bytes(Gm<uint8_t>* d, const Gm<uint8_t>* s, uint32_t len) {
  const uint32_t n16 = len >> 4;
  for (uint32_t i = threadIdx.x; i < n16; i += kEB) ((Gm<uint4>*)d)[i] = ((const Gm<uint4>*)s)[i];
  for (uint32_t i = (n16 << 4) + threadIdx.x; i < len; i += kEB) d[i] = s[i];
}

// move the RStates of one node side between its slot and the LDS copy
__device__ inline void hot_store(Eng& E, uint32_t slot, uint32_t side) {
  Gm<RState>* d = E.sv(slot, side).rs;
  const Sh<RState>* h = E.L.hot + side * E.nmax;
  for (uint32_t r = threadIdx.x; r < E.n; r += kEB) rstate_store(&d[r], rstate_load(&h[r]));
}
__device__ inline void hot_fetch(Eng& E, uint32_t slot, uint32_t side) {
  const Gm<RState>* d = E.sv(slot, side).rs;
  Sh<RState>* h = E.L.hot + side * E.nmax;
  for (uint32_t r = threadIdx.x; r < E.n; r += kEB) rstate_store(&h[r], rstate_load(&d[r]));
}

// ---- clone a node: RState records, live wavefront rows, consensus bytes ----
// kSrcHot / kDstHot: the source's / destination's RStates are the LDS copy of
// the node being expanded. kCopyRs: copy the RStates too (the single engine's
// clones do not: their push writes the child's RStates straight into the slot).
template <bool kSrcHot, bool kDstHot = false, bool kCopyRs = !kSrcHot>
__device__ inline void copy_side(Eng& E, uint32_t src, uint32_t ssrc, uint32_t dst, uint32_t sdst, uint32_t len) {
  SideView a = E.sv(src, ssrc), b = E.sv(dst, sdst);
  const auto ars = node_rs<kSrcHot>(E, src, ssrc);
  const auto brs = node_rs<kDstHot>(E, dst, sdst);
  copy_bytes(b.con, a.con, len);
  // thread per read: its RState, then its wavefront row in 16-byte moves with
  // eight loads in flight, so the reads' copies overlap instead of queueing
  // behind one wave per read (rows are 16-byte aligned: wcap % 64 == 0)
  for (uint32_t r = threadIdx.x; r < E.n; r += kEB) {
    const RRaw st = rstate_load(&ars[r]);
    if (kCopyRs) rstate_store(&brs[r], st);
    const uint32_t e = rraw_e(st);
    if (e == kInactive) continue;
    const uint32_t n4 = (2 * e + 1 + 3) >> 2;
    const Gm<uint4>* wa = (const Gm<uint4>*)(a.wf + (uint64_t)r * E.wcap);
    Gm<uint4>* wb = (Gm<uint4>*)(b.wf + (uint64_t)r * E.wcap);
    // (rows hold wcap >= 64 entries, a multiple of 32: the eight loads stay inside)
    for (uint32_t i = 0; i < n4; i += 8) {
      const uint4 t0 = wa[i], t1 = wa[i + 1], t2 = wa[i + 2], t3 = wa[i + 3];
      const uint4 t4 = wa[i + 4], t5 = wa[i + 5], t6 = wa[i + 6], t7 = wa[i + 7];
      wb[i] = t0;
      if (i + 1 < n4) wb[i + 1] = t1;
      if (i + 2 < n4) wb[i + 2] = t2;
      if (i + 3 < n4) wb[i + 3] = t3;
      if (i + 4 < n4) wb[i + 4] = t4;
      if (i + 5 < n4) wb[i + 5] = t5;
      if (i + 6 < n4) wb[i + 6] = t6;
      if (i + 7 < n4) wb[i + 7] = t7;
    }
  }
}

// ---- offset activation of one node side (block-level, barriers) ----
// Every read whose activation length is `alen` (consensus.rs:330-334,
// dual_consensus.rs:633-639) is activated against this side's consensus
// con[0..clen) (consensus.rs:413-448 / dual_consensus.rs:866-906), one wave
// per read. Adds the new reads' costs to ctl.cost_acc (want_cost) and, when
// `info` is set, writes their nominations there (the pushed child's analysis
// cache) and counts their ends/multi. ctl.ovf: 4 wavefront capacity, 2 offset
// scratch, 16 an already active read (the reference's assert).
template <bool kHot>
WC_PHASE_FN void activate_side(Eng& E, Lo<Ctl>& ctl, uint32_t slot, uint32_t side, uint32_t clen, uint32_t alen,
                                     bool want_cost, Sh<RInfo>* info) {
  const int tid = threadIdx.x, lane = lane_id();
  if (tid == 0) ctl.nheavy = 0;
  __syncthreads();
  for (uint32_t r = tid; r < E.n; r += kEB)
    if (E.ract[E.P.read_begin + r] == (int64_t)alen) E.L.list[WC_IX(atomicAdd(&ctl.nheavy, 1u), list_entries(E.sides, E.nmax))] = r;
  __syncthreads();
  const uint32_t nh = uni(ctl.nheavy);
  SideView v = E.sv(slot, side);
  const auto dst = node_rs<kHot>(E, slot, side);
  WaveCounters cnt = {0, 0, 0, 0, 0, 0};
  for (uint32_t k = wave_id(); k < nh; k += kEW) {
    const uint32_t r = E.L.list[WC_IX(k, list_entries(E.sides, E.nmax))];
    if (uni(dst[r].e) != kInactive) {
      if (lane == 0) atomicOr(&ctl.ovf, 16u);
      continue;
    }
    Gm<uint32_t>* wf = v.wf + (uint64_t)r * E.wcap;
    uint32_t e = 0;
    const int rc = wave_activate(&dst[r], wf, E.read(r), E.rlen(r), v.con, clen, E.cfg, E.wcap, E.act_scr, E.act_m,
                                 cnt, e);
    if (rc != 0) {
      if (lane == 0) atomicOr(&ctl.ovf, rc == 1 ? 4u : 2u);
      continue;
    }
    if (info) {
      __builtin_amdgcn_wave_barrier();
      const bool ok = wave_analyze_read(wf, e, dst[r].off, E.read(r), E.rlen(r), clen, &info[r]);
      if (lane == 0) {
        if (!ok) atomicOr(&ctl.ovf, 1u);
        if (info[r].end) atomicAdd(&ctl.n_end[side], 1u);
        if (info[r].n > 1) atomicOr(&ctl.multi[side], 1u);
      }
    }
    if (want_cost && lane == 0)
      atomicAdd((unsigned long long*)&ctl.cost_acc, (unsigned long long)cost_of(e, E.cfg.cost_mode));
  }
  flush_counters(ctl, cnt);
  __syncthreads();
}

// ---- VOTES (consensus.rs:540-564 / dual_consensus.rs:1242-1290) ----
// One wave. Outer-map insertion order = first appearance over (read index,
// inner iteration position); values are summed per key strictly in read order
// (the reference's f64 order), weight * occ / split. When no read has two
// distinct symbols (and no weights), every contribution is exactly 1.0, so the
// per-key sums are exact integer counts (order-independent) and are taken
// with ballots. Weights follow get_ed_weights (dual_consensus.rs:1299-1336).
__device__ inline double vote_weight(const Sh<RInfo>* r0, const Sh<RInfo>* r1, uint32_t r, bool is_dual, bool side1) {
  if (!is_dual) return 1.0;
  const bool h1 = r0[r].e != kInactive, h2 = r1[r].e != kInactive;
  const double v1 = h1 ? fmax((double)r0[r].e, 0.5) : 0.0;
  const double v2 = h2 ? fmax((double)r1[r].e, 0.5) : 0.0;
  if (h1 && h2) return (side1 ? v2 : v1) / (v1 + v2);
  if ((h1 && side1) || (h2 && !side1)) return 1.0;
  return 0.0;
}

// One read's nominations in registers (RInfo is 32 bytes: two 16-byte LDS reads)
struct RInfoReg {
  uint32_t n, split, e;
  uint64_t sym;    // sym[k] = byte k
  uint4 occ;       // occ[k] = 16-bit halves: k=0,1 in .x ... k=6,7 in .w
};
__device__ __forceinline__ RInfoReg rinfo_load(const Sh<RInfo>* p) {
  static_assert(sizeof(RInfo) == 32, "RInfo layout");
  const uint4 a = ((const Sh<uint4>*)p)[0];
  const uint4 b = ((const Sh<uint4>*)p)[1];
  RInfoReg x;
  x.n = a.x & 0xFFu;
  x.split = a.x >> 16;
  x.sym = (uint64_t)a.y | ((uint64_t)a.z << 32);
  x.occ = make_uint4(a.w, b.x, b.y, b.z);
  x.e = b.w;
  return x;
}
__device__ __forceinline__ uint32_t occ_at(const uint4& o, uint32_t k) {
  const uint32_t w = k < 2 ? o.x : (k < 4 ? o.y : (k < 6 ? o.z : o.w));
  return (k & 1) ? (w >> 16) : (w & 0xFFFFu);
}

__device__ __forceinline__ double readlane_f64(double v, int l) {
  const long long b = __double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)b, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// acc + 1.0 + 1.0 + ... (t times) with IEEE round-to-nearest after every
// add, in closed form. Within one binade [2^p, 2^(p+1)) (acc < 2^53) every
// integer step is exact, so a run that stays below the next power of two is a
// single exact add; the step that crosses it is done as a real f64 add (the
// only step that can round). At most ~log2(t) crossings.
__device__ inline double add_ones(double acc, uint32_t t) {
  while (t) {
    if (acc == trunc(acc)) return acc + (double)t;  // integer + integer: exact
    int ex;
    frexp(acc, &ex);                          // acc in [2^(ex-1), 2^ex)
    const double room = ldexp(1.0, ex) - acc;  // exact (same ulp grid)
    const uint32_t k = min(t, (uint32_t)ceil(room) - 1u);  // steps staying below 2^ex
    acc += (double)k;
    t -= k;
    if (t) {
      acc += 1.0;
      t--;
    }
  }
  return acc;
}

// wave-uniform 256-bit symbol set
struct SymSet {
  uint64_t w0, w1, w2, w3;
  __device__ bool has(uint32_t s) const {
    const uint64_t w = s < 64 ? w0 : (s < 128 ? w1 : (s < 192 ? w2 : w3));
    return (w >> (s & 63)) & 1ull;
  }
  __device__ void add(uint32_t s) {
    const uint64_t b = 1ull << (s & 63);
    if (s < 64) w0 |= b;
    else if (s < 128) w1 |= b;
    else if (s < 192) w2 |= b;
    else w3 |= b;
  }
};

// Core of the votes over one node side (one wave). load(r) gives read r's
// nominations (e = kInactive for None), weight(r) its vote weight (weighted
// mode only). On return lane k < m holds the k-th key in iteration order and
// its f64 vote. Returns false when more than kKout distinct symbols occur.
template <class Load, class Weight>
__device__ inline bool wave_votes_core(Load load, Weight weight, uint32_t n, bool weighted, bool multi, int wc,
                                       uint64_t mc, bool odd_ok, uint32_t& m_out, uint32_t& key_out, double& val_out,
                                       Lo<uint64_t>* ph = nullptr, Lo<FxCache>* fxc = nullptr) {
  WC_FULL_EXEC();  // (ballots over every read lane, the DPP sums below)
  const int lane = lane_id();
#ifdef WC_PHASE_PROF
  uint64_t vt = __builtin_amdgcn_s_memtime();
#define VOTE_T(k)                                              \
  do {                                                         \
    if (ph && threadIdx.x == 0) {                              \
      const uint64_t t1 = __builtin_amdgcn_s_memtime();        \
      ph[k] += t1 - vt;                                        \
      vt = t1;                                                 \
    }                                                          \
  } while (0)
#else
#define VOTE_T(k) \
  do {            \
  } while (0)
#endif
  // 1. outer-map insertion order: first appearance over (read, inner order)
  uint64_t ins_lo = 0, ins_hi = 0;
  uint32_t nk = 0;
  SymSet known = {0, 0, 0, 0};
  auto ins_at = [&](uint32_t j) { return j < 8 ? byte_at(ins_lo, j) : byte_at(ins_hi, j - 8); };
  // Unweighted votes where no read has two distinct tip symbols (`multi`
  // false): every voter adds exactly 1.0 to its one symbol, so one ballot per
  // distinct symbol gives both the insertion order and the (exact) per-key
  // sums; lane i counts the reads of the i-th inserted key.
#ifdef WC_NO_SINGLE_SYM  // (diagnostic variant: every vote takes the general path)
  const bool single_sym = false;
#else
  const bool single_sym = !weighted && !multi;
#endif
  uint32_t cins = 0;
  for (uint32_t base = 0; base < n && single_sym; base += 64) {
    const uint32_t r = base + lane;
    RInfoReg x = {0, 0, kInactive, 0, make_uint4(0, 0, 0, 0)};
    if (r < n) x = load(r);
    const uint32_t s0 = (x.e != kInactive && x.n) ? byte_at(x.sym, 0) : 0x100u;
    uint64_t rem = ballot(s0 != 0x100u);
    while (rem) {
      const uint32_t s = (uint32_t)__builtin_amdgcn_readlane((int)s0, __builtin_ctzll(rem));
      const uint64_t mm = ballot(s0 == s);
      rem &= ~mm;
      uint32_t k = 0;
      if (known.has(s)) {
        while (ins_at(k) != s) ++k;
      } else {
        if (nk == (uint32_t)kKout) return false;
        if (nk < 8) ins_lo |= (uint64_t)s << (8 * nk);
        else ins_hi |= (uint64_t)s << (8 * (nk - 8));
        k = nk++;
        known.add(s);
      }
      if ((uint32_t)lane == k) cins += (uint32_t)__popcll((unsigned long long)mm);
    }
  }
  for (uint32_t base = 0; base < n && !single_sym; base += 64) {
    const uint32_t r = base + lane;
    RInfoReg x = {0, 0, kInactive, 0, make_uint4(0, 0, 0, 0)};
    if (r < n) x = load(r);
    bool voter = x.e != kInactive;
    if (voter && weighted) voter = weight(r) > 0.0;
    const uint32_t xn = voter ? x.n : 0u;
    // per lane, the high bit of byte j stays set while its symbol j (j < xn)
    // is not a key yet (a read's symbols are distinct); the keys of earlier
    // chunks are cleared first, eight bytes at a time
    constexpr uint64_t kHi = 0x8080808080808080ull, kOnes = 0x0101010101010101ull;
    uint64_t rem = xn >= 8u ? kHi : kHi & ((1ull << (8u * xn)) - 1ull);
    for (uint32_t k = 0; k < nk; ++k) rem &= nz_bytes(x.sym ^ (kOnes * ins_at(k)));
    for (;;) {
      // the first read (lane) with a symbol not yet a key, and its first one
      const uint64_t m = ballot(rem != 0);
      if (!m) break;
      const int first = __ffsll((unsigned long long)m) - 1;
      const uint64_t rf = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(rem >> 32), first) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)rem, first);
      const uint64_t sf = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x.sym >> 32), first) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x.sym, first);
      const uint32_t s = byte_at(sf, (uint32_t)__builtin_ctzll(rf) >> 3);
      if (nk == (uint32_t)kKout) return false;
      if (nk < 8) ins_lo |= (uint64_t)s << (8 * nk);
      else ins_hi |= (uint64_t)s << (8 * (nk - 8));
      nk++;
      known.add(s);
      rem &= nz_bytes(x.sym ^ (kOnes * s));
    }
  }
  VOTE_T(28);
  // 2. hashbrown iteration order, wildcard removed (consensus.rs:556-561);
  // consecutive pops mostly see the same keys in the same insertion order,
  // so the last order is kept (fxc) and reused on a match
  uint64_t ord = 0;
  const uint64_t tag = ins_hi | ((uint64_t)nk << 56);
  uint64_t hit = 0;
  if (fxc) {  // lanes 0..15 probe one entry each
    const uint32_t e = (uint32_t)lane & (kFxCache - 1);
    hit = ballot(lane < kFxCache && fxc->k0[e] == ins_lo && fxc->k1[e] == tag);
    if (hit) ord = fxc->ord[__builtin_ctzll(hit)];
  }
  if (!hit) {
    ord = fx_order_packed(nk, ins_at);
    if (fxc && lane == 0) {
      const uint32_t e = fxc->next++ & (kFxCache - 1);
      fxc->k0[e] = ins_lo;
      fxc->k1[e] = tag;
      fxc->ord[e] = ord;
    }
  }
  uint64_t k_lo = 0, k_hi = 0, k_ins = 0;  // k_ins: nibble j = insertion index of output key j
  uint32_t m = 0;
  const bool drop_wc = wc >= 0 && nk > 1;
  for (uint32_t k = 0; k < nk; ++k) {
    const uint32_t s = ins_at(nib(ord, k));
    if (drop_wc && s == (uint32_t)(uint8_t)wc) continue;
    if (m < 8) k_lo |= (uint64_t)s << (8 * m);
    else k_hi |= (uint64_t)s << (8 * (m - 8));
    k_ins |= (uint64_t)nib(ord, k) << (4 * m);
    m++;
  }
  auto key_at = [&](uint32_t j) { return j < 8 ? byte_at(k_lo, j) : byte_at(k_hi, j - 8); };
  VOTE_T(29);
  // 3. per-key sums; lane k keeps key k's running sum
  double accv = 0.0;
  // Unweighted votes: a read adds occ/split (tips) to each of its symbols.
  // They are counted exactly, in units of 1/U of a read, lane-parallel per
  // key (ballot counts where every voter nominates one symbol, else a wave
  // sum of each lane's units): U = 8 while every split is 1, 2, 4 or 8 (all
  // partial sums of the reference's f64 fold are then exact too, < 2^50, so
  // the count is its value), U = 840 = lcm(1..8) from the first split of 3,
  // 5, 6 or 7 on. The fold of such terms rounds, but every decision taken on
  // the votes compares two of them, or one with min_count (the
  // min(min_count, max) thresholds, the order of the split candidates):
  // distinct counts are at least 1/840 apart and the fold's error is below
  // 2^-40, so the counts decide alike unless two compared quantities are
  // exactly equal. Then, and for splits above 8 or min_af > 0 (the ceil of a
  // rounded sum), every key takes the ordered fold below.
  bool fold = weighted;
  if (single_sym) {
    // output key j (lane j) gets the read count of its insertion index
    const uint32_t src = (uint32_t)lane < m ? nib(k_ins, (uint32_t)lane) : 0u;
    const uint32_t c = (uint32_t)__shfl((int)cins, (int)src, 64);
    accv = (uint32_t)lane < m ? (double)c : 0.0;
  } else if (!weighted) {
    uint32_t U = 8u, cu = 0;  // lane k: key k's count in units of 1/U
    for (uint32_t base = 0; base < n && !fold; base += 64) {
      const uint32_t r = base + lane;
      RInfoReg x = {0, 0, kInactive, 0, make_uint4(0, 0, 0, 0)};
      if (r < n) x = load(r);
      const bool voter = x.e != kInactive;
      const bool mul = voter && x.n >= 2;
      const uint32_t s0 = voter && x.n == 1 ? byte_at(x.sym, 0) : 0x100u;
      if (!ballot(mul)) {
        for (uint32_t k = 0; k < m; ++k) {
          const uint32_t cnt = (uint32_t)__popcll((unsigned long long)ballot(s0 == key_at(k)));
          if ((uint32_t)lane == k) cu += U * cnt;
        }
        continue;
      }
      if (ballot(mul && x.split > 8u)) {
        fold = true;
        break;
      }
      if (U == 8u && ballot(mul && (x.split & (x.split - 1u)))) {
        if (!odd_ok) {
          fold = true;
          break;
        }
        U = 840u;
        cu *= 105u;
      }
      const uint32_t per = mul ? U / x.split : 0u;
      // this lane's symbol slots j < x.n of a multi-symbol read (byte high bits)
      constexpr uint64_t kHi = 0x8080808080808080ull, kOnes = 0x0101010101010101ull;
      const uint64_t slots = !mul ? 0ull : (x.n >= 8u ? kHi : kHi & ((1ull << (8u * x.n)) - 1ull));
      // units of key k on this lane: U for its one symbol, occ * U / split
      // for the slot holding it (a read's symbols are distinct)
      auto units = [&](uint32_t key) -> uint32_t {
        const uint64_t eq = slots & ~nz_bytes(x.sym ^ (kOnes * key));
        return s0 == key ? U : (eq ? occ_at(x.occ, (uint32_t)__builtin_ctzll(eq) >> 3) * per : 0u);
      };
      // two keys per wave sum: a key's units over 64 lanes stay below 2^16
      for (uint32_t k = 0; k < m; k += 2) {
        const uint32_t u = units(key_at(k)) | (k + 1 < m ? units(key_at(k + 1)) << 16 : 0u);
        const uint32_t t = wave_sum_u32(u);  // (the whole wave runs the votes)
        if ((uint32_t)lane == k) cu += t & 0xFFFFu;
        if ((uint32_t)lane == k + 1) cu += t >> 16;
      }
    }
    if (!fold && U != 8u) {  // exact ties (two keys, or a key and min_count): the f64 fold decides
      for (uint32_t k = 0; k < m && !fold; ++k) {
        const uint32_t ck = (uint32_t)__builtin_amdgcn_readlane((int)cu, (int)k);
        fold = __popcll((unsigned long long)ballot((uint32_t)lane < m && cu == ck)) > 1 || (uint64_t)ck == 840ull * mc;
      }
    }
    if (!fold) accv = (uint32_t)lane < m ? (double)cu / (double)U : 0.0;
  }
  // contributions computed lane-parallel (one read per lane), then folded
  // strictly in read order (the reference's f64 summation order); a read
  // without the key adds nothing (x + 0.0 == x, so skipping it is exact)
  auto fold_into = [&](double& acc_io) {
    for (uint32_t base = 0; base < n; base += 64) {
      const uint32_t r = base + lane;
      RInfoReg x = {0, 0, kInactive, 0, make_uint4(0, 0, 0, 0)};
      if (r < n) x = load(r);
      double w = 0.0;
      if (x.e != kInactive) w = weighted ? weight(r) : 1.0;
      const bool voter = w > 0.0;
      const double dsplit = (double)x.split;
      for (uint32_t k = 0; k < m; ++k) {
        const uint32_t key = key_at(k);
        uint32_t occ = 0;
        if (voter)
          for (uint32_t j = 0; j < x.n; ++j)
            if (byte_at(x.sym, j) == key) {
              occ = occ_at(x.occ, j);
              break;
            }
        const double c = occ ? w * (double)occ / dsplit : 0.0;
        // runs of exact 1.0 contributions are added in closed form
        // (add_ones); every other contribution is added one at a time
        const uint64_t ones = ballot(occ != 0 && c == 1.0);
        uint64_t frac = ballot(occ != 0 && c != 1.0);
        double acc = readlane_f64(acc_io, (int)k);
        uint64_t done = 0;
        while (frac) {
          const int l = __builtin_ctzll(frac);
          frac &= frac - 1;
          const uint64_t below = (1ull << l) - 1ull;
          acc = add_ones(acc, (uint32_t)__popcll((unsigned long long)(ones & below & ~done)));
          done = below | (1ull << l);
          acc += readlane_f64(c, l);
        }
        acc = add_ones(acc, (uint32_t)__popcll((unsigned long long)(ones & ~done)));
        if ((uint32_t)lane == k) acc_io = acc;
      }
    }
  };
  if (fold) {
    fold_into(accv);
  }
#ifdef WC_VOTE_XCHECK
  // (diagnostic build) the exact counts against the reference's ordered fold:
  // distinct counts are >= 1/840 apart, the fold's rounding error < 2^-40
  else if (!weighted) {
    double accf = 0.0;
    fold_into(accf);
    const bool bad = (uint32_t)lane < m && fabs(accf - accv) > 1e-9;
    const uint64_t bm = ballot(bad);
    if (bm && lane == __builtin_ctzll(bm))
      printf("[wc-xcheck] votes: wg %u wave %u n %u m %u key %u exact %.17g fold %.17g single %d\n", blockIdx.x,
             threadIdx.x >> 6, n, m, key_at((uint32_t)lane), accv, accf, (int)single_sym);
  }
#endif
  VOTE_T(30);
#undef VOTE_T
  m_out = m;
  key_out = (uint32_t)lane < m ? key_at(lane) : 0u;
  val_out = accv;
  return true;
}


WC_PHASE_FN bool wave_votes(Lo<Ctl>& ctl, uint32_t side, const Sh<RInfo>* ri, const Sh<RInfo>* r0, const Sh<RInfo>* r1,
                                  uint32_t n, bool weighted, bool is_dual, bool multi, int wc, uint64_t mc, bool odd_ok) {
  const int lane = lane_id();
  const bool side1 = side == 0;
  uint32_t m = 0, key = 0;
  double val = 0.0;
  const bool ok = wave_votes_core([&](uint32_t r) { return rinfo_load(&ri[r]); },
                                  [&](uint32_t r) { return vote_weight(r0, r1, r, is_dual, side1); }, n, weighted,
                                  multi, wc, mc, odd_ok, m, key, val,
#ifdef WC_PHASE_PROF
                                  ctl.ph,
#else
                                  nullptr,
#endif
#ifdef WC_NO_FXCACHE
                                  nullptr);
#else
                                  &ctl.fxc[side]);
#endif
  if (!ok) return false;
  if ((uint32_t)lane < m) {
    ctl.keys[side][lane] = (uint8_t)key;
    ctl.vals[side][lane] = val;
  }
  if (lane == 0) ctl.nkeys[side] = m;
  PH_MARK(12);
  return true;
}

#include "chain.hip.hpp"
#include "dual_chain.hip.hpp"

// ---- write one result record (finalized node) ----
WC_PHASE_FN void store_record(Eng& E, Lo<Ctl>& ctl, Gm<uint8_t>* outp, uint32_t slot, uint32_t nsides,
                                    uint32_t len0, uint32_t len1, bool is_dual) {
  const int tid = threadIdx.x;
  const uint64_t rb = result_bytes(E.sides, E.nmax, E.lcap);
  Gm<uint8_t>* rec = outp + 16 + (uint64_t)ctl.store_idx * rb;
  for (uint32_t s = 0; s < E.sides; ++s) {
    Gm<uint8_t>* rcon = rec + 16 + s * align16(E.lcap);
    Gm<uint32_t>* rfe = (Gm<uint32_t>*)(rec + 16 + E.sides * align16(E.lcap) + s * align16((uint64_t)E.nmax * 4));
    if (s < nsides) {
      SideView v = E.sv(slot, s);
      copy_bytes(rcon, v.con, s ? len1 : len0);  // both 16-byte aligned: 16-byte stores
    }
    for (uint32_t r = tid; r < E.n; r += kEB) rfe[r] = s < nsides ? E.L.fe[s * E.nmax + r] : kInactive;
  }
  if (tid == 0) {
    Gm<uint32_t>* h = (Gm<uint32_t>*)rec;
    h[0] = len0;
    h[1] = nsides > 1 ? len1 : 0;
    h[2] = is_dual ? 1u : 0u;
  }
}

__device__ inline void trace_pop(const EngineArgs& A, uint32_t prob, const HeapEntry& top, uint32_t flags,
                                 uint32_t extra) {
  if (!A.trace || prob != 0) return;
  const uint32_t k = A.trace[0];
  if (k >= A.trace_cap) return;
  uint32_t* rec = A.trace + 4 + 4 * k;
  rec[0] = (uint32_t)top.cost;
  rec[1] = top.len;
  rec[2] = flags;
  rec[3] = extra;
  A.trace[0] = k + 1;
}

__device__ inline void finish_problem(const EngineArgs& A, Lo<Ctl>& ctl, uint8_t* outp, uint32_t prob, uint32_t oslot) {
  // every wave's result-record stores complete (system scope) before the flag
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    // every tied result must have a record; otherwise rerun with more records
    if (ctl.status == ST_OK && ctl.n_ret > A.rmax) ctl.status = ST_RETRY | ST_RETRY_RMAX;
    ((uint32_t*)outp)[0] = min(ctl.n_ret, A.rmax);
    A.status[oslot] = ctl.status;
    for (int s = 0; s < S_NSTAT; ++s) A.stats[(uint64_t)oslot * S_NSTAT + s] = ctl.cnt[s];
#ifdef WC_PHASE_PROF
    if (A.phases)
      for (int k = 0; k < kPhases; ++k) atomicAdd(&A.phases[k], (unsigned long long)ctl.ph[k]);
#endif
    if (A.done) {
      // the host consumes this problem as soon as it sees the flag (while the
      // launch goes on): status, counters and records first, then the flag
      __threadfence_system();
      __hip_atomic_store(&A.done[oslot], A.stream ? prob + 1 : 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  __syncthreads();
}

// ---- DualConsensusDWFA: build every child of the popped node ----
// (dual_consensus.rs:554-734: per child a clone, activate_dual :957-976, the
// pushes :915-946, activation :633-639, prune_dwfa :1030-1045 and the
// priority :1092-1168.) The children of one node are independent: each has
// its own slot, and the clones copy the parent before the in-place child (the
// last one) changes it. So each step runs over up to kNCB children in one
// block-wide pass, and a group of children costs the latency of one.
// kDH (dual_hot): the popped node's RStates are the LDS copy (Lds::hot); the
// clones copy them into their slots, the in-place child is pushed there.
// the dual pushes' grouped ED increases (group_edinc): 8-lane groups, eight
// reads per wave, for rows of at most 64 entries; longer rows one read per
// wave (wave_heavy). Measured on cfg3 (200 reads, one box): 16-lane groups
// (four reads per wave, rows to 128) 214 loci/s, 8-lane groups 233; on
// another box 8-lane groups 216 against 212-215 for spreading each round's
// items evenly over the waves, 16-lane groups for the rows of 65-128 entries,
// or both, and 4-lane groups (16 reads per wave, rows to 32) 220 vs 233.
constexpr uint32_t kRowPush = 8u * kQ16;

template <bool kDH>
__device__ inline void dual_build_children(Eng& E, Lo<Ctl>& ctl, uint32_t top, const SlotMeta& tm, bool tdual,
                                           uint32_t nc) {
  const int tid = threadIdx.x, lane = lane_id();
  const DevConfig& cfg = E.cfg;
  const bool early = cfg.early != 0;
  const uint32_t n = E.n;
  for (uint32_t c0 = 0; c0 < nc; c0 += kNCB) {
    const uint32_t cn = min(kNCB, nc - c0);
    // slots in the reference's child order (clones first, the last child in
    // place), then every child's new symbols, locks and lengths: the new
    // consensus bytes sit past the copied prefix, so they go in before the copies
    if (tid == 0) {
      for (uint32_t c = c0; c < c0 + cn; ++c) {
        uint32_t slot = top;
        if (c + 1 < nc) {
          if (ctl.nfree == 0) {
            ctl.status = ST_RETRY | ST_RETRY_PCAP;
            break;
          }
          slot = E.L.freestack[WC_IX(--ctl.nfree, E.pcap)];
        }
        ctl.ch_slot[c] = slot;
        ctl.ch_cost[c] = 0;
        ctl.ch_some[c - c0][0] = ctl.ch_some[c - c0][1] = 0;
        const uint32_t kind = ctl.ch_kind[c];
        SlotMeta m = tm;
        if (kind == 2) {  // activate_dual
          m.flags |= 1u;
          m.len[1] = m.len[0];
          m.nsome[1] = m.nsome[0];
        }
#pragma unroll
        for (int sd = 0; sd < 2; ++sd) {
          const int sym = ctl.ch_s[c][sd];
          if (sym >= 0) {
            E.sv(slot, sd).con[WC_IX(m.len[sd], E.lcap)] = (uint8_t)sym;
            m.len[sd]++;
          } else if (kind == 0) {
            m.flags |= (sd == 0 ? 2u : 4u);  // lock_sequence
          }
        }
        meta_put(E.L.meta[slot], m);
      }
      ctl.nheavy = 0;
      ctl.nwide = 0;
      con_store_wait();  // (the children's consensus bytes: the ED increases below read them)
    }
    __syncthreads();
    if (uni(ctl.status) != ST_OK) return;
    // clones copy the parent (every side it has); activate_dual copies side 1
    // into side 2, straight from the parent (a split child's parent is single,
    // so the in-place child's side 2 is not read by any clone)
    for (uint32_t c = c0; c < c0 + cn; ++c) {
      const uint32_t slot = WC_IX(uni(ctl.ch_slot[c]), E.pcap);
      if (slot != top) {
        copy_side<kDH, false, true>(E, top, 0, slot, 0, tm.len[0]);
        if (tdual) copy_side<kDH, false, true>(E, top, 1, slot, 1, tm.len[1]);
      }
      if (uni((uint32_t)ctl.ch_kind[c]) == 2) {
        if (kDH && slot == top) copy_side<true, true, true>(E, top, 0, top, 1, tm.len[0]);
        else copy_side<kDH, false, true>(E, top, 0, slot, 1, tm.len[0]);
      }
    }
    __syncthreads();
    PH_MARK(4);
    // pushes: every (child, side) that appends a symbol, thread per read.
    // Reads that need the ED-increase loop go to the group list (rows that fit
    // kRow16, eight or four reads per wave) or, for wide frontiers and long
    // rows, to the wave list (filled from the top of E.L.list)
    const uint32_t lend = (uint32_t)list_entries(2, E.nmax) - 1;
    WaveCounters tc = {0, 0, 0, 0, 0, 0};
    for (uint32_t q = 0; q < 2 * cn; ++q) {
      const uint32_t c = c0 + q / 2, sd = q & 1u;
      const int sym = uni((int32_t)ctl.ch_s[c][sd]);
      Sh<uint16_t>* ceq = E.L.ce + (uint64_t)q * E.nmax;
      if (sym < 0) {
        // a side this child does not push keeps the parent's edit distances
        // (a locked side of a dual child); a single child has no side 1
        const bool keep = tdual;
        const Sh<RInfo>* par = E.L.rinfo + (sd ? E.nmax : 0u);  // the parent's analysis of this side
        for (uint32_t r = tid; r < n; r += kEB) ceq[r] = ce16(keep ? par[r].e : kInactive);
        continue;
      }
      const uint32_t slot = WC_IX(uni(ctl.ch_slot[c]), E.pcap);
      const uint32_t olen = uni(E.L.meta[slot].len[sd]);
      SideView v = E.sv(slot, sd);
      // the in-place child's RStates: the LDS copy (kDH), else its slot
      auto push_pass = [&](auto rsb) {
      for (uint32_t base = 0; base < n; base += kEB) {
        const uint32_t r = base + tid;
        uint32_t kind = 0;  // 1: group list, 2: wave list
        if (r < n) {
          const RRaw s = rstate_load(&rsb[r]);
          if (rraw_e(s) == kInactive) ceq[r] = (uint16_t)kCeNone;
          if (rraw_e(s) != kInactive) {
            if (rraw_flags(s) & kWide) {  // frontier too wide for the register path
              kind = 2;
            } else {
              Front f;
              front_load(s, f);
              uint32_t cmp = 0;
              const bool heavy = thread_push(f, GlobalBytes{E.read(r)}, E.rlen(r), olen - 1, (uint8_t)sym,
                                             cfg.wildcard, early, v.wf + (uint64_t)r * E.wcap, cmp);
              tc.compares += cmp;
              front_store(&rsb[r], f);
              if (heavy) {
                const uint32_t w2 = 2 * f.e + 3;
                kind = w2 <= kRowPush ? 1u : 2u;
              } else {
                tc.updates++;
                tc.w_out += 2 * f.e + 1;
                ceq[r] = ce16(f.e);
              }
            }
          }
        }
        const uint32_t kg = agg_append(&ctl.nheavy, kind == 1);
        const uint32_t kw = agg_append(&ctl.nwide, kind == 2);
        if (kind == 1) E.L.list[WC_IX(kg, list_entries(E.sides, E.nmax))] = q * n + r;
        if (kind == 2) E.L.list[WC_IX(lend - kw, list_entries(E.sides, E.nmax))] = q * n + r;
      }
      };
      if constexpr (kDH) push_pass(slot == top ? rs_generic(E.L.hot + sd * E.nmax) : rs_generic(v.rs));
      else push_pass(v.rs);
    }
    flush_thread_counters(ctl, tc);
    __syncthreads();
    PH_MARK(5);
    // the ED-increase loops: eight reads per wave in 8-lane groups ...
    const uint32_t nh = uni(ctl.nheavy), nw = uni(ctl.nwide);
    if (nh + nw) l1_drop();  // (they read the children's consensus bytes; con_store_wait above)
    SUB_CNT(16, nh);
    SUB_CNT(17, nw);
    SUB_T0(tg);
    WaveCounters cnt = {0, 0, 0, 0, 0, 0};
    GroupCnt gc = {0, 0, 0, 0, 0};
    // (up to one item per wave the 64-lane path is quicker: it goes to the wave loop)
    const uint32_t ng = nh > (uint32_t)kEW ? nh : 0u;
    // (8-lane groups: eight reads per wave, rows of at most kRowPush entries)
    constexpr uint32_t G = 8u;
    for (uint32_t b0 = wave_id() * (64u / G); b0 < ng; b0 += kEW * (64u / G)) {
      const uint32_t k = b0 + ((uint32_t)lane / G);
      const bool act = k < ng;
      const uint32_t it = act ? E.L.list[WC_IX(k, list_entries(E.sides, E.nmax))] : 0u;
      const uint32_t q = it / n, r = it - q * n;
      const uint32_t c = c0 + q / 2, sd = q & 1u;
      const uint32_t slot = ctl.ch_slot[c];
      SideView v = E.sv(slot, sd);
      GroupOut go;
      if constexpr (kDH) {
        const RSg rp = slot == top ? rs_generic(E.L.hot + sd * E.nmax + r) : rs_generic(&v.rs[r]);
        go = group_edinc<G>(act, rp, v.wf + (uint64_t)r * E.wcap, E.read(r), E.rlen(r), v.con, E.L.meta[slot].len[sd],
                         cfg.wildcard, early, E.wcap);
      } else {
        go = group_edinc<G>(act, &v.rs[r], v.wf + (uint64_t)r * E.wcap, E.read(r), E.rlen(r), v.con,
                         E.L.meta[slot].len[sd], cfg.wildcard, early, E.wcap);
      }
      const uint32_t g = go.st, e = go.e;
      if (act && (lane & (G - 1)) == 0 && g == kG_DONE) E.L.ce[WC_IX((uint64_t)q * E.nmax + r, (uint64_t)2 * kNCB * E.nmax)] = ce16(e);
      gc.edinc += go.edinc;
      gc.updates += go.updates;
      gc.w_out += go.w_out;
      gc.cmp += go.cmp;
      gc.rowb += go.rowb;
      if (act && (lane & (G - 1)) == 0 && g == kG_WCAP) atomicOr(&ctl.ovf, 4u);
      // ... a row that outgrew the group finishes with the whole wave
      uint64_t mem = ballot(act && (lane & (G - 1)) == 0 && g == kG_MEM);
      while (mem) {
        const int src = __builtin_ctzll(mem);
        mem &= mem - 1;
        const uint32_t it2 = (uint32_t)__builtin_amdgcn_readlane((int)it, src);
        const uint32_t e2 = (uint32_t)__builtin_amdgcn_readlane((int)e, src);
        const uint32_t q2 = it2 / n, r2 = it2 - q2 * n;
        const uint32_t c2 = c0 + q2 / 2, sd2 = q2 & 1u;
        SUB_CNT(18, 1);
        const uint32_t slot2 = uni(ctl.ch_slot[c2]);
        SideView v2 = E.sv(slot2, sd2);
        uint32_t eo = 0;
        bool okm;
        if constexpr (kDH) {
          const RSg rp = slot2 == top ? rs_generic(E.L.hot + sd2 * E.nmax + r2) : rs_generic(&v2.rs[r2]);
          okm = wave_edinc_mem(rp, v2.wf + (uint64_t)r2 * E.wcap, e2, E.read(r2), E.rlen(r2), v2.con,
                               uni(E.L.meta[slot2].len[sd2]), cfg.wildcard, early, E.wcap, cnt, eo);
        } else {
          okm = wave_edinc_mem(&v2.rs[r2], v2.wf + (uint64_t)r2 * E.wcap, e2, E.read(r2), E.rlen(r2), v2.con,
                               uni(E.L.meta[slot2].len[sd2]), cfg.wildcard, early, E.wcap, cnt, eo);
        }
        if (!okm) {
          if (lane == 0) atomicOr(&ctl.ovf, 4u);
        } else if (lane == 0) {
          E.L.ce[WC_IX((uint64_t)q2 * E.nmax + r2, (uint64_t)2 * kNCB * E.nmax)] = ce16(eo);
        }
      }
    }
    SUB_T1(19, tg);
    SUB_T0(tw);
    cnt.edinc += wave_sum_u32(gc.edinc);
    cnt.updates += wave_sum_u32(gc.updates);
    cnt.w_out += wave_sum_u32(gc.w_out);
    cnt.compares += wave_sum_u32(gc.cmp);
    cnt.rowb += wave_sum_u32(gc.rowb);
    // ... and wide frontiers / long rows (and a few group items) one read per wave
    const uint32_t nsolo = nw + (nh - ng);
    for (uint32_t k = wave_id(); k < nsolo; k += kEW) {
      const uint32_t it = uni(k < nw ? E.L.list[WC_IX(lend - k, list_entries(E.sides, E.nmax))] : E.L.list[WC_IX(k - nw, list_entries(E.sides, E.nmax))]);
      const uint32_t q = it / n, r = it - q * n;
      const uint32_t c = c0 + q / 2, sd = q & 1u;
      const uint32_t slot = WC_IX(uni(ctl.ch_slot[c]), E.pcap);
      SideView v = E.sv(slot, sd);
      uint32_t e = 0;
      bool okh;
      if constexpr (kDH) {
        const RSg rp = slot == top ? rs_generic(E.L.hot + sd * E.nmax + r) : rs_generic(&v.rs[r]);
        okh = wave_heavy(rp, v.wf + (uint64_t)r * E.wcap, E.read(r), E.rlen(r), v.con, uni(E.L.meta[slot].len[sd]),
                         (uint8_t)uni((int32_t)ctl.ch_s[c][sd]), cfg.wildcard, early, E.wcap, cnt, e);
      } else {
        okh = wave_heavy(&v.rs[r], v.wf + (uint64_t)r * E.wcap, E.read(r), E.rlen(r), v.con,
                         uni(E.L.meta[slot].len[sd]), (uint8_t)uni((int32_t)ctl.ch_s[c][sd]), cfg.wildcard, early,
                         E.wcap, cnt, e);
      }
      if (!okh) {
        if (lane == 0) atomicOr(&ctl.ovf, 4u);
      } else if (lane == 0) {
        E.L.ce[WC_IX((uint64_t)q * E.nmax + r, (uint64_t)2 * kNCB * E.nmax)] = ce16(e);
      }
    }
    SUB_T1(20, tw);
    flush_counters(ctl, cnt);
    __syncthreads();
    PH_MARK(6);
    // reads whose offset activates at a child's new max length
    // (dual_consensus.rs:633-639): consensus 1 always, consensus 2 too when dual
    bool activated = false;  // (uniform) then the prune pass reads the slots, not ce
    for (uint32_t c = c0; c < c0 + cn; ++c) {
      const uint32_t slot = WC_IX(uni(ctl.ch_slot[c]), E.pcap);
      const uint32_t nl0 = uni(E.L.meta[slot].len[0]), nl1 = uni(E.L.meta[slot].len[1]);
      if (max(nl0, nl1) > E.P.max_act) continue;
      if (!activated && nh + nw == 0) l1_drop();  // (activation reads the new consensus bytes too)
      activated = true;
      if (kDH && slot == top) {
        activate_side<true>(E, ctl, slot, 0, nl0, max(nl0, nl1), false, nullptr);
        if (uni(E.L.meta[slot].flags) & 1u) activate_side<true>(E, ctl, slot, 1, nl1, max(nl0, nl1), false, nullptr);
      } else {
        activate_side<false>(E, ctl, slot, 0, nl0, max(nl0, nl1), false, nullptr);
        if (uni(E.L.meta[slot].flags) & 1u) activate_side<false>(E, ctl, slot, 1, nl1, max(nl0, nl1), false, nullptr);
      }
    }
    PH_MARK(10);
    // prune + priority of every child of the group in one pass; every
    // child's edit distances are loaded before any is used
    SUB_T0(tp0);
    uint32_t cslot[kNCB], cdual = 0;
#pragma unroll
    for (uint32_t k = 0; k < kNCB; ++k) {
      cslot[k] = k < cn ? uni(ctl.ch_slot[c0 + k]) : 0u;
      if (k < cn && (uni(E.L.meta[cslot[k]].flags) & 1u)) cdual |= 1u << k;
    }
    SUB_T1(22, tp0);
    SUB_T0(tp1);
    // edit distances from the slots when an activation changed them, or when
    // they might not fit the u16 array (wavefront rows past 2^17 entries)
#ifdef WC_NO_CE  // (diagnostic variant: the prune pass reads every edit distance from the slots)
    const bool slot_e = true;
#else
    const bool slot_e = activated || E.wcap > 2u * kCeNone;
#endif
    uint64_t ccost[kNCB] = {0, 0, 0, 0};
    uint32_t cn0[kNCB] = {0, 0, 0, 0}, cn1[kNCB] = {0, 0, 0, 0};
    // child k's RState of read r on side sd (kDH: the in-place child's is the LDS copy)
    auto crs_e = [&](uint32_t k, uint32_t sd, uint32_t r) -> auto& {
      if constexpr (kDH)
        return (cslot[k] == top ? rs_generic(&E.L.hot[sd * E.nmax + r]) : rs_generic(&E.sv(cslot[k], sd).rs[r]))->e;
      else return E.sv(cslot[k], sd).rs[r].e;
    };
    for (uint32_t r = tid; r < n; r += kEB) {
      uint32_t e1[kNCB], e2[kNCB];
#pragma unroll
      for (uint32_t k = 0; k < kNCB; ++k) {
        e1[k] = e2[k] = kInactive;
        if (k < cn) {
          // each child's edit distances as its pushes left them (LDS), or
          // from its slot when an activation changed them
          e1[k] = slot_e ? crs_e(k, 0, r) : ce32(E.L.ce[WC_IX((uint64_t)(2 * k) * E.nmax + r, (uint64_t)2 * kNCB * E.nmax)]);
          if (cdual & (1u << k))
            e2[k] = slot_e ? crs_e(k, 1, r) : ce32(E.L.ce[WC_IX((uint64_t)(2 * k + 1) * E.nmax + r, (uint64_t)2 * kNCB * E.nmax)]);
        }
      }
#pragma unroll
      for (uint32_t k = 0; k < kNCB; ++k) {
        if (k >= cn) continue;
        if ((cdual & (1u << k)) && e1[k] != kInactive && e2[k] != kInactive) {
          if ((uint64_t)e1[k] + cfg.dual_max_ed_delta < (uint64_t)e2[k]) {
            crs_e(k, 1, r) = kInactive;
            e2[k] = kInactive;
          } else if ((uint64_t)e2[k] + cfg.dual_max_ed_delta < (uint64_t)e1[k]) {
            crs_e(k, 0, r) = kInactive;
            e1[k] = kInactive;
          }
        }
        uint64_t best = ~0ull;
        if (e1[k] != kInactive) best = cost_of(e1[k], cfg.cost_mode);
        if (e2[k] != kInactive && cost_of(e2[k], cfg.cost_mode) < best) best = cost_of(e2[k], cfg.cost_mode);
        if (best != ~0ull) ccost[k] += best;
        cn0[k] += e1[k] != kInactive;
        cn1[k] += e2[k] != kInactive;
      }
    }
    SUB_T1(23, tp1);
    SUB_T0(tp2);
#pragma unroll
    for (uint32_t k = 0; k < kNCB; ++k) {
      if (k >= cn) continue;
      agg_add64(&ctl.ch_cost[c0 + k], ccost[k]);
      agg_add(&ctl.ch_some[k][0], cn0[k]);
      agg_add(&ctl.ch_some[k][1], cn1[k]);
    }
    SUB_T1(24, tp2);
    SUB_T0(tp3);
    __syncthreads();
    SUB_T1(25, tp3);
    SUB_T0(tp4);
    if (tid == 0) {
      if (ctl.ovf & 16u) ctl.status = WC_E_INVARIANT_CODE;
      else if (ctl.ovf & 4u) ctl.status = ST_RETRY | ST_RETRY_WCAP;
      else if (ctl.ovf) ctl.status = limit_status(ctl.ovf);
      for (uint32_t c = c0; c < c0 + cn; ++c) {
        auto& m = E.L.meta[ctl.ch_slot[c]];
        m.nsome[0] = ctl.ch_some[c - c0][0];
        m.nsome[1] = ctl.ch_some[c - c0][1];
        ctl.ch_len[c] = max(m.len[0], m.len[1]);
      }
    }
    __syncthreads();
    SUB_T1(26, tp4);
    PH_MARK(11);
    if (uni(ctl.status) != ST_OK) return;
  }
}

// single-engine phases out of line (see WC_SINGLE_FN)
WC_SINGLE_FN WaveCounters single_finalize(Eng& E, Lo<Ctl>& ctl, uint32_t top, uint32_t len) {
  WaveCounters cnt = {0, 0, 0, 0, 0, 0};
  finalize_side<true>(E, ctl, top, 0, len, E.L.fe, cnt);
  return cnt;
}
WC_SINGLE_FN bool single_votes(Lo<Ctl>& ctl, Sh<RInfo>* ri, uint32_t n, bool multi, int wc, uint64_t mc) {
  return wave_votes(ctl, 0, ri, ri, ri, n, false, false, multi, wc, mc, true);
}
WC_SINGLE_FN void single_store(Eng& E, Lo<Ctl>& ctl, Gm<uint8_t>* outp, uint32_t top, uint32_t len) {
  store_record(E, ctl, outp, top, 1, len, 0, false);
}
WC_SINGLE_FN void single_activate(Eng& E, Lo<Ctl>& ctl, uint32_t slot, bool hot, uint32_t len) {
  if (hot) activate_side<true>(E, ctl, slot, 0, len, len, true, E.L.rinfo);
  else activate_side<false>(E, ctl, slot, 0, len, len, true, E.L.rinfo);
}

// =====================================================================
// ConsensusDWFA engine (consensus.rs:139-351)
// =====================================================================
#ifndef WC_DUAL_ONLY  // (engine_cu_dual.hip: the dual engine only)
__global__ void __launch_bounds__(kEB) __attribute__((amdgpu_waves_per_eu(WC_SINGLE_WAVES_PER_EU))) single_engine_kernel(EngineArgs A) {
  extern __shared__ __align__(16) uint8_t smem[];
  __shared__ Ctl ctl_lds;
  Lo<Ctl>& ctl = *(Lo<Ctl>*)&ctl_lds;
  const int tid = threadIdx.x;
  const int lane = lane_id();
  const DevConfig& cfg = A.cfg;
  const bool early = cfg.early != 0;
  Eng E = make_eng(A, state_base(A, smem));

  if (tid == 0) ctl.obuf = 1;
  for (;;) {
    uint32_t oslot = 0;
    const uint32_t prob = claim_problem(A, ctl, E, oslot);
    if (prob == ~0u) break;
    E.n = E.P.n_reads;
    Gm<uint8_t>* outp = (Gm<uint8_t>*)A.out + (uint64_t)oslot * A.out_stride;
    init_problem(E, ctl);

    for (;;) {
      // ---- pop (consensus.rs:224-251) ----
      if (tid == 0) {
        TrackerRef t = E.tracker(ctl, 0);
        ctl.cache_hit = 0;
        if (ctl.heap_n == 0) {
          ctl.action = 2;
        } else {
          ctl.cnt[S_PEAKQ] = max(ctl.cnt[S_PEAKQ], (uint64_t)ctl.heap_n);
          ctl.cnt[S_POPS]++;
          while ((ctl.trk_total[0] > cfg.max_queue_size || ctl.last_constraint[0] >= cfg.max_nodes_wo_constraint) &&
                 ctl.trk_thr[0] < ctl.farthest[0]) {
            t.increment_threshold();
            ctl.last_constraint[0] = 0;
          }
          HeapEntry top = heap_pop(E.L.heap, ctl.heap_n, E.pcap);
          t.remove(top.len);
          ctl.top_slot = top.slot;
          ctl.top_len = top.len;
          ctl.top_cost = top.cost;
          const bool at_cap = t.processed(top.len) >= t.cap;
          if (top.cost > ctl.max_err || top.len < ctl.trk_thr[0] || at_cap) {
            ctl.cnt[S_IGNORED]++;
            E.L.freestack[WC_IX(ctl.nfree++, E.pcap)] = top.slot;
            if (top.slot == ctl.hot_slot) ctl.hot_slot = kNoSlot;
            ctl.action = 1;
          } else {
            ctl.farthest[0] = max(ctl.farthest[0], (uint64_t)top.len);
            ctl.cnt[S_EXPLORED]++;
            ctl.last_constraint[0]++;
            t.process_unchecked(top.len);
            ctl.action = 0;
            ctl.cache_hit = top.slot == ctl.cache_slot;
            // the popped node's RStates move into LDS; the previous LDS
            // node (still queued) is written back to its slot first
            ctl.hot_prev = ctl.hot_slot;
            ctl.hot_load = top.slot != ctl.hot_slot;
            ctl.hot_slot = top.slot;
          }
          trace_pop(A, prob, top, ctl.action << 1, 0);
        }
        if (ctl.cache_hit) {
          ctl.n_end[0] = ctl.cache_nend;
          ctl.multi[0] = ctl.cache_multi;
        } else {
          ctl.n_end[0] = 0;
          ctl.multi[0] = 0;
        }
        ctl.cache_slot = kNoSlot;
        ctl.ovf = 0;
      }
      PH_MARK(13);
      __syncthreads();
      PH_MARK(0);
      if (uni(ctl.action) == 2) break;
      if (uni(ctl.action) == 1) continue;
      if (uni(ctl.status) != ST_OK) break;

      const uint32_t top = uni(ctl.top_slot);
      const uint32_t len = uni(ctl.top_len);
      if (uni(ctl.hot_load)) {
        // per read r the same thread stores then fetches: no barrier needed
        const uint32_t prev = uni(ctl.hot_prev);
        if (prev != kNoSlot) hot_store(E, prev, 0);
        hot_fetch(E, top, 0);
      }
      if (!uni(ctl.cache_hit)) analyze_side0<true>(E, ctl, top, len, E.L.rinfo);
      PH_MARK(1);
      if (tid == 0) {
        const uint32_t ne = ctl.n_end[0];
        ctl.reached = early ? (ne == E.n) : (ne > 0);  // consensus.rs:516-532
        if (ctl.ovf) ctl.status = limit_status(ctl.ovf);
      }
      __syncthreads();
      if (uni(ctl.status) != ST_OK) break;

      // ---- finalize a clone (consensus.rs:254-279) ----
      if (uni(ctl.reached)) {
        const WaveCounters cnt = single_finalize(E, ctl, top, len);
        flush_counters(ctl, cnt);
        __syncthreads();
        if (tid == 0) {
          ctl.store_idx = -1;
          if (ctl.ovf & 4u) {
            ctl.status = ST_RETRY | ST_RETRY_WCAP;
          } else {
            uint64_t total = 0;
            bool uninit = false;
            for (uint32_t r = 0; r < E.n; ++r) {
              if (E.L.fe[r] == kInactive) uninit = true;
              else total += cost_of(E.L.fe[r], cfg.cost_mode);
            }
            if (uninit) {
              ctl.status = 1;  // "Finalize called on DWFA that was never initialized."
            } else {
              if (total < ctl.max_err) {
                ctl.max_err = total;
                ctl.n_ret = 0;
              }
              if (total <= ctl.max_err && ctl.n_ret < cfg.max_return_size) {
                if (ctl.n_ret < A.rmax) ctl.store_idx = (int32_t)ctl.n_ret;
                ctl.n_ret++;
              }
            }
          }
        }
        __syncthreads();
        if (uni(ctl.status) != ST_OK) break;
        if (uni(ctl.store_idx) >= 0) {
          const uint32_t lens[2] = {len, 0};
          single_store(E, ctl, outp, top, lens[0]);
        }
        PH_MARK(2);
      }

      // ---- votes + child selection (consensus.rs:283-321) ----
      if (wave_id() == 0) {
        const bool ok = single_votes(ctl, E.L.rinfo, E.n, ctl.multi[0] != 0, cfg.wildcard, cfg.min_count);
        if (lane == 0) {
          if (!ok) {
            ctl.status = limit_status(LIM_VOTES);
          } else {
            double max_obs = 0.0;
            bool have = false;
            for (uint32_t k = 0; k < ctl.nkeys[0]; ++k) {
              if (!have || ctl.vals[0][k] >= max_obs) max_obs = ctl.vals[0][k];
              have = true;
            }
            if (!have) max_obs = (double)cfg.min_count;
            const double thr = fmin((double)cfg.min_count, max_obs);
            uint32_t nc = 0;
            for (uint32_t k = 0; k < ctl.nkeys[0]; ++k)
              if (ctl.vals[0][k] >= thr) {
                ctl.ch_s[nc][0] = ctl.keys[0][k];
                ctl.ch_s[nc][1] = -1;
                nc++;
              }
            ctl.nchild = nc;
          }
        }
      }
      __syncthreads();
      PH_MARK(3);
      if (uni(ctl.status) != ST_OK) break;
      const uint32_t nc = uni(ctl.nchild);
      if (nc == 0) {
        if (tid == 0) {
          if (len < E.P.max_act) {  // consensus.rs:303-305: coverage gap (the host formats the message)
            ctl.status = WC_E_COVERAGE_GAP_CODE;
            ((Gm<uint32_t>*)outp)[1] = len;
          }
          E.L.freestack[WC_IX(ctl.nfree++, E.pcap)] = top;
          ctl.hot_slot = kNoSlot;
        }
        __syncthreads();
        if (uni(ctl.status) != ST_OK) break;
        continue;
      }
      if (len + 1 > E.lcap) {
        if (tid == 0) ctl.status = ST_RETRY | ST_RETRY_LCAP;
        __syncthreads();
        break;
      }
      // ---- one child and nothing else queued: linear-chain run-ahead ----
      // (past the last activation point every read of this lineage is active)
      uint32_t plen = len;  // the expanded node's length (a chain that popped its last node moves it)
      if (nc == 1 && A.chain && uni(ctl.heap_n) == 0 && (E.P.n_active == E.n || len >= E.P.max_act)) {
#ifdef WC_CHAIN_REBUILD
        uint32_t jstar = run_chain_single_k(kernel_args(), E.P, state_base(A, smem), ctl, top, plen, uni((int32_t)ctl.ch_s[0][0]));
#else
        uint32_t jstar = run_chain_single(E, ctl, top, plen, uni((int32_t)ctl.ch_s[0][0]));
#endif
        PH_MARK(14);
        // a full chain that also popped its last node N_K (one child, no
        // queue): that child starts the next chain at once
        while (jstar && uni(ctl.chain_next)) {
          plen += jstar - 1;
          const int s1 = uni((int32_t)ctl.chain_sym);
#ifdef WC_CHAIN_REBUILD
          jstar = run_chain_single_k(kernel_args(), E.P, state_base(A, smem), ctl, top, plen, s1);
#else
          jstar = run_chain_single(E, ctl, top, plen, s1);
#endif
          PH_MARK(14);
          if (!jstar) {
            // the next chain did not start: N_K's one child is pushed literally below
            if (tid == 0) ctl.ch_s[0][0] = (int16_t)s1;
            __syncthreads();
          }
        }
        if (jstar) continue;
      }
      // ---- push every child: clones first, the last child in place ----
      for (uint32_t c = 0; c < nc; ++c) {
        if (tid == 0) {
          uint32_t slot = top;
          if (c + 1 < nc) {
            if (ctl.nfree == 0) ctl.status = ST_RETRY | ST_RETRY_PCAP;
            else slot = E.L.freestack[WC_IX(--ctl.nfree, E.pcap)];
          }
          ctl.cur_slot = slot;
          ctl.cost_acc = 0;
          ctl.n_end[0] = 0;
          ctl.multi[0] = 0;
        }
        __syncthreads();
        if (uni(ctl.status) != ST_OK) break;
        const uint32_t slot = uni(ctl.cur_slot);
        if (slot != top) copy_side<true>(E, top, 0, slot, 0, plen);
        if (tid == 0) {
          E.sv(slot, 0).con[plen] = (uint8_t)ctl.ch_s[c][0];
          con_store_wait();  // (the ED increases below read it)
        }
        __syncthreads();
        l1_drop();
        PH_MARK(4);
        // clones read the parent from LDS and write their own slot; the last
        // child is pushed in place on the LDS copy
        const int sym = uni((int32_t)ctl.ch_s[c][0]);
        if (slot != top) push_sides<true, false>(E, ctl, slot, sym, -1, plen + 1, 0, true, E.L.rinfo);
        else push_sides<true, true>(E, ctl, slot, sym, -1, plen + 1, 0, true, E.L.rinfo);
        // reads whose offset activates at this length (consensus.rs:327-335)
        if (plen + 1 <= E.P.max_act) {
          single_activate(E, ctl, slot, slot == top, plen + 1);
        }
        if (tid == 0) {
          if (ctl.ovf & 16u) ctl.status = WC_E_INVARIANT_CODE;
          else if (ctl.ovf & 4u) ctl.status = ST_RETRY | ST_RETRY_WCAP;
          else if (ctl.ovf) ctl.status = limit_status(ctl.ovf);
          ctl.ch_cost[c] = ctl.cost_acc;
          ctl.ch_slot[c] = slot;
          E.L.meta[slot].len[0] = plen + 1;
        }
        __syncthreads();
        if (uni(ctl.status) != ST_OK) break;
      }
      if (uni(ctl.status) != ST_OK) break;
      if (tid == 0) {
        TrackerRef t = E.tracker(ctl, 0);
        for (uint32_t c = 0; c < nc; ++c) {
          t.insert(plen + 1);
          heap_push(E.L.heap, ctl.heap_n, E.pcap, HeapEntry{ctl.ch_cost[c], plen + 1, ctl.ch_slot[c]});
        }
        // the last child's nominations are in LDS: reuse them if it is popped next
        ctl.cache_slot = ctl.ch_slot[nc - 1];
        ctl.cache_nend = ctl.n_end[0];
        ctl.cache_multi = ctl.multi[0];
      }
      __syncthreads();
      PH_MARK(7);
    }
    finish_problem(A, ctl, outp, prob, oslot);
  }
  stream_exit(A);
}
#endif  // WC_DUAL_ONLY

// =====================================================================
// DualConsensusDWFA engine (dual_consensus.rs:240-787)
// =====================================================================
// kDH (EngineArgs::dual_hot): the popped node's RStates (both sides) move into
// LDS (Lds::hot) and stay there while its in-place child is popped next; the
// previous hot node is written back to its slot when another node is popped.
template <bool kDH>
__device__ __forceinline__ void dual_main(const EngineArgs& A, uint8_t* smem, Lo<Ctl>& ctl) {
  const int tid = threadIdx.x;
  const int lane = lane_id();
  const DevConfig& cfg = A.cfg;
  const bool early = cfg.early != 0;
  const bool weighted = cfg.weighted != 0;
  Eng E = make_eng(A, state_base(A, smem));
  Sh<RInfo>* R0 = E.L.rinfo;
  Sh<RInfo>* R1 = E.L.rinfo + E.nmax;

  if (tid == 0) ctl.obuf = 1;
  for (;;) {
    uint32_t oslot = 0;
    const uint32_t prob = claim_problem(A, ctl, E, oslot);
    if (prob == ~0u) break;
    E.n = E.P.n_reads;
    Gm<uint8_t>* outp = (Gm<uint8_t>*)A.out + (uint64_t)oslot * A.out_stride;
    init_problem(E, ctl);
    if (tid == 0) ctl.top_dual = 0;  // (no stashed child from the last problem)
    const uint64_t full_min = max(cfg.min_count, ceil_u64(cfg.min_af * (double)E.n));

    for (;;) {
      // ---- pop (dual_consensus.rs:340-397) ----
      if (tid == 0) {
        if (ctl.heap_n == 0) {
          ctl.action = 2;
        } else {
          // the node to pop is heap[0] already (or the stashed in-place
          // child): its HBM-resident counts (processed per length of both
          // trackers, active_min) are loaded first, under one wait, while the
          // threshold walk and the sift run
          const bool stashed = ctl.top_dual == kTopStashed;
          const uint32_t plen = stashed ? ctl.top_len : E.L.heap[0].len;
          const uint32_t pc_pre[2] = {E.tracker(ctl, 0).processed(plen), E.tracker(ctl, 1).processed(plen)};
          const uint64_t am_pre = plen < ctl.am_len ? E.active_min[WC_IX(plen, E.lcap + 2)] : 0;
          ctl.cnt[S_PEAKQ] = max(ctl.cnt[S_PEAKQ], (uint64_t)ctl.heap_n);
          ctl.cnt[S_POPS]++;
          for (int k = 0; k < 2; ++k) {
            TrackerRef t = E.tracker(ctl, k);
            while ((ctl.trk_total[k] > cfg.max_queue_size || ctl.last_constraint[k] >= cfg.max_nodes_wo_constraint) &&
                   ctl.trk_thr[k] < ctl.farthest[k]) {
              t.increment_threshold();
              ctl.last_constraint[k] = 0;
            }
          }
          HeapEntry top;
          if (stashed) {
            top = HeapEntry{ctl.top_cost, ctl.top_len, ctl.top_slot};
            ctl.heap_n--;
          } else {
            top = heap_pop(E.L.heap, ctl.heap_n, E.pcap);
          }
          const auto& m = E.L.meta[top.slot];
          const uint32_t dual = m.flags & 1u;
          TrackerRef t = E.tracker(ctl, dual);
          t.remove(top.len);
          ctl.top_slot = top.slot;
          ctl.top_len = top.len;
          ctl.top_cost = top.cost;
          ctl.top_dual = dual;
          const uint64_t am = am_pre;
          const bool imbalanced = dual && (m.nsome[0] < am || m.nsome[1] < am);
          if (top.len >= ctl.am_len) ctl.status = WC_E_INVARIANT_CODE;
          const bool at_cap = pc_pre[dual] >= t.cap;
          if (top.cost > ctl.max_err || top.len < ctl.trk_thr[dual] || at_cap || imbalanced) {
            ctl.cnt[S_IGNORED]++;
            E.L.freestack[WC_IX(ctl.nfree++, E.pcap)] = top.slot;
            if (kDH && top.slot == ctl.hot_slot) ctl.hot_slot = kNoSlot;  // its LDS state is dropped
            ctl.action = 1;
          } else {
            ctl.farthest[dual] = max(ctl.farthest[dual], (uint64_t)top.len);
            ctl.last_constraint[dual]++;
            t.process_unchecked(top.len);
            ctl.cnt[S_EXPLORED]++;
            ctl.action = 0;
            if (kDH) {
              // the popped node moves into LDS unless it is there already
              // (the in-place child of the previous pop); the previous hot
              // node (still queued) goes back to its slot first
              ctl.hot_prev = ctl.hot_slot;
              ctl.hot_load = top.slot != ctl.hot_slot;
              ctl.hot_prev_dual = ctl.hot_slot != kNoSlot && (E.L.meta[ctl.hot_slot].flags & 1u) != 0;
              ctl.hot_slot = top.slot;
            }
          }
          trace_pop(A, prob, top, dual | (ctl.action << 1) | (m.nsome[0] << 8) | (m.nsome[1] << 20), (uint32_t)am);
        }
        ctl.n_end[0] = ctl.n_end[1] = 0;
        ctl.multi[0] = ctl.multi[1] = 0;
        ctl.n_either = 0;
        ctl.nheavy = 0;
        ctl.ovf = 0;
      }
      __syncthreads();
      PH_MARK(13);
      if (uni(ctl.action) == 2) break;
      if (uni(ctl.action) == 1) continue;
      if (uni(ctl.status) != ST_OK) break;

      const uint32_t top = uni(ctl.top_slot);
      const uint32_t tlen = uni(ctl.top_len);
      const bool tdual = uni(ctl.top_dual) != 0;
      const SlotMeta tm = meta_get(E.L.meta[top]);
      const uint32_t tlens[2] = {tm.len[0], tm.len[1]};
      if (kDH && uni(ctl.hot_load)) {
        // per read the same thread stores then fetches; the analysis below
        // maps items to threads differently, hence the barrier
        const uint32_t prev = uni(ctl.hot_prev);
        if (prev != kNoSlot) {
          hot_store(E, prev, 0);
          if (uni(ctl.hot_prev_dual)) hot_store(E, prev, 1);
        }
        hot_fetch(E, top, 0);
        if (tdual) hot_fetch(E, top, 1);
        __syncthreads();
      }

      analyze_sides<kDH>(E, ctl, top, tdual ? 2 : 1, tlens[0], tlens[1], R0, R1);
      // reached_all_end (dual_consensus.rs:1174-1195): per read, either side at its end
      {
        uint32_t ne = 0;
        for (uint32_t r = tid; r < E.n; r += kEB)
          ne += (R0[r].e != kInactive && R0[r].end) || (tdual && R1[r].e != kInactive && R1[r].end);
        agg_add(&ctl.n_either, ne);
      }
      __syncthreads();
      if (tid == 0) {
        ctl.reached = early ? (ctl.n_either == E.n) : (ctl.n_either > 0);
        // reached_consensus_end (dual_consensus.rs:1203-1233); inactive counts as require_all
        ctl.fin[0] = early ? (ctl.n_end[0] == tm.nsome[0]) : (ctl.n_end[0] > 0);
        ctl.fin[1] = !tdual ? 0u : (early ? (ctl.n_end[1] == tm.nsome[1]) : (ctl.n_end[1] > 0));
        if (ctl.ovf) ctl.status = limit_status(ctl.ovf);
      }
      __syncthreads();
      PH_MARK(1);
      if (uni(ctl.status) != ST_OK) break;

      // ---- finalize a clone (dual_consensus.rs:438-492) ----
      if (uni(ctl.reached)) {
        WaveCounters cnt = {0, 0, 0, 0, 0, 0};
        finalize_side<kDH>(E, ctl, top, 0, tlens[0], E.L.fe, cnt);
        if (tdual) finalize_side<kDH>(E, ctl, top, 1, tlens[1], E.L.fe + E.nmax, cnt);
        flush_counters(ctl, cnt);
        __syncthreads();
        if (tid == 0) {
          ctl.store_idx = -1;
          if (ctl.ovf & 4u) {
            ctl.status = ST_RETRY | ST_RETRY_WCAP;
          } else {
            uint64_t total = 0, c1 = 0;
            bool uninit = false;
            for (uint32_t r = 0; r < E.n; ++r) {
              const uint32_t f1 = E.L.fe[r];
              const uint32_t f2 = tdual ? E.L.fe[E.nmax + r] : kInactive;
              int idx = -1;
              uint64_t best = ~0ull;
              if (f1 != kInactive) {
                best = cost_of(f1, cfg.cost_mode);
                idx = 0;
              }
              if (f2 != kInactive && cost_of(f2, cfg.cost_mode) < best) {
                best = cost_of(f2, cfg.cost_mode);
                idx = 1;
              }
              if (idx < 0) uninit = true;
              else total += best;
              c1 += (idx == 0);
            }
            if (uninit) {
              ctl.status = 1;  // "Finalize called on DWFA that was never initialized."
            } else {
              const uint64_t c2 = E.n - c1;
              const bool imbalanced = tdual && (c1 < full_min || c2 < full_min);
              if (!imbalanced) {
                if (total < ctl.max_err) {
                  ctl.max_err = total;
                  ctl.n_ret = 0;
                }
                if (total <= ctl.max_err && ctl.n_ret < cfg.max_return_size) {
                  if (ctl.n_ret < A.rmax) ctl.store_idx = (int32_t)ctl.n_ret;
                  ctl.n_ret++;
                }
              }
            }
          }
        }
        __syncthreads();
        if (uni(ctl.status) != ST_OK) break;
        if (uni(ctl.store_idx) >= 0) store_record(E, ctl, outp, top, tdual ? 2 : 1, tlens[0], tlens[1], tdual);
        PH_MARK(2);
      }

      // ---- active_min_count growth (dual_consensus.rs:497-513) ----
      SUB_T0(tam);
      uint32_t nadd = 0;  // reads activating at tlen
      if (tlen <= E.P.max_act && uni(ctl.am_len) == tlen + 1) {
        if (tid == 0) ctl.act_cnt = 0;
        __syncthreads();
        for (uint32_t r = tid; r < E.n; r += kEB)
          if (E.ract[E.P.read_begin + r] == (int64_t)tlen) atomicAdd(&ctl.act_cnt, 1u);
        __syncthreads();
        nadd = uni(ctl.act_cnt);
      }
      if (tid == 0 && ctl.am_len == tlen + 1 && tlen + 1 < E.lcap + 2) {
        const uint32_t nt = E.total_active[tlen] + nadd;
        E.total_active[tlen + 1] = nt;
        E.active_min[tlen + 1] = (uint32_t)max(cfg.min_count, ceil_u64(cfg.min_af * (double)nt));
        ctl.am_len++;
      }
      SUB_T1(31, tam);

      // ---- votes on both sides (waves 0 and 1 in parallel; one after the
      // other in a one-wave workgroup) ----
      for (uint32_t side = wave_id(); side < (tdual ? 2u : 1u); side += (uint32_t)kEW) {
        const bool ok = wave_votes(ctl, side, side == 0 ? R0 : R1, R0, R1, E.n, weighted, tdual,
                                   ctl.multi[side] != 0, cfg.wildcard, cfg.min_count, cfg.min_af == 0.0);
        if (!ok && lane == 0) atomicOr(&ctl.ovf, (uint32_t)LIM_VOTES);
      }
      __syncthreads();
      if (tid == 0) {
        if (ctl.ovf) ctl.status = limit_status(ctl.ovf);
        double thr[2] = {0.0, 0.0};
        uint64_t mc[2] = {0, 0};
#pragma unroll
        for (uint32_t s = 0; s < 2u; ++s) {
          if (s == 1 && !tdual) break;
          double sum = -0.0, mx = 0.0;
          bool have = false;
          for (uint32_t k = 0; k < ctl.nkeys[s]; ++k) {
            sum += ctl.vals[s][k];
            if (!have || ctl.vals[s][k] >= mx) mx = ctl.vals[s][k];
            have = true;
          }
          mc[s] = max(cfg.min_count, ceil_u64(cfg.min_af * sum));
          if (!have) mx = (double)mc[s];
          thr[s] = fmin((double)mc[s], mx);
        }
        uint32_t nc = 0;
        bool overflow = false;
        if (tdual) {
          // dual_consensus.rs:554-650: options per side, None first
          auto& o = ctl.opt;
          uint32_t no[2] = {0, 0};
          const bool lock[2] = {(tm.flags & 2u) != 0, (tm.flags & 4u) != 0};
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            if (ctl.fin[s] || ctl.nkeys[s] == 0 || lock[s]) o[s][no[s]++] = -1;
            if (!lock[s])
              for (uint32_t k = 0; k < ctl.nkeys[s]; ++k)
                if (!(ctl.vals[s][k] < thr[s])) o[s][no[s]++] = ctl.keys[s][k];
          }
          for (uint32_t a = 0; a < no[0]; ++a)
            for (uint32_t b = 0; b < no[1]; ++b) {
              if (o[0][a] < 0 && o[1][b] < 0) continue;
              if (nc == kMaxChild) {
                overflow = true;
                continue;
              }
              ctl.ch_s[nc][0] = o[0][a];
              ctl.ch_s[nc][1] = o[1][b];
              ctl.ch_kind[nc] = 0;
              nc++;
            }
        } else {
          // stay-single children (dual_consensus.rs:655-679)
          for (uint32_t k = 0; k < ctl.nkeys[0]; ++k) {
            if (ctl.vals[0][k] < thr[0]) continue;
            ctl.ch_s[nc][0] = ctl.keys[0][k];
            ctl.ch_s[nc][1] = -1;
            ctl.ch_kind[nc] = 1;
            nc++;
          }
          // split children from every pair of sorted candidates (:682-734)
          Lo<double>* cv = ctl.srt_v;
          Lo<uint8_t>* cs = ctl.srt_s;
          uint32_t ns = 0, passing = 0;
          for (uint32_t k = 0; k < ctl.nkeys[0]; ++k) {
            if (cfg.wildcard >= 0 && ctl.keys[0][k] == (uint8_t)cfg.wildcard) continue;
            if (ctl.vals[0][k] >= (double)mc[0]) passing++;
            // stable insertion sort by (Reverse(count), symbol)
            uint32_t p = ns;
            while (p > 0 && (cv[p - 1] < ctl.vals[0][k] || (cv[p - 1] == ctl.vals[0][k] && cs[p - 1] > ctl.keys[0][k]))) {
              cv[p] = cv[p - 1];
              cs[p] = cs[p - 1];
              --p;
            }
            cv[p] = ctl.vals[0][k];
            cs[p] = ctl.keys[0][k];
            ns++;
          }
          if (passing > 1)
            for (uint32_t i = 0; i < ns; ++i)
              for (uint32_t j = i + 1; j < ns; ++j) {
                if (nc == kMaxChild) {
                  overflow = true;
                  continue;
                }
                ctl.ch_s[nc][0] = cs[i];
                ctl.ch_s[nc][1] = cs[j];
                ctl.ch_kind[nc] = 2;
                nc++;
              }
        }
        if (overflow) ctl.status = limit_status(LIM_CHILDREN);
        ctl.nchild = nc;
      }
      __syncthreads();
      PH_MARK(3);
      if (uni(ctl.status) != ST_OK) break;
      const uint32_t nc = uni(ctl.nchild);
      if (nc == 0) {
        if (tid == 0) {
          E.L.freestack[WC_IX(ctl.nfree++, E.pcap)] = top;
          if (kDH) ctl.hot_slot = kNoSlot;
        }
        __syncthreads();
        continue;
      }
      if (tlens[0] + 1 > E.lcap || tlens[1] + 1 > E.lcap) {
        if (tid == 0) ctl.status = ST_RETRY | ST_RETRY_LCAP;
        __syncthreads();
        break;
      }

      // ---- one child: linear-chain run-ahead (chain.hip.hpp, dual_chain.hip.hpp) ----
      // Past the last activation point. A single-consensus node's stay-single
      // child: the single engine's walk; a dual node's child: the two-sided
      // walk (unweighted votes; a walking side must be the longer one, so the
      // max length grows with every step).
#ifdef WC_DUAL_CHAIN_CALL  // (engine_dchain.hip: the default builds carry no call)
      if (E.chain && nc == 1 && (E.P.n_active == E.n || tlen >= E.P.max_act)) {
        const int x0 = uni((int32_t)ctl.ch_s[0][0]), x1 = uni((int32_t)ctl.ch_s[0][1]);
        uint32_t kind = 0, walk = 0;
        if (!tdual) {
          if (uni((uint32_t)ctl.ch_kind[0]) == 1 && (A.chain_kinds & 1u)) kind = 1;
        } else if (!weighted && (A.chain_kinds & 2u)) {
          walk = (x0 >= 0 ? 1u : 0u) | (x1 >= 0 ? 2u : 0u);
          const uint32_t L0 = max(tlens[0], tlens[1]);
          if (((walk & 1u) && tlens[0] == L0) || ((walk & 2u) && tlens[1] == L0)) kind = 2;
        }
        if (kind) {
          const uint32_t flags = tm.flags | (x0 < 0 ? 2u : 0u) | (x1 < 0 ? 4u : 0u);
          SUB_T0(tch);
          const uint32_t jstar = run_engine_chain(kernel_args(), E.P, state_base(A, smem), ctl, top, kind, tlens[0],
                                                  tlens[1], walk, (uint32_t)max(x0, 0), (uint32_t)max(x1, 0), flags);
          PH_MARK(14);
          // (phase builds) per chain kind: attempts, accepted nodes, speculative steps, cycles
          SUB_CNT(kind == 1 ? 32 : 35, 1);
          SUB_CNT(kind == 1 ? 33 : 36, jstar);
          SUB_CNT(kind == 1 ? 34 : 37, uni(ctl.chain_stop));
          SUB_T1(kind == 1 ? 38 : 39, tch);
          if (jstar) continue;
        }
      }
#endif

      // ---- build every child: clones first, the last child in place ----
      SUB_CNT(21, nc);
      dual_build_children<kDH>(E, ctl, top, tm, tdual, nc);
      if (uni(ctl.status) != ST_OK) break;
      if (tid == 0) {
        for (uint32_t c = 0; c < nc; ++c) {
          const uint32_t k = (E.L.meta[ctl.ch_slot[c]].flags & 1u) ? 1 : 0;
          E.tracker(ctl, k).insert(ctl.ch_len[c]);
          const HeapEntry ce{ctl.ch_cost[c], ctl.ch_len[c], ctl.ch_slot[c]};
          // the last (in-place) child: when the next pop would take it
          // straight back and leave the heap as it was, both are skipped
          if (kRepopBlock && c + 1 == nc && heap_push_pop_noop(E.L.heap, ctl.heap_n, ce)) {
            ctl.heap_n++;
            ctl.top_cost = ce.cost;
            ctl.top_len = ce.len;
            ctl.top_slot = ce.slot;
            ctl.top_dual = kTopStashed;
          } else {
            heap_push(E.L.heap, ctl.heap_n, E.pcap, ce);
          }
        }
      }
      // (no barrier: the next pop is thread 0's too, and the block meets after it)
      PH_MARK(7);
    }
    finish_problem(A, ctl, outp, prob, oslot);
  }
  stream_exit(A);
}

#ifdef WC_WAVE_DUAL
#include "wave_dual.hip.hpp"
#ifdef WC_COOP
// every problem on kEW cooperating waves, one read per lane (engine_coop.hip)
__global__ void __launch_bounds__(kEB) __attribute__((amdgpu_waves_per_eu(WC_DUAL_WAVES_PER_EU))) dual_coop_kernel(EngineArgs A) {
  extern __shared__ __align__(16) uint8_t smem[];
  __shared__ Ctl ctl_lds;
  dual_main_wave<1, false>(A, smem, *(Lo<Ctl>*)&ctl_lds);
}
#else
// one kernel per reads-per-lane count (engine_wave.hip): launches whose
// problems have <= 64 reads, and launches with larger ones (<= 128 reads, two
// per lane), where each problem of <= 64 reads still runs one read per lane
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WC_DUAL_WAVES_PER_EU))) dual_wave1_kernel(EngineArgs A) {
  extern __shared__ __align__(16) uint8_t smem[];
  __shared__ Ctl ctl_lds;
  dual_main_wave<1, false>(A, smem, *(Lo<Ctl>*)&ctl_lds);
}
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WC_WAVE2_WPE))) dual_wave2_kernel(EngineArgs A) {
  extern __shared__ __align__(16) uint8_t smem[];
  __shared__ Ctl ctl_lds;
  dual_main_wave<2, true>(A, smem, *(Lo<Ctl>*)&ctl_lds);
}
#endif  // WC_COOP
#elif !defined(WC_SINGLE_ONLY)  // (engine_cu.hip: the single engine only)
// two kernels, one per dual_hot: in one kernel the two paths' register
// allocations merge (the 4-wave build spilled 236 VGPRs instead of 84)
__global__ void __launch_bounds__(kEB) __attribute__((amdgpu_waves_per_eu(WC_DUAL_WAVES_PER_EU))) dual_engine_kernel(EngineArgs A) {
  extern __shared__ __align__(16) uint8_t smem[];
  __shared__ Ctl ctl_lds;
  dual_main<false>(A, smem, *(Lo<Ctl>*)&ctl_lds);
}
#if !defined(WC_GLOBAL_STATE) && !defined(WC_DUAL_CHAIN_CALL)  // (the host plans dual_hot for neither build)
__global__ void __launch_bounds__(kEB) __attribute__((amdgpu_waves_per_eu(WC_DUAL_WAVES_PER_EU))) dual_hot_engine_kernel(EngineArgs A) {
  extern __shared__ __align__(16) uint8_t smem[];
  __shared__ Ctl ctl_lds;
  dual_main<true>(A, smem, *(Lo<Ctl>*)&ctl_lds);
}
#endif
#endif  // WC_SINGLE_ONLY

#if !defined(WC_GLOBAL_STATE) && !defined(WC_NARROW) && !defined(WC_LOWLAT) && !defined(WC_CU) && !defined(WC_WAVE_DUAL)
// =====================================================================
// standalone DWFALite jobs (dynamic_wfa.rs:48-265): one wave per job
// =====================================================================
__global__ void __launch_bounds__(64) dwfa_jobs_kernel(DwfaDevJob* jobs) {
  DwfaDevJob& j = jobs[blockIdx.x];
  const int lane = lane_id();
  Gm<uint32_t>* wf = (Gm<uint32_t>*)j.wf;
  const Gm<uint8_t>* base = (const Gm<uint8_t>*)j.baseline;
  const Gm<uint8_t>* other = (const Gm<uint8_t>*)j.other;
  uint32_t e = j.e;
  WaveCounters cnt = {0, 0, 0, 0, 0, 0};
  uint32_t status = 0;
  if (j.op == 0) {
    uint32_t mo = 0, mb = 0;
    if (!wave_update_general(wf, e, j.offset, base, j.blen, other, j.olen, j.wildcard, j.early != 0, j.wf_cap,
                             cnt, mo, mb))
      status = WC_E_LIMIT_CODE;
    else if (!(mo == j.olen || (j.early && mb == j.blen)))
      status = WC_E_INVARIANT_CODE;  // dynamic_wfa.rs:94-97 assert
  } else if (j.op == 1) {
    uint32_t W = 2 * e + 1, mb = 0;
    for (uint32_t i = lane; i < W; i += 64) mb = max(mb, wf[i] + e - i);
    mb = wave_max_u32(mb);
    uint32_t cmp = 0;
    while (mb < j.blen) {
      if (W + 2 > j.wf_cap) {
        status = WC_E_LIMIT_CODE;
        break;
      }
      wave_grow(wf, W);
      W += 2;
      e += 1;
      uint32_t mo;
      wave_extend_all(wf, W, e, j.offset, base, j.blen, other, j.olen, j.wildcard, mo, mb, cmp);
    }
  } else {
    __shared__ RInfo ri_lds;
    Lo<RInfo>& ri = *(Lo<RInfo>*)&ri_lds;
    uint64_t ins = 0;
    if (!wave_analyze_read(wf, e, j.offset, base, j.blen, j.olen, &ri, &ins)) status = WC_E_LIMIT_CODE;
    __builtin_amdgcn_wave_barrier();
    if (lane == 0 && status == 0) {
      j.n_cand = ri.n;
      for (uint32_t k = 0; k < ri.n; ++k) {
        j.cand_syms[k] = ri.sym[k];
        j.cand_counts[k] = ri.occ[k];
        j.cand_first[k] = (uint8_t)byte_at(ins, k);
      }
    }
  }
  if (lane == 0) {
    j.e = e;
    j.status = status;
  }
}

#endif

#ifndef WC_DUAL_ONLY
void launch_single_engine(const EngineArgs& a, uint32_t grid, size_t lds, hipStream_t s) {
  hipLaunchKernelGGL(single_engine_kernel, dim3(grid), dim3(kEB), lds, s, a);
}
#endif
// waves per workgroup of this build (the host sizes the per-wave layouts)
int engine_waves() { return kEW; }
// Workgroups per CU of `kernel` at `lds` bytes of dynamic LDS. The runtime's
// occupancy query counts LDS more finely than gfx950 allocates it: a CU's
// 160 KB go out in granules of 1,280 bytes (tools/lds_occupancy.hip: 53,760
// bytes ran 3 per CU, 53,761 only 2, where the query answers 3 up to 54,613),
// so its answer is capped by the granule count of static + dynamic LDS.
template <class K>
static int blocks_per_cu(K kernel, int threads, size_t lds) {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, threads, lds) != hipSuccess || nb <= 0) return 1;
  hipFuncAttributes at;
  if (hipFuncGetAttributes(&at, (const void*)kernel) == hipSuccess) {
    constexpr size_t kGranule = 1280, kLdsPerCu = 160 * 1024;
    const size_t per_wg = (at.sharedSizeBytes + lds + kGranule - 1) / kGranule * kGranule;
    if (per_wg) nb = std::min<int>(nb, (int)(kLdsPerCu / per_wg));
  }
  return std::max(nb, 1);
}
#if defined(WC_WAVE_DUAL) && defined(WC_COOP)
void launch_dual_engine(const EngineArgs& a, uint32_t grid, size_t lds, hipStream_t s) {
  hipLaunchKernelGGL(dual_coop_kernel, dim3(grid), dim3(kEB), lds, s, a);
}
int coop_blocks_per_cu(size_t lds) { return blocks_per_cu(dual_coop_kernel, kEB, lds); }
#elif defined(WC_WAVE_DUAL)
// experiment hook: WC_WAVE_KERNEL=2 runs every problem on the two-reads-per-lane
// kernel (1 wave per SIMD) instead of the one-read kernel for <=64 reads
static bool wave_force2() {
  static const bool f = [] { const char* e = getenv("WC_WAVE_KERNEL"); return e && atoi(e) == 2; }();
  return f;
}
void launch_dual_engine(const EngineArgs& a, uint32_t grid, size_t lds, hipStream_t s) {
  if (a.nmax <= 64 && !wave_force2()) hipLaunchKernelGGL(dual_wave1_kernel, dim3(grid), dim3(64), lds, s, a);
  else hipLaunchKernelGGL(dual_wave2_kernel, dim3(grid), dim3(64), lds, s, a);
}
// workgroups per CU of the build that runs problems of nmax reads
int wave_blocks_per_cu(uint32_t nmax, size_t lds) {
  return nmax <= 64 && !wave_force2() ? blocks_per_cu(dual_wave1_kernel, 64, lds) : blocks_per_cu(dual_wave2_kernel, 64, lds);
}
#elif !defined(WC_SINGLE_ONLY)
void launch_dual_engine(const EngineArgs& a, uint32_t grid, size_t lds, hipStream_t s) {
#if !defined(WC_GLOBAL_STATE) && !defined(WC_DUAL_CHAIN_CALL)
  if (a.dual_hot) {
    hipLaunchKernelGGL(dual_hot_engine_kernel, dim3(grid), dim3(kEB), lds, s, a);
    return;
  }
#endif
  hipLaunchKernelGGL(dual_engine_kernel, dim3(grid), dim3(kEB), lds, s, a);
}
#endif
#ifndef WC_WAVE_DUAL
int engine_blocks_per_cu(uint32_t sides, size_t lds, bool dual_hot) {
#ifndef WC_DUAL_ONLY
  if (sides == 1) return blocks_per_cu(single_engine_kernel, kEB, lds);
#else
  if (sides == 1) return 1;
#endif
#ifndef WC_SINGLE_ONLY
#if !defined(WC_GLOBAL_STATE) && !defined(WC_DUAL_CHAIN_CALL)
  if (dual_hot) return blocks_per_cu(dual_hot_engine_kernel, kEB, lds);
#endif
  return blocks_per_cu(dual_engine_kernel, kEB, lds);
#endif
  return 1;
}
#endif
#if !defined(WC_GLOBAL_STATE) && !defined(WC_NARROW) && !defined(WC_LOWLAT) && !defined(WC_CU) && !defined(WC_WAVE_DUAL)
void launch_dwfa_jobs(DwfaDevJob* jobs, uint32_t n, hipStream_t s) {
  hipLaunchKernelGGL(dwfa_jobs_kernel, dim3(n), dim3(64), 0, s, jobs);
}
#endif

}  // namespace WC_ENGINE_NS
