// DualConsensusDWFA on one wave per problem (engine_wave.hip, namespace wcw).
//
// The dual search (dual_consensus.rs:240-787) of a PriorityConsensusDWFA
// sub-problem is a long sequence of dependent pops, and most pops expand the
// node the previous pop created in place (one child, popped next: 81-87% of
// cfg5's one-child pops). In the block engines (dual_main) every such pop
// re-reads every read's RState from its HBM slot twice (analysis, push), and
// the tip bytes of the read behind each wavefront tip twice, each a dependent
// HBM round trip, between barriers of 2-4 waves. That is the per-pop latency
// that bounds a deep locus (cfg5 locus 5949, 1.16M pops in
// sequence).
//
// Here one wave runs the whole search, lane r holding read r (and r + 64,
// r + 128, ... up to R reads per lane):
//  * the popped node's per-read state stays in LDS ("hot", Lds::hot) in an
//    uncompacted frontier format, written back to its slot only when another
//    node is popped, before clones copy it and before a finalize;
//  * the read bytes at each frontier tip are fetched into registers right
//    after the push that creates the frontier, so the next pop of that node
//    (its in-place child) nominates and pushes without a memory round trip;
//  * the push, the ED-increase hand-off, prune_dwfa (:1030-1045), the costs
//    (:1092-1168) and the Some counts of the in-place child are one lane pass.
// Search control (heap, trackers, thresholds, candidate order, f64 vote
// order) is dual_main's, unchanged; pops with several children or an
// activate_dual split (:682-734) take dual_build_children after a write-back.
// Problems with offsets (activation) run on the block engines (the host never
// plans this build for them).

// ---- the cooperative build (engine_coop.hip, kEW > 1 waves per problem) ----
// Wave w's lane l holds read 64 w + l (one read per lane); every wave runs the
// search control on the same values (what one wave learns about its reads, the
// others get through LDS: nominations in the RInfo area, flag words and
// partial sums in coopx()), and wave 0 alone writes the shared state: heap,
// trackers, free stack, slot metadata and consensus bytes (thread 0).
constexpr bool kCoop = kEW > 1;
// the lean path's pushes leave advancing tips' row entries to the RState
// (hot_flush_rows below); WC_EAGER_ROWS keeps every row entry written
#ifdef WC_EAGER_ROWS
constexpr bool kLazyRows = false;
#else
constexpr bool kLazyRows = true;
#endif
// an in-place child that the next pop would take straight back skips the
// heap (wheap_push_pop_noop); WC_NO_REPOP keeps every push and pop
#ifdef WC_NO_REPOP
constexpr bool kRepop = false;
#else
constexpr bool kRepop = true;
#endif
// the first read of this wave
__device__ __forceinline__ uint32_t read_base() { return kCoop ? 64u * (uint32_t)wave_id() : 0u; }
// (coop) between every wave's reads of shared state and wave 0's writes
__device__ __forceinline__ void coop_sync() {
  if constexpr (kCoop) __syncthreads();
}
// (coop) the waves' exchange area, a static LDS variable of its own that only
// the cooperative build references: Ctl keeps its size in every other build,
// whose LDS budgets sit at 1,280-byte allocation granules (§2.6 of DESIGN.md:
// 112 bytes more in Ctl cost cfg3's dual build a workgroup per CU)
struct CoopX {
  uint32_t flags[kEW];  // analysis flags of the wave's reads
  uint32_t nh[kEW];     // ED-increase overflow bits of the wave's reads
  uint32_t cc[kEW];     // Some counts of the in-place child (side 1 | side 2 << 16)
  uint64_t cost[kEW];   // the in-place child's cost over the wave's reads
  uint64_t top_cost[2];  // the node wave 0 popped for every wave (double-buffered by pop parity)
  uint32_t top_len[2], top_slot[2];
};
__device__ __forceinline__ CoopX& coopx() {
  __shared__ CoopX x;
  return x;
}
// a read's nominations (NomRaw) through the LDS area of its RInfo record
struct NomRaw;
__device__ __forceinline__ void nom_put(Sh<RInfo>* p, const NomRaw& o);
__device__ __forceinline__ NomRaw nom_get(const Sh<RInfo>* p);

// ---- the hot copy: the popped node's RStates (slot format) in LDS ----
// Lds::hot[side * nmax + r] is authoritative while the node is hot: pushes
// (front_store) and the ED-increase loops (wave_heavy's rebuild) write it
// there; the slot gets it back (a raw copy) when another node is popped.
// ---- tip bytes: the read byte behind every tip of a frontier ----
// (thread_tips' x[k] for the frontier as front_store compacts it: entry k is
// the k-th live slot in ascending order; byte k of lo/hi, valid bit k)
struct Tips {
  uint32_t lo, hi, valid;
};
__device__ __forceinline__ Tips tips_fetch(const Front& f, const Gm<uint8_t>* rd, uint32_t blen, uint32_t len) {
  Tips t = {0, 0, 0};
  uint32_t rank = 0;
  const uint32_t hi = f.mask ? 32u - (uint32_t)__builtin_clz(f.mask) : 0u;
#pragma unroll
  for (int k = 0; k < kF; ++k) {
    if ((uint32_t)k >= hi) break;
    if (!(f.mask & (1u << k))) continue;
    const uint32_t bo = f.fd[k] + f.e - f.fi[k];
    if (f.fd[k] + f.off == len && bo < blen) {
      const uint32_t b = rd[bo];
      t.valid |= 1u << rank;
      if (rank < 4) t.lo |= b << (8 * rank);
      else t.hi |= b << (8 * (rank - 4));
    }
    rank++;
  }
  return t;
}
__device__ __forceinline__ void tips_unpack(const Tips& t, uint32_t (&x)[kF]) {
#pragma unroll
  for (int k = 0; k < kF; ++k) {
    const uint32_t b = ((k < 4 ? t.lo : t.hi) >> (8 * (k & 3))) & 0xFFu;
    x[k] = (t.valid >> k) & 1u ? b : 0x100u;
  }
}

// thread_nominate on prefetched tip bytes (same arithmetic: every live slot
// counts for reached_baseline_end, the tips give the nominations), without
// the hashbrown order of several symbols (the lean path's votes do not depend
// on it): the distinct tip symbols in first-seen
// order (klo/khi bytes), their counts (nibbles of cnt), and in meta the
// number of symbols, reached_baseline_end (bit 8) and the split (bits 16+);
// e = the read's edit distance (kInactive: no DWFA). The order, and RInfo,
// are made only for the pops whose votes take the block engines' code
// (wave_fill_rinfo).
struct NomRaw {
  uint32_t klo, khi, cnt, meta, e;
};
__device__ inline NomRaw nominate_raw(const Front& f, const uint32_t (&x)[kF], uint32_t blen) {
  uint32_t mb = f.maxb;
  const uint32_t hi = f.mask ? 32u - (uint32_t)__builtin_clz(f.mask) : 0u;
#pragma unroll
  for (int k = 0; k < kF; ++k) {
    if ((uint32_t)k >= hi) break;
    if (f.mask & (1u << k)) mb = max(mb, f.fd[k] + f.e - f.fi[k]);
  }
  uint64_t keys = 0;
  uint32_t cnts = 0, nk = 0, split = 0;
#pragma unroll
  for (int k = 0; k < kF; ++k) {
    if ((uint32_t)k >= hi) break;
    const uint32_t s = x[k];
    if (s == 0x100u) continue;
    uint32_t j = 0;
    while (j < nk && byte_at(keys, j) != s) ++j;
    if (j == nk) {
      keys |= (uint64_t)s << (8 * nk);
      nk++;
    }
    cnts += 1u << (4 * j);
    split++;
  }
  return NomRaw{(uint32_t)keys, (uint32_t)(keys >> 32), cnts, nk | ((mb == blen) ? 256u : 0u) | (split << 16), f.e};
}
__device__ __forceinline__ void nom_put(Sh<RInfo>* p, const NomRaw& o) {
  static_assert(sizeof(RInfo) >= 20 && sizeof(RInfo) % 16 == 0, "RInfo holds a NomRaw");
  ((Sh<uint4>*)p)[0] = make_uint4(o.klo, o.khi, o.cnt, o.meta);
  ((Sh<uint32_t>*)p)[4] = o.e;
}
__device__ __forceinline__ NomRaw nom_get(const Sh<RInfo>* p) {
  const uint4 a = ((const Sh<uint4>*)p)[0];
  return NomRaw{a.x, a.y, a.z, a.w, ((const Sh<uint32_t>*)p)[4]};
}
// RInfo (thread_nominate's record, the order of several symbols included) of
// one read from its NomRaw, for the block engines' votes (WR_VOTES_SELECT)
__device__ inline void rinfo_from_raw(Sh<RInfo>* out, const NomRaw& r) {
  if (r.e == kInactive) {
    out->e = kInactive;
    out->n = 0;
    out->end = 0;
    return;
  }
  const uint32_t nk = r.meta & 0xFFu;
  const uint64_t keys = (uint64_t)r.klo | ((uint64_t)r.khi << 32);
  Nom o;
  o.n = nk;
  o.end = (r.meta >> 8) & 1u;
  if (nk <= 1) {
    o.sym = keys;
    o.occ = r.cnt;
    o.split = r.cnt;
  } else {
    const uint64_t ord = fx_order_packed(nk, [&](uint32_t j) { return byte_at(keys, j); });
    uint64_t sym = 0, occ = 0;
    uint32_t split = 0;
    for (uint32_t k = 0; k < nk; ++k) {
      const uint32_t j = nib(ord, k);
      const uint32_t c = (r.cnt >> (4 * j)) & 15u;
      sym |= (uint64_t)byte_at(keys, j) << (8 * k);
      occ |= (uint64_t)c << (8 * k);
      split += c;
    }
    o.sym = sym;
    o.occ = occ;
    o.split = split;
  }
  rinfo_store(out, o, r.e);
}

// the hot node (both sides when `dual`) back into slot `slot`
template <int R>
__device__ __forceinline__ void hot_writeback(Eng& E, uint32_t slot, bool dual) {
  const int lane = lane_id();
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const uint32_t r = read_base() + (uint32_t)lane + 64u * j;
    if (r >= E.n) continue;
    rstate_store(&E.sv(slot, 0).rs[r], rstate_load(&E.L.hot[r]));
    if (dual) rstate_store(&E.sv(slot, 1).rs[r], rstate_load(&E.L.hot[E.nmax + r]));
  }
}
template <int R>
__device__ __forceinline__ void hot_fetch_slot(Eng& E, uint32_t slot, bool dual) {
  const int lane = lane_id();
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const uint32_t r = read_base() + (uint32_t)lane + 64u * j;
    if (r >= E.n) continue;
    const RRaw a = rstate_load(&E.sv(slot, 0).rs[r]);
    RRaw b = a;
    if (dual) b = rstate_load(&E.sv(slot, 1).rs[r]);
    rstate_store(&E.L.hot[r], a);
    if (dual) rstate_store(&E.L.hot[E.nmax + r], b);
  }
}
// Lazy rows: the lean path's pushes (thread_apply<true>) do not write a tip's
// new value into its wavefront row when it advances, only a diagonal's final
// value when it leaves the frontier (stuck or at the read's end). Between the
// two the RState is authoritative for its frontier diagonals, and the row for
// every other diagonal. Readers of rows: the ED-increase loop (a read whose
// frontier emptied, so every diagonal has been written; wide-frontier reads
// never take the lean push), and the block engines' code (wave_rare), whose
// pushes assume rows complete: the hot node's frontier goes into its rows
// first (this function, at wave_rare's entry). Clones copy rows and RStates together, so the
// invariant carries over to them.
template <int R>
__device__ __forceinline__ void hot_flush_rows(Eng& E, uint32_t slot, bool dual) {
  const int lane = lane_id();
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const uint32_t r = read_base() + (uint32_t)lane + 64u * j;
    if (r >= E.n) continue;
#pragma unroll
    for (int sd = 0; sd < 2; ++sd) {
      if (sd == 1 && !dual) continue;
      const RRaw s = rstate_load(&E.L.hot[sd * E.nmax + r]);
      if (rraw_e(s) == kInactive || (rraw_flags(s) & kWide)) continue;
      Front f;
      front_load(s, f);
      front_flush(f, E.sv(slot, sd).wf + (uint64_t)r * E.wcap);
    }
  }
}

// ---- the rare paths, out of line (one call site each): the pop loop's
// register allocation does not carry theirs. The callee rebuilds the engine
// context from the kernel arguments (callee_eng); the hot area is the carve's
// start, so sbase = Lds::hot. ----
enum : uint32_t { WR_GENERAL_POP = 0, WR_VOTES_SELECT = 1, WR_CHILDREN = 3 };

// dual_main's thread-0 selection (dual_consensus.rs:520-734): thresholds from
// the votes in ctl.keys/vals, then the children in the reference's order
__device__ inline void wave_select_t0(const DevConfig& cfg, Lo<Ctl>& ctl, const SlotMeta& tm, bool tdual) {
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
    for (uint32_t k = 0; k < ctl.nkeys[0]; ++k) {
      if (ctl.vals[0][k] < thr[0]) continue;
      ctl.ch_s[nc][0] = ctl.keys[0][k];
      ctl.ch_s[nc][1] = -1;
      ctl.ch_kind[nc] = 1;
      nc++;
    }
    Lo<double>* cv = ctl.srt_v;
    Lo<uint8_t>* cs = ctl.srt_s;
    uint32_t ns = 0, passing = 0;
    for (uint32_t k = 0; k < ctl.nkeys[0]; ++k) {
      if (cfg.wildcard >= 0 && ctl.keys[0][k] == (uint8_t)cfg.wildcard) continue;
      if (ctl.vals[0][k] >= (double)mc[0]) passing++;
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

// the ED-increase loops (and wide frontiers) of the in-place push: one read
// per wave, on the hot copy (the rows are the slot's). A call of its own, with
// what it needs as arguments: the general paths' call saved and restored 42
// registers, and rebuilding the engine context from the kernel arguments
// (callee_eng) cost most of a call.
// (V: the kernel it is called from, so that each kernel's call has a body
// compiled for that kernel's register budget)
template <int R>
struct HeavyArgs {
  Sh<RState>* hot;
  const Sh<uint32_t>* list;
  Gm<uint32_t>* wf[2];
  const Gm<uint8_t>* con[2];
  const Gm<uint8_t>* rd[R];  // per lane: read lane + 64 j
  uint32_t bl[R];
  uint32_t list_cap, nmax, n, wcap, nl[2], sy[2];
  int wc;
  uint32_t early;
};
template <int R, int V>
__device__ __noinline__ uint32_t wave_heavy_call(HeavyArgs<R> h, Lo<Ctl>& ctl, uint32_t lbase, uint32_t nh) {
  const int lane = lane_id();
  WaveCounters cnt = {0, 0, 0, 0, 0, 0};
  uint32_t ovf = 0;  // (coop: returned, the caller exchanges it; else ctl.ovf)
  // (this wave's items: list entries [lbase, lbase + nh), its own reads; every
  // wave calls, for the barrier at the end)
  for (uint32_t k = 0; k < nh; ++k) {
    const uint32_t it = uni(h.list[WC_IX(lbase + k, h.list_cap)]);
    const uint32_t sd = it >= h.n ? 1u : 0u, r = it - sd * h.n;
    // read r's bytes and length from the lane that holds it
    const uint32_t rr = r - read_base();
    const uint32_t j = rr >> 6, l = rr & 63u;
    const Gm<uint8_t>* rp = h.rd[0];
    uint32_t bl = h.bl[0];
#pragma unroll
    for (int q = 1; q < R; ++q)
      if (j == (uint32_t)q) {
        rp = h.rd[q];
        bl = h.bl[q];
      }
    const uint64_t pv = (uint64_t)rp;
    const Gm<uint8_t>* rd = (const Gm<uint8_t>*)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(pv >> 32), l) << 32) |
                                                  (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)pv, l));
    bl = (uint32_t)__builtin_amdgcn_readlane((int)bl, l);
    uint32_t e = 0;
    const bool ok = wave_heavy(&h.hot[sd * h.nmax + r], (sd ? h.wf[1] : h.wf[0]) + (uint64_t)r * h.wcap, rd, bl,
                               sd ? h.con[1] : h.con[0], sd ? h.nl[1] : h.nl[0], (uint8_t)(sd ? h.sy[1] : h.sy[0]), h.wc,
                               h.early != 0, h.wcap, cnt, e);
    __builtin_amdgcn_wave_barrier();
    if (kCoop) ovf |= ok ? 0u : 4u;
    else if (!ok && lane == 0) atomicOr(&ctl.ovf, 4u);
  }
  flush_counters(ctl, cnt);
  if constexpr (!kCoop) __syncthreads();
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)ovf);
}

template <int R, int V>
__device__ __noinline__ void wave_rare(KArgs kp, DevProblem P, Sh<uint8_t>* sbase, Lo<Ctl>& ctl, uint32_t op,
                                       uint32_t top, uint32_t tdual_u, uint32_t a0, uint32_t a1, uint32_t a2,
                                       uint32_t a3, uint32_t a4) {
  Eng E = callee_eng(kp, P, sbase);
  const int tid = threadIdx.x, lane = lane_id();
  const DevConfig& cfg = E.cfg;
  const bool early = cfg.early != 0;
  const bool weighted = cfg.weighted != 0;
  const bool tdual = tdual_u != 0;
  const uint32_t n = E.n;
  const SlotMeta tm = meta_get(E.L.meta[top]);
  Sh<RInfo>* R0 = E.L.rinfo;
  Sh<RInfo>* R1 = E.L.rinfo + E.nmax;
  if constexpr (kLazyRows) {
    // (the block code below pushes and clones from the node's rows)
    if (op != WR_VOTES_SELECT) {
      hot_flush_rows<R>(E, top, tdual);
      __syncthreads();
    }
  }
  if (op == WR_VOTES_SELECT) {
    // the votes from the pop's RInfo (weighted, or splits that round, or
    // several children to order) and dual_main's selection; the caller
    // builds a single in-place child itself
    for (uint32_t side = wave_id(); side < (tdual ? 2u : 1u); side += (uint32_t)kEW) {
      const bool ok = wave_votes(ctl, side, side == 0 ? R0 : R1, R0, R1, n, weighted, tdual, ctl.multi[side] != 0,
                                 cfg.wildcard, cfg.min_count, cfg.min_af == 0.0);
      if (!ok && lane == 0) atomicOr(&ctl.ovf, (uint32_t)LIM_VOTES);
    }
    __syncthreads();
    if (tid == 0) wave_select_t0(cfg, ctl, tm, tdual);
    __syncthreads();
    return;
  }
  // the rest of the pop with the block engines' code (dual_main), from the
  // slot: the hot node goes back there first and is dropped
  const uint32_t tlens[2] = {tm.len[0], tm.len[1]};
  hot_writeback<R>(E, top, tdual);
  __threadfence_block();
  if (tid == 0) ctl.hot_slot = kNoSlot;
  __syncthreads();
  if (op == WR_CHILDREN) {  // after WR_VOTES_SELECT: several children, or an activate_dual split
    if (tlens[0] + 1 > E.lcap || tlens[1] + 1 > E.lcap) {
      if (tid == 0) ctl.status = ST_RETRY | ST_RETRY_LCAP;
      __syncthreads();
      return;
    }
    dual_build_children<false>(E, ctl, top, tm, tdual, uni(ctl.nchild));
    return;
  }
  if (op == WR_GENERAL_POP) {
    const uint64_t full_min = (uint64_t)a0 | (uint64_t)a1 << 32;
    const uint32_t oslot = a2;
    analyze_sides<false>(E, ctl, top, tdual ? 2 : 1, tlens[0], tlens[1], R0, R1);
    {
      uint32_t ne = 0;
      for (uint32_t r = tid; r < n; r += kEB)
        ne += (R0[r].e != kInactive && R0[r].end) || (tdual && R1[r].e != kInactive && R1[r].end);
      agg_add(&ctl.n_either, ne);
    }
    __syncthreads();
    if (tid == 0) {
      ctl.reached = early ? (ctl.n_either == n) : (ctl.n_either > 0);
      ctl.fin[0] = early ? (ctl.n_end[0] == tm.nsome[0]) : (ctl.n_end[0] > 0);
      ctl.fin[1] = !tdual ? 0u : (early ? (ctl.n_end[1] == tm.nsome[1]) : (ctl.n_end[1] > 0));
      if (ctl.ovf) ctl.status = limit_status(ctl.ovf);
    }
    __syncthreads();
    if (uni(ctl.status) != ST_OK) return;
    // finalize a clone (dual_consensus.rs:438-492)
    if (uni(ctl.reached)) {
      WaveCounters cnt = {0, 0, 0, 0, 0, 0};
      finalize_side<false>(E, ctl, top, 0, tlens[0], E.L.fe, cnt);
      if (tdual) finalize_side<false>(E, ctl, top, 1, tlens[1], E.L.fe + E.nmax, cnt);
      flush_counters(ctl, cnt);
      __syncthreads();
      const uint32_t rmax = kp->rmax;
      if (tid == 0) {
        ctl.store_idx = -1;
        if (ctl.ovf & 4u) {
          ctl.status = ST_RETRY | ST_RETRY_WCAP;
        } else {
          uint64_t total = 0, c1 = 0;
          bool uninit = false;
          for (uint32_t r = 0; r < n; ++r) {
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
            const uint64_t c2 = n - c1;
            const bool imbalanced = tdual && (c1 < full_min || c2 < full_min);
            if (!imbalanced) {
              if (total < ctl.max_err) {
                ctl.max_err = total;
                ctl.n_ret = 0;
              }
              if (total <= ctl.max_err && ctl.n_ret < cfg.max_return_size) {
                if (ctl.n_ret < rmax) ctl.store_idx = (int32_t)ctl.n_ret;
                ctl.n_ret++;
              }
            }
          }
        }
      }
      __syncthreads();
      if (uni(ctl.status) != ST_OK) return;
      if (uni(ctl.store_idx) >= 0) {
        Gm<uint8_t>* outp = (Gm<uint8_t>*)kp->out + (uint64_t)oslot * kp->out_stride;
        store_record(E, ctl, outp, top, tdual ? 2 : 1, tlens[0], tlens[1], tdual);
      }
    }
  }
  // votes on both sides, the selection, the children (dual_main)
  for (uint32_t side = wave_id(); side < (tdual ? 2u : 1u); side += (uint32_t)kEW) {
    const bool ok = wave_votes(ctl, side, side == 0 ? R0 : R1, R0, R1, n, weighted, tdual, ctl.multi[side] != 0,
                               cfg.wildcard, cfg.min_count, cfg.min_af == 0.0);
    if (!ok && lane == 0) atomicOr(&ctl.ovf, (uint32_t)LIM_VOTES);
  }
  __syncthreads();
  if (tid == 0) wave_select_t0(cfg, ctl, tm, tdual);
  __syncthreads();
  if (uni(ctl.status) != ST_OK) return;
  const uint32_t nc = uni(ctl.nchild);
  if (nc == 0) {  // no child: the slot is free (the main loop pushes nothing)
    if (tid == 0) E.L.freestack[WC_IX(ctl.nfree++, E.pcap)] = top;
    __syncthreads();
    return;
  }
  if (tlens[0] + 1 > E.lcap || tlens[1] + 1 > E.lcap) {
    if (tid == 0) ctl.status = ST_RETRY | ST_RETRY_LCAP;
    __syncthreads();
    return;
  }
  dual_build_children<false>(E, ctl, top, tm, tdual, nc);
}

// per-lane read pointers and lengths of the claimed problem (read lane + 64 j)
template <int R>
struct LaneReads {  // (R = 1, 2 or 4)
  const Gm<uint8_t>* rd[R];
  uint32_t bl[R];
};

// ---- register-resident search control ----
// The pop loop keeps the search control (heap size, free-stack top, the
// trackers' totals and thresholds, the work counters) in uniform registers:
// in LDS, thread 0 read and wrote each of them with a full LDS round trip, one
// after the other. The general path (wave_rare) still reads Ctl, so the
// fields it uses are synced around each call.
// Lengths, queue sizes and per-problem pop counts fit 32 bits (fewer SGPRs:
// the pop loop's uniform state spilled into VGPR lanes); the pop counters go
// to Ctl before they could wrap, lastc saturates.
struct WCtl {
  uint32_t heap_n, nfree, hot, hot_dual, am_len, n_ret, status;
  uint64_t max_err;
  uint32_t far[2], lastc[2], total[2], thr[2];
  uint32_t pops, explored, ignored, peakq;
};
__device__ __forceinline__ void wctl_to_ctl(const WCtl& W, Lo<Ctl>& ctl) {
  if (threadIdx.x == 0) {
    ctl.nfree = W.nfree;
    ctl.n_ret = W.n_ret;
    ctl.max_err = W.max_err;
    ctl.status = W.status;
    ctl.hot_slot = W.hot;
  }
  __syncthreads();
}
__device__ __forceinline__ void wctl_from_ctl(WCtl& W, Lo<Ctl>& ctl) {
  W.nfree = uni(ctl.nfree);
  W.n_ret = uni(ctl.n_ret);
  W.max_err = ((uint64_t)uni((uint32_t)(ctl.max_err >> 32)) << 32) | uni((uint32_t)ctl.max_err);
  W.status = uni(ctl.status);
  W.hot = uni(ctl.hot_slot);
}
// the pop counters (uniform) and the lanes' work counters into Ctl's u64
// counters: every 16,384 pops (a lane's w_out grows by at most 2 wcap + 1 per
// pop) and at the end of the problem
__device__ __forceinline__ void wave_flush_counters(Lo<Ctl>& ctl, WCtl& W, uint32_t (&lcnt)[3]) {
  const uint32_t u = wave_sum_u32(lcnt[0]), wo = wave_sum_u32(lcnt[1]), cm = wave_sum_u32(lcnt[2]);
  if (threadIdx.x == 0) {  // (the pop counters: every wave holds the same)
    ctl.cnt[S_POPS] += W.pops;
    ctl.cnt[S_EXPLORED] += W.explored;
    ctl.cnt[S_IGNORED] += W.ignored;
  }
  if (kCoop) {  // (each wave's reads)
    if (lane_id() == 0) {
      atomicAdd((unsigned long long*)&ctl.cnt[S_UPDATES], (unsigned long long)u);
      atomicAdd((unsigned long long*)&ctl.cnt[S_WOUT], (unsigned long long)wo);
      atomicAdd((unsigned long long*)&ctl.cnt[S_COMPARES], (unsigned long long)cm);
    }
  } else if (threadIdx.x == 0) {
    ctl.cnt[S_UPDATES] += u;
    ctl.cnt[S_WOUT] += wo;
    ctl.cnt[S_COMPARES] += cm;
  }
  W.pops = W.explored = W.ignored = 0;
  lcnt[0] = lcnt[1] = lcnt[2] = 0;
}
// priority-queue 1.x on the LDS heap with the size in a register: the
// reference's sift rules (strict comparisons), with the
// path's entries compared by lanes in parallel instead of one level at a time.
__device__ __forceinline__ HeapEntry heap_uni(const HeapEntry& e);
__device__ __forceinline__ uint64_t heap_cost(const HeapEntry& e) { return e.cost; }
// push (sift-up): e enters at position n and moves up while its parent has a
// lower priority. The ancestors' priorities never decrease going up (the heap
// property), so the ancestors e passes are exactly a prefix of the path: lane
// k reads ancestor k + 1 levels up, one ballot finds how many e passes, and
// those move one level down in one parallel store.
__device__ __forceinline__ void wheap_push(Sh<HeapEntry>* h, uint32_t n, HeapEntry e) {
  const uint32_t lane = (uint32_t)lane_id();
  const uint32_t depth = 31u - (uint32_t)__builtin_clz(n + 1);  // ancestors of position n
  bool less = false;
  uint32_t child = 0;
  HeapEntry a{};
  if (lane < depth) {
    const uint32_t anc = ((n + 1) >> (lane + 1)) - 1;
    child = ((n + 1) >> lane) - 1;
    a = h[anc];
    less = prio_less(a, e);
  }
  const uint64_t m = ballot(less);
  const uint32_t k = (uint32_t)__builtin_ctzll(~m);  // ancestors e moves past
  if (lane < k) h[child] = a;
  if (lane == 0) h[((n + 1) >> k) - 1] = e;
}
// pop: the root leaves, the last entry x (at position n after the pop) sifts
// down from the root. At node i the larger child (left on ties) takes i's
// place while x has a lower priority than it. Lanes compute that decision
// for the nodes of the top levels in parallel; the path is then a walk over
// two ballot masks, and the entries on it move up in one parallel store.
// Below the top levels (heaps of more than 63 entries) the walk goes on
// level by level.
__device__ __forceinline__ HeapEntry wheap_pop(Sh<HeapEntry>* h, uint32_t n) {
  const uint32_t lane = (uint32_t)lane_id();
  const HeapEntry top = heap_uni(h[0]);
  const HeapEntry x = heap_uni(h[n]);
  if (n <= 1) {
    if (lane == 0) h[0] = x;
    return top;
  }
  // node `lane` of the top 63: its larger child and whether x moves past it
  bool go = false, right = false;
  HeapEntry cm{};
  {
    const uint32_t l = 2 * lane + 1, r = 2 * lane + 2;
    if (lane < 63 && l < n) {
      const HeapEntry hl = h[l];
      cm = hl;
      if (r < n) {
        const HeapEntry hr = h[r];
        if (prio_less(hl, hr)) {
          right = true;
          cm = hr;
        }
      }
      go = prio_less(x, cm);
    }
  }
  const uint64_t gm = ballot(go), rm = ballot(right);
  uint64_t path = 0;  // nodes (< 64) whose entry is replaced by their larger child's
  uint32_t i = 0;
  while (i < 63 && ((gm >> i) & 1ull)) {
    path |= 1ull << i;
    i = 2 * i + 1 + (uint32_t)((rm >> i) & 1ull);
  }
  if ((path >> lane) & 1ull) h[lane] = cm;
  if (i >= 63) {
    // deeper levels, one at a time (x is still moving)
    for (;;) {
      const uint32_t l = 2 * i + 1, r = 2 * i + 2;
      uint32_t largest = i;
      HeapEntry best = x;
      if (l < n) {
        const HeapEntry hl = heap_uni(h[l]);
        const HeapEntry hr = heap_uni(h[r < n ? r : l]);
        if (prio_less(best, hl)) {
          largest = l;
          best = hl;
        }
        if (r < n && prio_less(best, hr)) {
          largest = r;
          best = hr;
        }
      }
      if (largest == i) break;
      if (lane == 0) h[i] = best;
      i = largest;
    }
  }
  if (lane == 0) h[i] = x;
  return top;
}
__device__ __forceinline__ HeapEntry heap_uni(const HeapEntry& e) {
  HeapEntry u;
  u.cost = ((uint64_t)uni((uint32_t)(e.cost >> 32)) << 32) | uni((uint32_t)e.cost);
  u.len = uni(e.len);
  u.slot = uni(e.slot);
  return u;
}
// push(e) and then pop() on a heap of n entries: true when that pair returns
// e and leaves every entry where it was, so the caller can skip both (the
// in-place child of a pop is most often the next pop). The push takes e to
// the root iff it beats the root strictly (ancestors of strictly lower
// priority move down one level along its path). The pop then sifts x, the
// entry the push moved into position n (n's parent's), down from the root; it
// retraces the path, putting every moved entry back, iff at each ancestor the
// path child is the child the sift picks (the larger, the left one on ties)
// and x has strictly lower priority than it. (At n's parent x stops by the
// heap property.) Lane k checks ancestor k + 1 levels above n.
__device__ __forceinline__ bool wheap_push_pop_noop(const Sh<HeapEntry>* h, uint32_t n, const HeapEntry& e) {
  if (n == 0) return true;
  if (!prio_less(heap_uni(h[0]), e)) return false;
  const uint32_t lane = (uint32_t)lane_id();
  const uint32_t depth = 31u - (uint32_t)__builtin_clz(n + 1);  // ancestors of position n
  const HeapEntry x = heap_uni(h[((n + 1) >> 1) - 1]);
  bool bad = false;
  if (lane >= 1 && lane < depth) {
    const uint32_t anc = ((n + 1) >> (lane + 1)) - 1;  // (moved down to pc by the push)
    const uint32_t pc = ((n + 1) >> lane) - 1;          // its child on the path
    const uint32_t sib = (pc & 1u) ? pc + 1 : pc - 1;
    const HeapEntry a = h[anc];
    bool path = true;
    if (sib < n) {
      const HeapEntry b = h[sib];
      path = (pc & 1u) ? !prio_less(a, b) : prio_less(b, a);
    }
    bad = !path || !prio_less(x, a);
  }
  return ballot(bad) == 0;
}

// ---- the in-place child of a one-child pop (dual_build_children for nc == 1,
// no activate_dual): pushes on the hot state, ED increases through the slot
// (out of line), prune + cost + Some counts in one lane pass; new tip bytes
// into tx. Returns the child's cost; its metadata goes to the slot. ----
template <int R, int V>
__device__ __forceinline__ uint64_t wave_push_fast(Eng& E, Lo<Ctl>& ctl, KArgs kp, WCtl& W, uint32_t top,
                                                   const SlotMeta& tm, bool tdual, uint32_t kind, const int (&sy)[2],
                                                   const LaneReads<R>& lr, Tips (&tx)[R][2], uint32_t (&nl)[2],
                                                   uint32_t (&lcnt)[3]) {
  const int lane = lane_id();
  const DevConfig& cfg = E.cfg;
  const bool early = cfg.early != 0;
  const uint32_t n = E.n;
  // the child's symbols, locks and lengths (the metadata goes out with its
  // Some counts below)
  SlotMeta m = tm;
#pragma unroll
  for (int sd = 0; sd < 2; ++sd) {
    if (sy[sd] >= 0) {
      m.len[sd]++;  // (the consensus byte is stored after the lane pass)
    } else if (kind == 0) {
      m.flags |= (sd == 0 ? 2u : 4u);  // lock_sequence
    }
  }
  nl[0] = m.len[0];
  nl[1] = m.len[1];
  uint32_t upd = 0, wout = 0, cmps = 0, nheavy = 0;
  uint32_t ee[R][2];  // the child's edit distances (kInactive = None)
  // (coop: each wave lists its heavy items in its own part of the list)
  const uint32_t hbase = kCoop ? (uint32_t)wave_id() * 2u * 64u : 0u;
  SUB_T0(t_pl);
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const uint32_t r = read_base() + (uint32_t)lane + 64u * j;
    const bool live = r < n;
#pragma unroll
    for (int sd = 0; sd < 2; ++sd) {
      bool heavy = false;
      ee[j][sd] = kInactive;
      if (live && (sd == 0 || tdual)) {
        Sh<RState>* hp = &E.L.hot[sd * E.nmax + r];
        const RRaw s = rstate_load(hp);
        ee[j][sd] = rraw_e(s);
        if (rraw_e(s) != kInactive && sy[sd] >= 0) {
          if (rraw_flags(s) & kWide) {
            heavy = true;  // (wave_heavy's full-scan push)
          } else {
            Front f;
            front_load(s, f);
            uint32_t x[kF];
            tips_unpack(tx[j][sd], x);
            uint32_t cmp = 0;
            heavy = thread_apply<kLazyRows>(f, x, lr.bl[j], nl[sd] - 1, (uint8_t)sy[sd], cfg.wildcard, early,
                                 E.sv(top, sd).wf + (uint64_t)r * E.wcap, cmp);
            cmps += cmp;
            front_store(hp, f);  // (a heavy read's ED-increase loop goes on from it)
            if (!heavy) {
              upd++;
              wout += 2 * f.e + 1;
              ee[j][sd] = f.e;
              tx[j][sd] = tips_fetch(f, lr.rd[j], lr.bl[j], nl[sd]);
            }
          }
        }
      }
      // heavy items into the work list (ballot prefix, no atomics)
      const uint64_t hm = ballot(heavy);
      if (heavy) {
        const uint32_t k = nheavy + (uint32_t)__popcll((unsigned long long)(hm & ((1ull << lane) - 1ull)));
        E.L.list[WC_IX(hbase + k, list_entries(E.sides, E.nmax))] = sd * n + r;
      }
      nheavy += (uint32_t)__popcll((unsigned long long)hm);
    }
  }
  // (per-lane work counters, summed over the wave once per problem)
  lcnt[0] += upd;
  lcnt[1] += wout;
  lcnt[2] += cmps;
  SUB_T1(48, t_pl);  // (push: the lane pass and its counters)
  // The consensus bytes, after the lane pass (which compares against sy, not
  // memory). The ED-increase loops below read them back: each wave stores
  // them itself (coop waves run those loops with no barrier) and, before the
  // loops, waits for its stores and invalidates the CU's vector L1, whose
  // copy of the line a byte store leaves stale (measured: without the
  // invalidate a 4-wave problem read the old byte and faulted; with the store
  // at the push's start instead, only the lane pass's traffic evicting the
  // line kept it right). The block code reads them later, after barriers.
#pragma unroll
  for (int sd = 0; sd < 2; ++sd)
    if (sy[sd] >= 0 && lane == 0) E.sv(top, sd).con[WC_IX(nl[sd] - 1, E.lcap)] = (uint8_t)sy[sd];
  uint32_t hovf = 0;  // (coop) this wave's ED-increase overflow bits, exchanged with the cost partials
  if (nheavy) {
    // the ED-increase loops, out of line; then the rebuilt states and their
    // tip bytes from the hot copy (coop: each wave its own reads', with no
    // barrier)
    SUB_CNT(53, 1);
    SUB_CNT(55, nheavy);
    SUB_T0(t_hv);
    con_store_wait();  // (this wave's consensus byte stores)
    l1_drop();
    if constexpr (!kCoop) {
      if (lane == 0) ctl.ovf = 0;
      __syncthreads();
    }
    {
      HeavyArgs<R> h;
      h.hot = E.L.hot;
      h.list = E.L.list;
      const SideView v0 = E.sv(top, 0), v1 = E.sv(top, tdual ? 1 : 0);
      h.wf[0] = v0.wf;
      h.wf[1] = v1.wf;
      h.con[0] = v0.con;
      h.con[1] = v1.con;
#pragma unroll
      for (int j = 0; j < R; ++j) {
        h.rd[j] = lr.rd[j];
        h.bl[j] = lr.bl[j];
      }
      h.list_cap = list_entries(E.sides, E.nmax);
      h.nmax = E.nmax;
      h.n = n;
      h.wcap = E.wcap;
      h.nl[0] = nl[0];
      h.nl[1] = nl[1];
      h.sy[0] = (uint32_t)sy[0];
      h.sy[1] = (uint32_t)sy[1];
      h.wc = cfg.wildcard;
      h.early = early ? 1u : 0u;
      hovf = wave_heavy_call<R, V>(h, ctl, hbase, nheavy);
    }
    SUB_T1(54, t_hv);
    const uint32_t ovf = kCoop ? 0u : uni(ctl.ovf);
    // (per-lane branches without continue, and the uniform status after
    // them: a join of lanes' paths that also carries search control makes
    // the compiler treat the whole pop loop's control state as divergent)
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const uint32_t r = read_base() + (uint32_t)lane + 64u * j;
#pragma unroll
      for (int sd = 0; sd < 2; ++sd) {
        if (r < n && !(sd == 1 && !tdual) && sy[sd] >= 0) {
          const RRaw s = rstate_load(&E.L.hot[sd * E.nmax + r]);
          if (!(ee[j][sd] == rraw_e(s) && ee[j][sd] != kInactive && !(rraw_flags(s) & kWide))) {
            ee[j][sd] = rraw_e(s);
            if (rraw_e(s) != kInactive && !(rraw_flags(s) & kWide)) {
              Front f;
              front_load(s, f);
              tx[j][sd] = tips_fetch(f, lr.rd[j], lr.bl[j], nl[sd]);
            }
          }
        }
      }
    }
    if (ovf & 16u) W.status = WC_E_INVARIANT_CODE;
    else if (ovf & 4u) W.status = ST_RETRY | ST_RETRY_WCAP;
    else if (ovf) W.status = limit_status(ovf);
  }
  // prune_dwfa (:1030-1045) of a dual child, then per read the cheaper side's
  // cost (strict <: ties keep consensus 1, :1092-1131) and the Some counts
  SUB_T0(t_pc);
  uint64_t cost = 0;
  uint32_t c0 = 0, c1 = 0;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const uint32_t r = read_base() + (uint32_t)lane + 64u * j;
    if (r >= n) continue;
    uint32_t e1 = ee[j][0];
    uint32_t e2 = tdual ? ee[j][1] : kInactive;
    if (tdual && e1 != kInactive && e2 != kInactive) {
      if ((uint64_t)e1 + cfg.dual_max_ed_delta < (uint64_t)e2) {
        E.L.hot[E.nmax + r].e = kInactive;
        e2 = kInactive;
      } else if ((uint64_t)e2 + cfg.dual_max_ed_delta < (uint64_t)e1) {
        E.L.hot[r].e = kInactive;
        e1 = kInactive;
      }
    }
    uint64_t best = ~0ull;
    if (e1 != kInactive) best = cost_of(e1, cfg.cost_mode);
    if (e2 != kInactive && cost_of(e2, cfg.cost_mode) < best) best = cost_of(e2, cfg.cost_mode);
    if (best != ~0ull) cost += best;
    c0 += e1 != kInactive;
    c1 += e2 != kInactive;
  }
  cost = wave_sum_u64(cost);
  uint32_t cc = wave_sum_u32(c0 | (c1 << 16));  // (<= 256 reads a side)
  if constexpr (kCoop) {  // the partial sums and overflow bits of every wave
    if (lane == 0) {
      coopx().cost[wave_id()] = cost;
      coopx().cc[wave_id()] = cc;
      coopx().nh[wave_id()] = hovf;
    }
    __syncthreads();
    cost = 0;
    cc = 0;
    uint32_t ovf = 0;
#pragma unroll
    for (int w = 0; w < kEW; ++w) {
      cost += ((uint64_t)uni((uint32_t)(coopx().cost[w] >> 32)) << 32) | uni((uint32_t)coopx().cost[w]);
      cc += uni(coopx().cc[w]);
      ovf |= uni(coopx().nh[w]);
    }
    if (ovf & 16u) W.status = WC_E_INVARIANT_CODE;
    else if (ovf & 4u) W.status = ST_RETRY | ST_RETRY_WCAP;
    else if (ovf) W.status = limit_status(ovf);
  }
  m.nsome[0] = cc & 0xFFFFu;
  m.nsome[1] = cc >> 16;
  if (threadIdx.x == 0) meta_put(E.L.meta[top], m);
  SUB_T1(49, t_pc);  // (push: prune, cost, Some counts)
  return cost;
}

// ---- the votes of one node side on the lean path (consensus.rs:540-564,
// dual_consensus.rs:1242-1290): the keys (the wildcard dropped when it is not
// the only one, :556-561) with their votes, their sum and maximum, the
// threshold min(max(min_count, ceil(min_af * sum)), max) (:520-552), and the
// keys passing it. Votes are exact integers in units of 1/U of a read: U = 8
// when every split is 1, 2, 4 or 8 (the reference's f64 sums are then exact
// too), U = 840 = lcm(1..8) otherwise. With other splits the reference's f64
// sums round; they decide the same as the exact values unless two of the
// compared quantities are exactly equal (a tie at the maximum, or a vote equal
// to min_count), so those sides are left to the block engines' f64 votes
// (exact = false), as are min_af > 0 with other splits. With one child the
// order of the keys (hashbrown) decides nothing, so none is computed. ----
struct SideVotes {
  uint32_t npass, nkeys;  // keys passing the threshold, keys
  int pk;                 // a passing key (the one, when npass == 1)
  bool split;             // single-consensus node: two candidates pass min_count (split children)
  bool exact;             // false: decide with the block engines' f64 votes
};
template <int R>
__device__ __forceinline__ SideVotes wave_side_votes(const DevConfig& cfg, const uint32_t (&ys)[R],
                                                     const uint64_t (&mmask)[R], const NomRaw (&mn)[R], bool odd) {
  const int wc = cfg.wildcard;
  // the common case: every voter nominates one symbol, the same one
  {
    uint64_t vm[R], any = 0, mm = 0;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      vm[j] = ballot(ys[j] != 0x100u);
      any |= vm[j];
      mm |= mmask[j];
    }
    if (!mm) {
      if (!any) {  // no key: no option but None; thr (unused) from min_count
        return SideVotes{0, 0, -1, false, true};
      }
      uint32_t first = 0x100u;
#pragma unroll
      for (int j = 0; j < R; ++j)
        if (first == 0x100u && vm[j]) first = (uint32_t)__builtin_amdgcn_readlane((int)ys[j], __builtin_ctzll(vm[j]));
      bool same = true;
#pragma unroll
      for (int j = 0; j < R; ++j) same = same && ballot(ys[j] == first) == vm[j];
      if (same) {
        // one key, not dropped (it is the only one); it passes min(mc, its own count)
        return SideVotes{1, 1, (int)first, false, true};
      }
    }
  }
  if (odd && cfg.min_af != 0.0) return SideVotes{0, 0, -1, false, false};
  const uint32_t U = odd ? 840u : 8u;
  // the distinct keys one at a time (single-symbol voters first, by ballots;
  // then the symbols of multi-symbol voters not counted yet, lanes in
  // parallel), each with its vote in units of 1/U; lane k keeps key k and its
  // vote for the threshold pass
  uint64_t rem[R];
  uint32_t mrem[R];  // per lane: its multi-symbol slots not counted yet
  uint32_t mul[R];   // per lane: U / split (units per occurrence)
  bool any_multi = false, big = false;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    rem[j] = ballot(ys[j] != 0x100u);
    mrem[j] = 0;
    const uint32_t split = max(mn[j].meta >> 16, 1u);
    mul[j] = U / split;
    if ((mmask[j] >> lane_id()) & 1ull) {
      mrem[j] = (1u << (mn[j].meta & 0xFFu)) - 1u;  // (slots < nk hold a symbol)
      big |= split > 8u;                            // (never: at most kF = 8 tips)
    }
    any_multi |= mmask[j] != 0;
  }
  if (ballot(big)) return SideVotes{0, 0, -1, false, false};
  // symbols per multi-symbol voter, at most (the slot loops below stop there)
  uint32_t kmax = 0;
#pragma unroll
  for (int j = 0; j < R; ++j) kmax = max(kmax, mrem[j] ? 32u - (uint32_t)__builtin_clz(mrem[j]) : 0u);
  kmax = any_multi ? wave_max_u32(kmax) : 0u;
  uint32_t nk = 0, total = 0, mx_all = 0, mx_nowc = 0, wcv = 0;
  bool wc_in = false;
  uint32_t tkey = 0x100u, tc = 0;  // lane k: key k and its vote
  for (;;) {
    uint32_t key = 0x100u;
#pragma unroll
    for (int j = 0; j < R; ++j)
      if (key == 0x100u && rem[j]) key = (uint32_t)__builtin_amdgcn_readlane((int)ys[j], __builtin_ctzll(rem[j]));
    if (key == 0x100u && any_multi) {
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const uint64_t lm = ballot(mrem[j] != 0u);
        if (key == 0x100u && lm) {
          const int l = __builtin_ctzll(lm);
          const uint32_t k = (uint32_t)__builtin_ctz((uint32_t)__builtin_amdgcn_readlane((int)mrem[j], l));
          const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)(k < 4 ? mn[j].klo : mn[j].khi), l);
          key = (w >> (8 * (k & 3))) & 0xFFu;
        }
      }
    }
    if (key == 0x100u) break;
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const uint64_t m = ballot(ys[j] == key);
      c += U * (uint32_t)__popcll((unsigned long long)m);
      rem[j] &= ~m;
    }
    if (any_multi) {
      uint32_t mine = 0;
#pragma unroll
      for (int j = 0; j < R; ++j) {
        uint32_t occ = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if ((uint32_t)k >= kmax) break;
          const uint32_t sk = ((k < 4 ? mn[j].klo : mn[j].khi) >> (8 * (k & 3))) & 0xFFu;
          if (((mrem[j] >> k) & 1u) && sk == key) {
            occ += (mn[j].cnt >> (4 * k)) & 15u;
            mrem[j] &= ~(1u << k);
          }
        }
        mine += occ * mul[j];
      }
      c += wave_sum_u32(mine);
    }
    if (lane_id() == (int)nk) {
      tkey = key;
      tc = c;
    }
    nk++;
    total += c;
    mx_all = max(mx_all, c);
    if (wc >= 0 && key == (uint32_t)(uint8_t)wc) {
      wc_in = true;
      wcv = c;
    } else {
      mx_nowc = max(mx_nowc, c);
    }
  }
  const bool drop = wc_in && nk > 1;
  const uint32_t nko = drop ? nk - 1 : nk;
  const uint32_t sum = drop ? total - wcv : total;
  const uint32_t mx = drop ? mx_nowc : mx_all;
  // min_count (and min_af * sum, exact for U = 8) in units; saturated far
  // above any vote (<= 128 reads)
  const uint64_t mc = max(cfg.min_count, odd ? 0ull : ceil_u64(cfg.min_af * ((double)sum * 0.125)));
  const uint64_t mcu = mc > (1ull << 32) ? (1ull << 48) : mc * U;
  const uint64_t thr = nko ? min(mcu, (uint64_t)mx) : mcu;
  // the threshold pass (:520-552, :655-679), key k on lane k
  const bool is_wc = wc >= 0 && tkey == (uint32_t)(uint8_t)wc;
  const bool valid = lane_id() < (int)nk && !(drop && is_wc);
  if (odd && (__popcll((unsigned long long)ballot(valid && tc == mx)) > 1 || ballot(valid && (uint64_t)tc == mcu) != 0))
    return SideVotes{0, 0, -1, false, false};
  const uint64_t pm = ballot(valid && (uint64_t)tc >= thr);
  const uint32_t np = (uint32_t)__popcll((unsigned long long)pm);
  const int pk = pm ? (int)__builtin_amdgcn_readlane((int)tkey, __builtin_ctzll(pm)) : -1;
  const uint32_t ns = (uint32_t)__popcll((unsigned long long)ballot(valid && !is_wc));
  const uint32_t npmc = (uint32_t)__popcll((unsigned long long)ballot(valid && !is_wc && (uint64_t)tc >= mcu));
  return SideVotes{np, nko, pk, npmc > 1 && ns > 1, true};
}

// ---- the search: dual_main's pop, with a lean path for the common pop ----
// The common pop (no read at a consensus end, no wide frontier, unweighted
// votes whose per-read splits are 1, 2, 4 or 8 tips, and exactly one child
// that pushes in place) runs below with the search control in registers:
// analysis on the hot state and prefetched tip bytes, the votes as exact
// counts of eighths (ballots), the selection on them (with one child the
// hashbrown order of the keys decides nothing), the lane push. Anything else
// goes to wave_rare's WR_GENERAL*, the block engines' code for the rest of
// the pop.
template <int R, int V>
__device__ __forceinline__ void wave_problem(const EngineArgs& A, Eng& E, Lo<Ctl>& ctl, uint32_t prob, uint32_t oslot,
                                             Gm<uint8_t>* outp) {
  const int lane = lane_id();
  const DevConfig& cfg = A.cfg;
  const bool early = cfg.early != 0;
  const bool weighted = cfg.weighted != 0;
  Sh<RInfo>* R0 = E.L.rinfo;
  Sh<RInfo>* R1 = E.L.rinfo + E.nmax;
  Tips tx[R][2];
#pragma unroll
  for (int j = 0; j < R; ++j) tx[j][0] = tx[j][1] = Tips{0, 0, 0};
  const uint64_t full_min = max(cfg.min_count, ceil_u64(cfg.min_af * (double)E.n));
  // active_min_count (:497-513) without activations: the root's count at
  // every length below am_len
  const uint64_t am0 = full_min;
  bool tips_ok = false;  // tx holds the hot node's tip bytes
  // (written out: a loop here was not unrolled, which would leave lr in scratch)
  LaneReads<R> lr;
  {
    const uint32_t r0 = read_base() + (uint32_t)lane;
    lr.rd[0] = E.rbytes + (r0 < E.n ? E.roff[E.P.read_begin + r0] : 0ull);
    lr.bl[0] = r0 < E.n ? E.rlenp[E.P.read_begin + r0] : 0u;
    if constexpr (R > 1) {
      const uint32_t r1 = (uint32_t)lane + 64u;
      lr.rd[1] = E.rbytes + (r1 < E.n ? E.roff[E.P.read_begin + r1] : 0ull);
      lr.bl[1] = r1 < E.n ? E.rlenp[E.P.read_begin + r1] : 0u;
    }
    if constexpr (R > 2) {
      const uint32_t r2 = (uint32_t)lane + 128u, r3 = (uint32_t)lane + 192u;
      lr.rd[2] = E.rbytes + (r2 < E.n ? E.roff[E.P.read_begin + r2] : 0ull);
      lr.bl[2] = r2 < E.n ? E.rlenp[E.P.read_begin + r2] : 0u;
      lr.rd[3] = E.rbytes + (r3 < E.n ? E.roff[E.P.read_begin + r3] : 0ull);
      lr.bl[3] = r3 < E.n ? E.rlenp[E.P.read_begin + r3] : 0u;
    }
  }
  const KArgs kp = kernel_args();
  Sh<uint8_t>* const sbase = (Sh<uint8_t>*)E.L.hot;
  // init_problem left: the root in the heap and tracker 0, slot 0 taken
  WCtl W;
  W.heap_n = 1;
  W.nfree = E.pcap - 1;
  W.hot = kNoSlot;
  W.hot_dual = 0;
  W.am_len = 1;
  W.n_ret = 0;
  W.status = ST_OK;
  W.max_err = ~0ull;
  W.far[0] = W.far[1] = W.lastc[0] = W.lastc[1] = W.thr[0] = W.thr[1] = 0;
  W.total[0] = 1;
  W.total[1] = 0;
  W.pops = W.explored = W.ignored = W.peakq = 0;
  uint32_t lcnt[3] = {0, 0, 0};  // this lane's updates, w_out, compares (wave_push_fast)
  const uint64_t L2 = E.lcap + 2;
  Gm<uint32_t>* const lc[2] = {E.trk, E.trk + 2 * L2};
  Gm<uint32_t>* const pc[2] = {E.trk + L2, E.trk + 3 * L2};
  const uint64_t cap = cfg.max_capacity_per_size;
  // the tracker limits against 32-bit totals (a total above 2^32 - 1 never exceeds a larger limit)
  const uint32_t mqs32 = (uint32_t)min(cfg.max_queue_size, (uint64_t)0xFFFFFFFFu);
  const uint32_t mnc32 = (uint32_t)min(cfg.max_nodes_wo_constraint, (uint64_t)0xFFFFFFFFu);

  uint32_t pb = 0;  // (coop) pop parity: which hand-off buffer of the popped node
  // the last pop's in-place child when pushing it and popping it again would
  // leave the heap as it was (wheap_push_pop_noop): it is the next top, and
  // the heap is not touched (every wave holds the same)
  bool stashed = false;
  HeapEntry stash{};
  uint32_t stash_k = 0;  // its tracker (1: dual)
  for (;;) {
    // ---- pop (dual_consensus.rs:340-397) ----
    if (W.heap_n == 0) break;
    if constexpr (kCoop) {
      // wave 0 pops (after its own writes of the last pop: heap, trackers,
      // metadata), every wave takes the node from Ctl after the barrier (the
      // other waves read the heap only when no wave writes it: between this
      // barrier and the push)
      if (!stashed) {
        if (wave_id() == 0) {
          const HeapEntry t = wheap_pop(E.L.heap, W.heap_n - 1);
          if (lane == 0) {
            coopx().top_cost[pb] = t.cost;
            coopx().top_len[pb] = t.len;
            coopx().top_slot[pb] = t.slot;
          }
        }
        __syncthreads();
      }
    }
    SUB_T0(t_pl);
    uint32_t plen;
    if (stashed) plen = stash.len;
    else if constexpr (kCoop) plen = uni(coopx().top_len[pb]);
    else plen = uni(E.L.heap[0].len);
    // the processed counts of the top's length, loaded first (HBM, under
    // one wait) while the threshold walks and the sift run
    const uint32_t pc_pre0 = trk_load(&pc[0][WC_IX(plen, L2)]), pc_pre1 = trk_load(&pc[1][WC_IX(plen, L2)]);
    const uint64_t am = plen < W.am_len ? am0 : 0;
    W.peakq = max(W.peakq, W.heap_n);
    if (W.pops >= 0x4000u) {  // (the 32-bit counters into Ctl, long before they could wrap)
      wave_flush_counters(ctl, W, lcnt);
    }
    W.pops++;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      while ((W.total[k] > mqs32 || W.lastc[k] >= mnc32) && W.thr[k] < W.far[k]) {
        W.total[k] -= uni(trk_load(&lc[k][WC_IX(W.thr[k], L2)])) +  // increment_threshold
                      ((stashed && stash_k == (uint32_t)k && stash.len == W.thr[k]) ? 1u : 0u);
        W.thr[k]++;
        W.lastc[k] = 0;
      }
    }
    SUB_T1(45, t_pl);  // (pop-logic: to the heap pop)
    SUB_T0(t_hp);
    W.heap_n--;
    HeapEntry top;
    const bool from_stash = stashed;
    if (stashed) {
      top = stash;
      stashed = false;
    } else if constexpr (kCoop) {
      top.cost = ((uint64_t)uni((uint32_t)(coopx().top_cost[pb] >> 32)) << 32) | uni((uint32_t)coopx().top_cost[pb]);
      top.len = uni(coopx().top_len[pb]);
      top.slot = uni(coopx().top_slot[pb]);
      pb ^= 1u;
    } else {
      top = wheap_pop(E.L.heap, W.heap_n);
    }
    SUB_T1(46, t_hp);  // (pop-logic: the heap pop)
    SUB_T0(t_pc);
    const SlotMeta tm = meta_get(E.L.meta[top.slot]);
    const uint32_t dual = uni(tm.flags) & 1u;
    const uint32_t ns0 = uni(tm.nsome[0]), ns1 = uni(tm.nsome[1]);
    // tracker(dual).remove(len)
    // (the per-tracker fields by constant index only: a runtime index into
    // WCtl's arrays keeps the whole struct in scratch memory)
    const uint32_t thr_d = dual ? W.thr[1] : W.thr[0];
    if (threadIdx.x == 0 && !from_stash) atomicSub((uint32_t*)&(dual ? lc[1] : lc[0])[WC_IX(top.len, L2)], 1u);
    if (top.len >= thr_d) {
      if (dual) W.total[1]--;
      else W.total[0]--;
    }
    const bool imbalanced = dual && (ns0 < am || ns1 < am);
    if (top.len >= W.am_len) W.status = WC_E_INVARIANT_CODE;
    SUB_T1(47, t_pc);  // (pop-logic: metadata, tracker)
    // the node is ignored (:372-386) when it costs more than the best result,
    // lies below its tracker's threshold, is imbalanced, or its length is at
    // capacity; the capacity check waits for the processed count's load and
    // comes after the analysis below (nothing before it has an effect that
    // outlives an ignored node), so that load's latency overlaps it
    const bool ign = top.cost > W.max_err || top.len < thr_d || imbalanced;
    if (ign) {
      if (A.trace && threadIdx.x == 0) trace_pop(A, prob, top, dual | (1u << 1) | (ns0 << 8) | (ns1 << 20), (uint32_t)am);
      W.ignored++;
      if (threadIdx.x == 0) E.L.freestack[WC_IX(W.nfree, E.pcap)] = top.slot;
      W.nfree++;
      if (top.slot == W.hot) W.hot = kNoSlot;  // its state is dropped with the slot
      continue;
    }
    PH_MARK(13);

    const uint32_t topslot = top.slot;
    const uint32_t tlen = top.len;
    const bool tdual = dual != 0;
    const uint32_t tlens[2] = {uni(tm.len[0]), uni(tm.len[1])};
    const uint32_t tflags = uni(tm.flags);
    SUB_T0(t_hot);
    if (topslot != W.hot) {
      SUB_CNT(33, 1);
      // the previous hot node, still queued, goes back to its slot first
      if (W.hot != kNoSlot) hot_writeback<R>(E, W.hot, W.hot_dual != 0);
      hot_fetch_slot<R>(E, topslot, tdual);
      tips_ok = false;
      W.hot = topslot;
      W.hot_dual = tdual ? 1u : 0u;
    }
    SUB_T1(32, t_hot);

    // ---- analysis of both sides from the hot state: thread_analyze on the
    // prefetched tip bytes; the nominations also go to RInfo (the general
    // path reads them there) ----
    SUB_T0(t_an);
    uint32_t ys[2][R];  // the read's one nominated symbol (0x100: none, several, or not a voter)
    uint64_t mmask[2][R];  // lanes whose read nominates several symbols
    NomRaw mn[2][R];  // every read's nominations (RInfo is made from them only when needed)
    bool any_wide = false, any_end = false, any_multi = false, odd_split = false;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const uint32_t r = read_base() + (uint32_t)lane + 64u * j;
      const bool live = r < E.n;
#pragma unroll
      for (int sd = 0; sd < 2; ++sd) {
        ys[sd][j] = 0x100u;
        mn[sd][j] = NomRaw{0, 0, 0, 1u << 16, kInactive};
        bool wide = false, end = false, multi = false;
        if (live && (sd == 0 || tdual)) {
          const RRaw s = rstate_load(&E.L.hot[sd * E.nmax + r]);
          if (rraw_e(s) == kInactive) {
            // (mn: no DWFA)
          } else if (rraw_flags(s) & kWide) {
            wide = true;
          } else {
            Front f;
            front_load(s, f);
            if (!tips_ok) tx[j][sd] = tips_fetch(f, lr.rd[j], lr.bl[j], tlens[sd]);
            uint32_t x[kF];
            tips_unpack(tx[j][sd], x);
            const NomRaw o = nominate_raw(f, x, lr.bl[j]);
            mn[sd][j] = o;
            const uint32_t nk = o.meta & 0xFFu, split = o.meta >> 16;
            end = (o.meta & 256u) != 0;
            multi = nk > 1;
            if (nk == 1) ys[sd][j] = o.klo & 0xFFu;
            if (multi && (split > 8u || (split & (split - 1u)))) odd_split = true;
          }
        }
        mmask[sd][j] = ballot(multi);
        any_wide |= ballot(wide) != 0;
        any_end |= ballot(end) != 0;
        any_multi |= mmask[sd][j] != 0;
      }
    }
    odd_split = ballot(odd_split) != 0;
    if constexpr (kCoop) {
      // every wave's nominations (the votes read every read's) and flags
      const uint32_t r = read_base() + (uint32_t)lane;
      if (r < E.n) {
        nom_put(R0 + r, mn[0][0]);
        if (tdual) nom_put(R1 + r, mn[1][0]);
      }
      if (lane == 0)
        coopx().flags[wave_id()] = (any_wide ? 1u : 0u) | (any_end ? 2u : 0u) | (any_multi ? 4u : 0u) | (odd_split ? 8u : 0u);
      __syncthreads();
      uint32_t fw = 0;
#pragma unroll
      for (int w = 0; w < kEW; ++w) fw |= uni(coopx().flags[w]);
      any_wide = fw & 1u;
      any_end = (fw & 2u) != 0;
      any_multi = (fw & 4u) != 0;
      odd_split = (fw & 8u) != 0;
    }
    tips_ok = true;
    SUB_T1(34, t_an);
    {
      const bool at_cap = uni(dual ? pc_pre1 : pc_pre0) >= cap;
      if (A.trace && threadIdx.x == 0)
        trace_pop(A, prob, top, dual | ((at_cap ? 1u : 0u) << 1) | (ns0 << 8) | (ns1 << 20), (uint32_t)am);
      if (at_cap) {
        W.ignored++;
        if (threadIdx.x == 0) E.L.freestack[WC_IX(W.nfree, E.pcap)] = topslot;
        W.nfree++;
        W.hot = kNoSlot;  // (the hot node: its state is dropped with the slot)
        continue;
      }
    }
    if (dual) {
      W.far[1] = max(W.far[1], top.len);
      W.lastc[1] += W.lastc[1] != 0xFFFFFFFFu;
    } else {
      W.far[0] = max(W.far[0], top.len);
      W.lastc[0] += W.lastc[0] != 0xFFFFFFFFu;
    }
    if (threadIdx.x == 0) atomicAdd((uint32_t*)&(dual ? pc[1] : pc[0])[WC_IX(top.len, L2)], 1u);  // process_unchecked
    W.explored++;
    if (W.status != ST_OK) break;
    // active_min_count growth (:497-513): the count at every new length is
    // the root's (no activation in this build)
    if (W.am_len == tlen + 1 && tlen + 1 < E.lcap + 2) W.am_len++;
    PH_MARK(1);

    uint32_t nchild = 2;  // (0 or 1: decided on the lean path)
    int child[2] = {-1, -1};
    uint32_t kind = tdual ? 0u : 1u;
    uint32_t nc = 1;
    uint64_t ccost = 0;
    uint32_t clen = 0;
    bool general = false;  // children from Ctl (the block engines' passes)
    if (any_wide || any_end) {
      // wide frontiers or a read at a consensus end (finalize, reached_*):
      // the block engines' code for the rest of the pop, from the slot
      SUB_CNT(35, 1);
      if (threadIdx.x == 0) {
        ctl.n_end[0] = ctl.n_end[1] = 0;
        ctl.n_either = 0;
        ctl.nheavy = 0;
        ctl.ovf = 0;
        ctl.multi[0] = ctl.multi[1] = 0;
      }
      wctl_to_ctl(W, ctl);
      wave_rare<R, V>(kp, E.P, sbase, ctl, WR_GENERAL_POP, topslot, tdual, (uint32_t)full_min,
                   (uint32_t)(full_min >> 32), oslot, 0, 0);
      wctl_from_ctl(W, ctl);
      W.hot = kNoSlot;
      if (W.status != ST_OK) break;
      nc = uni(ctl.nchild);
      general = true;
    } else {
      SideVotes sv0 = {0, 0, -1, false, false}, sv1 = {0, 0, -1, false, true};
      if (!weighted) {
        if constexpr (kCoop) {
          // every read's nominations, read w * 64 + lane as this lane's w-th
          // (the single-wave build's two-reads-per-lane arrays, kEW of them)
          auto side_votes = [&](const Sh<RInfo>* Rs) {
            uint32_t ysA[kEW];
            uint64_t mmA[kEW];
            NomRaw mnA[kEW];
#pragma unroll
            for (int w = 0; w < kEW; ++w) {
              const uint32_t r = 64u * (uint32_t)w + (uint32_t)lane;
              const NomRaw o = r < E.n ? nom_get(Rs + r) : NomRaw{0, 0, 0, 1u << 16, kInactive};
              const uint32_t nk = o.meta & 0xFFu;
              ysA[w] = nk == 1 ? (o.klo & 0xFFu) : 0x100u;
              mmA[w] = ballot(nk > 1);
              mnA[w] = o;
            }
            return wave_side_votes<kEW>(cfg, ysA, mmA, mnA, odd_split);
          };
          sv0 = side_votes(R0);
          if (tdual && sv0.exact) sv1 = side_votes(R1);
        } else {
          sv0 = wave_side_votes<R>(cfg, ys[0], mmask[0], mn[0], odd_split);
          if (tdual && sv0.exact) sv1 = wave_side_votes<R>(cfg, ys[1], mmask[1], mn[1], odd_split);
        }
      }
      if (sv0.exact && sv1.exact) {
        // ---- votes and selection on the lean path ----
        SUB_T0(t_v);
        uint32_t npass[2] = {sv0.npass, sv1.npass};
        const uint32_t nkeys[2] = {sv0.nkeys, sv1.nkeys};
        const int pkey[2] = {sv0.pk, sv1.pk};
        if (tdual) {
          // options per side: None first (consensus end, no keys, locked),
          // then the passing keys; children = pairs but (None, None)
          // (dual_consensus.rs:554-650)
          bool has_none[2];
          uint32_t no[2];
#pragma unroll
          for (int sd = 0; sd < 2; ++sd) {
            const bool lock = (tflags & (sd == 0 ? 2u : 4u)) != 0;
            const bool fin = early && (sd == 0 ? ns0 : ns1) == 0;  // (no read at its end here)
            has_none[sd] = fin || nkeys[sd] == 0 || lock;
            if (lock) npass[sd] = 0;
            no[sd] = (has_none[sd] ? 1u : 0u) + npass[sd];
          }
          nchild = no[0] * no[1] - ((has_none[0] && has_none[1]) ? 1u : 0u);
          child[0] = npass[0] ? pkey[0] : -1;
          child[1] = npass[1] ? pkey[1] : -1;
        } else {
          // stay-single children, and split children from every pair of
          // candidates when two pass min_count (:655-734)
          nchild = npass[0] + (sv0.split ? 2u : 0u);
          child[0] = pkey[0];
        }
        SUB_T1(38, t_v);
      }
      if (nchild >= 2) {
        // weighted votes, rounding f64 votes at a tie, or several children
        // (their order): the block engines' votes and selection (from RInfo)
        SUB_CNT((!sv0.exact || !sv1.exact) ? 36 : 39, 1);
        if (threadIdx.x == 0) {
          ctl.ovf = 0;
          ctl.multi[0] = ctl.multi[1] = any_multi ? 1u : 0u;
          ctl.fin[0] = early && ns0 == 0;
          ctl.fin[1] = tdual && early && ns1 == 0;
          ctl.status = W.status;
        }
        // the block engines' votes read RInfo: made here, with the order of
        // several symbols, only for these pops (coop: over the nominations the
        // other waves may still be reading)
        coop_sync();
#pragma unroll
        for (int j = 0; j < R; ++j) {
          const uint32_t r = read_base() + (uint32_t)lane + 64u * j;
          if (r < E.n) {
            rinfo_from_raw(R0 + r, mn[0][j]);
            if (tdual) rinfo_from_raw(R1 + r, mn[1][j]);
          }
        }
        __syncthreads();
        wave_rare<R, V>(kp, E.P, sbase, ctl, WR_VOTES_SELECT, topslot, tdual, 0, 0, 0, 0, 0);
        W.status = uni(ctl.status);
        if (W.status != ST_OK) break;
        nchild = uni(ctl.nchild);
        if (nchild == 1) {
          child[0] = uni((int32_t)ctl.ch_s[0][0]);
          child[1] = uni((int32_t)ctl.ch_s[0][1]);
          kind = uni((uint32_t)ctl.ch_kind[0]);
        }
      }
      if (nchild == 0) {
        if (threadIdx.x == 0) E.L.freestack[WC_IX(W.nfree, E.pcap)] = topslot;
        W.nfree++;
        W.hot = kNoSlot;
        PH_MARK(3);
        continue;
      }
      if (tlens[0] + 1 > E.lcap || tlens[1] + 1 > E.lcap) {
        W.status = ST_RETRY | ST_RETRY_LCAP;
        break;
      }
      PH_MARK(3);
      if (nchild == 1 && kind != 2) {
        SUB_CNT(37, 1);
        uint32_t nl[2];
        ccost = wave_push_fast<R, V>(E, ctl, kp, W, topslot, tm, tdual, kind, child, lr, tx, nl, lcnt);
        clen = max(nl[0], nl[1]);
        if (W.status != ST_OK) break;
        PH_MARK(11);
      } else {
        // clones, activate_dual: dual_build_children from the slot
        wctl_to_ctl(W, ctl);
        wave_rare<R, V>(kp, E.P, sbase, ctl, WR_CHILDREN, topslot, tdual, 0, 0, 0, 0, 0);
        wctl_from_ctl(W, ctl);
        W.hot = kNoSlot;
        if (W.status != ST_OK) break;
        nc = nchild;
        general = true;
      }
    }
    // ---- the children into the queue and their trackers ----
    for (uint32_t c = 0; c < nc; ++c) {
      uint32_t cslot = topslot;
      if (general) {
        cslot = uni(ctl.ch_slot[c]);
        ccost = ((uint64_t)uni((uint32_t)(ctl.ch_cost[c] >> 32)) << 32) | uni((uint32_t)ctl.ch_cost[c]);
        clen = uni(ctl.ch_len[c]);
      }
      const uint32_t k = !general ? (tdual ? 1u : 0u) : ((uni(E.L.meta[cslot].flags) & 1u) ? 1u : 0u);
      if (k) W.total[1] += clen >= W.thr[1];
      else W.total[0] += clen >= W.thr[0];
      const HeapEntry ce{ccost, clen, cslot};
      if (kRepop && !general && wheap_push_pop_noop(E.L.heap, W.heap_n, ce)) {
        // (nc == 1: the in-place child) its tracker count too stays out of
        // HBM: the next pop's remove cancels the insert, and the threshold
        // walk between them adds it (stash_k)
        stashed = true;
        stash = ce;
        stash_k = k;
      } else {
        if (threadIdx.x == 0) atomicAdd((uint32_t*)&(k ? lc[1] : lc[0])[WC_IX(clen, L2)], 1u);  // tracker(k).insert(len)
        if (!kCoop || wave_id() == 0) wheap_push(E.L.heap, W.heap_n, ce);
      }
      W.heap_n++;
    }
    PH_MARK(7);
  }
  wave_flush_counters(ctl, W, lcnt);
  // the register state back into Ctl for finish_problem
  if (threadIdx.x == 0) {
    ctl.cnt[S_PEAKQ] = max(ctl.cnt[S_PEAKQ], (uint64_t)W.peakq);
  }
  wctl_to_ctl(W, ctl);
  finish_problem(A, ctl, outp, prob, oslot);
}

// the claim loop: every problem on the build of its read count (R = 1 for
// <= 64 reads, 2 for <= 128) when `mixed`, else on R's
template <int R, bool mixed>
__device__ __forceinline__ void dual_main_wave(const EngineArgs& A, uint8_t* smem, Lo<Ctl>& ctl) {
  const int tid = threadIdx.x;
  Eng E = make_eng(A, state_base(A, smem));
  if (tid == 0) ctl.obuf = 1;
  for (;;) {
    uint32_t oslot = 0;
    const uint32_t prob = claim_problem(A, ctl, E, oslot);
    if (prob == ~0u) break;
    E.n = E.P.n_reads;
    Gm<uint8_t>* outp = (Gm<uint8_t>*)A.out + (uint64_t)oslot * A.out_stride;
    init_problem(E, ctl);
    // what this build runs (the host plans it so): no offsets, <= 64 R reads
    if (E.n > 64u * R * (uint32_t)kEW || E.P.max_act != 0 || E.P.n_active != E.n) {
      if (tid == 0) ctl.status = WC_E_INVARIANT_CODE;
      __syncthreads();
      finish_problem(A, ctl, outp, prob, oslot);
      continue;
    }
    constexpr int V = mixed ? R : 0;
    if (mixed && E.n <= 64u) wave_problem<1, V>(A, E, ctl, prob, oslot, outp);
    else wave_problem<R, V>(A, E, ctl, prob, oslot, outp);
  }
  stream_exit(A);
}
