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

// ---- the hot format: a slot RState with the frontier left uncompacted ----
// word 3 = nscmp | live-slot mask << 16 | flags << 24 (slot RStates keep nf in
// byte 2; a kWide or inactive read keeps its slot RState as it is)
__device__ __forceinline__ RRaw hot_pack(const Front& f) {
  RRaw s;
  s.a = make_uint4(f.e, f.off, f.maxb, (f.nscmp & 0xFFFFu) | (f.mask << 16));
  s.b = make_uint4(f.fi[0] | f.fi[1] << 16, f.fi[2] | f.fi[3] << 16, f.fi[4] | f.fi[5] << 16, f.fi[6] | f.fi[7] << 16);
  s.c = make_uint4(f.fd[0], f.fd[1], f.fd[2], f.fd[3]);
  s.d = make_uint4(f.fd[4], f.fd[5], f.fd[6], f.fd[7]);
  return s;
}
__device__ __forceinline__ void hot_unpack(const RRaw& s, Front& f) {
  front_load(s, f);
  f.mask = (s.a.w >> 16) & 0xFFu;
}
// a slot RState (compacted: nf live slots) in the hot format
__device__ __forceinline__ RRaw slot_to_hot(RRaw s) {
  if (rraw_e(s) != kInactive && !(rraw_flags(s) & kWide)) {
    const uint32_t nf = (s.a.w >> 16) & 0xFFu;
    s.a.w = (s.a.w & 0xFF00FFFFu) | (((1u << nf) - 1u) << 16);
  }
  return s;
}
// and back (front_store compacts the live slots)
__device__ __forceinline__ void hot_to_slot(Gm<RState>* p, const RRaw& s) {
  if (rraw_e(s) != kInactive && !(rraw_flags(s) & kWide)) {
    Front f;
    hot_unpack(s, f);
    front_store(p, f);
  } else {
    rstate_store(p, s);
  }
}

// ---- tip bytes: the read byte behind every tip of a frontier ----
// (thread_tips' x[k], packed: byte k of lo/hi, valid bit k; 0x100 = no tip)
struct Tips {
  uint32_t lo, hi, valid;
};
__device__ __forceinline__ Tips tips_fetch(const Front& f, const Gm<uint8_t>* rd, uint32_t blen, uint32_t len) {
  uint32_t x[kF];
  thread_tips(f, GlobalBytes{rd}, blen, len, x);
  Tips t = {0, 0, 0};
#pragma unroll
  for (int k = 0; k < kF; ++k) {
    if (x[k] == 0x100u) continue;
    t.valid |= 1u << k;
    if (k < 4) t.lo |= (x[k] & 0xFFu) << (8 * k);
    else t.hi |= (x[k] & 0xFFu) << (8 * (k - 4));
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
// counts for reached_baseline_end, the tips give the nominations)
__device__ inline Nom nominate_tips(const Front& f, const uint32_t (&x)[kF], uint32_t blen) {
  uint32_t mb = f.maxb;
  const uint32_t hi = f.mask ? 32u - (uint32_t)__builtin_clz(f.mask) : 0u;
#pragma unroll
  for (int k = 0; k < kF; ++k) {
    if ((uint32_t)k >= hi) break;
    if (f.mask & (1u << k)) mb = max(mb, f.fd[k] + f.e - f.fi[k]);
  }
  uint64_t keys = 0;
  uint32_t cnts = 0, nk = 0;
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
  }
  Nom o;
  o.n = nk;
  o.end = mb == blen;
  if (nk <= 1) {
    o.sym = keys;
    o.occ = cnts;
    o.split = cnts;
    return o;
  }
  const uint64_t ord = fx_order_packed(nk, [&](uint32_t j) { return byte_at(keys, j); });
  uint64_t sym = 0, occ = 0;
  uint32_t split = 0;
  for (uint32_t k = 0; k < nk; ++k) {
    const uint32_t j = nib(ord, k);
    const uint32_t c = (cnts >> (4 * j)) & 15u;
    sym |= (uint64_t)byte_at(keys, j) << (8 * k);
    occ |= (uint64_t)c << (8 * k);
    split += c;
  }
  o.sym = sym;
  o.occ = occ;
  o.split = split;
  return o;
}

// the hot node (both sides when `dual`) back into slot `slot`
template <int R>
__device__ __forceinline__ void hot_writeback(Eng& E, uint32_t slot, bool dual) {
  const int lane = lane_id();
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const uint32_t r = (uint32_t)lane + 64u * j;
    if (r >= E.n) continue;
    hot_to_slot(&E.sv(slot, 0).rs[r], rstate_load(&E.L.hot[r]));
    if (dual) hot_to_slot(&E.sv(slot, 1).rs[r], rstate_load(&E.L.hot[E.nmax + r]));
  }
}
template <int R>
__device__ __forceinline__ void hot_fetch_slot(Eng& E, uint32_t slot, bool dual) {
  const int lane = lane_id();
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const uint32_t r = (uint32_t)lane + 64u * j;
    if (r >= E.n) continue;
    const RRaw a = rstate_load(&E.sv(slot, 0).rs[r]);
    RRaw b = a;
    if (dual) b = rstate_load(&E.sv(slot, 1).rs[r]);
    rstate_store(&E.L.hot[r], slot_to_hot(a));
    if (dual) rstate_store(&E.L.hot[E.nmax + r], slot_to_hot(b));
  }
}

// ---- the rare paths, out of line (one call site each): the pop loop's
// register allocation does not carry theirs. The callee rebuilds the engine
// context from the kernel arguments (callee_eng); the hot area is the carve's
// start, so sbase = Lds::hot. ----
enum : uint32_t { WR_GENERAL_POP = 0, WR_GENERAL_VOTES = 1, WR_HEAVY = 2 };

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

template <int R>
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
  if (op == WR_HEAVY) {
    // the ED-increase loops (and wide frontiers) of the in-place push: one
    // read per wave, through the slot; the rebuilt RState goes back to the
    // hot copy
    const uint32_t nl[2] = {a0, a1};
    const int sy[2] = {(int32_t)a2, (int32_t)a3};
    const uint32_t nh = uni(ctl.nheavy);
    WaveCounters cnt = {0, 0, 0, 0, 0, 0};
    for (uint32_t k = 0; k < nh; ++k) {
      const uint32_t it = uni(E.L.list[WC_IX(k, list_entries(E.sides, E.nmax))]);
      const uint32_t sd = it >= n ? 1u : 0u, r = it - sd * n;
      SideView v = E.sv(top, sd);
      uint32_t e = 0;
      const bool ok = wave_heavy(&v.rs[r], v.wf + (uint64_t)r * E.wcap, E.read(r), E.rlen(r), v.con, nl[sd],
                                 (uint8_t)sy[sd], cfg.wildcard, early, E.wcap, cnt, e);
      __threadfence_block();
      __builtin_amdgcn_wave_barrier();
      if (!ok) {
        if (lane == 0) atomicOr(&ctl.ovf, 4u);
        continue;
      }
      if (lane == 0) rstate_store(&E.L.hot[sd * E.nmax + r], slot_to_hot(rstate_load(&v.rs[r])));
    }
    flush_counters(ctl, cnt);
    __syncthreads();
    return;
  }
  // the rest of the pop with the block engines' code (dual_main), from the
  // slot: the hot node goes back there first and is dropped
  const SlotMeta tm = meta_get(E.L.meta[top]);
  const uint32_t tlens[2] = {tm.len[0], tm.len[1]};
  hot_writeback<R>(E, top, tdual);
  __threadfence_block();
  if (tid == 0) ctl.hot_slot = kNoSlot;
  __syncthreads();
  Sh<RInfo>* R0 = E.L.rinfo;
  Sh<RInfo>* R1 = E.L.rinfo + E.nmax;
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
  for (uint32_t side = 0; side < (tdual ? 2u : 1u); ++side) {
    const bool ok = wave_votes(ctl, side, side == 0 ? R0 : R1, R0, R1, n, weighted, tdual, ctl.multi[side] != 0,
                               cfg.wildcard);
    if (!ok && lane == 0) atomicOr(&ctl.ovf, (uint32_t)LIM_VOTES);
  }
  __syncthreads();
  if (tid == 0) wave_select_t0(cfg, ctl, tm, tdual);
  __syncthreads();
  if (uni(ctl.status) != ST_OK) return;
  const uint32_t nc = uni(ctl.nchild);
  if (nc == 0) {
    if (tid == 0) {
      E.L.freestack[WC_IX(ctl.nfree++, E.pcap)] = top;
      ctl.action = 3;  // no child (the main loop pushes nothing)
    }
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
struct LaneReads {
  const Gm<uint8_t>* rd[R];
  uint32_t bl[R];
};

// ---- the in-place child of a one-child pop (dual_build_children for nc == 1,
// no activate_dual): pushes on the hot state, ED increases through the slot,
// prune + cost + Some counts in one lane pass; new tip bytes into tx ----
template <int R>
__device__ __forceinline__ void wave_push_inplace(Eng& E, Lo<Ctl>& ctl, KArgs kp, uint32_t top, const SlotMeta& tm,
                                                  bool tdual, const LaneReads<R>& lr, Tips (&tx)[R][2]) {
  const int tid = threadIdx.x, lane = lane_id();
  const DevConfig& cfg = E.cfg;
  const bool early = cfg.early != 0;
  const uint32_t n = E.n;
  if (tid == 0) {
    ctl.ch_slot[0] = top;
    ctl.ch_cost[0] = 0;
    SlotMeta m = tm;
    const uint32_t kind = ctl.ch_kind[0];
#pragma unroll
    for (int sd = 0; sd < 2; ++sd) {
      const int sym = ctl.ch_s[0][sd];
      if (sym >= 0) {
        E.sv(top, sd).con[WC_IX(m.len[sd], E.lcap)] = (uint8_t)sym;
        m.len[sd]++;
      } else if (kind == 0) {
        m.flags |= (sd == 0 ? 2u : 4u);  // lock_sequence
      }
    }
    meta_put(E.L.meta[top], m);
    ctl.nheavy = 0;
  }
  __syncthreads();
  PH_MARK(4);
  const int sy[2] = {uni((int32_t)ctl.ch_s[0][0]), uni((int32_t)ctl.ch_s[0][1])};
  const uint32_t nl[2] = {uni(E.L.meta[top].len[0]), uni(E.L.meta[top].len[1])};
  WaveCounters tc = {0, 0, 0, 0, 0, 0};
  uint32_t refetch = 0;  // bit 2j+sd: tips to fetch after the heavy pass
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const uint32_t r = (uint32_t)lane + 64u * j;
    const bool live = r < n;
    const Gm<uint8_t>* rd = lr.rd[j];
    const uint32_t blen = lr.bl[j];
#pragma unroll
    for (int sd = 0; sd < 2; ++sd) {
      bool heavy = false;
      if (live && (sd == 0 || tdual) && sy[sd] >= 0) {
        Sh<RState>* hp = &E.L.hot[sd * E.nmax + r];
        const RRaw s = rstate_load(hp);
        if (rraw_e(s) != kInactive) {
          if (rraw_flags(s) & kWide) {
            heavy = true;  // the slot's RState is current (a wide read's hot copy is the slot's)
          } else {
            Front f;
            hot_unpack(s, f);
            uint32_t x[kF];
            tips_unpack(tx[j][sd], x);
            uint32_t cmp = 0;
            SideView v = E.sv(top, sd);
            heavy = thread_apply(f, x, blen, nl[sd] - 1, (uint8_t)sy[sd], cfg.wildcard, early,
                                 v.wf + (uint64_t)r * E.wcap, cmp);
            tc.compares += cmp;
            if (heavy) {
              front_store(&v.rs[r], f);  // the ED-increase loop reads it from the slot
            } else {
              rstate_store(hp, hot_pack(f));
              tc.updates++;
              tc.w_out += 2 * f.e + 1;
              tx[j][sd] = tips_fetch(f, rd, blen, nl[sd]);
            }
          }
        }
      }
      if (heavy) refetch |= 1u << (2 * j + sd);
      const uint32_t k = agg_append(&ctl.nheavy, heavy);
      if (heavy) E.L.list[WC_IX(k, list_entries(E.sides, E.nmax))] = sd * n + r;
    }
  }
  flush_thread_counters(ctl, tc);
  __syncthreads();
  PH_MARK(5);
  if (uni(ctl.nheavy))
    wave_rare<R>(kp, E.P, (Sh<uint8_t>*)E.L.hot, ctl, WR_HEAVY, top, tdual, nl[0], nl[1], (uint32_t)sy[0],
                 (uint32_t)sy[1], 0);
  PH_MARK(6);
  // prune_dwfa (:1030-1045) of a dual child, then per read the cheaper side's
  // cost (strict <: ties keep consensus 1, :1092-1131) and the Some counts
  uint64_t cost = 0;
  uint32_t c0 = 0, c1 = 0;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const uint32_t r = (uint32_t)lane + 64u * j;
    if (r >= n) continue;
    Sh<RState>* h0 = &E.L.hot[r];
    Sh<RState>* h1 = &E.L.hot[E.nmax + r];
    uint32_t e1 = h0->e;
    uint32_t e2 = tdual ? h1->e : kInactive;
    if (tdual && e1 != kInactive && e2 != kInactive) {
      if ((uint64_t)e1 + cfg.dual_max_ed_delta < (uint64_t)e2) {
        h1->e = kInactive;
        e2 = kInactive;
      } else if ((uint64_t)e2 + cfg.dual_max_ed_delta < (uint64_t)e1) {
        h0->e = kInactive;
        e1 = kInactive;
      }
    }
    uint64_t best = ~0ull;
    if (e1 != kInactive) best = cost_of(e1, cfg.cost_mode);
    if (e2 != kInactive && cost_of(e2, cfg.cost_mode) < best) best = cost_of(e2, cfg.cost_mode);
    if (best != ~0ull) cost += best;
    c0 += e1 != kInactive;
    c1 += e2 != kInactive;
    // tips of the reads that went through the ED-increase loop
#pragma unroll
    for (int sd = 0; sd < 2; ++sd) {
      if (!((refetch >> (2 * j + sd)) & 1u)) continue;
      const RRaw s = rstate_load(sd ? h1 : h0);
      if (rraw_e(s) == kInactive || (rraw_flags(s) & kWide)) continue;
      Front f;
      hot_unpack(s, f);
      tx[j][sd] = tips_fetch(f, lr.rd[j], lr.bl[j], nl[sd]);
    }
  }
  cost = wave_sum_u64(cost);
  c0 = wave_sum_u32(c0);
  c1 = wave_sum_u32(c1);
  if (tid == 0) {
    if (ctl.ovf & 16u) ctl.status = WC_E_INVARIANT_CODE;
    else if (ctl.ovf & 4u) ctl.status = ST_RETRY | ST_RETRY_WCAP;
    else if (ctl.ovf) ctl.status = limit_status(ctl.ovf);
    auto& m = E.L.meta[top];
    m.nsome[0] = c0;
    m.nsome[1] = c1;
    ctl.ch_cost[0] = cost;
    ctl.ch_len[0] = max(nl[0], nl[1]);
  }
  __syncthreads();
  PH_MARK(11);
}

// ---- the search: dual_main's pop, with a lean path for the common pop ----
// The common pop (no read at a consensus end, no wide frontier, every read
// nominating at most one symbol, unweighted votes, and exactly one child that
// pushes in place) runs below: analysis on the hot state and prefetched tip
// bytes, the votes as ballot counts (exact integers), the selection on those
// counts (with one child the hashbrown order of the keys decides nothing), the
// lane push. Anything else goes to wave_rare's WR_GENERAL*, which runs the
// block engines' code for the rest of the pop.
template <int R>
__device__ __forceinline__ void dual_main_wave(const EngineArgs& A, uint8_t* smem, Lo<Ctl>& ctl) {
  const int tid = threadIdx.x;
  const int lane = lane_id();
  const DevConfig& cfg = A.cfg;
  const bool early = cfg.early != 0;
  const bool weighted = cfg.weighted != 0;
  const int wc = cfg.wildcard;
  Eng E = make_eng(A, state_base(A, smem));
  Sh<RInfo>* R0 = E.L.rinfo;
  Sh<RInfo>* R1 = E.L.rinfo + E.nmax;
  Tips tx[R][2];
#pragma unroll
  for (int j = 0; j < R; ++j) tx[j][0] = tx[j][1] = Tips{0, 0, 0};

  if (tid == 0) ctl.obuf = 1;
  for (;;) {
    uint32_t oslot = 0;
    const uint32_t prob = claim_problem(A, ctl, E, oslot);
    if (prob == ~0u) break;
    E.n = E.P.n_reads;
    Gm<uint8_t>* outp = (Gm<uint8_t>*)A.out + (uint64_t)oslot * A.out_stride;
    init_problem(E, ctl);
    if (tid == 0) ctl.hot_prev_dual = 0;  // (here: the hot node has side 2)
    // what this build runs (the host plans it so): no offsets, <= 64 R reads
    if (E.n > 64u * R || E.P.max_act != 0 || E.P.n_active != E.n) {
      if (tid == 0) ctl.status = WC_E_INVARIANT_CODE;
      __syncthreads();
      finish_problem(A, ctl, outp, prob, oslot);
      continue;
    }
    const uint64_t full_min = max(cfg.min_count, ceil_u64(cfg.min_af * (double)E.n));
    bool tips_ok = false;  // tx holds the hot node's tip bytes
    LaneReads<R> lr;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const uint32_t r = (uint32_t)lane + 64u * j;
      lr.rd[j] = r < E.n ? E.read(r) : E.rbytes;
      lr.bl[j] = r < E.n ? E.rlen(r) : 0u;
    }
    const KArgs kp = kernel_args();
    Sh<uint8_t>* const sbase = (Sh<uint8_t>*)E.L.hot;

    for (;;) {
      // ---- pop (dual_consensus.rs:340-397) ----
      if (tid == 0) {
        if (ctl.heap_n == 0) {
          ctl.action = 2;
        } else {
          const uint32_t plen = E.L.heap[0].len;
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
          HeapEntry top = heap_pop(E.L.heap, ctl.heap_n, E.pcap);
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
            if (top.slot == ctl.hot_slot) ctl.hot_slot = kNoSlot;  // its state is dropped with the slot
            ctl.action = 1;
          } else {
            ctl.farthest[dual] = max(ctl.farthest[dual], (uint64_t)top.len);
            ctl.last_constraint[dual]++;
            t.process_unchecked(top.len);
            ctl.cnt[S_EXPLORED]++;
            ctl.action = 0;
            // the popped node's state into the hot area, unless it is there
            // (the in-place child of the previous pop); the previous hot node,
            // still queued, goes back to its slot first
            ctl.hot_prev = ctl.hot_slot;
            ctl.hot_load = top.slot != ctl.hot_slot;
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
      SUB_T0(t_hot);
      if (uni(ctl.hot_load)) {
        SUB_CNT(33, 1);
        const uint32_t prev = uni(ctl.hot_prev);
        if (prev != kNoSlot) hot_writeback<R>(E, prev, uni(ctl.hot_prev_dual) != 0);
        hot_fetch_slot<R>(E, top, tdual);
        tips_ok = false;
        if (tid == 0) {
          ctl.hot_slot = top;
          ctl.hot_prev_dual = tdual ? 1u : 0u;
        }
        __syncthreads();
      }
      SUB_T1(32, t_hot);

      // ---- analysis of both sides from the hot state: thread_analyze on the
      // prefetched tip bytes; the nominations also go to RInfo (the general
      // path reads them there) ----
      SUB_T0(t_an);
      uint32_t ys[R][2];  // the read's one nominated symbol (0x100: none or not a voter)
      bool any_wide = false, any_end = false, any_multi = false;
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const uint32_t r = (uint32_t)lane + 64u * j;
        const bool live = r < E.n;
#pragma unroll
        for (int sd = 0; sd < 2; ++sd) {
          ys[j][sd] = 0x100u;
          bool wide = false, end = false, multi = false;
          if (live && (sd == 0 || tdual)) {
            Sh<RInfo>* out = (sd ? R1 : R0) + r;
            const RRaw s = rstate_load(&E.L.hot[sd * E.nmax + r]);
            if (rraw_e(s) == kInactive) {
              out->e = kInactive;
              out->n = 0;
              out->end = 0;
            } else if (rraw_flags(s) & kWide) {
              wide = true;
            } else {
              Front f;
              hot_unpack(s, f);
              if (!tips_ok) tx[j][sd] = tips_fetch(f, lr.rd[j], lr.bl[j], tlens[sd]);
              uint32_t x[kF];
              tips_unpack(tx[j][sd], x);
              const Nom o = nominate_tips(f, x, lr.bl[j]);
              rinfo_store(out, o, f.e);
              end = o.end != 0;
              multi = o.n > 1;
              if (o.n == 1) ys[j][sd] = byte_at(o.sym, 0);
            }
          }
          any_wide |= ballot(wide) != 0;
          any_end |= ballot(end) != 0;
          any_multi |= ballot(multi) != 0;
        }
      }
      tips_ok = true;
      SUB_T1(34, t_an);
      // ---- active_min_count growth (dual_consensus.rs:497-513; no activation
      // in this build, so the count stays the root's) ----
      if (tid == 0 && ctl.am_len == tlen + 1 && tlen + 1 < E.lcap + 2) {
        const uint32_t nt = E.total_active[tlen];
        E.total_active[tlen + 1] = nt;
        E.active_min[tlen + 1] = (uint32_t)max(cfg.min_count, ceil_u64(cfg.min_af * (double)nt));
        ctl.am_len++;
      }
      PH_MARK(1);
      if (any_wide || any_end) {
        // wide frontiers (nominated from the row) or a read at a consensus
        // end (finalize, reached_*): the general pop from its analysis on
        wave_rare<R>(kp, E.P, sbase, ctl, WR_GENERAL_POP, top, tdual, (uint32_t)full_min, (uint32_t)(full_min >> 32),
                     oslot, 0, 0);
      } else {
        // ---- votes (consensus.rs:540-564, dual_consensus.rs:1242-1290):
        // every voter adds 1.0 to its one symbol, so each key's value is an
        // exact count. Per side: the keys (wildcard dropped when it is not the
        // only one, :556-561), their sum and maximum, the threshold
        // min(max(min_count, ceil(min_af * sum)), max) (:520-552), the keys
        // passing it ----
        SUB_T0(t_v);
        int child[2] = {-1, -1};
        uint32_t nchild = 2;  // (anything but 0 or 1: the general path)
        uint32_t kind = tdual ? 0u : 1u;
        if (!any_multi && !weighted) {
          uint32_t npass[2] = {0, 0}, nkeys[2] = {0, 0};
          int pkey[2] = {-1, -1};
          bool split = false;
#pragma unroll
          for (int sd = 0; sd < 2; ++sd) {
            if (sd == 1 && !tdual) break;
            // pass 1: distinct keys, their counts, sum and maximum
            uint64_t rem[R];
#pragma unroll
            for (int j = 0; j < R; ++j) rem[j] = ballot(ys[j][sd] != 0x100u);
            uint32_t nk = 0, total = 0, mx_all = 0, mx_nowc = 0, wc_cnt = 0;
            bool wc_in = false;
            for (;;) {
              int jj = -1;
#pragma unroll
              for (int j = R - 1; j >= 0; --j)
                if (rem[j]) jj = j;
              if (jj < 0) break;
              uint32_t key = 0;
#pragma unroll
              for (int j = 0; j < R; ++j)
                if (j == jj) key = (uint32_t)__builtin_amdgcn_readlane((int)ys[j][sd], __builtin_ctzll(rem[j]));
              uint32_t cnt = 0;
#pragma unroll
              for (int j = 0; j < R; ++j) {
                const uint64_t m = ballot(ys[j][sd] == key);
                cnt += (uint32_t)__popcll((unsigned long long)m);
                rem[j] &= ~m;
              }
              nk++;
              total += cnt;
              mx_all = max(mx_all, cnt);
              if (wc >= 0 && key == (uint32_t)(uint8_t)wc) {
                wc_in = true;
                wc_cnt = cnt;
              } else {
                mx_nowc = max(mx_nowc, cnt);
              }
            }
            const bool drop = wc_in && nk > 1;
            const uint32_t nko = drop ? nk - 1 : nk;
            const uint32_t sum = drop ? total - wc_cnt : total;
            const uint32_t mx = drop ? mx_nowc : mx_all;
            const uint64_t mc = max(cfg.min_count, ceil_u64(cfg.min_af * (double)sum));
            const double thr = nko ? fmin((double)mc, (double)mx) : (double)mc;
            // pass 2: keys passing the threshold (and, single-consensus
            // nodes, the split candidates: non-wildcard keys, those >= mc)
            uint32_t np = 0, ns = 0, npmc = 0;
            int pk = -1;
#pragma unroll
            for (int j = 0; j < R; ++j) rem[j] = ballot(ys[j][sd] != 0x100u);
            for (;;) {
              int jj = -1;
#pragma unroll
              for (int j = R - 1; j >= 0; --j)
                if (rem[j]) jj = j;
              if (jj < 0) break;
              uint32_t key = 0;
#pragma unroll
              for (int j = 0; j < R; ++j)
                if (j == jj) key = (uint32_t)__builtin_amdgcn_readlane((int)ys[j][sd], __builtin_ctzll(rem[j]));
              uint32_t cnt = 0;
#pragma unroll
              for (int j = 0; j < R; ++j) {
                const uint64_t m = ballot(ys[j][sd] == key);
                cnt += (uint32_t)__popcll((unsigned long long)m);
                rem[j] &= ~m;
              }
              const bool is_wc = wc >= 0 && key == (uint32_t)(uint8_t)wc;
              if (drop && is_wc) continue;
              if (!((double)cnt < thr)) {
                np++;
                pk = (int)key;
              }
              if (!is_wc) {
                ns++;
                if ((double)cnt >= (double)mc) npmc++;
              }
            }
            npass[sd] = np;
            nkeys[sd] = nko;
            pkey[sd] = pk;
            if (!tdual) split = npmc > 1 && ns > 1;
          }
          if (tdual) {
            // options per side: None first (consensus end, no keys, locked),
            // then the passing keys; children = pairs but (None, None)
            // (dual_consensus.rs:554-650)
            bool has_none[2];
            uint32_t no[2];
#pragma unroll
            for (int sd = 0; sd < 2; ++sd) {
              const bool lock = (tm.flags & (sd == 0 ? 2u : 4u)) != 0;
              const bool fin = early && tm.nsome[sd] == 0;  // (no read at its end here)
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
            nchild = npass[0] + (split ? 2u : 0u);
            child[0] = pkey[0];
          }
        }
        SUB_T1(38, t_v);
        if (nchild == 0) {
          if (tid == 0) {
            E.L.freestack[WC_IX(ctl.nfree++, E.pcap)] = top;
            ctl.hot_slot = kNoSlot;
          }
          __syncthreads();
          PH_MARK(3);
          continue;
        }
        if (nchild == 1 && (tlens[0] + 1 > E.lcap || tlens[1] + 1 > E.lcap)) {
          if (tid == 0) ctl.status = ST_RETRY | ST_RETRY_LCAP;
          __syncthreads();
          break;
        }
        PH_MARK(3);
        if (nchild == 1) {
          SUB_CNT(37, 1);
          if (tid == 0) {
            ctl.ch_s[0][0] = (int16_t)child[0];
            ctl.ch_s[0][1] = (int16_t)child[1];
            ctl.ch_kind[0] = (uint8_t)kind;
            ctl.nchild = 1;
          }
          __syncthreads();
          wave_push_inplace<R>(E, ctl, kp, top, tm, tdual, lr, tx);  // the hot node becomes the child
        } else {
          // several children, or multi-symbol reads / weighted votes: the
          // block engines' votes, selection and children
          if (tid == 0) {
            ctl.multi[0] = ctl.multi[1] = any_multi ? 1u : 0u;
            ctl.fin[0] = early && tm.nsome[0] == 0;
            ctl.fin[1] = tdual && early && tm.nsome[1] == 0;
          }
          __syncthreads();
          wave_rare<R>(kp, E.P, sbase, ctl, WR_GENERAL_VOTES, top, tdual, 0, 0, 0, 0, 0);
        }
      }
      if (uni(ctl.status) != ST_OK) break;
      if (uni(ctl.action) == 3) continue;  // (the general path: no child; the slot is free)
      if (tid == 0) {
        for (uint32_t c = 0; c < ctl.nchild; ++c) {
          const uint32_t k = (E.L.meta[ctl.ch_slot[c]].flags & 1u) ? 1 : 0;
          E.tracker(ctl, k).insert(ctl.ch_len[c]);
          heap_push(E.L.heap, ctl.heap_n, E.pcap, HeapEntry{ctl.ch_cost[c], ctl.ch_len[c], ctl.ch_slot[c]});
        }
      }
      __syncthreads();
      PH_MARK(7);
    }
    finish_problem(A, ctl, outp, prob, oslot);
  }
  stream_exit(A);
}
