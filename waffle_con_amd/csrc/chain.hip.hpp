// Linear-chain run-ahead for the ConsensusDWFA engine (included by engine.hip).
//
// The least-cost-first search of consensus.rs:139-351 is, almost everywhere, a
// single chain: the popped node has exactly one passing candidate, the pushed
// child is the only queued node and is popped next. Executed literally, every
// consensus base costs a full pop: a block-wide push over all reads, the
// votes, and a handful of barriers — latency, not bandwidth.
//
// run_chain executes up to K steps of such a chain speculatively and then
// proves, step by step, that the reference search would have taken exactly
// those steps:
//   1. predict the next K-1 symbols (plurality of the reads' upcoming bases);
//   2. every thread pushes the K symbols through its own read's DWFA
//      (DWFALite::update, dynamic_wfa.rs:75-99; edit-distance increases are
//      done by the thread's wave over the full wavefront) and records each
//      step's nominations (dynamic_wfa.rs:241-255), cost and end flag;
//   3. the votes of every step are evaluated exactly (consensus.rs:540-564,
//      f64 order and hashbrown order as in the one-step path) and the pop
//      sequence is replayed on the scalar search state: PQueueTracker
//      threshold/capacity (consensus.rs:224-251), reached_end (:254), the
//      candidate filter (:283-321). Step j is accepted only if the node would
//      be popped next, explored, not reach an end, and have exactly one passing
//      candidate equal to the predicted symbol j+1;
//   4. the accepted prefix N_1..N_j* is committed: all counters, tracker and
//      pool state are exactly those of j* literal iterations. If a step is
//      rejected, the node's wavefront rows are restored from a backup slot and
//      the accepted prefix is replayed.
// The last accepted node is handed back to the literal path (pushed to the
// queue with its nominations cached), which handles ends, branching and
// everything else.

// nomination record of one read at one chain step (u16)
constexpr uint32_t kNomSymMask = 0xFFu;   // the symbol, or the ChainOvf index with kNomOvf
constexpr uint32_t kNomOne = 1u << 8;     // exactly one distinct symbol
constexpr uint32_t kNomEnd = 1u << 12;    // reached_baseline_end
constexpr uint32_t kNomActive = 1u << 13; // Some(dwfa)
constexpr uint32_t kNomOvf = 1u << 14;    // >= 2 symbols: ChainOvf[code & kNomSymMask]
constexpr uint32_t kNomQuiet = 1u << 15;  // a quiet step: one symbol, the step's next prediction
constexpr uint16_t kNomQuietCode = (uint16_t)(kNomActive | kNomOne | kNomQuiet);

__device__ __forceinline__ RInfoReg nom_decode(uint32_t c, const Sh<ChainOvf>* ovf, uint32_t qsym) {
  RInfoReg x = {0, 0, kInactive, 0, make_uint4(0, 0, 0, 0)};
  if (!(c & kNomActive)) return x;
  x.e = 0;
  if (c & kNomOvf) {
    const ChainOvf o = ovf[c & kNomSymMask];
    x.n = o.n();
    x.split = o.split();
    x.sym = o.sym;
    x.occ = make_uint4(o.occ_at(0) | o.occ_at(1) << 16, o.occ_at(2) | o.occ_at(3) << 16,
                       o.occ_at(4) | o.occ_at(5) << 16, o.occ_at(6) | o.occ_at(7) << 16);
  } else if (c & kNomOne) {
    x.n = 1;
    x.split = 1;  // occ / split = 1.0 exactly for a single symbol
    x.sym = (c & kNomQuiet) ? qsym : (c & kNomSymMask);
    x.occ = make_uint4(1, 0, 0, 0);
  }
  return x;
}
__device__ __forceinline__ RInfoReg nom_load(const Sh<uint16_t>* nom, const Sh<ChainOvf>* ovf, uint32_t r,
                                             uint32_t qsym = 0) {
  return nom_decode(nom[r], ovf, qsym);
}

// 8 bytes of an LDS byte array from byte q (the array is dword aligned; bytes
// the three dword loads touch past its end are never counted)
__device__ __forceinline__ uint64_t lds_bytes8(const Sh<uint8_t>* a, uint32_t q) {
  const Sh<uint32_t>* w32 = (const Sh<uint32_t>*)a + (q >> 2);
  const uint32_t d0 = w32[0], d1 = w32[1], d2 = w32[2], sh = q & 3u;
  return (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, sh) | (uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sh) << 32;
}

// LDS window slot of read r (the walk deals read r to wave r % kEW, lane
// r / kEW): the lanes of one wave read consecutive slots (engine_shared.hpp
// kWinStride). kEW * ceil(n / kEW) <= win_slots(nmax, kEW), the carve.
__device__ __forceinline__ uint32_t cwin_slot(uint32_t r, uint32_t n) {
  return (r % (uint32_t)kEW) * ((n + kEW - 1) / (uint32_t)kEW) + r / (uint32_t)kEW;
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ double wave_max_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

// (B) backup wavefront rows to slot S, stage read windows in LDS, prefetch
// capacities, predict symbols.
__device__ inline void chain_prepare(Eng& E, Lo<Ctl>& ctl, uint32_t top, uint32_t L0, uint32_t K, uint32_t S) {
  const int tid = threadIdx.x, lane = lane_id();
  SideView v = E.sv(top, 0);
  SUB_T0(ta);
  // windows: 64 bytes from the lowest tip, 16-byte aligned (reads are
  // 16-byte aligned and the read buffer has 64 bytes of tail padding)
  uint64_t c0 = 0;
  for (uint32_t r = tid; r < E.n; r += kEB) {
    const RRaw h = rstate_load(&E.L.hot[r]);
    if (rraw_e(h) != kInactive && (rraw_flags(h) & kWide)) atomicOr(&ctl.chain_nochain, 1u);
    Front f;
    front_load(h, f);
    uint32_t lo = kInactive, tip = kInactive;
    if (f.e != kInactive) {
      const uint32_t blen = E.rlen(r);
#pragma unroll
      for (int k = kF - 1; k >= 0; --k)
        if ((f.mask >> k) & 1u) {
          const uint32_t bo = f.fd[k] + f.e - f.fi[k];
          lo = min(lo, min(bo, blen));
          if (f.fd[k] + f.off == L0 && bo < blen) tip = bo;  // the first tip at the node's end
        }
    }
    if (lo == kInactive) lo = 0;
    const uint32_t wb = lo & ~15u;
    // the predictions below read that tip's window offset (cm0 is free until the deal)
    E.L.cm0[r] = (uint8_t)(tip != kInactive && tip - wb < 64u ? tip - wb : 0xFFu);
    const Gm<uint4>* g = (const Gm<uint4>*)(E.read(r) + wb);
    Sh<uint32_t>* w = (Sh<uint32_t>*)(E.L.cwin + (uint64_t)cwin_slot(r, E.n) * kWinStride);
    const uint4 a0 = g[0], a1 = g[1], a2 = g[2], a3 = g[3];
    w[0] = a0.x, w[1] = a0.y, w[2] = a0.z, w[3] = a0.w;
    w[4] = a1.x, w[5] = a1.y, w[6] = a1.z, w[7] = a1.w;
    w[8] = a2.x, w[9] = a2.y, w[10] = a2.z, w[11] = a2.w;
    w[12] = a3.x, w[13] = a3.y, w[14] = a3.z, w[15] = a3.w;
    E.L.cwb[r] = wb;
    // Every step of an active read starts as a quiet step (it nominates the
    // step's next prediction with weight 1); the walk stores the code of every
    // other step. An inactive read nominates nothing. The node's cost is the
    // base of the steps' costs (chain_votes adds the walk's changes).
    const bool act = rraw_e(h) != kInactive;
    const uint16_t qc = act ? kNomQuietCode : (uint16_t)0;
    Sh<uint16_t>* nm = E.L.cnom + r * (K + 1);  // read r's row: step j at nm[j]
    for (uint32_t j = 1; j <= K; ++j) nm[j] = qc;
    if (act) c0 += cost_of(rraw_e(h), E.cfg.cost_mode);
  }
  c0 = wave_sum_u64(c0);
  const Gm<uint32_t>* pc = E.trk + (E.lcap + 2);  // PQueueTracker processed counts
  for (uint32_t j = tid; j <= K; j += kEB) E.L.cpc[j] = (j >= 1) ? trk_load(&pc[L0 + j]) : 0u;
  __syncthreads();
  if (lane == 0 && c0) atomicAdd((unsigned long long*)&E.L.cstep[0].cost, (unsigned long long)c0);
  SUB_T1(23, ta);
  SUB_T0(tb);
  {
    // upcoming bases of each read's first tip (reads 0..63); every wave
    // predicts the steps t = 1 + wave (mod kEW)
    const uint32_t wave = (uint32_t)wave_id();
    // (the window loop left each read's first tip at the node's end as an
    // offset into its window, 0xFF = none or outside it)
    uint32_t q0 = 0xFFu, blen = 0, wb = 0;
    const Sh<uint8_t>* win = E.L.cwin + (uint64_t)cwin_slot(min((uint32_t)lane, E.n - 1), E.n) * kWinStride;
    if ((uint32_t)lane < E.n) {
      q0 = E.L.cm0[lane];
      wb = E.L.cwb[lane];
      blen = E.rlen(lane);
    }
    // all of this wave's bytes under one wait; LDS windows only: a read whose
    // next bases lie past its window does not vote (the prediction is a
    // guess, acceptance is exact)
    constexpr uint32_t kPer = (kChainMax + kEW - 1) / kEW;
    uint32_t xs[kPer];
#pragma unroll
    for (uint32_t u = 0; u < kPer; ++u) {
      const uint32_t t = 1 + wave + kEW * u;
      const uint32_t q = q0 + t;
      xs[u] = (q0 != 0xFFu && t <= K && wb + q < blen && q < 64u) ? (uint32_t)win[q] : 0x100u;
    }
#pragma unroll
    for (uint32_t u = 0; u < kPer; ++u) {
      const uint32_t t = 1 + wave + kEW * u;
      if (t > K) break;  // (t = K predicts N_K's child: chain_votes decides N_K too)
      const uint32_t x = xs[u];
      // plurality of x over the wave (ties: the first-seen symbol); a
      // first-seen symbol held by a strict majority is the plurality
      uint64_t rem = ballot(x != 0x100u);
      uint32_t best = 0x100u, bestc = 0;
      if (rem) {
        const uint32_t s = (uint32_t)__builtin_amdgcn_readlane((int)x, __builtin_ctzll(rem));
        const uint64_t mm = ballot(x == s);
        const uint32_t c = (uint32_t)__popcll((unsigned long long)mm);
        if (2 * c > (uint32_t)__popcll((unsigned long long)rem)) {
          best = s;
          rem = 0;
        }
      }
      while (rem) {
        const int l = __builtin_ctzll(rem);
        const uint32_t s = (uint32_t)__builtin_amdgcn_readlane((int)x, l);
        const uint64_t mm = ballot(x == s);
        const uint32_t c = (uint32_t)__popcll((unsigned long long)mm);
        if (c > bestc) {
          bestc = c;
          best = s;
        }
        rem &= ~mm;
      }
      if (best == 0x100u) {
        if (lane == 0 && t < K) atomicMin(&ctl.chain_stop, t);  // nothing to predict N_{t+1} from
        break;
      }
      if (lane == 0) {
        E.L.cpred[t + 1] = (uint8_t)best;
        if (t == K) ctl.chain_pk = 1;
      }
    }
  }
  __syncthreads();
  SUB_T1(44, tb);
  // the predicted symbols extend the node's own consensus buffer in place
  // (positions >= L0 are not part of the node)
  if (tid >= 1 && (uint32_t)tid <= K) v.con[L0 + tid - 1] = E.L.cpred[tid];
  // Deal the reads to the walk's positions (position p: wave p % kEW, lane
  // p / kEW). A wave runs its reads' edit-distance increases one at a time
  // and the walk ends with its slowest wave, so the reads whose every tip
  // disagrees with the predictions within the chain (each costs its wave an
  // increase) go first, spread evenly over the waves; the others follow. Any
  // order gives the same results (reads are walked independently).
  {
    const uint32_t r = (uint32_t)tid;  // (n <= kEB with chains: one read per thread)
    bool hv = false;
    if (r < E.n) {
      Front f;
      front_load(rstate_load(&E.L.hot[r]), f);
      if (f.e != kInactive) {
        const uint32_t wb = E.L.cwb[r], blen = E.rlen(r);
        const Sh<uint8_t>* win = E.L.cwin + (uint64_t)cwin_slot(r, E.n) * kWinStride;
        bool any = false, lives = false, fail = false;
        uint32_t m0 = K;
#pragma unroll
        for (int k = 0; k < kF; ++k) {
          if (!((f.mask >> k) & 1u)) continue;
          const uint32_t bo = f.fd[k] + f.e - f.fi[k], q = bo - wb;
          if (f.fd[k] + f.off != L0 || bo >= blen || q >= 64u) {
            fail = true;
            continue;
          }
          any = true;
          const uint32_t lim = min(K, min(blen - bo, 64u - q));
          // the first mismatch within K <= 40 bases: five 8-byte compares,
          // all loaded under one wait (bytes past the window or the
          // predictions are read but never counted: c is clamped to lim)
          static_assert(kChainMax <= 40, "five 8-byte chunks cover a chain");
          uint64_t mmv[5];
#pragma unroll
          for (uint32_t u = 0; u < 5; ++u)
            mmv[u] = nz_bytes(lds_bytes8(win, q + 8 * u) ^ lds_bytes8(E.L.cpred, 1 + 8 * u));
          uint32_t c = 40;
#pragma unroll
          for (int u = 4; u >= 0; --u)
            if (mmv[u]) c = 8 * (uint32_t)u + ((uint32_t)__builtin_ctzll(mmv[u]) >> 3);
          c = min(c, lim);
          lives |= c >= lim;
          m0 = min(m0, min(c, lim));
        }
        hv = any && !lives;
        // the walk's first quiet run (lane_run at step 1, which returns 0 when
        // a live tip is not at the end)
        E.L.cm0[r] = (uint8_t)(fail || !any ? 0u : m0);
      }
    }
    const uint64_t hm = ballot(hv);
    if (lane == 0) ctl.deal_cnt[wave_id()] = (uint32_t)__popcll((unsigned long long)hm);
    if (tid >= 1 && (uint32_t)tid <= K) con_store_wait();  // (the predictions stored above: the walk's ED increases read them)
    __syncthreads();
    l1_drop();
    uint32_t hb = 0, H = 0;
    for (uint32_t w = 0; w < (uint32_t)kEW; ++w) {
      const uint32_t c = ctl.deal_cnt[w];
      if (w < (uint32_t)wave_id()) hb += c;
      H += c;
    }
    if (r < E.n) {
      const uint32_t hr = hb + (uint32_t)__popcll((unsigned long long)(hm & ((1ull << lane) - 1ull)));
      E.L.cperm[hv ? hr : H + r - hr] = (uint8_t)r;
    }
  }
  SUB_T1(24, tb);
}

// ---- thread-level step primitives over the LDS read window ----
// A thread's read window: 64 bytes of its read staged in LDS from wb.
// the bytes at a read's (up to kF) tips, packed four to a register (the walk
// keeps them live across its loop; eight registers of them spilled)
struct TipBytes {
  uint32_t lo, hi;
  __device__ __forceinline__ uint32_t at(int k) const {
    return k < 4 ? (lo >> (8 * k)) & 0xFFu : (hi >> (8 * (k - 4))) & 0xFFu;
  }
};
struct Win {
  const Sh<uint8_t>* w;
  uint32_t wb;
};
// Bytes at the tip positions bo_k = d_k + e - i_k of all frontier entries.
// The loads are unconditional (clamped into the window) so the eight LDS reads
// issue back to back under one wait. Returns whether a tip inside the read lies
// outside the window (the chain then stops before this step's node).
__device__ __forceinline__ bool win_tip_bytes(const Win& W, const Front& f, uint32_t blen, uint32_t kb,
                                              TipBytes& x) {
  uint32_t b[kF];
  bool oob = false;
#pragma unroll
  for (int k = 0; k < kF; ++k) {
    if ((uint32_t)k >= kb) break;
    const uint32_t bo = f.fd[k] + f.e - f.fi[k];
    const uint32_t q = bo - W.wb;
    const bool in = q < 64u;
    b[k] = W.w[in ? q : 0u];
    oob |= ((f.mask >> k) & 1u) && !in && bo < blen;
  }
  x.lo = x.hi = 0;
#pragma unroll
  for (int k = 0; k < kF; ++k) {
    if ((uint32_t)k >= kb) break;
    if (k < 4) x.lo |= b[k] << (8 * k);
    else x.hi |= b[k] << (8 * (k - 4));
  }
  return oob;
}
// DWFALite::update's extend for one appended symbol on the frontier
// (thread_push<kLazy> semantics), comparing against the preloaded tip bytes.
__device__ __forceinline__ bool chain_push(Front& f, const TipBytes& x, uint32_t blen, uint32_t old_len,
                                           uint32_t sym, int wc, bool early, Gm<uint32_t>* row, uint32_t kb,
                                           uint32_t& cmp) {
  uint32_t c = f.nscmp, mb = 0;
#pragma unroll
  for (int k = 0; k < kF; ++k) {
    if ((uint32_t)k >= kb) break;
    if (!(f.mask & (1u << k))) continue;
    const uint32_t d = f.fd[k];
    const uint32_t bo = d + f.e - f.fi[k];
    if (d + f.off == old_len) {
      if (bo < blen) {
        c++;
        if (x.at(k) == sym || (wc >= 0 && x.at(k) == (uint32_t)(uint8_t)wc)) {
          f.fd[k] = d + 1;
          mb = max(mb, bo + 1);
          continue;
        }
        f.nscmp++;  // stuck on a mismatch: compared (and failing) on every later push
      }
      row[f.fi[k]] = d;  // leaves the frontier: the row gets its final value
      f.maxb = max(f.maxb, bo);
      f.mask &= ~(1u << k);
    } else {
      mb = max(mb, bo);
    }
  }
  mb = max(mb, f.maxb);
  cmp = c;
  return f.mask == 0 && !(early && mb == blen);
}
// get_extension_candidates + reached_baseline_end of one read from its
// frontier and the bytes at its tips (thread_nominate semantics).
__device__ __forceinline__ Nom chain_nominate(const Front& f, const TipBytes& x, uint32_t blen, uint32_t len,
                                          uint32_t kb) {
  uint32_t mb = f.maxb;
  uint64_t keys = 0;
  uint32_t cnts = 0, nk = 0;
#pragma unroll
  for (int k = 0; k < kF; ++k) {
    if ((uint32_t)k >= kb) break;
    if (!(f.mask & (1u << k))) continue;
    const uint32_t bo = f.fd[k] + f.e - f.fi[k];
    mb = max(mb, bo);
    if (!(f.fd[k] + f.off == len && bo < blen)) continue;
    const uint32_t s = x.at(k);
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

// Votes in exact rational form: a read's contribution occ/split to a symbol
// (split <= kF = 8) is an integer number of 1/840ths (840 = lcm(1..8)).
constexpr uint32_t kVoteDen = 840;
// kVoteDen / split for split in 1..kF, without an integer division
__device__ __forceinline__ uint32_t vote_unit(uint32_t split) {
  return split <= 4 ? (split <= 2 ? (split == 1 ? 840u : 420u) : (split == 3 ? 280u : 210u))
                    : (split <= 6 ? (split == 5 ? 168u : 140u) : (split == 7 ? 120u : 105u));
}
static_assert(kF == 8, "vote_unit covers split <= 8");

// The ED-increase step of one read inside the chain walk (rare: ~0.5% of the
// updates at cfg2) as a call, so its registers do not add to the walk's
// per-step register pressure (the walk keeps a frontier per lane in registers).
// Arguments and result by value (no stack objects): returns the new edit
// distance, or kInactive on wavefront capacity overflow; the work counters go
// straight to the chain totals.
#ifdef WC_INLINE_HEAVY  // (experiment build: the increase inlined into the walk)
#define WC_HEAVY_FN __device__ __forceinline__
#else
#define WC_HEAVY_FN __device__ __noinline__
#endif
WC_HEAVY_FN uint32_t chain_heavy(Sh<RState>* tmp, Gm<uint32_t>* wf, const Gm<uint8_t>* rd, uint32_t blen,
                                             const Gm<uint8_t>* con, uint32_t olen, uint32_t sym, int wc, bool early,
                                             uint32_t wcap, Lo<uint64_t>* tot, Gm<uint32_t>* bak) {
  WaveCounters cnt = {0, 0, 0, 0, 0, 0};
  uint32_t e_out = 0;
  const bool ok = wave_heavy(tmp, wf, rd, blen, con, olen, (uint8_t)sym, wc, early, wcap, cnt, e_out, bak);
  if (lane_id() == 0) {
    atomicAdd((unsigned long long*)&tot[0], (unsigned long long)cnt.updates);
    atomicAdd((unsigned long long*)&tot[1], (unsigned long long)cnt.w_out);
    atomicAdd((unsigned long long*)&tot[2], (unsigned long long)cnt.compares);
    atomicAdd((unsigned long long*)&tot[3], (unsigned long long)cnt.edinc);
    atomicAdd((unsigned long long*)&tot[4], (unsigned long long)cnt.rowb);
#ifdef WC_PHASE_PROF
    for (int k = 0; k < 3; ++k) atomicAdd((unsigned long long*)&tot[5 + k], (unsigned long long)cnt.tq[k]);
#endif
  }
  return ok ? e_out : kInactive;
}


// The quiet run of one read from step j: the number m (<= lim) of consecutive
// pushes N_j, N_j+1, ... under which every live tip extends (its read bytes
// equal the predictions; 8-byte XOR + ctz of the LDS window against the LDS
// predictions, chunk after chunk). 0 when a live tip is not at the end of the
// consensus (olen = |N_j-1|), lies at the read's end, or outside the window.
__device__ __forceinline__ uint32_t lane_run(const Front& f, const Win& W, const Sh<uint8_t>* pred, uint32_t blen,
                                             uint32_t olen, uint32_t j, uint32_t lim, uint32_t kb, uint32_t& nlive) {
  uint32_t m = lim;
  nlive = 0;
#pragma unroll
  for (int k = 0; k < kF; ++k) {
    if ((uint32_t)k >= kb) break;
    if (!(f.mask & (1u << k))) continue;
    const uint32_t bo = f.fd[k] + f.e - f.fi[k];
    const uint32_t q = bo - W.wb;
    if (f.fd[k] + f.off != olen || bo >= blen || q >= 64u) return 0;
    const uint32_t mk = min(m, min(blen - bo, 64u - q));
    uint32_t c = 0;
    while (c < mk) {
      const uint64_t mm = nz_bytes(lds_bytes8(W.w, q + c) ^ lds_bytes8(pred, j + c));
      if (mm) {
        c += (uint32_t)__builtin_ctzll(mm) >> 3;
        break;
      }
      c += 8;
    }
    m = min(mk, c);
    nlive++;
  }
  return m;
}

// The walk's edit-distance increases for up to four reads of one wave at
// once, one per 16-lane group (group_edinc, the dual engine's path: the same
// arithmetic as wave_heavy's register path; a row that outgrows a group's
// registers goes on in wave_edinc_mem). ls[q] (q < ng) are the lanes whose
// frontiers wait in gtmp[q]; their reads are perm[ls[q] * kEW + wave], their steps
// j of those lanes. kFirst: the first rewrite of a row in the chain leaves a
// copy in slot S (the rows are otherwise only touched at frontier diagonals,
// which a rollback restores from the node's LDS RStates), and each step's
// cost change goes to its ChainStep. Returns the backed-up-lanes mask and the
// groups whose wavefront outgrew its capacity (the chain stops before them).
struct GHOut {
  uint64_t bak;
  uint32_t fail;
};
template <bool kFirst>
__device__ __noinline__ GHOut chain_group_heavy(Lo<Ctl>& ctl, uint32_t j, uint32_t ls0, uint32_t ls1, uint32_t ls2,
                                                uint32_t ls3, uint32_t ng, uint64_t bak) {
  const int lane = lane_id();
  const uint32_t wave = (uint32_t)wave_id();
  // the chain's uniform arguments (run_chain_impl stores them)
  Sh<RState>* gtmp0 = ctl.gh_tmp + 4 * wave;
  Gm<uint32_t>* nwf = ctl.gh_nwf;
  Gm<uint32_t>* swf = ctl.gh_swf;
  const Gm<uint8_t>* rbytes = ctl.gh_rbytes;
  const Sh<uint2>* rt = ctl.gh_rt;
  const Gm<uint8_t>* con = ctl.gh_con;
  const uint32_t L0 = uni(ctl.gh_L0), wcap = uni(ctl.gh_wcap), list_n = uni(ctl.gh_list_n);
  (void)list_n;  // (bounds of the checked build's WC_IX)
  const uint32_t flags = uni(ctl.gh_flags);
  const bool early = (flags & 1u) != 0;
  const int cost_mode = (int)(flags >> 1);
  const int wc = uni(ctl.gh_wc);
  Sh<ChainStep>* cstep = ctl.gh_cstep;
  Sh<uint32_t>* list = ctl.gh_list;
  const uint32_t g = (uint32_t)lane >> 4, gl = (uint32_t)lane & 15u;
  const uint32_t ls[4] = {uni(ls0), uni(ls1), uni(ls2), uni(ls3)};
  ng = uni(ng);
  const uint32_t lsel = g == 0 ? ls[0] : g == 1 ? ls[1] : g == 2 ? ls[2] : ls[3];
  const bool gact = g < ng;
  Sh<RState>* gtmp = gtmp0 + g;
  const uint32_t rl = ctl.gh_perm[lsel * kEW + wave];
  const uint32_t jl = (uint32_t)__shfl((int)j, (int)lsel, 64);
  const uint32_t e_in = gact ? gtmp->e : 0u;
  Gm<uint32_t>* gwf = nwf + (uint64_t)rl * wcap;
  // (the read table: the LDS copy, or the HBM tables in the dual engine)
  const Gm<uint8_t>* rd = rt ? rbytes + (uint64_t)rt[rl].x * 16 : rbytes + ctl.gh_roff[ctl.gh_rbegin + rl];
  const uint32_t blen = rt ? rt[rl].y : ctl.gh_rlenp[ctl.gh_rbegin + rl];
  if (kFirst) {
    const bool first = gact && !((bak >> lsel) & 1ull);
    if (first) {
      Gm<uint32_t>* bdst = swf + (uint64_t)rl * wcap;
      for (uint32_t i = gl; i < 2 * e_in + 1; i += 16) bdst[i] = gwf[i];
      if (gl == 0) {
        const uint32_t k = atomicAdd(&ctl.chain_nbak, 1u);
        list[WC_IX(2 * k, list_n)] = rl;
        list[WC_IX(2 * k + 1, list_n)] = 2 * e_in + 1;
      }
    }
    const uint64_t fm = ballot(first && gl == 0);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if ((fm >> (16 * q)) & 1ull) bak |= 1ull << ls[q];
    __builtin_amdgcn_wave_barrier();
  }
  const GroupOut go = group_edinc<16>(gact, gtmp, gwf, rd, blen, con, L0 + jl, wc, early, wcap);
  uint32_t st = go.st, e_out = go.e;
  uint32_t t_ed = go.edinc, t_up = go.updates, t_wo = go.w_out, t_rb = go.rowb, t_cm = go.cmp;
  // rows that outgrew the group's registers (rare): the wave goes on with each
  uint64_t mem = ballot(gact && gl == 0 && st == kG_MEM);
  while (mem) {
    const uint32_t q = (uint32_t)__builtin_ctzll(mem) >> 4;
    mem &= mem - 1;
    const uint32_t rq = ctl.gh_perm[ls[q] * kEW + wave];
    const uint32_t jq = (uint32_t)__builtin_amdgcn_readlane((int)j, (int)ls[q]);
    const uint32_t eq = (uint32_t)__builtin_amdgcn_readlane((int)e_out, (int)(16 * q));
    WaveCounters cnt = {0, 0, 0, 0, 0, 0};
    uint32_t eo = 0;
    const Gm<uint8_t>* rdq = rt ? rbytes + (uint64_t)rt[rq].x * 16 : rbytes + ctl.gh_roff[ctl.gh_rbegin + rq];
    const uint32_t blq = rt ? rt[rq].y : ctl.gh_rlenp[ctl.gh_rbegin + rq];
    const bool okq = wave_edinc_mem(gtmp0 + q, nwf + (uint64_t)rq * wcap, eq, rdq, blq, con, L0 + jq, wc, early,
                                    wcap, cnt, eo);
    if (lane == 0) {
      t_ed += (uint32_t)cnt.edinc;
      t_up += (uint32_t)cnt.updates;
      t_wo += (uint32_t)cnt.w_out;
      t_rb += (uint32_t)cnt.rowb;
      t_cm += (uint32_t)cnt.compares;
    }
    if (g == q) {
      st = okq ? kG_DONE : kG_WCAP;
      e_out = eo;
    }
  }
  const uint32_t s_up = wave_sum_u32(t_up), s_wo = wave_sum_u32(t_wo), s_cm = wave_sum_u32(t_cm),
                 s_ed = wave_sum_u32(t_ed), s_rb = wave_sum_u32(t_rb);
  if (lane == 0) {
    atomicAdd((unsigned long long*)&ctl.chain_tot[0], (unsigned long long)s_up);
    atomicAdd((unsigned long long*)&ctl.chain_tot[1], (unsigned long long)s_wo);
    atomicAdd((unsigned long long*)&ctl.chain_tot[2], (unsigned long long)s_cm);
    atomicAdd((unsigned long long*)&ctl.chain_tot[3], (unsigned long long)s_ed);
    atomicAdd((unsigned long long*)&ctl.chain_tot[4], (unsigned long long)s_rb);
  }
  if (gact && gl == 0) {
    if (st == kG_WCAP) atomicMin(&ctl.chain_stop, jl - 1);
    else if (kFirst && e_out != e_in)  // the node cost from step jl on (chain_votes sums the changes)
      atomicAdd((unsigned long long*)&cstep[jl].cost,
                (unsigned long long)(cost_of(e_out, cost_mode) - cost_of(e_in, cost_mode)));
  }
  const uint64_t fb = ballot(gact && gl == 0 && st == kG_WCAP);
  GHOut o;
  o.bak = bak;
  o.fail = (uint32_t)((fb & 1ull) | ((fb >> 15) & 2ull) | ((fb >> 30) & 4ull) | ((fb >> 45) & 8ull));
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  return o;
}

// (C) push the K predicted symbols through every read, thread per read.
// Each lane walks its own read through the steps (a run-length walk): from
// step j, a read whose live tips all match the next m predictions takes the
// first m - 1 of those steps at once (their pushes extend every tip, and each
// of them nominates exactly the next prediction with weight 1: the code
// chain_prepare stored for every (step, read)); the step after the run, and
// any step where a tip mismatches or the read ends, takes the step path (push,
// tip bytes, nominations). A lane stops when its push needs an edit-distance
// increase; the wave then runs those, one read at a time (wave_heavy), and the
// lanes go on. The step aggregates are computed from the nominations after
// the walk (chain_votes); the walk only adds each step's cost change.
// kFirst: speculative pass; stores each step's nominations, leaves the final
// RStates in slot S. Replay pass: writes the final RStates to the LDS copy and
// the last step's nominations to rinfo (the analysis cache). Both passes add
// their work counters to ctl.chain_tot. Wavefront rows are written lazily
// (thread_push<kLazy>): only when a diagonal leaves the frontier, plus one
// flush of the final frontier.
template <bool kFirst>
__device__ inline void chain_walk(Eng& E, Lo<Ctl>& ctl, uint32_t top, uint32_t L0, uint32_t K, uint32_t S) {
  const int lane = lane_id(), wave = wave_id();
  // reads are dealt round-robin over the waves (read = lane * kEW + wave):
  // every wave walks a quarter of the reads, so the edit-distance increases,
  // which a wave handles one read at a time, are spread over all four
  if ((uint32_t)wave >= E.n) return;  // no reads in this wave (no barriers below)
  SUB_T0(tw);
  const DevConfig& cfg = E.cfg;
  const bool early = cfg.early != 0;
  const int wc = cfg.wildcard;
  SideView v = E.sv(top, 0);
  const uint32_t pos = (uint32_t)lane * kEW + (uint32_t)wave;
  const bool has = pos < E.n;
  const uint32_t r = has ? (uint32_t)E.L.cperm[pos] : pos;  // (chain_prepare's deal)
  Front f;
  f.e = kInactive;
  f.off = f.maxb = f.nscmp = f.mask = 0;
#pragma unroll
  for (int k = 0; k < kF; ++k) f.fi[k] = f.fd[k] = 0;
  Win W{E.L.cwin + (uint64_t)cwin_slot(min(r, E.n - 1), E.n) * kWinStride, 0};
  uint32_t blen = 0;
  if (has) {
    front_load(rstate_load(&E.L.hot[r]), f);
    W.wb = E.L.cwb[r];
    blen = E.rlen(r);
  }
  const bool active = has && f.e != kInactive;
  const uint32_t m0 = active ? (uint32_t)E.L.cm0[r] : 0u;  // the first quiet run (chain_prepare)
  Gm<uint32_t>* wf_row = v.wf + (uint64_t)r * E.wcap;
  uint32_t t_upd = 0, t_wout = 0, t_cmp = 0;
  uint64_t bak = 0;  // lanes whose row was backed up (wave-uniform)
  TipBytes x;        // bytes at the current tips
  // frontier entries sit at mask bits below 32 - clz(mask) (entries only
  // leave between rebuilds): kb, the wave's largest such bound, is a scalar
  // loop bound for the per-entry work (typically 1-3 of the kF = 8 slots)
  auto front_bound = [&]() {
    return wave_max_u32(active && f.mask ? 32u - (uint32_t)__builtin_clz(f.mask) : 0u);
  };
  uint32_t kb = front_bound();
  {
    const bool oob = win_tip_bytes(W, f, blen, kb, x) && active;
    if (kFirst && ballot(oob) && lane == 0) atomicMin(&ctl.chain_stop, 0u);
  }
  const Sh<uint8_t>* pred = E.L.cpred;  // pred[t] = N_t's symbol
#ifdef WC_NO_FF
  const bool ffon = false;
#else
  // (a wildcard read byte matches any push but nominates itself; it never
  // equals another prediction byte, so the byte compare ends a run there and
  // the step path takes it)
  const bool ffon = true;
#endif
  Sh<uint16_t>* nom_r = E.L.cnom + r * (K + 1);  // read r's row: cnom[r * (K + 1) + j]
  uint32_t j = 1;                      // this lane's next step
  uint32_t jend = active ? K : 0u;     // its last step (lowered when it stops the chain)
  bool pend = false;                   // step j's push needs an edit-distance increase
  // the rest of step j after its push: the bytes at the new tips and the
  // node's nominations (kFirst: into cnom; replay: the analysis cache at K)
  auto step_tail = [&]() {
    const bool oob = win_tip_bytes(W, f, blen, kb, x);
    const Nom o = chain_nominate(f, x, blen, L0 + j, kb);
    if (kFirst) {
      bool stop = oob;
      uint32_t code = kNomActive | (o.end ? kNomEnd : 0u) | (uint32_t)(o.sym & 0xFF) | (o.n == 1 ? kNomOne : 0u);
      if (o.n > 1) {
        const uint32_t idx = atomicAdd(&ctl.chain_novf, 1u);
        if (idx < kChainOvf) {
          E.L.covf[idx].set(o.sym, o.occ, o.split, o.n);
          code = (code & ~kNomSymMask) | kNomOvf | idx;
        } else {
          stop = true;
        }
      }
      nom_r[j] = (uint16_t)code;
      if (stop) {
        atomicMin(&ctl.chain_stop, j - 1);
        jend = j - 1;
      }
    } else if (j == K) {
      rinfo_store(&E.L.rinfo[r], o, f.e);
    }
    ++j;
  };
  for (;;) {
    const uint32_t stopv =
        kFirst ? uni(__hip_atomic_load(&ctl.chain_stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) : K;
    uint32_t lim = min(jend, stopv);
    SUB_T0(ta);
#ifdef WC_PHASE_PROF
    uint32_t it = 0;
#endif
    while (j <= lim) {
#ifdef WC_PHASE_PROF
      ++it;
#endif
      // ---- this read's quiet run from step j ----
      if (ffon && j < K && f.mask != 0 && f.maxb != blen) {
        uint32_t nlive;
        uint32_t m;
        if (j == 1) {  // chain_prepare computed it (cm0)
          m = min(m0, K);
          nlive = (uint32_t)__popc(f.mask);
        } else {
          m = lane_run(f, W, pred, blen, L0 + j - 1, j, K - j + 1, kb, nlive);
        }
        // the run's last push nominates the byte after the run: the step path takes it
        const uint32_t Q = m >= 1 ? min(m - 1, lim - j) : 0u;
        if (Q > 0) {
#pragma unroll
          for (int k = 0; k < kF; ++k) {
            if ((uint32_t)k >= kb) break;
            if (f.mask & (1u << k)) f.fd[k] += Q;
          }
          t_upd += Q;
          t_wout += Q * (2 * f.e + 1);
          t_cmp += Q * (f.nscmp + nlive);
          j += Q;
          win_tip_bytes(W, f, blen, kb, x);  // the tips moved (all inside the window)
        }
      }
      // ---- step j ----
      uint32_t cmp = 0;
      const bool heavy = chain_push(f, x, blen, L0 + j - 1, (uint32_t)pred[j], wc, early, wf_row, kb, cmp);
      t_cmp += cmp;
      if (heavy) {
        pend = true;
        break;
      }
      t_upd++;
      t_wout += 2 * f.e + 1;
      step_tail();
      lim = min(lim, jend);
    }
#ifdef WC_PHASE_PROF
    SUB_CNT(27, wave_max_u32(it));
    SUB_CNT(42, it);
    SUB_CNT(26, 1);
#endif
    SUB_T1(16, ta);
    uint64_t hm = ballot(pend);
    if (!hm) break;
    SUB_CNT(19, __popcll(hm));
    SUB_WADD(46, __popcll(hm));
    SUB_T0(tb);
// The 2-waves-per-SIMD build (WC_LOWLAT, 256 VGPRs) runs the edit-distance
// increases of up to four reads at once (chain_group_heavy); in the 4-wave build the call's
// register needs make the walk spill, which cost more than the overlap saves
// under load (cfg2 batch 32.7 vs 27.6 ms; one locus alone 19.1 vs 19.9 ms in
// the 2-wave build): one read at a time there.
#if (!defined(WC_LOWLAT) && !defined(WC_GROUP_HEAVY)) || defined(WC_SEQ_HEAVY)
    while (hm) {  // edit-distance increases: the wave works on one read at a time
      const int l = __builtin_ctzll(hm);
      hm &= hm - 1;
      const uint32_t jl = (uint32_t)__builtin_amdgcn_readlane((int)j, l);
      if (lane == l) front_store(&E.L.ctmp[4 * wave], f);
      wave_lds_sync();
      const uint32_t rl = (uint32_t)__builtin_amdgcn_readlane((int)r, l);
      const uint32_t e_in = uni(E.L.ctmp[4 * wave].e);
      Gm<uint32_t>* bdst = nullptr;
      if (kFirst && !((bak >> l) & 1ull)) {
        // first rewrite of this row in the chain: chain_heavy keeps a copy in
        // slot S (the rows are otherwise only touched at frontier diagonals,
        // which a rollback restores from the node's LDS RStates)
        bdst = E.sv(S, 0).wf + (uint64_t)rl * E.wcap;
        if (lane == 0) {
          const uint32_t k = atomicAdd(&ctl.chain_nbak, 1u);
          E.L.list[WC_IX(2 * k, list_entries(E.sides, E.nmax))] = rl;
          E.L.list[WC_IX(2 * k + 1, list_entries(E.sides, E.nmax))] = 2 * e_in + 1;
        }
        bak |= 1ull << l;
      }
      SUB_T0(tc);
      const uint32_t e_out = uni(chain_heavy(&E.L.ctmp[4 * wave], v.wf + (uint64_t)rl * E.wcap, E.read(rl), E.rlen(rl), v.con, L0 + jl,
                                             (uint32_t)pred[jl], wc, early, E.wcap, ctl.chain_tot, bdst));
      SUB_T1(51, tc);
      const bool ok = e_out != kInactive;
      wave_lds_sync();
      if (lane == 0) {
        if (!ok) atomicMin(&ctl.chain_stop, jl - 1);
        else if (kFirst && e_out != e_in)  // the node cost from step jl on (chain_votes sums the changes)
          atomicAdd((unsigned long long*)&E.L.cstep[jl].cost,
                    (unsigned long long)(cost_of(e_out, cfg.cost_mode) - cost_of(e_in, cfg.cost_mode)));
      }
      if (lane == l) {
        const RRaw t = rstate_load(&E.L.ctmp[4 * wave]);
        bool stop = !ok;
        if (kFirst && (rraw_flags(t) & kWide)) {  // not a thread-path state
          atomicMin(&ctl.chain_stop, jl - 1);
          stop = true;
        }
        if (stop) jend = jl - 1;
        front_load(t, f);
      }
      wave_lds_sync();
    }
#else
    // edit-distance increases: up to four reads at once, one per 16-lane
    // group (chain_group_heavy); the selected lanes hand their frontiers over
    // in LDS, so the call keeps the walk's register allocation
    while (hm) {
      uint32_t ls[4], ng = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        ls[q] = hm ? (uint32_t)__builtin_ctzll(hm) : 0u;
        if (hm) {
          hm &= hm - 1;
          ng++;
        }
      }
      const bool mine = (uint32_t)lane == ls[0] || (ng > 1 && (uint32_t)lane == ls[1]) ||
                        (ng > 2 && (uint32_t)lane == ls[2]) || (ng > 3 && (uint32_t)lane == ls[3]);
      const uint32_t myg = (uint32_t)lane == ls[0] ? 0u : (uint32_t)lane == ls[1] ? 1u : (uint32_t)lane == ls[2] ? 2u : 3u;
      if (mine) front_store(&E.L.ctmp[4 * wave + myg], f);
      wave_lds_sync();
      const GHOut gh = chain_group_heavy<kFirst>(ctl, j, ls[0], ls[1], ls[2], ls[3], ng, bak);
      bak = gh.bak;
      if (mine) {
        const RRaw t = rstate_load(&E.L.ctmp[4 * wave + myg]);
        bool stop = ((gh.fail >> myg) & 1u) != 0;
        if (kFirst && (rraw_flags(t) & kWide)) {  // not a thread-path state
          atomicMin(&ctl.chain_stop, j - 1);
          stop = true;
        }
        if (stop) jend = j - 1;
        front_load(t, f);
      }
      wave_lds_sync();
    }
#endif
    SUB_T0(td);
    kb = front_bound();  // rebuilt frontiers
    if (pend) {
      pend = false;
      if (j <= jend) step_tail();
    }
    SUB_T1(52, td);
    SUB_T1(17, tb);
  }
  if (!kFirst && has && !active) {
    Nom o;
    o.sym = o.occ = 0;
    o.n = o.split = o.end = 0;
    rinfo_store(&E.L.rinfo[r], o, f.e);
  }
  if (active) front_flush(f, wf_row);  // lazy rows: write the final frontier
  if (has) {
    if (kFirst) front_store(&E.sv(S, 0).rs[r], f);
    else front_store(&E.L.hot[r], f);
  }
  const uint32_t s_upd = wave_sum_u32(t_upd);
  const uint32_t s_wout = wave_sum_u32(t_wout);
  const uint32_t s_cmp = wave_sum_u32(t_cmp);
  if (lane == 0) {
    atomicAdd((unsigned long long*)&ctl.chain_tot[0], (unsigned long long)s_upd);
    atomicAdd((unsigned long long*)&ctl.chain_tot[1], (unsigned long long)s_wout);
    atomicAdd((unsigned long long*)&ctl.chain_tot[2], (unsigned long long)s_cmp);
  }
  SUB_T1(18, tw);
  SUB_WADD(45, __builtin_amdgcn_s_memtime() - tw);
}

// (D) Step aggregates, then per chain node N_j, j < Keff: ok[j] = exactly one
// passing candidate and it is the predicted symbol j+1 (consensus.rs:283-321).
// Aggregates of step j (1 <= j <= Keff) from the walk's nomination codes: the
// node cost (N_0's plus the walk's changes up to j), reads at their end, and
// the votes for the predicted next symbol (P) and for all other non-wildcard
// symbols (O) in exact 1/840ths, with the counts of multi-symbol reads and of
// fractional votes for the prediction. Lane j of every wave sums step j over
// the wave's share of the reads (a read's codes are one row: the lanes read
// consecutive entries) and adds it to the step with two LDS atomics. Then
// wave 0 decides the steps lane-parallel: unless the wildcard is predicted, P
// and O decide almost every step; the rest take the exact path, the wave per
// step (per-key f64 sums in read order, hashbrown key order).
__device__ inline void chain_votes(Eng& E, Lo<Ctl>& ctl, uint32_t Keff, uint32_t K) {
  const int lane = lane_id();
  const DevConfig& cfg = E.cfg;
  const uint32_t wsym = cfg.wildcard >= 0 ? (uint32_t)(uint8_t)cfg.wildcard : 0x100u;
  const uint32_t jl = (uint32_t)lane;  // Keff <= K < 64: one step per lane
  const bool lact = jl >= 1 && jl <= Keff;
  // N_K's next symbol is predicted too (chain_prepare, chain_pk): a full chain
  // decides N_K's votes, and its pop can be replayed like the others
  const bool pk = Keff == K && uni(ctl.chain_pk) != 0;
  const uint32_t pred = lact && (jl < K || pk) ? (uint32_t)E.L.cpred[jl + 1] : 0x100u;
  SUB_T0(ta);
  if (Keff > 0 && (uint32_t)wave_id() < E.n) {
    uint32_t np = 0, no = 0, nend = 0, nmul = 0, nfrac = 0, vpx = 0, vox = 0;
    const Sh<uint16_t>* col = E.L.cnom + (lact ? jl : 0u);
    // eight reads' codes per batch, loaded under one wait
    for (uint32_t r0 = (uint32_t)wave_id(); r0 < E.n; r0 += 8u * kEW) {
      uint32_t cc[8];
#pragma unroll
      for (uint32_t u = 0; u < 8; ++u) {
        const uint32_t r = r0 + u * kEW;
        cc[u] = lact && r < E.n ? (uint32_t)col[r * (K + 1)] : 0u;
      }
      uint32_t ovfm = 0;
#pragma unroll
      for (uint32_t u = 0; u < 8; ++u) {
        const uint32_t c = cc[u];
        if (c & kNomEnd) nend++;  // (kNomEnd only with kNomActive)
        const uint32_t s0 = (c & kNomQuiet) ? pred : (c & kNomSymMask);
        if (c & kNomOne) {
          if (s0 == pred) np++;
          else if (s0 != wsym) no++;
        }
        if (c & kNomOvf) ovfm |= 1u << u;
      }
      while (ovfm) {  // multi-symbol reads (rare): their fractions
        const uint32_t u = (uint32_t)__builtin_ctz(ovfm);
        ovfm &= ovfm - 1;
        const ChainOvf q = E.L.covf[cc[u] & kNomSymMask];
        const uint32_t unit = vote_unit(q.split());
        bool frac = false;
        for (uint32_t k = 0; k < q.n(); ++k) {
          const uint32_t w = unit * q.occ_at(k);
          const uint32_t sk = (uint32_t)((q.sym >> (8 * k)) & 0xFF);
          if (sk == pred) {
            vpx += w;
            frac = true;
          } else if (sk != wsym) {
            vox += w;
          }
        }
        nmul++;
        if (frac) nfrac++;
      }
    }
    if (lact) {
      const uint64_t P = (uint64_t)kVoteDen * np + vpx, O = (uint64_t)kVoteDen * no + vox;
      atomicAdd((unsigned long long*)&E.L.cstep[jl].po, (unsigned long long)(P | O << 32));
      atomicAdd((unsigned long long*)&E.L.cstep[jl].ef,
                (unsigned long long)((uint64_t)nend | (uint64_t)nmul << 16 | (uint64_t)nfrac << 32));
    }
  }
  __syncthreads();
  SUB_T1(20, ta);
  if (wave_id() != 0) return;
  SUB_T0(tb);
  // step costs: the running sum of the per-step changes
  {
    uint64_t d = lact ? E.L.cstep[jl].cost : 0ull;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t t = __shfl_up(d, (unsigned)o, 64);
      if (lane >= o) d += t;
    }
    if (lact) E.L.cstep[jl].cost = E.L.cstep[0].cost + d;
  }
  // Exact rational votes (P, O in 1/840ths); the f64 sums of the reference
  // differ from them by far less than 1/840, so strict inequalities carry
  // over. Only exact ties with fractional terms need the f64 path. With a
  // wildcard (not predicted here), its votes are left out of O: any other key
  // present drops it from the candidates (consensus.rs:556-561), and P > 0 is
  // one.
  int dec = 0;  // 1 ok, 0 not ok, -1 undecided
  if (jl >= 1 && (jl < Keff || (pk && jl == K))) {
    const auto& st = E.L.cstep[jl];
    const uint64_t P = st.po & 0xFFFFFFFFull, O = st.po >> 32;
    const uint64_t M = (uint64_t)kVoteDen * cfg.min_count;
    dec = -1;
    if (cfg.wildcard < 0 || pred != (uint32_t)(uint8_t)cfg.wildcard) {
      if (P == 0) dec = 0;  // the prediction is not a candidate
      else if (O < P && O < M) {
        // thr = min(min_count, max) and max = P when P < M: the prediction
        // passes, every other key stays below the threshold
        if (P != M || step_nfrac(st.ef) == 0) dec = 1;
      }
    }
    E.L.cstep[jl].ok = dec == 1 ? 1u : 0u;
  }
  uint64_t und = ballot(dec < 0);
  while (und) {
    const uint32_t j = (uint32_t)__builtin_ctzll(und);
    und &= und - 1;
    const uint32_t pj = (uint32_t)E.L.cpred[j + 1];
    const uint32_t multi = step_nmulti(E.L.cstep[j].ef) ? 1u : 0u;
    uint32_t m = 0, key = 0;
    double val = 0.0;
    bool ok = wave_votes_core([&](uint32_t r) { return nom_decode(E.L.cnom[r * (K + 1) + j], E.L.covf, pj); },
                              [&](uint32_t) { return 1.0; }, E.n, false, multi != 0, cfg.wildcard, cfg.min_count,
                              cfg.min_af == 0.0, m, key, val);
    if (ok) {
      const double max_obs = m ? wave_max_f64((uint32_t)lane < m ? val : 0.0) : (double)cfg.min_count;
      const double thr = fmin((double)cfg.min_count, max_obs);
      const uint64_t pass = ballot((uint32_t)lane < m && val >= thr);
      ok = __popcll((unsigned long long)pass) == 1 &&
           (uint32_t)__builtin_amdgcn_readlane((int)key, __builtin_ctzll(pass)) == pj;
    }
    SUB_CNT(25, 1);
    if (lane == 0) E.L.cstep[j].ok = ok ? 1u : 0u;
  }
  SUB_T1(21, tb);
}

// (E) wave 0: replay the pops of N_1.. on the scalar search state
// (consensus.rs:224-251 / dual_consensus.rs:340-397) and commit the accepted
// prefix. Returns j* = number of chain nodes generated. The step-local tests
// (max_err, capacity, reached_end, one passing candidate, and N_j popping
// next: strictly above the best other queued node, whatever the heap's tie
// order) are evaluated by lanes over j at once; only the PQueueTracker
// threshold walk is sequential, on registers. Other queued nodes of the
// tracker count in its total: when the threshold passes a length, their
// count there (HBM) leaves the total, as increment_threshold does. A dual
// search's consensus-2 tracker does not change during a chain of
// single-consensus nodes (its loop at N_0's pop already left it stable).
__device__ inline uint32_t chain_accept(Eng& E, Lo<Ctl>& ctl, uint32_t L0, uint32_t Keff) {
  const DevConfig& cfg = E.cfg;
  const bool early = cfg.early != 0;
  const uint32_t lane = (uint32_t)lane_id();
  const Gm<uint32_t>* lc = E.trk;  // PQueueTracker length counts of the queued nodes
  Gm<uint32_t>* pc = E.trk + (E.lcap + 2);
  const uint32_t jl = 1 + lane;  // Keff <= kChainMax < 64: one step per lane
  const uint32_t hn = ctl.heap_n;  // other queued nodes (N_0 is popped)
  bool bad = true;
  if (jl < Keff) {
    const auto& st = E.L.cstep[jl];
    const uint32_t n_end = step_nend(st.ef);
    const bool reached = early ? (n_end == E.n) : (n_end > 0);
    bad = st.cost > ctl.max_err || (uint64_t)E.L.cpc[jl] >= cfg.max_capacity_per_size || reached || !st.ok;
    if (hn > 0) bad |= !prio_less(E.L.heap[0], HeapEntry{st.cost, L0 + jl, 0u});
  }
  const uint32_t jbad = 1 + (uint32_t)__builtin_ctzll(ballot(bad));  // lane 63 is always bad
  uint32_t jstar = Keff >= 1 ? 1u : 0u;
  uint64_t thr = ctl.trk_thr[0], farthest = ctl.farthest[0], lcnst = ctl.last_constraint[0];
  uint64_t others = ctl.trk_total[0];
  SUB_T0(ta);
  // Fast path, exact: with others + 1 <= max_queue_size the queue-size clause
  // of the threshold loop is false at every step (others does not change
  // while no threshold moves), and the constraint clause stays false while
  // last_constraint + (j - 1) < max_nodes_wo_constraint; L0 + 1 >= thr keeps
  // every L above the threshold. Then every step up to the first bad one
  // passes with the tracker untouched but for the constraint count and
  // farthest.
  const uint32_t jlim = min(Keff, jbad);
  const bool fast = jlim >= 2 && others + 1 <= cfg.max_queue_size &&
                    lcnst + (uint64_t)(jlim - 2) < cfg.max_nodes_wo_constraint && (uint64_t)L0 + 1 >= thr;
  if (fast) {
    lcnst += jlim - 1;
    farthest = max(farthest, (uint64_t)(L0 + jlim - 1));
    jstar = jlim;
  }
  for (uint32_t j = 1; !fast && j < Keff && j < jbad; ++j) {
    const uint64_t L = L0 + j;
    uint64_t t_thr = thr, t_l = lcnst, t_oth = others;
    while ((t_oth + (L >= t_thr ? 1u : 0u) > cfg.max_queue_size || t_l >= cfg.max_nodes_wo_constraint) &&
           t_thr < farthest) {
      SUB_CNT(40, 1);
      if (t_oth) t_oth -= trk_load(&lc[t_thr]);
      t_thr++;
      t_l = 0;
    }
    if (L < t_thr) break;
    thr = t_thr;
    others = t_oth;
    lcnst = t_l + 1;
    farthest = max(farthest, L);
    jstar = j + 1;
  }
  SUB_T1(41, ta);
  if (jl < jstar) pc[L0 + jl] = E.L.cpc[jl] + 1;
  if (lane == 0) {
    ctl.trk_thr[0] = thr;
    ctl.trk_total[0] = others;
    ctl.farthest[0] = farthest;
    ctl.last_constraint[0] = lcnst;
    if (jstar > 1) {
      ctl.cnt[S_POPS] += jstar - 1;
      ctl.cnt[S_EXPLORED] += jstar - 1;
      ctl.cnt[S_PEAKQ] = max(ctl.cnt[S_PEAKQ], (uint64_t)hn + 1);
    }
  }
  return jstar;
}

// Not inlined: the chain has its own register allocation (no spills in the
// walk); the caller saves its live registers once per chain.
// Run one chain from the popped node `top` (length L0, hot in LDS) whose
// single child symbol is s1. Returns j* (uniform); for j* > 0 the chain node
// N_j* is in slot `top`/LDS, queued, with its nominations cached; j* == 0
// leaves everything as it was. kDual: `top` is a single-consensus node of a
// DualConsensusDWFA search (its stay-single children, dual_consensus.rs:
// 655-679); the virtual pops also grow the active-read minimum per length
// (:497-513).
template <bool kDual>
__device__ __forceinline__ uint32_t run_chain_impl(Eng E, Lo<Ctl>& ctl, uint32_t top, uint32_t L0, int s1) {
  const int tid = threadIdx.x;
  SUB_T0(te);
  if (tid == 0) {
    ctl.chain_pk = 0;
    // (the dual engine's chains end at forks of its search more often: their
    // length adapts, so a chain that ends early wastes few speculative steps)
    const uint32_t K = min(kDual ? min(E.chain, ctl.chain_kcur) : E.chain, E.lcap - L0);
    ctl.chain_k = 0;
    if (K >= 2 && ctl.nfree > 0 && E.n <= (uint32_t)kEB) {  // (the walk deals one read per thread)
      ctl.chain_k = K;
      ctl.chain_slot = E.L.freestack[WC_IX(--ctl.nfree, E.pcap)];
      ctl.chain_stop = K;
      ctl.chain_novf = 0;
      ctl.chain_nochain = 0;
      ctl.chain_nbak = 0;
      for (int k = 0; k < (int)(sizeof(ctl.chain_tot) / 8); ++k) ctl.chain_tot[k] = 0;
      E.L.cpred[1] = (uint8_t)s1;
    }
  }
  __syncthreads();
  const uint32_t K = uni(ctl.chain_k);
  // (reset only here: every wave has read the previous chain's chain_next in
  // the kernel's loop condition before it reached the barrier above)
  if (tid == 0) ctl.chain_next = 0;
  if (K == 0) return 0;
  const uint32_t S = uni(ctl.chain_slot);
  if (tid == 0) {  // chain_group_heavy's arguments (read after chain_prepare's barriers)
    ctl.gh_nwf = E.sv(top, 0).wf;
    ctl.gh_swf = E.sv(S, 0).wf;
    ctl.gh_rbytes = E.rbytes;
    ctl.gh_con = E.sv(top, 0).con;
    ctl.gh_rt = E.L.rt;
    ctl.gh_roff = E.roff;
    ctl.gh_rlenp = E.rlenp;
    ctl.gh_rbegin = E.P.read_begin;
    ctl.gh_tmp = E.L.ctmp;
    ctl.gh_cstep = E.L.cstep;
    ctl.gh_list = E.L.list;
    ctl.gh_perm = E.L.cperm;
    ctl.gh_L0 = L0;
    ctl.gh_wcap = E.wcap;
    ctl.gh_list_n = (uint32_t)list_entries(E.sides, E.nmax);
    ctl.gh_flags = (E.cfg.early ? 1u : 0u) | (uint32_t)E.cfg.cost_mode << 1;
    ctl.gh_wc = E.cfg.wildcard;
  }
  for (uint32_t i = tid; i < (K + 1) * (uint32_t)(sizeof(ChainStep) / 4); i += kEB)
    ((Sh<uint32_t>*)E.L.cstep)[i] = 0;
  SUB_T1(43, te);
  chain_prepare(E, ctl, top, L0, K, S);
  __syncthreads();
  PH_MARK(8);
  if (uni(ctl.chain_nochain)) {
    if (tid == 0) E.L.freestack[WC_IX(ctl.nfree++, E.pcap)] = S;
    __syncthreads();
    return 0;
  }
  chain_walk<true>(E, ctl, top, L0, K, S);
  __syncthreads();
  PH_MARK(9);
  const uint32_t Keff = uni(ctl.chain_stop);
  chain_votes(E, ctl, Keff, K);
  __syncthreads();
  PH_MARK(10);
  // A full chain whose N_K has exactly one passing candidate (its predicted
  // child) replays N_K's pop too, and its child starts the next chain at
  // once (single engine; the kernel falls back to pushing that child when
  // the next chain does not start): no literal pop between the chains.
  // Only where the next chain can start (room for two more steps).
  const bool ext = !kDual && Keff == K && uni(ctl.chain_pk) != 0 && L0 + K + 2 <= E.lcap;
  if (wave_id() == 0) {
    const uint32_t js = chain_accept(E, ctl, L0, ext ? K + 1 : Keff);
    if (tid == 0) {
      ctl.chain_len = js;
      if (js >= K && Keff == K) {  // the speculative pass is the committed work
        ctl.cnt[S_UPDATES] += ctl.chain_tot[0];
        ctl.cnt[S_WOUT] += ctl.chain_tot[1];
        ctl.cnt[S_COMPARES] += ctl.chain_tot[2];
        ctl.cnt[S_EDINC] += ctl.chain_tot[3];
        ctl.cnt[S_ROWB] += ctl.chain_tot[4];
      }
      for (int k = 0; k < 5; ++k) ctl.chain_tot[k] = 0;
    }
  }
  __syncthreads();
  PH_MARK(11);
  const uint32_t jstar = uni(ctl.chain_len);
  const bool full = jstar >= K && Keff == K;  // (jstar = K + 1: N_K popped too)
  SideView v = E.sv(top, 0), b = E.sv(S, 0);
  if (full) {
    // every step accepted: the speculative final state is the node
    for (uint32_t r = tid; r < E.n; r += kEB) {
      const RRaw t = rstate_load(&b.rs[r]);
      rstate_store(&E.L.hot[r], t);
      RInfoReg x = nom_decode(E.L.cnom[r * (K + 1) + K], E.L.covf, 0u);
      Nom o;
      o.n = x.n;
      o.split = x.split;
      o.sym = x.sym;
      o.end = (E.L.cnom[r * (K + 1) + K] & kNomEnd) ? 1u : 0u;
      o.occ = (uint64_t)(x.occ.x & 0xFF) | (uint64_t)((x.occ.x >> 16) & 0xFF) << 8 |
              (uint64_t)(x.occ.y & 0xFF) << 16 | (uint64_t)((x.occ.y >> 16) & 0xFF) << 24 |
              (uint64_t)(x.occ.z & 0xFF) << 32 | (uint64_t)((x.occ.z >> 16) & 0xFF) << 40 |
              (uint64_t)(x.occ.w & 0xFF) << 48 | (uint64_t)((x.occ.w >> 16) & 0xFF) << 56;
      rinfo_store(&E.L.rinfo[r], o, rraw_e(t));
    }
  } else {
    // roll the node's wavefront rows back: rows rewritten by an edit-distance
    // increase come back from their copies, then every frontier diagonal of
    // the node gets its value from the node's RState (the only entries the
    // thread path writes)
    const int lane = lane_id();
    const uint32_t nb = uni(ctl.chain_nbak);
    for (uint32_t k = wave_id(); k < nb; k += kEW) {
      const uint32_t r = E.L.list[WC_IX(2 * k, list_entries(E.sides, E.nmax))], W = E.L.list[WC_IX(2 * k + 1, list_entries(E.sides, E.nmax))];
      const Gm<uint32_t>* src = b.wf + (uint64_t)r * E.wcap;
      Gm<uint32_t>* dst = v.wf + (uint64_t)r * E.wcap;
      for (uint32_t i = lane; i < W; i += 64) dst[i] = src[i];
    }
    __syncthreads();
    for (uint32_t r = tid; r < E.n; r += kEB) {
      Front f;
      front_load(rstate_load(&E.L.hot[r]), f);
      if (f.e == kInactive) continue;
      Gm<uint32_t>* row = v.wf + (uint64_t)r * E.wcap;
#pragma unroll
      for (int k = 0; k < kF; ++k)
        if ((f.mask >> k) & 1u) row[f.fi[k]] = f.fd[k];
    }
    __syncthreads();
    if (jstar > 0) chain_walk<false>(E, ctl, top, L0, jstar, S);
  }
  __syncthreads();
  if (tid == 0) {
    if (!full) {  // the replay pass is the committed work
      ctl.cnt[S_UPDATES] += ctl.chain_tot[0];
      ctl.cnt[S_WOUT] += ctl.chain_tot[1];
      ctl.cnt[S_COMPARES] += ctl.chain_tot[2];
      ctl.cnt[S_EDINC] += ctl.chain_tot[3];
      ctl.cnt[S_ROWB] += ctl.chain_tot[4];
    }
#ifdef WC_PHASE_PROF
    ctl.ph[15] += 1ull + (full ? (1ull << 20) : 0ull) + ((uint64_t)min(jstar, K) << 40);
    for (int k = 0; k < 3; ++k) {  // wave_heavy's timers over every wave (both passes)
      ctl.ph[48 + k] += ctl.chain_tot[5 + k];
      ctl.chain_tot[5 + k] = 0;
    }
#endif
    E.L.freestack[WC_IX(ctl.nfree++, E.pcap)] = S;
    if (kDual) ctl.chain_kcur = full ? min(2 * K, E.chain) : max(4u, jstar + 1);
    // the queue as the literal pops leave it: each N_j (j < j*) was pushed,
    // then popped as the maximum, which moves the other entries along its
    // path (their tie order depends on the layout)
    if (ctl.heap_n > 1)
      for (uint32_t j = 1; j < jstar; ++j) {
        heap_push(E.L.heap, ctl.heap_n, E.pcap, HeapEntry{E.L.cstep[j].cost, L0 + j, top});
        (void)heap_pop(E.L.heap, ctl.heap_n, E.pcap);
      }
    if (kDual) {
      // every explored N_j (j < j*) extends the per-length active counts
      // (no read activates past the last activation point)
      // (one HBM load: the count repeats along the chain)
      uint32_t nt = ~0u, amv = 0;
      for (uint32_t j = 1; j < jstar; ++j) {
        const uint32_t tl = L0 + j;
        if (ctl.am_len == tl + 1 && tl + 1 < E.lcap + 2) {
          if (nt == ~0u) {
            nt = E.total_active[tl];
            amv = (uint32_t)max(E.cfg.min_count, ceil_u64(E.cfg.min_af * (double)nt));
          }
          E.total_active[tl + 1] = nt;
          E.active_min[tl + 1] = amv;
          ctl.am_len++;
        }
      }
    }
    if (jstar == K + 1) {
      // N_K was popped (virtually, like N_1..N_K-1): its one child, the
      // predicted symbol, is the kernel's next chain (or, if that chain does
      // not start, its literal push); nothing is queued
      E.L.meta[top].len[0] = L0 + K;
      ctl.chain_next = 1;
      ctl.chain_sym = E.L.cpred[K + 1];
    } else if (jstar > 0) {
      const auto& st = E.L.cstep[jstar];
      const uint32_t clen = L0 + jstar;
      E.L.meta[top].len[0] = clen;
      E.tracker(ctl, 0).insert(clen);
      heap_push(E.L.heap, ctl.heap_n, E.pcap, HeapEntry{st.cost, clen, top});
      ctl.cache_slot = top;
      ctl.cache_nend = step_nend(st.ef);
      ctl.cache_multi = step_nmulti(st.ef) ? 1u : 0u;
    }
  }
  __syncthreads();
  return jstar;
}
// the out-of-line entries (plain functions: their register allocation is
// fitted to the one caller, so the call saves no callee-saved registers)
// The single engine passes its context by reference: measured faster on cfg2
// than rebuilding it in the callee (34.5 vs 33.3 ms per launch; the callee
// then saves ~45 callee-saved VGPRs per chain), at the price of the context
// living in scratch in that kernel. The dual engine's chain builds (wcd)
// rebuild it from the kernel arguments (callee_eng).
__device__ __noinline__ uint32_t run_chain_single(Eng& Eref, Lo<Ctl>& ctl, uint32_t top, uint32_t L0, int s1) {
  return run_chain_impl<false>(eng_uniform(Eref), ctl, top, L0, s1);
}
#ifdef WC_CHAIN_REBUILD  // (experiment build: the context rebuilt from the kernel arguments)
__device__ __noinline__ uint32_t run_chain_single_k(KArgs kp, DevProblem P, Sh<uint8_t>* sbase, Lo<Ctl>& ctl,
                                                    uint32_t top, uint32_t L0, int s1) {
  return run_chain_impl<false>(callee_eng(kp, P, sbase), ctl, top, L0, s1);
}
#endif
__device__ __noinline__ uint32_t run_chain_dual_single(KArgs kp, DevProblem P, Sh<uint8_t>* sbase, Lo<Ctl>& ctl,
                                                       uint32_t top, uint32_t L0, int s1) {
  return run_chain_impl<true>(callee_eng(kp, P, sbase), ctl, top, L0, s1);
}
