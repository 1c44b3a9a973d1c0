// Linear-chain run-ahead over dual-consensus nodes (included by engine.hip,
// after chain.hip.hpp whose primitives it uses).
//
// In a DualConsensusDWFA search (dual_consensus.rs:240-787) a dual node with
// both consensuses still open mostly has exactly one child: one passing
// symbol per side, pushed on both sides at once (:554-650), and that child is
// popped next. run_dual_chain walks up to K such steps speculatively, thread
// per read over both sides of the read:
//   1. per walking side, predict the next K-1 symbols (plurality of the
//      side's reads' upcoming bases);
//   2. every thread pushes the predictions through its read's DWFAs of both
//      sides (DWFALite::update, dynamic_wfa.rs:75-99; ED increases by the
//      thread's wave), prunes the side that fell dual_max_ed_delta behind
//      (prune_dwfa, :1030-1045), and records each step's nominations per side,
//      the read's cost (the cheaper side, :1092-1168), its end flags and the
//      Some(dwfa) counts;
//   3. per step the votes of each walking side are evaluated exactly (as in
//      chain_votes), with reached_all_end / reached_consensus_end (:1174-1233)
//      and the imbalance test at pop (:340-397); the pops are replayed on the
//      scalar search state (consensus-2 PQueueTracker, the queue's best other
//      node, max_err, active_min_count growth);
//   4. the accepted prefix is committed exactly as that many literal pops;
//      on a rejected step the rows are restored and the prefix is replayed.
// A side locked before the chain (a child that took None there) is not
// walked: its DWFAs only take part in pruning, cost and end flags.

// one side's end flag (reached_baseline_end, dynamic_wfa.rs:232-234) from its frontier
__device__ __forceinline__ bool front_end(const Front& f, uint32_t blen) {
  uint32_t mb = f.maxb;
#pragma unroll
  for (int k = 0; k < kF; ++k)
    if ((f.mask >> k) & 1u) mb = max(mb, f.fd[k] + f.e - f.fi[k]);
  return mb == blen;
}

// per-side views of the chain area (engine_shared chain_lds_bytes)
struct DualChainArea {
  Sh<DualStep>* step;
  Sh<uint16_t>* nom[2];
  Sh<uint8_t>* win[2];
  Sh<uint32_t>* wb[2];
  Sh<uint8_t>* pred[2];
};
__device__ __forceinline__ DualChainArea dual_area(const Eng& E) {
  DualChainArea a;
  const uint32_t K = E.chain;
  a.step = (Sh<DualStep>*)E.L.cstep;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    a.nom[s] = E.L.cnom + (uint64_t)s * (K + 1) * E.nmax;
    a.win[s] = E.L.cwin + (uint64_t)s * win_slots(E.nmax, chain_waves(kEW)) * kWinStride;
    a.wb[s] = E.L.cwb + (uint64_t)s * E.nmax;
    a.pred[s] = E.L.cpred + (uint64_t)s * (K + 2);
  }
  return a;
}

// (B) read windows of the walking sides, capacities, predictions
__device__ inline void dual_chain_prepare(Eng& E, Lo<Ctl>& ctl, const DualChainArea& A, uint32_t top, uint32_t L0,
                                          uint32_t K, uint32_t walk, const uint32_t (&l0)[2]) {
  const int tid = threadIdx.x, lane = lane_id();
  for (uint32_t it = tid; it < 2 * E.n; it += kEB) {
    const uint32_t s = it >= E.n ? 1u : 0u, r = it - s * E.n;
    if (!((walk >> s) & 1u)) continue;
    const RRaw h = rstate_load(&E.sv(top, s).rs[r]);
    if (rraw_e(h) != kInactive && (rraw_flags(h) & kWide)) atomicOr(&ctl.chain_nochain, 1u);
    Front f;
    front_load(h, f);
    uint32_t lo = kInactive;
    if (f.e != kInactive) {
      const uint32_t blen = E.rlen(r);
#pragma unroll
      for (int k = 0; k < kF; ++k)
        if ((f.mask >> k) & 1u) lo = min(lo, min(f.fd[k] + f.e - f.fi[k], blen));
    }
    if (lo == kInactive) lo = 0;
    const uint32_t wb = lo & ~15u;
    const Gm<uint4>* g = (const Gm<uint4>*)(E.read(r) + wb);
    Sh<uint32_t>* w = (Sh<uint32_t>*)(A.win[s] + (uint64_t)cwin_slot(r, E.n) * kWinStride);
    const uint4 a0 = g[0], a1 = g[1], a2 = g[2], a3 = g[3];
    w[0] = a0.x, w[1] = a0.y, w[2] = a0.z, w[3] = a0.w;
    w[4] = a1.x, w[5] = a1.y, w[6] = a1.z, w[7] = a1.w;
    w[8] = a2.x, w[9] = a2.y, w[10] = a2.z, w[11] = a2.w;
    w[12] = a3.x, w[13] = a3.y, w[14] = a3.z, w[15] = a3.w;
    A.wb[s][r] = wb;
  }
  const Gm<uint32_t>* pc = E.trk + 3 * (E.lcap + 2);  // the consensus-2 tracker's processed counts
  for (uint32_t j = tid; j <= K; j += kEB) E.L.cpc[j] = (j >= 1) ? trk_load(&pc[L0 + j]) : 0u;
  __syncthreads();
  // predictions: every wave predicts the steps t = 1 + wave (mod kEW) of both
  // walking sides from the upcoming bases of reads 0..63 on that side
  const uint32_t wave = (uint32_t)wave_id();
  for (uint32_t s = 0; s < 2; ++s) {
    if (!((walk >> s) & 1u)) continue;
    uint32_t bo_tip = kInactive, blen = 0, wb = 0;
    const Sh<uint8_t>* win = A.win[s] + (uint64_t)cwin_slot(min((uint32_t)lane, E.n - 1), E.n) * kWinStride;
    if ((uint32_t)lane < E.n) {
      Front f;
      front_load(rstate_load(&E.sv(top, s).rs[lane]), f);
      if (f.e != kInactive) {
        wb = A.wb[s][lane];
        blen = E.rlen(lane);
#pragma unroll
        for (int k = kF - 1; k >= 0; --k)
          if ((f.mask >> k) & 1u) {
            const uint32_t bo = f.fd[k] + f.e - f.fi[k];
            if (f.fd[k] + f.off == l0[s] && bo < blen) bo_tip = bo;
          }
      }
    }
    for (uint32_t t = 1 + wave; t < K; t += kEW) {
      const uint32_t q = bo_tip + t - wb;
      const uint32_t x = (bo_tip != kInactive && bo_tip + t < blen && q < 64u) ? (uint32_t)win[q] : 0x100u;
      uint64_t rem = ballot(x != 0x100u);
      uint32_t best = 0x100u, bestc = 0;
      while (rem) {
        const int l = __builtin_ctzll(rem);
        const uint32_t sy = (uint32_t)__builtin_amdgcn_readlane((int)x, l);
        const uint64_t mm = ballot(x == sy);
        const uint32_t c = (uint32_t)__popcll((unsigned long long)mm);
        if (c > bestc) {
          bestc = c;
          best = sy;
        }
        rem &= ~mm;
      }
      if (best == 0x100u) {
        if (lane == 0) atomicMin(&ctl.chain_stop, t);
        break;
      }
      if (lane == 0) A.pred[s][t + 1] = (uint8_t)best;
    }
  }
  __syncthreads();
  // the predictions extend each walking side's consensus buffer in place
  // (positions >= its length are not part of the node)
  for (uint32_t s = 0; s < 2; ++s)
    if (((walk >> s) & 1u) && tid >= 1 && (uint32_t)tid <= K) E.sv(top, s).con[l0[s] + tid - 1] = A.pred[s][tid];
  con_store_wait();  // (the walk's ED increases read them)
  __syncthreads();
  l1_drop();
}

// (C) push the predictions through both sides of every read, thread per read,
// from the node's RStates in its slot. kFirst: speculative pass (step
// records, final RStates to slot S, the node's own stay as they were); replay
// pass: final RStates to the node's slot. Rows are written lazily (chain_push).
template <bool kFirst>
__device__ inline void dual_chain_walk(Eng& E, Lo<Ctl>& ctl, const DualChainArea& A, uint32_t top, uint32_t K,
                                       uint32_t S, uint32_t walk, const uint32_t (&l0)[2]) {
  const int lane = lane_id(), wave = wave_id();
  if ((uint32_t)wave >= E.n) return;
  const DevConfig& cfg = E.cfg;
  const bool early = cfg.early != 0;
  const int wc = cfg.wildcard;
  const uint32_t wsym = wc >= 0 ? (uint32_t)(uint8_t)wc : 0x100u;
  const uint64_t delta = cfg.dual_max_ed_delta;
  const uint32_t r = (uint32_t)lane * kEW + (uint32_t)wave;
  const bool has = r < E.n;
  const uint32_t blen = has ? E.rlen(r) : 0u;
  Front f[2];
  Win W[2];
  TipBytes x[2];
  uint32_t kb[2];
  bool act[2], lend[2];
  Gm<uint32_t>* row[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    f[s].e = kInactive;
    f[s].off = f[s].maxb = f[s].nscmp = f[s].mask = 0;
#pragma unroll
    for (int k = 0; k < kF; ++k) f[s].fi[k] = f[s].fd[k] = 0;
    W[s] = Win{A.win[s] + (uint64_t)cwin_slot(min(r, E.n - 1), E.n) * kWinStride, 0};
    if (has) {
      front_load(rstate_load(&E.sv(top, s).rs[r]), f[s]);
      W[s].wb = A.wb[s][r];
    }
    act[s] = has && f[s].e != kInactive;
    lend[s] = act[s] && front_end(f[s], blen);  // a locked side's end flag never changes
    row[s] = E.sv(top, s).wf + (uint64_t)r * E.wcap;
    kb[s] = wave_max_u32(act[s] && f[s].mask ? 32u - (uint32_t)__builtin_clz(f[s].mask) : 0u);
    x[s].lo = x[s].hi = 0;
    if ((walk >> s) & 1u) {
      const bool oob = win_tip_bytes(W[s], f[s], blen, kb[s], x[s]) && act[s];
      if (kFirst && ballot(oob) && lane == 0) atomicMin(&ctl.chain_stop, 0u);
    }
  }
  Sh<RState>* tmp = &E.L.ctmp[wave];
  uint32_t t_upd = 0, t_wout = 0, t_cmp = 0;
  uint64_t bak[2] = {0, 0};  // lanes whose row of side s was backed up (wave-uniform)
  uint64_t a_cost = 0, a_po0 = 0, a_po1 = 0, a_ef0 = 0, a_ef1 = 0;
  uint32_t a_some = 0, jlast = 0;
  for (uint32_t j = 1; j <= K; ++j) {
    const uint32_t stopv =
        kFirst ? uni(__hip_atomic_load(&ctl.chain_stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) : K;
    if (kFirst && j > stopv) break;
    bool heavy[2] = {false, false};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (!((walk >> s) & 1u) || !act[s]) continue;
      uint32_t cmp = 0;
      heavy[s] = chain_push(f[s], x[s], blen, l0[s] + j - 1, (uint32_t)A.pred[s][j], wc, early, row[s], kb[s], cmp);
      t_cmp += cmp;
      if (!heavy[s]) {
        t_upd++;
        t_wout += 2 * f[s].e + 1;
      }
    }
    bool rebuilt = false;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (!((walk >> s) & 1u)) continue;
      uint64_t hm = ballot(heavy[s]);
      rebuilt |= hm != 0;
      const uint32_t olen = l0[s] + j;
      while (hm) {  // edit-distance increase: the wave works on one read at a time
        const int l = __builtin_ctzll(hm);
        hm &= hm - 1;
        if (lane == l) front_store(tmp, f[s]);
        wave_lds_sync();
        const uint32_t rl = (uint32_t)l * kEW + (uint32_t)wave;
        const uint32_t e_in = uni(tmp->e);
        Gm<uint32_t>* bdst = nullptr;
        if (kFirst && !((bak[s] >> l) & 1ull)) {
          bdst = E.sv(S, s).wf + (uint64_t)rl * E.wcap;
          if (lane == 0) {
            const uint32_t k = atomicAdd(&ctl.chain_nbak, 1u);
            E.L.list[WC_IX(2 * k, list_entries(E.sides, E.nmax))] = rl | (uint32_t)s << 31;
            E.L.list[WC_IX(2 * k + 1, list_entries(E.sides, E.nmax))] = 2 * e_in + 1;
          }
          bak[s] |= 1ull << l;
        }
        SideView v = E.sv(top, s);
        const uint32_t e_out = chain_heavy(tmp, v.wf + (uint64_t)rl * E.wcap, E.read(rl), E.rlen(rl), v.con, olen,
                                           (uint32_t)A.pred[s][j], wc, early, E.wcap, ctl.chain_tot, bdst);
        wave_lds_sync();
        if (e_out == kInactive && lane == 0) atomicMin(&ctl.chain_stop, j - 1);
        if (lane == l) {
          const RRaw t = rstate_load(tmp);
          if (kFirst && (rraw_flags(t) & kWide)) atomicMin(&ctl.chain_stop, j - 1);  // not a thread-path state
          front_load(t, f[s]);
        }
        wave_lds_sync();
      }
    }
    if (rebuilt)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        kb[s] = wave_max_u32(act[s] && f[s].mask ? 32u - (uint32_t)__builtin_clz(f[s].mask) : 0u);
    // prune_dwfa (dual_consensus.rs:1030-1045): the side more than delta behind
    // is dropped for this read
    if (act[0] && act[1]) {
      if ((uint64_t)f[0].e + delta < (uint64_t)f[1].e) {
        act[1] = false;
        f[1].e = kInactive;
      } else if ((uint64_t)f[1].e + delta < (uint64_t)f[0].e) {
        act[0] = false;
        f[0].e = kInactive;
      }
    }
    // bytes at the new tips, this node's nominations per walking side
    bool oob = false;
    Nom o[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      o[s].sym = o[s].occ = 0;
      o[s].n = o[s].split = o[s].end = 0;
      if (!((walk >> s) & 1u)) {
        o[s].end = lend[s] ? 1u : 0u;
        continue;
      }
      oob |= win_tip_bytes(W[s], f[s], blen, kb[s], x[s]) && act[s];
      if (act[s]) o[s] = chain_nominate(f[s], x[s], blen, l0[s] + j, kb[s]);
    }
    if (kFirst) {
      bool stop = oob;
      uint64_t po[2] = {0, 0}, ef[2] = {0, 0};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if (!((walk >> s) & 1u)) {
          ef[s] = (uint64_t)__popcll((unsigned long long)ballot(act[s] && o[s].end));
          continue;
        }
        if (has) {
          uint32_t code = 0;
          if (act[s]) {
            code = kNomActive | (o[s].end ? kNomEnd : 0u) | (uint32_t)(o[s].sym & 0xFF) | (o[s].n == 1 ? kNomOne : 0u);
            if (o[s].n > 1) {
              const uint32_t idx = atomicAdd(&ctl.chain_novf, 1u);
              if (idx < kChainOvf) {
                E.L.covf[idx].set(o[s].sym, o[s].occ, o[s].split, o[s].n);
                code = (code & ~kNomSymMask) | kNomOvf | idx;
              } else {
                stop = true;
              }
            }
          }
          A.nom[s][(uint64_t)j * E.nmax + r] = (uint16_t)code;
        }
        // votes for the side's predicted next symbol (P) and every other
        // non-wildcard symbol (O), in 1/840ths (chain_votes)
        const uint32_t pred = j < K ? (uint32_t)A.pred[s][j + 1] : 0x100u;
        uint32_t vp = 0, vo = 0;
        bool frac = false;
        if (act[s] && o[s].n > 0) {
          if (o[s].n == 1) {
            const uint32_t s0 = (uint32_t)(o[s].sym & 0xFF);
            if (s0 == pred) vp = kVoteDen;
            else if (s0 != wsym) vo = kVoteDen;
          } else {
            const uint32_t unit = vote_unit(o[s].split);
            for (uint32_t k = 0; k < o[s].n; ++k) {
              const uint32_t c = unit * (uint32_t)((o[s].occ >> (8 * k)) & 0xFF);
              const uint32_t sk = (uint32_t)((o[s].sym >> (8 * k)) & 0xFF);
              if (sk == pred) {
                vp += c;
                frac = true;
              } else if (sk != wsym) {
                vo += c;
              }
            }
          }
        }
        const uint64_t nend = (uint64_t)__popcll((unsigned long long)ballot(act[s] && o[s].end));
        const uint64_t mm = ballot(act[s] && o[s].n > 1);
        const uint64_t nmul = (uint64_t)__popcll((unsigned long long)mm);
        const uint64_t nfrac = (uint64_t)__popcll((unsigned long long)ballot(frac));
        if (mm == 0)
          po[s] = (uint64_t)kVoteDen * (uint64_t)__popcll((unsigned long long)ballot(vp != 0)) |
                  ((uint64_t)kVoteDen * (uint64_t)__popcll((unsigned long long)ballot(vo != 0)) << 32);
        else
          po[s] = (uint64_t)wave_sum_u32(vp) | ((uint64_t)wave_sum_u32(vo) << 32);
        ef[s] = nend | nmul << 16 | nfrac << 32;
      }
      // the read's cost: the cheaper of its Some sides (dual_consensus.rs:1092-1168)
      uint64_t best = ~0ull;
#pragma unroll
      for (int s = 0; s < 2; ++s)
        if (act[s]) best = min(best, cost_of(f[s].e, cfg.cost_mode));
      const uint64_t wcost = wave_sum_u64(best == ~0ull ? 0ull : best);
      const uint32_t n0 = (uint32_t)__popcll((unsigned long long)ballot(act[0]));
      const uint32_t n1 = (uint32_t)__popcll((unsigned long long)ballot(act[1]));
      const uint32_t ne = (uint32_t)__popcll((unsigned long long)ballot((act[0] && o[0].end) || (act[1] && o[1].end)));
      if (ballot(stop) && lane == 0) atomicMin(&ctl.chain_stop, j - 1);
      if ((uint32_t)lane == j) {
        a_cost = wcost;
        a_po0 = po[0];
        a_po1 = po[1];
        a_ef0 = ef[0];
        a_ef1 = ef[1];
        a_some = n0 | n1 << 10 | ne << 20;
      }
      jlast = j;
    }
  }
  if (kFirst && lane >= 1 && (uint32_t)lane <= jlast) {
    auto& st = A.step[lane];
    atomicAdd((unsigned long long*)&st.cost, (unsigned long long)a_cost);
    atomicAdd((unsigned long long*)&st.po[0], (unsigned long long)a_po0);
    atomicAdd((unsigned long long*)&st.po[1], (unsigned long long)a_po1);
    atomicAdd((unsigned long long*)&st.ef[0], (unsigned long long)a_ef0);
    atomicAdd((unsigned long long*)&st.ef[1], (unsigned long long)a_ef1);
    atomicAdd(&st.some, a_some);
  }
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    if (((walk >> s) & 1u) && act[s]) front_flush(f[s], row[s]);  // lazy rows: write the final frontier
    if (has) front_store(&E.sv(kFirst ? S : top, s).rs[r], f[s]);
  }
  const uint32_t s_upd = wave_sum_u32(t_upd);
  const uint32_t s_wout = wave_sum_u32(t_wout);
  const uint32_t s_cmp = wave_sum_u32(t_cmp);
  if (lane == 0) {
    atomicAdd((unsigned long long*)&ctl.chain_tot[0], (unsigned long long)s_upd);
    atomicAdd((unsigned long long*)&ctl.chain_tot[1], (unsigned long long)s_wout);
    atomicAdd((unsigned long long*)&ctl.chain_tot[2], (unsigned long long)s_cmp);
  }
}

// (D) per chain node N_j, j < K: every walking side has exactly one passing
// candidate, its predicted symbol (dual_consensus.rs:554-601 with min_af 0:
// thr = min(min_count, max)), and has not reached its consensus end (then
// None would be an option as well: a second child)
__device__ inline void dual_chain_votes(Eng& E, Lo<Ctl>& ctl, const DualChainArea& A, uint32_t K, uint32_t walk) {
  const int lane = lane_id();
  const DevConfig& cfg = E.cfg;
  const bool early = cfg.early != 0;
  for (uint32_t j = 1 + wave_id(); j < K; j += kEW) {
    auto& st = A.step[j];
    const uint32_t some = st.some;
    bool ok = true;
    for (uint32_t s = 0; s < 2 && ok; ++s) {
      if (!((walk >> s) & 1u)) continue;
      const uint64_t po = st.po[s], ef = st.ef[s];
      const uint32_t nsome = (some >> (10 * s)) & 1023u, nend = step_nend(ef);
      if (early ? nend == nsome : nend > 0) {  // reached_consensus_end (:1203-1233)
        ok = false;
        break;
      }
      const uint32_t pred = (uint32_t)A.pred[s][j + 1];
      const uint64_t P = po & 0xFFFFFFFFull, O = po >> 32;
      const uint64_t M = (uint64_t)kVoteDen * cfg.min_count;
      int dec = -1;
      if (cfg.wildcard < 0 || pred != (uint32_t)(uint8_t)cfg.wildcard) {
        if (P == 0) dec = 0;
        else if (O < P && O < M && (P != M || step_nfrac(ef) == 0)) dec = 1;
      }
      if (dec < 0) {
        const Sh<uint16_t>* nom = A.nom[s] + (uint64_t)j * E.nmax;
        uint32_t m = 0, key = 0;
        double val = 0.0;
        bool vok = wave_votes_core([&](uint32_t r) { return nom_load(nom, E.L.covf, r); },
                                   [&](uint32_t) { return 1.0; }, E.n, false, step_nmulti(ef) != 0, cfg.wildcard,
                                   cfg.min_count, cfg.min_af == 0.0, m, key, val);
        if (vok) {
          const double max_obs = m ? wave_max_f64((uint32_t)lane < m ? val : 0.0) : (double)cfg.min_count;
          const double thr = fmin((double)cfg.min_count, max_obs);
          const uint64_t pass = ballot((uint32_t)lane < m && val >= thr);
          vok = __popcll((unsigned long long)pass) == 1 &&
                (uint32_t)__builtin_amdgcn_readlane((int)key, __builtin_ctzll(pass)) == pred;
        }
        dec = vok ? 1 : 0;
      }
      ok = dec == 1;
    }
    if (lane == 0) st.ok = ok ? 1u : 0u;
  }
}

// (E) wave 0: replay the pops of N_1.. (dual_consensus.rs:340-397 on the
// consensus-2 tracker; N_j has length L0 + j) and commit the accepted prefix.
__device__ inline uint32_t dual_chain_accept(Eng& E, Lo<Ctl>& ctl, const DualChainArea& A, uint32_t L0, uint32_t Keff) {
  const DevConfig& cfg = E.cfg;
  const bool early = cfg.early != 0;
  const uint32_t lane = (uint32_t)lane_id();
  const Gm<uint32_t>* lc = E.trk + 2 * (E.lcap + 2);
  Gm<uint32_t>* pc = E.trk + 3 * (E.lcap + 2);
  const uint32_t jl = 1 + lane;
  const uint32_t hn = ctl.heap_n;
  const uint64_t am = cfg.min_count;  // active_min_count at every length (min_af 0, dual_consensus.rs:497-513)
  bool bad = true;
  if (jl < Keff) {
    const auto& st = A.step[jl];
    const uint32_t some = st.some;
    const uint32_t n0 = some & 1023u, n1 = (some >> 10) & 1023u, ne = (some >> 20) & 1023u;
    const bool reached = early ? (ne == E.n) : (ne > 0);
    bad = st.cost > ctl.max_err || (uint64_t)E.L.cpc[jl] >= cfg.max_capacity_per_size || reached || !st.ok ||
          n0 < am || n1 < am;
    if (hn > 0) bad |= !prio_less(E.L.heap[0], HeapEntry{st.cost, L0 + jl, 0u});
  }
  const uint32_t jbad = 1 + (uint32_t)__builtin_ctzll(ballot(bad));
  uint32_t jstar = Keff >= 1 ? 1u : 0u;
  uint64_t thr = ctl.trk_thr[1], farthest = ctl.farthest[1], lcnst = ctl.last_constraint[1];
  uint64_t others = ctl.trk_total[1];
  for (uint32_t j = 1; j < Keff && j < jbad; ++j) {
    const uint64_t L = L0 + j;
    uint64_t t_thr = thr, t_l = lcnst, t_oth = others;
    while ((t_oth + (L >= t_thr ? 1u : 0u) > cfg.max_queue_size || t_l >= cfg.max_nodes_wo_constraint) &&
           t_thr < farthest) {
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
  if (jl < jstar) pc[L0 + jl] = E.L.cpc[jl] + 1;
  if (lane == 0) {
    ctl.trk_thr[1] = thr;
    ctl.trk_total[1] = others;
    ctl.farthest[1] = farthest;
    ctl.last_constraint[1] = lcnst;
    if (jstar > 1) {
      ctl.cnt[S_POPS] += jstar - 1;
      ctl.cnt[S_EXPLORED] += jstar - 1;
      ctl.cnt[S_PEAKQ] = max(ctl.cnt[S_PEAKQ], (uint64_t)hn + 1);
    }
  }
  return jstar;
}

// Run one chain from the popped dual node `top` (lengths tl[0..1], max L0)
// whose only child pushes syms[s] on the sides in `walk` (the others stay
// locked; `flags` = the child's flags). Returns j* (uniform): for j* > 0 the
// node N_j* is in slot `top`, queued.
__device__ __noinline__ uint32_t run_dual_chain(KArgs kp, DevProblem P, Sh<uint8_t>* sbase, Lo<Ctl>& ctl, uint32_t top,
                                                uint32_t tl0, uint32_t tl1, uint32_t walk, uint32_t sym0, uint32_t sym1,
                                                uint32_t flags) {
  Eng E = callee_eng(kp, P, sbase);
  const int tid = threadIdx.x;
  const uint32_t l0[2] = {tl0, tl1};
  const uint32_t L0 = max(tl0, tl1);
  const DualChainArea A = dual_area(E);
  if (tid == 0) {
    uint32_t K = min(min(E.chain, ctl.chain_kcur), E.lcap - L0);  // (adaptive, as in run_chain)
    ctl.chain_k = 0;
    if (K >= 2 && ctl.nfree > 0) {
      ctl.chain_k = K;
      ctl.chain_slot = E.L.freestack[WC_IX(--ctl.nfree, E.pcap)];
      ctl.chain_stop = K;
      ctl.chain_novf = 0;
      ctl.chain_nochain = 0;
      ctl.chain_nbak = 0;
      for (int k = 0; k < 5; ++k) ctl.chain_tot[k] = 0;
      A.pred[0][1] = (uint8_t)sym0;
      A.pred[1][1] = (uint8_t)sym1;
    }
  }
  __syncthreads();
  const uint32_t K = uni(ctl.chain_k);
  if (K == 0) return 0;
  const uint32_t S = uni(ctl.chain_slot);
  for (uint32_t i = tid; i < (K + 1) * (uint32_t)(sizeof(DualStep) / 4); i += kEB) ((Sh<uint32_t>*)A.step)[i] = 0;
  __syncthreads();
  dual_chain_prepare(E, ctl, A, top, L0, K, walk, l0);
  __syncthreads();
  if (uni(ctl.chain_nochain)) {
    if (tid == 0) E.L.freestack[WC_IX(ctl.nfree++, E.pcap)] = S;
    __syncthreads();
    return 0;
  }
  dual_chain_walk<true>(E, ctl, A, top, K, S, walk, l0);
  __syncthreads();
  const uint32_t Keff = uni(ctl.chain_stop);
  dual_chain_votes(E, ctl, A, Keff, walk);
  __syncthreads();
  if (wave_id() == 0) {
    const uint32_t js = dual_chain_accept(E, ctl, A, L0, Keff);
    if (tid == 0) {
      ctl.chain_len = js;
      if (js == K && Keff == K) {
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
  const uint32_t jstar = uni(ctl.chain_len);
  if (jstar == K && Keff == K) {
    // every step accepted: the speculative final RStates are the node's
    for (uint32_t s = 0; s < 2; ++s)
      for (uint32_t r = tid; r < E.n; r += kEB) rstate_store(&E.sv(top, s).rs[r], rstate_load(&E.sv(S, s).rs[r]));
  } else {
    // roll the rows back (ED-increase copies, then the frontier diagonals of
    // the node's RStates) and replay the accepted prefix
    const int lane = lane_id();
    const uint32_t nb = uni(ctl.chain_nbak);
    for (uint32_t k = wave_id(); k < nb; k += kEW) {
      const uint32_t rs = E.L.list[WC_IX(2 * k, list_entries(E.sides, E.nmax))];
      const uint32_t W = E.L.list[WC_IX(2 * k + 1, list_entries(E.sides, E.nmax))];
      const uint32_t r = rs & 0x7FFFFFFFu, s = rs >> 31;
      const Gm<uint32_t>* src = E.sv(S, s).wf + (uint64_t)r * E.wcap;
      Gm<uint32_t>* dst = E.sv(top, s).wf + (uint64_t)r * E.wcap;
      for (uint32_t i = lane; i < W; i += 64) dst[i] = src[i];
    }
    __syncthreads();
    for (uint32_t it = tid; it < 2 * E.n; it += kEB) {
      const uint32_t s = it >= E.n ? 1u : 0u, r = it - s * E.n;
      if (!((walk >> s) & 1u)) continue;
      Front f;
      front_load(rstate_load(&E.sv(top, s).rs[r]), f);
      if (f.e == kInactive) continue;
      Gm<uint32_t>* row = E.sv(top, s).wf + (uint64_t)r * E.wcap;
#pragma unroll
      for (int k = 0; k < kF; ++k)
        if ((f.mask >> k) & 1u) row[f.fi[k]] = f.fd[k];
    }
    __syncthreads();
    if (jstar > 0) dual_chain_walk<false>(E, ctl, A, top, jstar, S, walk, l0);
  }
  __syncthreads();
  // the node N_j*: metadata, queued
  if (tid == 0) {
    if (!(jstar == K && Keff == K)) {
      ctl.cnt[S_UPDATES] += ctl.chain_tot[0];
      ctl.cnt[S_WOUT] += ctl.chain_tot[1];
      ctl.cnt[S_COMPARES] += ctl.chain_tot[2];
      ctl.cnt[S_EDINC] += ctl.chain_tot[3];
      ctl.cnt[S_ROWB] += ctl.chain_tot[4];
    }
    E.L.freestack[WC_IX(ctl.nfree++, E.pcap)] = S;
    ctl.chain_kcur = (jstar == K && Keff == K) ? min(2 * K, E.chain) : max(4u, jstar + 1);
    if (ctl.heap_n > 1)
      for (uint32_t j = 1; j < jstar; ++j) {
        heap_push(E.L.heap, ctl.heap_n, E.pcap, HeapEntry{A.step[j].cost, L0 + j, top});
        (void)heap_pop(E.L.heap, ctl.heap_n, E.pcap);
      }
    uint32_t nt = ~0u, amv = 0;  // (one HBM load: the count repeats along the chain)
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
    if (jstar > 0) {
      const auto& st = A.step[jstar];
      SlotMeta m;
      m.len[0] = l0[0] + ((walk & 1u) ? jstar : 0u);
      m.len[1] = l0[1] + ((walk & 2u) ? jstar : 0u);
      m.nsome[0] = st.some & 1023u;
      m.nsome[1] = (st.some >> 10) & 1023u;
      m.flags = flags;
      meta_put(E.L.meta[top], m);
      const uint32_t clen = L0 + jstar;
      E.tracker(ctl, 1).insert(clen);
      heap_push(E.L.heap, ctl.heap_n, E.pcap, HeapEntry{st.cost, clen, top});
    }
  }
  __syncthreads();
  return jstar;
}

// The dual engine's one out-of-line call into a chain (kind 1: the
// single-consensus walk of chain.hip.hpp on an LDS copy of side 1; kind 2: the
// two-sided walk): one call site keeps the kernel's register allocation
// around it small.
__device__ __noinline__ uint32_t run_engine_chain(KArgs kp, DevProblem P, Sh<uint8_t>* sbase, Lo<Ctl>& ctl,
                                                  uint32_t top, uint32_t kind, uint32_t tl0, uint32_t tl1,
                                                  uint32_t walk, uint32_t sym0, uint32_t sym1, uint32_t flags) {
  if (kind == 2) return run_dual_chain(kp, P, sbase, ctl, top, tl0, tl1, walk, sym0, sym1, flags);
  Eng E = callee_eng(kp, P, sbase);
  hot_fetch(E, top, 0);
  __syncthreads();
  const uint32_t jstar = run_chain_dual_single(kp, P, sbase, ctl, top, tl0, (int)sym0);
  if (jstar) {
    hot_store(E, top, 0);
    __syncthreads();
  }
  return jstar;
}
