// Device-resident consensus engines for MI355X (gfx950).
//
// ConsensusDWFA::consensus (consensus.rs:139-351) runs entirely on the GPU:
// one workgroup per consensus problem pulls problems from a global work
// counter and executes the reference's least-cost-first search with the
// reference's exact pop order (priority-queue 1.x heap),
// candidate order (hashbrown/FxHash iteration, Appendix B) and f64 vote
// summation order. Node DWFA state lives in a per-workgroup node pool in HBM
// (copy on branch, in place on single extension); the heap, node metadata and
// per-read nomination summaries live in LDS.
//
// Per pop: ANALYZE (per-read tips + end flags), optional FINALIZE of the
// popped node on scratch, VOTES (ordered f64 sums), then PUSH of every child
// (the per-read DWFA update, dynamic_wfa.rs:75-99) with the cost reduction
// fused in.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "engine_common.hip.hpp"

namespace wc {

struct Ctl {
  uint32_t prob, n, read_begin, max_read_len;
  uint32_t heap_n, nfree;
  uint32_t status;
  uint32_t action;  // 0 expand, 1 ignore, 2 done
  uint32_t top_slot, top_len;
  uint64_t top_cost;
  uint32_t n_end;
  uint32_t multi;
  uint32_t ovf;
  uint32_t reached;
  uint64_t cost_acc;
  uint64_t max_err;
  uint64_t farthest[2], last_constraint[2];
  uint64_t trk_total[2], trk_thr[2];
  uint32_t n_ret;
  int32_t store_idx;
  uint32_t nchild;
  uint32_t cur_child;
  uint8_t child_sym[kKout];
  uint32_t child_slot[kKout];
  uint64_t child_cost[kKout];
  uint32_t nkeys;
  uint8_t keys[kKout];
  double vals[kKout];
  uint64_t cnt[S_NSTAT];
};

struct Lds {
  HeapEntry* heap;
  uint32_t* freestack;
  SlotMeta* meta;
  RInfo* rinfo;    // [sides][nmax]
  uint32_t* fe;    // [sides][nmax]
};

__device__ inline Lds carve(uint8_t* smem, uint32_t sides, uint32_t pcap, uint32_t nmax) {
  Lds l;
  uint8_t* p = smem;
  l.heap = (HeapEntry*)p;
  p += (uint64_t)pcap * sizeof(HeapEntry);
  l.freestack = (uint32_t*)p;
  p += align16((uint64_t)pcap * 4);
  l.meta = (SlotMeta*)p;
  p += (uint64_t)pcap * sizeof(SlotMeta);
  l.rinfo = (RInfo*)p;
  p += (uint64_t)sides * nmax * sizeof(RInfo);
  l.fe = (uint32_t*)p;
  return l;
}

// ---- priority-queue 1.x emulation (thread 0 only) ----
__device__ inline bool prio_less(const HeapEntry& a, const HeapEntry& b) {
  if (a.cost != b.cost) return a.cost > b.cost;  // Reverse(cost)
  return a.len < b.len;
}
__device__ inline void heap_push(HeapEntry* h, uint32_t& n, HeapEntry e) {
  uint32_t pos = n++;
  while (pos > 0) {
    uint32_t parent = (pos - 1) / 2;
    if (!prio_less(h[parent], e)) break;
    h[pos] = h[parent];
    pos = parent;
  }
  h[pos] = e;
}
__device__ inline HeapEntry heap_pop(HeapEntry* h, uint32_t& n) {
  HeapEntry top = h[0];
  n--;
  h[0] = h[n];
  uint32_t i = 0;
  if (n > 1) {
    for (;;) {
      uint32_t l = 2 * i + 1, r = 2 * i + 2, largest = i;
      if (l < n) {
        if (prio_less(h[largest], h[l])) largest = l;
        if (r < n && prio_less(h[largest], h[r])) largest = r;
      }
      if (largest == i) break;
      HeapEntry t = h[i];
      h[i] = h[largest];
      h[largest] = t;
      i = largest;
    }
  }
  return top;
}

// ---- PQueueTracker (pqueue_tracker.rs:10-144), thread 0 only ----
struct TrackerRef {
  uint32_t* lc;
  uint32_t* pc;
  uint64_t* total;
  uint64_t* thr;
  uint64_t cap;
  __device__ void insert(uint32_t v) {
    lc[v]++;
    if (v >= *thr) (*total)++;
  }
  __device__ void remove(uint32_t v) {
    lc[v]--;
    if (v >= *thr) (*total)--;
  }
  __device__ void increment_threshold() {
    *total -= lc[*thr];
    (*thr)++;
  }
  __device__ bool at_capacity(uint32_t v) const { return pc[v] >= cap; }
  __device__ bool process(uint32_t v) {
    if (pc[v] >= cap) return false;
    pc[v]++;
    return true;
  }
};

__device__ inline void flush_counters(Ctl& ctl, const WaveCounters& wc) {
  if (lane_id() == 0) {
    if (wc.updates) atomicAdd((unsigned long long*)&ctl.cnt[S_UPDATES], (unsigned long long)wc.updates);
    if (wc.w_out) atomicAdd((unsigned long long*)&ctl.cnt[S_WOUT], (unsigned long long)wc.w_out);
    if (wc.compares) atomicAdd((unsigned long long*)&ctl.cnt[S_COMPARES], (unsigned long long)wc.compares);
    if (wc.edinc) atomicAdd((unsigned long long*)&ctl.cnt[S_EDINC], (unsigned long long)wc.edinc);
    if (wc.finalizes) atomicAdd((unsigned long long*)&ctl.cnt[S_FINALIZES], (unsigned long long)wc.finalizes);
  }
}

// ---- VOTES: ConsensusNode::get_extension_candidates (consensus.rs:540-564) ----
// Wave 0 only. Outer-map insertion order = first appearance over (read index,
// inner iteration position); values are summed per key strictly in read order
// (the reference's f64 order). Writes ctl.keys/vals in iteration order, with
// the wildcard removed when other keys exist. Returns false on > kKout keys.
__device__ inline bool wave_votes(Ctl& ctl, const RInfo* ri, uint32_t n, const float* weights_unused, int wc) {
  const int lane = lane_id();
  uint32_t known[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint8_t ins[kKout];
  uint32_t nk = 0;
  bool ok = true;
  for (uint32_t base = 0; base < n && ok; base += 64) {
    uint32_t r = base + lane;
    for (;;) {
      uint32_t cand = 0xFFFF;
      if (r < n && ri[r].e != kInactive) {
        const RInfo& x = ri[r];
        for (uint32_t k = 0; k < x.n; ++k) {
          uint8_t s = x.sym[k];
          if (!((known[s >> 5] >> (s & 31)) & 1u)) {
            cand = s;
            break;
          }
        }
      }
      uint64_t m = ballot(cand != 0xFFFF);
      if (!m) break;
      int first = __ffsll((unsigned long long)m) - 1;
      uint32_t s = (uint32_t)__shfl((int)cand, first, 64);
      if (nk == kKout) {
        ok = false;
        break;
      }
      ins[nk++] = (uint8_t)s;
      known[s >> 5] |= 1u << (s & 31);
    }
  }
  if (!ok) return false;
  uint8_t ord[kKout];
  fx_order(ins, nk, ord);
  // iteration order keys, wildcard removal (consensus.rs:556-561)
  uint8_t keys[kKout];
  uint32_t m = 0;
  bool drop_wc = wc >= 0 && nk > 1;
  for (uint32_t k = 0; k < nk; ++k) {
    uint8_t s = ins[ord[k]];
    if (drop_wc && s == (uint8_t)wc) continue;
    keys[m++] = s;
  }
  // per-key ordered sums: lane j owns key j
  double acc = 0.0;
  if ((uint32_t)lane < m) {
    uint8_t key = keys[lane];
    for (uint32_t r = 0; r < n; ++r) {
      const RInfo& x = ri[r];
      if (x.e == kInactive) continue;
      for (uint32_t k = 0; k < x.n; ++k) {
        if (x.sym[k] == key) {
          acc += (double)x.occ[k] / (double)x.split;
          break;
        }
      }
    }
    ctl.keys[lane] = key;
    ctl.vals[lane] = acc;
  }
  if (lane == 0) ctl.nkeys = m;
  return true;
}

// ---- ConsensusDWFA engine ----
__global__ void __launch_bounds__(kBlock) single_engine_kernel(EngineArgs A) {
  extern __shared__ __align__(16) uint8_t smem[];
  __shared__ Ctl ctl;
  const int tid = threadIdx.x;
  const int lane = lane_id();
  const int wave = wave_id();
  const DevConfig& cfg = A.cfg;
  const int wc = cfg.wildcard;
  const bool early = cfg.early != 0;
  const uint32_t nmax = A.nmax, wcap = A.wcap, lcap = A.lcap, pcap = A.pcap;
  Lds L = carve(smem, 1, pcap, nmax);
  uint8_t* ws = A.ws + (uint64_t)blockIdx.x * A.ws_stride;
  const uint64_t sbytes = slot_bytes(1, nmax, wcap, lcap);
  uint32_t* trk_lc = (uint32_t*)(ws + (uint64_t)pcap * sbytes);
  uint32_t* trk_pc = trk_lc + (lcap + 2);
  uint32_t* scratch_base =
      (uint32_t*)(ws + (uint64_t)pcap * sbytes + align16((uint64_t)4 * (lcap + 2) * 4) + align16((uint64_t)2 * (lcap + 2) * 4));
  uint32_t* scratch = scratch_base + (uint64_t)wave * (wcap + 2);
  const uint32_t rmax = A.rmax;
  const uint64_t rbytes_sz = result_bytes(1, nmax, lcap);

  for (;;) {
    if (tid == 0) ctl.prob = atomicAdd(A.work_counter, 1u);
    __syncthreads();
    const uint32_t prob = ctl.prob;
    if (prob >= A.n_problems) break;
    const DevProblem P = A.problems[prob];
    const uint32_t n = P.n_reads;
    uint8_t* outp = A.out + (uint64_t)prob * A.out_stride;

    // ---- init ----
    if (tid == 0) {
      ctl.heap_n = 0;
      ctl.nfree = pcap;
      ctl.status = ST_OK;
      ctl.max_err = ~0ull;
      ctl.farthest[0] = 0;
      ctl.last_constraint[0] = 0;
      ctl.trk_total[0] = 0;
      ctl.trk_thr[0] = 0;
      ctl.n_ret = 0;
      for (int s = 0; s < S_NSTAT; ++s) ctl.cnt[s] = 0;
    }
    for (uint32_t i = tid; i < pcap; i += kBlock) L.freestack[i] = pcap - 1 - i;
    for (uint32_t i = tid; i < 2 * (lcap + 2); i += kBlock) trk_lc[i] = 0;
    __syncthreads();
    // root node (consensus.rs:384-403): reads with offset None start active
    const uint32_t root = pcap - 1;  // top of the free stack
    {
      SideView v = side_view(ws + (uint64_t)root * sbytes, 0, nmax, wcap, lcap);
      for (uint32_t r = tid; r < n; r += kBlock) {
        const bool act = A.ractivate[P.read_begin + r] < 0;
        v.e[r] = act ? 0u : kInactive;
        v.off[r] = 0;
        v.wf[(uint64_t)r * wcap] = 0;
      }
    }
    if (tid == 0) {
      ctl.nfree = pcap - 1;
      L.meta[root].len[0] = 0;
      L.meta[root].flags = 0;
      TrackerRef t{trk_lc, trk_pc, &ctl.trk_total[0], &ctl.trk_thr[0], cfg.max_capacity_per_size};
      t.insert(0);
      heap_push(L.heap, ctl.heap_n, HeapEntry{0, 0, root});
    }
    __syncthreads();

    // ---- search loop (consensus.rs:224-340) ----
    for (;;) {
      if (tid == 0) {
        TrackerRef t{trk_lc, trk_pc, &ctl.trk_total[0], &ctl.trk_thr[0], cfg.max_capacity_per_size};
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
          HeapEntry top = heap_pop(L.heap, ctl.heap_n);
          t.remove(top.len);
          ctl.top_slot = top.slot;
          ctl.top_len = top.len;
          ctl.top_cost = top.cost;
          if (top.cost > ctl.max_err || top.len < ctl.trk_thr[0] || t.at_capacity(top.len)) {
            ctl.cnt[S_IGNORED]++;
            L.freestack[ctl.nfree++] = top.slot;
            ctl.action = 1;
          } else {
            ctl.farthest[0] = max(ctl.farthest[0], (uint64_t)top.len);
            ctl.cnt[S_EXPLORED]++;
            ctl.last_constraint[0]++;
            if (!t.process(top.len)) ctl.status = 4;  // "Capacity is full"
            ctl.action = 0;
          }
        }
        ctl.n_end = 0;
        ctl.multi = 0;
        ctl.ovf = 0;
        ctl.cost_acc = 0;
      }
      __syncthreads();
      if (ctl.action == 2) break;
      if (ctl.action == 1) continue;
      if (ctl.status != ST_OK) break;

      const uint32_t top = ctl.top_slot;
      const uint32_t len = ctl.top_len;
      SideView tv = side_view(ws + (uint64_t)top * sbytes, 0, nmax, wcap, lcap);

      // ---- ANALYZE: tips + reached_baseline_end per read ----
      {
        for (uint32_t r = wave; r < n; r += kWaves) {
          const uint32_t e = tv.e[r];
          if (e == kInactive) {
            if (lane == 0) {
              L.rinfo[r].e = kInactive;
              L.rinfo[r].n = 0;
              L.rinfo[r].end = 0;
            }
            continue;
          }
          const uint64_t ro = A.roff[P.read_begin + r];
          const uint32_t blen = A.rlen[P.read_begin + r];
          bool ok = wave_analyze_read(tv.wf + (uint64_t)r * wcap, e, tv.off[r], A.rbytes + ro, blen, len, &L.rinfo[r]);
          if (lane == 0) {
            if (!ok) atomicOr(&ctl.ovf, 1u);
            if (L.rinfo[r].end) atomicAdd(&ctl.n_end, 1u);
          }
        }
      }
      __syncthreads();
      if (tid == 0) {
        const uint32_t ne = ctl.n_end;
        ctl.reached = early ? (ne == n) : (ne > 0);
        if (ctl.ovf) ctl.status = 11u;
      }
      __syncthreads();
      if (ctl.status != ST_OK) break;

      // ---- FINALIZE a clone when any (all, with early termination) read is at its end ----
      if (ctl.reached) {
        WaveCounters cnt = {0, 0, 0, 0, 0};
        for (uint32_t r = wave; r < n; r += kWaves) {
          const uint32_t e = tv.e[r];
          if (e == kInactive) {
            if (lane == 0) atomicOr(&ctl.ovf, 2u);  // Finalize called on DWFA that was never initialized.
            continue;
          }
          const uint64_t ro = A.roff[P.read_begin + r];
          const uint32_t blen = A.rlen[P.read_begin + r];
          uint32_t fe;
          bool ok = wave_finalize_read(tv.wf + (uint64_t)r * wcap, e, tv.off[r], A.rbytes + ro, blen, tv.con, len, wc,
                                       scratch, wcap, fe, cnt);
          if (!ok) {
            if (lane == 0) atomicOr(&ctl.ovf, 4u);
            continue;
          }
          if (lane == 0) L.fe[r] = fe;
          __builtin_amdgcn_wave_barrier();
        }
        flush_counters(ctl, cnt);
        __syncthreads();
        if (tid == 0) {
          ctl.store_idx = -1;
          if (ctl.ovf & 2u) {
            ctl.status = 1;
          } else if (ctl.ovf & 4u) {
            ctl.status = ST_RETRY | ST_RETRY_WCAP;
          } else {
            uint64_t total = 0;
            for (uint32_t r = 0; r < n; ++r) total += cost_of(L.fe[r], cfg.cost_mode);
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
        __syncthreads();
        if (ctl.status != ST_OK) break;
        if (ctl.store_idx >= 0) {
          uint8_t* rec = outp + 16 + (uint64_t)ctl.store_idx * rbytes_sz;
          uint8_t* rcon = rec + 16;
          uint32_t* rfe = (uint32_t*)(rec + 16 + align16(lcap));
          for (uint32_t i = tid; i < len; i += kBlock) rcon[i] = tv.con[i];
          for (uint32_t r = tid; r < n; r += kBlock) rfe[r] = L.fe[r];
          if (tid == 0) {
            uint32_t* h = (uint32_t*)rec;
            h[0] = len;
            h[1] = 0;
            h[2] = 0;
          }
        }
      }

      // ---- VOTES + child selection (consensus.rs:283-321) ----
      if (wave == 0) {
        bool ok = wave_votes(ctl, L.rinfo, n, nullptr, wc);
        if (lane == 0) {
          if (!ok) {
            ctl.status = 11u;
          } else {
            double max_obs = 0.0;
            bool have = false;
            for (uint32_t k = 0; k < ctl.nkeys; ++k) {
              if (!have || ctl.vals[k] >= max_obs) max_obs = ctl.vals[k];
              have = true;
            }
            if (!have) max_obs = (double)cfg.min_count;
            const double thr = fmin((double)cfg.min_count, max_obs);
            uint32_t nc = 0;
            for (uint32_t k = 0; k < ctl.nkeys; ++k)
              if (ctl.vals[k] >= thr) ctl.child_sym[nc++] = ctl.keys[k];
            ctl.nchild = nc;
            if (nc == 0 && len < ctl.max_read_len) {
              // coverage gap: only reachable with activation offsets (max_activate)
            }
          }
        }
      }
      __syncthreads();
      if (ctl.status != ST_OK) break;

      const uint32_t nc = ctl.nchild;
      if (nc == 0) {
        if (tid == 0) L.freestack[ctl.nfree++] = top;
        __syncthreads();
        continue;
      }
      if (len + 1 > lcap) {
        if (tid == 0) ctl.status = ST_RETRY | ST_RETRY_LCAP;
        __syncthreads();
        break;
      }
      // ---- PUSH each child: clone when 2+, in place when 1 ----
      for (uint32_t c = 0; c < nc; ++c) {
        if (tid == 0) {
          uint32_t slot = top;
          if (nc > 1) {
            if (ctl.nfree == 0) {
              ctl.status = ST_RETRY | ST_RETRY_PCAP;
            } else {
              slot = L.freestack[--ctl.nfree];
            }
          }
          ctl.child_slot[c] = slot;
          ctl.cost_acc = 0;
          ctl.ovf = 0;
        }
        __syncthreads();
        if (ctl.status != ST_OK) break;
        const uint32_t slot = ctl.child_slot[c];
        SideView cv = side_view(ws + (uint64_t)slot * sbytes, 0, nmax, wcap, lcap);
        const uint8_t sym = ctl.child_sym[c];
        if (slot != top) {
          // clone: consensus bytes + per-read (e, off, live wavefront)
          for (uint32_t i = tid; i < len; i += kBlock) cv.con[i] = tv.con[i];
          for (uint32_t r = wave; r < n; r += kWaves) {
            const uint32_t e = tv.e[r];
            if (lane == 0) {
              cv.e[r] = e;
              cv.off[r] = tv.off[r];
            }
            if (e == kInactive) continue;
            const uint32_t W = 2 * e + 1;
            for (uint32_t i = lane; i < W; i += 64) cv.wf[(uint64_t)r * wcap + i] = tv.wf[(uint64_t)r * wcap + i];
          }
        }
        if (tid == 0) cv.con[len] = sym;
        __syncthreads();
        WaveCounters cnt = {0, 0, 0, 0, 0};
        uint64_t cost = 0;
        for (uint32_t r = wave; r < n; r += kWaves) {
          uint32_t e = cv.e[r];
          if (e == kInactive) continue;
          const uint64_t ro = A.roff[P.read_begin + r];
          const uint32_t blen = A.rlen[P.read_begin + r];
          bool ok = wave_push_read(cv.wf + (uint64_t)r * wcap, e, cv.off[r], A.rbytes + ro, blen, cv.con, len + 1, sym,
                                   wc, early, wcap, cnt);
          if (!ok) {
            if (lane == 0) atomicOr(&ctl.ovf, 4u);
            continue;
          }
          if (lane == 0) cv.e[r] = e;
          cost += cost_of(e, cfg.cost_mode);
        }
        flush_counters(ctl, cnt);
        if (lane == 0 && cost) atomicAdd((unsigned long long*)&ctl.cost_acc, (unsigned long long)cost);
        __syncthreads();
        if (tid == 0) {
          if (ctl.ovf & 4u) ctl.status = ST_RETRY | ST_RETRY_WCAP;
          ctl.child_cost[c] = ctl.cost_acc;
          L.meta[slot].len[0] = len + 1;
        }
        __syncthreads();
        if (ctl.status != ST_OK) break;
      }
      if (ctl.status != ST_OK) break;
      if (tid == 0) {
        if (nc > 1) L.freestack[ctl.nfree++] = top;
        TrackerRef t{trk_lc, trk_pc, &ctl.trk_total[0], &ctl.trk_thr[0], cfg.max_capacity_per_size};
        for (uint32_t c = 0; c < nc; ++c) {
          t.insert(len + 1);
          if (ctl.heap_n >= pcap) {
            ctl.status = ST_RETRY | ST_RETRY_HEAP;
            break;
          }
          heap_push(L.heap, ctl.heap_n, HeapEntry{ctl.child_cost[c], len + 1, ctl.child_slot[c]});
        }
      }
      __syncthreads();
      if (ctl.status != ST_OK) break;
    }

    // ---- outputs ----
    __syncthreads();
    if (tid == 0) {
      uint32_t* h = (uint32_t*)outp;
      h[0] = min(ctl.n_ret, rmax);
      A.status[prob] = ctl.status;
      for (int s = 0; s < S_NSTAT; ++s) A.stats[(uint64_t)prob * S_NSTAT + s] = ctl.cnt[s];
    }
    __syncthreads();
  }
}

}  // namespace wc

namespace wc {
void launch_single_engine(const EngineArgs& a, uint32_t grid, size_t lds, hipStream_t s) {
  hipLaunchKernelGGL(single_engine_kernel, dim3(grid), dim3(kBlock), lds, s, a);
}
void launch_dual_engine(const EngineArgs& a, uint32_t grid, size_t lds, hipStream_t s) {
  (void)a; (void)grid; (void)lds; (void)s;
}
int engine_blocks_per_cu(uint32_t sides, size_t lds) {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, single_engine_kernel, kBlock, lds) != hipSuccess) nb = 1;
  return nb;
}
}  // namespace wc
