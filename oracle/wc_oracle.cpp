// ORACLE — TEST INFRASTRUCTURE ONLY (see rust_compat.hpp header).
// CPU restatement of waffle_con v0.4.4 (reference @ /root/reference, read-only):
//   DWFALite            src/dynamic_wfa.rs:48-265
//   wfa_ed_config       src/sequence_alignment.rs:36-87
//   PQueueTracker       src/pqueue_tracker.rs:23-144
//   ConsensusDWFA       src/consensus.rs:139-564
//   DualConsensusDWFA   src/dual_consensus.rs:79-150, 240-787, 822-1349
//   PriorityConsensus   src/priority_consensus.rs:129-341
// Rust-crate behaviour (heap ties, hash iteration order) comes from rust_compat.hpp.
#include "wc_oracle.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <unordered_map>

namespace wco {

// ===========================================================================
// DWFALite
// ===========================================================================

// dynamic_wfa.rs:109-153 — extend every diagonal while bytes match; the
// wildcard is honoured on the baseline (read) side only (:138-140).
void Dwfa::extend(Seq b, Seq o, Counters* c) {
  uint64_t cmp = 0;
  for (size_t i = 0; i < wf.size(); ++i) {
    size_t d = wf[i];
    for (;;) {
      size_t bo = d + e - i;
      size_t oo = d + offset;
      if (bo >= b.n || oo >= o.n) break;
      cmp++;
      uint8_t x = b.p[bo];
      if (x != o.p[oo] && (wildcard < 0 || x != (uint8_t)wildcard)) break;
      d++;
    }
    wf[i] = d;
  }
  if (c) c->compares += cmp;
}

// dynamic_wfa.rs:162-191
void Dwfa::increase(Seq b, Seq o, Counters* c) {
  e += 1;
  std::vector<size_t> nw(wf.size() + 2, 0);
  for (size_t i = 0; i < wf.size(); ++i) {
    size_t d = wf[i];
    nw[i] = std::max(nw[i], d);
    nw[i + 1] = std::max(nw[i + 1], d + 1);
    nw[i + 2] = std::max(nw[i + 2], d + 1);
  }
  wf.swap(nw);
  if (c) c->ed_increases++;
  extend(b, o, c);
}

// dynamic_wfa.rs:213-220
size_t Dwfa::max_baseline() const {
  size_t m = 0;
  for (size_t i = 0; i < wf.size(); ++i) m = std::max(m, wf[i] + e - i);
  return m;
}

// dynamic_wfa.rs:224-227
size_t Dwfa::max_other() const { return offset + *std::max_element(wf.begin(), wf.end()); }

// dynamic_wfa.rs:75-99
size_t Dwfa::update(Seq b, Seq o, Counters* c) {
  extend(b, o, c);
  const size_t w_in = wf.size();
  size_t mo = max_other();
  while (mo < o.n && !(early && reached_end(b))) {
    increase(b, o, c);
    mo = max_other();
  }
  if (!(mo == o.n || (early && max_baseline() == b.n)))
    throw Error(E_INVARIANT, "DWFA update invariant violated");
  if (c) {
    c->updates++;
    c->w_out += wf.size();
    // a grown wavefront is read and written whole (u32 entries): the row
    // traffic of the roofline model
    if (wf.size() != w_in) c->row_bytes += 4 * (w_in + wf.size());
  }
  return e;
}

// dynamic_wfa.rs:201-210 (never sets is_finalized)
void Dwfa::finalize(Seq b, Seq o, Counters* c) {
  if (c) c->finalizes++;
  const size_t w_in = wf.size();
  while (max_baseline() < b.n) increase(b, o, c);
  if (c && wf.size() != w_in) c->row_bytes += 4 * w_in;  // read once, grown on a copy
}

// dynamic_wfa.rs:241-255 — tips are diagonals at the consensus end; insertion
// order is ascending diagonal index.
FxByteMap<uint64_t> Dwfa::candidates(Seq b, Seq o) const {
  FxByteMap<uint64_t> m;
  for (size_t i = 0; i < wf.size(); ++i) {
    size_t d = wf[i];
    if (d + offset == o.n) {
      size_t bo = d + e - i;
      if (bo < b.n) m.entry(b.p[bo], 0) += 1;
    }
  }
  return m;
}

// ===========================================================================
// sequence_alignment.rs:36-87
// ===========================================================================
size_t wfa_ed_config(Seq v1, Seq v2, bool require_both_end, int wildcard) {
  typedef std::pair<size_t, size_t> P;
  const size_t l1 = v1.n, l2 = v2.n;
  auto wc_match = [&](uint8_t a) { return wildcard >= 0 && a == (uint8_t)wildcard; };
  std::vector<P> cur(1, P(0, 0));
  std::vector<P> nxt(3, P(0, 0));
  size_t edits = 0;
  for (;;) {
    for (size_t k = 0; k < cur.size(); ++k) {
      size_t i = cur[k].first, j = cur[k].second;
      while (i < l1 && j < l2 && (v1.p[i] == v2.p[j] || wc_match(v1.p[i]) || wc_match(v2.p[j]))) {
        ++i;
        ++j;
      }
      if ((i == l1 || !require_both_end) && j == l2) return edits;
      if (i == l1) {
        nxt[k] = std::max(nxt[k], P(i, j));
        nxt[k + 1] = std::max(nxt[k + 1], P(i, j + 1));
        nxt[k + 2] = std::max(nxt[k + 2], P(i, j + 1));
      } else if (j == l2) {
        nxt[k] = std::max(nxt[k], P(i + 1, j));
        nxt[k + 1] = std::max(nxt[k + 1], P(i + 1, j));
        nxt[k + 2] = std::max(nxt[k + 2], P(i, j));
      } else {
        nxt[k] = std::max(nxt[k], P(i + 1, j));
        nxt[k + 1] = std::max(nxt[k + 1], P(i + 1, j + 1));
        nxt[k + 2] = std::max(nxt[k + 2], P(i, j + 1));
      }
    }
    edits++;
    cur.swap(nxt);
    nxt.assign(3 + 2 * edits, P(0, 0));
  }
}

// ===========================================================================
// pqueue_tracker.rs:10-144
// ===========================================================================
struct Tracker {
  std::vector<uint64_t> length_counts, processed_counts;
  uint64_t total = 0, threshold = 0, cap;
  Tracker(size_t initial, uint64_t capacity) : length_counts(initial, 0), processed_counts(initial, 0), cap(capacity) {}
  void insert(size_t v) {
    if (v >= length_counts.size()) length_counts.resize(v + 1, 0);
    length_counts[v]++;
    if (v >= threshold) total++;
  }
  void remove(size_t v) {
    if (v >= length_counts.size() || length_counts[v] == 0) throw Error(E_INVARIANT, "tracker remove of absent length");
    length_counts[v]--;
    if (v >= threshold) {
      if (total == 0) throw Error(E_INVARIANT, "tracker total underflow");
      total--;
    }
  }
  void increment_threshold() {
    // increase_threshold(threshold + 1)
    if (threshold < length_counts.size()) total -= length_counts[threshold];
    threshold++;
  }
  void process(size_t v) {
    if (v >= processed_counts.size()) processed_counts.resize(v + 1, 0);
    if (processed_counts[v] >= cap) throw Error(E_CAPACITY, "Capacity is full");
    processed_counts[v]++;
  }
  uint64_t processed(size_t v) const { return v >= processed_counts.size() ? 0 : processed_counts[v]; }
  bool at_capacity(size_t v) const { return processed(v) >= cap; }
  uint64_t len() const { return total; }
  uint64_t unfiltered_len() const {
    uint64_t s = 0;
    for (auto x : length_counts) s += x;
    return s;
  }
};

static inline uint64_t cost_of(size_t e, int mode) { return mode == 0 ? (uint64_t)e : (uint64_t)e * (uint64_t)e; }

// consensus.rs:151-181 / dual_consensus.rs:254-284
static std::vector<int64_t> shift_offsets(const Config& cfg, const std::vector<int64_t>& offs) {
  if (!cfg.auto_shift_offsets) return offs;
  int64_t mn = INT64_MAX;
  bool start = false;
  for (auto o : offs) {
    if (o < 0) start = true;
    else mn = std::min(mn, o);
  }
  if (start) return offs;
  std::vector<int64_t> r;
  for (auto o : offs) r.push_back(o == mn ? -1 : o - mn);
  return r;
}

// consensus.rs:413-448 / dual_consensus.rs:877-903 — pick the best start offset
// inside the window by semi-global ED of the read prefix, then a full update.
static Dwfa activate_one(const std::vector<uint8_t>& con, Seq seq, const Config& cfg, Counters* c) {
  const size_t con_len = con.size();
  const size_t ocl = std::min<size_t>(cfg.offset_compare_length, seq.n);
  auto sat = [](size_t a, size_t b) { return a > b ? a - b : 0; };
  const size_t start = sat(con_len, cfg.offset_window + ocl);
  const size_t end = sat(con_len, ocl);
  size_t best = sat(con_len, ocl + cfg.offset_window / 2);
  Seq prefix{seq.p, ocl};
  size_t min_ed = wfa_ed_config(Seq{con.data() + best, con_len - best}, prefix, false, cfg.wildcard);
  for (size_t p = start; p < end; ++p) {
    size_t ed = wfa_ed_config(Seq{con.data() + p, con_len - p}, prefix, false, cfg.wildcard);
    if (ed < min_ed) {
      min_ed = ed;
      best = p;
    }
  }
  Dwfa d;
  d.wildcard = cfg.wildcard;
  d.early = cfg.allow_early_termination;
  d.offset = best;
  d.update(seq, Seq{con.data(), con_len}, c);
  return d;
}

// ===========================================================================
// ConsensusDWFA (consensus.rs)
// ===========================================================================
namespace {
struct SNode {
  std::vector<uint8_t> con;
  std::vector<Dwfa> dw;
  std::vector<uint8_t> act;  // Option<DWFALite>::is_some
};

// consensus.rs:455-463
void snode_push(SNode& n, const std::vector<Seq>& seqs, uint8_t sym, Counters* c) {
  n.con.push_back(sym);
  Seq o{n.con.data(), n.con.size()};
  for (size_t r = 0; r < seqs.size(); ++r)
    if (n.act[r]) n.dw[r].update(seqs[r], o, c);
}

// consensus.rs:480-499
uint64_t snode_total(const SNode& n, int mode) {
  uint64_t t = 0;
  for (size_t r = 0; r < n.dw.size(); ++r)
    if (n.act[r]) t += cost_of(n.dw[r].e, mode);
  return t;
}

// consensus.rs:540-564 — outer map keyed by symbol, reads in index order,
// per-read inner map in its own iteration order; f64 sums in that order.
FxByteMap<double> snode_candidates(const SNode& n, const std::vector<Seq>& seqs, int wildcard) {
  FxByteMap<double> cand;
  Seq o{n.con.data(), n.con.size()};
  for (size_t r = 0; r < seqs.size(); ++r) {
    if (!n.act[r]) continue;
    FxByteMap<uint64_t> m = n.dw[r].candidates(seqs[r], o);
    uint64_t split_i = 0;
    m.for_each([&](uint8_t, uint64_t v) { split_i += v; });
    double split = (double)split_i;
    m.for_each([&](uint8_t k, uint64_t occ) { cand.entry(k, 0.0) += (double)occ / split; });
  }
  if (wildcard >= 0 && cand.size() > 1) cand.remove((uint8_t)wildcard);
  return cand;
}
}  // namespace

// consensus.rs:139-351
std::vector<ConsensusOut> consensus_single(const Config& cfg, const std::vector<Seq>& seqs,
                                           const std::vector<int64_t>& offsets_in, Counters* c) {
  if (seqs.empty()) throw Error(E_BAD_INPUT, "No sequences provided");
  const int mode = cfg.consensus_cost;
  uint64_t maximum_error = UINT64_MAX;
  uint64_t farthest = 0, last_constraint = 0;

  std::vector<int64_t> offsets = shift_offsets(cfg, offsets_in);
  std::map<size_t, std::vector<size_t>> activate_points;
  size_t max_activate = 0, initially_active = 0;
  for (size_t i = 0; i < offsets.size(); ++i) {
    if (offsets[i] >= 0) {
      size_t al = (size_t)offsets[i] + cfg.offset_compare_length;
      activate_points[al].push_back(i);
      max_activate = std::max(max_activate, al);
    } else {
      initially_active++;
    }
  }
  if (initially_active == 0) throw Error(E_NO_START, "Must have at least one initial offset of None to see the consensus.");

  size_t initial_size = 0;
  for (auto& s : seqs) initial_size = std::max(initial_size, s.n);
  Tracker tracker(initial_size, cfg.max_capacity_per_size);

  std::vector<SNode> pool;
  std::vector<int> free_ids;
  auto alloc = [&]() -> int {
    if (!free_ids.empty()) {
      int id = free_ids.back();
      free_ids.pop_back();
      return id;
    }
    pool.emplace_back();
    return (int)pool.size() - 1;
  };

  int root = alloc();
  {
    SNode& n = pool[root];
    n.con.clear();
    n.dw.assign(seqs.size(), Dwfa());
    n.act.assign(seqs.size(), 0);
    for (size_t r = 0; r < seqs.size(); ++r) {
      n.dw[r].wildcard = cfg.wildcard;
      n.dw[r].early = cfg.allow_early_termination;
      n.act[r] = offsets[r] < 0;
    }
  }
  PQHeap pq;
  tracker.insert(0);
  pq.push(root, Prio{snode_total(pool[root], mode), 0});

  std::vector<ConsensusOut> ret;
  while (!pq.empty()) {
    if (c) {
      c->peak_queue_size = std::max<uint64_t>(c->peak_queue_size, pq.size());
      c->pops++;
    }
    while ((tracker.len() > cfg.max_queue_size || last_constraint >= cfg.max_nodes_wo_constraint) &&
           tracker.threshold < farthest) {
      tracker.increment_threshold();
      last_constraint = 0;
    }
    PQHeap::Entry top = pq.pop();
    const size_t top_len = pool[top.id].con.size();
    tracker.remove(top_len);
    if (top.p.cost > maximum_error || top.p.len < tracker.threshold || tracker.at_capacity(top_len)) {
      if (c) c->nodes_ignored++;
      free_ids.push_back(top.id);
      continue;
    }
    farthest = std::max<uint64_t>(farthest, top_len);
    if (c) c->nodes_explored++;
    last_constraint++;
    tracker.process(top_len);

    // consensus.rs:254-279 reached_end (:516-532) → finalize a clone
    {
      const SNode& n = pool[top.id];
      Seq o{n.con.data(), n.con.size()};
      bool any = false, all = true;
      for (size_t r = 0; r < seqs.size(); ++r) {
        bool at = n.act[r] && n.dw[r].reached_end(seqs[r]);
        any |= at;
        all &= at;
      }
      bool reached = cfg.allow_early_termination ? all : any;
      if (reached) {
        std::vector<uint64_t> costs(seqs.size(), 0);
        uint64_t total = 0;
        for (size_t r = 0; r < seqs.size(); ++r) {
          if (!n.act[r]) throw Error(E_FINALIZE_UNINIT, "Finalize called on DWFA that was never initialized.");
          Dwfa f = n.dw[r];
          f.finalize(seqs[r], o, c);
          costs[r] = cost_of(f.e, mode);
          total += costs[r];
        }
        if (total < maximum_error) {
          maximum_error = total;
          ret.clear();
        }
        if (total <= maximum_error && ret.size() < cfg.max_return_size) ret.push_back(ConsensusOut{n.con, costs});
      }
    }

    // consensus.rs:283-321
    FxByteMap<double> cand = snode_candidates(pool[top.id], seqs, cfg.wildcard);
    double max_obs = 0.0;
    bool have = false;
    cand.for_each([&](uint8_t, double v) {
      if (!have || v >= max_obs) max_obs = v;  // max_by(total_cmp): last max wins, value identical
      have = true;
    });
    if (!have) max_obs = (double)cfg.min_count;
    double thr = std::min((double)cfg.min_count, max_obs);
    std::vector<uint8_t> passing;
    cand.for_each([&](uint8_t k, double v) {
      if (v >= thr) passing.push_back(k);
    });

    std::vector<int> new_nodes;
    if (passing.empty()) {
      if (top_len < max_activate)
        throw Error(E_COVERAGE_GAP, "Encountered coverage gap: consensus is length " + std::to_string(top_len) +
                                        " with no candidates, but sequences activate at " + std::to_string(max_activate));
      free_ids.push_back(top.id);
    } else if (passing.size() == 1) {
      snode_push(pool[top.id], seqs, passing[0], c);
      new_nodes.push_back(top.id);
    } else {
      for (uint8_t sym : passing) {
        int id = alloc();
        pool[id] = pool[top.id];
        snode_push(pool[id], seqs, sym, c);
        new_nodes.push_back(id);
      }
      free_ids.push_back(top.id);
    }

    for (int id : new_nodes) {
      SNode& n = pool[id];
      auto it = activate_points.find(n.con.size());
      if (it != activate_points.end()) {
        for (size_t si : it->second) {
          if (n.act[si]) throw Error(E_INVARIANT, "activation of an active sequence");
          n.dw[si] = activate_one(n.con, seqs[si], cfg, c);
          n.act[si] = 1;
        }
      }
      Prio p{snode_total(n, mode), n.con.size()};
      tracker.insert(n.con.size());
      pq.push(id, p);
    }
  }
  if (tracker.len() != 0) throw Error(E_INVARIANT, "tracker not drained");
  std::stable_sort(ret.begin(), ret.end(),
                   [](const ConsensusOut& a, const ConsensusOut& b) { return a.sequence < b.sequence; });
  return ret;
}

// ===========================================================================
// DualConsensusDWFA (dual_consensus.rs)
// ===========================================================================
namespace {
struct DNode {
  bool is_dual = false, lock1 = false, lock2 = false;
  std::vector<uint8_t> con1, con2;
  std::vector<Dwfa> dw1, dw2;
  std::vector<uint8_t> a1, a2;
  size_t max_len() const { return std::max(con1.size(), con2.size()); }
};

// dual_consensus.rs:915-946
void dnode_push(DNode& n, const std::vector<Seq>& seqs, uint8_t sym, bool side1, Counters* c) {
  if (side1 && n.lock1) throw Error(E_LOCKED, "Consensus 1 is locked, cannot modify");
  if (!side1 && n.lock2) throw Error(E_LOCKED, "Consensus 2 is locked, cannot modify");
  std::vector<uint8_t>& con = side1 ? n.con1 : n.con2;
  std::vector<Dwfa>& dw = side1 ? n.dw1 : n.dw2;
  std::vector<uint8_t>& a = side1 ? n.a1 : n.a2;
  con.push_back(sym);
  Seq o{con.data(), con.size()};
  for (size_t r = 0; r < seqs.size(); ++r)
    if (a[r]) dw[r].update(seqs[r], o, c);
}

// dual_consensus.rs:957-976
void dnode_activate_dual(DNode& n, const std::vector<Seq>& seqs, uint8_t s1, uint8_t s2, Counters* c) {
  if (n.is_dual) throw Error(E_DUAL_TWICE, "Cannot activate dual on a dual node");
  n.is_dual = true;
  if (s1 == s2) throw Error(E_SAME_SYMBOL, "Cannot activate dual mode with the same extension symbols");
  n.con2 = n.con1;
  n.dw2 = n.dw1;
  n.a2 = n.a1;
  dnode_push(n, seqs, s1, true, c);
  dnode_push(n, seqs, s2, false, c);
}

// dual_consensus.rs:981-991
bool dnode_imbalanced(const DNode& n, uint64_t min_count) {
  if (!n.is_dual) return false;
  uint64_t c1 = 0, c2 = 0;
  for (auto x : n.a1) c1 += x;
  for (auto x : n.a2) c2 += x;
  return c1 < min_count || c2 < min_count;
}

// dual_consensus.rs:1030-1045
void dnode_prune(DNode& n, uint64_t delta) {
  if (!n.is_dual) return;
  for (size_t r = 0; r < n.a1.size(); ++r) {
    if (n.a1[r] && n.a2[r]) {
      size_t e1 = n.dw1[r].e, e2 = n.dw2[r].e;
      if (e1 + delta < e2) n.a2[r] = 0;
      else if (e2 + delta < e1) n.a1[r] = 0;
    }
  }
}

// dual_consensus.rs:1092-1131 — per read min over sides, strict < (ties → side 1)
void dnode_costs(const DNode& n, int mode, std::vector<size_t>& idx, std::vector<uint64_t>& score) {
  const size_t N = n.a1.size();
  idx.assign(N, SIZE_MAX);
  score.assign(N, UINT64_MAX);
  for (int side = 0; side < 2; ++side) {
    const std::vector<Dwfa>& dw = side == 0 ? n.dw1 : n.dw2;
    const std::vector<uint8_t>& a = side == 0 ? n.a1 : n.a2;
    for (size_t r = 0; r < N; ++r) {
      if (!a[r]) continue;
      uint64_t s = cost_of(dw[r].e, mode);
      if (s < score[r]) {
        score[r] = s;
        idx[r] = (size_t)side;
      }
    }
  }
  for (size_t r = 0; r < N; ++r)
    if (idx[r] == SIZE_MAX && score[r] == UINT64_MAX) score[r] = 0;
}

uint64_t dnode_total(const DNode& n, int mode) {
  std::vector<size_t> idx;
  std::vector<uint64_t> sc;
  dnode_costs(n, mode, idx, sc);
  uint64_t t = 0;
  for (auto s : sc) t += s;
  return t;
}

// dual_consensus.rs:1174-1195
bool dnode_reached_all_end(const DNode& n, const std::vector<Seq>& seqs, bool require_all) {
  bool any = false, all = true;
  for (size_t r = 0; r < seqs.size(); ++r) {
    bool p1 = n.a1[r] && n.dw1[r].reached_end(seqs[r]);
    bool p2 = n.a2[r] && n.dw2[r].reached_end(seqs[r]);
    bool v = p1 || p2;
    any |= v;
    all &= v;
  }
  return require_all ? all : any;
}

// dual_consensus.rs:1203-1233
bool dnode_reached_con_end(const DNode& n, const std::vector<Seq>& seqs, bool side1, bool require_all) {
  if (!side1 && !n.is_dual) return false;
  const std::vector<Dwfa>& dw = side1 ? n.dw1 : n.dw2;
  const std::vector<uint8_t>& a = side1 ? n.a1 : n.a2;
  bool any = false, all = true;
  for (size_t r = 0; r < seqs.size(); ++r) {
    bool v = a[r] ? dw[r].reached_end(seqs[r]) : require_all;
    any |= v;
    all &= v;
  }
  return require_all ? all : any;
}

// dual_consensus.rs:1299-1336
std::vector<double> dnode_ed_weights(const DNode& n, bool side1, bool weight_by_ed) {
  const size_t N = n.a1.size();
  if (!n.is_dual) return std::vector<double>(N, 1.0);
  std::vector<double> w(N, 0.0);
  for (size_t r = 0; r < N; ++r) {
    bool h1 = n.a1[r], h2 = n.a2[r];
    double v1 = h1 ? std::max((double)n.dw1[r].e, 0.5) : 0.0;
    double v2 = h2 ? std::max((double)n.dw2[r].e, 0.5) : 0.0;
    if (h1 && h2) {
      if (weight_by_ed) {
        double numer = side1 ? v2 : v1;
        w[r] = numer / (v1 + v2);
      } else if (v1 == v2) {
        w[r] = 0.5;
      } else if ((side1 && v1 < v2) || (!side1 && v2 < v1)) {
        w[r] = 1.0;
      } else {
        w[r] = 0.0;
      }
    } else if ((h1 && side1) || (h2 && !side1)) {
      w[r] = 1.0;
    } else {
      w[r] = 0.0;
    }
  }
  return w;
}

// dual_consensus.rs:1242-1290
FxByteMap<double> dnode_candidates(const DNode& n, const std::vector<Seq>& seqs, int wildcard, bool side1,
                                   bool weighted) {
  const std::vector<Dwfa>& dw = side1 ? n.dw1 : n.dw2;
  const std::vector<uint8_t>& a = side1 ? n.a1 : n.a2;
  const std::vector<uint8_t>& con = side1 ? n.con1 : n.con2;
  std::vector<double> w = weighted ? dnode_ed_weights(n, side1, true) : std::vector<double>(seqs.size(), 1.0);
  FxByteMap<double> cand;
  Seq o{con.data(), con.size()};
  for (size_t r = 0; r < seqs.size(); ++r) {
    if (!(w[r] > 0.0)) continue;
    if (!a[r]) continue;
    FxByteMap<uint64_t> m = dw[r].candidates(seqs[r], o);
    uint64_t split_i = 0;
    m.for_each([&](uint8_t, uint64_t v) { split_i += v; });
    double split = (double)split_i;
    m.for_each([&](uint8_t k, uint64_t occ) { cand.entry(k, 0.0) += w[r] * (double)occ / split; });
  }
  if (wildcard >= 0 && cand.size() > 1) cand.remove((uint8_t)wildcard);
  return cand;
}

// dual_consensus.rs:102-150
DualOut dual_from_node(const DNode& n, int mode) {
  std::vector<size_t> idx;
  std::vector<uint64_t> sc;
  dnode_costs(n, mode, idx, sc);
  bool swap = n.is_dual && (n.con2 < n.con1);
  DualOut out;
  std::vector<uint64_t> scores[2];
  for (size_t r = 0; r < idx.size(); ++r) {
    if (idx[r] > 1) throw Error(E_INVARIANT, "read without a tracked consensus in a result");
    out.is_c1.push_back((uint8_t)((idx[r] == 0) ^ swap));
    scores[idx[r]].push_back(sc[r]);
  }
  ConsensusOut c1{n.con1, scores[0]};
  ConsensusOut c2{n.con2, scores[1]};
  if (swap) {
    out.c1 = c2;
    out.has_c2 = true;
    out.c2 = c1;
  } else {
    out.c1 = c1;
    out.has_c2 = n.is_dual;
    if (n.is_dual) out.c2 = c2;
  }
  std::vector<int64_t> s1, s2;
  for (size_t r = 0; r < n.a1.size(); ++r) {
    s1.push_back(n.a1[r] ? (int64_t)cost_of(n.dw1[r].e, mode) : -1);
    s2.push_back(n.a2[r] ? (int64_t)cost_of(n.dw2[r].e, mode) : -1);
  }
  out.scores1 = swap ? s2 : s1;
  out.scores2 = swap ? s1 : s2;
  return out;
}

uint64_t ceil_u64(double x) {
  double c = std::ceil(x);
  if (!(c > 0.0)) return 0;  // Rust `as u64` saturates negatives/NaN to 0
  if (c >= 18446744073709551615.0) return UINT64_MAX;
  return (uint64_t)c;
}
}  // namespace

// dual_consensus.rs:240-787
std::vector<DualOut> consensus_dual(const Config& cfg, const std::vector<Seq>& seqs,
                                    const std::vector<int64_t>& offsets_in, Counters* c) {
  if (seqs.empty()) throw Error(E_BAD_INPUT, "No sequences provided");
  const int mode = cfg.consensus_cost;
  const bool early = cfg.allow_early_termination;
  uint64_t maximum_error = UINT64_MAX;
  uint64_t far_single = 0, far_dual = 0, single_lc = 0, dual_lc = 0;

  std::vector<int64_t> offsets = shift_offsets(cfg, offsets_in);
  std::map<size_t, std::vector<size_t>> activate_points;
  size_t initially_active = 0;
  for (size_t i = 0; i < offsets.size(); ++i) {
    if (offsets[i] >= 0) activate_points[(size_t)offsets[i] + cfg.offset_compare_length].push_back(i);
    else initially_active++;
  }
  if (initially_active == 0) throw Error(E_NO_START, "Must have at least one initial offset of None to see the consensus.");

  size_t initial_size = 0;
  for (auto& s : seqs) initial_size = std::max(initial_size, s.n);
  Tracker st(initial_size, cfg.max_capacity_per_size), dt(initial_size, cfg.max_capacity_per_size);

  std::vector<DNode> pool;
  std::vector<int> free_ids;
  auto alloc = [&]() -> int {
    if (!free_ids.empty()) {
      int id = free_ids.back();
      free_ids.pop_back();
      return id;
    }
    pool.emplace_back();
    return (int)pool.size() - 1;
  };
  const size_t N = seqs.size();
  auto make_root = [&](const std::vector<int64_t>& offs) {
    DNode n;
    n.dw1.assign(N, Dwfa());
    n.dw2.assign(N, Dwfa());
    n.a1.assign(N, 0);
    n.a2.assign(N, 0);
    for (size_t r = 0; r < N; ++r) {
      n.dw1[r].wildcard = n.dw2[r].wildcard = cfg.wildcard;
      n.dw1[r].early = n.dw2[r].early = early;
      n.a1[r] = offs[r] < 0;
    }
    return n;
  };

  int root = alloc();
  pool[root] = make_root(offsets);
  PQHeap pq;
  // debug trace of pops (ORC_TRACE=<file>), same record shape as the device trace
  FILE* trace = getenv("ORC_TRACE") ? fopen(getenv("ORC_TRACE"), "w") : nullptr;
  struct TraceCloser {
    FILE*& f;
    ~TraceCloser() {
      if (f) fclose(f);
    }
  } trace_closer{trace};
  st.insert(0);
  pq.push(root, Prio{dnode_total(pool[root], mode), 0});

  std::vector<DualOut> ret;
  const uint64_t full_min_count = std::max<uint64_t>(cfg.min_count, ceil_u64(cfg.min_af * (double)N));
  std::vector<uint64_t> total_active{initially_active};
  std::vector<uint64_t> active_min{std::max<uint64_t>(cfg.min_count, ceil_u64(cfg.min_af * (double)initially_active))};

  auto activate_node = [&](DNode& n) {
    auto it = activate_points.find(n.max_len());
    if (it == activate_points.end()) return;
    for (size_t si : it->second) {
      // dual_consensus.rs:866-906: con1 always, con2 as well when dual
      if (n.a1[si]) throw Error(E_INVARIANT, "activation of an active sequence");
      n.dw1[si] = activate_one(n.con1, seqs[si], cfg, c);
      n.a1[si] = 1;
      if (n.is_dual) {
        if (n.a2[si]) throw Error(E_INVARIANT, "activation of an active sequence");
        n.dw2[si] = activate_one(n.con2, seqs[si], cfg, c);
        n.a2[si] = 1;
      }
    }
  };

  while (!pq.empty()) {
    if (c) {
      c->peak_queue_size = std::max<uint64_t>(c->peak_queue_size, pq.size());
      c->pops++;
    }
    while ((st.len() > cfg.max_queue_size || single_lc >= cfg.max_nodes_wo_constraint) && st.threshold < far_single) {
      st.increment_threshold();
      single_lc = 0;
    }
    while ((dt.len() > cfg.max_queue_size || dual_lc >= cfg.max_nodes_wo_constraint) && dt.threshold < far_dual) {
      dt.increment_threshold();
      dual_lc = 0;
    }
    PQHeap::Entry top = pq.pop();
    const int tid = top.id;
    const size_t top_len = pool[tid].max_len();
    uint64_t thr_cut;
    bool at_cap;
    if (pool[tid].is_dual) {
      dt.remove(top_len);
      thr_cut = dt.threshold;
      at_cap = dt.at_capacity(top_len);
    } else {
      st.remove(top_len);
      thr_cut = st.threshold;
      at_cap = st.at_capacity(top_len);
    }
    if (top_len >= active_min.size()) throw Error(E_INVARIANT, "active_min_count index out of range");
    const bool ignore =
        top.p.cost > maximum_error || top_len < thr_cut || at_cap || dnode_imbalanced(pool[tid], active_min[top_len]);
    if (trace) {
      uint64_t s1 = 0, s2 = 0;
      for (auto x : pool[tid].a1) s1 += x;
      for (auto x : pool[tid].a2) s2 += x;
      fprintf(trace, "%u %u %u %u\n", (unsigned)top.p.cost, (unsigned)top_len,
              (unsigned)(pool[tid].is_dual | ((ignore ? 1 : 0) << 1) | (s1 << 8) | (s2 << 20)),
              (unsigned)active_min[top_len]);
    }
    if (ignore) {
      if (c) c->nodes_ignored++;
      free_ids.push_back(tid);
      continue;
    }
    if (pool[tid].is_dual) {
      far_dual = std::max<uint64_t>(far_dual, top_len);
      dual_lc++;
      dt.process(top_len);
    } else {
      far_single = std::max<uint64_t>(far_single, top_len);
      single_lc++;
      st.process(top_len);
    }
    if (c) c->nodes_explored++;

    // :438-492 finalize a clone
    if (dnode_reached_all_end(pool[tid], seqs, early)) {
      DNode f = pool[tid];
      for (size_t r = 0; r < N; ++r) {
        bool done = false;
        if (f.a1[r]) {
          f.dw1[r].finalize(seqs[r], Seq{f.con1.data(), f.con1.size()}, c);
          done = true;
        }
        if (f.is_dual && f.a2[r]) {
          f.dw2[r].finalize(seqs[r], Seq{f.con2.data(), f.con2.size()}, c);
          done = true;
        }
        if (!done) throw Error(E_FINALIZE_UNINIT, "Finalize called on DWFA that was never initialized.");
      }
      f.lock1 = f.lock2 = true;
      bool imbalanced = false;
      if (f.is_dual) {
        std::vector<size_t> idx;
        std::vector<uint64_t> sc;
        dnode_costs(f, mode, idx, sc);
        uint64_t c1 = 0;
        for (auto i : idx) c1 += (i == 0);
        uint64_t c2 = idx.size() - c1;
        imbalanced = c1 < full_min_count || c2 < full_min_count;
      }
      if (!imbalanced) {
        uint64_t fs = dnode_total(f, mode);
        if (fs < maximum_error) {
          maximum_error = fs;
          ret.clear();
        }
        if (fs <= maximum_error && ret.size() < cfg.max_return_size) ret.push_back(dual_from_node(f, mode));
      }
    }

    // :497-513
    if (active_min.size() == top_len + 1) {
      auto it = activate_points.find(top_len);
      uint64_t nt = total_active[top_len] + (it == activate_points.end() ? 0 : it->second.size());
      total_active.push_back(nt);
      active_min.push_back(std::max<uint64_t>(cfg.min_count, ceil_u64(cfg.min_af * (double)nt)));
    }

    const DNode& tn = pool[tid];
    FxByteMap<double> ec1 = dnode_candidates(tn, seqs, cfg.wildcard, true, cfg.weighted_by_ed);
    double sum1 = -0.0;
    ec1.for_each([&](uint8_t, double v) { sum1 += v; });
    uint64_t min_count1 = std::max<uint64_t>(cfg.min_count, ceil_u64(cfg.min_af * sum1));
    double max1 = 0.0;
    bool have1 = false;
    ec1.for_each([&](uint8_t, double v) {
      if (!have1 || v >= max1) max1 = v;
      have1 = true;
    });
    if (!have1) max1 = (double)min_count1;
    double thr1 = std::min((double)min_count1, max1);

    std::vector<int> children;
    if (tn.is_dual) {
      FxByteMap<double> ec2 = dnode_candidates(tn, seqs, cfg.wildcard, false, cfg.weighted_by_ed);
      double sum2 = -0.0;
      ec2.for_each([&](uint8_t, double v) { sum2 += v; });
      uint64_t min_count2 = std::max<uint64_t>(cfg.min_count, ceil_u64(cfg.min_af * sum2));
      double max2 = 0.0;
      bool have2 = false;
      ec2.for_each([&](uint8_t, double v) {
        if (!have2 || v >= max2) max2 = v;
        have2 = true;
      });
      if (!have2) max2 = (double)min_count2;
      double thr2 = std::min((double)min_count2, max2);
      bool fin1 = dnode_reached_con_end(tn, seqs, true, early);
      bool fin2 = dnode_reached_con_end(tn, seqs, false, early);
      // :554-601 — None first, then passing symbols in iteration order
      std::vector<int> o1, o2;
      if (fin1 || ec1.empty() || tn.lock1) o1.push_back(-1);
      if (!tn.lock1) ec1.for_each([&](uint8_t k, double v) {
        if (!(v < thr1)) o1.push_back(k);
      });
      if (fin2 || ec2.empty() || tn.lock2) o2.push_back(-1);
      if (!tn.lock2) ec2.for_each([&](uint8_t k, double v) {
        if (!(v < thr2)) o2.push_back(k);
      });
      if (o1.empty() || o2.empty()) throw Error(E_INVARIANT, "empty dual option list");
      for (int x1 : o1) {
        for (int x2 : o2) {
          if (x1 < 0 && x2 < 0) continue;
          int id = alloc();
          pool[id] = pool[tid];
          DNode& n = pool[id];
          if (x1 >= 0) dnode_push(n, seqs, (uint8_t)x1, true, c);
          else n.lock1 = true;
          if (x2 >= 0) dnode_push(n, seqs, (uint8_t)x2, false, c);
          else n.lock2 = true;
          activate_node(n);
          dnode_prune(n, cfg.dual_max_ed_delta);
          Prio p{dnode_total(n, mode), n.max_len()};
          dt.insert(n.max_len());
          pq.push(id, p);
        }
      }
    } else {
      // :655-679 stay-single children
      std::vector<std::pair<uint8_t, double>> items;
      ec1.for_each([&](uint8_t k, double v) { items.push_back({k, v}); });
      for (auto& kv : items) {
        if (kv.second < thr1) continue;
        int id = alloc();
        pool[id] = pool[tid];
        DNode& n = pool[id];
        dnode_push(n, seqs, kv.first, true, c);
        activate_node(n);
        Prio p{dnode_total(n, mode), n.max_len()};
        st.insert(n.max_len());
        pq.push(id, p);
      }
      // :682-734 split children from every ordered pair of sorted candidates
      int num_passing = 0;
      std::vector<std::pair<double, uint8_t>> sc;
      for (auto& kv : items) {
        if (cfg.wildcard >= 0 && kv.first == (uint8_t)cfg.wildcard) continue;
        if (kv.second >= (double)min_count1) num_passing++;
        sc.push_back({kv.second, kv.first});
      }
      std::stable_sort(sc.begin(), sc.end(), [](const std::pair<double, uint8_t>& a, const std::pair<double, uint8_t>& b) {
        if (a.first != b.first) return a.first > b.first;  // Reverse(count)
        return a.second < b.second;
      });
      if (num_passing > 1) {
        for (size_t i = 0; i < sc.size(); ++i) {
          for (size_t j = i + 1; j < sc.size(); ++j) {
            int id = alloc();
            pool[id] = pool[tid];
            DNode& n = pool[id];
            dnode_activate_dual(n, seqs, sc[i].second, sc[j].second, c);
            activate_node(n);
            dnode_prune(n, cfg.dual_max_ed_delta);
            Prio p{dnode_total(n, mode), n.max_len()};
            dt.insert(n.max_len());
            pq.push(id, p);
          }
        }
      }
    }
    free_ids.push_back(tid);
    if (pq.size() != st.unfiltered_len() + dt.unfiltered_len()) throw Error(E_INVARIANT, "queue/tracker mismatch");
  }
  if (st.len() != 0 || dt.len() != 0) throw Error(E_INVARIANT, "tracker not drained");

  if (ret.size() > 1) {
    std::stable_sort(ret.begin(), ret.end(), [](const DualOut& a, const DualOut& b) {
      static const std::vector<uint8_t> empty;
      const std::vector<uint8_t>& a2 = a.has_c2 ? a.c2.sequence : empty;
      const std::vector<uint8_t>& b2 = b.has_c2 ? b.c2.sequence : empty;
      if (a.c1.sequence != b.c1.sequence) return a.c1.sequence < b.c1.sequence;
      return a2 < b2;
    });
  }
  if (ret.empty()) {
    // :772-779 fallback: root with every read active, empty consensus
    std::vector<int64_t> none(N, -1);
    DNode r = make_root(none);
    ret.push_back(dual_from_node(r, mode));
  }
  return ret;
}

// ===========================================================================
// PriorityConsensusDWFA (priority_consensus.rs:172-341)
// ===========================================================================
// FxHashSet<Option<usize>> iteration order (priority_consensus.rs:180): hash of
// Option<usize> = derive(Hash): discriminant (as isize) then payload.
static uint64_t fx_add(uint64_t h, uint64_t w) { return (((h << 5) | (h >> 59)) ^ w) * kFxSeed; }
static uint64_t fx_hash_opt(int64_t v) {
  if (v < 0) return fx_add(0, 0);
  return fx_add(fx_add(0, 1), (uint64_t)v);
}

std::vector<int64_t> seed_group_order(const std::vector<int64_t>& groups) {
  // PARITY UNPINNED: no reference fixture observes this order. It restates
  // hashbrown on x86_64 with SSE2 (probe group width 16; NEON/generic builds
  // of the reference use 8 and would iterate differently).
  // hashbrown table of Option<usize> keys (16-B entries): same placement rules as
  // FxByteMap but with a 64-bit hash
  // built by `.collect()` (priority_consensus.rs:180): hashbrown's extend
  // reserves the iterator's exact size hint (n_chains) up front, so the table
  // starts at capacity_to_buckets(n_chains) buckets
  std::vector<int64_t> keys;
  std::vector<int64_t> table(fx_buckets_for(std::max<size_t>(groups.size(), 1)), -1);  // slot -> key index
  std::vector<uint64_t> hashes;
  size_t items = 0, growth_left = fx_capacity(table.size());
  auto insert_slot = [&](uint64_t h) -> size_t {
    size_t B = table.size(), mask = B - 1, pos = (size_t)h & mask;
    if (B < 16) {
      for (size_t i = pos; i < B; ++i)
        if (table[i] < 0) return i;
      for (size_t i = 0; i < B; ++i)
        if (table[i] < 0) return i;
      return SIZE_MAX;
    }
    size_t stride = 0;
    for (;;) {
      for (size_t j = 0; j < 16; ++j)
        if (table[(pos + j) & mask] < 0) return (pos + j) & mask;
      stride += 16;
      pos = (pos + stride) & mask;
    }
  };
  for (int64_t g : groups) {
    bool found = false;
    for (auto k : keys)
      if (k == g) found = true;
    if (found) continue;
    uint64_t h = fx_hash_opt(g);
    if (growth_left == 0) {
      size_t want = std::max(items + 1, fx_capacity(table.size()) + 1);
      size_t nb = fx_buckets_for(want);
      std::vector<int64_t> old = table;
      table.assign(nb, -1);
      for (size_t i = 0; i < old.size(); ++i)
        if (old[i] >= 0) table[insert_slot(hashes[old[i]])] = old[i];
      growth_left = fx_capacity(nb) - items;
    }
    keys.push_back(g);
    hashes.push_back(h);
    table[insert_slot(h)] = (int64_t)keys.size() - 1;
    items++;
    growth_left--;
  }
  std::vector<int64_t> order;
  for (auto s : table)
    if (s >= 0) order.push_back(keys[s]);
  return order;
}

PriorityOut consensus_priority(const Config& cfg, const std::vector<std::vector<Seq>>& chains,
                               const std::vector<std::vector<int64_t>>& offsets,
                               const std::vector<int64_t>& seed_groups, Counters* c) {
  if (chains.empty()) throw Error(E_BAD_INPUT, "No sequence chains provided");
  const size_t max_level = chains[0].size();
  const size_t M = chains.size();
  struct Work {
    std::vector<uint8_t> inc;
    size_t level;
    std::vector<ConsensusOut> chain;
  };
  std::vector<Work> stack;
  for (int64_t g : seed_group_order(seed_groups)) {
    Work w;
    w.inc.resize(M);
    for (size_t i = 0; i < M; ++i) w.inc[i] = seed_groups[i] == g;
    w.level = 0;
    stack.push_back(w);
  }
  std::vector<std::vector<ConsensusOut>> cons;
  std::vector<std::vector<uint8_t>> assigns;
  while (!stack.empty()) {
    Work w = std::move(stack.back());
    stack.pop_back();
    std::vector<Seq> seqs;
    std::vector<int64_t> offs;
    for (size_t i = 0; i < M; ++i) {
      if (!w.inc[i]) continue;
      seqs.push_back(chains[i][w.level]);
      offs.push_back(offsets[i][w.level]);
    }
    std::vector<DualOut> res = consensus_dual(cfg, seqs, offs, c);
    const DualOut& ch = res[0];
    if (ch.has_c2) {
      std::vector<uint8_t> as1(M, 0), as2(M, 0);
      size_t k = 0;
      for (size_t i = 0; i < M; ++i) {
        if (!w.inc[i]) continue;
        if (ch.is_c1[k]) as1[i] = 1;
        else as2[i] = 1;
        k++;
      }
      if (k != ch.is_c1.size()) throw Error(E_INVARIANT, "assignment length mismatch");
      stack.push_back(Work{as1, w.level, w.chain});
      stack.push_back(Work{as2, w.level, w.chain});
    } else {
      w.chain.push_back(ch.c1);
      if (w.level + 1 == max_level) {
        cons.push_back(w.chain);
        assigns.push_back(w.inc);
      } else {
        stack.push_back(Work{w.inc, w.level + 1, w.chain});
      }
    }
  }
  PriorityOut out;
  if (cons.size() > 1) {
    std::vector<size_t> ord(cons.size());
    for (size_t i = 0; i < ord.size(); ++i) ord[i] = i;
    std::stable_sort(ord.begin(), ord.end(), [&](size_t a, size_t b) {
      const auto& ca = cons[a];
      const auto& cb = cons[b];
      size_t n = std::min(ca.size(), cb.size());
      for (size_t i = 0; i < n; ++i)
        if (ca[i].sequence != cb[i].sequence) return ca[i].sequence < cb[i].sequence;
      return ca.size() < cb.size();
    });
    out.indices.assign(M, UINT64_MAX);
    for (size_t ci = 0; ci < ord.size(); ++ci) {
      for (size_t i = 0; i < M; ++i) {
        if (!assigns[ord[ci]][i]) continue;
        if (out.indices[i] != UINT64_MAX) throw Error(E_INVARIANT, "sequence assigned twice");
        out.indices[i] = ci;
      }
      out.chains.push_back(cons[ord[ci]]);
    }
  } else {
    out.chains = cons;
    out.indices.assign(M, 0);
  }
  return out;
}

// test hook: dual_consensus.rs:1362-1382 (test_get_ed_weights)
std::vector<double> test_ed_weights(const std::vector<Seq>& seqs, uint8_t s1, uint8_t s2, bool early, bool side1,
                                    bool weight_by_ed) {
  DNode n;
  const size_t N = seqs.size();
  n.dw1.assign(N, Dwfa());
  n.dw2.assign(N, Dwfa());
  n.a1.assign(N, 1);
  n.a2.assign(N, 0);
  for (size_t r = 0; r < N; ++r) n.dw1[r].early = n.dw2[r].early = early;
  dnode_activate_dual(n, seqs, s1, s2, nullptr);
  return dnode_ed_weights(n, side1, weight_by_ed);
}

}  // namespace wco
