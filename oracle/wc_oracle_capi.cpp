// ORACLE — TEST INFRASTRUCTURE ONLY (see rust_compat.hpp header).
// ctypes-friendly C ABI over the CPU restatement. Results come back as a
// malloc'd JSON string (free with orc_free); sequences are hex encoded so raw
// byte alphabets (example_gen's 0..3) survive.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "wc_oracle.hpp"

using namespace wco;

extern "C" {

struct orc_config {
  int32_t consensus_cost;
  int32_t wildcard;  // -1 = None
  uint64_t max_queue_size;
  uint64_t max_capacity_per_size;
  uint64_t max_return_size;
  uint64_t max_nodes_wo_constraint;
  uint64_t min_count;
  double min_af;
  uint64_t dual_max_ed_delta;
  uint64_t offset_window;
  uint64_t offset_compare_length;
  uint8_t weighted_by_ed;
  uint8_t allow_early_termination;
  uint8_t auto_shift_offsets;
  uint8_t _pad[5];
};

struct orc_counters {
  uint64_t updates, w_out, compares, ed_increases, finalizes, nodes_explored, nodes_ignored, peak_queue_size, pops,
      row_bytes;
};

void orc_free(char* p) { free(p); }
}

namespace {
Config to_cfg(const orc_config* c) {
  Config k;
  k.consensus_cost = c->consensus_cost;
  k.wildcard = c->wildcard;
  k.max_queue_size = c->max_queue_size;
  k.max_capacity_per_size = c->max_capacity_per_size;
  k.max_return_size = c->max_return_size;
  k.max_nodes_wo_constraint = c->max_nodes_wo_constraint;
  k.min_count = c->min_count;
  k.min_af = c->min_af;
  k.dual_max_ed_delta = c->dual_max_ed_delta;
  k.offset_window = c->offset_window;
  k.offset_compare_length = c->offset_compare_length;
  k.weighted_by_ed = c->weighted_by_ed;
  k.allow_early_termination = c->allow_early_termination;
  k.auto_shift_offsets = c->auto_shift_offsets;
  return k;
}

std::string hex(const std::vector<uint8_t>& v) {
  static const char* d = "0123456789abcdef";
  std::string s;
  s.reserve(v.size() * 2);
  for (uint8_t b : v) {
    s.push_back(d[b >> 4]);
    s.push_back(d[b & 15]);
  }
  return s;
}

template <class T>
std::string arr(const std::vector<T>& v) {
  std::string s = "[";
  for (size_t i = 0; i < v.size(); ++i) {
    if (i) s += ",";
    s += std::to_string(v[i]);
  }
  return s + "]";
}

std::string cons_json(const ConsensusOut& c) {
  return "{\"sequence\":\"" + hex(c.sequence) + "\",\"scores\":" + arr(c.scores) + "}";
}

char* dup(const std::string& s) {
  char* p = (char*)malloc(s.size() + 1);
  memcpy(p, s.c_str(), s.size() + 1);
  return p;
}

std::string err_json(const Error& e) {
  std::string m;
  for (char ch : std::string(e.what())) {
    if (ch == '"' || ch == '\\') m.push_back('\\');
    m.push_back(ch);
  }
  return "{\"ok\":false,\"code\":" + std::to_string(e.code) + ",\"error\":\"" + m + "\"}";
}

void copy_counters(const Counters& c, orc_counters* o) {
  if (!o) return;
  o->updates = c.updates;
  o->w_out = c.w_out;
  o->compares = c.compares;
  o->ed_increases = c.ed_increases;
  o->finalizes = c.finalizes;
  o->nodes_explored = c.nodes_explored;
  o->nodes_ignored = c.nodes_ignored;
  o->peak_queue_size = c.peak_queue_size;
  o->pops = c.pops;
  o->row_bytes = c.row_bytes;
}

std::vector<Seq> to_seqs(uint32_t n, const uint8_t* const* seqs, const uint64_t* lens) {
  std::vector<Seq> v;
  for (uint32_t i = 0; i < n; ++i) v.push_back(Seq{seqs[i], (size_t)lens[i]});
  return v;
}
}  // namespace

extern "C" {

// ConsensusDWFA::consensus (consensus.rs:139)
char* orc_consensus(const orc_config* cfg, uint32_t n, const uint8_t* const* seqs, const uint64_t* lens,
                    const int64_t* offsets, orc_counters* counters) {
  Counters c;
  try {
    std::vector<int64_t> offs(n, -1);
    if (offsets) offs.assign(offsets, offsets + n);
    auto res = consensus_single(to_cfg(cfg), to_seqs(n, seqs, lens), offs, &c);
    copy_counters(c, counters);
    std::string s = "{\"ok\":true,\"results\":[";
    for (size_t i = 0; i < res.size(); ++i) s += (i ? "," : "") + cons_json(res[i]);
    return dup(s + "]}");
  } catch (const Error& e) {
    copy_counters(c, counters);
    return dup(err_json(e));
  }
}

// DualConsensusDWFA::consensus (dual_consensus.rs:240)
char* orc_dual_consensus(const orc_config* cfg, uint32_t n, const uint8_t* const* seqs, const uint64_t* lens,
                         const int64_t* offsets, orc_counters* counters) {
  Counters c;
  try {
    std::vector<int64_t> offs(n, -1);
    if (offsets) offs.assign(offsets, offsets + n);
    auto res = consensus_dual(to_cfg(cfg), to_seqs(n, seqs, lens), offs, &c);
    copy_counters(c, counters);
    std::string s = "{\"ok\":true,\"results\":[";
    for (size_t i = 0; i < res.size(); ++i) {
      const DualOut& d = res[i];
      if (i) s += ",";
      std::vector<int> isc(d.is_c1.begin(), d.is_c1.end());
      s += "{\"consensus1\":" + cons_json(d.c1) + ",\"consensus2\":" + (d.has_c2 ? cons_json(d.c2) : "null") +
           ",\"is_consensus1\":" + arr(isc) + ",\"scores1\":" + arr(d.scores1) + ",\"scores2\":" + arr(d.scores2) +
           "}";
    }
    return dup(s + "]}");
  } catch (const Error& e) {
    copy_counters(c, counters);
    return dup(err_json(e));
  }
}

// PriorityConsensusDWFA::consensus (priority_consensus.rs:172)
// chains are laid out row-major: seqs[i*levels + l]; offsets likewise; seed_groups[i] (-1 None)
char* orc_priority_consensus(const orc_config* cfg, uint32_t n_chains, uint32_t levels, const uint8_t* const* seqs,
                             const uint64_t* lens, const int64_t* offsets, const int64_t* seed_groups,
                             orc_counters* counters) {
  Counters c;
  try {
    std::vector<std::vector<Seq>> chains(n_chains);
    std::vector<std::vector<int64_t>> offs(n_chains, std::vector<int64_t>(levels, -1));
    std::vector<int64_t> groups(n_chains, -1);
    for (uint32_t i = 0; i < n_chains; ++i) {
      for (uint32_t l = 0; l < levels; ++l) {
        chains[i].push_back(Seq{seqs[i * levels + l], (size_t)lens[i * levels + l]});
        if (offsets) offs[i][l] = offsets[i * levels + l];
      }
      if (seed_groups) groups[i] = seed_groups[i];
    }
    auto res = consensus_priority(to_cfg(cfg), chains, offs, groups, &c);
    copy_counters(c, counters);
    std::string s = "{\"ok\":true,\"consensuses\":[";
    for (size_t i = 0; i < res.chains.size(); ++i) {
      if (i) s += ",";
      s += "[";
      for (size_t j = 0; j < res.chains[i].size(); ++j) s += (j ? "," : "") + cons_json(res.chains[i][j]);
      s += "]";
    }
    return dup(s + "],\"sequence_indices\":" + arr(res.indices) + "}");
  } catch (const Error& e) {
    copy_counters(c, counters);
    return dup(err_json(e));
  }
}

// Standalone DWFALite driving (dynamic_wfa.rs unit tests). ops: for each k in
// [0, n_updates): update(baseline, other[0..upd_lens[k]]). Then finalize when
// do_finalize. Returns e after each update in eds_out, wavefront in wf_out (cap).
int orc_dwfa_run(const uint8_t* baseline, uint64_t blen, const uint8_t* other, const uint64_t* upd_lens,
                 uint32_t n_updates, int32_t wildcard, uint8_t early, uint64_t offset, uint8_t do_finalize,
                 uint64_t* eds_out, uint64_t* final_e, uint64_t* wf_out, uint64_t wf_cap, uint64_t* wf_len) {
  try {
    Dwfa d;
    d.wildcard = wildcard;
    d.early = early;
    d.offset = offset;
    Seq b{baseline, (size_t)blen};
    for (uint32_t k = 0; k < n_updates; ++k) eds_out[k] = d.update(b, Seq{other, (size_t)upd_lens[k]}, nullptr);
    if (do_finalize) {
      uint64_t ol = n_updates ? upd_lens[n_updates - 1] : 0;
      d.finalize(b, Seq{other, (size_t)ol}, nullptr);
    }
    *final_e = d.e;
    *wf_len = d.wf.size();
    for (size_t i = 0; i < d.wf.size() && i < wf_cap; ++i) wf_out[i] = d.wf[i];
    return 0;
  } catch (const Error& e) {
    return e.code;
  }
}

// Tip nomination of a DWFA after updates: returns symbols in FxHashMap
// iteration order and their counts (dynamic_wfa.rs:241-255).
int orc_dwfa_candidates(const uint8_t* baseline, uint64_t blen, const uint8_t* other, uint64_t olen, int32_t wildcard,
                        uint8_t* syms, uint64_t* counts, uint32_t cap, uint32_t* n_out) {
  Dwfa d;
  d.wildcard = wildcard;
  Seq b{baseline, (size_t)blen};
  for (uint64_t l = 1; l <= olen; ++l) d.update(b, Seq{other, (size_t)l}, nullptr);
  auto m = d.candidates(b, Seq{other, (size_t)olen});
  uint32_t k = 0;
  m.for_each([&](uint8_t s, uint64_t v) {
    if (k < cap) {
      syms[k] = s;
      counts[k] = v;
    }
    k++;
  });
  *n_out = k;
  return 0;
}

// The same nomination's keys in insertion order: dynamic_wfa.rs:244-250 calls
// entry(read[bo]).or_insert(0) tip by tip in ascending diagonal index, so the
// k-th key is the k-th distinct tip symbol. (Replaying these inserts through
// FxByteMap gives orc_dwfa_candidates' iteration order.)
int orc_dwfa_candidate_first(const uint8_t* baseline, uint64_t blen, const uint8_t* other, uint64_t olen,
                             int32_t wildcard, uint8_t* syms, uint32_t cap, uint32_t* n_out) {
  Dwfa d;
  d.wildcard = wildcard;
  Seq b{baseline, (size_t)blen};
  for (uint64_t l = 1; l <= olen; ++l) d.update(b, Seq{other, (size_t)l}, nullptr);
  bool seen[256] = {false};
  uint32_t k = 0;
  for (size_t i = 0; i < d.wf.size(); ++i) {
    const size_t dd = d.wf[i];
    if (dd + d.offset != (size_t)olen) continue;
    const size_t bo = dd + d.e - i;
    if (bo >= (size_t)blen || seen[baseline[bo]]) continue;
    seen[baseline[bo]] = true;
    if (k < cap) syms[k] = baseline[bo];
    k++;
  }
  *n_out = k;
  return 0;
}

// One DWFALite operation on an explicit state (clone = copy the state on the
// caller side). op 0 = update(baseline, other), 1 = finalize(baseline, other).
// State: *e, wf[0..*wf_len] (in/out, capacity wf_cap).
int orc_dwfa_step(const uint8_t* baseline, uint64_t blen, const uint8_t* other, uint64_t olen, int32_t wildcard,
                  uint8_t early, uint64_t offset, int op, uint64_t* e, uint64_t* wf, uint64_t* wf_len,
                  uint64_t wf_cap) {
  try {
    Dwfa d;
    d.wildcard = wildcard;
    d.early = early;
    d.offset = offset;
    d.e = *e;
    d.wf.assign(wf, wf + *wf_len);
    Seq b{baseline, (size_t)blen}, o{other, (size_t)olen};
    if (op == 0) d.update(b, o, nullptr);
    else d.finalize(b, o, nullptr);
    if (d.wf.size() > wf_cap) return E_INVARIANT;
    *e = d.e;
    *wf_len = d.wf.size();
    for (size_t i = 0; i < d.wf.size(); ++i) wf[i] = d.wf[i];
    return 0;
  } catch (const Error& ex) {
    return ex.code;
  }
}

// dual_consensus.rs:1299-1336 restated on a node built by new_root_node +
// activate_dual(s1, s2) (the shape of test_get_ed_weights, :1362-1382).
int orc_test_ed_weights(uint32_t n, const uint8_t* const* seqs, const uint64_t* lens, uint8_t s1, uint8_t s2,
                        uint8_t early, uint8_t side1, uint8_t weight_by_ed, double* out) {
  try {
    auto w = test_ed_weights(to_seqs(n, seqs, lens), s1, s2, early, side1, weight_by_ed);
    for (size_t i = 0; i < w.size(); ++i) out[i] = w[i];
    return 0;
  } catch (const Error& e) {
    return e.code;
  }
}

uint64_t orc_wfa_ed_config(const uint8_t* v1, uint64_t l1, const uint8_t* v2, uint64_t l2, uint8_t require_both,
                           int32_t wildcard) {
  return wfa_ed_config(Seq{v1, (size_t)l1}, Seq{v2, (size_t)l2}, require_both, wildcard);
}

// FxByteMap<usize> iteration order after inserting keys in order (Appendix B check)
uint32_t orc_fxmap_order(const uint8_t* keys, uint32_t n, uint8_t* out) {
  FxByteMap<uint64_t> m;
  for (uint32_t i = 0; i < n; ++i) m.entry(keys[i], 0) += 1;
  uint32_t k = 0;
  m.for_each([&](uint8_t s, uint64_t) { out[k++] = s; });
  return k;
}

// seed-group processing order (priority_consensus.rs:180), -1 = None; returns the key count
uint32_t orc_seed_group_order(const int64_t* groups, uint32_t n, int64_t* out) {
  std::vector<int64_t> g(groups, groups + n);
  std::vector<int64_t> o = seed_group_order(g);
  for (size_t i = 0; i < o.size(); ++i) out[i] = o[i];
  return (uint32_t)o.size();
}
}
