// ORACLE — TEST INFRASTRUCTURE ONLY (see rust_compat.hpp header).
// CPU restatement of the reference's DWFA scoring path and the three
// consensus engines. Every function cites the reference file:line it follows.
#pragma once
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "rust_compat.hpp"

namespace wco {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// error codes shared with include/waffle_con.h (same numbering)
enum : int {
  E_OK = 0,
  E_FINALIZE_UNINIT = 1,   // consensus.rs:473, dual_consensus.rs:1078
  E_NO_START = 2,          // consensus.rs:205, dual_consensus.rs:303
  E_COVERAGE_GAP = 3,      // consensus.rs:305
  E_CAPACITY = 4,          // pqueue_tracker.rs:90
  E_LOCKED = 5,            // dual_consensus.rs:917,919
  E_DUAL_TWICE = 6,        // dual_consensus.rs:959
  E_SAME_SYMBOL = 7,       // dual_consensus.rs:964
  E_ROOT_INACTIVE = 8,     // consensus.rs:396, dual_consensus.rs:843
  E_BAD_INPUT = 9,         // priority_consensus.rs:144,148 / empty inputs
  E_INVARIANT = 10,        // reference assert!/panic sites
};

// cdwfa_config.rs:38-103
struct Config {
  int consensus_cost = 0;  // 0 = L1Distance, 1 = L2Distance
  uint64_t max_queue_size = 20;
  uint64_t max_capacity_per_size = 20;
  uint64_t max_return_size = 10;
  uint64_t max_nodes_wo_constraint = 1000;
  uint64_t min_count = 3;
  double min_af = 0.0;
  bool weighted_by_ed = false;
  int wildcard = -1;  // -1 = None
  uint64_t dual_max_ed_delta = 20;
  bool allow_early_termination = false;
  bool auto_shift_offsets = true;
  uint64_t offset_window = 50;
  uint64_t offset_compare_length = 50;
};

// deterministic work counters
struct Counters {
  uint64_t updates = 0;        // DWFALite::update calls
  uint64_t w_out = 0;          // sum of post-update wavefront lengths
  uint64_t compares = 0;       // byte compares reached in extend
  uint64_t ed_increases = 0;   // increase_edit_distance calls
  uint64_t finalizes = 0;      // DWFALite::finalize calls
  uint64_t nodes_explored = 0;
  uint64_t nodes_ignored = 0;
  uint64_t peak_queue_size = 0;
  uint64_t pops = 0;
  uint64_t row_bytes = 0;      // wavefront bytes read + written by updates/finalizes that grow e
};

struct Seq {
  const uint8_t* p;
  size_t n;
};

// dynamic_wfa.rs:12-265
struct Dwfa {
  size_t e = 0;
  std::vector<size_t> wf{0};
  int wildcard = -1;
  bool early = false;
  size_t offset = 0;

  bool operator==(const Dwfa& o) const {
    return e == o.e && wf == o.wf && wildcard == o.wildcard && early == o.early && offset == o.offset;
  }

  size_t update(Seq b, Seq o, Counters* c);
  void extend(Seq b, Seq o, Counters* c);
  void increase(Seq b, Seq o, Counters* c);
  void finalize(Seq b, Seq o, Counters* c);
  size_t max_baseline() const;
  size_t max_other() const;
  bool reached_end(Seq b) const { return max_baseline() == b.n; }
  FxByteMap<uint64_t> candidates(Seq b, Seq o) const;
};

size_t wfa_ed_config(Seq v1, Seq v2, bool require_both_end, int wildcard);

// ---- results ----
struct ConsensusOut {
  std::vector<uint8_t> sequence;
  std::vector<uint64_t> scores;
};

struct DualOut {
  ConsensusOut c1;
  bool has_c2 = false;
  ConsensusOut c2;
  std::vector<uint8_t> is_c1;
  std::vector<int64_t> scores1, scores2;  // -1 = None
};

struct PriorityOut {
  std::vector<std::vector<ConsensusOut>> chains;
  std::vector<uint64_t> indices;
};

// offsets: -1 = None
std::vector<ConsensusOut> consensus_single(const Config& cfg, const std::vector<Seq>& seqs,
                                           const std::vector<int64_t>& offsets, Counters* c);
std::vector<DualOut> consensus_dual(const Config& cfg, const std::vector<Seq>& seqs,
                                    const std::vector<int64_t>& offsets, Counters* c);
// chains[i][level]; offsets[i][level]; seed_groups[i] (-1 = None)
PriorityOut consensus_priority(const Config& cfg, const std::vector<std::vector<Seq>>& chains,
                               const std::vector<std::vector<int64_t>>& offsets,
                               const std::vector<int64_t>& seed_groups, Counters* c);

std::vector<double> test_ed_weights(const std::vector<Seq>& seqs, uint8_t s1, uint8_t s2, bool early, bool side1,
                                    bool weight_by_ed);

// FxHashSet<Option<usize>> iteration order of the seed groups (priority_consensus.rs:180); -1 = None
std::vector<int64_t> seed_group_order(const std::vector<int64_t>& groups);
}  // namespace wco
