// sequence_alignment.rs:18-87 — pairwise WFA edit distance, host reference
// API (wc_wfa_ed_config). Not on the consensus hot path; the device engine
// uses its own copy for offset activation.
#include <algorithm>
#include <cstdint>
#include <utility>
#include <vector>

#include "../../include/waffle_con.h"

extern "C" uint64_t wc_wfa_ed_config(const uint8_t* v1, uint64_t l1, const uint8_t* v2, uint64_t l2,
                                     uint8_t require_both_end, int32_t wildcard) {
  typedef std::pair<uint64_t, uint64_t> P;  // (i into v1, j into v2), compared lexicographically
  auto wc = [&](uint8_t a) { return wildcard >= 0 && a == (uint8_t)wildcard; };
  std::vector<P> cur(1, P(0, 0)), nxt(3, P(0, 0));
  for (uint64_t edits = 0;; ++edits) {
    for (size_t k = 0; k < cur.size(); ++k) {
      uint64_t i = cur[k].first, j = cur[k].second;
      while (i < l1 && j < l2 && (v1[i] == v2[j] || wc(v1[i]) || wc(v2[j]))) ++i, ++j;
      if ((i == l1 || !require_both_end) && j == l2) return edits;
      const P a = i == l1 ? P(i, j) : P(i + 1, j);
      const P b = i == l1 ? P(i, j + 1) : (j == l2 ? P(i + 1, j) : P(i + 1, j + 1));
      const P c = j == l2 && i != l1 ? P(i, j) : P(i, j + 1);
      nxt[k] = std::max(nxt[k], a);
      nxt[k + 1] = std::max(nxt[k + 1], b);
      nxt[k + 2] = std::max(nxt[k + 2], c);
    }
    cur.swap(nxt);
    nxt.assign(3 + 2 * (edits + 1), P(0, 0));
  }
}
