// ORACLE — TEST INFRASTRUCTURE ONLY.
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
// anything under oracle/. The product path (waffle_con_amd/) never links it.
//
// Emulators for the observable behaviour of the third-party Rust crates the
// reference depends on (none of their sources are in the container; see
// SURVEY.md Appendix A/B):
//   * priority-queue 1.x binary heap tie order   (consensus.rs:217-219,235,338)
//   * std HashMap (hashbrown, SSE2 groups) + rustc-hash 1.1 FxHasher iteration
//     order for u8 keys                          (dynamic_wfa.rs:241-254,
//                                                 consensus.rs:540-563)
#pragma once
#include <cstdint>
#include <cstring>
#include <utility>
#include <vector>

namespace wco {

// ---------------------------------------------------------------------------
// FxHashMap<u8, V> with hashbrown (group width 16) bucket placement.
// Iteration = ascending bucket index; inserts probe from h1 = hash & mask.
// ---------------------------------------------------------------------------
constexpr uint64_t kFxSeed = 0x517cc1b727220a95ULL;

inline uint64_t fx_hash_u8(uint8_t b) { return (uint64_t)b * kFxSeed; }

// capacity of a table with `buckets` buckets (hashbrown bucket_mask_to_capacity)
inline size_t fx_capacity(size_t buckets) {
  if (buckets == 0) return 0;
  if (buckets < 8) return buckets - 1;
  return buckets / 8 * 7;
}

// buckets chosen for a requested capacity (hashbrown capacity_to_buckets, 16-B entries)
inline size_t fx_buckets_for(size_t cap) {
  if (cap < 8) return cap < 4 ? 4 : 8;
  size_t adj = cap * 8 / 7;
  size_t p = 1;
  while (p < adj) p <<= 1;
  return p;
}

template <class V>
class FxByteMap {
 public:
  // slot key: -1 = EMPTY, -2 = DELETED, 0..255 = key
  std::vector<int16_t> key;
  std::vector<V> val;
  size_t items = 0;
  size_t growth_left = 0;

  size_t buckets() const { return key.size(); }

  int find(uint8_t k) const {
    for (size_t i = 0; i < key.size(); ++i)
      if (key[i] == k) return (int)i;
    return -1;
  }

  // returns reference to the value for k, inserting `init` when absent
  // (entry(k).or_insert(init); reserve(1) happens only for vacant keys)
  V& entry(uint8_t k, const V& init) {
    int f = find(k);
    if (f >= 0) return val[f];
    if (growth_left == 0) grow(items + 1);
    size_t slot = insert_slot(fx_hash_u8(k));
    key[slot] = k;
    val[slot] = init;
    items++;
    growth_left--;
    return val[slot];
  }

  bool remove(uint8_t k) {
    int f = find(k);
    if (f < 0) return false;
    key[f] = -2;  // order of the others is unchanged
    items--;
    return true;
  }

  size_t size() const { return items; }
  bool empty() const { return items == 0; }

  template <class F>
  void for_each(F&& fn) const {
    for (size_t i = 0; i < key.size(); ++i)
      if (key[i] >= 0) fn((uint8_t)key[i], val[i]);
  }

 private:
  size_t insert_slot(uint64_t hash) const {
    const size_t B = key.size();
    const size_t mask = B - 1;
    size_t pos = (size_t)hash & mask;
    if (B < 16) {
      // group load covers [pos, B) then trailing EMPTY fakes; a fake hit maps to
      // bucket 0 and is fixed up by rescanning from 0 (fix_insert_slot)
      for (size_t i = pos; i < B; ++i)
        if (key[i] < 0) return i;
      for (size_t i = 0; i < B; ++i)
        if (key[i] < 0) return i;
      return (size_t)-1;
    }
    size_t stride = 0;
    for (;;) {
      for (size_t j = 0; j < 16; ++j) {
        size_t idx = (pos + j) & mask;
        if (key[idx] < 0) return idx;
      }
      stride += 16;
      pos = (pos + stride) & mask;
    }
  }

  void grow(size_t need) {
    size_t full_cap = fx_capacity(key.size());
    size_t want = need > full_cap + 1 ? need : full_cap + 1;
    size_t nb = fx_buckets_for(want);
    std::vector<int16_t> ok = std::move(key);
    std::vector<V> ov = std::move(val);
    key.assign(nb, -1);
    val.assign(nb, V());
    for (size_t i = 0; i < ok.size(); ++i) {
      if (ok[i] < 0) continue;
      size_t s = insert_slot(fx_hash_u8((uint8_t)ok[i]));
      key[s] = ok[i];
      val[s] = ov[i];
    }
    growth_left = fx_capacity(nb) - items;
  }
};

// ---------------------------------------------------------------------------
// priority-queue 1.x max-heap of item ids with priority (Reverse(cost), len).
// push: sift up while parent < new (strict). pop: swap_remove(0) + heapify
// with strict comparisons (left checked before right).
// ---------------------------------------------------------------------------
struct Prio {
  uint64_t cost;
  uint64_t len;
};
inline bool prio_less(const Prio& a, const Prio& b) {
  // (Reverse(cost), len) lexicographic "<"
  if (a.cost != b.cost) return a.cost > b.cost;
  return a.len < b.len;
}

class PQHeap {
 public:
  struct Entry {
    Prio p;
    int id;
  };
  std::vector<Entry> h;

  size_t size() const { return h.size(); }
  bool empty() const { return h.empty(); }

  void push(int id, Prio p) {
    h.push_back({p, id});
    size_t pos = h.size() - 1;
    Entry e = h[pos];
    while (pos > 0) {
      size_t parent = (pos - 1) / 2;
      if (!prio_less(h[parent].p, e.p)) break;
      h[pos] = h[parent];
      pos = parent;
    }
    h[pos] = e;
  }

  Entry pop() {
    Entry top = h[0];
    h[0] = h.back();
    h.pop_back();
    size_t n = h.size();
    size_t i = 0;
    if (n > 1) {
      for (;;) {
        size_t l = 2 * i + 1, r = 2 * i + 2, largest = i;
        if (l < n) {
          if (prio_less(h[largest].p, h[l].p)) largest = l;
          if (r < n && prio_less(h[largest].p, h[r].p)) largest = r;
        }
        if (largest == i) break;
        std::swap(h[i], h[largest]);
        i = largest;
      }
    }
    return top;
  }
};

}  // namespace wco
