// Device building blocks shared by the consensus engines (engine.hip).
//
// Mapping: one workgroup (4 x wave64) owns one consensus
// problem for its whole search. Per-read DWFA work is spread over the waves
// (read r -> wave r % 4) with the 64 lanes over the read's wavefront
// diagonals. Host-style control logic (heap, tracker, thresholds) runs on
// thread 0 against LDS and is broadcast through LDS between barriers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "engine_shared.hpp"

namespace wc {

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
  return v;
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

__device__ __forceinline__ uint64_t cost_of(uint32_t e, int mode) {
  return mode == 0 ? (uint64_t)e : (uint64_t)e * (uint64_t)e;
}

// --- FxHashMap<u8,_> iteration order (oracle rust_compat.hpp) ---
// Given distinct keys in insertion order, produce the bucket-ascending order.
// Supports up to 16 keys (tables of 4, 8, 16 or 32 buckets).
__device__ inline uint32_t fx_cap(uint32_t b) { return b == 0 ? 0 : (b < 8 ? b - 1 : b / 8 * 7); }
__device__ inline uint32_t fx_buckets_for(uint32_t cap) {
  if (cap < 8) return cap < 4 ? 4 : 8;
  uint32_t adj = cap * 8 / 7, p = 1;
  while (p < adj) p <<= 1;
  return p;
}
__device__ inline uint32_t fx_slot(const int16_t* tab, uint32_t B, uint8_t k) {
  uint64_t h = (uint64_t)k * 0x517cc1b727220a95ULL;
  uint32_t mask = B - 1, pos = (uint32_t)h & mask;
  if (B < 16) {
    for (uint32_t i = pos; i < B; ++i)
      if (tab[i] < 0) return i;
    for (uint32_t i = 0; i < B; ++i)
      if (tab[i] < 0) return i;
    return 0;
  }
  uint32_t stride = 0;
  for (;;) {
    for (uint32_t j = 0; j < 16; ++j)
      if (tab[(pos + j) & mask] < 0) return (pos + j) & mask;
    stride += 16;
    pos = (pos + stride) & mask;
  }
}
// keys[0..n) distinct in insertion order -> out[0..n) iteration order (indices into keys)
__device__ inline void fx_order(const uint8_t* keys, uint32_t n, uint8_t* out) {
  int16_t tab[32];
  uint32_t B = 0, items = 0, growth = 0;
  for (uint32_t k = 0; k < n; ++k) {
    if (growth == 0) {
      uint32_t want = max(items + 1, fx_cap(B) + 1);
      uint32_t nb = fx_buckets_for(want);
      int16_t old[32];
      for (uint32_t i = 0; i < B; ++i) old[i] = tab[i];
      for (uint32_t i = 0; i < nb; ++i) tab[i] = -1;
      for (uint32_t i = 0; i < B; ++i)
        if (old[i] >= 0) tab[fx_slot(tab, nb, keys[old[i]])] = old[i];
      B = nb;
      growth = fx_cap(nb) - items;
    }
    tab[fx_slot(tab, B, keys[k])] = (int16_t)k;
    items++;
    growth--;
  }
  uint32_t m = 0;
  for (uint32_t i = 0; i < B; ++i)
    if (tab[i] >= 0) out[m++] = (uint8_t)tab[i];
}

// --- per-read DWFA views ---
struct SideView {
  uint32_t* e;    // [nmax]
  uint32_t* off;  // [nmax]
  uint32_t* wf;   // [nmax * wcap]
  uint8_t* con;   // [lcap]
};

__device__ inline SideView side_view(uint8_t* slot_base, uint32_t side, uint32_t nmax, uint32_t wcap, uint32_t lcap) {
  uint8_t* b = slot_base + (uint64_t)side * side_bytes(nmax, wcap, lcap);
  SideView v;
  v.e = (uint32_t*)b;
  v.off = v.e + nmax;
  v.wf = v.off + nmax;
  v.con = b + align16((uint64_t)nmax * 8 + (uint64_t)nmax * wcap * 4);
  return v;
}

struct WaveCounters {
  uint32_t updates, w_out, compares, edinc, finalizes;
};

// Full extend of every diagonal of `wf[0..W)` (dynamic_wfa.rs:109-153),
// lanes over diagonals. Returns (via refs) wave-reduced max_other - off and
// max_baseline. Counts byte compares as the reference loop would.
__device__ inline void wave_extend_all(uint32_t* wf, uint32_t W, uint32_t e, uint32_t off, const uint8_t* rd,
                                       uint32_t blen, const uint8_t* con, uint32_t olen, int wc, uint32_t& maxo,
                                       uint32_t& maxb, uint32_t& cmp) {
  const int lane = lane_id();
  uint32_t mo = 0, mb = 0, c = 0;
  for (uint32_t base = 0; base < W; base += 64) {
    uint32_t i = base + lane;
    if (i < W) {
      uint32_t d = wf[i];
      uint32_t d0 = d;
      for (;;) {
        uint32_t bo = d + e - i;
        uint32_t oo = d + off;
        if (bo >= blen || oo >= olen) break;
        c++;
        uint8_t x = rd[bo];
        if (x != con[oo] && !(wc >= 0 && x == (uint8_t)wc)) break;
        d++;
      }
      if (d != d0) wf[i] = d;
      mo = max(mo, d);
      mb = max(mb, d + e - i);
    }
  }
  maxo = wave_max_u32(mo);
  maxb = wave_max_u32(mb);
  cmp += c;
}

// increase_edit_distance in place (dynamic_wfa.rs:162-183): W -> W+2.
// Chunks are processed from the top so a chunk never reads an entry that a
// previously processed chunk overwrote.
__device__ inline void wave_grow(uint32_t* wf, uint32_t Wold) {
  const int lane = lane_id();
  const uint32_t Wn = Wold + 2;
  for (int base = (int)((Wn - 1) / 64) * 64; base >= 0; base -= 64) {
    uint32_t j = (uint32_t)base + lane;
    uint32_t nv = 0;
    if (j < Wn) {
      if (j < Wold) nv = wf[j];
      if (j >= 1 && j - 1 < Wold) nv = max(nv, wf[j - 1] + 1);
      if (j >= 2 && j - 2 < Wold) nv = max(nv, wf[j - 2] + 1);
    }
    __builtin_amdgcn_wave_barrier();
    if (j < Wn) wf[j] = nv;
    __builtin_amdgcn_wave_barrier();
  }
}

// DWFALite::update for one appended symbol (consensus grew from olen-1 to
// olen, con[olen-1] == sym). Only diagonals sitting exactly at the old end can
// move (by one); every other diagonal is provably blocked by the same
// mismatch / read end as in the previous extend, so it is only counted, not
// re-compared. Then the ED-increase loop of dynamic_wfa.rs:84-91.
// Returns false on wavefront capacity overflow.
__device__ inline bool wave_push_read(uint32_t* wf, uint32_t& e, uint32_t off, const uint8_t* rd, uint32_t blen,
                                      const uint8_t* con, uint32_t olen, uint8_t sym, int wc, bool early,
                                      uint32_t wcap, WaveCounters& cnt) {
  const int lane = lane_id();
  uint32_t W = 2 * e + 1;
  const uint32_t old_end = olen - 1;
  uint32_t mo = 0, mb = 0, c = 0;
  for (uint32_t base = 0; base < W; base += 64) {
    uint32_t i = base + lane;
    if (i < W) {
      uint32_t d = wf[i];
      uint32_t bo = d + e - i;
      if (bo < blen && d + off < olen) {
        c++;  // the reference compares here (and fails unless this is a tip)
        if (d + off == old_end) {
          uint8_t x = rd[bo];
          if (x == sym || (wc >= 0 && x == (uint8_t)wc)) {
            d++;
            wf[i] = d;
          }
        }
      }
      mo = max(mo, d);
      mb = max(mb, d + e - i);
    }
  }
  mo = wave_max_u32(mo) + off;
  mb = wave_max_u32(mb);
  uint32_t cmp = c;
  while (mo < olen && !(early && mb == blen)) {
    if (W + 2 > wcap) return false;
    wave_grow(wf, W);
    W += 2;
    e += 1;
    cnt.edinc++;
    uint32_t m;
    wave_extend_all(wf, W, e, off, rd, blen, con, olen, wc, m, mb, cmp);
    mo = m + off;
  }
  cnt.updates++;
  cnt.w_out += W;
  cnt.compares += wave_sum_u32(cmp);
  return true;
}

// General DWFALite::update (other may have grown by any amount):
// dynamic_wfa.rs:75-99 with a full extend first.
__device__ inline bool wave_update_general(uint32_t* wf, uint32_t& e, uint32_t off, const uint8_t* rd, uint32_t blen,
                                           const uint8_t* con, uint32_t olen, int wc, bool early, uint32_t wcap,
                                           WaveCounters& cnt, uint32_t& mo, uint32_t& mb) {
  uint32_t W = 2 * e + 1, cmp = 0;
  wave_extend_all(wf, W, e, off, rd, blen, con, olen, wc, mo, mb, cmp);
  mo += off;
  while (mo < olen && !(early && mb == blen)) {
    if (W + 2 > wcap) return false;
    wave_grow(wf, W);
    W += 2;
    e += 1;
    cnt.edinc++;
    wave_extend_all(wf, W, e, off, rd, blen, con, olen, wc, mo, mb, cmp);
    mo += off;
  }
  cnt.updates++;
  cnt.w_out += W;
  cnt.compares += wave_sum_u32(cmp);
  return true;
}

// DWFALite::finalize (dynamic_wfa.rs:201-210) on a scratch copy of the
// wavefront; the node itself is untouched (the reference finalizes a clone).
__device__ inline bool wave_finalize_read(const uint32_t* wf, uint32_t e, uint32_t off, const uint8_t* rd,
                                          uint32_t blen, const uint8_t* con, uint32_t olen, int wc, uint32_t* scratch,
                                          uint32_t wcap, uint32_t& e_out, WaveCounters& cnt) {
  const int lane = lane_id();
  uint32_t W = 2 * e + 1;
  uint32_t mb = 0;
  for (uint32_t base = 0; base < W; base += 64) {
    uint32_t i = base + lane;
    if (i < W) {
      uint32_t d = wf[i];
      scratch[i] = d;
      mb = max(mb, d + e - i);
    }
  }
  mb = wave_max_u32(mb);
  uint32_t cmp = 0;
  cnt.finalizes++;
  while (mb < blen) {
    if (W + 2 > wcap) return false;
    __builtin_amdgcn_wave_barrier();
    wave_grow(scratch, W);
    W += 2;
    e += 1;
    cnt.edinc++;
    uint32_t mo;
    wave_extend_all(scratch, W, e, off, rd, blen, con, olen, wc, mo, mb, cmp);
  }
  cnt.compares += wave_sum_u32(cmp);
  e_out = e;
  return true;
}

// Tip nomination of one read (dynamic_wfa.rs:241-255) plus reached_baseline_end
// (:232-234). Distinct symbols are found in first-appearance order (ascending
// diagonal), then permuted into FxHashMap iteration order. Returns false when
// more than kKmax distinct symbols sit at the tips.
__device__ inline bool wave_analyze_read(const uint32_t* wf, uint32_t e, uint32_t off, const uint8_t* rd,
                                         uint32_t blen, uint32_t olen, RInfo* out) {
  const int lane = lane_id();
  const uint32_t W = 2 * e + 1;
  uint8_t keys[kKmax];
  uint32_t cnts[kKmax];
  uint32_t nk = 0;
  uint32_t mb = 0;
  bool ok = true;
  for (uint32_t base = 0; base < W; base += 64) {
    uint32_t i = base + lane;
    bool tip = false;
    uint32_t s = 0;
    if (i < W) {
      uint32_t d = wf[i];
      uint32_t bo = d + e - i;
      mb = max(mb, bo);
      if (d + off == olen && bo < blen) {
        tip = true;
        s = rd[bo];
      }
    }
    uint64_t m = ballot(tip);
    while (m) {
      int first = __ffsll((unsigned long long)m) - 1;
      uint32_t sym = (uint32_t)__shfl((int)s, first, 64);
      uint64_t ms = ballot(tip && s == sym);
      uint32_t k = 0;
      while (k < nk && keys[k] != (uint8_t)sym) ++k;
      if (k == nk) {
        if (nk == kKmax) {
          ok = false;
          break;
        }
        keys[nk] = (uint8_t)sym;
        cnts[nk] = 0;
        nk++;
      }
      cnts[k] += (uint32_t)__popcll((unsigned long long)ms);
      m &= ~ms;
    }
  }
  mb = wave_max_u32(mb);
  if (lane == 0) {
    uint8_t ord[kKmax];
    fx_order(keys, nk, ord);
    uint32_t split = 0;
    for (uint32_t k = 0; k < nk; ++k) {
      out->sym[k] = keys[ord[k]];
      out->occ[k] = (uint16_t)cnts[ord[k]];
      split += cnts[ord[k]];
    }
    out->n = (uint8_t)nk;
    out->split = (uint16_t)split;
    out->end = (mb == blen);
    out->e = e;
  }
  return ok;
}

}  // namespace wc
