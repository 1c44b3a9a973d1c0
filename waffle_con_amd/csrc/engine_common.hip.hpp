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

// The engine is compiled twice: normally (namespace wc, per-problem search
// state in LDS) and as engine_gstate.hip (namespace wcg, WC_GLOBAL_STATE: the
// same state in a per-workgroup HBM region) for problems whose state does not
// fit one workgroup's 160 KiB of LDS (many reads, deep queues).
#ifndef WC_ENGINE_NS
#define WC_ENGINE_NS wc
#endif

namespace WC_ENGINE_NS {
using namespace ::wc;

// threads per engine workgroup of this build (engine_narrow.hip: 128,
// engine_cu.hip: 1024); problems have at most kBlock = 256 reads, and the
// LDS/HBM layouts' per-wave parts are sized for the build (engine_shared.hpp)
#ifndef WC_BLOCK
#define WC_BLOCK 256
#endif
constexpr int kEB = WC_BLOCK;
constexpr int kEW = kEB / 64;
// thread paths skip frontier slots past the lane's last live one; the
// 256-thread build (128 VGPRs) spills more with the extra control flow than it
// saves (cfg3 -6%), the 128-thread build has the registers (cfg5 +4%)
constexpr bool kSlotBound = kEB <= 128;
static_assert(kEB % 64 == 0 && kEB <= 64 * kMaxWaves, "engine workgroup size");

// Explicit address spaces: HBM (global) and LDS pointers compile to global_* /
// ds_* instructions instead of flat_* (which wait on both counters and take
// the slower path). The engines keep every pointer in one of these types:
// Gm = HBM, Lo = LDS, Sh = the search state (LDS, or HBM in the global-state
// build). (The host pass of this single-source file only parses device code;
// it sees plain types.)
#if defined(__HIP_DEVICE_COMPILE__)
template <class T> using Gm = __attribute__((address_space(1))) T;
template <class T> using Lo = __attribute__((address_space(3))) T;
#ifdef WC_GLOBAL_STATE
template <class T> using Sh = __attribute__((address_space(1))) T;
#else
template <class T> using Sh = __attribute__((address_space(3))) T;
#endif
#else
template <class T> using Gm = T;
template <class T> using Lo = T;
template <class T> using Sh = T;
#endif

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

// Bounds-checked debug builds (-DWC_CHECK, `make check`): every index into the
// node pool, the search state (heap, free stack, work list, slot metadata),
// the read table and the tracker arrays goes through WC_IX(i, n). An index out
// of range is reported (file line, index, bound, workgroup, thread) and
// replaced by 0, so the access stays inside its buffer instead of faulting;
// the host reads the hit count back after the launch (wc_check_hits).
#ifdef WC_CHECK
__device__ unsigned int wc_chk_hits;
__device__ __noinline__ uint32_t wc_chk_fail(uint32_t line, uint64_t i, uint64_t n) {
  if (atomicAdd(&wc_chk_hits, 1u) < 64u)
    printf("[wc-check] line %u: index %llu >= bound %llu (workgroup %u thread %u)\n", line, (unsigned long long)i,
           (unsigned long long)n, blockIdx.x, threadIdx.x);
  return 0;
}
__device__ __forceinline__ uint32_t wc_ix(uint64_t i, uint64_t n, uint32_t line) {
  return i < n ? (uint32_t)i : wc_chk_fail(line, i, n);
}
#define WC_IX(i, n) wc_ix((i), (n), __LINE__)
// Wave-wide reductions and ballot-driven code (the DPP row sums read lanes 0,
// 16, 32, 48 and every lane's neighbours) are only correct with all 64 lanes
// in exec; checked builds report every call site reached with a partial mask.
__device__ __noinline__ void wc_chk_exec_fail(uint32_t line, uint64_t exec) {
  if (atomicAdd(&wc_chk_hits, 1u) < 64u)
    printf("[wc-check] line %u: partial exec 0x%016llx (workgroup %u wave %u)\n", line, (unsigned long long)exec,
           blockIdx.x, threadIdx.x >> 6);
}
#define WC_FULL_EXEC()                                                     \
  do {                                                                     \
    const uint64_t _ex = __builtin_amdgcn_read_exec();                     \
    if (_ex != ~0ull && (threadIdx.x & 63) == (uint32_t)__builtin_ctzll(_ex)) \
      wc_chk_exec_fail(__LINE__, _ex);                                     \
  } while (0)
// a per-wave LDS index (wave w of the build's kEW) in range
#define WC_WAVE_IX(w, n) wc_ix((w), (n), __LINE__)
#else
#define WC_IX(i, n) (i)
#define WC_FULL_EXEC() \
  do {                 \
  } while (0)
#define WC_WAVE_IX(w, n) (w)
#endif

// Wave64 reductions through DPP lane moves (VALU, no LDS round trips): quad
// swaps, half-row and row mirrors leave every lane with its 16-lane row
// result; the four row results are read into scalar registers. Lanes outside
// exec read as 0 (bound_ctrl), the identity of max and sum.
template <int kCtrl>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, 0xf, 0xf, true);
}
__device__ __forceinline__ uint32_t row_max_u32(uint32_t v) {
  v = max(v, dpp_u32<0xb1>(v));   // quad_perm [1,0,3,2]
  v = max(v, dpp_u32<0x4e>(v));   // quad_perm [2,3,0,1]
  v = max(v, dpp_u32<0x141>(v));  // row_half_mirror
  v = max(v, dpp_u32<0x140>(v));  // row_mirror
  return v;
}
__device__ __forceinline__ uint32_t row_sum_u32(uint32_t v) {
  v += dpp_u32<0xb1>(v);
  v += dpp_u32<0x4e>(v);
  v += dpp_u32<0x141>(v);
  v += dpp_u32<0x140>(v);
  return v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  WC_FULL_EXEC();
  v = row_max_u32(v);
  return max(max((uint32_t)__builtin_amdgcn_readlane((int)v, 0), (uint32_t)__builtin_amdgcn_readlane((int)v, 16)),
             max((uint32_t)__builtin_amdgcn_readlane((int)v, 32), (uint32_t)__builtin_amdgcn_readlane((int)v, 48)));
}
// lane i reads lane i-1 (row_ror: within its 16-lane row, wave_ror: of the wave), cyclically
__device__ __forceinline__ uint32_t row_ror1(uint32_t v) { return dpp_u32<0x121>(v); }
__device__ __forceinline__ uint32_t row_ror2(uint32_t v) { return dpp_u32<0x122>(v); }
__device__ __forceinline__ uint32_t wave_ror1(uint32_t v) { return dpp_u32<0x13c>(v); }
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
  WC_FULL_EXEC();
  v = row_sum_u32(v);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) + (uint32_t)__builtin_amdgcn_readlane((int)v, 16) +
         (uint32_t)__builtin_amdgcn_readlane((int)v, 32) + (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

__device__ __forceinline__ uint64_t cost_of(uint32_t e, int mode) {
  return mode == 0 ? (uint64_t)e : (uint64_t)e * (uint64_t)e;
}

// --- FxHashMap<u8,_> iteration order (oracle rust_compat.hpp) ---
// hashbrown with FxHasher over u8 keys: the table (4, 8 or 16 buckets for up
// to 14 keys) is kept in one u64 of 4-bit bucket tags (key index + 1), so no
// private array (and no scratch memory) is needed. Insertion is the first
// empty bucket cyclically from h1 = (k * FxSEED) & (B - 1); growth rebuilds in
// ascending bucket order; iteration is ascending bucket order.
__device__ inline uint32_t fx_cap(uint32_t b) { return b == 0 ? 0 : (b < 8 ? b - 1 : b / 8 * 7); }
__device__ inline uint32_t fx_buckets_for(uint32_t cap) { return cap < 4 ? 4 : (cap < 8 ? 8 : 16); }
// h1 = (k * FxSEED) & (B - 1) only depends on FxSEED mod B; B <= 16 and
// FxSEED = 0x517cc1b727220a95 = 5 (mod 16), so h1 = (5k) & (B - 1).
__device__ inline uint64_t fx_put(uint64_t T, uint32_t B, uint32_t key, uint32_t tag) {
  uint32_t pos = ((key & 0xFFu) * 5u) & (B - 1);
  for (uint32_t t = 0; t < B; ++t) {
    const uint32_t b = (pos + t) & (B - 1);
    if (((T >> (4 * b)) & 15ull) == 0) return T | ((uint64_t)tag << (4 * b));
  }
  return T;
}
// keys: key(k) for k in [0, n) distinct, in insertion order (n <= 14).
// Returns the iteration order as 4-bit key indices (nibble m = m-th key).
template <class KeyFn>
__device__ inline uint64_t fx_order_packed(uint32_t n, KeyFn key) {
  uint64_t T = 0;
  uint32_t B = 0, items = 0, growth = 0;
  for (uint32_t k = 0; k < n; ++k) {
    if (growth == 0) {
      const uint32_t nb = fx_buckets_for(max(items + 1, fx_cap(B) + 1));
      const uint64_t old = T;
      T = 0;
      for (uint32_t b = 0; b < B; ++b) {
        const uint32_t v = (uint32_t)(old >> (4 * b)) & 15u;
        if (v) T = fx_put(T, nb, key(v - 1), v);
      }
      B = nb;
      growth = fx_cap(nb) - items;
    }
    T = fx_put(T, B, key(k), k + 1);
    items++;
    growth--;
  }
  uint64_t out = 0;
  uint32_t m = 0;
  for (uint32_t b = 0; b < B; ++b) {
    const uint32_t v = (uint32_t)(T >> (4 * b)) & 15u;
    if (v) {
      out |= (uint64_t)(v - 1) << (4 * m);
      m++;
    }
  }
  return out;
}
__device__ __forceinline__ uint32_t nib(uint64_t x, uint32_t i) { return (uint32_t)(x >> (4 * i)) & 15u; }
__device__ __forceinline__ uint32_t byte_at(uint64_t x, uint32_t i) { return (uint32_t)(x >> (8 * i)) & 0xFFu; }

// --- per-read DWFA views ---
struct SideView {
  Gm<RState>* rs;    // [nmax]
  Gm<uint32_t>* wf;  // [nmax * wcap]
  Gm<uint8_t>* con;  // [lcap]
};

__device__ inline SideView side_view(Gm<uint8_t>* slot_base, uint32_t side, uint32_t nmax, uint32_t wcap,
                                     uint32_t lcap) {
  Gm<uint8_t>* b = slot_base + (uint64_t)side * side_bytes(nmax, wcap, lcap);
  SideView v;
  v.rs = (Gm<RState>*)b;
  v.wf = (Gm<uint32_t>*)(b + (uint64_t)nmax * sizeof(RState));
  v.con = b + align16((uint64_t)nmax * sizeof(RState) + (uint64_t)nmax * wcap * 4);
  return v;
}

// A 64-byte RState moves as four 16-byte accesses held in named registers
// (word 3 = nscmp | nf << 16 | flags << 24; words 4-7 = fi pairs; 8-15 = fd).
struct RRaw {
  uint4 a, b, c, d;
};
__device__ __forceinline__ RRaw rstate_load(const Gm<RState>* p) {
  const Gm<uint4>* q = (const Gm<uint4>*)p;
  return RRaw{q[0], q[1], q[2], q[3]};
}
#if defined(__HIP_DEVICE_COMPILE__) && !defined(WC_GLOBAL_STATE)
__device__ __forceinline__ RRaw rstate_load(const Sh<RState>* p) {
  const Sh<uint4>* q = (const Sh<uint4>*)p;
  return RRaw{q[0], q[1], q[2], q[3]};
}
#endif
__device__ __forceinline__ void rstate_store(Gm<RState>* p, const RRaw& s) {
  Gm<uint4>* q = (Gm<uint4>*)p;
  q[0] = s.a;
  q[1] = s.b;
  q[2] = s.c;
  q[3] = s.d;
}
#if defined(__HIP_DEVICE_COMPILE__) && !defined(WC_GLOBAL_STATE)
__device__ __forceinline__ void rstate_store(Sh<RState>* p, const RRaw& s) {
  Sh<uint4>* q = (Sh<uint4>*)p;
  q[0] = s.a;
  q[1] = s.b;
  q[2] = s.c;
  q[3] = s.d;
}
#endif
// A node's RStates through a generic (flat) pointer: the dual engine's
// in-place child lives in the LDS copy of the popped node (dual_hot), its
// clones in their HBM slots, and the same pass handles both
using RSg = RState*;
template <class P>
__device__ __forceinline__ RSg rs_generic(P p) {
  return (RSg)p;
}
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ RRaw rstate_load(const RState* p) {
  const uint4* q = (const uint4*)p;
  return RRaw{q[0], q[1], q[2], q[3]};
}
__device__ __forceinline__ void rstate_store(RState* p, const RRaw& s) {
  uint4* q = (uint4*)p;
  q[0] = s.a;
  q[1] = s.b;
  q[2] = s.c;
  q[3] = s.d;
}
#endif
__device__ __forceinline__ uint32_t rraw_e(const RRaw& s) { return s.a.x; }
__device__ __forceinline__ uint32_t rraw_flags(const RRaw& s) { return s.a.w >> 24; }

struct WaveCounters {
  uint32_t updates, w_out, compares, edinc, finalizes;
  uint32_t rowb;  // wavefront-row bytes read + written by updates (finalizes: read) that grow e
#ifdef WC_PHASE_PROF
  uint64_t tq[3];  // wave_heavy's register path: row load, increase loop, store + rebuild (cycles)
#endif
};

// The CU's vector L1 keeps its copy of a line across this workgroup's own
// byte stores to it: a wave that stored a consensus byte and read it back in
// its ED-increase loop got the old byte, even after waiting for the store
// (wave_dual.hip.hpp, a fault on a 4-wave problem). Code that stores
// consensus bytes which ED-increase loops then read waits for the stores
// (con_store_wait, in the storing waves) and, after whatever orders the
// readers behind them, drops the CU's L1 lines (l1_drop: buffer_inv sc1).
__device__ __forceinline__ void con_store_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void l1_drop() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent"); }

// ---- packed match runs (dynamic_wfa.rs:122-150) ----
// 8 bytes at p[pos..pos+8): two aligned 8-byte loads and a funnel shift.
// Reads start 16-byte aligned with 64 bytes of arena tail padding and the
// consensus rows are followed by more workspace, so the second word is always
// inside the allocation; bytes past a sequence's end are masked by the caller.
__device__ __forceinline__ uint64_t load8(const Gm<uint8_t>* p, uint32_t pos) {
  const Gm<uint64_t>* w = (const Gm<uint64_t>*)p + (pos >> 3);
  const uint32_t sh = (pos & 7u) * 8u;
  const uint64_t a = w[0], b = w[1];
  return sh ? (a >> sh) | (b << (64u - sh)) : a;
}
// 0x80 in every byte of v that is non-zero
__device__ __forceinline__ uint64_t nz_bytes(uint64_t v) {
  constexpr uint64_t lo7 = 0x7f7f7f7f7f7f7f7full;
  return (((v & lo7) + lo7) | v) & ~lo7;
}
// The extend loop of one diagonal from read position bo / consensus position
// oo, eight bytes per step: XOR of the packed bytes, the wildcard masked on the
// read side only (:138-140), ctz for the first mismatch. Returns how far d
// advances; `cmp` gets the compares the byte-at-a-time reference loop makes
// (one per matched byte, plus the failing one when the run stops on a
// mismatch rather than at a sequence end).
__device__ __forceinline__ uint32_t match_run(const Gm<uint8_t>* rd, uint32_t blen, const Gm<uint8_t>* con,
                                              uint32_t olen, uint32_t bo, uint32_t oo, int wc, uint32_t& cmp) {
  const uint64_t wcb = 0x0101010101010101ull * (uint64_t)(uint8_t)wc;
  uint32_t adv = 0;
  while (bo < blen && oo < olen) {
    const uint32_t rem = min(blen - bo, olen - oo);
    const uint64_t x = load8(rd, bo), y = load8(con, oo);
    uint64_t mm = nz_bytes(x ^ y);
    if (wc >= 0) mm &= nz_bytes(x ^ wcb);
    const uint32_t k = mm ? (uint32_t)__builtin_ctzll(mm) >> 3 : 8u;
    if (k >= rem) {  // everything up to the nearer sequence end matches
      adv += rem;
      cmp += rem;
      break;
    }
    if (k < 8) {  // mismatch at byte k
      adv += k;
      cmp += k + 1;
      break;
    }
    adv += 8;
    cmp += 8;
    bo += 8;
    oo += 8;
  }
  return adv;
}

// Full extend of every diagonal of `wf[0..W)` (dynamic_wfa.rs:109-153),
// lanes over diagonals. Returns (via refs) wave-reduced max_other - off and
// max_baseline. Counts byte compares as the reference loop would.
__device__ inline void wave_extend_all(Gm<uint32_t>* wf, uint32_t W, uint32_t e, uint32_t off, const Gm<uint8_t>* rd,
                                       uint32_t blen, const Gm<uint8_t>* con, uint32_t olen, int wc, uint32_t& maxo,
                                       uint32_t& maxb, uint32_t& cmp) {
  const int lane = lane_id();
  uint32_t mo = 0, mb = 0, c = 0;
  for (uint32_t base = 0; base < W; base += 64) {
    uint32_t i = base + lane;
    if (i < W) {
      const uint32_t d0 = wf[i];
      const uint32_t d = d0 + match_run(rd, blen, con, olen, d0 + e - i, d0 + off, wc, c);
      if (d != d0) wf[i] = d;
      mo = max(mo, d);
      mb = max(mb, d + e - i);
    }
  }
  maxo = wave_max_u32(mo);
  maxb = wave_max_u32(mb);
  cmp += c;
}

// ---- register-resident wavefronts ----
// The ED-increase loop (dynamic_wfa.rs:84-91 / :162-191) holds the row in
// registers, lane-strided (entry lane + 64 q in v[q]), for W <= 64 * kRegQ:
// one load and one store of the row per update instead of a round trip
// through memory per increase.
constexpr int kRegQ = 2;

// increase_edit_distance on the register row: W -> W + 2,
// new[j] = max(old[j] (j < W), old[j-1] + 1 (1 <= j <= W), old[j-2] + 1 (2 <= j <= W+1)).
__device__ __forceinline__ void regs_grow(uint32_t (&v)[kRegQ], uint32_t W) {
  const uint32_t lane = (uint32_t)lane_id();
  // descending q: v[q - 1] is still the old row when entry q is rebuilt.
  // Entry j - 1 is lane - 1 of v[q] (lane 0: lane 63 of v[q - 1]), entry
  // j - 2 is lane - 2 (lanes 0, 1: lanes 62, 63 of v[q - 1]): one wave
  // rotation of a per-lane selection of the two registers.
#pragma unroll
  for (int q = kRegQ - 1; q >= 0; --q) {
    const uint32_t j = lane + 64u * q;
    const uint32_t prev = q > 0 ? v[q > 0 ? q - 1 : 0] : 0u;
    const uint32_t m1 = wave_ror1(lane == 63 ? prev : v[q]);
    const uint32_t m2 = wave_ror1(wave_ror1(lane >= 62 ? prev : v[q]));
    uint32_t x = 0;
    if (j < W) x = v[q];
    if (j >= 1 && j <= W) x = max(x, m1 + 1);
    if (j >= 2 && j <= W + 1) x = max(x, m2 + 1);
    v[q] = x;
  }
}

// extend every diagonal of the register row (wave_extend_all semantics)
__device__ __forceinline__ void regs_extend(uint32_t (&v)[kRegQ], uint32_t W, uint32_t e, uint32_t off,
                                            const Gm<uint8_t>* rd, uint32_t blen, const Gm<uint8_t>* con,
                                            uint32_t olen, int wc, uint32_t& maxo, uint32_t& maxb, uint32_t& cmp) {
  const int lane = lane_id();
  uint32_t mo = 0, mb = 0;
#pragma unroll
  for (int q = 0; q < kRegQ; ++q) {
    const uint32_t i = (uint32_t)lane + 64u * q;
    if (i < W) {
      const uint32_t d = v[q] + match_run(rd, blen, con, olen, v[q] + e - i, v[q] + off, wc, cmp);
      v[q] = d;
      mo = max(mo, d);
      mb = max(mb, d + e - i);
    }
  }
  maxo = wave_max_u32(mo);
  maxb = wave_max_u32(mb);
}

__device__ __forceinline__ void regs_load(uint32_t (&v)[kRegQ], const Gm<uint32_t>* wf, uint32_t W) {
#pragma unroll
  for (int q = 0; q < kRegQ; ++q) {
    const uint32_t i = (uint32_t)lane_id() + 64u * q;
    v[q] = i < W ? wf[i] : 0u;
  }
}
__device__ __forceinline__ void regs_store(const uint32_t (&v)[kRegQ], Gm<uint32_t>* wf, uint32_t W) {
#pragma unroll
  for (int q = 0; q < kRegQ; ++q) {
    const uint32_t i = (uint32_t)lane_id() + 64u * q;
    if (i < W) wf[i] = v[q];
  }
}

// increase_edit_distance in place (dynamic_wfa.rs:162-183): W -> W+2.
// Chunks are processed from the top so a chunk never reads an entry that a
// previously processed chunk overwrote.
__device__ inline void wave_grow(Gm<uint32_t>* wf, uint32_t Wold) {
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
__device__ inline bool wave_push_read(Gm<uint32_t>* wf, uint32_t& e, uint32_t off, const Gm<uint8_t>* rd,
                                      uint32_t blen, const Gm<uint8_t>* con, uint32_t olen, uint8_t sym, int wc, bool early,
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
  const uint32_t w_in = W;
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
  if (W != w_in) cnt.rowb += 4 * (w_in + W);
  cnt.compares += wave_sum_u32(cmp);
  return true;
}

// General DWFALite::update (other may have grown by any amount):
// dynamic_wfa.rs:75-99 with a full extend first.
__device__ inline bool wave_update_general(Gm<uint32_t>* wf, uint32_t& e, uint32_t off, const Gm<uint8_t>* rd,
                                           uint32_t blen, const Gm<uint8_t>* con, uint32_t olen, int wc, bool early, uint32_t wcap,
                                           WaveCounters& cnt, uint32_t& mo, uint32_t& mb) {
  uint32_t W = 2 * e + 1, cmp = 0;
  const uint32_t w_in = W;
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
  if (W != w_in) cnt.rowb += 4 * (w_in + W);
  cnt.compares += wave_sum_u32(cmp);
  return true;
}

// DWFALite::finalize (dynamic_wfa.rs:201-210) on a copy of the wavefront (in
// registers while it fits, else the scratch row); the node itself is
// untouched (the reference finalizes a clone).
__device__ inline bool wave_finalize_read(const Gm<uint32_t>* wf, uint32_t e, uint32_t off, const Gm<uint8_t>* rd,
                                          uint32_t blen, const Gm<uint8_t>* con, uint32_t olen, int wc,
                                          Gm<uint32_t>* scratch,
                                          uint32_t wcap, uint32_t& e_out, WaveCounters& cnt) {
  uint32_t W = 2 * e + 1;
  const uint32_t w_in = W;
  uint32_t v[kRegQ];
  regs_load(v, wf, W);
  uint32_t mb = 0;
#pragma unroll
  for (int q = 0; q < kRegQ; ++q) {
    const uint32_t i = (uint32_t)lane_id() + 64u * q;
    if (i < W) mb = max(mb, v[q] + e - i);
  }
  for (uint32_t i = 64u * kRegQ + lane_id(); i < W; i += 64) mb = max(mb, wf[i] + e - i);
  mb = wave_max_u32(mb);
  uint32_t cmp = 0;
  cnt.finalizes++;
  bool regs = true;
  if (W > 64u * kRegQ) {
    for (uint32_t i = lane_id(); i < W; i += 64) scratch[i] = wf[i];
    regs = false;
  }
  while (mb < blen) {
    if (W + 2 > wcap) return false;
    if (regs && W + 2 > 64u * kRegQ) {
      regs_store(v, scratch, W);
      regs = false;
    }
    uint32_t mo;
    if (regs) {
      regs_grow(v, W);
      W += 2;
      e += 1;
      regs_extend(v, W, e, off, rd, blen, con, olen, wc, mo, mb, cmp);
    } else {
      __builtin_amdgcn_wave_barrier();
      wave_grow(scratch, W);
      W += 2;
      e += 1;
      wave_extend_all(scratch, W, e, off, rd, blen, con, olen, wc, mo, mb, cmp);
    }
    cnt.edinc++;
  }
  if (W != w_in) cnt.rowb += 4 * w_in;
  cnt.compares += wave_sum_u32(cmp);
  e_out = e;
  return true;
}

// Tip nomination of one read (dynamic_wfa.rs:241-255) plus reached_baseline_end
// (:232-234), one wave over the full wavefront. Distinct symbols are found in
// first-appearance order (ascending diagonal), then permuted into FxHashMap
// iteration order. Keys/counts are wave-uniform packed registers. Returns
// false when more than kKmax distinct symbols sit at the tips.
// (ins: when given, lane 0 also stores the symbols in insertion order, the
// order of the reference's entry().or_insert() calls, byte k = k-th key)
__device__ inline bool wave_analyze_read(const Gm<uint32_t>* wf, uint32_t e, uint32_t off, const Gm<uint8_t>* rd,
                                         uint32_t blen, uint32_t olen, Sh<RInfo>* out, uint64_t* ins = nullptr) {
  const int lane = lane_id();
  const uint32_t W = 2 * e + 1;
  uint64_t keys = 0, cnt_lo = 0, cnt_hi = 0;  // 8 keys (bytes), 8 x 16-bit counts
  uint32_t nk = 0;
  uint32_t mb = 0;
  bool ok = true;
  for (uint32_t base = 0; base < W; base += 64) {
    const uint32_t i = base + lane;
    bool tip = false;
    uint32_t s = 0;
    if (i < W) {
      const uint32_t d = wf[i];
      const uint32_t bo = d + e - i;
      mb = max(mb, bo);
      if (d + off == olen && bo < blen) {
        tip = true;
        s = rd[bo];
      }
    }
    uint64_t m = ballot(tip);
    while (m) {
      const int first = __ffsll((unsigned long long)m) - 1;
      const uint32_t sym = (uint32_t)__shfl((int)s, first, 64);
      const uint64_t ms = ballot(tip && s == sym);
      uint32_t k = 0;
      while (k < nk && byte_at(keys, k) != sym) ++k;
      if (k == nk) {
        if (nk == (uint32_t)kKmax) {
          ok = false;
          break;
        }
        keys |= (uint64_t)sym << (8 * nk);
        nk++;
      }
      const uint64_t add = (uint64_t)__popcll((unsigned long long)ms);
      if (k < 4) cnt_lo += add << (16 * k);
      else cnt_hi += add << (16 * (k - 4));
      m &= ~ms;
    }
  }
  mb = wave_max_u32(mb);
  if (lane == 0) {
    const uint64_t ord = fx_order_packed(nk, [&](uint32_t j) { return byte_at(keys, j); });
    uint32_t split = 0;
    for (uint32_t k = 0; k < nk; ++k) {
      const uint32_t j = nib(ord, k);
      const uint32_t c = (uint32_t)((j < 4 ? cnt_lo >> (16 * j) : cnt_hi >> (16 * (j - 4))) & 0xFFFFu);
      out->sym[k] = (uint8_t)byte_at(keys, j);
      out->occ[k] = (uint16_t)c;
      split += c;
    }
    if (ins) *ins = keys;
    out->n = (uint8_t)nk;
    out->split = (uint16_t)split;
    out->end = (mb == blen);
    out->e = e;
  }
  return ok;
}

// =====================================================================
// Frontier-cache (RState) operations. A push of one symbol only moves
// frontier diagonals, so the common case is one thread per read touching
// its 64-byte RState plus a few read bytes; the full wavefront is revisited
// (one wave, lanes over diagonals) only when the edit distance must grow.
// =====================================================================

// Per-read frontier in registers: entries k < kF with a keep mask (order =
// ascending diagonal index). Only static indices are used on it.
struct Front {
  uint32_t e, off, maxb, nscmp, mask;
  uint32_t fi[kF], fd[kF];
};
__device__ __forceinline__ void front_load(const RRaw& s, Front& f) {
  f.e = s.a.x;
  f.off = s.a.y;
  f.maxb = s.a.z;
  f.nscmp = s.a.w & 0xFFFFu;
  f.mask = (1u << ((s.a.w >> 16) & 0xFFu)) - 1u;
  f.fi[0] = s.b.x & 0xFFFFu;
  f.fi[1] = s.b.x >> 16;
  f.fi[2] = s.b.y & 0xFFFFu;
  f.fi[3] = s.b.y >> 16;
  f.fi[4] = s.b.z & 0xFFFFu;
  f.fi[5] = s.b.z >> 16;
  f.fi[6] = s.b.w & 0xFFFFu;
  f.fi[7] = s.b.w >> 16;
  f.fd[0] = s.c.x;
  f.fd[1] = s.c.y;
  f.fd[2] = s.c.z;
  f.fd[3] = s.c.w;
  f.fd[4] = s.d.x;
  f.fd[5] = s.d.y;
  f.fd[6] = s.d.z;
  f.fd[7] = s.d.w;
}
// write the compacted frontier back (memory stores at computed positions)
template <class P>
__device__ __forceinline__ void front_store(P p, const Front& f) {
  uint32_t n = 0;
#pragma unroll
  for (int k = 0; k < kF; ++k) {
    if (f.mask & (1u << k)) {
      p->fi[n] = (uint16_t)f.fi[k];
      p->fd[n] = f.fd[k];
      n++;
    }
  }
  p->e = f.e;
  p->off = f.off;
  p->maxb = f.maxb;
  p->nscmp = (uint16_t)f.nscmp;
  p->nf = (uint8_t)n;
  p->flags = 0;
}

// Nomination + end flag of one read from its frontier (thread-level),
// dynamic_wfa.rs:232-234 and :241-255: the distinct tip symbols in the
// per-read FxHashMap iteration order with their occurrence counts.
struct Nom {
  uint64_t sym;  // byte k = k-th symbol in iteration order
  uint64_t occ;  // byte k = its occurrences (<= kF tips)
  uint32_t n, split, end;
};
// read byte sources for the thread-level steps
struct GlobalBytes {
  const Gm<uint8_t>* rd;
  __device__ __forceinline__ uint32_t operator()(uint32_t p) const { return rd[p]; }
};
// a 64-byte window of the read staged in LDS ([wb, wb+64)), global beyond it
struct WindowBytes {
  const Gm<uint8_t>* rd;
  const Sh<uint8_t>* win;
  uint32_t wb;
  __device__ __forceinline__ uint32_t operator()(uint32_t p) const {
    const uint32_t q = p - wb;
    return q < 64u ? (uint32_t)win[q] : (uint32_t)rd[p];
  }
};

template <class RB>
__device__ inline Nom thread_nominate(const Front& f, RB rd, uint32_t blen, uint32_t len) {
  uint32_t mb = f.maxb;
  uint32_t tipsym[kF];
  // live slots sit below 32 - clz(mask): the slots past it are skipped (for
  // the whole wave when every lane's frontier is that short)
  const uint32_t hi = f.mask ? 32u - (uint32_t)__builtin_clz(f.mask) : 0u;
#pragma unroll
  for (int k = 0; k < kF; ++k) {
    tipsym[k] = 0x100;
    if (kSlotBound && (uint32_t)k >= hi) continue;
    if (f.mask & (1u << k)) {
      const uint32_t bo = f.fd[k] + f.e - f.fi[k];
      mb = max(mb, bo);
      if (f.fd[k] + f.off == len && bo < blen) tipsym[k] = rd(bo);
    }
  }
  uint64_t keys = 0;
  uint32_t cnts = 0, nk = 0;  // counts: 4-bit nibbles (<= kF tips)
#pragma unroll
  for (int k = 0; k < kF; ++k) {
    if (kSlotBound && (uint32_t)k >= hi) break;
    const uint32_t s = tipsym[k];
    if (s == 0x100) continue;
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
// RInfo from a nomination: two 16-byte stores
__device__ __forceinline__ void rinfo_store(Sh<RInfo>* out, const Nom& o, uint32_t e) {
  static_assert(sizeof(RInfo) == 32, "RInfo layout");
  const uint32_t o16[4] = {
      (uint32_t)(o.occ & 0xFF) | (uint32_t)((o.occ >> 8) & 0xFF) << 16,
      (uint32_t)((o.occ >> 16) & 0xFF) | (uint32_t)((o.occ >> 24) & 0xFF) << 16,
      (uint32_t)((o.occ >> 32) & 0xFF) | (uint32_t)((o.occ >> 40) & 0xFF) << 16,
      (uint32_t)((o.occ >> 48) & 0xFF) | (uint32_t)((o.occ >> 56) & 0xFF) << 16};
  Sh<uint4>* q = (Sh<uint4>*)out;
  q[0] = make_uint4(o.n | (o.end << 8) | (o.split << 16), (uint32_t)o.sym, (uint32_t)(o.sym >> 32), o16[0]);
  q[1] = make_uint4(o16[1], o16[2], o16[3], e);
}
__device__ inline void thread_analyze(const Front& f, const Gm<uint8_t>* rd, uint32_t blen, uint32_t len,
                                      Sh<RInfo>* out, bool& multi) {
  const Nom o = thread_nominate(f, GlobalBytes{rd}, blen, len);
  rinfo_store(out, o, f.e);
  multi = o.n > 1;
}

// The extend step of DWFALite::update for one appended symbol on the frontier
// (thread-level). Tips (d + off == old length) compare once and either advance
// by one or become stuck; everything else is unchanged. Returns true when the
// read needs the wave path: the ED-increase loop (dynamic_wfa.rs:84-91).
// `cmp` receives the compares the reference extend makes.
// kLazy (linear-chain walk): the row is not written when a tip advances, only
// when a diagonal leaves the frontier; front_flush writes the final frontier.
// Between the two, RState (not the row) is authoritative for frontier
// diagonals, so the hot loop issues no global stores.
// thread_push in two halves, so that several reads' (or sides') byte loads
// can be in flight together: the tip bytes, then the update on them
template <class RB>
__device__ __forceinline__ void thread_tips(const Front& f, RB rd, uint32_t blen, uint32_t old_len,
                                            uint32_t (&x)[kF]) {
  const uint32_t hi = f.mask ? 32u - (uint32_t)__builtin_clz(f.mask) : 0u;  // live slots: below hi
#pragma unroll
  for (int k = 0; k < kF; ++k) {
    x[k] = 0x100;
    if (kSlotBound && (uint32_t)k >= hi) continue;
    if (f.mask & (1u << k)) {
      const uint32_t bo = f.fd[k] + f.e - f.fi[k];
      if (f.fd[k] + f.off == old_len && bo < blen) x[k] = rd(bo);
    }
  }
}
template <bool kLazy = false>
__device__ __forceinline__ bool thread_apply(Front& f, const uint32_t (&x)[kF], uint32_t blen, uint32_t old_len,
                                             uint8_t sym, int wc, bool early, Gm<uint32_t>* wf_row, uint32_t& cmp) {
  const uint32_t hi = f.mask ? 32u - (uint32_t)__builtin_clz(f.mask) : 0u;
  uint32_t c = f.nscmp;
  uint32_t mb = 0;
#pragma unroll
  for (int k = 0; k < kF; ++k) {
    if (kSlotBound && (uint32_t)k >= hi) break;
    if (!(f.mask & (1u << k))) continue;
    const uint32_t d = f.fd[k];
    const uint32_t bo = d + f.e - f.fi[k];
    if (d + f.off == old_len) {
      if (bo < blen) {
        c++;
        if (x[k] == sym || (wc >= 0 && x[k] == (uint32_t)(uint8_t)wc)) {
          f.fd[k] = d + 1;
          if (!kLazy) wf_row[f.fi[k]] = d + 1;
          mb = max(mb, bo + 1);
          continue;
        }
        f.nscmp++;  // stuck on a mismatch: compared (and failing) on every later push
      }
      if (kLazy) wf_row[f.fi[k]] = d;
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
template <bool kLazy = false, class RB>
__device__ inline bool thread_push(Front& f, RB rd, uint32_t blen, uint32_t old_len, uint8_t sym, int wc,
                                   bool early, Gm<uint32_t>* wf_row, uint32_t& cmp) {
  uint32_t x[kF];
  thread_tips(f, rd, blen, old_len, x);
  return thread_apply<kLazy>(f, x, blen, old_len, sym, wc, early, wf_row, cmp);
}

// write the frontier diagonals back into the wavefront row (end of a lazy walk)
__device__ __forceinline__ void front_flush(const Front& f, Gm<uint32_t>* wf_row) {
#pragma unroll
  for (int k = 0; k < kF; ++k)
    if (f.mask & (1u << k)) wf_row[f.fi[k]] = f.fd[k];
}

// Rebuild an RState from the authoritative wavefront (one wave).
template <class P>
__device__ inline void wave_rebuild(const Gm<uint32_t>* wf, uint32_t e, uint32_t off, uint32_t blen, uint32_t len,
                                    P out) {
  const int lane = lane_id();
  const uint32_t W = 2 * e + 1;
  uint32_t nf = 0, mb = 0, nsc = 0;
  for (uint32_t base = 0; base < W; base += 64) {
    const uint32_t i = base + lane;
    const bool valid = i < W;
    const uint32_t d = valid ? wf[i] : 0;
    const uint32_t bo = d + e - i;
    const bool inF = valid && d + off >= len;
    const uint64_t m = ballot(inF);
    const uint32_t pos = nf + (uint32_t)__popcll((unsigned long long)(m & ((1ull << lane) - 1ull)));
    if (inF && pos < (uint32_t)kF) {
      out->fi[pos] = (uint16_t)i;
      out->fd[pos] = d;
    }
    nf += (uint32_t)__popcll((unsigned long long)m);
    if (valid && !inF) {
      mb = max(mb, bo);
      nsc += bo < blen;
    }
  }
  mb = wave_max_u32(mb);
  nsc = wave_sum_u32(nsc);
  if (lane == 0) {
    out->e = e;
    out->off = off;
    out->maxb = mb;
    out->nscmp = (uint16_t)min(nsc, 65535u);
    out->nf = (uint8_t)min(nf, (uint32_t)kF);
    out->flags = (nf > (uint32_t)kF || nsc > 65535u) ? kWide : 0;
  }
}

// RState from a register row (wave_rebuild semantics)
template <class P>
__device__ inline void regs_rebuild(const uint32_t (&v)[kRegQ], uint32_t e, uint32_t off, uint32_t blen, uint32_t len,
                                    P out) {
  const int lane = lane_id();
  const uint32_t W = 2 * e + 1;
  uint32_t nf = 0, mb = 0, nsc = 0;
#pragma unroll
  for (int q = 0; q < kRegQ; ++q) {
    const uint32_t i = (uint32_t)lane + 64u * q;
    const bool valid = i < W;
    const uint32_t d = v[q];
    const uint32_t bo = d + e - i;
    const bool inF = valid && d + off >= len;
    const uint64_t m = ballot(inF);
    const uint32_t pos = nf + (uint32_t)__popcll((unsigned long long)(m & ((1ull << lane) - 1ull)));
    if (inF && pos < (uint32_t)kF) {
      out->fi[pos] = (uint16_t)i;
      out->fd[pos] = d;
    }
    nf += (uint32_t)__popcll((unsigned long long)m);
    if (valid && !inF) {
      mb = max(mb, bo);
      nsc += bo < blen;
    }
  }
  mb = wave_max_u32(mb);
  nsc = wave_sum_u32(nsc);
  if (lane == 0) {
    out->e = e;
    out->off = off;
    out->maxb = mb;
    out->nscmp = (uint16_t)min(nsc, 65535u);
    out->nf = (uint8_t)min(nf, (uint32_t)kF);
    out->flags = (nf > (uint32_t)kF || nsc > 65535u) ? kWide : 0;
  }
}

// The wave part of a push for one read whose thread step returned true:
// full-scan push for a wide frontier, otherwise the ED-increase loop from the
// post-extend wavefront (in registers while W <= 64 * kRegQ); then rebuild the
// RState. Returns false on wavefront capacity overflow.
template <class P>
__device__ inline bool wave_heavy(P rsp, Gm<uint32_t>* wf, const Gm<uint8_t>* rd, uint32_t blen,
                                  const Gm<uint8_t>* con, uint32_t olen, uint8_t sym, int wc, bool early, uint32_t wcap, WaveCounters& cnt,
                                  uint32_t& e_out, Gm<uint32_t>* bak = nullptr) {
  // bak: a copy of the row as it is on entry goes there (the linear chain's
  // rollback copy), from the registers the row is loaded into anyway
  const uint32_t flags = rsp->flags;
  uint32_t e = rsp->e;
  const uint32_t off = rsp->off;
  if (bak && ((flags & kWide) || 2 * e + 3 > 64u * kRegQ)) {
    for (uint32_t i = (uint32_t)lane_id(); i < 2 * e + 1; i += 64) bak[i] = wf[i];
    bak = nullptr;
    __builtin_amdgcn_wave_barrier();
  }
  if (flags & kWide) {
    if (!wave_push_read(wf, e, off, rd, blen, con, olen, sym, wc, early, wcap, cnt)) return false;
    __builtin_amdgcn_wave_barrier();
    wave_rebuild(wf, e, off, blen, olen, rsp);
    e_out = e;
    return true;
  }
  uint32_t W = 2 * e + 1, mo, mb, cmp = 0;
  const uint32_t w_in = W;
  uint32_t v[kRegQ];
  bool regs = W + 2 <= 64u * kRegQ;
#ifdef WC_PHASE_PROF
  const uint64_t t_a = __builtin_amdgcn_s_memtime();
#endif
  if (regs) regs_load(v, wf, W);
#ifdef WC_PHASE_PROF
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const uint64_t t_b = __builtin_amdgcn_s_memtime();
#endif
  if (bak) regs_store(v, bak, W);
  do {
    if (W + 2 > wcap) return false;
    if (regs && W + 2 > 64u * kRegQ) {
      regs_store(v, wf, W);
      regs = false;
      __builtin_amdgcn_wave_barrier();
    }
    if (regs) {
      regs_grow(v, W);
      W += 2;
      e += 1;
      regs_extend(v, W, e, off, rd, blen, con, olen, wc, mo, mb, cmp);
    } else {
      wave_grow(wf, W);
      W += 2;
      e += 1;
      wave_extend_all(wf, W, e, off, rd, blen, con, olen, wc, mo, mb, cmp);
    }
    cnt.edinc++;
  } while (mo + off < olen && !(early && mb == blen));
#ifdef WC_PHASE_PROF
  const uint64_t t_c = __builtin_amdgcn_s_memtime();
#endif
  cnt.updates++;
  cnt.w_out += W;
  cnt.rowb += 4 * (w_in + W);
  cnt.compares += wave_sum_u32(cmp);
  if (regs) {
    regs_store(v, wf, W);
    regs_rebuild(v, e, off, blen, olen, rsp);
  } else {
    __builtin_amdgcn_wave_barrier();
    wave_rebuild(wf, e, off, blen, olen, rsp);
  }
#ifdef WC_PHASE_PROF
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  cnt.tq[0] += t_b - t_a;
  cnt.tq[1] += t_c - t_b;
  cnt.tq[2] += __builtin_amdgcn_s_memtime() - t_c;
#endif
  e_out = e;
  return true;
}

// ---- the ED-increase loop for four (eight) reads per wave, 16-lane (8-lane) groups ----
// A push's ED-increase work (dynamic_wfa.rs:84-91) is a short chain of
// dependent memory round trips per read (RState, row, the extend's read and
// consensus bytes), so one read per wave leaves the wave waiting on one chain
// at a time. Here each G-lane group of a wave runs its own read's loop, the
// row held lane-strided (entry G q + gl in v[q]) for W <= G kQ16, so 64 / G
// reads' chains overlap. Same arithmetic as wave_heavy's register path.
constexpr int kQ16 = 8;
constexpr uint32_t kRow16 = 16u * kQ16;

template <int G>
__device__ __forceinline__ uint32_t grp_max(uint32_t v) {
  if constexpr (G == 16) return row_max_u32(v);
  v = max(v, dpp_u32<0xb1>(v));  // quad_perm [1,0,3,2]
  v = max(v, dpp_u32<0x4e>(v));  // quad_perm [2,3,0,1]
  return max(v, dpp_u32<0x141>(v));  // row_half_mirror (within 8 lanes)
}
template <int G>
__device__ __forceinline__ uint32_t grp_sum(uint32_t v) {
  if constexpr (G == 16) return row_sum_u32(v);
  v += dpp_u32<0xb1>(v);
  v += dpp_u32<0x4e>(v);
  return v + dpp_u32<0x141>(v);
}

// Outcome per group: kG_DONE (RState rebuilt), kG_WCAP (wavefront capacity),
// kG_MEM (the row outgrew kRow16: stored back with e = `e_out`, the loop goes
// on in wave_edinc_mem). Counters are per lane (wave-sum them).
constexpr uint32_t kG_DONE = 0, kG_WCAP = 1, kG_MEM = 2, kG_RUN = 3;
struct GroupCnt {
  uint32_t edinc, updates, w_out, cmp, rowb;
};
// group_edinc's result, by value (registers): outcome, final e, per-lane counters
struct GroupOut {
  uint32_t st, e, edinc, updates, w_out, cmp, rowb;
};
// (P: the RState pointer, an HBM slot or, dual_hot, a generic pointer that
// may point into the LDS copy of the popped node)
template <int G, class P>
__device__ __noinline__ GroupOut group_edinc(bool act, P rsp, Gm<uint32_t>* wf, const Gm<uint8_t>* rd,
                                             uint32_t blen, const Gm<uint8_t>* con, uint32_t olen, int wc,
                                             bool early, uint32_t wcap) {
  static_assert(G == 16 || G == 8, "group width");
  constexpr uint32_t kRowG = (uint32_t)G * kQ16;
  GroupOut go_ = {kG_DONE, 0, 0, 0, 0, 0, 0};
  const int lane = lane_id();
  const uint32_t gl = (uint32_t)lane & (G - 1u), gb = (uint32_t)lane & ~(G - 1u);
  uint32_t e = 0, off = 0;
  if (act) {
    e = rsp->e;
    off = rsp->off;
  }
  uint32_t W = 2 * e + 1;
  const uint32_t w_in = W;
  // wave-uniform bound on every group's row length: entry blocks q with
  // 16 q >= wlim are skipped (scalar branches) instead of predicated
#ifdef WC_NO_WLIM
  uint32_t wlim = 1000000u;
#else
  uint32_t wlim = wave_max_u32(act ? W : 0u);
#endif
  uint32_t v[kQ16];
#pragma unroll
  for (int q = 0; q < kQ16; ++q) {
    const uint32_t j = (uint32_t)G * q + gl;
    v[q] = 0u;
    if ((uint32_t)G * q < wlim && act && j < W) v[q] = wf[j];
  }
  uint32_t st = act ? kG_RUN : kG_DONE;
  uint32_t mb = 0, cmp = 0;
  while (ballot(st == kG_RUN)) {
    if (st == kG_RUN && W + 2 > wcap) st = kG_WCAP;
    else if (st == kG_RUN && W + 2 > kRowG) st = kG_MEM;
    const bool go = st == kG_RUN;  // group-uniform
    wlim += 2;
    // increase_edit_distance: W -> W + 2 (lane moves run on every lane).
    // Descending q keeps v[q - 1] old; entries j - 1 and j - 2 are row
    // rotations of per-lane selections of v[q] and v[q - 1] (row_ror).
#pragma unroll
    for (int q = kQ16 - 1; q >= 0; --q) {
      if ((uint32_t)G * q >= wlim) continue;
      const uint32_t j = (uint32_t)G * q + gl;
      const uint32_t prev = q > 0 ? v[q > 0 ? q - 1 : 0] : 0u;
      uint32_t m1, m2;
      if constexpr (G == 16) {
        m1 = row_ror1(gl == 15 ? prev : v[q]);
        m2 = row_ror2(gl >= 14 ? prev : v[q]);
      } else {
        // two groups per 16-lane row: a group's first lanes take their
        // group's last lanes of the previous block (row_ror 9 / 10)
        const uint32_t p1 = dpp_u32<0x129>(prev), p2 = dpp_u32<0x12a>(prev);
        const uint32_t r1 = row_ror1(v[q]), r2 = row_ror2(v[q]);
        m1 = gl == 0 ? p1 : r1;
        m2 = gl <= 1 ? p2 : r2;
      }
      uint32_t x = 0;
      if (j < W) x = v[q];
      if (j >= 1 && j <= W) x = max(x, m1 + 1);
      if (j >= 2 && j <= W + 1) x = max(x, m2 + 1);
      if (go) v[q] = x;
    }
    if (go) {
      W += 2;
      e += 1;
      go_.edinc += gl == 0;
    }
    // extend every diagonal: the first 8-byte step of every entry is issued
    // before any is used; runs that go on past it finish in match_run
    const uint64_t wcb = 0x0101010101010101ull * (uint64_t)(uint8_t)wc;
    uint64_t xa[kQ16], ya[kQ16];
#pragma unroll
    for (int q = 0; q < kQ16; ++q) {
      const uint32_t j = (uint32_t)G * q + gl;
      const uint32_t bo = v[q] + e - j, oo = v[q] + off;
      xa[q] = ya[q] = 0;
      if ((uint32_t)G * q >= wlim) continue;
      if (go && j < W && bo < blen && oo < olen) {
        xa[q] = load8(rd, bo);
        ya[q] = load8(con, oo);
      }
    }
    uint32_t lmo = 0, lmb = 0;
#pragma unroll
    for (int q = 0; q < kQ16; ++q) {
      const uint32_t j = (uint32_t)G * q + gl;
      if ((uint32_t)G * q >= wlim) continue;
      if (!(go && j < W)) continue;
      uint32_t d = v[q];
      const uint32_t bo = d + e - j, oo = d + off;
      if (bo < blen && oo < olen) {
        const uint32_t rem = min(blen - bo, olen - oo);
        uint64_t mm = nz_bytes(xa[q] ^ ya[q]);
        if (wc >= 0) mm &= nz_bytes(xa[q] ^ wcb);
        const uint32_t k = mm ? (uint32_t)__builtin_ctzll(mm) >> 3 : 8u;
        if (k >= rem) {
          d += rem;
          cmp += rem;
        } else if (k < 8) {
          d += k;
          cmp += k + 1;
        } else {
          cmp += 8;
          d += 8 + match_run(rd, blen, con, olen, bo + 8, oo + 8, wc, cmp);
        }
      }
      v[q] = d;
      lmo = max(lmo, d);
      lmb = max(lmb, d + e - j);
    }
    lmo = grp_max<G>(lmo);
    lmb = grp_max<G>(lmb);
    if (go) {
      mb = lmb;
      if (!(lmo + off < olen && !(early && lmb == blen))) st = kG_DONE;
    }
  }
  go_.cmp = cmp;
  go_.e = e;
  go_.st = st;
  if (!act || st == kG_WCAP) return go_;
  // the row back to memory
#pragma unroll
  for (int q = 0; q < kQ16; ++q) {
    const uint32_t j = (uint32_t)G * q + gl;
    if ((uint32_t)G * q < wlim && j < W) wf[j] = v[q];
  }
  // row traffic: the load now; the store when the update ends here (a row
  // that outgrew the group is stored by wave_edinc_mem)
  go_.rowb = gl == 0 ? 4 * (w_in + (st == kG_MEM ? 0u : W)) : 0u;
  if (st == kG_MEM) return go_;
  go_.updates = gl == 0;
  go_.w_out = gl == 0 ? W : 0u;
  // RState from the register row (regs_rebuild semantics, group-wide)
  uint32_t nf = 0, mbx = 0, nsc = 0;
#pragma unroll
  for (int q = 0; q < kQ16; ++q) {
    if ((uint32_t)G * q >= wlim) continue;
    const uint32_t j = (uint32_t)G * q + gl;
    const bool valid = j < W;
    const uint32_t d = v[q];
    const uint32_t bo = d + e - j;
    const bool inF = valid && d + off >= olen;
    const uint32_t m = (uint32_t)(ballot(inF) >> gb) & ((1u << G) - 1u);
    const uint32_t pos = nf + (uint32_t)__popc(m & ((1u << gl) - 1u));
    if (inF && pos < (uint32_t)kF) {
      rsp->fi[pos] = (uint16_t)j;
      rsp->fd[pos] = d;
    }
    nf += (uint32_t)__popc(m);
    if (valid && !inF) {
      mbx = max(mbx, bo);
      nsc += bo < blen;
    }
  }
  (void)mb;
  mbx = grp_max<G>(mbx);
  nsc = grp_sum<G>(nsc);
  if (gl == 0) {
    rsp->e = e;
    rsp->maxb = mbx;
    rsp->nscmp = (uint16_t)min(nsc, 65535u);
    rsp->nf = (uint8_t)min(nf, (uint32_t)kF);
    rsp->flags = (nf > (uint32_t)kF || nsc > 65535u) ? kWide : 0;
  }
  go_.st = kG_DONE;
  return go_;
}

// Continue an ED-increase loop whose row (W = 2 e + 1 entries, post-extend, not
// yet done) is in memory: one wave, lanes over diagonals (wave_heavy's memory
// path). Returns false on wavefront capacity overflow.
template <class P>
__device__ inline bool wave_edinc_mem(P rsp, Gm<uint32_t>* wf, uint32_t e, const Gm<uint8_t>* rd, uint32_t blen,
                                      const Gm<uint8_t>* con, uint32_t olen, int wc, bool early, uint32_t wcap,
                                      WaveCounters& cnt, uint32_t& e_out) {
  const uint32_t off = rsp->off;
  uint32_t W = 2 * e + 1, mo, mb, cmp = 0;
  do {
    if (W + 2 > wcap) return false;
    wave_grow(wf, W);
    W += 2;
    e += 1;
    wave_extend_all(wf, W, e, off, rd, blen, con, olen, wc, mo, mb, cmp);
    cnt.edinc++;
  } while (mo + off < olen && !(early && mb == blen));
  cnt.updates++;
  cnt.w_out += W;
  cnt.rowb += 4 * W;  // the final store (group_edinc counted the first load)
  cnt.compares += wave_sum_u32(cmp);
  __builtin_amdgcn_wave_barrier();
  wave_rebuild(wf, e, off, blen, olen, rsp);
  e_out = e;
  return true;
}

// ---- offset activation (consensus.rs:413-448, dual_consensus.rs:866-906) ----
// wfa_ed_config(v1, v2, require_both_end = false, wildcard)
// (sequence_alignment.rs:36-87) for this lane's own (v1, v2): the same
// furthest-reaching (i, j) pairs, max-merged lexicographically (packed as
// i << 32 | j), and the same boundary rules. Each lane keeps its two pair
// arrays in the wave's scratch, lane-interleaved (entry k of lane l at
// k * 64 + l). Returns the edit count, or `cap` as soon as it reaches `cap`.
// `m` bounds the arrays (entries); edits <= |v2| always, so m >= 2|v2| + 5
// never truncates an uncapped run.
constexpr uint32_t kEdOverflow = 0xFFFFFFFEu;
__device__ inline uint32_t lane_wfa_ed(const Gm<uint8_t>* v1, uint32_t l1, const Gm<uint8_t>* v2, uint32_t l2, int wc,
                                       uint32_t cap, uint32_t m, Gm<uint64_t>* A, Gm<uint64_t>* B) {
  const int lane = lane_id();
  auto wcm = [&](uint8_t a) { return wc >= 0 && a == (uint8_t)wc; };
  Gm<uint64_t>* cur = A;
  Gm<uint64_t>* nxt = B;
  cur[lane] = 0;
  for (uint32_t k = 0; k < 3; ++k) nxt[k * 64 + lane] = 0;
  uint32_t edits = 0;
  for (;;) {
    const uint32_t ncur = 1 + 2 * edits;
    for (uint32_t k = 0; k < ncur; ++k) {
      const uint64_t pr = cur[k * 64 + lane];
      uint32_t i = (uint32_t)(pr >> 32), j = (uint32_t)pr;
      while (i < l1 && j < l2) {
        const uint8_t a = v1[i], b = v2[j];
        if (!(a == b || wcm(a) || wcm(b))) break;
        ++i;
        ++j;
      }
      if (j == l2) return edits;  // (i == l1 || !require_both_end) && j == l2
      const uint64_t ij = (uint64_t)i << 32 | j;
      uint64_t n0, n1, n2;
      if (i == l1) {
        n0 = ij;
        n1 = ij + 1;
        n2 = ij + 1;
      } else {
        n0 = ij + (1ull << 32);
        n1 = ij + (1ull << 32) + 1;
        n2 = ij + 1;
      }
      Gm<uint64_t>* q = nxt + (uint64_t)k * 64 + lane;
      q[0] = max(q[0], n0);
      q[64] = max(q[64], n1);
      q[128] = max(q[128], n2);
    }
    edits++;
    if (edits >= cap) return cap;
    if (3 + 2 * edits > m) return kEdOverflow;  // scratch too small (reported, never truncated)
    Gm<uint64_t>* t = cur;
    cur = nxt;
    nxt = t;
    for (uint32_t k = 0; k < 3 + 2 * edits; ++k) nxt[k * 64 + lane] = 0;
  }
}

// The best start offset of a read activated against con[0..clen)
// (consensus.rs:418-437): the middle of the window is the default, replaced by
// the first p in [start, end) whose prefix edit distance is strictly smaller
// than the best so far — i.e. the smallest p attaining min_p ed(p) if that is
// below ed(best0). Lanes take candidates in parallel; a first pass caps every
// edit count at kCap (exact whenever the winner is below the cap), and only an
// undecided window reruns uncapped. Wave-uniform result.
__device__ inline uint32_t wave_pick_offset(const Gm<uint8_t>* con, uint32_t clen, const Gm<uint8_t>* rd, uint32_t ocl,
                                            uint32_t window, int wc, Gm<uint64_t>* scr, uint32_t m) {
  const int lane = lane_id();
  auto sat = [](uint32_t a, uint32_t b) { return a > b ? a - b : 0u; };
  const uint32_t start = sat(clen, window + ocl), end = sat(clen, ocl);
  const uint32_t best0 = sat(clen, ocl + window / 2);
  Gm<uint64_t>* A = scr;
  Gm<uint64_t>* B = scr + (uint64_t)m * 64;
  constexpr uint32_t kCap = 12;
  for (int pass = 0; pass < 2; ++pass) {
    const uint32_t cap = pass == 0 ? kCap : 0xFFFFFFFFu;
    // best0 (lane 0 of the first chunk is spent on it)
    uint32_t e0 = lane == 0 ? lane_wfa_ed(con + best0, clen - best0, rd, ocl, wc, cap, m, A, B) : 0u;
    e0 = __shfl(e0, 0);
    uint32_t mbest = 0xFFFFFFFFu, pbest = 0xFFFFFFFFu;  // min over [start, end), smallest p
    for (uint32_t base = start; base < end; base += 64) {
      const uint32_t p = base + lane;
      uint32_t ed = 0xFFFFFFFFu;
      if (p < end) ed = lane_wfa_ed(con + p, clen - p, rd, ocl, wc, cap, m, A, B);
      // wave min of (ed, p)
      uint64_t key = (uint64_t)ed << 32 | p;
      for (int o = 32; o >= 1; o >>= 1) {
        const uint64_t y = __shfl_xor(key, o);
        key = min(key, y);
      }
      if (ballot(ed == kEdOverflow) || e0 == kEdOverflow) return kEdOverflow;
      if ((uint32_t)(key >> 32) < mbest) {
        mbest = (uint32_t)(key >> 32);
        pbest = (uint32_t)key;
      }
    }
    if (e0 == kEdOverflow) return kEdOverflow;
    if (mbest < cap && mbest < e0) return pbest;      // exact strict win inside the window
    if (e0 < cap && !(mbest < e0)) return best0;      // e0 exact and nothing below it
    // undecided (everything reached the cap): rerun uncapped
    if (pass == 1) return mbest < e0 ? pbest : best0;
  }
  return best0;
}

// Activate read (rd, blen) on one node side whose consensus is con[0..clen):
// pick the offset, then DWFALite::new + set_offset + update (dynamic_wfa.rs:52-99)
// on the read's wavefront row, and write the RState. Returns false on
// wavefront capacity or offset-scratch overflow. e_out = the new edit distance.
// Return: 0 ok, 1 wavefront capacity (retry with a larger wcap), 2 offset scratch.
template <class P>
__device__ inline int wave_activate(P rsp, Gm<uint32_t>* wf, const Gm<uint8_t>* rd, uint32_t blen,
                                     const Gm<uint8_t>* con, uint32_t clen, const DevConfig& cfg, uint32_t wcap,
                                     Gm<uint64_t>* scr, uint32_t m, WaveCounters& cnt, uint32_t& e_out) {
  const uint32_t ocl = (uint32_t)min((uint64_t)cfg.offset_compare_length, (uint64_t)blen);
  const uint32_t off = wave_pick_offset(con, clen, rd, ocl, (uint32_t)cfg.offset_window, cfg.wildcard, scr, m);
  if (off == kEdOverflow) return 2;
  if (lane_id() == 0) wf[0] = 0;
  __builtin_amdgcn_wave_barrier();
  uint32_t e = 0, mo, mb;
  if (!wave_update_general(wf, e, off, rd, blen, con, clen, cfg.wildcard, cfg.early != 0, wcap, cnt, mo, mb))
    return 1;
  __builtin_amdgcn_wave_barrier();
  wave_rebuild(wf, e, off, blen, clen, rsp);
  e_out = e;
  return 0;
}

}  // namespace WC_ENGINE_NS
