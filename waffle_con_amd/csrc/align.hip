// Batched wfa_ed / wfa_ed_config on the device (sequence_alignment.rs:18-87).
//
// One wave64 per pair. The wavefront of iteration `edits` has 2*edits+1
// entries, entry k holding the furthest (i into v1, j into v2) pair the
// reference keeps at index k (sequence_alignment.rs:62-85). Because of the
// boundary rules at i == l1 / j == l2 an entry is not tied to one diagonal, so
// the pairs are stored whole, packed as i << 32 | j (u64 order = the
// reference's lexicographic tuple max). Lanes own entries k = lane + 64 c.
// Each iteration is two passes over the wave's scratch rows in HBM:
//   1. extend every entry in place along its diagonal (the match loop at
//      :62-64; the wildcard matches on either side), and stop with `edits`
//      as soon as any entry sits at the end (:66-69);
//   2. next[k] = max(a(cur[k]), b(cur[k-1]), c(cur[k-2])) — the same three
//      candidates per entry as :70-84, gathered per output entry instead of
//      scattered, which is the same max.
// The rows are sized on the host to the worst case (2*(l1+l2)+3 entries), so a
// pair never overflows; the edit count is exact.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "engine_shared.hpp"

namespace wc {

__device__ __forceinline__ bool ed_match(uint8_t a, uint8_t b, int wc) {
  return a == b || (wc >= 0 && (a == (uint8_t)wc || b == (uint8_t)wc));
}

// extend (i, j) while the symbols match (sequence_alignment.rs:62-64);
// four independent byte loads per round while both sides have 4 left
__device__ __forceinline__ void ed_extend(const uint8_t* __restrict__ v1, uint32_t l1, const uint8_t* __restrict__ v2,
                                          uint32_t l2, int wc, uint32_t& i, uint32_t& j) {
  while (i + 4 <= l1 && j + 4 <= l2) {
    const uint8_t a0 = v1[i], a1 = v1[i + 1], a2 = v1[i + 2], a3 = v1[i + 3];
    const uint8_t b0 = v2[j], b1 = v2[j + 1], b2 = v2[j + 2], b3 = v2[j + 3];
    const uint32_t n = !ed_match(a0, b0, wc) ? 0u
                       : !ed_match(a1, b1, wc) ? 1u
                       : !ed_match(a2, b2, wc) ? 2u
                       : !ed_match(a3, b3, wc) ? 3u
                                               : 4u;
    i += n;
    j += n;
    if (n < 4) return;
  }
  while (i < l1 && j < l2 && ed_match(v1[i], v2[j], wc)) {
    ++i;
    ++j;
  }
}

__device__ __forceinline__ void ed_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

constexpr uint64_t kJ1 = 1ull;         // (i, j + 1)
constexpr uint64_t kI1 = 1ull << 32;   // (i + 1, j)

__global__ void __launch_bounds__(256) wfa_ed_batch_kernel(const EdDevJob* __restrict__ jobs, uint32_t n,
                                                           const uint8_t* __restrict__ seqs,
                                                           uint64_t* __restrict__ scratch, int wc, uint32_t both,
                                                           uint64_t* __restrict__ out) {
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t id = blockIdx.x * (blockDim.x >> 6) + wave;
  if (id >= n) return;  // wave-uniform
  const EdDevJob J = jobs[id];
  const uint8_t* v1 = seqs + J.v1_off;
  const uint8_t* v2 = seqs + J.v2_off;
  const uint32_t l1 = J.l1, l2 = J.l2;
  uint64_t* cur = scratch + J.scr_off;
  uint64_t* nxt = cur + J.cap;
  if (lane == 0) cur[0] = 0;
  ed_wave_sync();
  for (uint32_t edits = 0;; ++edits) {
    const uint32_t W = 2 * edits + 1;
    bool done = false;
    for (uint32_t k = lane; k < W; k += 64) {
      const uint64_t p = cur[k];
      uint32_t i = (uint32_t)(p >> 32), j = (uint32_t)p;
      ed_extend(v1, l1, v2, l2, wc, i, j);
      cur[k] = (uint64_t)i << 32 | j;
      done |= (i == l1 || !both) && j == l2;
    }
    if (__builtin_amdgcn_ballot_w64(done)) {
      if (lane == 0) out[id] = edits;
      return;
    }
    ed_wave_sync();
    // every unfinished iteration raises the largest i + j by at least one, so
    // edits < l1 + l2 here and the host's rows (2 (l1 + l2) + 3) always fit;
    // checked anyway: a short row is reported, never truncated
    if (W + 2 > J.cap) {
      if (lane == 0) out[id] = ~0ull;
      return;
    }
    for (uint32_t k = lane; k < W + 2; k += 64) {
      uint64_t v = 0;
#pragma unroll
      for (uint32_t s = 0; s < 3; ++s) {
        if (k < s || k - s >= W) continue;
        const uint64_t p = cur[k - s];
        const uint32_t i = (uint32_t)(p >> 32), j = (uint32_t)p;
        uint64_t c;
        if (i == l1) c = s == 0 ? p : p + kJ1;                        // :70-74
        else if (j == l2) c = s == 2 ? p : p + kI1;                   // :75-79
        else c = s == 0 ? p + kI1 : (s == 1 ? p + kI1 + kJ1 : p + kJ1);  // :80-84
        v = c > v ? c : v;
      }
      nxt[k] = v;
    }
    ed_wave_sync();
    uint64_t* t = cur;
    cur = nxt;
    nxt = t;
  }
}

void launch_wfa_ed_batch(const EdDevJob* jobs, uint32_t n, const uint8_t* seqs, uint64_t* scratch, int wc,
                         uint32_t both, uint64_t* out, hipStream_t s) {
  const uint32_t per_block = 4;
  hipLaunchKernelGGL(wfa_ed_batch_kernel, dim3((n + per_block - 1) / per_block), dim3(64 * per_block), 0, s, jobs, n,
                     seqs, scratch, wc, both, out);
}

}  // namespace wc
