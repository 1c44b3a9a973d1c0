// Latency probe for the engine's building blocks on the GPU box (not part of
// the library): cycles (s_memtime) of
//   1. a dependent HBM load chain over a cold 512 MiB buffer,
//   2. the same chain over an L2-resident 1 MiB buffer,
//   3. a load of a 4-byte field of a 64-byte record this wave just wrote
//      field by field (the RState read-after-write pattern),
//   4. the same after full 16-byte stores of the record,
//   5. __syncthreads() with 4 waves, and
//   6. a dependent LDS load chain.
// Build: hipcc -O3 --offload-arch=gfx950 tools/latency_probe.hip -o tools/latency_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memtime(); }

__global__ void probe(uint32_t* big, uint64_t big_n, uint32_t* small, uint64_t small_n, uint4* rec,
                      unsigned long long* out, int iters) {
  __shared__ uint32_t lds[4096];
  const int tid = threadIdx.x;
  for (int i = tid; i < 4096; i += blockDim.x) lds[i] = (i * 97 + 13) & 4095;
  __syncthreads();
  if (tid == 0) {
    // 1. cold HBM chain
    uint32_t p = 0;
    uint64_t t0 = now();
    for (int i = 0; i < iters; ++i) p = big[p];
    uint64_t t1 = now();
    out[0] = (t1 - t0) / iters;
    out[10] = p;
    // 2. warm chain (prime first)
    p = 0;
    for (int i = 0; i < iters; ++i) p = small[p];
    p = 0;
    t0 = now();
    for (int i = 0; i < iters; ++i) p = small[p];
    t1 = now();
    out[1] = (t1 - t0) / iters;
    out[11] = p;
    // 3. read-after-partial-write
    uint64_t acc = 0;
    t0 = now();
    for (int i = 0; i < iters; ++i) {
      uint32_t* r = (uint32_t*)(rec + 4 * (uint64_t)(i & 1023));
      r[0] = i;
      r[5] = i + 1;
      r[9] = (uint32_t)acc;
      __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
      acc += r[1 + (acc & 1)];
    }
    t1 = now();
    out[2] = (t1 - t0) / iters;
    // 3b. the same, but the record was read (line valid in L2) before the writes
    t0 = now();
    for (int i = 0; i < iters; ++i) {
      uint32_t* r = (uint32_t*)(rec + 4 * (uint64_t)(2048 + (i & 1023)));
      acc += r[2];
      r[0] = i;
      r[5] = i + 1;
      r[9] = (uint32_t)acc;
      __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
      acc += r[1 + (acc & 1)];
    }
    t1 = now();
    out[7] = (t1 - t0) / iters;
    // 3c. read only (line valid, no writes)
    t0 = now();
    for (int i = 0; i < iters; ++i) {
      uint32_t* r = (uint32_t*)(rec + 4 * (uint64_t)(3072 + (i & 1023)));
      acc += r[(acc & 1) + 1];
      __asm__ volatile("" ::: "memory");
    }
    t1 = now();
    out[8] = (t1 - t0) / iters;
    // 4. read-after-full-16B-write
    t0 = now();
    for (int i = 0; i < iters; ++i) {
      uint4* r = rec + 4 * (uint64_t)(1024 + (i & 1023));
      r[0] = make_uint4(i, (uint32_t)acc, 0, 0);
      r[1] = make_uint4(1, 2, 3, 4);
      r[2] = make_uint4(1, 2, 3, 4);
      r[3] = make_uint4(1, 2, 3, (uint32_t)acc);
      __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
      acc += ((uint32_t*)r)[2 + (acc & 1)];
    }
    t1 = now();
    out[3] = (t1 - t0) / iters;
    out[12] = acc;
  }
  __syncthreads();
  // 5. barrier cost
  uint64_t t0 = now();
  for (int i = 0; i < iters; ++i) __syncthreads();
  uint64_t t1 = now();
  if (tid == 0) out[4] = (t1 - t0) / iters;
  // 6. LDS chain
  if (tid == 0) {
    uint32_t p = 0;
    t0 = now();
    for (int i = 0; i < iters; ++i) p = lds[p];
    t1 = now();
    out[5] = (t1 - t0) / iters;
    out[13] = p;
  }
  // 7. s_memtime overhead
  if (tid == 0) {
    t0 = now();
    uint64_t x = 0;
    for (int i = 0; i < iters; ++i) x += now();
    t1 = now();
    out[6] = (t1 - t0) / iters;
    out[14] = x;
  }
}

int main() {
  const uint64_t big_n = 128ull << 20, small_n = 256ull << 10;  // 512 MiB / 1 MiB of u32
  std::vector<uint32_t> h(big_n);
  // a random cycle with 4 KiB strides so each step is a new line
  uint64_t stride = 1031 * 1024 + 7;
  for (uint64_t i = 0; i < big_n; ++i) h[i] = (uint32_t)((i + stride) % big_n);
  uint32_t *big, *small;
  uint4* rec;
  unsigned long long* out;
  hipMalloc(&big, big_n * 4);
  hipMalloc(&small, small_n * 4);
  hipMalloc(&rec, 4096 * 64);
  hipMalloc(&out, 16 * 8);
  hipMemcpy(big, h.data(), big_n * 4, hipMemcpyHostToDevice);
  for (uint64_t i = 0; i < small_n; ++i) h[i] = (uint32_t)((i + 1031 * 16 + 3) % small_n);
  hipMemcpy(small, h.data(), small_n * 4, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(256), 0, 0, big, big_n, small, small_n, rec, out, 2000);
    hipDeviceSynchronize();
  }
  unsigned long long o[16];
  hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost);
  printf("{\"hbm_chain\": %llu, \"l2_chain\": %llu, \"raw_partial\": %llu, \"raw_full16\": %llu, \"barrier\": %llu, "
         "\"lds_chain\": %llu, \"memtime\": %llu, \"raw_partial_line_read_first\": %llu, \"load_only\": %llu, "
         "\"unit\": \"s_memtime ticks per step\"}\n",
         o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7], o[8]);
  return 0;
}
