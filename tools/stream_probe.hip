// Host-to-device visibility probe for the stream-mode control words (not part
// of the library). One workgroup per CU waits the way engine.hip claim_problem
// does (8-byte acquire load of {tail, stop}, relaxed heartbeat load, s_sleep
// backoff) while the host bumps the heartbeat every ~20 us and the tail every
// ~1 ms for `secs` seconds, then sets stop. Every workgroup reports how many
// distinct heartbeats and tails it saw and the longest gap (wall-clock ticks)
// between two heartbeat changes.
// Build: hipcc -O3 --offload-arch=gfx950 tools/stream_probe.hip -o tools/stream_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

struct alignas(16) Ctl {
  uint32_t tail, stop, abort, heartbeat;
};

__global__ void waiter(Ctl* c, unsigned long long* out, uint64_t give_up) {
  if (threadIdx.x != 0) return;
  uint32_t hb_seen = ~0u, tail_seen = ~0u, nhb = 0, ntail = 0, nap = 1;
  uint64_t t0 = wall_clock64(), tstart = t0, maxgap = 0, last_change = t0;
  for (;;) {
    const uint64_t ts = __hip_atomic_load(reinterpret_cast<uint64_t*>(c), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (ts >> 32) break;
    if ((uint32_t)ts != tail_seen) {
      tail_seen = (uint32_t)ts;
      ntail++;
    }
    const uint32_t hb = __hip_atomic_load(&c->heartbeat, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t now = wall_clock64();
    if (hb != hb_seen) {
      hb_seen = hb;
      nhb++;
      if (now - last_change > maxgap) maxgap = now - last_change;
      last_change = now;
    } else if (now - tstart > give_up) {
      __hip_atomic_store(&c->abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    for (uint32_t k = 0; k < nap; ++k) __builtin_amdgcn_s_sleep(127);
    nap = nap * 2 < 256 ? nap * 2 : 256;
  }
  out[blockIdx.x * 4 + 0] = nhb;
  out[blockIdx.x * 4 + 1] = ntail;
  out[blockIdx.x * 4 + 2] = maxgap;
  out[blockIdx.x * 4 + 3] = wall_clock64() - t0;
}

int main(int argc, char** argv) {
  const double secs = argc > 1 ? atof(argv[1]) : 3.0;
  int ncu = 0, clk = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeWallClockRate, 0);
  printf("CUs %d wall clock %d kHz\n", ncu, clk);
  Ctl* h = nullptr;
  if (hipHostMalloc((void**)&h, sizeof(Ctl), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 1;
  *h = Ctl{0, 0, 0, 0};
  Ctl* d = nullptr;
  (void)hipHostGetDevicePointer((void**)&d, h, 0);
  unsigned long long* out = nullptr;
  (void)hipMalloc(&out, (size_t)ncu * 32);
  const uint64_t give_up = (uint64_t)clk * 1000ull * (uint64_t)(secs + 5);
  hipLaunchKernelGGL(waiter, dim3(ncu), dim3(64), 0, 0, d, out, give_up);
  const auto t0 = std::chrono::steady_clock::now();
  uint32_t beat = 0, tail = 0;
  auto last_tail = t0;
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < secs) {
    __atomic_store_n(&h->heartbeat, ++beat, __ATOMIC_RELAXED);
    const auto now = std::chrono::steady_clock::now();
    if (std::chrono::duration<double, std::milli>(now - last_tail).count() > 1.0) {
      __atomic_store_n(&h->tail, ++tail, __ATOMIC_RELEASE);
      last_tail = now;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
  __atomic_store_n(&h->stop, 1u, __ATOMIC_RELEASE);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::vector<unsigned long long> r((size_t)ncu * 4);
  (void)hipMemcpy(r.data(), out, r.size() * 8, hipMemcpyDeviceToHost);
  unsigned long long minhb = ~0ull, mintail = ~0ull, maxgap = 0;
  for (int b = 0; b < ncu; ++b) {
    minhb = std::min(minhb, r[b * 4]);
    mintail = std::min(mintail, r[b * 4 + 1]);
    maxgap = std::max(maxgap, r[b * 4 + 2]);
  }
  printf("host: %u heartbeats, %u tails; device (min over %d workgroups): %llu heartbeats, %llu tails seen; "
         "longest heartbeat gap %.3f ms; abort %u\n",
         beat, tail, ncu, minhb, mintail, maxgap / (clk / 1000.0), h->abort);
  return h->abort ? 3 : 0;
}
