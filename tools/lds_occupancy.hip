// How many workgroups of a given LDS size does a gfx950 CU hold at once?
// Launches k x (CUs) one-wave workgroups that each spin for ~2 ms of wall
// clock with `bytes` of dynamic LDS, for k = 2..5 and a sweep of sizes, and
// prints the elapsed time beside the runtime's occupancy answer: when k per
// CU fit, the launch takes one spin; when they do not, two.
//   hipcc --offload-arch=gfx950 -O2 -o /tmp/lds_occ tools/lds_occupancy.hip && /tmp/lds_occ
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void spin(unsigned long long ticks, unsigned int* sink) {
  extern __shared__ unsigned int lds[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
  if (threadIdx.x == 0) lds[0] = blockIdx.x;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  __syncthreads();
  if (threadIdx.x == 0 && lds[0] == 0xFFFFFFFFu) sink[0] = 1;  // (never: keeps the LDS live)
}

int main() {
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
  const int cus = p.multiProcessorCount;
  printf("CUs %d, sharedMemPerMultiprocessor %zu, sharedMemPerBlock %zu\n", cus, (size_t)p.maxSharedMemoryPerMultiProcessor,
         (size_t)p.sharedMemPerBlock);
  unsigned int* sink = nullptr;
  if (hipMalloc(&sink, 4) != hipSuccess) return 1;
  hipFuncSetAttribute((const void*)spin, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  const size_t sizes[] = {40960, 40961, 41984, 52224, 53760, 53761, 53872, 54272, 54613, 54614, 55040, 65536, 81920, 81921};
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const unsigned long long ticks = 200000;  // 2 ms at 100 MHz
  // warm-up
  hipLaunchKernelGGL(spin, dim3(cus), dim3(64), 1024, 0, ticks, sink);
  hipDeviceSynchronize();
  for (size_t s : sizes) {
    int api = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&api, spin, 64, s);
    printf("bytes %6zu api %d |", s, api);
    for (int k = 2; k <= 5; ++k) {
      hipEventRecord(a, 0);
      hipLaunchKernelGGL(spin, dim3(k * cus), dim3(64), s, 0, ticks, sink);
      hipEventRecord(b, 0);
      if (hipEventSynchronize(b) != hipSuccess) {
        printf(" launch failed\n");
        return 1;
      }
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      printf(" k=%d %.2f ms", k, ms);
    }
    printf("\n");
    fflush(stdout);
  }
  return 0;
}
