// 2-bit packed read upload: the device side. A batch whose
// reads use a four-symbol alphabet (raw codes 0..3, or ASCII A/C/G/T) crosses
// PCIe as 2 bits per base (host.cpp pack_reads) and is expanded here into the
// byte arena the engines read: one workgroup per read, each thread writing 16
// bytes (one 32-bit packed word) per step; bytes past the read's end (its
// 16-byte padding and the arena's 64-byte tail) are zero, as in the byte path.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace wc {

// code k of packed byte b: (b >> 2k) & 3; lut maps codes to the alphabet
__global__ void __launch_bounds__(256) unpack2_kernel(const uint32_t* __restrict__ packed, const uint64_t* __restrict__ roff,
                                                      const uint32_t* __restrict__ rlen, uint32_t lut,
                                                      uint8_t* __restrict__ out) {
  const uint32_t r = blockIdx.x;
  const uint64_t off = roff[r];       // 16-byte aligned
  const uint32_t len = rlen[r];
  const uint32_t padded = (len + 15) & ~15u;
  const uint32_t* src = packed + off / 16;  // 4 packed bytes per 16 bases
  uint4* dst = (uint4*)(out + off);
  for (uint32_t w = threadIdx.x; w < padded / 16; w += blockDim.x) {
    const uint32_t p = src[w];
    uint32_t v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t x = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t pos = w * 16 + q * 4 + k;
        const uint32_t code = (p >> (2 * (q * 4 + k))) & 3u;
        const uint32_t byte = pos < len ? (lut >> (8 * code)) & 0xFFu : 0u;
        x |= byte << (8 * k);
      }
      v[q] = x;
    }
    dst[w] = make_uint4(v[0], v[1], v[2], v[3]);
  }
}

__global__ void zero_tail_kernel(uint8_t* __restrict__ out, uint64_t pos) {
  if (threadIdx.x < 64) out[pos + threadIdx.x] = 0;
}

void launch_unpack2(const uint32_t* packed, const uint64_t* roff, const uint32_t* rlen, uint32_t nreads, uint32_t lut,
                    uint8_t* out, uint64_t pos, hipStream_t s) {
  if (nreads) hipLaunchKernelGGL(unpack2_kernel, dim3(nreads), dim3(256), 0, s, packed, roff, rlen, lut, out);
  hipLaunchKernelGGL(zero_tail_kernel, dim3(1), dim3(64), 0, s, out, pos);
}

}  // namespace wc
