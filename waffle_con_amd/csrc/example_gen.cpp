// Synthetic input generator: waffle_con's generate_test (src/example_gen.rs:11-64)
// with the reference's RNG stack restated:
//   rand 0.8.5 StdRng = rand_chacha 0.3 ChaCha12Rng (64-bit counter, stream 0,
//   4-block / 64-word output buffer), rand_core 0.6 seed_from_u64 (PCG32 fill),
//   UniformInt widening-multiply rejection, UniformFloat [1,2)-1 mapping.
// The reference hardcodes seed 0 (example_gen.rs:15); `seed` generalises it.
// Host-side input generation only: it is not on the GPU hot path.
#include <cstdint>
#include <cstring>
#include <vector>

#include "waffle_con_internal.hpp"

namespace wc {

namespace {
inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

inline void quarter(uint32_t* s, int a, int b, int c, int d) {
  s[a] += s[b]; s[d] ^= s[a]; s[d] = rotl32(s[d], 16);
  s[c] += s[d]; s[b] ^= s[c]; s[b] = rotl32(s[b], 12);
  s[a] += s[b]; s[d] ^= s[a]; s[d] = rotl32(s[d], 8);
  s[c] += s[d]; s[b] ^= s[c]; s[b] = rotl32(s[b], 7);
}
}  // namespace

ChaChaRng::ChaChaRng(const uint8_t seed[32], int rounds) : rounds_(rounds) {
  for (int i = 0; i < 8; ++i) {
    key_[i] = (uint32_t)seed[4 * i] | ((uint32_t)seed[4 * i + 1] << 8) | ((uint32_t)seed[4 * i + 2] << 16) |
              ((uint32_t)seed[4 * i + 3] << 24);
  }
  counter_ = 0;
  index_ = 64;
}

ChaChaRng ChaChaRng::seed_from_u64(uint64_t state, int rounds) {
  uint8_t seed[32];
  for (int k = 0; k < 8; ++k) {
    state = state * 6364136223846793005ULL + 11634580027462260723ULL;
    uint32_t xorshifted = (uint32_t)(((state >> 18) ^ state) >> 27);
    uint32_t rot = (uint32_t)(state >> 59);
    uint32_t x = (xorshifted >> rot) | (xorshifted << ((32 - rot) & 31));
    std::memcpy(seed + 4 * k, &x, 4);  // little-endian host
  }
  return ChaChaRng(seed, rounds);
}

void ChaChaRng::refill() {
  static const uint32_t kConst[4] = {0x61707865, 0x3320646e, 0x79622d32, 0x6b206574};
  for (int blk = 0; blk < 4; ++blk) {
    uint32_t in[16], s[16];
    std::memcpy(in, kConst, 16);
    std::memcpy(in + 4, key_, 32);
    uint64_t ctr = counter_ + (uint64_t)blk;
    in[12] = (uint32_t)ctr;
    in[13] = (uint32_t)(ctr >> 32);
    in[14] = 0;
    in[15] = 0;
    std::memcpy(s, in, 64);
    for (int r = 0; r < rounds_; r += 2) {
      quarter(s, 0, 4, 8, 12); quarter(s, 1, 5, 9, 13); quarter(s, 2, 6, 10, 14); quarter(s, 3, 7, 11, 15);
      quarter(s, 0, 5, 10, 15); quarter(s, 1, 6, 11, 12); quarter(s, 2, 7, 8, 13); quarter(s, 3, 4, 9, 14);
    }
    for (int i = 0; i < 16; ++i) buf_[blk * 16 + i] = s[i] + in[i];
  }
  counter_ += 4;
  index_ = 0;
}

uint32_t ChaChaRng::next_u32() {
  if (index_ >= 64) refill();
  return buf_[index_++];
}

// rand_core BlockRng::next_u64 (low word first; straddles a refill)
uint64_t ChaChaRng::next_u64() {
  if (index_ < 63) {
    uint64_t lo = buf_[index_], hi = buf_[index_ + 1];
    index_ += 2;
    return (hi << 32) | lo;
  }
  if (index_ >= 64) {
    refill();
    index_ = 2;
    return ((uint64_t)buf_[1] << 32) | buf_[0];
  }
  uint64_t lo = buf_[63];
  refill();
  index_ = 1;
  return ((uint64_t)buf_[0] << 32) | lo;
}

// UniformInt::sample for u8 / i32 with a u32 draw (rand 0.8.5)
uint32_t ChaChaRng::uniform_u32(uint32_t range) {
  uint32_t z = (uint32_t)((0x100000000ULL - range) % range);
  uint32_t zone = 0xFFFFFFFFu - z;
  for (;;) {
    uint32_t v = next_u32();
    uint64_t m = (uint64_t)v * (uint64_t)range;
    uint32_t lo = (uint32_t)m, hi = (uint32_t)(m >> 32);
    if (lo <= zone) return hi;
  }
}

// UniformFloat<f64>::new(0.0, 1.0).sample
double ChaChaRng::uniform_unit_f64() {
  uint64_t v = next_u64();
  uint64_t bits = (v >> 12) | 0x3FF0000000000000ULL;
  double x;
  std::memcpy(&x, &bits, 8);
  return x - 1.0;
}

// example_gen.rs:11-64
void generate_test(uint8_t alphabet, size_t seq_len, size_t num_samples, double error_rate, uint64_t seed,
                   std::vector<uint8_t>& consensus, std::vector<std::vector<uint8_t>>& samples) {
  ChaChaRng rng = ChaChaRng::seed_from_u64(seed, 12);
  consensus.resize(seq_len);
  for (size_t i = 0; i < seq_len; ++i) consensus[i] = (uint8_t)rng.uniform_u32(alphabet);
  samples.assign(num_samples, {});
  for (size_t s = 0; s < num_samples; ++s) {
    std::vector<uint8_t>& seq = samples[s];
    seq.reserve(seq_len + seq_len / 16 + 8);
    size_t ci = 0;
    while (ci < consensus.size()) {
      uint8_t c = consensus[ci];
      bool is_error = rng.uniform_unit_f64() < error_rate;
      if (is_error) {
        uint32_t t = rng.uniform_u32(3);
        if (t == 0) {
          uint8_t off = (uint8_t)rng.uniform_u32((uint32_t)(alphabet - 1));
          seq.push_back((uint8_t)((c + off) % alphabet));
          ci++;
        } else if (t == 1) {
          ci++;
        } else {
          seq.push_back((uint8_t)rng.uniform_u32(alphabet));
        }
      } else {
        seq.push_back(c);
        ci++;
      }
    }
  }
}

}  // namespace wc
