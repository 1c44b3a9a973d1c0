// Internal host-side declarations of the waffle_con MI355X library.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace wc {

// rand 0.8 StdRng (ChaCha12) restated for generate_test
class ChaChaRng {
 public:
  ChaChaRng(const uint8_t seed[32], int rounds);
  static ChaChaRng seed_from_u64(uint64_t state, int rounds);
  uint32_t next_u32();
  uint64_t next_u64();
  uint32_t uniform_u32(uint32_t range);  // UniformInt<u8|i32>::new(0, range)
  double uniform_unit_f64();             // Uniform<f64>::new(0.0, 1.0)

 private:
  void refill();
  uint32_t key_[8];
  uint32_t buf_[64];
  uint64_t counter_;
  int index_;
  int rounds_;
};

void generate_test(uint8_t alphabet, size_t seq_len, size_t num_samples, double error_rate, uint64_t seed,
                   std::vector<uint8_t>& consensus, std::vector<std::vector<uint8_t>>& samples);

}  // namespace wc
