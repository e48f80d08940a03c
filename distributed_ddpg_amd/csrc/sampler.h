// Host MT19937 + CPython random.sample restatement (see sampler.cpp).
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace ddpg {

struct Mt19937 {
  uint32_t mt[624];
  int mti = 625;
  void init_genrand(uint32_t s);
  void init_by_array(const uint32_t* key, size_t len);
  void seed_int(int64_t seed);  // random.seed(int)
  uint32_t genrand_uint32();
  uint64_t getrandbits(int k);
  uint64_t randbelow(uint64_t n);
};

int sample_setsize(int k);

struct Sampler {
  Mt19937 rng;
  std::vector<int64_t> pool;
  std::vector<uint64_t> bitmap;
  explicit Sampler(int64_t seed) { rng.seed_int(seed); }
  // random.sample(range(n), k) -> out[0..k)
  int sample(int64_t n, int k, int64_t* out);
};

}  // namespace ddpg
