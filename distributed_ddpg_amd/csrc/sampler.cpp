// Host restatement of CPython's random.seed(int) / random.sample as used by
// the reference ReplayBuffer (replay_buffer.py:19 `random.seed(random_seed)`,
// replay_buffer.py:36-39 `random.sample(self.buffer, k)`).
//
// Bit-exact with CPython 3.x (3.10 in this image):
//   * seed: init_by_array(key = 32-bit little-endian words of |seed|)
//     (Modules/_randommodule.c random_seed / init_by_array / init_genrand);
//   * getrandbits(k<=32) = genrand_uint32() >> (32-k);
//   * _randbelow(n): k = n.bit_length(); rejection-sample getrandbits(k) < n;
//   * sample(population, k) (Lib/random.py): setsize = 21 (+ 4**ceil(log(3k, 4))
//     when k > 5); pool branch (partial Fisher-Yates on a list copy) when
//     n <= setsize, else set branch (rejection of already-selected indices).
// The result is the list of drawn POSITIONS; callers map deque positions to
// ring slots (distributed_ddpg_amd/csrc/replay.hip).
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <unordered_set>
#include <vector>

#include "sampler.h"

namespace ddpg {

static constexpr int kN = 624;
static constexpr int kM = 397;

void Mt19937::init_genrand(uint32_t s) {
  mt[0] = s;
  for (int i = 1; i < kN; ++i)
    mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + static_cast<uint32_t>(i);
  mti = kN;
}

void Mt19937::init_by_array(const uint32_t* key, size_t len) {
  init_genrand(19650218u);
  size_t i = 1, j = 0;
  size_t k = (kN > len ? kN : len);
  for (; k; --k) {
    mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] +
            static_cast<uint32_t>(j);
    ++i;
    ++j;
    if (i >= static_cast<size_t>(kN)) {
      mt[0] = mt[kN - 1];
      i = 1;
    }
    if (j >= len) j = 0;
  }
  for (k = kN - 1; k; --k) {
    mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - static_cast<uint32_t>(i);
    ++i;
    if (i >= static_cast<size_t>(kN)) {
      mt[0] = mt[kN - 1];
      i = 1;
    }
  }
  mt[0] = 0x80000000u;
  mti = kN;
}

void Mt19937::seed_int(int64_t seed) {
  // random_seed(): n = abs(arg); key = 32-bit chunks, little-endian, at least one.
  uint64_t n = seed < 0 ? static_cast<uint64_t>(-(seed + 1)) + 1u : static_cast<uint64_t>(seed);
  uint32_t key[2];
  size_t used;
  if (n == 0) {
    key[0] = 0;
    used = 1;
  } else {
    key[0] = static_cast<uint32_t>(n & 0xffffffffu);
    key[1] = static_cast<uint32_t>(n >> 32);
    used = key[1] ? 2 : 1;
  }
  init_by_array(key, used);
}

uint32_t Mt19937::genrand_uint32() {
  static const uint32_t mag01[2] = {0x0u, 0x9908b0dfu};
  uint32_t y;
  if (mti >= kN) {
    int kk;
    for (kk = 0; kk < kN - kM; ++kk) {
      y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
      mt[kk] = mt[kk + kM] ^ (y >> 1) ^ mag01[y & 0x1u];
    }
    for (; kk < kN - 1; ++kk) {
      y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
      mt[kk] = mt[kk + (kM - kN)] ^ (y >> 1) ^ mag01[y & 0x1u];
    }
    y = (mt[kN - 1] & 0x80000000u) | (mt[0] & 0x7fffffffu);
    mt[kN - 1] = mt[kM - 1] ^ (y >> 1) ^ mag01[y & 0x1u];
    mti = 0;
  }
  y = mt[mti++];
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

// getrandbits(k) for 0 < k <= 64 (CPython: words generated least-significant first)
uint64_t Mt19937::getrandbits(int k) {
  if (k <= 32) return genrand_uint32() >> (32 - k);
  uint64_t lo = genrand_uint32();
  uint64_t hi = genrand_uint32() >> (64 - k);
  return lo | (hi << 32);
}

static int bit_length(uint64_t n) {
  int b = 0;
  while (n) {
    ++b;
    n >>= 1;
  }
  return b;
}

uint64_t Mt19937::randbelow(uint64_t n) {
  if (n == 0) return 0;
  int k = bit_length(n);
  uint64_t r = getrandbits(k);
  while (r >= n) r = getrandbits(k);
  return r;
}

int sample_setsize(int k) {
  int setsize = 21;
  if (k > 5) {
    // 4 ** _ceil(_log(k * 3, 4)) ; math.log(x, b) == log(x) / log(b)
    double e = std::ceil(std::log(static_cast<double>(k) * 3.0) / std::log(4.0));
    setsize += static_cast<int>(std::llround(std::pow(4.0, e)));
  }
  return setsize;
}

int Sampler::sample(int64_t n, int k, int64_t* out) {
  if (k < 0 || n < 0 || k > n) return -1;
  if (k == 0) return 0;
  const int setsize = sample_setsize(k);
  if (n <= setsize) {
    pool.resize(static_cast<size_t>(n));
    for (int64_t i = 0; i < n; ++i) pool[i] = i;
    for (int i = 0; i < k; ++i) {
      uint64_t j = rng.randbelow(static_cast<uint64_t>(n - i));
      out[i] = pool[j];
      pool[j] = pool[n - i - 1];
    }
    return 0;
  }
  // set branch
  if (n <= (int64_t(1) << 27)) {
    size_t words = static_cast<size_t>((n + 63) / 64);
    if (bitmap.size() < words) bitmap.assign(words, 0);
    for (int i = 0; i < k; ++i) {
      uint64_t j = rng.randbelow(static_cast<uint64_t>(n));
      while (bitmap[j >> 6] & (1ull << (j & 63))) j = rng.randbelow(static_cast<uint64_t>(n));
      bitmap[j >> 6] |= 1ull << (j & 63);
      out[i] = static_cast<int64_t>(j);
    }
    for (int i = 0; i < k; ++i) bitmap[out[i] >> 6] &= ~(1ull << (out[i] & 63));
    return 0;
  }
  std::unordered_set<int64_t> selected;
  selected.reserve(static_cast<size_t>(k) * 2);
  for (int i = 0; i < k; ++i) {
    int64_t j = static_cast<int64_t>(rng.randbelow(static_cast<uint64_t>(n)));
    while (selected.count(j)) j = static_cast<int64_t>(rng.randbelow(static_cast<uint64_t>(n)));
    selected.insert(j);
    out[i] = j;
  }
  return 0;
}

}  // namespace ddpg
