// CRC-32C (Castagnoli) for the TF V2 checkpoint writer/reader
// (distributed_ddpg_amd/checkpoint.py): LevelDB block trailers and
// BundleEntryProto.crc32c of every tensor.  Slicing-by-8, host only.
#include <cstddef>
#include <cstdint>
#include <cstring>

#include "../../include/ddpg_hip.h"

namespace {
struct Tables {
  uint32_t t[8][256];
  Tables() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFF];
  }
};
const Tables& tables() {
  static const Tables tb;
  return tb;
}
}  // namespace

extern "C" uint32_t ddpg_crc32c(uint32_t crc, const void* data, size_t n) {
  const auto& T = tables().t;
  const uint8_t* p = static_cast<const uint8_t*>(data);
  crc = ~crc;
  while (n >= 8) {
    uint32_t lo, hi;
    memcpy(&lo, p, 4);
    memcpy(&hi, p + 4, 4);
    lo ^= crc;
    crc = T[7][lo & 0xFF] ^ T[6][(lo >> 8) & 0xFF] ^ T[5][(lo >> 16) & 0xFF] ^ T[4][lo >> 24] ^
          T[3][hi & 0xFF] ^ T[2][(hi >> 8) & 0xFF] ^ T[1][(hi >> 16) & 0xFF] ^ T[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) crc = T[0][(crc ^ *p++) & 0xFF] ^ (crc >> 8);
  return ~crc;
}
