// CRC32C (Castagnoli, reflected polynomial 0x82F63B78) as used by the TFRecord framing. The SSE4.2 `crc32`
// instruction handles 8 bytes per cycle-ish; a slicing-by-8 table is the fallback for CPUs without it.
#include <nmmintrin.h>

#include <cstring>
#include <mutex>
#include <string>

#include "rt.h"

namespace rt {
namespace {

uint32_t g_table[8][256];
std::once_flag g_once;
bool g_hw = false;

void init_tables() {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    g_table[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; ++i)
    for (int s = 1; s < 8; ++s) g_table[s][i] = (g_table[s - 1][i] >> 8) ^ g_table[0][g_table[s - 1][i] & 0xff];
  __builtin_cpu_init();
  g_hw = __builtin_cpu_supports("sse4.2");
}

uint32_t crc_sw(const uint8_t* p, size_t n, uint32_t c) {
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    v ^= c;
    c = g_table[7][v & 0xff] ^ g_table[6][(v >> 8) & 0xff] ^ g_table[5][(v >> 16) & 0xff] ^
        g_table[4][(v >> 24) & 0xff] ^ g_table[3][(v >> 32) & 0xff] ^ g_table[2][(v >> 40) & 0xff] ^
        g_table[1][(v >> 48) & 0xff] ^ g_table[0][v >> 56];
    p += 8;
    n -= 8;
  }
  while (n--) c = (c >> 8) ^ g_table[0][(c ^ *p++) & 0xff];
  return c;
}

__attribute__((target("sse4.2"))) uint32_t crc_hw(const uint8_t* p, size_t n, uint32_t c) {
  uint64_t c64 = c;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    c64 = _mm_crc32_u64(c64, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = static_cast<uint32_t>(c64);
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return c32;
}

}  // namespace

uint32_t crc32c(const void* data, size_t n, uint32_t crc) {
  std::call_once(g_once, init_tables);
  const uint8_t* p = static_cast<const uint8_t*>(data);
  uint32_t c = ~crc;
  c = g_hw ? crc_hw(p, n, c) : crc_sw(p, n, c);
  return ~c;
}

}  // namespace rt

extern "C" {
uint32_t rt_crc32c(const void* data, int64_t n, uint32_t crc) { return rt::crc32c(data, (size_t)n, crc); }
uint32_t rt_masked_crc32c(const void* data, int64_t n) { return rt::mask_crc(rt::crc32c(data, (size_t)n)); }
}
