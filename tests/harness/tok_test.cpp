// tests/harness/tok_test.cpp — the walk tokenizer's word-level helpers
// (keys.h slash_mask16 / align_byte, used by match.hip k_walk) against a
// plain byte scan: for random topics at every alignment, lane gl's 16 bytes
// [16 gl, 16 gl + 16) taken from 5 aligned words as k_walk takes them (loads
// clamped into the topic's last word, bytes past the end zeroed), the '/'
// positions found by the masks must equal the byte scan's, including a '.'
// (0x2E) right after a '/' (the byte the borrow-based zero test misflags).
// Test infrastructure: built by tests/harness/Makefile, run by
// tests/test_capi_host.py.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../maxmq_amd/csrc/keys.h"

int main() {
  std::mt19937 rng(7);
  std::vector<uint8_t> mem(4096 + 64);
  uint64_t checked = 0;
  for (int it = 0; it < 100000; it++) {
    const uint32_t len = rng() % 130;
    const size_t off = 8 + rng() % 1024;
    for (auto &b : mem) b = (uint8_t)rng();
    for (uint32_t i = 0; i < len; i++) {
      const uint32_t c = rng() % 5;
      mem[off + i] = c == 0 ? '/' : c == 1 ? '.' : c == 2 ? 0xAF : (uint8_t)('a' + rng() % 3);
    }
    const uint8_t *tp = mem.data() + off;
    for (uint32_t base = 0; base < len; base += 64)
      for (uint32_t gl = 0; gl < 4; gl++) {
        const uint32_t p0 = base + 16 * gl;
        const uint64_t first = reinterpret_cast<uint64_t>(tp + p0);
        const uint64_t lastw = reinterpret_cast<uint64_t>(tp + len - 1) & ~3ull;
        const uint64_t a0 = first & ~3ull;
        const uint32_t r = (uint32_t)(first & 3u);
        uint32_t w[5], b4[4];
        for (int k = 0; k < 5; k++) memcpy(&w[k], reinterpret_cast<const void *>(std::min(a0 + 4 * k, lastw)), 4);
        for (int k = 0; k < 4; k++) b4[k] = mqm::align_byte(w[k + 1], w[k], r);
        for (int k = 0; k < 4; k++) {
          const uint32_t pk = p0 + 4 * k;
          if (pk >= len) b4[k] = 0;
          else if (pk + 4 > len) b4[k] &= 0xFFFFFFFFu >> (8 * (pk + 4 - len));
        }
        uint32_t want = 0;
        for (uint32_t i = 0; i < 16; i++)
          if (p0 + i < len && tp[p0 + i] == '/') want |= 1u << i;
        const uint32_t got = mqm::slash_mask16(b4);
        uint8_t bytes[16];
        memcpy(bytes, b4, 16);
        for (uint32_t i = 0; i < 16; i++)
          if (bytes[i] != (p0 + i < len ? tp[p0 + i] : 0)) {
            printf("FAIL bytes len %u off %zu p0 %u i %u\n", len, off, p0, i);
            return 1;
          }
        if (got != want) {
          printf("FAIL mask len %u off %zu p0 %u: %04x vs %04x\n", len, off, p0, got, want);
          return 1;
        }
        checked++;
      }
  }
  printf("OK %llu lane chunks\n", (unsigned long long)checked);
  return 0;
}
