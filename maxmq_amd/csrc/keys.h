// maxmq_amd/csrc/keys.h — level-token keys and hashes shared by the host
// snapshot builder and the gfx950 kernels (compiled by both g++ and hipcc).
//
// A topic/filter level ("particle", topics.go:558-577) becomes a 128-bit key:
//   * len <= 15 : the bytes themselves, little-endian in k0 | k1[0..55], and
//                 the length in k1's top byte (0..15).  Exact: no collisions.
//   * len >= 16 : a 120-bit hash with k1's top byte = 0xFF; a probe hit is
//                 verified against the token byte pool, so matching stays exact.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define MQM_HD __host__ __device__ __forceinline__
#else
#define MQM_HD inline
#endif

namespace mqm {

constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint32_t kInlineMax = 15;

struct Key {
  uint64_t k0, k1;
};

MQM_HD uint64_t fmix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

MQM_HD uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

// 128-bit hash of a long token (>= 16 bytes); reads whole 8-byte words through
// the caller-supplied byte accessor so host and device share one definition.
template <class ByteAt>
MQM_HD Key hash_long_token(ByteAt at, uint32_t len) {
  uint64_t h0 = 0x9E3779B97F4A7C15ull ^ len, h1 = 0xC2B2AE3D27D4EB4Full ^ ((uint64_t)len << 32);
  uint32_t i = 0;
  for (; i + 8 <= len; i += 8) {
    uint64_t w = 0;
    for (int b = 0; b < 8; b++) w |= (uint64_t)at(i + b) << (8 * b);
    h0 = rotl64(h0 ^ (w * 0x87c37b91114253d5ull), 31) * 0x4cf5ad432745937full;
    h1 = rotl64(h1 + (w * 0x4cf5ad432745937full), 33) * 0x87c37b91114253d5ull;
  }
  uint64_t w = 0;
  for (uint32_t b = 0; i + b < len; b++) w |= (uint64_t)at(i + b) << (8 * b);
  h0 ^= w * 0x9E3779B97F4A7C15ull;
  h1 ^= rotl64(w, 17) * 0xC2B2AE3D27D4EB4Full;
  h0 = fmix64(h0 + h1);
  h1 = fmix64(h1 + h0);
  Key k;
  k.k0 = h0;
  k.k1 = (h1 & 0x00FFFFFFFFFFFFFFull) | (0xFFull << 56);
  return k;
}

template <class ByteAt>
MQM_HD Key make_key(ByteAt at, uint32_t len) {
  if (len > kInlineMax) return hash_long_token(at, len);
  Key k;
  k.k0 = 0;
  k.k1 = (uint64_t)len << 56;
  for (uint32_t i = 0; i < len; i++) {
    uint64_t b = (uint64_t)at(i);
    if (i < 8)
      k.k0 |= b << (8 * i);
    else
      k.k1 |= b << (8 * (i - 8));
  }
  return k;
}

MQM_HD bool key_is_long(const Key &k) { return (k.k1 >> 56) == 0xFF; }

// Edge hash: one 64-bit multiply and a 32x32 range reduction — the walk
// hashes every literal probe twice (the push-time filter check, the probe),
// and 64-bit integer multiplies are multi-cycle VALU instructions (round 2's
// fmix64 with a 64x64 reduction measured slower, profiles/r03/r03k).

// bucket of an edge among n buckets (multiply-shift range reduction: any n)
MQM_HD uint64_t bucket_of(uint64_t h, uint64_t n) {
  if (n <= 0xFFFFFFFFull) return ((h >> 32) * n) >> 32;  // the hash's top 32 bits
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(h, n);
#else
  return (uint64_t)(((unsigned __int128)h * n) >> 64);
#endif
}

// bucket hash of an edge (parent node, child key)
MQM_HD uint64_t edge_hash(uint32_t parent, const Key &k) {
  // one multiply: every product bit above bit i depends on every input bit up
  // to i, and the fold brings the well-mixed top half down for the low bits
  const uint64_t x = k.k0 ^ rotl64(k.k1, 29) ^ ((uint64_t)parent * 0x9E3779B97F4A7C15ull);
  uint64_t h = (x ^ (x >> 31)) * 0xff51afd7ed558ccdull;
  return h ^ (h >> 32);
}

// edge-existence filter (DeviceSnapshot::bloom): a blocked Bloom filter, the 3
// bits of an edge hash in one 64-bit word (bits independent of bucket_of's)
MQM_HD uint64_t bloom_word(uint64_t h, uint64_t mask) { return (h ^ (h >> 31)) & mask; }
MQM_HD uint64_t bloom_bits(uint64_t h) {
  return (1ull << ((h >> 34) & 63)) | (1ull << ((h >> 40) & 63)) | (1ull << ((h >> 46) & 63));
}

// The walk's tokenizer (match.hip k_walk): a lane holds 16 topic bytes as 4
// little-endian words, bytes at or past the topic's end zeroed.  -> a 16-bit
// mask of the '/' bytes (bit i = byte i).  Per byte exactly: the high bit of
// ((x & 0x7F..) + 0x7F..) | x is set for every non-zero byte of x and no carry
// crosses a byte, so no borrow from a '/' can flag its neighbour (the usual
// (x - 0x01..) & ~x trick flags a '.' after a '/').  tests/harness/tok_test.cpp
// checks it against a byte scan.
MQM_HD uint32_t slash_mask16(const uint32_t (&b4)[4]) {
  uint32_t sm = 0;
  for (int k = 0; k < 4; k++) {
    const uint32_t x = b4[k] ^ 0x2F2F2F2Fu;  // zero byte where '/'
    const uint32_t y = (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
    const uint32_t z = ~y & 0x80808080u;
    sm |= (((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u)) << (4 * k);
  }
  return sm;
}
// bytes [r, r + 4) of the 8-byte little-endian pair (lo, hi), r in 0..3
// (v_alignbyte_b32 on the device)
MQM_HD uint32_t align_byte(uint32_t hi, uint32_t lo, uint32_t r) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbyte(hi, lo, r);
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * r));
#endif
}

}  // namespace mqm
