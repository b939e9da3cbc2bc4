// maxmq_amd/csrc/device.h — trie lookups shared by the gfx950 kernels
// (match.hip: forward match; retained.hip: reverse match).
#pragma once
#include <hip/hip_runtime.h>

#include "snapshot.h"

namespace mqm {

__device__ __forceinline__ NodeDesc load_desc(const NodeDesc *p) {
  const uint4 *q = reinterpret_cast<const uint4 *>(p);
  uint4 a = q[0], b = q[1];
  NodeDesc d;
  d.plus = a.x;
  d.hash = a.y;
  d.sub_off = a.z;
  d.sub_cnt = a.w;
  d.multi = b.x;
  d.hsub_cnt = b.y;
  d.sh_off = b.z;
  d.sh_cnt_flags = b.w;
  return d;
}

// Literal child lookup: open-addressed edge table, 2 entries per 128-B bucket.
// Long keys (>= 16 bytes) are verified byte-for-byte against the token pool.
__device__ inline uint32_t probe_edge(const DeviceSnapshot &s, uint32_t parent, uint64_t k0, uint64_t k1,
                               const uint8_t *tok, uint32_t tok_len, NodeDesc *desc) {
  const uint64_t nslots = s.n_buckets * kEdgesPerBucket;
  Key key{k0, k1};
  uint64_t slot = bucket_of(edge_hash(parent, key), s.n_buckets) * kEdgesPerBucket;
  for (;;) {
    // the whole 64-B entry in one round trip: key, header and the child's descriptor
    const uint4 *q = reinterpret_cast<const uint4 *>(s.edges + slot);
    const uint4 kk = q[0], pc = q[1], d0 = q[2], d1 = q[3];
    if (pc.x == kNone) return kNone;
    if (pc.x == parent && (((uint64_t)kk.y << 32) | kk.x) == k0 && (((uint64_t)kk.w << 32) | kk.z) == k1) {
      bool ok = true;
      if (key_is_long(key)) {
        ok = pc.w == tok_len;
        for (uint32_t i = 0; ok && i < tok_len; i++) ok = s.tok_pool[pc.z + i] == tok[i];
      }
      if (ok) {
        desc->plus = d0.x;
        desc->hash = d0.y;
        desc->sub_off = d0.z;
        desc->sub_cnt = d0.w;
        desc->multi = d1.x;
        desc->hsub_cnt = d1.y;
        desc->sh_off = d1.z;
        desc->sh_cnt_flags = d1.w;
        return pc.y;
      }
    }
    slot = slot + 1 == nslots ? 0 : slot + 1;
  }
}

}  // namespace mqm
