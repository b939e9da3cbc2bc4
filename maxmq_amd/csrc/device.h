// maxmq_amd/csrc/device.h — trie lookups shared by the gfx950 kernels
// (match.hip: forward match; retained.hip: reverse match).
#pragma once
#include <hip/hip_runtime.h>

#include "snapshot.h"

namespace mqm {

// MQM_SNAP_STAMP=1 (snapshot.h DeviceSnapshot::stamp): 0 when every stamp
// equals the snapshot's version; else bit 0: a stamp read through the caches
// differs, bit 1: the stamp in memory (a system-scope load) differs — (1)
// alone is a stale cached line over refilled memory, (3) a buffer refilled
// for another snapshot while this reader still runs on it
__device__ inline uint32_t stamp_mismatch(const DeviceSnapshot &s, unsigned long long *seen_cached,
                                          unsigned long long *seen_memory) {
  uint32_t bad = 0;
  for (int i = 0; i < 4; i++) {
    const unsigned long long c = s.stamp[i][0];  // (a plain load: through L1 / L2)
    const unsigned long long m = __hip_atomic_load(s.stamp[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (c != s.version && !(bad & 1)) *seen_cached = c, bad |= 1;
    if (m != s.version && !(bad & 2)) *seen_memory = m, bad |= 2;
  }
  return bad;
}

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

// One step of the level walk for one lane, with a single load group: either
// the literal probe's home slot (64 B: key, header, the child's descriptor) or
// a wildcard child's descriptor (the node array is padded so 64-B reads of its
// last entry stay in bounds).  Both kinds issue the same loads unconditionally,
// so the lanes of a wavefront have them in flight together; only a probe chain
// that continues past its home slot (rare at the table's load factor) loops.
__device__ __forceinline__ uint32_t walk_step(const DeviceSnapshot &s, bool do_probe, bool do_desc, uint32_t parent,
                                              uint32_t wc, uint64_t k0, uint64_t k1, const uint8_t *tok, uint32_t tok_len, NodeDesc *desc) {
  const Key key{k0, k1};
  const uint64_t nslots = s.n_buckets * kEdgesPerBucket;
  const uint64_t h = do_probe ? edge_hash(parent, key) : 0;
  uint64_t slot = do_probe ? bucket_of(h, s.n_buckets) * kEdgesPerBucket : 0;
  const uint4 *q = do_probe ? reinterpret_cast<const uint4 *>(s.edges + slot)
                            : reinterpret_cast<const uint4 *>(s.nodes + (do_desc ? wc : 0));
  uint4 x0 = q[0], x1 = q[1], x2, x3;
  // a descriptor is 32 B: a wildcard step's lanes skip the entry's second half
  // (the next descriptor, for an odd id in the next 64-B sector) — every load
  // instruction costs the memory pipeline one access per distinct line it
  // touches, so a masked lane saves an access, not only bytes
  if (do_probe) {
    x2 = q[2];
    x3 = q[3];
  } else {
    x2 = x3 = make_uint4(0, 0, 0, 0);
  }
  uint32_t c = kNone;
  bool more = false;
  if (do_desc) {
    c = wc;
    *desc = NodeDesc{x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
  }
  for (;;) {
    if (do_probe && x1.x != kNone) {
      const bool hit = x1.x == parent && (((uint64_t)x0.y << 32) | x0.x) == k0 &&
                       (((uint64_t)x0.w << 32) | x0.z) == k1;
      bool ok = hit;
      if (hit && key_is_long(key)) {  // hashed long token: verify the bytes
        ok = x1.w == tok_len;
        for (uint32_t i = 0; ok && i < tok_len; i++) ok = s.tok_pool[x1.z + i] == tok[i];
      }
      if (ok) {
        c = x1.y;
        *desc = NodeDesc{x2.x, x2.y, x2.z, x2.w, x3.x, x3.y, x3.z, x3.w};
      }
      more = !ok;
    } else {
      more = false;
    }
    if (!__any(more)) break;  // wave-uniform
    if (more) {
      slot = slot + 1 == nslots ? 0 : slot + 1;
      const uint4 *e = reinterpret_cast<const uint4 *>(s.edges + slot);
      x0 = e[0];
      x1 = e[1];
      x2 = e[2];
      x3 = e[3];
    }
    do_probe = more;
  }
  return c;
}

// walk_step over the paired node slots (snapshot.h DeviceSnapshot::slots):
// a wildcard child's step loads its whole 64-B slot — one sector, as its
// 32-B descriptor was — and hands the child's own '+' child's descriptor to
// `carry` as well.  Probes as in walk_step.
template <class Carry>
__device__ __forceinline__ uint32_t walk_step_slot(const DeviceSnapshot &s, bool do_probe, bool do_desc,
                                                   uint32_t parent, uint32_t wc, uint64_t k0, uint64_t k1,
                                                   const uint8_t *tok, uint32_t tok_len, NodeDesc *desc,
                                                   Carry &&carry) {
  const Key key{k0, k1};
  const uint64_t nslots = s.n_buckets * kEdgesPerBucket;
  const uint64_t h = do_probe ? edge_hash(parent, key) : 0;
  uint64_t slot = do_probe ? bucket_of(h, s.n_buckets) * kEdgesPerBucket : 0;
  const uint4 *q = do_probe ? reinterpret_cast<const uint4 *>(s.edges + slot)
                            : reinterpret_cast<const uint4 *>(s.slots + 2 * (uint64_t)(do_desc ? wc : 0));
  uint4 x0 = q[0], x1 = q[1], x2 = q[2], x3 = q[3];
  uint32_t c = kNone;
  bool more = false;
  // carry(do_desc, the node's descriptor halves, its '+' child's halves): called
  // by every lane (it may use wave ops) before the probe loop, so the '+'
  // child's descriptor is consumed at once and holds no registers past here
  carry(do_desc, x0, x1, x2, x3);
  if (do_desc) {
    c = wc;
    *desc = NodeDesc{x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
  }
  for (;;) {
    if (do_probe && x1.x != kNone) {
      const bool hit = x1.x == parent && (((uint64_t)x0.y << 32) | x0.x) == k0 &&
                       (((uint64_t)x0.w << 32) | x0.z) == k1;
      bool ok = hit;
      if (hit && key_is_long(key)) {  // hashed long token: verify the bytes
        ok = x1.w == tok_len;
        for (uint32_t i = 0; ok && i < tok_len; i++) ok = s.tok_pool[x1.z + i] == tok[i];
      }
      if (ok) {
        c = x1.y;
        *desc = NodeDesc{x2.x, x2.y, x2.z, x2.w, x3.x, x3.y, x3.z, x3.w};
      }
      more = !ok;
    } else {
      more = false;
    }
    if (!__any(more)) break;  // wave-uniform
    if (more) {
      slot = slot + 1 == nslots ? 0 : slot + 1;
      const uint4 *e = reinterpret_cast<const uint4 *>(s.edges + slot);
      x0 = e[0];
      x1 = e[1];
      x2 = e[2];
      x3 = e[3];
    }
    do_probe = more;
  }
  return c;
}

}  // namespace mqm
