// maxmq_amd/csrc/device.h — trie lookups shared by the gfx950 kernels
// (match.hip: forward match; retained.hip: reverse match).
#pragma once
#include <hip/hip_runtime.h>

#include "snapshot.h"

#ifndef MQM_DESC32
#define MQM_DESC32 1
#endif

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

// One step of the level walk for one lane, with a single load group: either
// the literal probe's home slot (64 B: key, header, the child's descriptor) or
// a wildcard child's descriptor (the node array is padded so 64-B reads of its
// last entry stay in bounds).  Both kinds issue the same loads unconditionally,
// so the lanes of a wavefront have them in flight together; only a probe chain
// that continues past its home slot (rare at the table's load factor) loops.
__device__ __forceinline__ uint32_t walk_step(const DeviceSnapshot &s, bool do_probe, bool do_desc, bool use_bloom,
                                              uint32_t parent, uint32_t wc, uint64_t k0, uint64_t k1,
                                              const uint8_t *tok, uint32_t tok_len, NodeDesc *desc) {
  const Key key{k0, k1};
  const uint64_t nslots = s.n_buckets * kEdgesPerBucket;
  const uint64_t h = do_probe ? edge_hash(parent, key) : 0;
  if (s.bloom) {  // a literal no edge has: no probe (its bucket would be a DRAM request)
    const bool chk = do_probe && use_bloom;
    const uint64_t w = chk ? s.bloom[bloom_word(h, s.bloom_mask)] : ~0ull;
    const uint64_t b = bloom_bits(h);
    do_probe = do_probe && (w & b) == b;
  }
  uint64_t slot = do_probe ? bucket_of(h, s.n_buckets) * kEdgesPerBucket : 0;
  const uint4 *q = do_probe ? reinterpret_cast<const uint4 *>(s.edges + slot)
                            : reinterpret_cast<const uint4 *>(s.nodes + (do_desc ? wc : 0));
  uint4 x0 = q[0], x1 = q[1], x2, x3;
#if MQM_DESC32
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
#else
  x2 = q[2];
  x3 = q[3];
#endif
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

// ---- cooperative form for a 4-lane group (k_walk<4>) ------------------------
// A lane that loads a 64-B entry by itself issues four 16-B loads, each a line
// access of its own, so a wave-instruction touches 64 lines and the memory
// pipeline's per-line address work — not DRAM — bounds random gathers
// (tools/calib_fetch: k_gather64 vs k_coop4x16).  Here the four lanes of a
// group load each of their four items' blocks together, 16 B per lane (one
// line per group per instruction), and a quad transpose (DPP, no LDS) hands
// every lane its own item's block.
template <int kCtrl>
__device__ __forceinline__ uint32_t quad_dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kCtrl, 0xF, 0xF, true);
}
typedef unsigned int U32x4 __attribute__((ext_vector_type(4)));  // native vector: no struct copies
typedef const U32x4 __attribute__((address_space(1))) *GPtr4;     // global_load, not flat_load
template <int kCtrl>
__device__ __forceinline__ U32x4 quad_dpp4(U32x4 v) {
  U32x4 r;
  r.x = quad_dpp<kCtrl>(v.x);
  r.y = quad_dpp<kCtrl>(v.y);
  r.z = quad_dpp<kCtrl>(v.z);
  r.w = quad_dpp<kCtrl>(v.w);
  return r;
}
// lane q of a quad holds r0..r3 = chunk q of items 0..3; afterwards r0..r3 =
// chunks 0..3 of item q (two butterfly stages over the quad, no LDS)
__device__ __forceinline__ void quad_transpose(U32x4 &r0, U32x4 &r1, U32x4 &r2, U32x4 &r3, int q) {
  const bool h2 = q & 2, h1 = q & 1;
  {  // 2x2 blocks: lanes q, q ^ 2 swap the off-diagonal pair (quad_perm [2, 3, 0, 1])
    const U32x4 v0 = quad_dpp4<0x4E>(h2 ? r0 : r2), v1 = quad_dpp4<0x4E>(h2 ? r1 : r3);
    if (h2) {
      r0 = v0;
      r1 = v1;
    } else {
      r2 = v0;
      r3 = v1;
    }
  }
  {  // inside each block: lanes q, q ^ 1 (quad_perm [1, 0, 3, 2])
    const U32x4 v0 = quad_dpp4<0xB1>(h1 ? r0 : r1), v1 = quad_dpp4<0xB1>(h1 ? r2 : r3);
    if (h1) {
      r0 = v0;
      r2 = v1;
    } else {
      r1 = v0;
      r3 = v1;
    }
  }
}

// walk_step for lane q of a 4-lane group whose four lanes all call it together
// (same arguments as walk_step)
__device__ __forceinline__ uint32_t walk_step_quad(const DeviceSnapshot &s, bool do_probe, bool do_desc, bool use_bloom,
                                                   uint32_t parent, uint32_t wc, uint64_t k0, uint64_t k1,
                                                   const uint8_t *tok, uint32_t tok_len, NodeDesc *desc, int q) {
  const Key key{k0, k1};
  const uint64_t nslots = s.n_buckets * kEdgesPerBucket;
  const uint64_t h = do_probe ? edge_hash(parent, key) : 0;
  if (s.bloom) {
    const bool chk = do_probe && use_bloom;
    const uint64_t w = chk ? s.bloom[bloom_word(h, s.bloom_mask)] : ~0ull;
    const uint64_t b = bloom_bits(h);
    do_probe = do_probe && (w & b) == b;
  }
  uint64_t slot = do_probe ? bucket_of(h, s.n_buckets) * kEdgesPerBucket : 0;
  // this lane's block | 1 (64-B edge entry) or | 2 (32-B descriptor); blocks are 32-B aligned
  const uint64_t a = do_probe ? (reinterpret_cast<uint64_t>(s.edges + slot) | 1u)
                              : do_desc ? (reinterpret_cast<uint64_t>(s.nodes + wc) | 2u) : 0;
  const uint32_t alo = (uint32_t)a, ahi = (uint32_t)(a >> 32);
  // every lane loads unconditionally (one basic block: the four loads are in
  // flight together): a descriptor's lanes 2, 3 re-read its 32 B (same line),
  // an empty item's lanes the root descriptor (a line every CU holds)
  const uint64_t dummy = reinterpret_cast<uint64_t>(s.nodes);
#define MQM_QUAD_ADDR(j)                                                                          \
  [&] {                                                                                           \
    const uint32_t lo = quad_dpp<(j) * 0x55>(alo), hi = quad_dpp<(j) * 0x55>(ahi);                \
    const uint32_t kd = lo & 3u;                                                                  \
    const uint64_t base = kd ? ((((uint64_t)hi << 32) | lo) & ~3ull) : dummy;                     \
    return (GPtr4)(base + 16u * (uint32_t)(kd == 1u ? q : (q & 1)));                              \
  }()
  const GPtr4 p0 = MQM_QUAD_ADDR(0), p1 = MQM_QUAD_ADDR(1), p2 = MQM_QUAD_ADDR(2), p3 = MQM_QUAD_ADDR(3);
#undef MQM_QUAD_ADDR
  U32x4 r0 = *p0, r1 = *p1, r2 = *p2, r3 = *p3;
  quad_transpose(r0, r1, r2, r3, q);
  uint4 x0 = make_uint4(r0.x, r0.y, r0.z, r0.w), x1 = make_uint4(r1.x, r1.y, r1.z, r1.w);
  uint4 x2 = make_uint4(r2.x, r2.y, r2.z, r2.w), x3 = make_uint4(r3.x, r3.y, r3.z, r3.w);
  uint32_t c = kNone;
  bool more = false;
  if (do_desc) {
    c = wc;
    *desc = NodeDesc{x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
  }
  for (;;) {  // a probe chain past its home slot (rare): per lane, as walk_step
    if (do_probe && x1.x != kNone) {
      const bool hit = x1.x == parent && (((uint64_t)x0.y << 32) | x0.x) == k0 &&
                       (((uint64_t)x0.w << 32) | x0.z) == k1;
      bool ok = hit;
      if (hit && key_is_long(key)) {
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
    if (!__any(more)) break;
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
