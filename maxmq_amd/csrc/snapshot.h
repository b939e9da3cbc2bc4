// maxmq_amd/csrc/snapshot.h — the GPU-resident CSR level-trie ("snapshot").
//
// Built on the host from the authoritative store (store.h) and uploaded as a
// handful of flat arrays.  Node ids are the DFS PREORDER of the trie with the
// children of every node ordered (literals..., '+', '#'), the same order in
// which scanSubscribers (topics.go:503) probes them.  That makes
//   rank(hit) = 2 * node + slot   (slot 1 = the parent-'#' probe, :507-509)
// a total order equal to the reference walk's emission order, so
// "first-merged subscription" (packets.go:250-255) = minimum rank.
#pragma once
#include <stdint.h>

#include "keys.h"

namespace mqm {

enum : uint32_t {
  kFlagHasChildren = 1u,  // any child (literal, '+', '#')
  kFlagDollarWild = 2u,   // node lies under a root child whose key starts with '+'/'#'
                          // == the `$` rule's Filter[0] test (topics.go:527)
};

struct NodeDesc {         // 32 B
  uint32_t plus;          // '+' child or kNone
  uint32_t hash;          // '#' child or kNone
  uint32_t sub_off;       // non-shared subscriptions [sub_off, sub_off + sub_cnt)
  uint32_t sub_cnt;
  uint32_t hsub_off;      // copy of the '#' child's non-shared range (parent probe)
  uint32_t hsub_cnt;
  uint32_t sh_off;        // shared subscriptions [sh_off, sh_off + sh_cnt)
  uint32_t sh_cnt_flags;  // sh_cnt (low 24 bits) | flags << 24
};
static_assert(sizeof(NodeDesc) == 32, "NodeDesc layout");

constexpr uint32_t kShCntMask = 0x00FFFFFFu;

struct EdgeEntry {        // 64 B; two per 128-B bucket
  uint64_t k0, k1;        // child key (keys.h)
  uint32_t parent;        // kNone = empty slot
  uint32_t child;
  uint32_t tok_off;       // long keys: bytes at tok_pool[tok_off .. +tok_len)
  uint32_t tok_len;
  NodeDesc desc;          // the child's descriptor, inline
};
static_assert(sizeof(EdgeEntry) == 64, "EdgeEntry layout");

constexpr uint32_t kEdgesPerBucket = 2;

// non-shared subscription entry; sid = index into the array
struct SubEnt {
  uint32_t client;
  uint32_t meta;          // qos[1:0] | no_local[2] | rap[3] | rh[5:4]
};

// delivery written by the matcher (one per (topic, client)):
//   bits  0..31 client id
//   bits 32..59 sid of the first-merged subscription
//   bits 60..61 max QoS, bit 62 NoLocal (OR)
constexpr uint32_t kSidBits = 28;
constexpr uint32_t kMaxSubs = 1u << kSidBits;

struct DeviceSnapshot {
  const NodeDesc *nodes;
  const EdgeEntry *edges;
  const SubEnt *subs;
  const uint8_t *tok_pool;
  uint64_t bucket_mask;   // number of buckets - 1 (power of two)
  uint32_t n_nodes;
  uint32_t n_subs;
  uint32_t n_shared;
  uint32_t height;        // max node depth (root = 0)
};

}  // namespace mqm
