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
  kFlagHasLiteral = 4u,   // some child is a literal (else the edge probe is skipped)
  kFlagMultiSat = 8u,     // a multi count in NodeDesc::multi saturated (topics -> DFS path)
  kFlagHashLeaf = 16u,    // the '#' child exists, has no children and no shared subscriptions:
                          //   everything its gather needs is in this descriptor (its range
                          //   follows this node's, its multi count is multi >> 16, its `$`
                          //   flag equals this node's), so the walk records it without a load
  kFlagParentLit = 32u,   // a '#' node whose parent is a non-root node with a literal key: the
                          //   parent is only ever reached by a literal probe, whose parent-'#'
                          //   probe (topics.go:507-509) gathers this node's subscriptions, and
                          //   this node's own visit (the next level's '#' probe, :503) happens
                          //   only when that probe did, so the walks skip the own visit's
                          //   (non-shared) gather: a set gathered twice is the same set once
  kFlagHeavyOwn = 64u,    // the node's own range has a multi entry the merge by resolution cannot take
                          //   (pinfo kPInfoHeavy): a topic gathering it merges by hash table
  kFlagHeavyHash = 128u,  // likewise the '#' child's range (gathered by the parent probe / at push)
};

struct NodeDesc {         // 32 B
  uint32_t plus;          // '+' child or kNone
  uint32_t hash;          // '#' child or kNone
  uint32_t sub_off;       // non-shared subscriptions [sub_off, sub_off + sub_cnt)
  uint32_t sub_cnt;
  uint32_t multi;         // multi entries (kMetaMulti) of the own range (low 16 bits)
                          //   and of the '#' child's range (high 16), saturating
  uint32_t hsub_cnt;      // the '#' child's non-shared range (parent probe) is
                          //   [sub_off + sub_cnt, + hsub_cnt): laid out right after
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

// Edge-table layout (flatten.cpp builds it on the host, edges.hip on the
// device — the same bytes): the slots fall into kEdgeParts contiguous
// partitions; each partition takes the edges whose home slot is inside it, in
// edge order, by linear probing that stops at the partition's end; the edges
// that ran past it are then placed in partition order by probing with
// wrap-around.  A slot is in partition edge_part_of(slot) and partition p
// starts at edge_part_lo(p) (slot * kEdgeParts < 2^64: n_slots < 2^50).
constexpr uint32_t kEdgeParts = 16384;
MQM_HD uint32_t edge_part_of(uint64_t slot, uint64_t n_slots) { return (uint32_t)(slot * kEdgeParts / n_slots); }
MQM_HD uint64_t edge_part_lo(uint32_t p, uint64_t n_slots) {
  return (n_slots * p + kEdgeParts - 1) / kEdgeParts;
}
// home slot of an edge among nb buckets
MQM_HD uint64_t edge_home(const EdgeEntry &e, uint64_t nb) {
  return bucket_of(edge_hash(e.parent, Key{e.k0, e.k1}), nb) * kEdgesPerBucket;
}
// one slot's term of the edge-table digest (the digest sums them over the
// slots, so host and device reductions in any order agree)
MQM_HD uint64_t edge_slot_mix(uint64_t slot, const EdgeEntry &e) {
  const uint64_t *w = reinterpret_cast<const uint64_t *>(&e);
  uint64_t h = slot * 0x9E3779B97F4A7C15ull ^ 0x6D716D2D65646765ull;
  for (int i = 0; i < 8; i++) {
    h ^= w[i];
    h *= 0xFF51AFD7ED558CCDull;
    h ^= h >> 32;
  }
  return h;
}

// non-shared subscription entry as the device reads it; sid = its index.  A
// node's range holds its solo entries first, then its multi entries, and the
// range of a node's '#' child follows it directly.
//   client
//   word = sid (bits 0..27) | qos << 28 | no_local << 30 | ident << 31
// (client, word & 0x7FFFFFFF) is exactly the delivery the matcher writes for
// the entry when it is its client's only gathered entry (see kMetaMulti), so a
// solo range is emitted by a masked copy.  Bit 31 (kWordIdent): Identifier > 0
// (read by the identifiers pass).  RAP / RH / the identifier value stay on the
// host (SubInfo), resolved through the delivery's sid.
struct SubEnt {
  uint32_t client;
  uint32_t word;  // while flatten() builds the snapshot: the build-time meta bits below
};
constexpr uint32_t kWordSidMask = 0x0FFFFFFFu;
constexpr uint32_t kWordIdent = 1u << 31;
constexpr uint32_t kPackedMask = 0x7FFFFFFFu;  // word -> packed delivery (sid | qos << 28 | no_local << 30)

// build-time meta (flatten.cpp): qos[1:0] | no_local[2] | rap[3] | rh[5:4] |
// multi[6] | ident[7], rewritten into the device word at the end of flatten().
// Bit 6 ("multi"): this entry may meet another entry of the same client
// in one topic's gather, so it must go through the per-topic merge
// (packets.go:250-270).  Clear ("solo") only when the flattener proved that
// no topic emits it twice (it is not on a '#' node, whose subscriptions the
// parent probe of topics.go:507-509 can emit a second time) and that none of
// the client's other filters is level-compatible with it (two filters can
// both be gathered for one topic only if, at every level both have, the
// levels are equal or one is a wildcard).  A solo entry is its client's
// merged delivery as is.
constexpr uint32_t kMetaMulti = 1u << 6;
// meta bit 7: Identifier > 0 — Subscription.Merge adds the entry to the
// client's Identifiers map (packets.go:257-259); becomes kWordIdent
constexpr uint32_t kMetaIdent = 1u << 7;

// delivery written by the matcher (one per (topic, client)), 4 bytes:
//   bits  0..27 sid of the first-merged subscription (its client is the
//               delivery's client: subs[sid].client)
//   bits 28..29 max QoS, bit 30 NoLocal (OR)
// A solo entry's delivery is its word & kPackedMask, precomputed in `words`,
// so the solo part of a topic is a plain copy of word ranges.  The dense form
// (densify) resolves the client: {client, packed}, 8 bytes.
constexpr uint32_t kSidBits = 28;
constexpr uint32_t kMaxSubs = 1u << kSidBits;

// Merge by resolution (match.hip k_resolve).  pinfo[sid] of a multi entry
// lists its partners — the other subscriptions of its client whose filters are
// level-compatible with its own (flatten.cpp mark_multi), i.e. every entry it
// can meet in one topic's gather (the parent-'#' double gather is gone:
// kFlagParentLit).  A partner is encoded as the multi-tail start of its
// node's range (the range start of the walk's multi part when that range is
// gathered) | QoS << 28 | NoLocal << 30: {p0, p1} inline for one or two
// partners, kNone when absent; {offset into partners, kPInfoList | count} for up to kMaxPartners;
// {kNone, kPInfoHeavy}: merged by hash table only (an inline partner has bit 31
// clear, so kPInfoList | count, kNone and kPInfoHeavy stay distinct).  A
// gathered entry whose gathered partners all come later in the reference's
// order (hit rank) is its client's first-merged entry and writes the delivery with every gathered
// partner's QoS / NoLocal folded in (packets.go:250-270); the others write
// nothing (partners sit on other nodes than the entry, so their hit ranks
// differ from its own).  Solo entries: {0, 0} (unused).
constexpr uint32_t kPInfoList = 0x80000000u, kPInfoHeavy = 0xFFFFFFFEu;
constexpr uint32_t kMaxPartners = 15;

struct DeviceSnapshot {
  const NodeDesc *nodes;
  // paired node slots, 64 B per node (derived on the device at upload):
  // slots[i] = {nodes[i], nodes[nodes[i].plus] (zeros without a '+' child)}.
  // The batch walk loads a '+' / '#' child's slot instead of its descriptor —
  // the same one 64-B sector, so the same one DRAM request — and gets that
  // child's own '+' child's descriptor with it: the next level's '+' item
  // then costs no load (C3: 2.1 of the 4.9 '+' loads per topic, and the
  // root's '+' child for every topic; tools/walk_census CENSUS_SLOTS=1)
  const NodeDesc *slots;
  const EdgeEntry *edges;
  const SubEnt *subs;
  const uint32_t *words;  // n_subs: subs[i].word & kPackedMask (the entry's own delivery)
  // bit i = subs[i].word & kWordIdent (Identifier > 0), 1 bit per entry
  // (1.25 MB at C3: stays in L2; the identifiers pass reads it instead of
  // the 8-B entries)
  const uint32_t *ident_bits;
  const uint8_t *tok_pool;
  uint64_t n_buckets;     // edge buckets (kEdgesPerBucket entries each; any count)
  // literal-edge existence filter, >= 16 bits per edge (64 MB at 10M filters:
  // it stays in the Infinity Cache), checked before a literal probe: half the
  // walk's probes are for tokens no edge has (random topic levels under a
  // node that also has a '+' child), and each would cost a DRAM request
  const uint2 *pinfo;     // n_subs: partners of a multi entry (above)
  const uint32_t *partners;
  const uint64_t *bloom;  // nullptr: no filter
  uint64_t bloom_mask;    // words - 1 (a power of two)
  uint32_t n_nodes;
  uint32_t n_subs;
  uint32_t n_shared;
  uint32_t height;        // max node depth (root = 0)
  // the store version this snapshot reflects.  MQM_SNAP_STAMP=1 (diagnostic):
  // the upload's last step writes it past the end of the nodes, subs and words
  // buffers and into a buffer of its own (stamp[0..3]; nullptr: off), and the
  // per-publish kernels compare each stamp with `version` (device.h
  // stamp_mismatch) — a reader of a retired snapshot whose recycled buffers
  // were refilled for a newer one sees another version there
  const unsigned long long *stamp[4];
  uint64_t version;
};

// one (token, depth) group of the reverse walk's literal-edge index
struct RevGroup {
  uint64_t k0, k1;    // the token's level key (keys.h); count == 0: empty slot
  uint32_t depth_len; // child depth | token length << 16 (long tokens: bytes verified)
  uint32_t tok_off;   // long tokens: bytes at tok_pool[tok_off ..)
  uint32_t start, count;  // its edges: inv[start, start + count)
};
static_assert(sizeof(RevGroup) == 32, "RevGroup layout");

// Retained-message side of the snapshot (TopicsIndex.Messages, topics.go:426-480),
// built only when the store holds retained messages.  Preorder ids make every
// subtree the contiguous id range [i, i + subtree[i]), so "all retained
// messages below a node" ('#') is a range of `refs`, located with `cum`.
struct DeviceRetained {
  const uint32_t *subtree;    // n_nodes: nodes in the subtree of i, i included
  const uint32_t *child_off;  // n_nodes + 1: children of i = child_ids[child_off[i] ..)
  const uint32_t *child_ids;  // in preorder
  const uint32_t *cum;        // n_nodes + 1: retained nodes with id < i
  const uint64_t *refs;       // n_ret + 1: message refs in preorder; refs[n_ret] = the
                              //   message retained at topic "" (has_empty), see below
  const uint32_t *rch_off;    // n_nodes + 1: retained children of i = rch_refs[rch_off[i] ..)
  const uint64_t *rch_refs;   // (the root's list leaves out the root child "$SYS")
  const uint8_t *nflags;      // n_nodes: NodeDesc flags (kFlagHasChildren, kFlagHasLiteral) of every
                              //   node, one byte each (79 MB at config 5: stays in the Infinity Cache),
                              //   so a wildcard's expansion drops children that cannot continue
                              //   without reading their descriptors
  uint64_t n_ret;
  // literal-edge index for a wildcard followed by a literal level: the edges
  // (parent, child) grouped by (child token, child depth), each group sorted
  // by parent.  Children of node p are the ids in (p, p + subtree[p]) at
  // depth(p) + 1, so "every child x of p, then the literal K under x" is one
  // binary-searched range of group (K, depth(p) + 2): no per-child probe.
  const uint2 *inv;           // {parent, child} per literal edge, by (group, parent)
  const struct RevGroup *groups;  // open-addressed (linear probing), n_gslots slots
  uint64_t n_gslots;          // 0: no index (the walk probes every child)
  uint32_t n_nodes;
  uint32_t sys_child;         // the root child named exactly "$SYS", or kNone
  uint32_t has_empty;         // a message is retained at topic "": its retainPath is ""
                              //   (topics.go:362), so Retained.Get(particle.retainPath) of
                              //   every literal-final node without one returns it (:474)
};

}  // namespace mqm
