// maxmq_amd/csrc/flatten.h — host store -> GPU-resident CSR level-trie.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <memory>
#include <utility>
#include <vector>

#include "snapshot.h"
#include "store.h"

namespace mqm {

// an allocator that default-initialises (no zero fill): the big snapshot
// arrays are first touched by the threads that fill them (huge pages: HugeAlloc)
template <class T>
struct NoInitAlloc : HugeAlloc<T> {
  template <class U>
  struct rebind {
    using other = NoInitAlloc<U>;
  };
  NoInitAlloc() = default;
  template <class U>
  NoInitAlloc(const NoInitAlloc<U> &) {}
  template <class U, class... A>
  void construct(U *p, A &&...a) {
    if constexpr (sizeof...(A) == 0)
      ::new ((void *)p) U;
    else
      ::new ((void *)p) U(std::forward<A>(a)...);
  }
};

// per-subscription side information, kept on the host to resolve result ids
struct SubInfo {
  uint32_t filter;
  uint32_t client;
  int32_t ident;
  uint8_t qos, no_local, rap, rh;
};

using EdgeVec = std::vector<EdgeEntry, NoInitAlloc<EdgeEntry>>;

struct HostSnapshot {
  std::vector<NodeDesc, NoInitAlloc<NodeDesc>> nodes;  // (every field is written by flatten)
  EdgeVec edges;   // n_buckets * kEdgesPerBucket (empty after upload, and when built on the device)
  // the literal edges in (parent store id, child store id) order, while the
  // device builds the table (shared with the builder's FlattenCache)
  std::shared_ptr<EdgeVec> staged;
  uint64_t edges_digest = 0;  // edges_digest_of(edges), kept when the host copy is released
  std::vector<SubEnt> subs;
  std::vector<uint32_t> words;       // subs[i].word & kPackedMask (mqm_result_runs: a run's deliveries)
  std::vector<SubInfo> sub_info;     // by non-shared sid
  std::vector<SubInfo> shared_info;  // by shared sid
  std::vector<uint8_t> tok_pool;
  std::vector<uint64_t> bloom;       // DeviceSnapshot::bloom (empty: none)
  std::vector<uint2> pinfo;          // DeviceSnapshot::pinfo (by final sid)
  std::vector<uint32_t> partners;    // DeviceSnapshot::partners
  uint64_t n_buckets = 0;
  uint32_t height = 0;
  uint64_t n_edges = 0;
  uint64_t n_solo = 0;  // subscriptions without kMetaMulti
  // retained side (DeviceRetained), empty when nothing is retained
  std::vector<uint32_t> subtree, child_off, child_ids, cum, rch_off;
  std::vector<uint64_t> refs, rch_refs;
  std::vector<uint2> rinv;           // DeviceRetained::inv
  std::vector<RevGroup> rgroups;     // DeviceRetained::groups (empty: no index)
  uint32_t sys_child = kNone;
  bool has_empty = false;
  // the store version this snapshot reflects (set by the committer after
  // flatten; equal versions mean equal snapshots: flatten is deterministic)
  uint64_t version = 0;
  // MQM_CFG_FRESH (fresh.h): the subscriptions by client, built after flatten
  // (build_client_index) — client c's sids at client_subs[client_off[c] ..
  // client_off[c + 1]), its shared sids likewise; empty when not built
  std::vector<uint32_t> client_off, client_subs, client_shoff, client_shared;
};

// What a rebuild of the same trie shape can reuse (the background builder
// keeps one): the preorder numbering, the staged edge list (its inline child
// descriptors refreshed) and the edge filter.  Valid while the store's
// structure_version and token count are those it was built at, no message is
// retained and the table is built where it was.  Subscribe / Unsubscribe of
// filters that exist (and keep other subscribers) leave the shape alone.
// a node's children (flatten.cpp): literal ones at lch[off, off + cnt)
struct FlatKids {
  uint32_t off, cnt;
  uint32_t pc, hc;  // '+' / '#' child (kNone: none)
};
using ScratchU32 = std::vector<uint32_t, NoInitAlloc<uint32_t>>;

struct FlattenCache {
  bool valid = false;
  uint64_t structure = 0, n_tokens = 0;
  bool host_edges = false;
  U32Vec order, new_id, pc_of, hc_of, nlit;
  std::shared_ptr<EdgeVec> staged;
  std::vector<uint64_t> bloom;
  uint64_t reuses = 0;  // builds that took the cache (statistics)
  // working arrays kept from build to build (their pages stay mapped: a fresh
  // 2-MB page costs its zeroing and, when memory is fragmented, compaction)
  std::vector<FlatKids, NoInitAlloc<FlatKids>> kid;
  ScratchU32 lpar, ktok, lch, kch;
};

// Build the snapshot; returns MQM_OK or MQM_ELIMIT.  host_edges = false: the
// edge table is left to upload(), which builds it on the device from
// `staged` (the host fill of the table and its transfer were most of a
// rebuild: 18.5 GB at config 3 against 2.2 GB of staged edges).
int flatten(const Store &st, HostSnapshot *out, bool host_edges = true, FlattenCache *cache = nullptr);
// the snapshot's subscriptions by client (HostSnapshot::client_off ..), for
// the fresh overlay's first look at a client (fresh.h)
void build_client_index(HostSnapshot &hs);
// MQM_HOST_EDGES=1 (A/B, diagnostics): the edge table is built on the host
// and copied, never on the device (edges.hip)
bool host_edges_forced();
// the edge table from the staged edges, on the host (snapshot.h layout)
void insert_edges_host(HostSnapshot &hs, const EdgeVec &staged);
// the same table built on the device into `table` (n_buckets * kEdgesPerBucket
// slots) from the staged edges (host memory: copied in first), and its digest
// (the sum of edge_slot_mix over the slots); 1: a partition's run-past list
// overflowed its buffer (the caller builds the table on the host instead).
// The staged copy and every temporary live in a per-device scratch region
// that is kept from build to build (edges.hip; MQM_EDGE_POOL=1: the
// stream-ordered pool instead, round 5's form)
int build_edges_device(const EdgeEntry *h_staged, uint64_t n_edges, uint64_t n_buckets, EdgeEntry *table,
                       hipStream_t stream, uint64_t *digest_sum);
// host threads a flatten (and the snapshot digest) runs on: mqm_build_threads,
// else MQM_BUILD_THREADS, else min(16, hardware threads)
uint32_t build_threads();
void set_build_threads(uint32_t n);  // 0: back to the default
void serve_count(int delta);         // a per-publish server started (+1) / stopped (-1): the default drops to 4

// Device copy of a HostSnapshot.  Host side tables stay shared with results
// (shared_ptr) so a result can outlive the next commit.
struct GpuSnapshot {
  DeviceSnapshot dev{};
  std::shared_ptr<const HostSnapshot> host;
  static constexpr int kNumBuffers = 13;
  void *buffers[kNumBuffers] = {};
  void *words = nullptr;  // DeviceSnapshot::words (derived on the device at upload)
  void *slots = nullptr;  // DeviceSnapshot::slots (derived on the device at upload)
  void *ident_bits = nullptr;  // DeviceSnapshot::ident_bits (derived on the device at upload)
  void *nflags = nullptr; // DeviceRetained::nflags (derived on the device at upload)
  void *bloom = nullptr;  // DeviceSnapshot::bloom
  void *pinfo = nullptr, *partners = nullptr;  // DeviceSnapshot::pinfo / partners
  DeviceRetained ret{};
  bool has_retained = false;
  int device = -1;  // the buffers' device
  std::vector<std::pair<void *, size_t>> held;  // every device buffer above, with its capacity (recycled)
  uint64_t device_bytes = 0;
  uint64_t stamp_host = 0;  // MQM_SNAP_STAMP=1: the copy source of the stamps (lives as long as the copies)
  ~GpuSnapshot();
};

// Device buffers of a destroyed snapshot, freed later by the index layer
// (capi.cpp): hipFree waits for every kernel on the device, the per-publish
// server included, so the frees run on a thread of their own with the
// servers stopped.
void retire_device_buffers(int device, std::vector<void *> bufs);

// Copies on `stream` and waits for them (nullptr: the null stream).  device < 0
// (MQM_DEVICE_NONE) wraps the host snapshot without device buffers, so a
// host-only index still has stats and a digest.
// The host copy of the edge table (the snapshot's largest array: 18.5 GB at
// config 3) is released once it is on the device; its digest is kept.
int upload(std::shared_ptr<HostSnapshot> hs, int device, hipStream_t stream, std::unique_ptr<GpuSnapshot> *out);

}  // namespace mqm
