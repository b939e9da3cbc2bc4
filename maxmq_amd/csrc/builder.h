// maxmq_amd/csrc/builder.h — delta log + background snapshot builder
// (incremental Subscribe/Unsubscribe at rate).
//
// The reference mutates its live trie under the root mutex and readers see a
// change at once (topics.go:303-349,354-377; no snapshot).  Here the
// authoritative Store answers every mutation with the reference's return
// value, and the mutation is also appended to a DeltaLog.  A commit hands the
// log to the Builder's worker thread, which replays it into a private shadow
// Store (same calls, same order, so the same interned ids and trie shape),
// flattens the shadow into a new HostSnapshot and uploads it on its own HIP
// stream into the back buffer.  The index publishes the back buffer at its
// next call (double buffering): matches keep running against the front
// snapshot while the next one is built, and no mutation waits for a rebuild.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string_view>
#include <thread>
#include <vector>

#include "flatten.h"
#include "store.h"

namespace mqm {

// Store mutations in call order; strings packed into one arena.
class DeltaLog {
 public:
  // fp: the authoritative store's footprint of the call just made
  // (Store::last_footprint); a call that was not structural is replayed on its
  // node directly (no path walk, no interning)
  void subscribe(std::string_view client, std::string_view filter, uint8_t qos, uint8_t no_local, uint8_t rap,
                 uint8_t rh, int32_t ident, const Store::Footprint *fp = nullptr);
  void unsubscribe(std::string_view filter, std::string_view client, const Store::Footprint *fp = nullptr);
  uint64_t fast_ops() const { return fast_; }  // calls recorded with a usable footprint (statistics)
  void retain(std::string_view topic, uint64_t msg_ref, uint32_t payload_len, bool retain_flag);
  // re-run the first `limit` recorded calls on st, in order
  void replay(Store &st, size_t limit = SIZE_MAX) const;
  void append(DeltaLog &&o);  // o's ops after ours
  size_t size() const { return ops_.size(); }
  bool empty() const { return ops_.empty(); }
  void clear() {
    ops_.clear();
    bytes_.clear();
    fast_ = 0;
  }

 private:
  enum Kind : uint8_t { kSub, kUnsub, kRetain };
  struct Op {
    uint8_t kind, qos, no_local, rap, rh, retain_flag;
    int32_t ident;
    uint32_t payload_len;
    uint32_t a_len, b_len;  // strings at bytes_[a_off ..), then b
    uint64_t a_off;
    uint64_t msg_ref;
    Store::Footprint fp;    // fp.structural: replay by the strings
  };
  Op &push(Kind k, std::string_view a, std::string_view b);
  std::vector<Op> ops_;
  std::vector<char> bytes_;
  uint64_t fast_ = 0;
};

// A snapshot ready to be published: device copy (or host-only when the index
// has no device) plus the store version it reflects.
struct BuiltSnapshot {
  std::unique_ptr<GpuSnapshot> snap;
  uint64_t version = 0;
  double build_ms = 0;  // replay + flatten + upload
  double phase_ms[3] = {0, 0, 0};  // replay, flatten, upload
  bool kept_shape = false;         // the flatten reused the previous build's preorder and edges (FlattenCache)
  uint64_t n_ops = 0;   // delta-log entries folded in
};

class Builder {
 public:
  explicit Builder(int device);  // device < 0: host snapshots only
  ~Builder();                    // finishes the queued work, joins the worker
  Builder(const Builder &) = delete;
  Builder &operator=(const Builder &) = delete;

  // queue a delta log whose replay brings the shadow store to `version`
  void submit(DeltaLog &&log, uint64_t version);
  // replace the shadow store with a copy of the authoritative one (taken by the
  // caller under the index mutex, so it holds every mutation up to `version`);
  // queued logs are dropped: the copy already contains them
  void submit_full(const Store &st, uint64_t version);
  // the last build failed: the next commit must build even with an empty log
  bool dirty();
  // a replay failed part-way: the shadow store no longer mirrors the
  // authoritative one, and only submit_full repairs it (plain logs are refused)
  bool shadow_bad();
  // fault injection for tests (mqm_debug_fault): the next `count` builds fail
  // in `stage` (1 = part-way through the replay, 2 = flatten, 3 = upload)
  void inject_fault(int stage, int count);
  // the newest finished snapshot, if any (older unpublished ones are dropped)
  bool take(BuiltSnapshot *out);
  // take() would return a snapshot (no lock: the per-publish path checks it per call)
  bool has_ready() const { return ready_flag_.load(std::memory_order_acquire); }
  // block until every submitted log is built; returns the first build error
  int wait_idle();
  bool busy();
  // builds also index their subscriptions by client (MQM_CFG_FRESH: fresh.h)
  void set_client_index(bool on) { client_index_.store(on, std::memory_order_relaxed); }

 private:
  void run();
  const int device_;
  Store shadow_;  // touched only by the worker thread
  FlattenCache shape_;  // the last build's preorder and edge list (worker thread)
  hipStream_t stream_ = nullptr;
  std::mutex mu_;
  std::condition_variable cv_;
  DeltaLog queued_;
  std::unique_ptr<Store> full_;  // submit_full's copy, applied before queued_
  uint64_t queued_version_ = 0;
  bool has_queued_ = false, working_ = false, stop_ = false;
  bool dirty_ = false, shadow_bad_ = false;
  bool has_ready_ = false;
  std::atomic<bool> ready_flag_{false};  // has_ready_, readable without mu_
  std::atomic<bool> client_index_{false};
  BuiltSnapshot ready_;
  int err_ = 0;
  int fault_stage_ = 0, fault_count_ = 0;
  std::thread th_;
};

// 64-bit digest of a snapshot's arrays (replicas / shards compare it)
uint64_t snapshot_digest(const HostSnapshot &hs);
// digest of the edge table (a sum of per-slot terms, so the host's chunks and
// the device's reduction agree); snapshot_digest uses the kept value once the
// host copy is released or when the device built the table
uint64_t edges_digest_of(const HostSnapshot &hs);
// its parts: the sum of edge_slot_mix over the slots (snapshot.h; the device
// computes the same sum), then the final mix with the slot count
uint64_t edges_digest_sum(const EdgeEntry *edges, uint64_t n);
uint64_t edges_digest_final(uint64_t sum, uint64_t n);

}  // namespace mqm
