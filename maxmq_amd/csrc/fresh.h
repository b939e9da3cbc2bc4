// maxmq_amd/csrc/fresh.h — read-your-writes for per-publish calls while the
// snapshot is rebuilt in the background (MQM_CFG_FRESH).
//
// The reference has no snapshot: a Subscribe is visible to the next
// Subscribers call (topics.go:303-321, 484-518).  With MQM_CFG_ASYNC_COMMIT a
// match reads the published snapshot, which lags the store by a rebuild (7 s
// at config 3 on 2 build threads: DESIGN §9).  The overlay closes that gap for
// mqm_subscribers without waiting for a build: it holds, for every client a
// mutation touched since the snapshot before the published one, that client's
// complete current subscription set, in a small trie keyed by the path each
// subscription is stored at.  A result matched on snapshot version Vs is
// corrected by
//   * dropping the deliveries, shared candidates and listed Identifiers of the
//     clients touched after Vs (their rows in the snapshot may be stale), and
//   * adding those clients' rows recomputed from the overlay: the reference's
//     scan (scanSubscribers, topics.go:493-518: {key, "+", "#"} per level,
//     gather at every visited node, the parent-"#" probe after a literal, the
//     "$" rule of gatherSubscriptions, topics.go:521-538) over their current
//     subscriptions, merged per client as Subscription.Merge does
//     (packets.go:250-270: first-gathered fields, QoS max, NoLocal or).
// Clients nobody touched since Vs keep their snapshot rows, which are current.
// The first time a mutation touches a client, its subscriptions are read from
// the published snapshot (HostSnapshot::client_off, built for fresh indexes)
// and the mutation is applied on top; later mutations update the set.  The
// overlay starts at the first publish (switched on again: at the first publish
// that has every mutation made while it was off); the clients mutated since
// that snapshot was built are read from the store then (load_dirty).  At each
// publish the clients whose last mutation is no newer than the previous
// snapshot are dropped, a few at each mutation: a result on the published or
// the previous snapshot still finds every client it needs; one on an older
// snapshot is retried.
//
// Who does what.  The mutating thread (index mutex held) turns each mutation
// into self-contained operations — a client's first touch carries its
// snapshot subscriptions, names resolved — and queues them; it decides which
// clients are held and dropped, so the overlay copies never read the store.
// An applier thread applies the queue every kApplyNs (or at kBatch queued).
// Calls never wait for it: the overlay is kept in kCopies copies
// (left-right), calls read the current copy, the applier brings a copy no
// call is in up to date from its log of operations and makes it current.
// (A third copy, so that a caller preempted inside a copy never holds the
// applier up, tripled the applier's work and lost: r06ad, r06ag.)  A call whose own thread made a mutation still queued waits for the
// applier (read-your-writes); other threads' mutations reach calls within
// about kApplyNs; every result reports the version it reflects.  (One
// reader-writer-locked overlay updated at every mutation, with 64 callers
// reading, held the mutations to 28k/s and the calls to 276k/s: r06q.)
#pragma once
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "flatten.h"
#include "store.h"

namespace mqm {

class FreshOverlay {
 public:
  static constexpr size_t kBatch = 1024;
  static constexpr int64_t kApplyNs = 250000;  // 0.25 ms

  FreshOverlay();
  ~FreshOverlay();  // stops the applier
  FreshOverlay(const FreshOverlay &) = delete;
  FreshOverlay &operator=(const FreshOverlay &) = delete;

  // ---- the mutating side: the index mutex held (it orders mutations and publishes) ----
  // a snapshot was published (hs built with a client index)
  void on_install(std::shared_ptr<const HostSnapshot> hs, const Store &st);
  // after Store::subscribe (its footprint is current)
  void on_subscribe(const Store &st, std::string_view filter, const SubRec &rec);
  // after a Store::unsubscribe that found its node (returned true)
  void on_unsubscribe(const Store &st, std::string_view filter);
  // any other mutation (RetainMessage): the version only
  void on_version(const Store &st);
  // mqm_fresh_policy: off drops the overlay (mutations cost nothing more); on
  // starts it again from the published snapshot
  void set_enabled(bool on, std::shared_ptr<const HostSnapshot> published, const Store &st);

  // ---- calls ----
  // a mutation of the calling thread is still queued: wait until it is applied
  void await_own_writes();
  // every operation queued so far applied (false: not within ms)
  bool await_all(int64_t ms);

  struct Gathered {
    uint32_t client;
    SubInfo info;
  };
  struct Match {
    uint64_t version = 0;  // store version the overlay reflects
    // per touched client with a row, first-gathered order: its first-merged
    // entry (index into subs), merged QoS and NoLocal
    struct Row {
      uint32_t client, first;
      uint8_t qos, no_local;
    };
    std::vector<Row> rows;
    std::vector<Gathered> subs;  // every gathered non-shared entry of a touched client, gather order
    std::vector<SubInfo> shared; // shared candidates of touched clients
  };

  // statistics: operations applied (per copy), applier rounds, calls
  // corrected, ns in their read sections (sum), clients held
  struct Stats {
    uint64_t ops, rounds, corrected, read_ns, held, match_ns;
    uint64_t max_age_ns, max_round_ns, max_wait_ns;  // oldest batch taken, longest round, longest wait for a free copy
  };
  Stats stats() const {
    return Stats{ops_.load(std::memory_order_relaxed),         rounds_.load(std::memory_order_relaxed),
                 corrected_.load(std::memory_order_relaxed),   read_ns_.load(std::memory_order_relaxed),
                 held_n_.load(std::memory_order_relaxed),      match_ns_.load(std::memory_order_relaxed),
                 max_age_ns_.load(std::memory_order_relaxed),  max_round_ns_.load(std::memory_order_relaxed),
                 max_wait_ns_.load(std::memory_order_relaxed)};
  }
  void count_match(uint64_t ns) const { match_ns_.fetch_add(ns, std::memory_order_relaxed); }
  void count_read(uint64_t ns) const {
    corrected_.fetch_add(1, std::memory_order_relaxed);
    read_ns_.fetch_add(ns, std::memory_order_relaxed);
  }

 private:
  static constexpr uint32_t kNone = 0xFFFFFFFFu;
  struct Load {  // a client's subscription as the snapshot has it
    std::string filter;
    uint8_t shared;
    SubInfo info;
  };
  struct Op {
    enum Kind : uint8_t { kPut, kDrop, kVersion, kInstall, kLoad, kPrune, kReset } kind;
    uint8_t shared = 0;
    uint32_t client = kNone;
    uint64_t version = 0;
    std::string filter;          // kPut / kDrop: the filter as called (path and group derived)
    SubInfo info{};              // kPut
    uint64_t floor = 0;          // kInstall (and the snapshot's node count: the copies' tables sized from it)
    uint64_t nodes_hint = 0;
    std::vector<Load> loads;     // kLoad
    uint64_t last = 0;           // kLoad at a start: the client's last mutation (else op.version)
    uint64_t seq = 0;            // queue order (await_own_writes)
  };
  // one copy of the overlay (written by the applier only)
  class State {
   public:
    void apply(const Op &op);
    int status(uint64_t vs) const {
      if (!active_) return 0;
      if (vs < floor_) return -1;
      return version_ > vs ? 1 : 0;
    }
    // held bit first (a 1.3-MB bitmap at config 3: the per-delivery check of
    // a result mostly stops there), then the client's last mutation
    bool touched(uint32_t c, uint64_t vs) const {
      return c < held_bits_.size() * 64 && ((held_bits_[c >> 6] >> (c & 63)) & 1) && last_mut_[c] > vs;
    }
    void match(std::string_view topic, uint64_t vs, Match *out) const;

   private:
    struct Ent {
      uint32_t client;
      uint32_t group;      // overlay token of the $SHARE group (shared), else kNone
      uint8_t shared;
      uint8_t dollar_skip; // non-shared filter starting with '+' or '#' (topics.go:527)
      SubInfo info;
    };
    struct Node {
      std::vector<Ent> ents;
      uint32_t plus = kNone, hash = kNone;  // the '+' / '#' child (no table probe for them)
    };
    // (parent << 32 | token) -> child: open addressing, insert-only
    // (the big arrays on 2-MB pages: a call's scan and checks are random reads
    // into tens of MB, a TLB miss each on 4-KB pages)
    template <class T>
    using HVec = std::vector<T, HugeAlloc<T>>;
    struct Kids {
      HVec<uint64_t> key = HVec<uint64_t>(1024, ~0ull);
      HVec<uint32_t> val = HVec<uint32_t>(1024, 0);
      uint64_t n = 0;
      static uint64_t mix(uint64_t k) {
        k ^= k >> 31;
        k *= 0x9E3779B97F4A7C15ull;
        return k ^ (k >> 29);
      }
      uint32_t find(uint64_t k) const {
        const uint64_t m = key.size() - 1;
        for (uint64_t i = mix(k) & m;; i = (i + 1) & m) {
          if (key[i] == k) return val[i];
          if (key[i] == ~0ull) return kNone;
        }
      }
      void insert(uint64_t k, uint32_t v);
      void reserve(uint64_t slots);  // (a rehash inside a round delays every call's view)
    };
    uint32_t token(std::string_view s, bool create);
    uint32_t find_token(std::string_view s) const;
    uint32_t child(uint32_t parent, uint32_t tok) const { return kids_.find((uint64_t)parent << 32 | tok); }
    uint32_t path(std::string_view filter, int d, bool create);
    void put_sub(uint32_t client, std::string_view filter, uint8_t shared, const SubInfo &si);
    void stamp(uint32_t client, uint64_t v);  // last_mut_ and the held bit
    void put(uint32_t node, const Ent &e);
    void drop(uint32_t node, uint32_t client, uint8_t shared, uint32_t group);
    void gather(uint32_t node, std::string_view topic, uint64_t vs, bool with_shared, Match *m,
                std::unordered_map<uint32_t, uint32_t> *row_of) const;
    void scan(std::string_view topic, const uint32_t *lt, int nl, int d, uint32_t node, uint64_t vs, Match *m,
              std::unordered_map<uint32_t, uint32_t> *row_of) const;

    bool active_ = false;
    uint64_t floor_ = 0;    // results on snapshots older than this are retried
    uint64_t version_ = 0;  // the store version the overlay reflects
    HVec<uint64_t> last_mut_;   // by client: the version after its last mutation (0: not held)
    HVec<uint64_t> held_bits_;  // by client: held (last_mut_ != 0)
    std::unordered_map<uint32_t, std::vector<uint32_t>> held_;  // client -> nodes holding its entries
    // the trie: nodes, (parent, token) -> child, tokens by hash (chained)
    HVec<Node> nodes_{Node()};
    Kids kids_;
    std::vector<std::string> tok_str_;
    std::vector<uint32_t> tok_next_;
    std::unordered_map<uint64_t, uint32_t> tok_head_;
    int32_t hash_tok_ = -1, plus_tok_ = -1;
  };

  // the mutating side (index mutex)
  void enqueue(Op &&op);
  void emit_prunes(size_t n);
  void hold(const Store &st, uint32_t c, uint64_t v);  // a Load op at a client's first touch
  void load_dirty(const Store &st);                    // at a start: the clients mutated since its snapshot
  bool enabled_ = true, mactive_ = false;
  std::shared_ptr<const HostSnapshot> mbase_;
  uint64_t mfloor_ = 0, queued_version_ = 0;
  std::unordered_map<uint32_t, uint64_t> mirror_;  // held clients -> their last mutation's version
  std::vector<uint32_t> mprune_;                   // candidates to drop (last mutation <= floor at a publish)
  // not holding clients yet (no snapshot, or on again): the clients mutated
  // meanwhile, and the version a snapshot must have to start from (0: any)
  std::unordered_map<uint32_t, uint64_t> mdirty_;
  uint64_t mwait_ = 0;
  std::atomic<uint64_t> held_n_{0};
  // the queue (qmu_) and the applier
  std::mutex qmu_;
  std::condition_variable qcv_, done_cv_;
  std::vector<Op> q_;
  std::atomic<int64_t> oldest_ns_{0};
  std::mutex round_mu_;  // one round at a time (the applier, or a call helping)
  bool urgent_ = false, stop_ = false;
  std::atomic<uint64_t> applied_{0};    // the newest version the current copy holds
  std::atomic<uint64_t> seq_{0}, applied_seq_{0};  // operations queued / in the current copy
  void run();
  void round(std::vector<Op> &batch);
  bool await_seq(uint64_t w, int64_t ms);
  // the copies, the operations since the least up-to-date one (applier)
  static constexpr int kCopies = 2;
  State s_[kCopies];
  std::atomic<int> cur_{0};
  std::vector<Op> log_;       // operations log_base_ .. log_base_ + log_.size()
  uint64_t log_base_ = 0;
  uint64_t pos_[kCopies] = {};  // operations each copy holds (absolute)
  // calls inside each copy, counted in per-thread slots (64 callers on one
  // counter made its cache line the hot spot)
  static constexpr int kSlots = 16;
  struct alignas(64) Count {
    std::atomic<int> n{0};
  };
  mutable Count readers_[kCopies][kSlots];
  static int slot();
  bool drained(int copy) const {
    for (int k = 0; k < kSlots; k++)
      if (readers_[copy][k].n.load(std::memory_order_seq_cst) != 0) return false;
    return true;
  }
  std::atomic<uint64_t> ops_{0}, rounds_{0}, max_age_ns_{0}, max_round_ns_{0}, max_wait_ns_{0};
  mutable std::atomic<uint64_t> corrected_{0}, read_ns_{0}, match_ns_{0};
  std::thread th_;

 public:
  class Reader {
   public:
    explicit Reader(const FreshOverlay &o) : o_(o), k_(slot()) {
      for (;;) {  // (left-right: enter the current copy, then check it still is)
        i_ = o.cur_.load(std::memory_order_seq_cst);
        o.readers_[i_][k_].n.fetch_add(1, std::memory_order_seq_cst);
        if (o.cur_.load(std::memory_order_seq_cst) == i_) break;
        o.readers_[i_][k_].n.fetch_sub(1, std::memory_order_seq_cst);
      }
    }
    ~Reader() { o_.readers_[i_][k_].n.fetch_sub(1, std::memory_order_release); }
    Reader(const Reader &) = delete;
    Reader &operator=(const Reader &) = delete;
    // 0: nothing newer than vs (or no overlay), 1: correct the result, -1: vs
    // is older than the overlay covers (match again on the newer snapshot)
    int status(uint64_t vs) const { return o_.s_[i_].status(vs); }
    bool touched(uint32_t client, uint64_t vs) const { return o_.s_[i_].touched(client, vs); }
    void match(std::string_view topic, uint64_t vs, Match *out) const { o_.s_[i_].match(topic, vs, out); }

   private:
    const FreshOverlay &o_;
    int k_, i_ = 0;
  };
};

}  // namespace mqm
