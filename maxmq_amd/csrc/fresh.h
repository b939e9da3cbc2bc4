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
// and the mutation is applied on top; later mutations update the set.  At each
// publish the clients whose last mutation is no newer than the previous
// snapshot are dropped: a result on the published or the previous snapshot
// still finds every client it needs; one on an older snapshot is retried.
#pragma once
#include <stdint.h>

#include <memory>
#include <shared_mutex>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "flatten.h"
#include "store.h"

namespace mqm {

class FreshOverlay {
 public:
  // ---- writers: the index mutex held (it orders mutations and publishes) ----
  // a snapshot was published (hs built with a client index)
  void on_install(std::shared_ptr<const HostSnapshot> hs, const Store &st);
  // after Store::subscribe (its footprint is current)
  void on_subscribe(const Store &st, std::string_view filter, const SubRec &rec);
  // after a Store::unsubscribe that found its node (returned true)
  void on_unsubscribe(const Store &st, std::string_view filter);
  // any other mutation (RetainMessage): the version only
  void on_version(const Store &st);

  // ---- readers ----
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
  class Reader {
   public:
    explicit Reader(const FreshOverlay &o) : o_(o), lk_(o.rw_) {}
    // 0: nothing newer than vs (or no overlay), 1: correct the result, -1: vs
    // is older than the overlay covers (match again on the newer snapshot)
    int status(uint64_t vs) const;
    bool touched(uint32_t client, uint64_t vs) const {
      return client < o_.last_mut_.size() && o_.last_mut_[client] > vs;
    }
    void match(std::string_view topic, uint64_t vs, Match *out) const;

   private:
    const FreshOverlay &o_;
    std::shared_lock<std::shared_mutex> lk_;
  };

  // statistics (writers' lock not needed: approximate)
  uint64_t clients() const { return n_clients_; }

 private:
  static constexpr uint32_t kNone = 0xFFFFFFFFu;
  struct Ent {
    uint32_t client;
    uint32_t group;      // overlay token of the $SHARE group (shared), else kNone
    uint8_t shared;
    uint8_t dollar_skip; // non-shared filter starting with '+' or '#' (topics.go:527)
    SubInfo info;
  };
  struct Node {
    std::vector<Ent> ents;
  };
  uint32_t token(std::string_view s, bool create);
  uint32_t child(uint32_t parent, uint32_t tok) const;
  uint32_t path(std::string_view filter, int d, bool create);
  void touch(const Store &st, uint32_t client);
  void put(uint32_t node, const Ent &e);
  void drop(uint32_t node, uint32_t client, uint8_t shared, uint32_t group);
  void gather(uint32_t node, std::string_view topic, uint64_t vs, bool with_shared, Match *m,
              std::unordered_map<uint32_t, uint32_t> *row_of) const;
  void scan(std::string_view topic, int d, uint32_t node, uint64_t vs, Match *m,
            std::unordered_map<uint32_t, uint32_t> *row_of) const;

  mutable std::shared_mutex rw_;
  bool active_ = false;
  std::shared_ptr<const HostSnapshot> base_;  // the published snapshot
  uint64_t floor_ = 0;    // results on snapshots older than this are retried
  uint64_t version_ = 0;  // the store version the overlay reflects
  std::vector<uint64_t> last_mut_;  // by client: the version after its last mutation (0: not held)
  std::unordered_map<uint32_t, std::vector<uint32_t>> held_;  // client -> nodes holding its entries
  uint64_t n_clients_ = 0;
  // the trie: nodes, (parent, token) -> child, tokens by hash (chained)
  std::vector<Node> nodes_{Node()};
  std::unordered_map<uint64_t, uint32_t> kids_;
  std::vector<std::string> tok_str_;
  std::vector<uint32_t> tok_next_;
  std::unordered_map<uint64_t, uint32_t> tok_head_;
  int32_t hash_tok_ = -1, plus_tok_ = -1;
};

}  // namespace mqm
