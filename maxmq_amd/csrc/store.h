// maxmq_amd/csrc/store.h — host-authoritative subscription/retained store.
//
// The mutable side of the drop-in: it keeps the reference's trie SHAPE and
// mutation semantics (vendor/github.com/mochi-co/mqtt/v2/topics.go:303-423)
// so Subscribe/Unsubscribe/RetainMessage return exactly what the reference
// returns, and it is what the snapshot builder (flatten.cpp) turns into the
// GPU-resident CSR level-trie.  Strings are interned: tokens (level keys),
// clients and filters each get dense u32 ids in first-appearance order.
#pragma once
#include <atomic>
#include <stdint.h>
#include <sys/mman.h>

#include <memory>
#include <new>

#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

namespace mqm {

// std::allocator whose large blocks (>= 4 MB) are 2-MB aligned anonymous
// mappings marked MADV_HUGEPAGE: the flatten reads the node array (3.7 GB at
// C3) and its own per-node arrays in store-id or preorder order, i.e. at
// random in the other, and with 4-KB pages nearly every such read also
// missed the TLB
template <class T>
struct HugeAlloc : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = HugeAlloc<U>;
  };
  static constexpr size_t kHuge = 2ull << 20, kMin = 4ull << 20;
  HugeAlloc() = default;
  template <class U>
  HugeAlloc(const HugeAlloc<U> &) {}
  static size_t span(size_t n) { return (n * sizeof(T) + kHuge - 1) & ~(kHuge - 1); }
  T *allocate(size_t n) {
    if (n * sizeof(T) < kMin) return std::allocator<T>::allocate(n);
    const size_t len = span(n);
    char *base = (char *)mmap(nullptr, len + kHuge, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (base == MAP_FAILED) throw std::bad_alloc();
    char *p = (char *)(((uintptr_t)base + kHuge - 1) & ~(uintptr_t)(kHuge - 1));
    if (p > base) munmap(base, (size_t)(p - base));  // trim to the aligned span
    if (base + len + kHuge > p + len) munmap(p + len, (size_t)(base + len + kHuge - (p + len)));
    (void)madvise(p, len, MADV_HUGEPAGE);
    return (T *)p;
  }
  void deallocate(T *p, size_t n) {
    if (n * sizeof(T) < kMin) return std::allocator<T>::deallocate(p, n);
    munmap((void *)p, span(n));
  }
};
template <class T, class U>
bool operator==(const HugeAlloc<T> &, const HugeAlloc<U> &) { return true; }
template <class T, class U>
bool operator!=(const HugeAlloc<T> &, const HugeAlloc<U> &) { return false; }

using U32Vec = std::vector<uint32_t, HugeAlloc<uint32_t>>;

struct SubRec {       // packets.Subscription (packets.go:168-178), interned
  uint32_t client;
  uint32_t filter;
  int32_t ident;
  uint8_t qos, no_local, rap, rh;
};

struct SharedRec {
  uint32_t group;     // token id of the $SHARE group name
  SubRec sub;
};

struct HNode {        // particle (topics.go:627-635)
  uint32_t key = 0;   // token id
  uint32_t parent = 0xFFFFFFFFu;
  uint32_t first_child = 0xFFFFFFFFu, next_sibling = 0xFFFFFFFFu, prev_sibling = 0xFFFFFFFFu;
  uint32_t n_children = 0;
  uint32_t depth = 0;
  uint32_t subtree = 1;          // nodes in the subtree rooted here (itself included; flatten's preorder bases)
  bool retain_path = false;      // retainPath != ""
  uint64_t ret_ref = 0;          // caller's message ref of the retained packet (retain_path)
  bool live = false;
  std::vector<SubRec> subs;      // particle.subscriptions, unique by client
  std::vector<SharedRec> shared; // particle.shared, unique by (group, client)
};

// string -> dense id, first-appearance order.  Bytes live in one arena; the
// index is an open-addressed table of (hash, id) probed with string_views, so
// lookups allocate nothing.
class Interner {
 public:
  uint32_t intern(std::string_view s);
  uint32_t find(std::string_view s) const;  // kNone if absent
  std::string_view name(uint32_t id) const {
    return std::string_view(arena_.data() + offs_[id], offs_[id + 1] - offs_[id]);
  }
  uint32_t size() const { return (uint32_t)(offs_.size() - 1); }

 private:
  uint64_t slot_of(std::string_view s, uint64_t h) const;
  void grow();
  std::vector<char> arena_;
  std::vector<uint64_t> offs_{0};
  std::vector<uint64_t> table_;  // (hash high 32 bits << 32) | (id + 1); 0 = empty
};

// (parent << 32 | token) -> child: open addressing, linear probing,
// backward-shift deletion (no tombstones), so lookups on the mutation path
// touch one or two cache lines instead of a node-based bucket chain.
class EdgeMap {
 public:
  uint32_t find(uint64_t key) const;  // kNone if absent
  void insert(uint64_t key, uint32_t val);  // key must be absent
  void erase(uint64_t key);
  uint64_t size() const { return n_; }

 private:
  void grow();
  static uint64_t mix(uint64_t k) {
    k ^= k >> 31;
    k *= 0x9E3779B97F4A7C15ull;
    return k ^ (k >> 29);
  }
  std::vector<uint64_t> keys_;  // ~0 = empty
  std::vector<uint32_t> vals_;
  uint64_t n_ = 0, mask_ = 0;
};

struct RetainedRec {
  uint64_t msg_ref;
  uint32_t payload_len;
  bool retain_flag;
};

class Store {
 public:
  Store();

  bool subscribe(std::string_view client, std::string_view filter, uint8_t qos, uint8_t no_local, uint8_t rap,
                 uint8_t rh, int32_t ident);                                   // topics.go:303-321
  bool unsubscribe(std::string_view filter, std::string_view client);         // topics.go:325-349
  // What the last subscribe / unsubscribe touched: its node, the client's,
  // filter's and share group's interned ids, whether it was a shared
  // subscription, and whether it changed anything but that node's lists (a
  // node created or removed, a string interned for the first time).  A store
  // replaying the same calls in the same order (the builder's shadow) holds
  // the same ids, so a call that was not `structural` can be replayed on the
  // node directly (subscribe_at / unsubscribe_at) instead of walking the path.
  struct Footprint {
    uint32_t node = 0xFFFFFFFFu, client = 0xFFFFFFFFu, filter = 0xFFFFFFFFu, group = 0xFFFFFFFFu;
    bool shared = false, structural = true;
  };
  const Footprint &last_footprint() const { return last_; }
  bool subscribe_at(const Footprint &fp, uint8_t qos, uint8_t no_local, uint8_t rap, uint8_t rh, int32_t ident);
  void unsubscribe_at(const Footprint &fp);
  int64_t retain_message(std::string_view topic, uint64_t msg_ref, uint32_t payload_len,
                         bool retain_flag);                                    // topics.go:354-377
  uint64_t retained_len() const { return retained_.size(); }

  const Interner &tokens() const { return tokens_; }
  const Interner &clients() const { return clients_; }
  const Interner &filters() const { return filters_; }
  const std::vector<HNode, HugeAlloc<HNode>> &nodes() const { return nodes_; }
  uint32_t root() const { return 0; }
  // moves whenever a node is created or removed (the trie's shape, which
  // flatten's preorder and edge list depend on; subscriptions do not move it)
  uint64_t structure_version() const { return structure_version_; }
  uint32_t plus_token() const { return plus_tok_; }
  uint32_t hash_token() const { return hash_tok_; }
  uint32_t child(uint32_t parent, uint32_t tok) const;
  uint64_t version() const { return version_.v.load(std::memory_order_acquire); }
  const std::unordered_map<std::string, RetainedRec> &retained() const { return retained_; }

 private:
  uint32_t set_path(std::string_view s, int d);          // set  (topics.go:380-397)
  uint32_t seek_path(std::string_view s, int d) const;   // seek (topics.go:400-414)
  void trim(uint32_t n);                                 // trim (topics.go:417-423)
  void drop_sub(const Footprint &fp);
  uint32_t new_node(uint32_t parent, uint32_t tok);
  void unlink(uint32_t n);

  std::vector<HNode, HugeAlloc<HNode>> nodes_;
  uint64_t structure_version_ = 0;
  Footprint last_;
  // sizes that a structural call moves (Footprint::structural)
  uint64_t shape_mark() const {
    return structure_version_ + tokens_.size() + clients_.size() + filters_.size();
  }
  std::vector<uint32_t> free_;
  EdgeMap children_;
  Interner tokens_, clients_, filters_;
  std::unordered_map<std::string, RetainedRec> retained_;  // packets.Packets (Retained)
  uint32_t plus_tok_, hash_tok_;
  // bumped by every mutation (under the index lock); read without it by the
  // per-publish server's snapshot check (capi.cpp front_fast)
  struct Version {
    std::atomic<uint64_t> v{0};
    Version() = default;
    Version(const Version &o) : v(o.v.load(std::memory_order_relaxed)) {}
    Version &operator=(const Version &o) {
      v.store(o.v.load(std::memory_order_relaxed), std::memory_order_relaxed);
      return *this;
    }
  } version_;
};

// isolateParticle (topics.go:558-577) over a byte string: level d and hasNext.
bool isolate_particle(std::string_view s, int d, std::string_view *out);
// strings.EqualFold(level, "$SHARE") with Go's simple folding (U+017F ~ 's')
bool equal_fold_share(std::string_view s);
bool is_valid_filter(std::string_view f, bool for_publish);  // topics.go:586-624
bool is_shared_filter(std::string_view f);                   // topics.go:580-583

}  // namespace mqm
