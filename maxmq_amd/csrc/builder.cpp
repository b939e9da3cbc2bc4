// maxmq_amd/csrc/builder.cpp — delta log replay and the background snapshot
// builder (see builder.h).
#include "builder.h"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <new>
#include <thread>

#include <sys/resource.h>
#include <sys/syscall.h>
#include <unistd.h>

#include "../../include/mqmatch.h"

namespace mqm {

DeltaLog::Op &DeltaLog::push(Kind k, std::string_view a, std::string_view b) {
  Op op{};
  op.kind = k;
  op.a_off = bytes_.size();
  op.a_len = (uint32_t)a.size();
  op.b_len = (uint32_t)b.size();
  bytes_.insert(bytes_.end(), a.begin(), a.end());
  bytes_.insert(bytes_.end(), b.begin(), b.end());
  ops_.push_back(op);
  return ops_.back();
}

void DeltaLog::subscribe(std::string_view client, std::string_view filter, uint8_t qos, uint8_t no_local,
                         uint8_t rap, uint8_t rh, int32_t ident, const Store::Footprint *fp) {
  Op &op = push(kSub, client, filter);
  op.qos = qos;
  op.no_local = no_local;
  op.rap = rap;
  op.rh = rh;
  op.ident = ident;
  if (fp) op.fp = *fp;
  fast_ += !op.fp.structural;
}

void DeltaLog::unsubscribe(std::string_view filter, std::string_view client, const Store::Footprint *fp) {
  Op &op = push(kUnsub, filter, client);
  if (fp) op.fp = *fp;
  fast_ += !op.fp.structural;
}

void DeltaLog::retain(std::string_view topic, uint64_t msg_ref, uint32_t payload_len, bool retain_flag) {
  Op &op = push(kRetain, topic, std::string_view());
  op.msg_ref = msg_ref;
  op.payload_len = payload_len;
  op.retain_flag = retain_flag ? 1 : 0;
}

// non-structural calls replayed on their node (the footprint the
// authoritative store recorded; the shadow store has the same node ids);
// MQM_FAST_REPLAY=0: every call replayed through the path (A/B).  It was
// opt-in after the served-churn stall of r05ac; with the served path's
// counter restart and forced relaunch since (capi.cpp Server) the runs with
// it on are clean (r05ae churnfast, r05af)
static bool fast_replay() {
  static const bool v = !getenv("MQM_FAST_REPLAY") || atoi(getenv("MQM_FAST_REPLAY")) != 0;
  return v;
}

void DeltaLog::replay(Store &st, size_t limit) const {
  const char *base = bytes_.data();
  const bool fast = fast_replay();
  for (const Op &op : ops_) {
    if (limit-- == 0) return;
    const std::string_view a(base + op.a_off, op.a_len), b(base + op.a_off + op.a_len, op.b_len);
    switch (op.kind) {
      case kSub:
        if (fast && !op.fp.structural)
          st.subscribe_at(op.fp, op.qos, op.no_local, op.rap, op.rh, op.ident);
        else
          st.subscribe(a, b, op.qos, op.no_local, op.rap, op.rh, op.ident);
        break;
      case kUnsub:
        if (fast && !op.fp.structural)
          st.unsubscribe_at(op.fp);
        else
          st.unsubscribe(a, b);
        break;
      default:
        st.retain_message(a, op.msg_ref, op.payload_len, op.retain_flag != 0);
        break;
    }
  }
}

void DeltaLog::append(DeltaLog &&o) {
  if (ops_.empty()) {
    ops_.swap(o.ops_);
    bytes_.swap(o.bytes_);
    fast_ = o.fast_;
    o.clear();
    return;
  }
  const uint64_t shift = bytes_.size();
  bytes_.insert(bytes_.end(), o.bytes_.begin(), o.bytes_.end());
  // (no exact reserve: logs coalesce 20 times a second while a build runs,
  // and an exact reserve copied the whole queue each time — up to 44 ms under
  // the index lock at 100k mutations/s, r05k)
  for (Op op : o.ops_) {
    op.a_off += shift;
    ops_.push_back(op);
  }
  fast_ += o.fast_;
  o.clear();
}

Builder::Builder(int device) : device_(device) { th_ = std::thread([this] { run(); }); }

Builder::~Builder() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  th_.join();
  if (stream_) (void)hipStreamDestroy(stream_);
}

void Builder::submit(DeltaLog &&log, uint64_t version) {
  {
    std::lock_guard<std::mutex> g(mu_);
    queued_.append(std::move(log));  // logs submitted while a build runs are coalesced
    queued_version_ = version;
    has_queued_ = true;
  }
  cv_.notify_all();
}

void Builder::submit_full(const Store &st, uint64_t version) {
  auto copy = std::make_unique<Store>(st);  // outside mu_: the worker may be mid-build
  {
    std::lock_guard<std::mutex> g(mu_);
    full_ = std::move(copy);
    queued_.clear();
    queued_version_ = version;
    has_queued_ = true;
  }
  cv_.notify_all();
}

void Builder::inject_fault(int stage, int count) {
  std::lock_guard<std::mutex> g(mu_);
  fault_stage_ = stage;
  fault_count_ = count;
}

bool Builder::dirty() {
  std::lock_guard<std::mutex> g(mu_);
  return dirty_;
}

bool Builder::shadow_bad() {
  std::lock_guard<std::mutex> g(mu_);
  return shadow_bad_;
}

bool Builder::take(BuiltSnapshot *out) {
  std::lock_guard<std::mutex> g(mu_);
  if (!has_ready_) return false;
  *out = std::move(ready_);
  ready_ = BuiltSnapshot();
  has_ready_ = false;
  ready_flag_.store(false, std::memory_order_release);
  return true;
}

int Builder::wait_idle() {
  std::unique_lock<std::mutex> g(mu_);
  cv_.wait(g, [this] { return !has_queued_ && !working_; });
  const int e = err_;
  err_ = 0;
  return e;
}

bool Builder::busy() {
  std::lock_guard<std::mutex> g(mu_);
  return has_queued_ || working_;
}

void Builder::run() {
  // a background rebuild yields the CPU to the callers it publishes for (its
  // flatten threads inherit the nice value)
  (void)setpriority(PRIO_PROCESS, (id_t)syscall(SYS_gettid), 5);
  if (device_ >= 0) {
    if (hipSetDevice(device_) != hipSuccess ||
        hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking) != hipSuccess) {
      std::lock_guard<std::mutex> g(mu_);
      err_ = MQM_EHIP;
    }
  }
  for (;;) {
    DeltaLog log;
    uint64_t version;
    std::unique_ptr<Store> full;
    bool stale;
    int fault;
    {
      std::unique_lock<std::mutex> g(mu_);
      cv_.wait(g, [this] { return has_queued_ || stop_; });
      if (!has_queued_) return;  // stop_ with nothing left to build
      full = std::move(full_);
      log.append(std::move(queued_));
      version = queued_version_;
      has_queued_ = false;
      working_ = true;
      stale = shadow_bad_ && !full;
      fault = fault_count_ > 0 ? fault_stage_ : 0;
      if (fault) fault_count_--;
    }
    const auto t0 = std::chrono::steady_clock::now();
    int rc = MQM_OK;
    bool replayed = false;
    BuiltSnapshot b;
    if (stale) {
      rc = MQM_EINVAL;  // a log on top of a half-replayed shadow would build a wrong trie
    } else {
      try {
        if (full) {
          shadow_ = std::move(*full);
          shape_.valid = false;  // (another store instance)
        }
        if (fault == 1) {  // stop half-way, as a bad_alloc while interning would
          log.replay(shadow_, log.size() / 2);
          throw std::bad_alloc();
        }
        using ms = std::chrono::duration<double, std::milli>;
        log.replay(shadow_);
        replayed = true;
        const auto t1 = std::chrono::steady_clock::now();
        auto hs = std::make_shared<HostSnapshot>();
        const uint64_t reuses = shape_.reuses;
        rc = fault == 2 ? MQM_ENOMEM : flatten(shadow_, hs.get(), device_ < 0 || host_edges_forced(), &shape_);
        b.kept_shape = shape_.reuses != reuses;
        if (rc == MQM_OK && client_index_.load(std::memory_order_relaxed)) build_client_index(*hs);
        hs->version = version;  // (after flatten, which starts from an empty snapshot)
        const auto t2 = std::chrono::steady_clock::now();
        if (rc == MQM_OK && device_ >= 0 && !stream_) rc = MQM_EHIP;
        if (rc == MQM_OK) rc = fault == 3 ? MQM_ENOMEM : upload(std::move(hs), device_, stream_, &b.snap);
        b.phase_ms[0] = ms(t1 - t0).count();
        b.phase_ms[1] = ms(t2 - t1).count();
        b.phase_ms[2] = ms(std::chrono::steady_clock::now() - t2).count();
      } catch (const std::bad_alloc &) {
        rc = MQM_ENOMEM;
      } catch (...) {
        rc = MQM_EINVAL;
      }
    }
    b.version = version;
    b.n_ops = log.size();
    b.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    {
      std::lock_guard<std::mutex> g(mu_);
      working_ = false;
      if (rc == MQM_OK) {
        ready_ = std::move(b);  // replaces an unpublished older build
        has_ready_ = true;
        ready_flag_.store(true, std::memory_order_release);
        dirty_ = false;
        shadow_bad_ = false;
      } else {
        if (!err_) err_ = rc;
        dirty_ = true;
        shape_.valid = false;
        if (!stale && !replayed) shadow_bad_ = true;  // the replay stopped part-way
      }
    }
    cv_.notify_all();
  }
}

namespace {
// 64-bit multiply-xorshift over 8-byte words (tail zero-padded)
struct Digest {
  uint64_t h = 0x6D716D2D64696730ull;
  void add(const void *p, size_t n) {
    const auto *b = static_cast<const uint8_t *>(p);
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
      uint64_t w;
      std::memcpy(&w, b + i, 8);
      mix(w);
    }
    uint64_t w = 0;
    std::memcpy(&w, b + i, n - i);
    mix(w ^ ((uint64_t)n << 56));
  }
  void mix(uint64_t w) {
    h ^= w + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    h *= 0xFF51AFD7ED558CCDull;
    h ^= h >> 33;
  }
  template <class V>
  void vec(const V &v) {
    add(v.data(), v.size() * sizeof(v[0]));
  }
};
}  // namespace

uint64_t edges_digest_sum(const EdgeEntry *edges, uint64_t n) {
  constexpr uint64_t kChunks = 64;
  std::vector<uint64_t> part(kChunks, 0);
  std::vector<std::thread> th;
  const uint32_t nt = build_threads();
  for (uint32_t w = 0; w < nt; w++)
    th.emplace_back([&, w] {
      for (uint64_t c = w; c < kChunks; c += nt) {
        const uint64_t lo = n * c / kChunks, hi = n * (c + 1) / kChunks;
        uint64_t sum = 0;
        for (uint64_t s = lo; s < hi; s++) sum += edge_slot_mix(s, edges[s]);
        part[c] = sum;
      }
    });
  for (auto &x : th) x.join();
  uint64_t sum = 0;
  for (uint64_t v : part) sum += v;
  return sum;
}

uint64_t edges_digest_final(uint64_t sum, uint64_t n) {
  Digest d;
  d.mix(sum);
  d.mix(n);
  return d.h;
}

uint64_t edges_digest_of(const HostSnapshot &hs) {
  return edges_digest_final(edges_digest_sum(hs.edges.data(), hs.edges.size()), hs.edges.size());
}

uint64_t snapshot_digest(const HostSnapshot &hs) {
  Digest d;
  d.vec(hs.nodes);
  d.mix(hs.edges.empty() ? hs.edges_digest : edges_digest_of(hs));
  d.vec(hs.subs);
  d.vec(hs.sub_info);
  d.vec(hs.shared_info);
  d.vec(hs.tok_pool);
  d.vec(hs.bloom);
  d.vec(hs.pinfo);
  d.vec(hs.partners);
  d.vec(hs.subtree);
  d.vec(hs.child_off);
  d.vec(hs.child_ids);
  d.vec(hs.cum);
  d.vec(hs.rch_off);
  d.vec(hs.refs);
  d.vec(hs.rch_refs);
  d.vec(hs.rinv);
  d.vec(hs.rgroups);
  d.mix(hs.n_buckets);
  d.mix(hs.height);
  d.mix(hs.sys_child);
  d.mix(hs.has_empty);
  return d.h;
}

}  // namespace mqm
