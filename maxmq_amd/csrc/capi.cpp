// maxmq_amd/csrc/capi.cpp — the C ABI (include/mqmatch.h) over the host
// store, the snapshot builder and the HIP match pipeline.
//
// Threading (the reference runs Subscribers() concurrently from
// one goroutine per connection, listeners/tcp.go:83, clients.go:331-356):
//   * h->mu guards the store, the delta log, the builder and the front-buffer
//     pointer.  Mutations and commits hold it; a match holds it only to
//     publish / read the front buffer (RCU style: it takes a shared_ptr).
//   * Host-path matches (mqm_match_batch, mqm_subscribers, mqm_messages_*)
//     borrow a MatchCtx (workspace + HIP stream) from a per-index pool, so
//     any number of threads match concurrently against one snapshot, each on
//     its own stream; results land in pinned host blocks from a shared pool.
//   * The device-result API (mqm_match_device and its follow-ups, whose
//     results live in library memory "until the next call") uses one default
//     MatchCtx under its own mutex.
//   * A snapshot is freed when its last holder drops it: the front-buffer
//     pointer, a running call, or the default context (which keeps the
//     snapshot its device results refer to until its next call).
#include <hip/hip_runtime.h>

#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <shared_mutex>
#include <new>
#include <string_view>
#include <thread>
#include <vector>

#include "../../include/mqmatch.h"
#include "builder.h"
#include "bulkload.h"
#include "flatten.h"
#include "fresh.h"
#include "match.h"
#include "retained.h"
#include "serve_slots.h"
#include "shard.h"
#include "store.h"

using namespace mqm;

namespace {

// Pinned host blocks for results: D2H into pinned memory runs at the link
// rate; pageable memory costs an extra staging copy.  Blocks are recycled
// (best fit), so steady-state batches allocate nothing.
class PinnedPool {
 public:
  ~PinnedPool() {
    for (auto &kv : free_) (void)hipHostFree(kv.second);
  }
  void *get(size_t need, size_t *cap) {
    need = std::max<size_t>(need, 4096);
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = free_.lower_bound(need);
      // slack proportional to the request (a small single-topic result never
      // holds on to a large batch block)
      if (it != free_.end() && it->first <= 2 * need + std::min<size_t>(need, 64u << 20)) {
        *cap = it->first;
        void *p = it->second;
        cached_ -= it->first;
        free_.erase(it);
        return p;
      }
    }
    const size_t n = need + need / 8;
    void *p = nullptr;
    if (hipHostMalloc(&p, n, hipHostMallocDefault) != hipSuccess) return nullptr;
    *cap = n;
    return p;
  }
  void put(void *p, size_t cap) {
    if (!p) return;
    std::lock_guard<std::mutex> g(mu_);
    free_.emplace(cap, p);
    cached_ += cap;
    while (cached_ > kMaxCached && !free_.empty()) {  // drop the largest
      auto it = std::prev(free_.end());
      cached_ -= it->first;
      (void)hipHostFree(it->second);
      free_.erase(it);
    }
  }

 private:
  static constexpr size_t kMaxCached = size_t(16) << 30;
  std::mutex mu_;
  std::multimap<size_t, void *> free_;
  size_t cached_ = 0;
};

// one caller's pipeline state
struct MatchCtx {
  Workspace ws;
  hipStream_t stream = nullptr;         // own stream (host-path calls)
  std::shared_ptr<GpuSnapshot> snap;    // what the device results below were computed on
  bool has_mo = false;
  MatchOutput last_mo;
  void *staging = nullptr;              // pinned input staging (topic offsets)
  size_t staging_cap = 0;
  ~MatchCtx() {
    snap.reset();
    if (staging) (void)hipHostFree(staging);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

}  // namespace

namespace {
struct Collector;
struct Server;
}

struct mqm_index {
  mqm_config cfg{};
  std::mutex mu;  // store, journal, builder, front buffer
  Store store;
  std::shared_ptr<GpuSnapshot> snap;     // front buffer: what matches read
  uint64_t snap_version = ~0ull;         // store version the front buffer reflects
  std::shared_mutex snap_rw;             // snap / snap_version: written under mu + this, read under either
  // MQM_CFG_ASYNC_COMMIT: mutations since the last submit, and the builder
  // that turns them into the back buffer (builder.h)
  DeltaLog journal;
  std::unique_ptr<Builder> builder;
  std::atomic<bool> ident_early{false};         // mqm_identifiers_early: device matches compute Identifiers beside
  std::atomic<Builder *> builder_pub{nullptr};  // builder.get(), readable without mu (front_fast)
  std::atomic<int64_t> submit_due_ns{0};        // policy_ms: when the logged mutations are due (0: none)
  uint64_t policy_ops = 0;               // auto-submit after this many logged mutations (0 = off)
  uint32_t policy_ms = 0;                // ... or when the oldest one is this old (0 = off)
  std::chrono::steady_clock::time_point journal_t0;  // when the oldest unsubmitted mutation was logged
  bool journal_dated = false;                          // (journal_t0 is set for the current journal)
  uint64_t builds = 0, last_build_ops = 0;
  double last_build_ms = 0, last_build_phase_ms[3] = {0, 0, 0};
  bool last_build_kept_shape = false;
  bool fast_path = true;  // MQM_NO_FAST=1: small batches also take the batch pipeline (A/B, tests)
  // MQM_CFG_FRESH: the touched clients' current subscriptions (fresh.h), written
  // under mu with every mutation and publish, read by mqm_subscribers
  std::unique_ptr<FreshOverlay> fresh;
  std::atomic<bool> fresh_reads{true};  // mqm_fresh_policy: calls corrected (the overlay is kept either way)
  bool async() const { return (cfg.flags & MQM_CFG_ASYNC_COMMIT) != 0; }
  // the device-result API's context (mqm_match_device & follow-ups)
  std::mutex dev_mu;
  MatchCtx dev;
  // host-path contexts, one per concurrent caller
  std::mutex pool_mu;
  std::vector<std::unique_ptr<MatchCtx>> pool;
  std::shared_ptr<PinnedPool> pinned = std::make_shared<PinnedPool>();
  // MQM_CFG_BATCHING: declared last, so it stops (joins its thread) before
  // anything it uses is destroyed.  `collector` is what callers read (no
  // lock: an acquire load), published once with a release store under mu;
  // collector_owner keeps it alive until the index is destroyed
  std::unique_ptr<Collector> collector_owner;
  // MQM_CFG_SERVE: the persistent per-publish server (published like the collector)
  std::atomic<Server *> server{nullptr};
  std::unique_ptr<Server> server_owner;
  void stop_server();
  std::atomic<Collector *> collector{nullptr};
  std::atomic<uint32_t> live_ctxs{0};  // mqm_match_ctx objects of this index (mqm_destroy refuses while any live)
  // single-topic calls on the direct small-batch path (mqm_direct_host_us):
  // per phase (front buffer, context, launch + wait, result), summed and max ns
  std::atomic<uint64_t> direct_ns[4] = {}, direct_max_ns[4] = {}, direct_calls{0};
  // batch-pipeline host-path calls (mqm_batch_host_us): per phase ns, summed
  // — front buffer + context, topics H2D, match (walk .. merges, collected),
  // runs / identifiers / densify, result D2H + synchronisation
  std::atomic<uint64_t> batch_ns[5] = {}, batch_calls{0};
  void stop_collector();
  ~mqm_index();
};

struct mqm_messages {
  uint32_t n = 0;
  std::vector<uint64_t> offsets, refs;
};

struct mqm_result {
  uint32_t n = 0;
  // one pinned block: offsets | shared_offsets | ident_offsets | deliveries | shared | idents
  std::shared_ptr<PinnedPool> pool;
  void *blk = nullptr;
  size_t blk_cap = 0;
  const uint64_t *offsets = nullptr, *shared_offsets = nullptr, *ident_offsets = nullptr;
  const mqm_delivery *deliveries = nullptr;  // nullptr for a packed result
  const uint32_t *packed = nullptr;           // mqm_match_batch_packed: 4-B packed words
  const uint32_t *shared = nullptr, *idents = nullptr;
  bool has_idents = false;               // MQM_CFG_IDENTIFIERS
  // the runs form (mqm_match_batch_runs): offsets / packed are the merged
  // winners; topic t's solo deliveries are snap->words over its runs
  const uint64_t *run_offsets = nullptr;
  const mqm_run *runs = nullptr;
  uint64_t n_solo = 0;
  std::shared_ptr<const HostSnapshot> snap;
  // MQM_CFG_FRESH (freshen): subscriptions past the snapshot's sids (sid
  // snap->sub_info.size() + k is extra[k]; shared likewise), and the store
  // version the corrected result reflects (0: the snapshot's)
  std::vector<SubInfo> extra, extra_shared;
  uint64_t version = 0;
  bool heap = false;  // blk from malloc (results filled by host copies, no DMA into them)
  ~mqm_result() {
    if (heap)
      free(blk);
    else if (pool)
      pool->put(blk, blk_cap);
  }
  // the result's block: pinned (from the index's pool) when a DMA fills it,
  // plain host memory when host copies do
  bool alloc(const std::shared_ptr<PinnedPool> &p, size_t bytes, bool pinned) {
    if (pinned) {
      pool = p;
      blk = p->get(bytes, &blk_cap);
      if (!blk) pool.reset();
    } else {
      heap = true;
      blk = malloc(std::max<size_t>(bytes, 64));
      blk_cap = bytes;
    }
    return blk != nullptr;
  }
};

namespace {

template <class F>
int guarded(F &&f) {
  try {
    return f();
  } catch (const std::bad_alloc &) {
    return MQM_ENOMEM;
  } catch (...) {
    return MQM_EINVAL;
  }
}

std::string_view sv(const char *p, size_t n) { return std::string_view(p ? p : "", p ? n : 0); }

int hip_rc(int rc) { return rc == -2 ? MQM_ENOMEM : rc == -1 ? MQM_EINVAL : rc < 0 ? MQM_EHIP : rc; }

// make g the front buffer; readers that hold the old one keep it alive
// Snapshot references dropped on a latency path (a publish, a server
// relaunch, a served result freed) are handed to this thread, so the last one
// — which frees gigabytes of host arrays (HostSnapshot) and retires the device
// buffers — is never dropped by a caller, let alone under the index's or the
// server's lock (r05: served calls paused ~0.2 s around each publish).
struct Releaser {
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::shared_ptr<const void>> q;
  Releaser() {
    std::thread([this] {
      for (;;) {
        std::vector<std::shared_ptr<const void>> batch;
        {
          std::unique_lock<std::mutex> g(mu);
          cv.wait(g, [this] { return !q.empty(); });
          batch.swap(q);
        }
        batch.clear();  // (the last references: the destructors run here)
      }
    }).detach();
  }
};
void defer_release(std::shared_ptr<const void> p) {
  // (only a reference that looks like the last one goes to the thread: a
  // served call's own reference to a live snapshot is dropped here, no lock)
  if (!p || p.use_count() > 1) return;
  static auto *r = new Releaser;  // (never destroyed, like its thread)
  {
    std::lock_guard<std::mutex> g(r->mu);
    r->q.push_back(std::move(p));
  }
  r->cv.notify_one();
}

int install(mqm_index *h, std::shared_ptr<GpuSnapshot> g, uint64_t version) {
  std::shared_ptr<GpuSnapshot> old;
  std::shared_ptr<const HostSnapshot> host = g ? g->host : nullptr;
  {
    std::unique_lock<std::shared_mutex> w(h->snap_rw);
    old = std::move(h->snap);
    h->snap = std::move(g);
    h->snap_version = version;
  }
  if (h->fresh) h->fresh->on_install(std::move(host), h->store);
  defer_release(std::move(old));
  return MQM_OK;
}

// after a Store::subscribe (mu held): the overlay takes the record
void fresh_subscribe(mqm_index *h, std::string_view filter, uint8_t qos, uint8_t no_local, uint8_t rap, uint8_t rh,
                     int32_t ident) {
  if (!h->fresh) return;
  const Store::Footprint &fp = h->store.last_footprint();
  h->fresh->on_subscribe(h->store, filter, SubRec{fp.client, fp.filter, ident, qos, no_local, rap, rh});
}

int64_t steady_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// MQM_SERVE_TRACE=1: the served path's slow steps (publish, server relaunch)
// to stderr with their durations
bool serve_trace() {
  static const bool v = getenv("MQM_SERVE_TRACE") && atoi(getenv("MQM_SERVE_TRACE")) != 0;
  return v;
}
struct TraceSpan {
  const char *what;
  int64_t t0 = serve_trace() ? steady_ns() : 0;
  explicit TraceSpan(const char *w) : what(w) {}
  void mark(const char *step) {
    if (!t0) return;
    const int64_t t = steady_ns();
    if (t - t0 > 5000000) fprintf(stderr, "[serve-trace] %.6f %s: %s after %.1f ms\n", t * 1e-9, what, step, (t - t0) / 1e6);
    t0 = t;
  }
};

// the index's builder, created on first use (mu held)
Builder *builder_locked(mqm_index *h) {
  if (!h->builder) {
    h->builder = std::make_unique<Builder>(h->cfg.device);
    if (h->fresh) h->builder->set_client_index(true);
    h->builder_pub.store(h->builder.get(), std::memory_order_release);
  }
  return h->builder.get();
}

// hand the journal to the builder (MQM_CFG_ASYNC_COMMIT); after a replay that
// failed part-way the builder gets a full copy of the store instead
void submit_locked(mqm_index *h) {
  // the builder starts empty: the journal of an async index holds every
  // mutation since mqm_create
  builder_locked(h);
  if (h->builder->shadow_bad())
    h->builder->submit_full(h->store, h->store.version());
  else
    h->builder->submit(std::move(h->journal), h->store.version());
  h->journal.clear();
  h->journal_dated = false;
  h->submit_due_ns.store(0, std::memory_order_relaxed);
}

// publish the builder's newest finished snapshot, if any
int publish_locked(mqm_index *h, int *published) {
  if (published) *published = 0;
  if (!h->builder) return MQM_OK;
  BuiltSnapshot b;
  if (!h->builder->take(&b)) return MQM_OK;
  h->builds++;
  h->last_build_ms = b.build_ms;
  h->last_build_ops = b.n_ops;
  for (int i = 0; i < 3; i++) h->last_build_phase_ms[i] = b.phase_ms[i];
  h->last_build_kept_shape = b.kept_shape;
  if (published) *published = 1;
  return install(h, std::shared_ptr<GpuSnapshot>(std::move(b.snap)), b.version);
}

// after a logged mutation: the periodic-rebuild policy (mqm_commit_policy)
void maybe_submit(mqm_index *h) {
  if (!h->async() || h->journal.empty()) return;
  if (h->policy_ops && h->journal.size() >= h->policy_ops) return submit_locked(h);
  if (!h->journal_dated) {  // the first mutation since the last submit
    h->journal_t0 = std::chrono::steady_clock::now();
    h->journal_dated = true;
  }
  if (h->policy_ms) {
    const auto due = h->journal_t0 + std::chrono::milliseconds(h->policy_ms);
    if (std::chrono::steady_clock::now() >= due) return submit_locked(h);
    // (front_fast submits when this passes without another mutation)
    h->submit_due_ns.store(std::chrono::duration_cast<std::chrono::nanoseconds>(due.time_since_epoch()).count(),
                           std::memory_order_relaxed);
  }
}

int commit_locked(mqm_index *h) {
  if (h->snap && h->snap_version == h->store.version()) return MQM_OK;
  if (h->async()) {  // through the builder, so its shadow store stays in step
    if (!h->journal.empty() || !h->builder || h->builder->dirty() || h->builder->shadow_bad()) submit_locked(h);
    int rc = h->builder->wait_idle();
    if (rc != MQM_OK && h->builder->shadow_bad()) {  // a replay stopped part-way: rebuild from a copy once
      submit_locked(h);
      rc = h->builder->wait_idle();
    }
    if (rc != MQM_OK) return rc;
    rc = publish_locked(h, nullptr);
    if (rc != MQM_OK) return rc;
    // every submitted mutation is built and published, or this is an error
    return h->snap && h->snap_version == h->store.version() ? MQM_OK : MQM_EINVAL;
  }
  auto hs = std::make_shared<HostSnapshot>();
  int rc = flatten(h->store, hs.get(), h->cfg.device < 0 || host_edges_forced());  // (a device builds the edge table itself)
  if (rc != MQM_OK) return rc;
  if (h->fresh) build_client_index(*hs);
  hs->version = h->store.version();  // (after flatten, which starts from an empty snapshot; mu held)
  std::unique_ptr<GpuSnapshot> g;
  rc = upload(std::move(hs), h->cfg.device, h->dev.stream, &g);
  if (rc != MQM_OK) return rc;
  return install(h, std::shared_ptr<GpuSnapshot>(std::move(g)), h->store.version());
}

int ensure_snapshot_locked(mqm_index *h) {
  if (!h->snap || (h->cfg.flags & MQM_CFG_AUTOCOMMIT)) return commit_locked(h);
  if (h->async()) {
    maybe_submit(h);
    return publish_locked(h, nullptr);
  }
  return MQM_OK;
}

// the front buffer for a match (committing first per the index's flags)
int front(mqm_index *h, std::shared_ptr<GpuSnapshot> *out) {
  std::lock_guard<std::mutex> g(h->mu);
  const int rc = ensure_snapshot_locked(h);
  if (rc != MQM_OK) return rc;
  if (!h->snap) return MQM_EINVAL;
  *out = h->snap;
  return MQM_OK;
}

// front() without waiting for the index lock (the per-publish server's
// callers: 64 of them on mu queue up behind every mutation).  The front buffer
// is returned when it exists and, with MQM_CFG_AUTOCOMMIT, reflects the
// store's current version; false: take front() (it commits first).  With
// MQM_CFG_ASYNC_COMMIT and no autocommit a finished build is published (or a
// due policy submit made) by whichever caller gets the lock without waiting;
// the others match the current front buffer meanwhile.
bool front_fast(mqm_index *h, std::shared_ptr<GpuSnapshot> *out) {
  const bool autoc = (h->cfg.flags & MQM_CFG_AUTOCOMMIT) != 0;
  if (h->async() && !autoc) {
    const Builder *b = h->builder_pub.load(std::memory_order_acquire);
    const int64_t due = h->submit_due_ns.load(std::memory_order_relaxed);
    if ((b && b->has_ready()) || (due && steady_ns() >= due)) {
      std::unique_lock<std::mutex> g(h->mu, std::try_to_lock);
      if (g.owns_lock()) {
        TraceSpan ts("front_fast");
        maybe_submit(h);
        ts.mark("submit");
        (void)publish_locked(h, nullptr);
        ts.mark("publish");
      }
    }
  }
  std::shared_lock<std::shared_mutex> r(h->snap_rw);
  if (!h->snap) return false;
  if (autoc && h->snap_version != h->store.version()) return false;
  *out = h->snap;
  return true;
}

int ctx_init(mqm_index *, MatchCtx *c) {
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    c->stream = nullptr;
    return MQM_EHIP;
  }
  return MQM_OK;
}

// a host-path context from the pool (a new one when all are busy)
std::unique_ptr<MatchCtx> ctx_acquire(mqm_index *h, int *rc) {
  {
    std::lock_guard<std::mutex> g(h->pool_mu);
    if (!h->pool.empty()) {
      auto c = std::move(h->pool.back());
      h->pool.pop_back();
      *rc = MQM_OK;
      return c;
    }
  }
  auto c = std::make_unique<MatchCtx>();
  *rc = ctx_init(h, c.get());
  return c;
}

void ctx_release(mqm_index *h, std::unique_ptr<MatchCtx> c) {
  c->snap.reset();  // the call synchronised its stream: nothing reads the snapshot any more
  c->has_mo = false;
  std::lock_guard<std::mutex> g(h->pool_mu);
  h->pool.push_back(std::move(c));
}

// MQM_D2H_KERNEL=1: a host-path call's result parts go to its pinned block by
// one copy kernel (match.hip k_copy_out) instead of a DMA copy each (read per
// call: tests switch it)
bool d2h_kernel() {
  const char *e = getenv("MQM_D2H_KERNEL");
  return e && atoi(e) != 0;
}

// pinned staging for n + 1 rebased offsets
uint64_t *ctx_staging(MatchCtx *c, size_t bytes) {
  if (c->staging_cap < bytes) {
    if (c->staging) (void)hipHostFree(c->staging);
    c->staging = nullptr;
    c->staging_cap = 0;
    if (hipHostMalloc(&c->staging, bytes + bytes / 4, hipHostMallocDefault) != hipSuccess) return nullptr;
    c->staging_cap = bytes + bytes / 4;
  }
  return static_cast<uint64_t *>(c->staging);
}

// topic / filter batch from host memory into the context's input buffers
int upload_batch(MatchCtx *c, Workspace::Slot sb, Workspace::Slot so, const char *bytes, const uint64_t *offs,
                 uint32_t n, const uint8_t **d_bytes, const uint64_t **d_offs) {
  Workspace &ws = c->ws;
  const uint64_t base = offs[0], nbytes = offs[n] - base;
  if (ws.get(sb, nbytes + 16) || ws.get(so, sizeof(uint64_t) * (n + 1))) return MQM_ENOMEM;
  uint64_t *st = ctx_staging(c, sizeof(uint64_t) * (n + 1));
  if (!st) return MQM_ENOMEM;
  if (hipStreamSynchronize(c->stream) != hipSuccess) return MQM_EHIP;  // the staging block is reused
  for (uint32_t i = 0; i <= n; i++) st[i] = offs[i] - base;
  if (nbytes && hipMemcpyAsync(ws.ptr(sb), bytes + base, nbytes, hipMemcpyHostToDevice, c->stream) != hipSuccess)
    return MQM_EHIP;
  if (hipMemcpyAsync(ws.ptr(so), st, sizeof(uint64_t) * (n + 1), hipMemcpyHostToDevice, c->stream) != hipSuccess)
    return MQM_EHIP;
  *d_bytes = (const uint8_t *)ws.ptr(sb);
  *d_offs = (const uint64_t *)ws.ptr(so);
  return MQM_OK;
}

int fill_info(const SubInfo &s, mqm_sub_info *out) {
  out->filter = s.filter;
  out->client = s.client;
  out->identifier = s.ident;
  out->qos = s.qos;
  out->no_local = s.no_local;
  out->retain_as_published = s.rap;
  out->retain_handling = s.rh;
  return MQM_OK;
}

bool bad_sub(const mqm_subscription &s) { return s.qos > 2 || s.retain_handling > 3; }

void fill_device_result(const MatchOutput &mo, const Workspace &ws, mqm_device_result *out) {
  out->n_topics = mo.n_topics;
  out->n_deliveries = mo.n_deliveries;
  out->n_shared = mo.n_shared;
  out->starts = mo.starts;
  out->counts = mo.counts;
  out->deliveries = mo.deliveries;
  out->shared_starts = mo.shared_starts;
  out->shared_counts = mo.shared_counts;
  out->shared = mo.shared;
  out->n_fallback = mo.n_fallback;
  out->n_big = mo.n_big;
  for (int i = 0; i < 5; i++) out->fallback_why[i] = ws.why[i];
  out->n_merge_small = mo.n_merge_small;
  out->n_merge_wave = mo.n_merge_wave;
  out->n_solo_ranges = mo.n_solo_ranges;
  out->n_tier2 = mo.n_tier2;
  out->n_tier3 = mo.n_tier3;
  for (int i = 0; i < 3; i++) out->multi_entries[i] = mo.multi_entries[i];
  out->n_part = mo.n_part;
  out->n_resolve = mo.n_resolve;
  out->n_solo = mo.n_solo;
}

// a result block laid out like mqm_match_batch's: offsets | shared_offsets |
// deliveries | shared (16-B aligned parts), from per-topic counts
struct ResultLayout {
  uint64_t o_sh = 0, o_io = 0, o_d = 0, o_s = 0, o_i = 0, total = 0;
  ResultLayout(uint64_t n1, uint64_t nd, uint64_t ns, uint64_t dsize, uint64_t ni = 0, bool ids = false) {
    auto up = [](uint64_t b) { return (b + 15) & ~15ull; };
    o_sh = up(8 * n1);
    o_io = o_sh + up(8 * n1);
    o_d = o_io + (ids ? up(8 * n1) : 0);
    o_s = o_d + up(dsize * nd);
    o_i = o_s + up(4 * ns);
    total = o_i + up(4 * ni);
  }
};

// the small-batch path's per-topic segments (FastRec: anywhere in the pinned
// output blocks, in completion order) -> one result block in topic order
int fast_result(mqm_index *h, const std::shared_ptr<GpuSnapshot> &snap, const FastOutput &fo, bool packed,
                mqm_result *r) {
  const uint32_t n = fo.n_topics;
  const bool ids = fo.iout != nullptr;
  uint64_t nd = 0, ns = 0, ni = 0;
  for (uint32_t i = 0; i < n; i++) {
    nd += fo.recs[i].dcount;
    ns += fo.recs[i].hcount;
    ni += ids ? fo.recs[i].icount : 0;
  }
  const ResultLayout lay(n + 1ull, nd, ns, packed ? 4 : 8, ni, ids);
  if (!r->alloc(h->pinned, lay.total, false)) return MQM_ENOMEM;
  char *B = static_cast<char *>(r->blk);
  auto *off = reinterpret_cast<uint64_t *>(B), *soff = reinterpret_cast<uint64_t *>(B + lay.o_sh);
  auto *ioff = reinterpret_cast<uint64_t *>(B + lay.o_io);
  auto *dl = reinterpret_cast<uint64_t *>(B + lay.o_d);
  auto *sh = reinterpret_cast<uint32_t *>(B + lay.o_s);
  auto *idv = reinterpret_cast<uint32_t *>(B + lay.o_i);
  uint64_t d = 0, q = 0, k = 0;
  for (uint32_t i = 0; i < n; i++) {
    const FastRec &x = fo.recs[i];
    off[i] = d;
    soff[i] = q;
    if (ids) {
      ioff[i] = k;
      if (x.icount) memcpy(idv + k, fo.iout + x.ibase, 4ull * x.icount);
      k += x.icount;
    }
    if (packed) {
      uint32_t *p4 = reinterpret_cast<uint32_t *>(dl) + d;
      for (uint32_t j = 0; j < x.dcount; j++) p4[j] = (uint32_t)(fo.dout[x.dbase + j] >> 32);
    } else if (x.dcount) {
      memcpy(dl + d, fo.dout + x.dbase, 8ull * x.dcount);
    }
    if (x.hcount) memcpy(sh + q, fo.hout + x.hbase, 4ull * x.hcount);
    d += x.dcount;
    q += x.hcount;
  }
  off[n] = d;
  soff[n] = q;
  if (ids) {
    ioff[n] = k;
    r->has_idents = true;
    r->ident_offsets = ioff;
    r->idents = idv;
  }
  r->n = n;
  r->offsets = off;
  r->shared_offsets = soff;
  if (packed)
    r->packed = reinterpret_cast<const uint32_t *>(dl);
  else
    r->deliveries = reinterpret_cast<const mqm_delivery *>(dl);
  r->shared = sh;
  r->snap = snap->host;
  return MQM_OK;
}

}  // namespace

extern "C" {

const char *mqm_version(void) { return "mqmatch 0.1 (gfx950)"; }

int mqm_profile_enable(mqm_index *h, int on) {
  if (!h) return MQM_EINVAL;
  std::lock_guard<std::mutex> g(h->dev_mu);
  h->dev.ws.profile = on != 0;
  h->dev.ws.reset_profile();
  return MQM_OK;
}

int mqm_profile_read(mqm_index *h, mqm_profile *out) {
  if (!h || !out) return MQM_EINVAL;
  std::lock_guard<std::mutex> g(h->dev_mu);
  out->calls = h->dev.ws.prof_calls;
  out->fallback_topics = h->dev.ws.prof_fallback_topics;
  out->walk_ms = h->dev.ws.prof_walk_ms;
  out->dedupe_ms = h->dev.ws.prof_dedupe_ms;
  out->total_ms = h->dev.ws.prof_total_ms;
  return MQM_OK;
}

int mqm_create(const mqm_config *cfg, mqm_index **out) {
  if (!out) return MQM_EINVAL;
  *out = nullptr;
  return guarded([&] {
    auto h = std::make_unique<mqm_index>();
    if (cfg) h->cfg = *cfg;
    if (h->cfg.device == MQM_DEVICE_NONE) {  // host-only store: mutations, no matching
      *out = h.release();
      return MQM_OK;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return MQM_ENODEV;
    if (h->cfg.device < 0 || h->cfg.device >= ndev) return MQM_EINVAL;
    if (hipSetDevice(h->cfg.device) != hipSuccess) return MQM_EHIP;
    if (const char *e = getenv("MQM_NO_FAST")) h->fast_path = atoi(e) == 0;
    if (h->cfg.flags & MQM_CFG_FRESH) h->fresh = std::make_unique<FreshOverlay>();
    if (ctx_init(h.get(), &h->dev) != MQM_OK) return MQM_EHIP;
    if ((h->cfg.flags & MQM_CFG_SERVE) && mqm_serve_policy(h.get(), 0, 0) != MQM_OK) return MQM_EHIP;
    if (h->cfg.flags & MQM_CFG_BATCHING) {
      h->collector_owner = std::make_unique<Collector>(h.get());
      h->collector.store(h->collector_owner.get(), std::memory_order_release);
    }
    *out = h.release();
    return MQM_OK;
  });
}

int mqm_destroy(mqm_index *h) {
  if (!h) return MQM_EINVAL;
  // a match context reads the index: it must be destroyed first
  if (h->live_ctxs.load(std::memory_order_acquire) != 0) return MQM_EINVAL;
  h->stop_server();     // first: its kernel reads the snapshot
  h->stop_collector();  // its thread matches (and may commit) through this index
  h->builder_pub.store(nullptr, std::memory_order_release);
  h->builder.reset();    // finishes a running build and joins the worker
  if (h->cfg.device != MQM_DEVICE_NONE) {
    (void)hipSetDevice(h->cfg.device);
    (void)hipDeviceSynchronize();
  }
  delete h;
  return MQM_OK;
}

int mqm_debug_fault(mqm_index *h, int stage, int count) {
  if (!h || stage < 1 || stage > 3 || count < 0) return MQM_EINVAL;
  std::lock_guard<std::mutex> g(h->mu);
  if (!h->async()) return MQM_EINVAL;
  builder_locked(h)->inject_fault(stage, count);
  return MQM_OK;
}

int mqm_subscribe(mqm_index *h, const char *client, size_t client_len, const char *filter, size_t filter_len,
                  const mqm_subscription *sub, int *is_new) {
  if (!h || !sub || bad_sub(*sub)) return MQM_EINVAL;
  return guarded([&] {
    std::lock_guard<std::mutex> g(h->mu);
    bool n = h->store.subscribe(sv(client, client_len), sv(filter, filter_len), sub->qos, sub->no_local,
                                sub->retain_as_published, sub->retain_handling, sub->identifier);
    fresh_subscribe(h, sv(filter, filter_len), sub->qos, sub->no_local, sub->retain_as_published,
                    sub->retain_handling, sub->identifier);
    if (h->async()) {
      h->journal.subscribe(sv(client, client_len), sv(filter, filter_len), sub->qos, sub->no_local,
                           sub->retain_as_published, sub->retain_handling, sub->identifier,
                           &h->store.last_footprint());
      maybe_submit(h);
    }
    if (is_new) *is_new = n ? 1 : 0;
    return MQM_OK;
  });
}

int mqm_subscribe_many(mqm_index *h, size_t n, const char *client_bytes, const uint64_t *client_offs,
                       const char *filter_bytes, const uint64_t *filter_offs, const mqm_subscription *subs,
                       uint8_t *is_new) {
  if (!h || !client_offs || !filter_offs || !subs) return MQM_EINVAL;
  for (size_t i = 0; i < n; i++)  // nothing is applied when any record is out of range
    if (bad_sub(subs[i])) return MQM_EINVAL;
  return guarded([&] {
    std::lock_guard<std::mutex> g(h->mu);
    for (size_t i = 0; i < n; i++) {
      const mqm_subscription &s = subs[i];
      const auto c = sv(client_bytes + client_offs[i], client_offs[i + 1] - client_offs[i]);
      const auto f = sv(filter_bytes + filter_offs[i], filter_offs[i + 1] - filter_offs[i]);
      bool r = h->store.subscribe(c, f, s.qos, s.no_local, s.retain_as_published, s.retain_handling, s.identifier);
      fresh_subscribe(h, f, s.qos, s.no_local, s.retain_as_published, s.retain_handling, s.identifier);
      if (h->async())
        h->journal.subscribe(c, f, s.qos, s.no_local, s.retain_as_published, s.retain_handling, s.identifier,
                             &h->store.last_footprint());
      if (is_new) is_new[i] = r ? 1 : 0;
    }
    maybe_submit(h);
    return MQM_OK;
  });
}

int mqm_unsubscribe(mqm_index *h, const char *filter, size_t filter_len, const char *client, size_t client_len,
                    int *existed) {
  if (!h) return MQM_EINVAL;
  return guarded([&] {
    std::lock_guard<std::mutex> g(h->mu);
    bool r = h->store.unsubscribe(sv(filter, filter_len), sv(client, client_len));
    if (r && h->fresh) h->fresh->on_unsubscribe(h->store, sv(filter, filter_len));
    if (r && h->async()) {  // false: no node, nothing changed (topics.go:334-336)
      h->journal.unsubscribe(sv(filter, filter_len), sv(client, client_len), &h->store.last_footprint());
      maybe_submit(h);
    }
    if (existed) *existed = r ? 1 : 0;
    return MQM_OK;
  });
}

int mqm_load_subscriptions_json(mqm_index *h, const char *json, size_t len, uint64_t *n_loaded, uint64_t *n_new) {
  if (!h || (len && !json)) return MQM_EINVAL;
  if (n_loaded) *n_loaded = 0;
  if (n_new) *n_new = 0;
  return guarded([&] {
    std::lock_guard<std::mutex> g(h->mu);
    uint64_t fresh = 0;
    auto sink = [&](const std::string &client, const std::string &filter, const SubscriptionRecord &r) {
      // the snapshot packs QoS in 2 bits and RH in 2; the identifier is int32
      if (r.qos > 2 || r.retain_handling > 3 || r.identifier < INT32_MIN || r.identifier > INT32_MAX) return false;
      const uint8_t nl = r.no_local ? 1 : 0, rap = r.retain_as_published ? 1 : 0;
      if (h->store.subscribe(client, filter, r.qos, nl, rap, r.retain_handling, (int32_t)r.identifier)) fresh++;
      fresh_subscribe(h, filter, r.qos, nl, rap, r.retain_handling, (int32_t)r.identifier);
      if (h->async()) h->journal.subscribe(client, filter, r.qos, nl, rap, r.retain_handling, (int32_t)r.identifier);
      return true;
    };
    const int rc = parse_subscription_records(json, len, sink, n_loaded);
    if (n_new) *n_new = fresh;
    maybe_submit(h);
    return rc == 0 ? MQM_OK : rc == -2 ? MQM_ELIMIT : MQM_EINVAL;
  });
}

int mqm_unsubscribe_many(mqm_index *h, size_t n, const char *filter_bytes, const uint64_t *filter_offs,
                         const char *client_bytes, const uint64_t *client_offs, uint8_t *existed) {
  if (!h || !filter_offs || !client_offs) return MQM_EINVAL;
  return guarded([&] {
    std::lock_guard<std::mutex> g(h->mu);
    for (size_t i = 0; i < n; i++) {
      const auto f = sv(filter_bytes + filter_offs[i], filter_offs[i + 1] - filter_offs[i]);
      const auto c = sv(client_bytes + client_offs[i], client_offs[i + 1] - client_offs[i]);
      bool r = h->store.unsubscribe(f, c);
      if (r && h->fresh) h->fresh->on_unsubscribe(h->store, f);
      if (r && h->async()) h->journal.unsubscribe(f, c, &h->store.last_footprint());
      if (existed) existed[i] = r ? 1 : 0;
    }
    maybe_submit(h);
    return MQM_OK;
  });
}

int mqm_retain_message(mqm_index *h, const char *topic, size_t topic_len, uint64_t message_ref,
                       uint32_t payload_len, int retain_flag, int64_t *result) {
  if (!h) return MQM_EINVAL;
  return guarded([&] {
    std::lock_guard<std::mutex> g(h->mu);
    int64_t r = h->store.retain_message(sv(topic, topic_len), message_ref, payload_len, retain_flag != 0);
    if (h->fresh) h->fresh->on_version(h->store);
    if (h->async()) {
      h->journal.retain(sv(topic, topic_len), message_ref, payload_len, retain_flag != 0);
      maybe_submit(h);
    }
    if (result) *result = r;
    return MQM_OK;
  });
}

int mqm_retain_many(mqm_index *h, size_t n, const char *topic_bytes, const uint64_t *topic_offs,
                    const uint64_t *message_refs, const uint32_t *payload_lens, const uint8_t *retain_flags,
                    int64_t *results) {
  if (!h || !topic_offs || !message_refs || !payload_lens || (n && !topic_bytes)) return MQM_EINVAL;
  return guarded([&] {
    std::lock_guard<std::mutex> g(h->mu);
    for (size_t i = 0; i < n; i++) {
      const auto t = sv(topic_bytes + topic_offs[i], topic_offs[i + 1] - topic_offs[i]);
      const bool flag = retain_flags ? retain_flags[i] != 0 : true;
      int64_t r = h->store.retain_message(t, message_refs[i], payload_lens[i], flag);
      if (h->fresh) h->fresh->on_version(h->store);
      if (h->async()) h->journal.retain(t, message_refs[i], payload_lens[i], flag);
      if (results) results[i] = r;
    }
    maybe_submit(h);
    return MQM_OK;
  });
}

int mqm_retained_len(mqm_index *h, uint64_t *out) {
  if (!h || !out) return MQM_EINVAL;
  std::lock_guard<std::mutex> g(h->mu);
  *out = h->store.retained_len();
  return MQM_OK;
}

int mqm_commit(mqm_index *h) {
  if (!h) return MQM_EINVAL;
  return guarded([&] {
    std::lock_guard<std::mutex> g(h->mu);
    if (h->cfg.device != MQM_DEVICE_NONE && hipSetDevice(h->cfg.device) != hipSuccess) return MQM_EHIP;
    return commit_locked(h);
  });
}

int mqm_match_device(mqm_index *h, const uint8_t *d_topic_bytes, const uint64_t *d_topic_offsets, uint32_t n_topics,
                     void *hip_stream, mqm_device_result *out) {
  if (!h || !out || (n_topics && (!d_topic_bytes || !d_topic_offsets))) return MQM_EINVAL;
  return guarded([&] {
    if (h->cfg.device == MQM_DEVICE_NONE) return MQM_ENODEV;
    if (hipSetDevice(h->cfg.device) != hipSuccess) return MQM_EHIP;
    std::shared_ptr<GpuSnapshot> snap;
    int rc = front(h, &snap);
    if (rc != MQM_OK) return rc;
    std::lock_guard<std::mutex> g(h->dev_mu);
    MatchCtx &c = h->dev;
    const hipStream_t st = (hipStream_t)hip_stream;
    // earlier device results (and follow-ups queued on other streams) read the
    // workspace and their snapshot: wait for them before either is replaced
    if (c.ws.drain()) return MQM_EHIP;
    c.has_mo = false;
    c.snap = snap;
    c.ws.begin(st);
    c.ws.ident_early = h->ident_early.load(std::memory_order_relaxed);
    MatchOutput mo;
    rc = match_device(snap->dev, c.ws, d_topic_bytes, d_topic_offsets, n_topics, st, &mo);
    if (c.ws.end(st)) rc = rc ? rc : -3;
    if (rc != 0) return hip_rc(rc);
    c.last_mo = mo;
    c.has_mo = true;
    fill_device_result(mo, c.ws, out);
    return MQM_OK;
  });
}

}  // extern "C"

// skip_small: the caller already ran this batch on the small-batch path and
// it fell back (a topic past one of its capacities): go straight to the pipeline
// runs: the runs form (mqm_match_batch_runs): solo parts as runs of the
// snapshot's words, the merged winners packed (implies packed)
static int match_batch_impl(mqm_index *h, const char *topic_bytes, const uint64_t *topic_offsets, uint32_t n_topics,
                            bool packed, mqm_result **out, bool skip_small = false, bool runs = false) {
  packed = packed || runs;
  skip_small = skip_small || runs;  // (the small-batch path writes deliveries, not runs)
  if (!h || !out || !topic_offsets || (n_topics && !topic_bytes)) return MQM_EINVAL;
  *out = nullptr;
  return guarded([&] {
    if (h->cfg.device == MQM_DEVICE_NONE) return MQM_ENODEV;
    if (hipSetDevice(h->cfg.device) != hipSuccess) return MQM_EHIP;
    using clk = std::chrono::steady_clock;
    clk::time_point ts[5];
    ts[0] = clk::now();
    std::shared_ptr<GpuSnapshot> snap;
    int rc = front_fast(h, &snap) ? MQM_OK : front(h, &snap);  // (commits first with MQM_CFG_AUTOCOMMIT)
    if (rc != MQM_OK) return rc;
    ts[1] = clk::now();
    auto c = ctx_acquire(h, &rc);
    if (rc != MQM_OK) return rc;
    ts[2] = clk::now();
    auto r = std::make_unique<mqm_result>();
    const bool want_ids = (h->cfg.flags & MQM_CFG_IDENTIFIERS) != 0;
    // small batches (the per-publish call shape): the one-launch path, unless
    // a topic is past one of its capacities (then the pipeline below)
    if (n_topics <= kFastMaxTopics && h->fast_path && !skip_small) {
      c->ws.begin(c->stream);
      FastOutput fo;
      const int e = match_small(snap->dev, c->ws, topic_bytes, topic_offsets, n_topics, c->stream, &fo, want_ids);
      const int e2 = c->ws.end(c->stream);
      if (e < 0 || e2) {
        ctx_release(h, std::move(c));
        return e < 0 ? hip_rc(e) : MQM_EHIP;
      }
      if (e == 0) {
        ts[3] = clk::now();
        rc = fast_result(h, snap, fo, packed, r.get());
        ctx_release(h, std::move(c));
        if (rc != MQM_OK) return rc;
        *out = r.release();
        if (n_topics == 1) {  // the direct per-publish call: its phases (mqm_direct_host_us)
          ts[4] = clk::now();
          for (int i = 0; i < 4; i++) {
            const uint64_t d = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(ts[i + 1] - ts[i]).count();
            h->direct_ns[i].fetch_add(d, std::memory_order_relaxed);
            uint64_t m = h->direct_max_ns[i].load(std::memory_order_relaxed);
            while (d > m && !h->direct_max_ns[i].compare_exchange_weak(m, d, std::memory_order_relaxed)) {
            }
          }
          h->direct_calls.fetch_add(1, std::memory_order_relaxed);
        }
        return MQM_OK;
      }
    }
    clk::time_point tb[5];
    tb[0] = clk::now();
    rc = [&]() -> int {
      Workspace &ws = c->ws;
      const hipStream_t st = c->stream;
      ws.begin(st);
      const uint8_t *d_bytes = nullptr;
      const uint64_t *d_offs = nullptr;
      int e = upload_batch(c.get(), Workspace::kInBytes, Workspace::kInOffs, topic_bytes, topic_offsets, n_topics,
                           &d_bytes, &d_offs);
      if (e != MQM_OK) return e;
      tb[1] = clk::now();
      MatchOutput mo;
      ws.runs = runs;
      ws.ident_early = want_ids;  // (listed by the merges, or a pass beside them)
      e = match_device(snap->dev, ws, d_bytes, d_offs, n_topics, st, &mo);
      ws.runs = false;
      if (e != 0) return hip_rc(e);
      tb[2] = clk::now();
      RunsOutput ro;
      if (runs && (e = runs_device(ws, st, mo, &ro)) != 0) return hip_rc(e);
      IdentOutput io;
      if (want_ids && (e = identifiers_device(snap->dev, ws, st, &io)) != 0) return hip_rc(e);
      DenseOutput dn;
      if ((e = densify(snap->dev, ws, mo, st, &dn, packed)) != 0) return hip_rc(e);
      tb[3] = clk::now();
      // one pinned block: three offset arrays, then the entries (16-B aligned parts)
      const uint64_t n1 = (uint64_t)n_topics + 1, ni = want_ids ? io.n_idents : 0;
      auto up = [](uint64_t b) { return (b + 15) & ~15ull; };
      const uint64_t o_off = 0, o_sh = up(8 * n1), o_io = o_sh + up(8 * n1), o_d = o_io + (want_ids ? up(8 * n1) : 0);
      const uint64_t dsz = packed ? 4 : 8;
      const uint64_t o_s = o_d + up(dsz * mo.n_deliveries), o_i = o_s + up(4 * mo.n_shared), o_ro = o_i + up(4 * ni);
      const uint64_t o_r = o_ro + (runs ? up(8 * n1) : 0), total = o_r + (runs ? up(8 * ro.n_runs) : 0);
      r->pool = h->pinned;
      r->blk = h->pinned->get(total, &r->blk_cap);
      if (!r->blk) {
        r->pool.reset();
        return MQM_ENOMEM;
      }
      char *B = static_cast<char *>(r->blk);
      r->n = n_topics;
      r->offsets = reinterpret_cast<const uint64_t *>(B + o_off);
      r->shared_offsets = reinterpret_cast<const uint64_t *>(B + o_sh);
      if (packed)
        r->packed = reinterpret_cast<const uint32_t *>(B + o_d);
      else
        r->deliveries = reinterpret_cast<const mqm_delivery *>(B + o_d);
      r->shared = reinterpret_cast<const uint32_t *>(B + o_s);
      r->snap = snap->host;
      // the parts: DMA copies, or (MQM_D2H_KERNEL=1) one kernel storing into
      // the block's device view (tools/duplex_probe)
      CopyOut co;
      char *dB = nullptr;
      if (d2h_kernel()) {
        void *v = nullptr;
        if (hipHostGetDevicePointer(&v, B, 0) == hipSuccess) dB = static_cast<char *>(v);
      }
      auto part = [&](uint64_t off, const void *src, uint64_t bytes) -> bool {
        if (!bytes) return true;
        if (dB && co.n < CopyOut::kMax) {
          co.src[co.n] = src;
          co.dst[co.n] = dB + off;
          co.bytes[co.n++] = bytes;
          return true;
        }
        return hipMemcpyAsync(B + off, src, bytes, hipMemcpyDeviceToHost, st) == hipSuccess;
      };
      if (!part(o_off, dn.offsets, 8 * n1) || !part(o_sh, dn.shared_offsets, 8 * n1)) return MQM_EHIP;
      if (mo.n_deliveries && !part(o_d, dn.deliveries, dsz * mo.n_deliveries)) return MQM_EHIP;
      if (mo.n_shared && !part(o_s, dn.shared, 4 * mo.n_shared)) return MQM_EHIP;
      if (runs) {
        r->run_offsets = reinterpret_cast<const uint64_t *>(B + o_ro);
        r->runs = reinterpret_cast<const mqm_run *>(B + o_r);
        r->n_solo = mo.n_solo;
        if (!part(o_ro, ro.offsets, 8 * n1)) return MQM_EHIP;
        if (ro.n_runs && !part(o_r, ro.runs, 8 * ro.n_runs)) return MQM_EHIP;
      }
      if (want_ids) {
        r->has_idents = true;
        r->ident_offsets = reinterpret_cast<const uint64_t *>(B + o_io);
        r->idents = reinterpret_cast<const uint32_t *>(B + o_i);
        if (!part(o_io, io.offsets, 8 * n1)) return MQM_EHIP;
        if (ni && !part(o_i, io.sids, 4 * ni)) return MQM_EHIP;
      }
      if (co.n) {
        const int ce = copy_out_device(co, st);
        if (ce == -4) {  // (a part off the kernel's alignment: the DMA copies)
          for (int k = 0; k < co.n; k++)
            if (hipMemcpyAsync(B + (static_cast<char *>(co.dst[k]) - dB), co.src[k], co.bytes[k],
                               hipMemcpyDeviceToHost, st) != hipSuccess)
              return MQM_EHIP;
        } else if (ce != 0) {
          return hip_rc(ce);
        }
      }
      if (ws.end(st) || hipStreamSynchronize(st) != hipSuccess) return MQM_EHIP;
      tb[4] = clk::now();
      auto ns = [](clk::duration x) { return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(x).count(); };
      h->batch_ns[0].fetch_add(ns(tb[0] - ts[0]), std::memory_order_relaxed);
      for (int i = 1; i < 5; i++) h->batch_ns[i].fetch_add(ns(tb[i] - tb[i - 1]), std::memory_order_relaxed);
      h->batch_calls.fetch_add(1, std::memory_order_relaxed);
      if (runs && r->run_offsets[n_topics] != ro.n_runs) {  // the records' part counts vs the walk's tally
        fprintf(stderr, "mqmatch: runs form: %llu runs listed, %llu counted by the walk\n",
                (unsigned long long)r->run_offsets[n_topics], (unsigned long long)ro.n_runs);
        return MQM_EHIP;
      }
      return MQM_OK;
    }();
    ctx_release(h, std::move(c));
    if (rc != MQM_OK) return rc;
    *out = r.release();
    return MQM_OK;
  });
}

extern "C" {

int mqm_match_batch(mqm_index *h, const char *topic_bytes, const uint64_t *topic_offsets, uint32_t n_topics,
                    mqm_result **out) {
  return match_batch_impl(h, topic_bytes, topic_offsets, n_topics, false, out);
}

int mqm_match_batch_packed(mqm_index *h, const char *topic_bytes, const uint64_t *topic_offsets, uint32_t n_topics,
                           mqm_result **out) {
  return match_batch_impl(h, topic_bytes, topic_offsets, n_topics, true, out);
}

int mqm_match_batch_runs(mqm_index *h, const char *topic_bytes, const uint64_t *topic_offsets, uint32_t n_topics,
                         mqm_result **out) {
  return match_batch_impl(h, topic_bytes, topic_offsets, n_topics, true, out, false, true);
}

}  // extern "C"

// a caller-owned context of the queued device API (mqm_match_device_async)
struct mqm_match_ctx {
  mqm_index *h = nullptr;
  MatchCtx c;
  hipStream_t st = nullptr;
  const uint8_t *bytes = nullptr;
  const uint64_t *offs = nullptr;
  uint32_t n = 0;
  bool queued = false;
};

extern "C" {

int mqm_match_ctx_create(mqm_index *h, mqm_match_ctx **out) {
  if (!h || !out) return MQM_EINVAL;
  *out = nullptr;
  return guarded([&] {
    if (h->cfg.device == MQM_DEVICE_NONE) return MQM_ENODEV;
    if (hipSetDevice(h->cfg.device) != hipSuccess) return MQM_EHIP;
    auto x = std::make_unique<mqm_match_ctx>();
    x->h = h;
    h->live_ctxs.fetch_add(1, std::memory_order_acq_rel);
    *out = x.release();
    return MQM_OK;
  });
}

int mqm_match_ctx_destroy(mqm_match_ctx *x) {
  if (!x) return MQM_EINVAL;
  if (x->queued) (void)hipStreamSynchronize(x->st);
  (void)x->c.ws.drain();
  mqm_index *h = x->h;
  delete x;
  h->live_ctxs.fetch_sub(1, std::memory_order_acq_rel);
  return MQM_OK;
}

int mqm_match_device_async(mqm_match_ctx *x, const uint8_t *d_topic_bytes, const uint64_t *d_topic_offsets,
                           uint32_t n_topics, void *hip_stream) {
  if (!x || x->queued || (n_topics && (!d_topic_bytes || !d_topic_offsets))) return MQM_EINVAL;
  return guarded([&] {
    mqm_index *h = x->h;
    if (hipSetDevice(h->cfg.device) != hipSuccess) return MQM_EHIP;
    std::shared_ptr<GpuSnapshot> snap;
    int rc = front(h, &snap);
    if (rc != MQM_OK) return rc;
    const hipStream_t st = (hipStream_t)hip_stream;
    x->c.snap = snap;  // held until the next call on this context
    x->c.has_mo = false;
    x->c.ws.begin(st);
    x->c.ws.ident_early = h->ident_early.load(std::memory_order_relaxed);
    rc = match_enqueue(snap->dev, x->c.ws, d_topic_bytes, d_topic_offsets, n_topics, st, false);
    if (x->c.ws.end(st)) rc = rc ? rc : -3;
    if (rc != 0) return hip_rc(rc);
    x->st = st;
    x->bytes = d_topic_bytes;
    x->offs = d_topic_offsets;
    x->n = n_topics;
    x->queued = true;
    return MQM_OK;
  });
}

int mqm_match_ctx_wait(mqm_match_ctx *x, mqm_device_result *out) {
  if (!x || !out || !x->queued) return MQM_EINVAL;
  return guarded([&] {
    x->queued = false;
    if (hipSetDevice(x->h->cfg.device) != hipSuccess) return MQM_EHIP;
    MatchOutput mo;
    int rc = match_collect(x->c.ws, x->st, &mo);
    if (rc == 1) {  // outgrew the buffers earlier calls sized: again, sized exactly
      x->c.ws.begin(x->st);
      rc = match_enqueue(x->c.snap->dev, x->c.ws, x->bytes, x->offs, x->n, x->st, true);
      if (x->c.ws.end(x->st)) rc = rc ? rc : -3;
      if (rc == 0) rc = match_collect(x->c.ws, x->st, &mo);
      if (rc == 0) x->c.ws.requeued++;
    }
    if (rc != 0) return hip_rc(rc);
    x->c.last_mo = mo;
    x->c.has_mo = true;
    fill_device_result(mo, x->c.ws, out);
    return MQM_OK;
  });
}

int mqm_match_ctx_stats(mqm_match_ctx *x, uint64_t *requeued) {
  if (!x || !requeued) return MQM_EINVAL;
  *requeued = x->c.ws.requeued;
  return MQM_OK;
}

int mqm_identifiers_device(mqm_index *h, void *hip_stream, mqm_device_identifiers *out) {
  if (!h || !out) return MQM_EINVAL;
  return guarded([&] {
    if (h->cfg.device == MQM_DEVICE_NONE) return MQM_ENODEV;
    std::lock_guard<std::mutex> g(h->dev_mu);
    MatchCtx &c = h->dev;
    if (!c.has_mo) return MQM_EINVAL;  // the records of the last mqm_match_device call
    if (hipSetDevice(h->cfg.device) != hipSuccess) return MQM_EHIP;
    const hipStream_t st = (hipStream_t)hip_stream;
    c.ws.begin(st);
    IdentOutput io;
    int rc = identifiers_device(c.snap->dev, c.ws, st, &io);
    if (c.ws.end(st)) rc = rc ? rc : -3;
    if (rc != 0) return hip_rc(rc);
    out->n_topics = io.n_topics;
    out->n_idents = io.n_idents;
    out->offsets = io.offsets;
    out->sids = io.sids;
    return MQM_OK;
  });
}

int mqm_dense_device(mqm_index *h, void *hip_stream, mqm_device_dense *out) {
  if (!h || !out) return MQM_EINVAL;
  return guarded([&] {
    if (h->cfg.device == MQM_DEVICE_NONE) return MQM_ENODEV;
    std::lock_guard<std::mutex> g(h->dev_mu);
    MatchCtx &c = h->dev;
    if (!c.has_mo) return MQM_EINVAL;
    if (hipSetDevice(h->cfg.device) != hipSuccess) return MQM_EHIP;
    const hipStream_t st = (hipStream_t)hip_stream;
    c.ws.begin(st);
    DenseOutput dn;
    int rc = densify(c.snap->dev, c.ws, c.last_mo, st, &dn);
    if (c.ws.end(st)) rc = rc ? rc : -3;
    if (rc != 0) return hip_rc(rc);
    out->n_topics = c.last_mo.n_topics;
    out->n_deliveries = c.last_mo.n_deliveries;
    out->n_shared = c.last_mo.n_shared;
    out->offsets = dn.offsets;
    out->deliveries = reinterpret_cast<const mqm_delivery *>(dn.deliveries);
    out->shared_offsets = dn.shared_offsets;
    out->shared = dn.shared;
    return MQM_OK;
  });
}

namespace {
// device-visible status word for the gather kernels (pinned, mapped)
int gather_status(unsigned int **host, unsigned int **dev) {
  static unsigned int *bad = nullptr;
  if (!bad && hipHostMalloc((void **)&bad, sizeof(unsigned int), hipHostMallocMapped) != hipSuccess) {
    bad = nullptr;
    return MQM_EHIP;
  }
  *bad = 0;
  *host = bad;
  return hipHostGetDevicePointer((void **)dev, bad, 0) == hipSuccess ? MQM_OK : MQM_EHIP;
}
std::mutex gather_mu;
}  // namespace

int mqm_gather_shards(uint32_t n_topics, uint32_t n_shards, const mqm_shard_part *parts, void *hip_stream,
                      uint64_t *d_out_offsets, mqm_delivery *d_out) {
  if (!parts || !d_out_offsets || n_shards == 0 || n_shards > (uint32_t)kMaxShards) return MQM_EINVAL;
  return guarded([&] {
    std::lock_guard<std::mutex> g(gather_mu);
    unsigned int *bad = nullptr, *dbad = nullptr;
    if (gather_status(&bad, &dbad) != MQM_OK) return MQM_EHIP;
    ShardPart p[kMaxShards];
    for (uint32_t r = 0; r < n_shards; r++)
      p[r] = ShardPart{parts[r].offsets, reinterpret_cast<const uint64_t *>(parts[r].deliveries),
                       parts[r].client_map, parts[r].n_map};
    const int rc = gather_shards(n_topics, n_shards, p, (hipStream_t)hip_stream, d_out_offsets,
                                 reinterpret_cast<uint64_t *>(d_out), dbad);
    if (rc == -1) return MQM_EINVAL;
    if (rc != 0) return MQM_EHIP;
    if (hipStreamSynchronize((hipStream_t)hip_stream) != hipSuccess) return MQM_EHIP;
    return *(volatile unsigned int *)bad ? MQM_EINVAL : MQM_OK;
  });
}

int mqm_gather_shards_shared(uint32_t n_topics, uint32_t n_shards, const mqm_shard_shared_part *parts,
                             void *hip_stream, uint64_t *d_out_offsets, uint32_t *d_out) {
  if (!parts || !d_out_offsets || n_shards == 0 || n_shards > (uint32_t)kMaxShards) return MQM_EINVAL;
  return guarded([&] {
    std::lock_guard<std::mutex> g(gather_mu);
    unsigned int *bad = nullptr, *dbad = nullptr;
    if (gather_status(&bad, &dbad) != MQM_OK) return MQM_EHIP;
    const uint64_t *offs[kMaxShards];
    const uint32_t *ids[kMaxShards];
    for (uint32_t r = 0; r < n_shards; r++) {
      offs[r] = parts[r].offsets;
      ids[r] = parts[r].shared;
    }
    const int rc = gather_shards_shared(n_topics, n_shards, offs, ids, (hipStream_t)hip_stream, d_out_offsets, d_out,
                                        dbad);
    if (rc == -1) return MQM_EINVAL;
    if (rc != 0) return MQM_EHIP;
    if (hipStreamSynchronize((hipStream_t)hip_stream) != hipSuccess) return MQM_EHIP;
    return *(volatile unsigned int *)bad ? MQM_EINVAL : MQM_OK;
  });
}

int mqm_result_identifiers(const mqm_result *r, const uint64_t **offsets, const uint32_t **sids) {
  if (!r || !offsets || !sids || !r->has_idents) return MQM_EINVAL;
  *offsets = r->ident_offsets;
  *sids = r->idents;
  return MQM_OK;
}

int mqm_messages_device(mqm_index *h, const uint8_t *d_filter_bytes, const uint64_t *d_filter_offsets,
                        uint32_t n_filters, void *hip_stream, mqm_device_messages *out) {
  if (!h || !out || (n_filters && (!d_filter_bytes || !d_filter_offsets))) return MQM_EINVAL;
  return guarded([&] {
    if (h->cfg.device == MQM_DEVICE_NONE) return MQM_ENODEV;
    if (hipSetDevice(h->cfg.device) != hipSuccess) return MQM_EHIP;
    std::shared_ptr<GpuSnapshot> snap;
    int rc = front(h, &snap);
    if (rc != MQM_OK) return rc;
    std::lock_guard<std::mutex> g(h->dev_mu);
    MatchCtx &c = h->dev;
    if (c.ws.drain()) return MQM_EHIP;
    c.has_mo = false;  // the forward-match records share nothing, but the snapshot changes
    c.snap = snap;
    const hipStream_t st = (hipStream_t)hip_stream;
    c.ws.begin(st);
    MessagesOutput mo;
    rc = messages_device(snap->dev, snap->has_retained ? &snap->ret : nullptr, c.ws, d_filter_bytes,
                         d_filter_offsets, n_filters, st, &mo);
    if (c.ws.end(st)) rc = rc ? rc : -3;
    if (rc != 0) return hip_rc(rc);
    out->n_filters = mo.n_filters;
    out->n_refs = mo.n_refs;
    out->offsets = mo.offsets;
    out->refs = mo.refs;
    out->n_ranges = mo.n_emissions;
    out->n_items = mo.n_items;
    out->n_skipped = mo.n_skipped;
    return MQM_OK;
  });
}

int mqm_messages_batch(mqm_index *h, const char *filter_bytes, const uint64_t *filter_offsets, uint32_t n_filters,
                       mqm_messages **out) {
  if (!h || !out || !filter_offsets || (n_filters && !filter_bytes)) return MQM_EINVAL;
  *out = nullptr;
  return guarded([&] {
    if (h->cfg.device == MQM_DEVICE_NONE) return MQM_ENODEV;
    if (hipSetDevice(h->cfg.device) != hipSuccess) return MQM_EHIP;
    std::shared_ptr<GpuSnapshot> snap;
    int rc = front(h, &snap);
    if (rc != MQM_OK) return rc;
    auto c = ctx_acquire(h, &rc);
    if (rc != MQM_OK) return rc;
    auto m = std::make_unique<mqm_messages>();
    rc = [&]() -> int {
      Workspace &ws = c->ws;
      const hipStream_t st = c->stream;
      ws.begin(st);
      const uint8_t *d_bytes = nullptr;
      const uint64_t *d_offs = nullptr;
      int e = upload_batch(c.get(), Workspace::kRInBytes, Workspace::kRInOffs, filter_bytes, filter_offsets,
                           n_filters, &d_bytes, &d_offs);
      if (e != MQM_OK) return e;
      MessagesOutput mo;
      e = messages_device(snap->dev, snap->has_retained ? &snap->ret : nullptr, ws, d_bytes, d_offs, n_filters, st,
                          &mo);
      if (e != 0) return hip_rc(e);
      m->n = n_filters;
      m->offsets.resize(n_filters + 1);
      m->refs.resize(mo.n_refs);
      if (hipMemcpyAsync(m->offsets.data(), mo.offsets, sizeof(uint64_t) * (n_filters + 1), hipMemcpyDeviceToHost,
                         st) != hipSuccess)
        return MQM_EHIP;
      if (mo.n_refs &&
          hipMemcpyAsync(m->refs.data(), mo.refs, sizeof(uint64_t) * mo.n_refs, hipMemcpyDeviceToHost, st) != hipSuccess)
        return MQM_EHIP;
      if (ws.end(st) || hipStreamSynchronize(st) != hipSuccess) return MQM_EHIP;
      return MQM_OK;
    }();
    ctx_release(h, std::move(c));
    if (rc != MQM_OK) return rc;
    *out = m.release();
    return MQM_OK;
  });
}

int mqm_messages_one(mqm_index *h, const char *filter, size_t filter_len, mqm_messages **out) {
  uint64_t offs[2] = {0, filter_len};
  return mqm_messages_batch(h, filter ? filter : "", offs, 1, out);
}

uint32_t mqm_messages_num_filters(const mqm_messages *m) { return m ? m->n : 0; }
const uint64_t *mqm_messages_offsets(const mqm_messages *m) { return m ? m->offsets.data() : nullptr; }
const uint64_t *mqm_messages_refs(const mqm_messages *m) { return m ? m->refs.data() : nullptr; }
void mqm_messages_free(mqm_messages *m) { delete m; }

namespace {

// MQM_CFG_BATCHING: single-topic calls queue a request and wait; worker
// threads drain the queue into GPU batches.  Calls that arrive while a batch
// runs form the next one, so batches grow with the offered load and an idle
// index adds no latency.  MQM_BATCH_WORKERS workers (default 3): while one
// waits for its batch on the GPU, the others gather and launch the next ones
// (each borrows its own context: workspace, stream, pinned blocks).  A batch
// takes the small-batch path (fast.hip: one launch); each caller is woken on
// its own futex and copies its own topic's result out of the batch's pinned
// blocks (in parallel, on the callers' threads); the last one returns the
// context to the pool.  With a topic past the small-batch path's capacities
// the worker runs mqm_match_batch and splits the result.
struct Collector {
  struct Req;
  struct Batch {  // one small-batch call, shared by its callers until they have copied their results
    mqm_index *h = nullptr;
    std::unique_ptr<MatchCtx> ctx;
    std::shared_ptr<GpuSnapshot> snap;
    FastOutput fo;
    std::atomic<uint32_t> refs{0};
    void release() {
      if (refs.fetch_sub(1, std::memory_order_acq_rel) == 1) {
        ctx_release(h, std::move(ctx));
        delete this;
      }
    }
  };
  struct Req {
    const char *topic;
    size_t len;
    mqm_result *res = nullptr;
    int rc = MQM_OK;
    Batch *batch = nullptr;  // set: copy topic `index` of the batch's result
    uint32_t index = 0;
    std::atomic<uint32_t> state{0};  // futex word: 0 waiting, 1 done
    void wake() {
      state.store(1, std::memory_order_release);
      syscall(SYS_futex, reinterpret_cast<uint32_t *>(&state), FUTEX_WAKE_PRIVATE, 1, nullptr, nullptr, 0);
    }
    void wait() {
      while (state.load(std::memory_order_acquire) == 0)
        syscall(SYS_futex, reinterpret_cast<uint32_t *>(&state), FUTEX_WAIT_PRIVATE, 0, nullptr, nullptr, 0);
    }
  };
  mqm_index *h;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<Req *> q;
  bool stop = false;
  uint32_t max_batch = 8192, linger_us = 0;
  uint64_t batches = 0, topics = 0;
  std::vector<std::thread> ths;

  explicit Collector(mqm_index *idx) : h(idx) {
    int workers = 3;
    if (const char *e = getenv("MQM_BATCH_WORKERS")) workers = std::max(1, std::min(16, atoi(e)));
    for (int i = 0; i < workers; i++) ths.emplace_back([this] { run(); });
  }
  ~Collector() {
    {
      std::lock_guard<std::mutex> g(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto &t : ths) t.join();
  }

  int submit(const char *topic, size_t len, mqm_result **out) {
    Req r{topic ? topic : "", len};
    {
      std::lock_guard<std::mutex> g(mu);
      q.push_back(&r);
    }
    cv.notify_one();
    r.wait();
    if (r.batch) {  // the small-batch path: this caller's topic, copied off the batch's blocks
      const FastOutput &fo = r.batch->fo;
      const FastRec &x = fo.recs[r.index];
      try {
        r.rc = single(r.batch->snap->host, fo.dout + x.dbase, x.dcount, fo.hout + x.hbase, x.hcount,
                      fo.iout ? fo.iout + x.ibase : nullptr, fo.iout ? x.icount : 0, fo.iout != nullptr, &r.res);
      } catch (const std::bad_alloc &) {
        r.rc = MQM_ENOMEM;
      }
      r.batch->release();
    }
    *out = r.res;
    return r.rc;
  }

  // one topic's deliveries / shared candidates as a result of its own (host memory)
  static int single(std::shared_ptr<const HostSnapshot> hs, const uint64_t *dl, uint64_t d, const uint32_t *sh,
                    uint64_t sn, const uint32_t *ids, uint64_t in, bool has_ids, mqm_result **out) {
    auto r = std::make_unique<mqm_result>();
    auto up = [](uint64_t x) { return (x + 15) & ~15ull; };
    const uint64_t o_sh = 16, o_io = 32, o_d = 48, o_s = o_d + up(8 * d), o_i = o_s + up(4 * sn), total = o_i + up(4 * in);
    if (!r->alloc(nullptr, total, false)) return MQM_ENOMEM;
    char *B = static_cast<char *>(r->blk);
    uint64_t *off = reinterpret_cast<uint64_t *>(B), *soff = reinterpret_cast<uint64_t *>(B + o_sh),
             *ioff = reinterpret_cast<uint64_t *>(B + o_io);
    off[0] = soff[0] = ioff[0] = 0;
    off[1] = d;
    soff[1] = sn;
    ioff[1] = in;
    if (d) memcpy(B + o_d, dl, 8 * d);
    if (sn) memcpy(B + o_s, sh, 4 * sn);
    if (in) memcpy(B + o_i, ids, 4 * in);
    r->n = 1;
    r->offsets = off;
    r->shared_offsets = soff;
    r->deliveries = reinterpret_cast<const mqm_delivery *>(B + o_d);
    r->shared = reinterpret_cast<const uint32_t *>(B + o_s);
    if (has_ids) {
      r->has_idents = true;
      r->ident_offsets = ioff;
      r->idents = reinterpret_cast<const uint32_t *>(B + o_i);
    }
    r->snap = std::move(hs);
    *out = r.release();
    return MQM_OK;
  }

  // topic i of batch result b as a result of its own
  static int split(const mqm_result *b, uint32_t i, mqm_result **out) {
    const uint64_t d0 = b->offsets[i], d = b->offsets[i + 1] - d0;
    const uint64_t s0 = b->shared_offsets[i], sn = b->shared_offsets[i + 1] - s0;
    const uint64_t i0 = b->has_idents ? b->ident_offsets[i] : 0, in = b->has_idents ? b->ident_offsets[i + 1] - i0 : 0;
    return single(b->snap, reinterpret_cast<const uint64_t *>(b->deliveries) + d0, d, b->shared + s0, sn,
                  b->has_idents ? b->idents + i0 : nullptr, in, b->has_idents, out);
  }

  // the batch on the small-batch path: a Batch the callers copy their results
  // from; nullptr when not taken (the worker falls back to the batch pipeline;
  // *ran: the small-batch kernel ran and reported a topic past its capacities)
  Batch *run_fast(const std::vector<Req *> &batch, const std::string &bytes, const std::vector<uint64_t> &offs,
                  bool *ran) {
    *ran = false;
    if (!h->fast_path || batch.size() > kFastMaxTopics) return nullptr;
    if (hipSetDevice(h->cfg.device) != hipSuccess) return nullptr;
    auto b = std::make_unique<Batch>();
    b->h = h;
    if (front(h, &b->snap) != MQM_OK) return nullptr;
    int rc = MQM_OK;
    b->ctx = ctx_acquire(h, &rc);
    if (rc != MQM_OK) return nullptr;
    b->ctx->ws.begin(b->ctx->stream);
    const int e = match_small(b->snap->dev, b->ctx->ws, bytes.data(), offs.data(), (uint32_t)batch.size(),
                              b->ctx->stream, &b->fo, (h->cfg.flags & MQM_CFG_IDENTIFIERS) != 0);
    const int e2 = b->ctx->ws.end(b->ctx->stream);
    if (e != 0 || e2) {
      *ran = e == 1 && !e2;
      ctx_release(h, std::move(b->ctx));
      return nullptr;
    }
    b->refs.store((uint32_t)batch.size(), std::memory_order_relaxed);
    return b.release();
  }

  void run() {
    std::vector<Req *> batch;
    std::string bytes;
    std::vector<uint64_t> offs;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return stop || !q.empty(); });
        if (q.empty()) return;  // stop requested and nothing pending
        if (linger_us && q.size() < max_batch) {
          cv.wait_for(lk, std::chrono::microseconds(linger_us), [&] { return stop || q.size() >= max_batch; });
          // another worker lingering on the same queue may have taken it all:
          // never run (or count) an empty batch
          if (q.empty()) {
            if (stop) return;
            continue;
          }
        }
        const size_t n = std::min<size_t>(q.size(), max_batch);
        batch.assign(q.begin(), q.begin() + n);
        q.erase(q.begin(), q.begin() + n);
        batches++;
        topics += n;
        if (!q.empty()) cv.notify_one();  // more queued than one batch: wake another worker
      }
      bytes.clear();
      offs.assign(1, 0);
      for (Req *r : batch) {
        bytes.append(r->topic, r->len);
        offs.push_back(bytes.size());
      }
      Batch *fb = nullptr;
      bool ran_small = false;
      try {
        fb = run_fast(batch, bytes, offs, &ran_small);
      } catch (...) {
        fb = nullptr;
      }
      if (fb) {
        for (uint32_t i = 0; i < batch.size(); i++) {
          batch[i]->batch = fb;
          batch[i]->index = i;
        }
        for (Req *r : batch) r->wake();
        continue;
      }
      mqm_result *b = nullptr;
      // (a batch the small-batch kernel already rejected skips it: one launch, not two)
      const int rc = match_batch_impl(h, bytes.data(), offs.data(), (uint32_t)batch.size(), false, &b, ran_small);
      for (uint32_t i = 0; i < batch.size(); i++) {
        batch[i]->rc = rc;
        if (rc == MQM_OK) {
          try {
            batch[i]->rc = split(b, i, &batch[i]->res);
          } catch (const std::bad_alloc &) {
            batch[i]->rc = MQM_ENOMEM;
          }
        }
      }
      if (b) mqm_result_free(b);
      for (Req *r : batch) r->wake();
    }
  }
};

// MQM_CFG_SERVE: the persistent per-publish server (fast.hip k_serve).
//
// Snapshots: every launch serves one snapshot and writes its version into
// each slot it answers; the caller decodes the result's sids with the host
// snapshot of that version (the last kHist launches' are kept), never with a
// snapshot it merely read before posting.  The server only ever moves to a
// newer snapshot (a caller holding an older front buffer does not relaunch
// it), and a caller posts only once the running launch's snapshot is at least
// as new as its own front buffer, so a result never predates the caller's
// view of the store (MQM_CFG_AUTOCOMMIT: read-your-writes).
void server_register(Server *s);
void server_unregister(Server *s);

struct Server {
  mqm_index *h;
  ServeQueue *q = nullptr;            // pinned, coherent, device-mapped
  unsigned long long *ctr = nullptr;  // device: [0] the next request number a workgroup takes, [1] exited workgroups
  unsigned long long *restart = nullptr;  // pinned: ctr's values for the next launch (ensure)
  hipStream_t st = nullptr;
  std::mutex mu;                      // launches / snapshot switches
  std::shared_ptr<GpuSnapshot> snap;  // (mu) what the running launch reads
  bool launched = false;              // (mu) a launch may still run
  uint64_t gen = 0;                   // (mu) launches so far = the running launch's generation
  uint64_t seen = 0;                  // (mu) request numbers handed out by the launches so far
  uint32_t grid = 32, idle_us = 20000;
  uint32_t max_grid = 128;            // half the device's CUs (init): batch-path kernels keep the rest
  const bool want_ids;
  // the running launch, readable without mu: generation, snapshot version + 1 (0: none)
  std::atomic<uint64_t> run_gen{0}, run_ver{0};
  // host snapshots of recent launches (decoding a result whose launch served
  // a snapshot other than the caller's front buffer), with the generation of
  // the launch that added each.  At C3 a host snapshot is 1-2 GB, so an entry
  // is kept only while a request posted under its launch or a later one may
  // still be decoded: a caller stores the running generation + 1 in
  // post_gen[slot] before it posts and clears it after decoding, and ensure()
  // drops the entries older than the oldest such generation (at most kHist
  // are kept in any case; an evicted version decodes on the batch path)
  static constexpr uint32_t kHist = 8;
  std::mutex hist_mu;
  struct Hist {
    uint64_t gen = 0;
    std::shared_ptr<const HostSnapshot> host;
  };
  Hist hist[kHist];
  uint32_t hist_next = 0;
  std::unique_ptr<std::atomic<uint64_t>[]> post_gen;  // slot -> launch generation + 1 at post (0: none in flight)
  std::atomic<uint64_t> ticket{0};
  std::unique_ptr<SlotOwners> slots;  // which ticket owns each ring slot (serve_slots.h; created by init)
  std::atomic<uint64_t> served{0}, fallbacks{0}, launches{0}, stale{0}, forced{0};
  std::atomic<uint64_t> result_timeouts{0};  // (mqm_serve_counters; slot timeouts: SlotOwners)
  std::atomic<uint64_t> device_ticks{0};  // claim -> publish on the device, summed (100 MHz ticks)
  std::atomic<uint64_t> phase_ticks[3] = {};  // stage + keys, walk, emission + publish
  std::atomic<uint64_t> timed{0};
  // host-side time per call (ns, summed; mqm_serve_host_us reads and resets):
  // entry -> posted, posted -> result seen, result seen -> returned; calls that slept
  std::atomic<uint64_t> host_ns[3] = {}, host_calls{0}, host_slept{0};
  // the longest call per host phase (ns; mqm_serve_host_max_us reads and
  // resets): front buffer, server check / relaunch, slot wait + post, result
  // wait, result block; then the longest batch-path fallback, calls > 10 ms
  std::atomic<uint64_t> host_max_ns[6] = {}, host_slow{0};
  static void note_max(std::atomic<uint64_t> &m, uint64_t v) {
    uint64_t c = m.load(std::memory_order_relaxed);
    while (v > c && !m.compare_exchange_weak(c, v, std::memory_order_relaxed)) {
    }
  }
  // completion pollers: callers that stopped spinning sleep on waitw[slot];
  // poller p watches the done words of the sleepers on slots i = p mod
  // n_pollers and wakes them (one thread's FUTEX_WAKE calls cap the wake rate
  // near 0.6M/s)
  std::unique_ptr<std::atomic<uint64_t>[]> waiting;  // slot -> the done value its sleeper waits for (0: none)
  std::unique_ptr<std::atomic<uint32_t>[]> waitw;    // futex words
  struct Poller {
    std::atomic<uint32_t> sleepers{0}, word{0};
    std::thread th;
  };
  // 3: measured on the 16-CPU box (r04p-r04r, 1M-filter index): 1 / 2 / 3 / 4
  // pollers give 0.51 / 0.78 / 1.07 / 1.07M calls/s from 64 callers, and
  // with 128 callers 3 pollers keep 0.96M where 4 spin the process into its
  // CPU quota (0.37M)
  static constexpr uint32_t n_pollers = 3;
  Poller pollers[n_pollers];
  std::atomic<uint32_t> inflight{0};
  std::atomic<int64_t> last_check_ns{0};  // the last liveness check of a late caller (steady clock)
  std::atomic<bool> poller_quit{false};
  bool counted = false;  // (serve_count: the rebuild's default thread count while a server lives)
  void poke_poller(Poller &pl) {
    pl.word.fetch_add(1, std::memory_order_acq_rel);
    syscall(SYS_futex, reinterpret_cast<uint32_t *>(&pl.word), FUTEX_WAKE_PRIVATE, 1, nullptr, nullptr, 0);
  }
  void poll_loop(uint32_t p) {
    Poller &pl = pollers[p];
    while (!poller_quit.load(std::memory_order_acquire)) {
      const uint32_t pw = pl.word.load(std::memory_order_acquire);
      if (pl.sleepers.load(std::memory_order_acquire) == 0) {
        const struct timespec ts = {0, 1000000};  // 1 ms (quit is checked at least that often)
        syscall(SYS_futex, reinterpret_cast<uint32_t *>(&pl.word), FUTEX_WAIT_PRIVATE, pw, &ts, nullptr, 0);
        continue;
      }
      for (uint32_t i = p; i < kServeSlots; i += n_pollers) {
        const uint64_t w = waiting[i].load(std::memory_order_acquire);
        if (w && __atomic_load_n(&q->done[i], __ATOMIC_ACQUIRE) == w && !waitw[i].load(std::memory_order_relaxed)) {
          waitw[i].store(1, std::memory_order_release);
          syscall(SYS_futex, reinterpret_cast<uint32_t *>(&waitw[i]), FUTEX_WAKE_PRIVATE, 1, nullptr, nullptr, 0);
        }
      }
      __builtin_ia32_pause();
    }
  }

  explicit Server(mqm_index *idx) : h(idx), want_ids((idx->cfg.flags & MQM_CFG_IDENTIFIERS) != 0) {
    waiting.reset(new std::atomic<uint64_t>[kServeSlots]);
    waitw.reset(new std::atomic<uint32_t>[kServeSlots]);
    for (uint32_t i = 0; i < kServeSlots; i++) {
      waiting[i].store(0);
      waitw[i].store(0);
    }
  }
  int init() {
    if (hipSetDevice(h->cfg.device) != hipSuccess) return MQM_EHIP;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->cfg.device) == hipSuccess && cus > 1)
      max_grid = (uint32_t)cus / 2;
    void *p = nullptr;
    if (hipHostMalloc(&p, sizeof(ServeQueue), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
      return MQM_ENOMEM;
    q = static_cast<ServeQueue *>(p);
    memset((void *)q, 0, sizeof(ServeQueue));
    slots = std::make_unique<SlotOwners>(kServeSlots, q->done);
    post_gen.reset(new std::atomic<uint64_t>[kServeSlots]);
    for (uint32_t i = 0; i < kServeSlots; i++) post_gen[i].store(0);
    if (hipMalloc(&ctr, 2 * sizeof(unsigned long long)) != hipSuccess) return MQM_ENOMEM;
    if (hipHostMalloc(&restart, 2 * sizeof(unsigned long long), hipHostMallocDefault) != hipSuccess) {
      restart = nullptr;
      return MQM_ENOMEM;
    }
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return MQM_EHIP;
    if (hipMemsetAsync(ctr, 0, 2 * sizeof(unsigned long long), st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return MQM_EHIP;
    for (uint32_t p = 0; p < n_pollers; p++) pollers[p].th = std::thread([this, p] { poll_loop(p); });
    serve_count(+1);
    counted = true;
    server_register(this);
    return MQM_OK;
  }
  // (mu held) stop a running kernel and wait for it
  void halt() {
    run_ver.store(0, std::memory_order_release);
    if (!launched) return;
    __atomic_store_n(&q->stop, 1ull, __ATOMIC_SEQ_CST);
    const auto t0 = std::chrono::steady_clock::now();
    (void)hipStreamSynchronize(st);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (ms > 50.0) fprintf(stderr, "mqmatch: per-publish server: stopping the kernel took %.1f ms\n", ms);
    __atomic_store_n(&q->stop, 0ull, __ATOMIC_SEQ_CST);
    launched = false;
  }
  ~Server() {
    if (counted) {
      server_unregister(this);  // (waits for a reaper pass that holds this server stopped)
      serve_count(-1);
    }
    poller_quit.store(true, std::memory_order_release);
    for (uint32_t p = 0; p < n_pollers; p++)
      if (pollers[p].th.joinable()) {
        poke_poller(pollers[p]);
        pollers[p].th.join();
      }
    if (q) {
      std::lock_guard<std::mutex> g(mu);
      halt();
    }
    if (st) (void)hipStreamDestroy(st);
    if (ctr) (void)hipFree(ctr);
    if (restart) (void)hipHostFree(restart);
    if (q) (void)hipHostFree(q);
  }
  // the running launch's last workgroup has exited (idle): a posted request
  // waits for a relaunch
  bool exited() const {
    return __atomic_load_n(&q->exited, __ATOMIC_ACQUIRE) == run_gen.load(std::memory_order_acquire);
  }
  // (mu held) a launch runs on a snapshot at least as new as `cur`: relaunch
  // when the server has exited or reads an older one.  Never moves back to an
  // older snapshot than the one it has run (a caller may hold a stale front
  // buffer: it then gets the newer snapshot's result, and decodes with it).
  int ensure(const std::shared_ptr<GpuSnapshot> &cur) {
    std::shared_ptr<GpuSnapshot> want = snap && snap->host->version >= cur->host->version ? snap : cur;
    if (launched && want == snap && !exited() && hipStreamQuery(st) == hipErrorNotReady) return MQM_OK;
    TraceSpan ts("ensure");
    halt();
    ts.mark("halt");
    defer_release(std::move(snap));  // (the launch that read it has stopped)
    snap = std::move(want);
    ts.mark("snapshot switch");
    if (hipSetDevice(h->cfg.device) != hipSuccess) return MQM_EHIP;
    // (no kernel runs now) the device counter restarts at the oldest request
    // not yet served (SlotOwners::oldest_unserved: exact however long a caller
    // sat between taking its ticket and posting — round 5 scanned the posted
    // slots plus the last kServeSlots tickets and skipped such a ticket, whose
    // request then waited for the forced relaunch, r05af).  A caller may move
    // on meanwhile: the minimum can only come out low, and the launch skips
    // served numbers below `seen` (k_serve) instead of serving them again.
    {
      unsigned long long c0 = 0;
      if (hipMemcpyAsync(&c0, ctr, sizeof(c0), hipMemcpyDeviceToHost, st) != hipSuccess ||
          hipStreamSynchronize(st) != hipSuccess)
        return MQM_EHIP;
      seen = std::max<uint64_t>(seen, c0);
    }
    const uint64_t T = ticket.load(std::memory_order_acquire);
    // (pinned: the copy reads it after this returns; the next ensure's halt
    // synchronises the stream before it is written again)
    restart[0] = slots->oldest_unserved(T);
    restart[1] = 0;
    if (hipMemcpyAsync(ctr, restart, 2 * sizeof(unsigned long long), hipMemcpyHostToDevice, st) != hipSuccess)
      return MQM_EHIP;
    const uint64_t ver = snap->host->version;
    if (serve_launch(snap->dev, q, ctr, grid, idle_us, want_ids, ver, gen + 1, std::max<uint64_t>(seen, T), st) != 0)
      return MQM_EHIP;
    gen++;
    launched = true;
    launches++;
    {
      // the oldest generation a result still to be decoded may carry
      uint64_t oldest = gen;
      for (uint32_t i = 0; i < kServeSlots; i++) {
        const uint64_t pg = post_gen[i].load(std::memory_order_seq_cst);
        if (pg) oldest = std::min(oldest, pg - 1);
      }
      std::lock_guard<std::mutex> g(hist_mu);
      const uint32_t last = (hist_next + kHist - 1) % kHist;
      for (uint32_t j = 0; j < kHist; j++)  // (the evicted host snapshots go to the releaser if this held the last reference)
        if (j != last && hist[j].host && hist[j].gen < oldest) defer_release(std::move(hist[j].host));
      if (hist[last].host && hist[last].host->version == ver) {
        hist[last].gen = gen;  // (the newest launch that served it)
      } else {
        defer_release(std::move(hist[hist_next].host));
        hist[hist_next] = Hist{gen, snap->host};
        hist_next = (hist_next + 1) % kHist;
      }
    }
    run_gen.store(gen, std::memory_order_release);
    run_ver.store(ver + 1, std::memory_order_release);
    ts.mark("relaunch");
    return MQM_OK;
  }
  // the host snapshot a launch of version `ver` served (nullptr: no longer kept)
  std::shared_ptr<const HostSnapshot> host_of(uint64_t ver, const std::shared_ptr<GpuSnapshot> &cur) {
    if (cur->host->version == ver) return cur->host;
    std::lock_guard<std::mutex> g(hist_mu);
    for (const auto &x : hist)
      if (x.host && x.host->version == ver) return x.host;
    return nullptr;
  }
  int submit(const char *topic, size_t len, mqm_result **out) {
    if (len > kServeTopic) {  // longer than a slot's topic bytes
      fallbacks++;
      return direct(topic, len, out);
    }
    using clk = std::chrono::steady_clock;
    const auto t_in = clk::now();
    std::shared_ptr<GpuSnapshot> cur;
    struct DeferCur {  // the caller's reference is dropped on the releaser thread
      std::shared_ptr<GpuSnapshot> &p;
      ~DeferCur() { defer_release(std::move(p)); }
    } defer_cur{cur};
    int rc = front_fast(h, &cur) ? MQM_OK : front(h, &cur);  // (commits first with MQM_CFG_AUTOCOMMIT)
    if (rc != MQM_OK) return rc;
    const auto t_front = clk::now();
    // before posting: the running launch serves a snapshot at least as new as
    // the caller's (any later launch is newer still)
    const uint64_t rv = run_ver.load(std::memory_order_acquire);
    if (rv == 0 || rv - 1 < cur->host->version || exited()) {
      std::lock_guard<std::mutex> g(mu);
      if ((rc = ensure(cur)) != MQM_OK) return rc;
    }
    const auto t_ens = clk::now();
    const uint64_t k = ticket.fetch_add(1, std::memory_order_relaxed);
    const uint32_t i = (uint32_t)(k % kServeSlots);
    if (!slots->wait(k, std::chrono::seconds(10))) {
      // (the slot's previous request never completed: the device is gone.
      // Request k is never posted: the slot passes on past it, and the next
      // relaunch skips its number)
      slots->give_up_unposted(k);
      fprintf(stderr,
              "mqmatch: per-publish server: ring slot %u not free after 10 s (request %llu; slot owner %llu, "
              "abandoned %llu, done %llu; ticket %llu, run_gen %llu, exited %llu, run_ver %llu)\n",
              i, (unsigned long long)k, (unsigned long long)slots->owner(i),
              (unsigned long long)slots->abandoned(i), (unsigned long long)slots->done(i),
              (unsigned long long)ticket.load(), (unsigned long long)run_gen.load(),
              (unsigned long long)__atomic_load_n(&q->exited, __ATOMIC_ACQUIRE), (unsigned long long)run_ver.load());
      return MQM_EHIP;
    }
    ServeSlot &sl = q->slot[i];
    memcpy(sl.topic, topic, len);
    sl.len = (uint32_t)len;
    // the length rides in the word the server polls, the first kServeHead
    // topic bytes in the same 64-B line (one PCIe read for a short topic),
    // checked by chk
    const unsigned long long seqw = (k + 1) | ((unsigned long long)len << kServeSeqBits);
    unsigned long long head[kServeHead / 8];
    memcpy(head, sl.topic, kServeHead);
    sl.chk = serve_check(seqw, head);
    // (before the post: a relaunch from here on keeps the host snapshots this
    // result may be decoded with — this launch's and every later one)
    post_gen[i].store(run_gen.load(std::memory_order_acquire) + 1, std::memory_order_seq_cst);
    __atomic_store_n(&sl.seq, seqw, __ATOMIC_RELEASE);
    // the server exited (idle) since the check above: relaunch now rather
    // than at the liveness check below (no HIP call on the common path)
    if (exited() || run_ver.load(std::memory_order_acquire) == 0) {
      std::lock_guard<std::mutex> g(mu);
      if ((rc = ensure(cur)) != MQM_OK) {
        post_gen[i].store(0, std::memory_order_release);
        slots->abandon(k);
        return rc;
      }
    }
    // spin on the slot's done word for a while (the single-caller latency
    // path), then sleep on a futex the completion poller wakes (more callers
    // than CPUs: a spinning caller would delay the ones whose results are
    // ready); a caller still without a result after 200 us makes sure a server
    // is still running (it exits after idle_us without a request; the request
    // then waits in the ring for the relaunch)
    const auto t0 = clk::now();
    bool ready = false;
    // (few callers in flight: spin through a whole call; many: sleep almost
    // at once — a spinning caller holds a CPU another caller's finished
    // result is waiting for)
    const auto spin_for = std::chrono::microseconds(inflight.fetch_add(1, std::memory_order_acq_rel) < 4 ? 300 : 2);
    for (uint32_t spin = 0; !ready; spin++) {
      __builtin_ia32_pause();
      ready = __atomic_load_n(&q->done[i], __ATOMIC_ACQUIRE) == k + 1;
      if (!ready && (spin & 15) == 15 && clk::now() - t0 > spin_for) break;
    }
    if (!ready) {
      waitw[i].store(0, std::memory_order_relaxed);
      waiting[i].store(k + 1, std::memory_order_release);
      Poller &pl = pollers[i % n_pollers];
      if (pl.sleepers.fetch_add(1, std::memory_order_acq_rel) == 0) poke_poller(pl);
      auto give_up = [&](int code) {
        waiting[i].store(0, std::memory_order_release);
        pl.sleepers.fetch_sub(1, std::memory_order_acq_rel);
        inflight.fetch_sub(1, std::memory_order_acq_rel);
        post_gen[i].store(0, std::memory_order_release);
        slots->abandon(k);
        return code;
      };
      while (__atomic_load_n(&q->done[i], __ATOMIC_ACQUIRE) != k + 1) {
        const struct timespec ts = {0, 500000};  // 500 us (a late result: the liveness check below)
        syscall(SYS_futex, reinterpret_cast<uint32_t *>(&waitw[i]), FUTEX_WAIT_PRIVATE, 0, &ts, nullptr, 0);
        if (__atomic_load_n(&q->done[i], __ATOMIC_ACQUIRE) == k + 1) break;
        // a wake meant for this slot's previous request (a waker that read
        // `waiting` before this call stored it): re-arm, so the wait sleeps
        waitw[i].store(0, std::memory_order_release);
        if (__atomic_load_n(&q->done[i], __ATOMIC_ACQUIRE) == k + 1) break;
        const auto now = clk::now();
        if (now - t0 > std::chrono::seconds(10)) {
          fprintf(stderr, "mqmatch: per-publish server: no result for 10 s\n");
          result_timeouts++;
          return give_up(MQM_EHIP);
        }
        // one liveness check per 200 us across all late callers (each is a
        // HIP call under mu; 64 callers checking at once cost more CPU than
        // the calls they wait for)
        const int64_t now_ns = std::chrono::duration_cast<std::chrono::nanoseconds>(now.time_since_epoch()).count();
        int64_t last = last_check_ns.load(std::memory_order_relaxed);
        if (now - t0 > std::chrono::microseconds(200) && now_ns - last > 200000 &&
            last_check_ns.compare_exchange_strong(last, now_ns, std::memory_order_acq_rel)) {
          std::lock_guard<std::mutex> g(mu);
          // a request unserved for a second while the launch runs: its number
          // was skipped or a workgroup waits on one never posted — stop and
          // relaunch (the counter restarts at the oldest unserved request)
          if (now - t0 > std::chrono::seconds(1) && launched && run_gen.load() == gen) {
            forced++;
            fprintf(stderr, "mqmatch: per-publish server: request %llu unserved for %.1f s, relaunching\n",
                    (unsigned long long)k, std::chrono::duration<double>(now - t0).count());
            halt();
          }
          if ((rc = ensure(cur)) != MQM_OK) return give_up(rc);
        }
      }
      waiting[i].store(0, std::memory_order_release);
      pl.sleepers.fetch_sub(1, std::memory_order_acq_rel);
      host_slept++;
    }
    const auto t_seen = clk::now();
    inflight.fetch_sub(1, std::memory_order_acq_rel);
    uint32_t status = sl.status;
    if (sl.t_done > sl.t_claim && sl.t_phase[0] >= sl.t_claim && sl.t_phase[1] >= sl.t_phase[0] &&
        sl.t_done >= sl.t_phase[1]) {
      device_ticks += sl.t_done - sl.t_claim;
      phase_ticks[0] += sl.t_phase[0] - sl.t_claim;
      phase_ticks[1] += sl.t_phase[1] - sl.t_phase[0];
      phase_ticks[2] += sl.t_done - sl.t_phase[1];
      timed++;
    }
    if (status == kServeOk) {
      // the sids are positions in the snapshot the launch served
      std::shared_ptr<const HostSnapshot> hs = host_of(sl.ver, cur);
      if (!hs) {
        stale++;
        status = kServeFallback;
      } else {
        try {
          rc = Collector::single(std::move(hs), sl.dout, sl.dcount, sl.hout, sl.hcount, want_ids ? sl.iout : nullptr,
                                 want_ids ? sl.icount : 0, want_ids, out);
        } catch (const std::bad_alloc &) {
          rc = MQM_ENOMEM;
        }
        served++;
      }
    }
    post_gen[i].store(0, std::memory_order_release);
    slots->release(k);
    const auto t_end = clk::now();
    auto ns = [](clk::duration d) { return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(d).count(); };
    host_ns[0] += ns(t0 - t_in);
    host_ns[1] += ns(t_seen - t0);
    host_ns[2] += ns(t_end - t_seen);
    host_calls++;
    note_max(host_max_ns[0], ns(t_front - t_in));
    note_max(host_max_ns[1], ns(t_ens - t_front));
    note_max(host_max_ns[2], ns(t0 - t_ens));
    note_max(host_max_ns[3], ns(t_seen - t0));
    note_max(host_max_ns[4], ns(t_end - t_seen));
    if (status == kServeOk) {
      if (t_end - t_in > std::chrono::milliseconds(10)) host_slow++;
      return rc;
    }
    fallbacks++;
    rc = direct(topic, len, out);
    note_max(host_max_ns[5], ns(clk::now() - t_end));
    if (clk::now() - t_in > std::chrono::milliseconds(10)) host_slow++;
    return rc;
  }
  int direct(const char *topic, size_t len, mqm_result **out) {
    uint64_t offs[2] = {0, len};
    return mqm_match_batch(h, topic ? topic : "", offs, 1, out);
  }
};

// Live servers, for the reaper to stop while it frees.
struct ServerRegistry {
  std::mutex mu;
  std::vector<Server *> list;
};
ServerRegistry &server_registry() {
  static auto *r = new ServerRegistry;  // (never destroyed: the reaper thread outlives static destruction)
  return *r;
}
void server_register(Server *s) {
  ServerRegistry &r = server_registry();
  std::lock_guard<std::mutex> g(r.mu);
  r.list.push_back(s);
}
void server_unregister(Server *s) {
  ServerRegistry &r = server_registry();
  std::lock_guard<std::mutex> g(r.mu);
  r.list.erase(std::remove(r.list.begin(), r.list.end(), s), r.list.end());
}

// The device buffers of destroyed snapshots, freed on a thread of their own
// (flatten.h retire_device_buffers).  hipFree waits until every kernel on
// the device has finished (tools/free_probe.hip: it waited out a 1 s spinner),
// and a per-publish server runs for as long as calls arrive: a caller, the
// builder or the committing thread that dropped a snapshot's last reference
// used to block there — until the load stopped, or for good once a ring slot
// had been abandoned (r05i).  The reaper stops every live server (its lock
// held, so no caller relaunches it meanwhile), frees, and lets the next call
// relaunch.
struct BufReaper {
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::pair<int, std::vector<void *>>> q;
  BufReaper() {
    std::thread([this] { run(); }).detach();
  }
  void run() {
    for (;;) {
      std::vector<std::pair<int, std::vector<void *>>> batch;
      {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [this] { return !q.empty(); });
        batch.swap(q);
      }
      const int64_t t0 = steady_ns();
      ServerRegistry &r = server_registry();
      std::lock_guard<std::mutex> rg(r.mu);
      std::vector<std::unique_lock<std::mutex>> held;
      held.reserve(r.list.size());
      for (Server *sv : r.list) {
        held.emplace_back(sv->mu);
        sv->halt();
      }
      for (auto &x : batch) {
        if (x.first >= 0) (void)hipSetDevice(x.first);
        for (void *p : x.second) (void)hipFree(p);
      }
      const int64_t t1 = steady_ns();
      if (serve_trace() && t1 - t0 > 5000000)
        fprintf(stderr, "[serve-trace] %.6f reaper: %zu snapshot(s) freed with %zu server(s) stopped in %.1f ms\n",
                t1 * 1e-9, batch.size(), held.size(), (t1 - t0) / 1e6);
    }
  }
  void push(int device, std::vector<void *> bufs) {
    {
      std::lock_guard<std::mutex> g(mu);
      q.emplace_back(device, std::move(bufs));
    }
    cv.notify_one();
  }
};

}  // namespace

}  // extern "C" (a C++ function for flatten.cpp)
namespace mqm {
void retire_device_buffers(int device, std::vector<void *> bufs) {
  static auto *r = new BufReaper;  // (never destroyed, like its thread)
  r->push(device, std::move(bufs));
}
}  // namespace mqm
extern "C" {

void mqm_index::stop_server() {
  server.store(nullptr, std::memory_order_release);
  server_owner.reset();
}

void mqm_index::stop_collector() {
  collector.store(nullptr, std::memory_order_release);
  collector_owner.reset();
}

mqm_index::~mqm_index() {
  stop_server();     // first: its kernel reads this index's snapshot
  stop_collector();  // its thread matches through this index
  pool.clear();
}

// MQM_CFG_FRESH: a single-topic result brought to the store's current
// subscriptions (fresh.h).  Returns MQM_OK (the result replaced when a client
// in it, or one that now matches, was touched after its snapshot), 1 when the
// result's snapshot is older than the overlay covers (match again), or an error.
static int freshen(mqm_index *h, std::string_view topic, mqm_result **res) {
  mqm_result *r = *res;
  if (!r || r->n != 1 || !r->snap) return MQM_OK;
  h->fresh->await_own_writes();  // (this thread's mutations still queued: applied first)
  const int64_t t_read = steady_ns();
  const uint64_t vs = r->snap->version;
  const HostSnapshot &hs = *r->snap;
  const uint64_t base = hs.sub_info.size(), sbase = hs.shared_info.size();
  const bool packed = r->deliveries == nullptr;
  // (per-thread scratch: their capacity kept from call to call)
  thread_local FreshOverlay::Match m;
  thread_local std::vector<mqm_delivery> dl;
  thread_local std::vector<uint32_t> sh, ids;
  dl.clear();
  sh.clear();
  ids.clear();
  {
    FreshOverlay::Reader rd(*h->fresh);
    const int st = rd.status(vs);
    if (st <= 0) return st < 0 ? 1 : MQM_OK;
    rd.match(topic, vs, &m);
    h->fresh->count_match((uint64_t)(steady_ns() - t_read));
    if (base + m.subs.size() > MQM_DELIVERY_SUB(~0u) + 1ull || sbase + m.shared.size() > MQM_DELIVERY_SUB(~0u) + 1ull)
      return MQM_ELIMIT;
    // the snapshot's rows of clients nobody touched since it, then the touched
    // clients' rows from the overlay
    dl.reserve(r->offsets[1] - r->offsets[0] + m.rows.size());
    for (uint64_t j = r->offsets[0]; j < r->offsets[1]; j++) {
      const uint32_t pk = packed ? r->packed[j] : r->deliveries[j].packed;
      const uint32_t client = packed ? hs.sub_info[MQM_DELIVERY_SUB(pk)].client : r->deliveries[j].client;
      if (!rd.touched(client, vs)) dl.push_back(mqm_delivery{client, pk});
    }
    for (uint64_t j = r->shared_offsets[0]; j < r->shared_offsets[1]; j++)
      if (!rd.touched(hs.shared_info[r->shared[j]].client, vs)) sh.push_back(r->shared[j]);
    if (r->has_idents)
      for (uint64_t j = r->ident_offsets[0]; j < r->ident_offsets[1]; j++)
        if (!rd.touched(hs.sub_info[r->idents[j]].client, vs)) ids.push_back(r->idents[j]);
  }
  h->fresh->count_read((uint64_t)(steady_ns() - t_read));
  for (const auto &row : m.rows)
    dl.push_back(mqm_delivery{row.client, (uint32_t)(base + row.first) | (uint32_t)(row.qos & 3u) << 28 |
                                              (uint32_t)(row.no_local & 1u) << 30});
  for (size_t k = 0; k < m.shared.size(); k++) sh.push_back((uint32_t)(sbase + k));
  if (r->has_idents)
    for (size_t g = 0; g < m.subs.size(); g++)  // (packets.go:257-259: Identifiers > 0)
      if (m.subs[g].info.ident > 0) ids.push_back((uint32_t)(base + g));
  auto r2 = std::make_unique<mqm_result>();
  const ResultLayout lay(2, dl.size(), sh.size(), packed ? 4 : 8, ids.size(), r->has_idents);
  if (!r2->alloc(h->pinned, lay.total, false)) return MQM_ENOMEM;
  char *B = static_cast<char *>(r2->blk);
  auto *off = reinterpret_cast<uint64_t *>(B), *soff = reinterpret_cast<uint64_t *>(B + lay.o_sh);
  off[0] = 0;
  off[1] = dl.size();
  soff[0] = 0;
  soff[1] = sh.size();
  if (packed) {
    auto *p4 = reinterpret_cast<uint32_t *>(B + lay.o_d);
    for (size_t j = 0; j < dl.size(); j++) p4[j] = dl[j].packed;
    r2->packed = p4;
  } else {
    if (!dl.empty()) memcpy(B + lay.o_d, dl.data(), sizeof(mqm_delivery) * dl.size());
    r2->deliveries = reinterpret_cast<const mqm_delivery *>(B + lay.o_d);
  }
  if (!sh.empty()) memcpy(B + lay.o_s, sh.data(), 4 * sh.size());
  if (r->has_idents) {
    auto *ioff = reinterpret_cast<uint64_t *>(B + lay.o_io);
    ioff[0] = 0;
    ioff[1] = ids.size();
    if (!ids.empty()) memcpy(B + lay.o_i, ids.data(), 4 * ids.size());
    r2->has_idents = true;
    r2->ident_offsets = ioff;
    r2->idents = reinterpret_cast<const uint32_t *>(B + lay.o_i);
  }
  r2->n = 1;
  r2->offsets = off;
  r2->shared_offsets = soff;
  r2->shared = reinterpret_cast<const uint32_t *>(B + lay.o_s);
  r2->snap = r->snap;
  r2->version = m.version;
  r2->extra.reserve(m.subs.size());
  for (const auto &g : m.subs) r2->extra.push_back(g.info);
  r2->extra_shared.assign(m.shared.begin(), m.shared.end());
  mqm_result_free(r);
  *res = r2.release();
  return MQM_OK;
}

static int subscribers_once(mqm_index *h, const char *topic, size_t topic_len, mqm_result **out) {
  if (Server *sv = h->server.load(std::memory_order_acquire)) {
    *out = nullptr;
    return guarded([&] { return sv->submit(topic ? topic : "", topic_len, out); });
  }
  if (Collector *c = h->collector.load(std::memory_order_acquire)) {
    *out = nullptr;
    return guarded([&] { return c->submit(topic, topic_len, out); });
  }
  uint64_t offs[2] = {0, topic_len};
  return mqm_match_batch(h, topic ? topic : "", offs, 1, out);
}

int mqm_subscribers(mqm_index *h, const char *topic, size_t topic_len, mqm_result **out) {
  if (!h || !out) return MQM_EINVAL;
  if (!h->fresh || !h->fresh_reads.load(std::memory_order_relaxed)) return subscribers_once(h, topic, topic_len, out);
  // (a result on a snapshot two publishes old: the newest one is at most one
  // publish behind the overlay, so the second attempt corrects)
  for (int attempt = 0; attempt < 8; attempt++) {
    int rc = subscribers_once(h, topic, topic_len, out);
    if (rc != MQM_OK) return rc;
    rc = guarded([&] { return freshen(h, std::string_view(topic ? topic : "", topic_len), out); });
    if (rc != 1) return rc;
    mqm_result_free(*out);
    *out = nullptr;
  }
  return MQM_EHIP;
}

int mqm_fresh_policy(mqm_index *h, int correct_calls) {
  if (!h || !h->fresh) return MQM_EINVAL;
  std::lock_guard<std::mutex> g(h->mu);
  // (off: the overlay is dropped and mutations cost nothing more; on: it
  // starts again from the published snapshot)
  h->fresh_reads.store(correct_calls != 0, std::memory_order_relaxed);
  h->fresh->set_enabled(correct_calls != 0, h->snap ? h->snap->host : nullptr, h->store);
  return MQM_OK;
}

int mqm_fresh_stats(mqm_index *h, uint64_t *out) {
  if (!h || !h->fresh || !out) return MQM_EINVAL;
  const FreshOverlay::Stats s = h->fresh->stats();
  out[0] = s.held;
  out[1] = s.ops;
  out[2] = s.rounds;
  out[3] = s.corrected;
  out[4] = s.read_ns;
  out[5] = s.match_ns;
  out[6] = s.max_age_ns;
  out[7] = s.max_round_ns;
  out[8] = s.max_wait_ns;
  return MQM_OK;
}

int mqm_batching_policy(mqm_index *h, uint32_t max_batch, uint32_t linger_us) {
  if (!h || h->cfg.device == MQM_DEVICE_NONE) return MQM_EINVAL;
  {
    // (turns batching on for an index created without MQM_CFG_BATCHING; calls
    // already inside mqm_subscribers finish on the direct path)
    std::lock_guard<std::mutex> g(h->mu);
    if (!h->collector_owner) {
      int rc = guarded([&] {
        h->collector_owner = std::make_unique<Collector>(h);
        return MQM_OK;
      });
      if (rc != MQM_OK) return rc;
      // published fully constructed: a concurrent mqm_subscribers either sees
      // nullptr (direct path) or this collector (release / acquire)
      h->collector.store(h->collector_owner.get(), std::memory_order_release);
    }
  }
  Collector *c = h->collector.load(std::memory_order_acquire);
  std::lock_guard<std::mutex> g(c->mu);
  c->max_batch = max_batch ? max_batch : 8192;
  c->linger_us = linger_us;
  return MQM_OK;
}

// (the server is created once and kept: calls in flight hold no reference
// beyond the index's lifetime)
static int serve_enable_impl(mqm_index *h) {
  std::lock_guard<std::mutex> g(h->mu);
  if (h->server_owner) return MQM_OK;
  return guarded([&] {
    auto sv = std::make_unique<Server>(h);
    const int rc = sv->init();
    if (rc != MQM_OK) return rc;
    h->server_owner = std::move(sv);
    h->server.store(h->server_owner.get(), std::memory_order_release);
    return MQM_OK;
  });
}

int mqm_serve_policy(mqm_index *h, uint32_t grid, uint32_t idle_us) {
  if (!h || h->cfg.device == MQM_DEVICE_NONE) return MQM_EINVAL;
  int rc = serve_enable_impl(h);
  if (rc != MQM_OK) return rc;
  Server *sv = h->server.load(std::memory_order_acquire);
  std::lock_guard<std::mutex> g(sv->mu);
  // (capped at half the CUs: a persistent grid that never idles out would
  // otherwise starve the batch-path kernels of fallback calls)
  sv->grid = std::min<uint32_t>(grid ? grid : 32, sv->max_grid);
  sv->idle_us = idle_us ? idle_us : 20000;
  sv->halt();  // the next call launches with these
  return MQM_OK;
}

int mqm_serve_stats(mqm_index *h, uint64_t *served, uint64_t *fallbacks, uint64_t *launches) {
  Server *sv = h ? h->server.load(std::memory_order_acquire) : nullptr;
  if (!sv || !served || !fallbacks || !launches) return MQM_EINVAL;
  *served = sv->served.load();
  *fallbacks = sv->fallbacks.load();
  *launches = sv->launches.load();
  return MQM_OK;
}

int mqm_serve_counters_get(mqm_index *h, mqm_serve_counters *out) {
  Server *sv = h ? h->server.load(std::memory_order_acquire) : nullptr;
  if (!sv || !out) return MQM_EINVAL;
  out->served = sv->served.load();
  out->fallbacks = sv->fallbacks.load();
  out->launches = sv->launches.load();
  out->stale = sv->stale.load();
  out->forced = sv->forced.load();
  out->slot_timeouts = sv->slots ? sv->slots->slot_timeouts.load() : 0;
  out->result_timeouts = sv->result_timeouts.load();
  out->skipped_slots = sv->slots ? sv->slots->skipped.load() : 0;
  return MQM_OK;
}

int mqm_debug_stamp_counts(uint64_t *checks, uint64_t *stale_cached, uint64_t *stale_memory) {
  if (!checks || !stale_cached || !stale_memory) return MQM_EINVAL;
  uint64_t v[3] = {};
  if (stamp_counts(v) != 0) return MQM_EHIP;
  *checks = v[0];
  *stale_cached = v[1];
  *stale_memory = v[2];
  return MQM_OK;
}

int mqm_serve_device_us(mqm_index *h, double *us) {
  Server *sv = h ? h->server.load(std::memory_order_acquire) : nullptr;
  if (!sv || !us) return MQM_EINVAL;
  const uint64_t n = sv->timed.load();
  // s_memrealtime: 100 MHz; us[0] claim -> published, us[1..3] its phases
  us[0] = n ? (double)sv->device_ticks.load() / 100.0 / (double)n : 0.0;
  for (int i = 0; i < 3; i++) us[1 + i] = n ? (double)sv->phase_ticks[i].load() / 100.0 / (double)n : 0.0;
  return MQM_OK;
}

int mqm_serve_host_max_us(mqm_index *h, double *us) {
  Server *sv = h ? h->server.load(std::memory_order_acquire) : nullptr;
  if (!sv || !us) return MQM_EINVAL;
  for (int i = 0; i < 6; i++) us[i] = (double)sv->host_max_ns[i].exchange(0) / 1e3;
  us[6] = (double)sv->host_slow.exchange(0);
  us[7] = 0.0;
  return MQM_OK;
}

int mqm_serve_host_us(mqm_index *h, double *us) {
  Server *sv = h ? h->server.load(std::memory_order_acquire) : nullptr;
  if (!sv || !us) return MQM_EINVAL;
  const uint64_t n = sv->host_calls.exchange(0);
  for (int i = 0; i < 3; i++) {
    const uint64_t t = sv->host_ns[i].exchange(0);
    us[i] = n ? (double)t / 1e3 / (double)n : 0.0;
  }
  const uint64_t sl = sv->host_slept.exchange(0);
  us[3] = n ? (double)sl / (double)n : 0.0;
  return MQM_OK;
}

int mqm_direct_host_us(mqm_index *h, double *us) {
  if (!h || !us) return MQM_EINVAL;
  const uint64_t n = h->direct_calls.exchange(0);
  for (int i = 0; i < 4; i++) {
    const uint64_t t = h->direct_ns[i].exchange(0), m = h->direct_max_ns[i].exchange(0);
    us[i] = n ? (double)t / 1e3 / (double)n : 0.0;
    us[4 + i] = (double)m / 1e3;
  }
  us[8] = (double)n;
  return MQM_OK;
}

int mqm_batch_host_us(mqm_index *h, double *us) {
  if (!h || !us) return MQM_EINVAL;
  const uint64_t n = h->batch_calls.exchange(0);
  for (int i = 0; i < 5; i++) {
    const uint64_t v = h->batch_ns[i].exchange(0);
    us[i] = n ? (double)v / 1e3 / (double)n : 0.0;
  }
  us[5] = (double)n;
  return MQM_OK;
}

int mqm_batching_stats(mqm_index *h, uint64_t *batches, uint64_t *topics) {
  Collector *c = h ? h->collector.load(std::memory_order_acquire) : nullptr;
  if (!c || !batches || !topics) return MQM_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  *batches = c->batches;
  *topics = c->topics;
  return MQM_OK;
}

uint32_t mqm_result_num_topics(const mqm_result *r) { return r ? r->n : 0; }
uint64_t mqm_result_snapshot_version(const mqm_result *r) {
  return !r ? 0 : r->version ? r->version : r->snap ? r->snap->version : 0;
}
const uint64_t *mqm_result_offsets(const mqm_result *r) { return r ? r->offsets : nullptr; }
const mqm_delivery *mqm_result_deliveries(const mqm_result *r) { return r ? r->deliveries : nullptr; }
const uint32_t *mqm_result_packed(const mqm_result *r) { return r ? r->packed : nullptr; }

int mqm_result_runs(const mqm_result *r, const uint64_t **run_offsets, const mqm_run **runs, const uint32_t **words,
                    uint64_t *n_words) {
  if (!r || !r->run_offsets || !r->snap || !run_offsets || !runs || !words) return MQM_EINVAL;
  *run_offsets = r->run_offsets;
  *runs = r->runs;
  *words = r->snap->words.data();
  if (n_words) *n_words = r->snap->words.size();
  return MQM_OK;
}

int mqm_result_expand(const mqm_result *r, uint32_t t0, uint32_t t1, uint64_t *offsets, uint32_t *dst) {
  if (!r || !r->packed || t0 > t1 || t1 > r->n || !offsets) return MQM_EINVAL;
  const uint32_t *W = r->run_offsets && r->snap ? r->snap->words.data() : nullptr;
  const uint64_t nw = W ? r->snap->words.size() : 0;
  uint64_t at = 0;
  for (uint32_t t = t0; t < t1; t++) {
    offsets[t - t0] = at;
    if (W) {
      for (uint64_t k = r->run_offsets[t]; k < r->run_offsets[t + 1]; k++) {
        const mqm_run run = r->runs[k];
        if ((uint64_t)run.off + run.count > nw) return MQM_EINVAL;
        if (dst) memcpy(dst + at, W + run.off, 4ull * run.count);
        at += run.count;
      }
    }
    const uint64_t w0 = r->offsets[t], w1 = r->offsets[t + 1];
    if (dst && w1 > w0) memcpy(dst + at, r->packed + w0, 4 * (w1 - w0));
    at += w1 - w0;
  }
  offsets[t1 - t0] = at;
  return MQM_OK;
}
const uint64_t *mqm_result_shared_offsets(const mqm_result *r) { return r ? r->shared_offsets : nullptr; }
const uint32_t *mqm_result_shared(const mqm_result *r) { return r ? r->shared : nullptr; }

// a result's subscription record: the snapshot's, or past its sids a fresh
// result's own (freshen)
static const SubInfo *result_info(const mqm_result *r, uint32_t sub, bool shared) {
  const auto &tab = shared ? r->snap->shared_info : r->snap->sub_info;
  if (sub < tab.size()) return &tab[sub];
  const auto &ext = shared ? r->extra_shared : r->extra;
  return sub - tab.size() < ext.size() ? &ext[sub - tab.size()] : nullptr;
}

int mqm_result_sub_info(const mqm_result *r, uint32_t sub, mqm_sub_info *out) {
  if (!r || !out || !r->snap) return MQM_EINVAL;
  const SubInfo *x = result_info(r, sub, false);
  return x ? fill_info(*x, out) : MQM_EINVAL;
}

int mqm_result_shared_info(const mqm_result *r, uint32_t shared_sub, mqm_sub_info *out) {
  if (!r || !out || !r->snap) return MQM_EINVAL;
  const SubInfo *x = result_info(r, shared_sub, true);
  return x ? fill_info(*x, out) : MQM_EINVAL;
}

int mqm_result_sub_infos(const mqm_result *r, int shared, const uint32_t *subs, size_t n, mqm_sub_info *out) {
  if (!r || !r->snap || (n && (!subs || !out))) return MQM_EINVAL;
  for (size_t i = 0; i < n; i++) {
    const SubInfo *x = result_info(r, subs[i], shared != 0);
    if (!x) return MQM_EINVAL;
    fill_info(*x, &out[i]);
  }
  return MQM_OK;
}

void mqm_result_free(mqm_result *r) {
  if (!r) return;
  defer_release(std::move(r->snap));  // (a served result may hold the last reference to its host snapshot)
  delete r;
}

static int copy_name(std::string_view s, char *buf, size_t cap, size_t *len) {
  if (len) *len = s.size();
  if (buf && cap) memcpy(buf, s.data(), s.size() < cap ? s.size() : cap);
  return MQM_OK;
}

int mqm_client_name(mqm_index *h, uint32_t client, char *buf, size_t cap, size_t *len) {
  if (!h) return MQM_EINVAL;
  std::lock_guard<std::mutex> g(h->mu);
  if (client >= h->store.clients().size()) return MQM_EINVAL;
  return copy_name(h->store.clients().name(client), buf, cap, len);
}

int mqm_filter_name(mqm_index *h, uint32_t filter, char *buf, size_t cap, size_t *len) {
  if (!h) return MQM_EINVAL;
  std::lock_guard<std::mutex> g(h->mu);
  if (filter >= h->store.filters().size()) return MQM_EINVAL;
  return copy_name(h->store.filters().name(filter), buf, cap, len);
}

int mqm_num_clients(mqm_index *h, uint32_t *out) {
  if (!h || !out) return MQM_EINVAL;
  std::lock_guard<std::mutex> g(h->mu);
  *out = h->store.clients().size();
  return MQM_OK;
}

int mqm_is_valid_filter(const char *filter, size_t len, int for_publish) {
  return is_valid_filter(sv(filter, len), for_publish != 0) ? 1 : 0;
}

int mqm_is_shared_filter(const char *filter, size_t len) { return is_shared_filter(sv(filter, len)) ? 1 : 0; }

int mqm_commit_async(mqm_index *h) {
  if (!h) return MQM_EINVAL;
  return guarded([&] {
    std::lock_guard<std::mutex> g(h->mu);
    if (!h->async()) return MQM_EINVAL;
    if (h->cfg.device != MQM_DEVICE_NONE && hipSetDevice(h->cfg.device) != hipSuccess) return MQM_EHIP;
    if (!h->journal.empty() || !h->builder || h->builder->dirty() || h->builder->shadow_bad()) submit_locked(h);
    return MQM_OK;
  });
}

int mqm_commit_poll(mqm_index *h, int wait, int *published) {
  if (!h) return MQM_EINVAL;
  return guarded([&] {
    std::lock_guard<std::mutex> g(h->mu);
    if (published) *published = 0;
    if (!h->async()) return MQM_EINVAL;
    if (h->cfg.device != MQM_DEVICE_NONE && hipSetDevice(h->cfg.device) != hipSuccess) return MQM_EHIP;
    if (wait) {
      if (h->builder && (h->builder->dirty() || h->builder->shadow_bad())) submit_locked(h);
      if (h->builder) {
        int rc = h->builder->wait_idle();
        if (rc != MQM_OK) return rc;
      }
    }
    return publish_locked(h, published);
  });
}

int mqm_commit_policy(mqm_index *h, uint64_t max_ops, uint32_t max_ms) {
  if (!h) return MQM_EINVAL;
  std::lock_guard<std::mutex> g(h->mu);
  if (!h->async()) return MQM_EINVAL;
  h->policy_ops = max_ops;
  h->policy_ms = max_ms;
  return MQM_OK;
}

int mqm_commit_state_get(mqm_index *h, mqm_commit_state *out) {
  if (!h || !out) return MQM_EINVAL;
  std::lock_guard<std::mutex> g(h->mu);
  memset(out, 0, sizeof(*out));
  out->store_version = h->store.version();
  out->snapshot_version = h->snap ? h->snap_version : 0;
  out->has_snapshot = h->snap ? 1 : 0;
  out->pending_ops = h->journal.size();
  out->building = h->builder && h->builder->busy() ? 1 : 0;
  out->builds = h->builds;
  out->last_build_ops = h->last_build_ops;
  out->last_build_ms = h->last_build_ms;
  return MQM_OK;
}

int mqm_identifiers_early(mqm_index *h, int on) {
  if (!h || h->cfg.device == MQM_DEVICE_NONE) return MQM_EINVAL;
  h->ident_early.store(on != 0, std::memory_order_relaxed);
  return MQM_OK;
}

int mqm_build_threads(uint32_t n) {
  if (n > 256) return MQM_EINVAL;
  set_build_threads(n);
  return MQM_OK;
}

int mqm_build_phases_ms(mqm_index *h, double *ms) {
  if (!h || !ms) return MQM_EINVAL;
  std::lock_guard<std::mutex> g(h->mu);
  for (int i = 0; i < 3; i++) ms[i] = h->last_build_phase_ms[i];
  ms[3] = (double)build_threads();
  ms[4] = h->last_build_kept_shape ? 1.0 : 0.0;
  return MQM_OK;
}

int mqm_snapshot_digest(mqm_index *h, uint64_t *out) {
  if (!h || !out) return MQM_EINVAL;
  return guarded([&] {
    std::lock_guard<std::mutex> g(h->mu);
    if (!h->snap) return MQM_EINVAL;
    *out = snapshot_digest(*h->snap->host);
    return MQM_OK;
  });
}

int mqm_snapshot_stats_get(mqm_index *h, mqm_snapshot_stats *out) {
  if (!h || !out) return MQM_EINVAL;
  std::lock_guard<std::mutex> g(h->mu);
  memset(out, 0, sizeof(*out));
  if (!h->snap) return MQM_OK;
  const HostSnapshot &hs = *h->snap->host;
  out->nodes = hs.nodes.size();
  out->edges = hs.n_edges;
  out->edge_buckets = hs.n_buckets;
  out->subs = hs.sub_info.size();
  out->shared = hs.shared_info.size();
  out->height = hs.height;
  out->device_bytes = h->snap->device_bytes;
  out->solo_subs = hs.n_solo;
  return MQM_OK;
}

}  // extern "C"
