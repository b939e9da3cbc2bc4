// maxmq_amd/csrc/capi.cpp — the C ABI (include/mqmatch.h) over the host
// store, the snapshot builder and the HIP match pipeline.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <string_view>
#include <vector>

#include "../../include/mqmatch.h"
#include "builder.h"
#include "bulkload.h"
#include "flatten.h"
#include "match.h"
#include "retained.h"
#include "shard.h"
#include "store.h"

using namespace mqm;

struct mqm_index {
  mqm_config cfg{};
  std::mutex mu;  // serialises mutations, commits and matches on this index
  Store store;
  std::unique_ptr<GpuSnapshot> snap;     // front buffer: what matches read
  uint64_t snap_version = ~0ull;         // store version the front buffer reflects
  uint64_t snap_serial = 0;              // bumped at every publish
  Workspace ws;
  hipStream_t stream = nullptr;
  uint64_t matched_serial = ~0ull;       // snapshot of the last forward match (identifiers pass)
  MatchOutput last_mo;                   // its segments (mqm_dense_device)
  std::vector<hipStream_t> used_streams; // streams that may still read the front buffer
  // MQM_CFG_ASYNC_COMMIT: mutations since the last submit, and the builder
  // that turns them into the back buffer (builder.h)
  DeltaLog journal;
  std::unique_ptr<Builder> builder;
  uint64_t policy_ops = 0;               // auto-submit after this many logged mutations (0 = off)
  uint32_t policy_ms = 0;                // ... or when the oldest one is this old (0 = off)
  std::chrono::steady_clock::time_point journal_t0;
  uint64_t builds = 0, last_build_ops = 0;
  double last_build_ms = 0;
  bool async() const { return (cfg.flags & MQM_CFG_ASYNC_COMMIT) != 0; }
};

struct mqm_messages {
  uint32_t n = 0;
  std::vector<uint64_t> offsets, refs;
};

struct mqm_result {
  uint32_t n = 0;
  std::vector<uint64_t> offsets, shared_offsets;
  std::vector<mqm_delivery> deliveries;
  std::vector<uint32_t> shared;
  bool has_idents = false;               // MQM_CFG_IDENTIFIERS
  std::vector<uint64_t> ident_offsets;   // n + 1
  std::vector<uint32_t> idents;          // sids with Identifier > 0, per topic
  std::shared_ptr<const HostSnapshot> snap;
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

void note_stream(mqm_index *h, hipStream_t s) {
  if (std::find(h->used_streams.begin(), h->used_streams.end(), s) == h->used_streams.end())
    h->used_streams.push_back(s);
}

// make g the front buffer; the old one is freed once the streams that may
// still read it have drained (the builder's upload stream is not waited on)
int install(mqm_index *h, std::unique_ptr<GpuSnapshot> g, uint64_t version) {
  if (h->snap && h->cfg.device != MQM_DEVICE_NONE) {
    for (hipStream_t s : h->used_streams)
      if (hipStreamSynchronize(s) != hipSuccess) return MQM_EHIP;
  }
  h->used_streams.clear();
  h->snap = std::move(g);
  h->snap_version = version;
  h->snap_serial++;
  return MQM_OK;
}

// hand the journal to the builder (MQM_CFG_ASYNC_COMMIT)
void submit_locked(mqm_index *h) {
  if (!h->builder) h->builder = std::make_unique<Builder>(h->cfg.device);
  h->builder->submit(std::move(h->journal), h->store.version());
  h->journal.clear();
  h->journal_t0 = std::chrono::steady_clock::now();
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
  if (published) *published = 1;
  return install(h, std::move(b.snap), b.version);
}

// after a logged mutation: the periodic-rebuild policy (mqm_commit_policy)
void maybe_submit(mqm_index *h) {
  if (!h->async() || h->journal.empty()) return;
  if (h->policy_ops && h->journal.size() >= h->policy_ops) return submit_locked(h);
  if (h->policy_ms && std::chrono::steady_clock::now() - h->journal_t0 >= std::chrono::milliseconds(h->policy_ms))
    submit_locked(h);
}

int commit_locked(mqm_index *h) {
  if (h->snap && h->snap_version == h->store.version()) return MQM_OK;
  if (h->async()) {  // through the builder, so its shadow store stays in step
    if (!h->journal.empty() || !h->builder) submit_locked(h);
    int rc = h->builder->wait_idle();
    if (rc != MQM_OK) return rc;
    return publish_locked(h, nullptr);
  }
  auto hs = std::make_shared<HostSnapshot>();
  int rc = flatten(h->store, hs.get());
  if (rc != MQM_OK) return rc;
  std::unique_ptr<GpuSnapshot> g;
  rc = upload(std::move(hs), h->cfg.device, h->stream, &g);
  if (rc != MQM_OK) return rc;
  return install(h, std::move(g), h->store.version());
}

int ensure_snapshot(mqm_index *h) {
  if (!h->snap || (h->cfg.flags & MQM_CFG_AUTOCOMMIT)) return commit_locked(h);
  if (h->async()) {
    maybe_submit(h);
    return publish_locked(h, nullptr);
  }
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

}  // namespace

extern "C" {

const char *mqm_version(void) { return "mqmatch 0.1 (gfx950)"; }

int mqm_profile_enable(mqm_index *h, int on) {
  if (!h) return MQM_EINVAL;
  std::lock_guard<std::mutex> g(h->mu);
  h->ws.profile = on != 0;
  h->ws.reset_profile();
  return MQM_OK;
}

int mqm_profile_read(mqm_index *h, mqm_profile *out) {
  if (!h || !out) return MQM_EINVAL;
  std::lock_guard<std::mutex> g(h->mu);
  out->calls = h->ws.prof_calls;
  out->fallback_topics = h->ws.prof_fallback_topics;
  out->walk_ms = h->ws.prof_walk_ms;
  out->dedupe_ms = h->ws.prof_dedupe_ms;
  out->total_ms = h->ws.prof_total_ms;
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
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) return MQM_EHIP;
    if (const char *e = getenv("MQM_WALK_LANES")) {
      const int g = atoi(e);
      h->ws.walk_lanes = g == 4 || g == 16 ? g : 8;
    }
    *out = h.release();
    return MQM_OK;
  });
}

int mqm_destroy(mqm_index *h) {
  if (!h) return MQM_EINVAL;
  h->builder.reset();  // finishes a running build and joins the worker
  if (h->cfg.device != MQM_DEVICE_NONE) {
    (void)hipSetDevice(h->cfg.device);
    (void)hipDeviceSynchronize();
    if (h->stream) (void)hipStreamDestroy(h->stream);
  }
  delete h;
  return MQM_OK;
}

int mqm_subscribe(mqm_index *h, const char *client, size_t client_len, const char *filter, size_t filter_len,
                  const mqm_subscription *sub, int *is_new) {
  if (!h || !sub) return MQM_EINVAL;
  return guarded([&] {
    std::lock_guard<std::mutex> g(h->mu);
    bool n = h->store.subscribe(sv(client, client_len), sv(filter, filter_len), sub->qos, sub->no_local,
                                sub->retain_as_published, sub->retain_handling, sub->identifier);
    if (h->async()) {
      h->journal.subscribe(sv(client, client_len), sv(filter, filter_len), sub->qos, sub->no_local,
                           sub->retain_as_published, sub->retain_handling, sub->identifier);
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
  return guarded([&] {
    std::lock_guard<std::mutex> g(h->mu);
    for (size_t i = 0; i < n; i++) {
      const mqm_subscription &s = subs[i];
      const auto c = sv(client_bytes + client_offs[i], client_offs[i + 1] - client_offs[i]);
      const auto f = sv(filter_bytes + filter_offs[i], filter_offs[i + 1] - filter_offs[i]);
      bool r = h->store.subscribe(c, f, s.qos, s.no_local, s.retain_as_published, s.retain_handling, s.identifier);
      if (h->async()) h->journal.subscribe(c, f, s.qos, s.no_local, s.retain_as_published, s.retain_handling, s.identifier);
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
    if (r && h->async()) {  // false: no node, nothing changed (topics.go:334-336)
      h->journal.unsubscribe(sv(filter, filter_len), sv(client, client_len));
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
      if (r && h->async()) h->journal.unsubscribe(f, c);
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
    std::lock_guard<std::mutex> g(h->mu);
    if (h->cfg.device == MQM_DEVICE_NONE) return MQM_ENODEV;
    if (hipSetDevice(h->cfg.device) != hipSuccess) return MQM_EHIP;
    int rc = ensure_snapshot(h);
    if (rc != MQM_OK) return rc;
    MatchOutput mo;
    note_stream(h, (hipStream_t)hip_stream);
    rc = match_device(h->snap->dev, h->ws, d_topic_bytes, d_topic_offsets, n_topics, (hipStream_t)hip_stream, &mo);
    if (rc != 0) return rc;
    h->matched_serial = h->snap_serial;
    h->last_mo = mo;
    out->n_topics = mo.n_topics;
    out->n_deliveries = mo.n_deliveries;
    out->n_shared = mo.n_shared;
    out->starts = mo.starts;
    out->counts = mo.counts;
    out->deliveries = reinterpret_cast<const mqm_delivery *>(mo.deliveries);
    out->shared_starts = mo.shared_starts;
    out->shared_counts = mo.shared_counts;
    out->shared = mo.shared;
    out->n_fallback = mo.n_fallback;
    out->n_big = mo.n_big;
    for (int i = 0; i < 5; i++) out->fallback_why[i] = h->ws.why[i];
    return MQM_OK;
  });
}

int mqm_match_batch(mqm_index *h, const char *topic_bytes, const uint64_t *topic_offsets, uint32_t n_topics,
                    mqm_result **out) {
  if (!h || !out || !topic_offsets || (n_topics && !topic_bytes)) return MQM_EINVAL;
  *out = nullptr;
  return guarded([&] {
    std::lock_guard<std::mutex> g(h->mu);
    if (h->cfg.device == MQM_DEVICE_NONE) return MQM_ENODEV;
    if (hipSetDevice(h->cfg.device) != hipSuccess) return MQM_EHIP;
    int rc = ensure_snapshot(h);
    if (rc != MQM_OK) return rc;
    const uint64_t base = topic_offsets[0];
    const uint64_t nbytes = topic_offsets[n_topics] - base;
    Workspace &ws = h->ws;
    if (ws.get(Workspace::kInBytes, nbytes + 16) || ws.get(Workspace::kInOffs, sizeof(uint64_t) * (n_topics + 1)))
      return MQM_ENOMEM;
    auto *d_bytes = (uint8_t *)ws.ptr(Workspace::kInBytes);
    auto *d_offs = (uint64_t *)ws.ptr(Workspace::kInOffs);
    std::vector<uint64_t> offs(topic_offsets, topic_offsets + n_topics + 1);
    for (auto &o : offs) o -= base;
    if (nbytes && hipMemcpyAsync(d_bytes, topic_bytes + base, nbytes, hipMemcpyHostToDevice, h->stream) != hipSuccess)
      return MQM_EHIP;
    if (hipMemcpyAsync(d_offs, offs.data(), sizeof(uint64_t) * (n_topics + 1), hipMemcpyHostToDevice, h->stream) !=
        hipSuccess)
      return MQM_EHIP;
    MatchOutput mo;
    note_stream(h, h->stream);
    rc = match_device(h->snap->dev, ws, d_bytes, d_offs, n_topics, h->stream, &mo);
    if (rc != 0) return rc;
    h->matched_serial = h->snap_serial;
    h->last_mo = mo;
    IdentOutput io;
    const bool want_ids = (h->cfg.flags & MQM_CFG_IDENTIFIERS) != 0;
    if (want_ids && (rc = identifiers_device(h->snap->dev, ws, h->stream, &io)) != 0) return rc;
    DenseOutput dn;
    rc = densify(ws, mo, h->stream, &dn);
    if (rc != 0) return rc;
    auto r = std::make_unique<mqm_result>();
    r->n = n_topics;
    r->offsets.resize(n_topics + 1);
    r->shared_offsets.resize(n_topics + 1);
    r->deliveries.resize(mo.n_deliveries);
    r->shared.resize(mo.n_shared);
    r->snap = h->snap->host;
    if (hipMemcpyAsync(r->offsets.data(), dn.offsets, sizeof(uint64_t) * (n_topics + 1), hipMemcpyDeviceToHost,
                       h->stream) != hipSuccess ||
        hipMemcpyAsync(r->shared_offsets.data(), dn.shared_offsets, sizeof(uint64_t) * (n_topics + 1),
                       hipMemcpyDeviceToHost, h->stream) != hipSuccess)
      return MQM_EHIP;
    if (mo.n_deliveries && hipMemcpyAsync(r->deliveries.data(), dn.deliveries, sizeof(uint64_t) * mo.n_deliveries,
                                          hipMemcpyDeviceToHost, h->stream) != hipSuccess)
      return MQM_EHIP;
    if (mo.n_shared && hipMemcpyAsync(r->shared.data(), dn.shared, sizeof(uint32_t) * mo.n_shared,
                                      hipMemcpyDeviceToHost, h->stream) != hipSuccess)
      return MQM_EHIP;
    if (want_ids) {
      r->has_idents = true;
      r->ident_offsets.resize(n_topics + 1);
      r->idents.resize(io.n_idents);
      if (hipMemcpyAsync(r->ident_offsets.data(), io.offsets, sizeof(uint64_t) * (n_topics + 1),
                         hipMemcpyDeviceToHost, h->stream) != hipSuccess)
        return MQM_EHIP;
      if (io.n_idents && hipMemcpyAsync(r->idents.data(), io.sids, sizeof(uint32_t) * io.n_idents,
                                        hipMemcpyDeviceToHost, h->stream) != hipSuccess)
        return MQM_EHIP;
    }
    if (hipStreamSynchronize(h->stream) != hipSuccess) return MQM_EHIP;
    *out = r.release();
    return MQM_OK;
  });
}

int mqm_identifiers_device(mqm_index *h, void *hip_stream, mqm_device_identifiers *out) {
  if (!h || !out) return MQM_EINVAL;
  return guarded([&] {
    std::lock_guard<std::mutex> g(h->mu);
    if (h->cfg.device == MQM_DEVICE_NONE) return MQM_ENODEV;
    // the records of the last forward match, against the snapshot it read
    if (!h->snap || h->matched_serial != h->snap_serial) return MQM_EINVAL;
    if (hipSetDevice(h->cfg.device) != hipSuccess) return MQM_EHIP;
    note_stream(h, (hipStream_t)hip_stream);
    IdentOutput io;
    const int rc = identifiers_device(h->snap->dev, h->ws, (hipStream_t)hip_stream, &io);
    if (rc != 0) return rc == -2 ? MQM_ENOMEM : rc == -1 ? MQM_EINVAL : MQM_EHIP;
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
    std::lock_guard<std::mutex> g(h->mu);
    if (h->cfg.device == MQM_DEVICE_NONE) return MQM_ENODEV;
    if (!h->snap || h->matched_serial != h->snap_serial) return MQM_EINVAL;
    if (hipSetDevice(h->cfg.device) != hipSuccess) return MQM_EHIP;
    note_stream(h, (hipStream_t)hip_stream);
    DenseOutput dn;
    const int rc = densify(h->ws, h->last_mo, (hipStream_t)hip_stream, &dn);
    if (rc != 0) return rc == -2 ? MQM_ENOMEM : MQM_EHIP;
    out->n_topics = h->last_mo.n_topics;
    out->n_deliveries = h->last_mo.n_deliveries;
    out->n_shared = h->last_mo.n_shared;
    out->offsets = dn.offsets;
    out->deliveries = reinterpret_cast<const mqm_delivery *>(dn.deliveries);
    out->shared_offsets = dn.shared_offsets;
    out->shared = dn.shared;
    return MQM_OK;
  });
}

int mqm_gather_shards(uint32_t n_topics, uint32_t n_shards, const mqm_shard_part *parts, void *hip_stream,
                      uint64_t *d_out_offsets, mqm_delivery *d_out) {
  if (!parts || !d_out_offsets || n_shards == 0 || n_shards > (uint32_t)kMaxShards) return MQM_EINVAL;
  return guarded([&] {
    // device-visible status word (pinned, mapped): a client id outside its map
    static std::mutex mu;
    static unsigned int *bad = nullptr;
    std::lock_guard<std::mutex> g(mu);
    if (!bad && hipHostMalloc((void **)&bad, sizeof(unsigned int), hipHostMallocMapped) != hipSuccess) {
      bad = nullptr;
      return MQM_EHIP;
    }
    *bad = 0;
    ShardPart p[kMaxShards];
    for (uint32_t r = 0; r < n_shards; r++)
      p[r] = ShardPart{parts[r].offsets, reinterpret_cast<const uint64_t *>(parts[r].deliveries),
                       parts[r].client_map, parts[r].n_map};
    unsigned int *dbad = nullptr;
    if (hipHostGetDevicePointer((void **)&dbad, bad, 0) != hipSuccess) return MQM_EHIP;
    const int rc = gather_shards(n_topics, n_shards, p, (hipStream_t)hip_stream, d_out_offsets,
                                 reinterpret_cast<uint64_t *>(d_out), dbad);
    if (rc == -1) return MQM_EINVAL;
    if (rc != 0) return MQM_EHIP;
    if (hipStreamSynchronize((hipStream_t)hip_stream) != hipSuccess) return MQM_EHIP;
    return *(volatile unsigned int *)bad ? MQM_EINVAL : MQM_OK;
  });
}

int mqm_result_identifiers(const mqm_result *r, const uint64_t **offsets, const uint32_t **sids) {
  if (!r || !offsets || !sids || !r->has_idents) return MQM_EINVAL;
  *offsets = r->ident_offsets.data();
  *sids = r->idents.data();
  return MQM_OK;
}

int mqm_messages_device(mqm_index *h, const uint8_t *d_filter_bytes, const uint64_t *d_filter_offsets,
                        uint32_t n_filters, void *hip_stream, mqm_device_messages *out) {
  if (!h || !out || (n_filters && (!d_filter_bytes || !d_filter_offsets))) return MQM_EINVAL;
  return guarded([&] {
    std::lock_guard<std::mutex> g(h->mu);
    if (h->cfg.device == MQM_DEVICE_NONE) return MQM_ENODEV;
    if (hipSetDevice(h->cfg.device) != hipSuccess) return MQM_EHIP;
    int rc = ensure_snapshot(h);
    if (rc != MQM_OK) return rc;
    MessagesOutput mo;
    note_stream(h, (hipStream_t)hip_stream);
    rc = messages_device(h->snap->dev, h->snap->has_retained ? &h->snap->ret : nullptr, h->ws, d_filter_bytes,
                         d_filter_offsets, n_filters, (hipStream_t)hip_stream, &mo);
    if (rc != 0) return rc;
    out->n_filters = mo.n_filters;
    out->n_refs = mo.n_refs;
    out->offsets = mo.offsets;
    out->refs = mo.refs;
    out->n_ranges = mo.n_emissions;
    out->n_items = mo.n_items;
    return MQM_OK;
  });
}

int mqm_messages_batch(mqm_index *h, const char *filter_bytes, const uint64_t *filter_offsets, uint32_t n_filters,
                       mqm_messages **out) {
  if (!h || !out || !filter_offsets || (n_filters && !filter_bytes)) return MQM_EINVAL;
  *out = nullptr;
  return guarded([&] {
    std::lock_guard<std::mutex> g(h->mu);
    if (h->cfg.device == MQM_DEVICE_NONE) return MQM_ENODEV;
    if (hipSetDevice(h->cfg.device) != hipSuccess) return MQM_EHIP;
    int rc = ensure_snapshot(h);
    if (rc != MQM_OK) return rc;
    const uint64_t base = filter_offsets[0];
    const uint64_t nbytes = filter_offsets[n_filters] - base;
    Workspace &ws = h->ws;
    if (ws.get(Workspace::kRInBytes, nbytes + 16) || ws.get(Workspace::kRInOffs, sizeof(uint64_t) * (n_filters + 1)))
      return MQM_ENOMEM;
    auto *d_bytes = (uint8_t *)ws.ptr(Workspace::kRInBytes);
    auto *d_offs = (uint64_t *)ws.ptr(Workspace::kRInOffs);
    std::vector<uint64_t> offs(filter_offsets, filter_offsets + n_filters + 1);
    for (auto &o : offs) o -= base;
    if (nbytes && hipMemcpyAsync(d_bytes, filter_bytes + base, nbytes, hipMemcpyHostToDevice, h->stream) != hipSuccess)
      return MQM_EHIP;
    if (hipMemcpyAsync(d_offs, offs.data(), sizeof(uint64_t) * (n_filters + 1), hipMemcpyHostToDevice, h->stream) !=
        hipSuccess)
      return MQM_EHIP;
    MessagesOutput mo;
    note_stream(h, h->stream);
    rc = messages_device(h->snap->dev, h->snap->has_retained ? &h->snap->ret : nullptr, ws, d_bytes, d_offs,
                         n_filters, h->stream, &mo);
    if (rc != 0) return rc;
    auto m = std::make_unique<mqm_messages>();
    m->n = n_filters;
    m->offsets.resize(n_filters + 1);
    m->refs.resize(mo.n_refs);
    if (hipMemcpyAsync(m->offsets.data(), mo.offsets, sizeof(uint64_t) * (n_filters + 1), hipMemcpyDeviceToHost,
                       h->stream) != hipSuccess)
      return MQM_EHIP;
    if (mo.n_refs && hipMemcpyAsync(m->refs.data(), mo.refs, sizeof(uint64_t) * mo.n_refs, hipMemcpyDeviceToHost,
                                    h->stream) != hipSuccess)
      return MQM_EHIP;
    if (hipStreamSynchronize(h->stream) != hipSuccess) return MQM_EHIP;
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

int mqm_subscribers(mqm_index *h, const char *topic, size_t topic_len, mqm_result **out) {
  uint64_t offs[2] = {0, topic_len};
  return mqm_match_batch(h, topic ? topic : "", offs, 1, out);
}

uint32_t mqm_result_num_topics(const mqm_result *r) { return r ? r->n : 0; }
const uint64_t *mqm_result_offsets(const mqm_result *r) { return r ? r->offsets.data() : nullptr; }
const mqm_delivery *mqm_result_deliveries(const mqm_result *r) { return r ? r->deliveries.data() : nullptr; }
const uint64_t *mqm_result_shared_offsets(const mqm_result *r) { return r ? r->shared_offsets.data() : nullptr; }
const uint32_t *mqm_result_shared(const mqm_result *r) { return r ? r->shared.data() : nullptr; }

int mqm_result_sub_info(const mqm_result *r, uint32_t sub, mqm_sub_info *out) {
  if (!r || !out || !r->snap || sub >= r->snap->sub_info.size()) return MQM_EINVAL;
  return fill_info(r->snap->sub_info[sub], out);
}

int mqm_result_shared_info(const mqm_result *r, uint32_t shared_sub, mqm_sub_info *out) {
  if (!r || !out || !r->snap || shared_sub >= r->snap->shared_info.size()) return MQM_EINVAL;
  return fill_info(r->snap->shared_info[shared_sub], out);
}

int mqm_result_sub_infos(const mqm_result *r, int shared, const uint32_t *subs, size_t n, mqm_sub_info *out) {
  if (!r || !r->snap || (n && (!subs || !out))) return MQM_EINVAL;
  const auto &tab = shared ? r->snap->shared_info : r->snap->sub_info;
  for (size_t i = 0; i < n; i++) {
    if (subs[i] >= tab.size()) return MQM_EINVAL;
    fill_info(tab[subs[i]], &out[i]);
  }
  return MQM_OK;
}

void mqm_result_free(mqm_result *r) { delete r; }

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
    if (!h->journal.empty() || !h->builder) submit_locked(h);
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
    if (wait && h->builder) {
      int rc = h->builder->wait_idle();
      if (rc != MQM_OK) return rc;
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
