// maxmq_amd/csrc/fresh.cpp — the fresh overlay (fresh.h).
#include "fresh.h"

#include <algorithm>
#include <chrono>

namespace mqm {

namespace {
uint64_t fnv(std::string_view s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
  return h;
}
// gatherSubscriptions' "$" rule (topics.go:527) tests the filter's first byte
uint8_t dollar_skip(std::string_view f) { return !f.empty() && (f[0] == '+' || f[0] == '#'); }
int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
// the calling thread's newest queued operation per overlay (a few overlays:
// the thread's own writes its next call on that index must see)
struct LastWrite {
  const void *owner = nullptr;
  uint64_t seq = 0;
};
thread_local LastWrite tl_writes[4];
void note_write(const void *o, uint64_t v) {
  for (auto &w : tl_writes)
    if (w.owner == o) {
      w.seq = v;
      return;
    }
  for (int i = 3; i > 0; i--) tl_writes[i] = tl_writes[i - 1];
  tl_writes[0] = LastWrite{o, v};
}
uint64_t last_write(const void *o) {
  for (const auto &w : tl_writes)
    if (w.owner == o) return w.seq;
  return 0;
}
}  // namespace

// ---- lifecycle, the applier ------------------------------------------------

int FreshOverlay::slot() {
  static std::atomic<int> next{0};
  thread_local const int k = next.fetch_add(1, std::memory_order_relaxed) % kSlots;
  return k;
}

FreshOverlay::FreshOverlay() { th_ = std::thread([this] { run(); }); }

FreshOverlay::~FreshOverlay() {
  {
    std::lock_guard<std::mutex> g(qmu_);
    stop_ = true;
  }
  qcv_.notify_all();
  done_cv_.notify_all();
  th_.join();
}

void FreshOverlay::run() {
  std::unique_lock<std::mutex> lk(qmu_);
  for (;;) {
    qcv_.wait(lk, [&] { return stop_ || !q_.empty(); });
    if (stop_) return;
    // let a batch gather for up to kApplyNs after its first operation
    const int64_t t0 = oldest_ns_.load(std::memory_order_relaxed);
    const auto due = std::chrono::steady_clock::time_point(std::chrono::nanoseconds((t0 ? t0 : now_ns()) + kApplyNs));
    qcv_.wait_until(lk, due, [&] { return stop_ || urgent_ || q_.size() >= kBatch; });
    if (stop_) return;
    lk.unlock();
    {
      std::lock_guard<std::mutex> r(round_mu_);
      std::vector<Op> batch;
      int64_t age = 0;
      {
        std::lock_guard<std::mutex> g(qmu_);
        batch.swap(q_);
        urgent_ = false;
        const int64_t t = oldest_ns_.exchange(0, std::memory_order_acq_rel);
        age = t ? now_ns() - t : 0;
      }
      if ((uint64_t)age > max_age_ns_.load(std::memory_order_relaxed)) max_age_ns_.store(age, std::memory_order_relaxed);
      const int64_t r0 = now_ns();
      round(batch);
      const uint64_t rd = (uint64_t)(now_ns() - r0);
      if (rd > max_round_ns_.load(std::memory_order_relaxed)) max_round_ns_.store(rd, std::memory_order_relaxed);
    }
    lk.lock();
    done_cv_.notify_all();
  }
}

// one round: the batch appended to the log; the least up-to-date copy no call
// is in (not the current one: the copies take turns, so the log stays short)
// brought up to the log's end and made current; the log trimmed to the least
// up-to-date copy
void FreshOverlay::round(std::vector<Op> &batch) {
  if (batch.empty()) return;
  for (Op &op : batch) log_.push_back(std::move(op));
  const uint64_t end = log_base_ + log_.size();
  const int c = cur_.load(std::memory_order_seq_cst);
  int t = -1;
  const int64_t w0 = now_ns();
  // (a caller preempted inside a copy: take another; all busy, yield)
  for (uint32_t spin = 0; t < 0; spin++) {
    for (int k = 0; k < kCopies; k++)
      if (k != c && drained(k) && (t < 0 || pos_[k] < pos_[t])) t = k;
    if (t >= 0) break;
    if (spin < 2048)
      __builtin_ia32_pause();
    else
      std::this_thread::yield();
  }
  const uint64_t wt = (uint64_t)(now_ns() - w0);
  if (wt > max_wait_ns_.load(std::memory_order_relaxed)) max_wait_ns_.store(wt, std::memory_order_relaxed);
  State &x = s_[t];
  for (uint64_t i = pos_[t]; i < end; i++) x.apply(log_[i - log_base_]);
  ops_.fetch_add(end - pos_[t], std::memory_order_relaxed);
  pos_[t] = end;
  cur_.store(t, std::memory_order_seq_cst);
  applied_.store(log_.back().version, std::memory_order_release);
  applied_seq_.store(log_.back().seq, std::memory_order_release);
  rounds_.fetch_add(1, std::memory_order_relaxed);
  uint64_t lo = end;
  for (int k = 0; k < kCopies; k++) lo = std::min(lo, pos_[k]);
  if (lo > log_base_) {
    log_.erase(log_.begin(), log_.begin() + (std::ptrdiff_t)(lo - log_base_));
    log_base_ = lo;
  }
  batch.clear();
}

bool FreshOverlay::await_seq(uint64_t w, int64_t ms) {
  if (w == 0 || applied_seq_.load(std::memory_order_acquire) >= w) return true;
  std::unique_lock<std::mutex> lk(qmu_);
  urgent_ = true;
  qcv_.notify_one();
  return done_cv_.wait_for(lk, std::chrono::milliseconds(ms),
                           [&] { return stop_ || applied_seq_.load(std::memory_order_acquire) >= w; });
}

// (bounded: a result that misses the write still reports its version)
void FreshOverlay::await_own_writes() { await_seq(last_write(this), 200); }

bool FreshOverlay::await_all(int64_t ms) { return await_seq(seq_.load(std::memory_order_acquire), ms); }

// ---- the mutating side (index mutex held) ----------------------------------

void FreshOverlay::enqueue(Op &&op) {
  // (by operation, not version: a publish or a policy change queues one at
  // the version of the mutation before it, and the thread's next call sees it)
  op.seq = seq_.fetch_add(1, std::memory_order_relaxed) + 1;
  note_write(this, op.seq);
  bool wake = false;
  {
    std::lock_guard<std::mutex> g(qmu_);
    if (q_.empty()) {
      oldest_ns_.store(now_ns(), std::memory_order_release);
      wake = true;
    }
    q_.push_back(std::move(op));
    wake |= q_.size() >= kBatch;
  }
  if (wake) qcv_.notify_one();
}

// a client's first touch since the overlay last held it: its subscriptions as
// the published snapshot has them (it had no mutation since: it would be held)
void FreshOverlay::hold(const Store &st, uint32_t c, uint64_t v) {
  auto it = mirror_.find(c);
  if (it != mirror_.end()) {
    it->second = v;
    return;
  }
  Op op;
  op.kind = Op::kLoad;
  op.client = c;
  op.version = v;
  const HostSnapshot &hs = *mbase_;
  if ((size_t)c + 1 < hs.client_off.size())
    for (uint32_t k = hs.client_off[c]; k < hs.client_off[c + 1]; k++) {
      const SubInfo &si = hs.sub_info[hs.client_subs[k]];
      op.loads.push_back(Load{std::string(st.filters().name(si.filter)), 0, si});
    }
  if ((size_t)c + 1 < hs.client_shoff.size())
    for (uint32_t k = hs.client_shoff[c]; k < hs.client_shoff[c + 1]; k++) {
      const SubInfo &si = hs.shared_info[hs.client_shared[k]];
      op.loads.push_back(Load{std::string(st.filters().name(si.filter)), 1, si});
    }
  enqueue(std::move(op));
  mirror_.emplace(c, v);
  held_n_.fetch_add(1, std::memory_order_relaxed);
}

// a few clients at a time: a publish under churn passes the floor over
// hundreds of thousands at once (their entries are ignored by every result the
// overlay still corrects until then: last mutation <= floor)
void FreshOverlay::emit_prunes(size_t n) {
  const uint64_t v = applied_.load(std::memory_order_relaxed);
  for (; n > 0 && !mprune_.empty(); n--) {
    const uint32_t c = mprune_.back();
    mprune_.pop_back();
    auto it = mirror_.find(c);
    if (it == mirror_.end() || it->second > mfloor_) continue;  // (touched again since)
    mirror_.erase(it);
    held_n_.fetch_sub(1, std::memory_order_relaxed);
    Op op;
    op.kind = Op::kPrune;
    op.client = c;
    op.version = std::max(v, queued_version_);
    enqueue(std::move(op));
  }
}

void FreshOverlay::on_subscribe(const Store &st, std::string_view filter, const SubRec &rec) {
  if (!enabled_) return;
  Op op;
  op.version = queued_version_ = st.version();
  if (!mactive_) {
    mdirty_[rec.client] = op.version;
    op.kind = Op::kVersion;
    return enqueue(std::move(op));
  }
  hold(st, rec.client, op.version);
  op.kind = Op::kPut;
  op.client = rec.client;
  op.filter = std::string(filter);
  op.shared = st.last_footprint().shared;
  op.info = SubInfo{rec.filter, rec.client, rec.ident, rec.qos, rec.no_local, rec.rap, rec.rh};
  enqueue(std::move(op));
  emit_prunes(2);
}

void FreshOverlay::on_unsubscribe(const Store &st, std::string_view filter) {
  if (!enabled_) return;
  const Store::Footprint &fp = st.last_footprint();
  Op op;
  op.version = queued_version_ = st.version();
  if (!mactive_ || fp.client == kNone) {  // (a client never seen: nothing of it changes)
    if (!mactive_ && fp.client != kNone) mdirty_[fp.client] = op.version;
    op.kind = Op::kVersion;
    return enqueue(std::move(op));
  }
  hold(st, fp.client, op.version);
  op.kind = Op::kDrop;
  op.client = fp.client;
  op.filter = std::string(filter);
  op.shared = fp.shared;
  enqueue(std::move(op));
  emit_prunes(2);
}

void FreshOverlay::on_version(const Store &st) {
  if (!enabled_) return;
  Op op;
  op.kind = Op::kVersion;
  op.version = queued_version_ = st.version();
  enqueue(std::move(op));
}

void FreshOverlay::on_install(std::shared_ptr<const HostSnapshot> hs, const Store &st) {
  if (!enabled_) return;
  Op op;
  op.version = queued_version_ = st.version();
  if (!hs || (hs->client_off.empty() && !hs->sub_info.empty()) ||
      (hs->client_shoff.empty() && !hs->shared_info.empty())) {  // (no client index: nothing to start from)
    // (the held clients are the ones mutated since the floor: remembered, so
    // that a later snapshot can start the overlay again)
    for (const auto &kv : mirror_) mdirty_[kv.first] = std::max(mdirty_[kv.first], kv.second);
    mactive_ = false;
    mbase_.reset();
    mirror_.clear();
    mprune_.clear();
    held_n_.store(0, std::memory_order_relaxed);
    op.kind = Op::kReset;
    return enqueue(std::move(op));
  }
  // (not holding clients yet, and mutations from before mwait_ were not
  // followed: only a snapshot that has them can start the overlay)
  if (!mactive_ && hs->version < mwait_) {
    op.kind = Op::kVersion;
    return enqueue(std::move(op));
  }
  const bool first = !mactive_;
  // results on the snapshot published before this one are still corrected;
  // the clients only older results would need are dropped
  mfloor_ = mactive_ && mbase_ ? mbase_->version : hs->version;
  mprune_.clear();
  for (const auto &kv : mirror_)
    if (kv.second <= mfloor_) mprune_.push_back(kv.first);
  // (the copies' per-client arrays sized for the snapshot's clients and a
  // quarter more: grown inside a round they cost that round its zeroing and
  // copy — a 306-ms round, r06af)
  const uint64_t nc = std::max<uint64_t>(hs->client_off.size(), hs->client_shoff.size());
  op.client = (uint32_t)std::min<uint64_t>(nc + nc / 4 + 1024, 0xFFFFFFF0u);
  op.nodes_hint = hs->nodes.size();
  mbase_ = std::move(hs);
  mactive_ = true;
  op.kind = Op::kInstall;
  op.floor = mfloor_;
  enqueue(std::move(op));
  if (first) load_dirty(st);
}

// The overlay starts (first install, or on again) from a snapshot that may be
// older than the store: the clients mutated since it was built are held from
// the start, with their subscriptions as the store has them now — one pass
// over the store's nodes under the index mutex, at a start only (a first
// publish under churn, mqm_fresh_policy on).  Every other client's first
// touch loads from the snapshot, which is then its state.
void FreshOverlay::load_dirty(const Store &st) {
  const uint64_t base = mbase_->version, now = st.version();
  std::vector<Op> ops;
  std::vector<uint32_t> at(st.clients().size(), kNone);  // client -> its op
  for (const auto &kv : mdirty_)
    if (kv.second > base && kv.first < at.size() && !mirror_.count(kv.first)) {
      at[kv.first] = (uint32_t)ops.size();
      Op op;
      op.kind = Op::kLoad;
      op.client = kv.first;
      op.version = now;       // (the overlay's version only moves forward)
      op.last = kv.second;    // the client's last mutation
      ops.push_back(std::move(op));
    }
  mdirty_.clear();
  if (ops.empty()) return;
  for (const HNode &n : st.nodes()) {
    if (!n.live) continue;
    for (const SubRec &r : n.subs)
      if (r.client < at.size() && at[r.client] != kNone)
        ops[at[r.client]].loads.push_back(Load{std::string(st.filters().name(r.filter)), 0,
                                               SubInfo{r.filter, r.client, r.ident, r.qos, r.no_local, r.rap, r.rh}});
    for (const SharedRec &x : n.shared) {
      const SubRec &r = x.sub;
      if (r.client < at.size() && at[r.client] != kNone)
        ops[at[r.client]].loads.push_back(Load{std::string(st.filters().name(r.filter)), 1,
                                               SubInfo{r.filter, r.client, r.ident, r.qos, r.no_local, r.rap, r.rh}});
    }
  }
  for (Op &op : ops) {
    mirror_.emplace(op.client, op.last);
    held_n_.fetch_add(1, std::memory_order_relaxed);
    enqueue(std::move(op));
  }
}

void FreshOverlay::set_enabled(bool on, std::shared_ptr<const HostSnapshot> published, const Store &st) {
  if (on == enabled_) return;
  if (!on) {
    Op op;
    op.kind = Op::kReset;
    op.version = queued_version_ = st.version();
    enqueue(std::move(op));
    enabled_ = mactive_ = false;
    mirror_.clear();
    mprune_.clear();
    mdirty_.clear();
    mbase_.reset();
    held_n_.store(0, std::memory_order_relaxed);
    return;
  }
  enabled_ = true;
  // (the mutations while off were not followed: a snapshot that has them all
  // starts the overlay — the published one when nothing changed since)
  mwait_ = st.version();
  on_install(std::move(published), st);
}

// ---- one copy (the applier) ------------------------------------------------

void FreshOverlay::State::Kids::reserve(uint64_t slots) {
  if (slots <= key.size()) return;
  uint64_t sz = key.size();
  while (sz < slots) sz *= 2;
  HVec<uint64_t> ok(sz, ~0ull);
  HVec<uint32_t> ov(sz, 0);
  ok.swap(key);
  ov.swap(val);
  n = 0;
  for (size_t i = 0; i < ok.size(); i++)
    if (ok[i] != ~0ull) insert(ok[i], ov[i]);
}

void FreshOverlay::State::Kids::insert(uint64_t k, uint32_t v) {
  if (2 * (n + 1) > key.size()) {  // load <= 0.5
    HVec<uint64_t> ok(key.size() * 2, ~0ull);
    HVec<uint32_t> ov(key.size() * 2, 0);
    ok.swap(key);
    ov.swap(val);
    n = 0;
    for (size_t i = 0; i < ok.size(); i++)
      if (ok[i] != ~0ull) insert(ok[i], ov[i]);
  }
  const uint64_t m = key.size() - 1;
  uint64_t i = mix(k) & m;
  while (key[i] != ~0ull) i = (i + 1) & m;
  key[i] = k;
  val[i] = v;
  n++;
}

uint32_t FreshOverlay::State::find_token(std::string_view s) const {
  auto it = tok_head_.find(fnv(s));
  if (it != tok_head_.end())
    for (uint32_t id = it->second; id != kNone; id = tok_next_[id])
      if (tok_str_[id] == s) return id;
  return kNone;
}

uint32_t FreshOverlay::State::token(std::string_view s, bool create) {
  const uint32_t found = find_token(s);
  if (found != kNone || !create) return found;
  const uint64_t h = fnv(s);
  auto it = tok_head_.find(h);
  const uint32_t id = (uint32_t)tok_str_.size();
  tok_str_.emplace_back(s);
  tok_next_.push_back(it != tok_head_.end() ? it->second : kNone);
  tok_head_[h] = id;
  if (s == "+") plus_tok_ = (int32_t)id;
  if (s == "#") hash_tok_ = (int32_t)id;
  return id;
}

// the node a filter's subscription is stored at: levels from d, as the store's
// set_path / seek_path walk them (topics.go:380-414)
uint32_t FreshOverlay::State::path(std::string_view filter, int d, bool create) {
  uint32_t n = 0;
  for (bool has_next = true; has_next; d++) {
    std::string_view key;
    has_next = isolate_particle(filter, d, &key);
    const uint32_t tok = token(key, create);
    if (tok == kNone) return kNone;
    uint32_t c = child(n, tok);
    if (c == kNone) {
      if (!create) return kNone;
      c = (uint32_t)nodes_.size();
      nodes_.emplace_back();
      kids_.insert((uint64_t)n << 32 | tok, c);
      if ((int32_t)tok == plus_tok_) nodes_[n].plus = c;
      if ((int32_t)tok == hash_tok_) nodes_[n].hash = c;
    }
    n = c;
  }
  return n;
}

void FreshOverlay::State::put(uint32_t node, const Ent &e) {
  for (Ent &x : nodes_[node].ents)
    if (x.client == e.client && x.shared == e.shared && x.group == e.group) {
      x = e;  // (a re-subscription replaces the record: topics.go:390-396)
      return;
    }
  nodes_[node].ents.push_back(e);
  auto &v = held_[e.client];
  if (v.empty() || v.back() != node) v.push_back(node);
}

// a subscription as Subscribe stores it: shared ones (level 0 EqualFolds
// "$SHARE") at levels >= 2 under group = level 1 (topics.go:306-318)
void FreshOverlay::State::put_sub(uint32_t c, std::string_view filter, uint8_t shared, const SubInfo &si) {
  if (shared) {
    std::string_view g;
    isolate_particle(filter, 1, &g);
    put(path(filter, 2, true), Ent{c, token(g, true), 1, 0, si});
  } else {
    put(path(filter, 0, true), Ent{c, kNone, 0, dollar_skip(filter), si});
  }
}

void FreshOverlay::State::drop(uint32_t node, uint32_t client, uint8_t shared, uint32_t group) {
  auto &es = nodes_[node].ents;
  for (size_t i = 0; i < es.size(); i++)
    if (es[i].client == client && es[i].shared == shared && es[i].group == group) {
      es.erase(es.begin() + (std::ptrdiff_t)i);
      return;
    }
}

void FreshOverlay::State::stamp(uint32_t c, uint64_t v) {
  if (c >= last_mut_.size()) {  // (clients new since the snapshot: doubled, so rarely)
    last_mut_.resize(std::max<size_t>((size_t)c + 1, 2 * last_mut_.size()), 0);
    held_bits_.resize((last_mut_.size() + 63) / 64, 0);
  }
  last_mut_[c] = v;
  if (v)
    held_bits_[c >> 6] |= 1ull << (c & 63);
  else
    held_bits_[c >> 6] &= ~(1ull << (c & 63));
}

void FreshOverlay::State::apply(const Op &op) {
  version_ = op.version;
  switch (op.kind) {
    case Op::kReset:
      *this = State();
      version_ = op.version;
      return;
    case Op::kInstall:
      floor_ = op.floor;
      active_ = true;
      if (op.client != kNone && last_mut_.size() < op.client) {
        last_mut_.resize(op.client, 0);
        held_bits_.resize((last_mut_.size() + 63) / 64, 0);
      }
      {  // room for an eighth of the snapshot's trie (at most 2M paths), once
        const uint64_t want = std::min<uint64_t>(op.nodes_hint / 8, 1u << 21);
        if (nodes_.capacity() < want) {
          kids_.reserve(2 * want);
          nodes_.reserve(want);
          held_.reserve(want / 2);
          tok_head_.reserve(want / 2);
        }
      }
      return;
    case Op::kVersion:
      return;
    case Op::kLoad:
      held_[op.client];  // (held from now on, even with no subscription)
      for (const Load &l : op.loads) put_sub(op.client, l.filter, l.shared, l.info);
      stamp(op.client, op.last ? op.last : op.version);
      return;
    case Op::kPut:
      put_sub(op.client, op.filter, op.shared, op.info);
      stamp(op.client, op.version);
      return;
    case Op::kDrop: {
      // the node the store looked at: levels from 2 only for a case-sensitive
      // "$SHARE" prefix (topics.go:330); the shared record dropped when level
      // 0 EqualFolds "$SHARE" (:337-341)
      const int d = std::string_view(op.filter).substr(0, 6) == "$SHARE" ? 2 : 0;
      const uint32_t n = path(op.filter, d, false);
      if (n != kNone) {
        if (op.shared) {
          std::string_view g;
          isolate_particle(op.filter, 1, &g);
          const uint32_t gt = find_token(g);
          if (gt != kNone) drop(n, op.client, 1, gt);
        } else {
          drop(n, op.client, 0, kNone);
        }
      }
      stamp(op.client, op.version);
      return;
    }
    case Op::kPrune: {
      const uint32_t c = op.client;
      auto it = held_.find(c);
      if (it != held_.end()) {
        for (uint32_t node : it->second) {
          auto &es = nodes_[node].ents;
          es.erase(std::remove_if(es.begin(), es.end(), [c](const Ent &e) { return e.client == c; }), es.end());
        }
        held_.erase(it);
      }
      stamp(c, 0);
      return;
    }
  }
}

void FreshOverlay::State::gather(uint32_t node, std::string_view topic, uint64_t vs, bool with_shared, Match *m,
                                 std::unordered_map<uint32_t, uint32_t> *row_of) const {
  for (const Ent &e : nodes_[node].ents) {
    if (!touched(e.client, vs)) continue;  // its snapshot rows stand
    if (e.shared) {  // gatherSharedSubscriptions (topics.go:541-555): no "$" rule
      if (with_shared) m->shared.push_back(e.info);
      continue;
    }
    if (topic[0] == '$' && e.dollar_skip) continue;  // [MQTT-4.7.1-1/2] (topics.go:527)
    const uint32_t gi = (uint32_t)m->subs.size();
    m->subs.push_back(Gathered{e.client, e.info});
    auto ins = row_of->emplace(e.client, (uint32_t)m->rows.size());
    if (ins.second) {
      m->rows.push_back(Match::Row{e.client, gi, e.info.qos, e.info.no_local});
    } else {  // Subscription.Merge (packets.go:250-270)
      Match::Row &r = m->rows[ins.first->second];
      r.qos = std::max(r.qos, e.info.qos);
      r.no_local |= e.info.no_local;
    }
  }
}

// scanSubscribers (topics.go:493-518), restated: the slice {key, "+", "#"} per
// level, gather at every visited node, the parent-"#" probe after a literal.
// lt[d]: level d's token (kNone: no overlay filter has it)
void FreshOverlay::State::scan(std::string_view topic, const uint32_t *lt, int nl, int d, uint32_t node, uint64_t vs,
                               Match *m, std::unordered_map<uint32_t, uint32_t> *row_of) const {
  const bool has_next = d + 1 < nl;
  const Node &nd = nodes_[node];
  // the key's child by the table (a key that is "+" or "#" itself: the
  // node's wildcard child, as the reference's map lookup would find), then
  // the '+' and '#' children from the node
  const uint32_t key = lt[d];
  const uint32_t kids[3] = {key == kNone ? kNone
                            : (int32_t)key == plus_tok_ ? nd.plus
                            : (int32_t)key == hash_tok_ ? nd.hash
                                                        : child(node, key),
                            nd.plus, nd.hash};
  for (int k = 0; k < 3; k++) {
    const uint32_t p = kids[k];
    if (p == kNone) continue;
    gather(p, topic, vs, true, m, row_of);
    const bool literal = k == 0 && (int32_t)key != plus_tok_ && (int32_t)key != hash_tok_;
    if (literal && nodes_[p].hash != kNone) gather(nodes_[p].hash, topic, vs, false, m, row_of);
    if (has_next) scan(topic, lt, nl, d + 1, p, vs, m, row_of);
  }
}

void FreshOverlay::State::match(std::string_view topic, uint64_t vs, Match *out) const {
  out->version = version_;
  out->rows.clear();
  out->subs.clear();
  out->shared.clear();
  if (topic.empty()) return;  // (topics.go:498)
  // the topic's levels as overlay tokens, once (isolateParticle, topics.go:558-577)
  thread_local std::vector<uint32_t> lt;
  lt.clear();
  for (bool has_next = true; has_next;) {
    std::string_view key;
    has_next = isolate_particle(topic, (int)lt.size(), &key);
    lt.push_back(find_token(key));
  }
  thread_local std::unordered_map<uint32_t, uint32_t> row_of;  // (its buckets kept from call to call)
  row_of.clear();
  scan(topic, lt.data(), (int)lt.size(), 0, 0, vs, out, &row_of);
}

}  // namespace mqm
