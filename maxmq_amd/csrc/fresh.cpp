// maxmq_amd/csrc/fresh.cpp — the fresh overlay (fresh.h).
#include "fresh.h"

#include <algorithm>
#include <mutex>

namespace mqm {

namespace {
uint64_t fnv(std::string_view s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
  return h;
}
// gatherSubscriptions' "$" rule (topics.go:527) tests the filter's first byte
uint8_t dollar_skip(std::string_view f) { return !f.empty() && (f[0] == '+' || f[0] == '#'); }
}  // namespace

uint32_t FreshOverlay::token(std::string_view s, bool create) {
  const uint64_t h = fnv(s);
  auto it = tok_head_.find(h);
  if (it != tok_head_.end())
    for (uint32_t id = it->second; id != kNone; id = tok_next_[id])
      if (tok_str_[id] == s) return id;
  if (!create) return kNone;
  const uint32_t id = (uint32_t)tok_str_.size();
  tok_str_.emplace_back(s);
  tok_next_.push_back(it != tok_head_.end() ? it->second : kNone);
  tok_head_[h] = id;
  if (s == "+") plus_tok_ = (int32_t)id;
  if (s == "#") hash_tok_ = (int32_t)id;
  return id;
}

uint32_t FreshOverlay::child(uint32_t parent, uint32_t tok) const {
  auto it = kids_.find((uint64_t)parent << 32 | tok);
  return it == kids_.end() ? kNone : it->second;
}

// the node a filter's subscription is stored at: levels from d, as the store's
// set_path / seek_path walk them (topics.go:380-414)
uint32_t FreshOverlay::path(std::string_view filter, int d, bool create) {
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
      kids_[(uint64_t)n << 32 | tok] = c;
    }
    n = c;
  }
  return n;
}

void FreshOverlay::put(uint32_t node, const Ent &e) {
  for (Ent &x : nodes_[node].ents)
    if (x.client == e.client && x.shared == e.shared && x.group == e.group) {
      x = e;  // (a re-subscription replaces the record: topics.go:390-396)
      return;
    }
  nodes_[node].ents.push_back(e);
  auto &v = held_[e.client];
  if (v.empty() || v.back() != node) v.push_back(node);
}

void FreshOverlay::drop(uint32_t node, uint32_t client, uint8_t shared, uint32_t group) {
  auto &es = nodes_[node].ents;
  for (size_t i = 0; i < es.size(); i++)
    if (es[i].client == client && es[i].shared == shared && es[i].group == group) {
      es.erase(es.begin() + (std::ptrdiff_t)i);
      return;
    }
}

// a client's first mutation since the overlay last held it: its subscriptions
// as the published snapshot has them (no mutation of it since: it would be held)
void FreshOverlay::touch(const Store &st, uint32_t c) {
  if (c >= last_mut_.size()) last_mut_.resize((size_t)c + 1 + last_mut_.size() / 2, 0);
  if (last_mut_[c] != 0) return;
  n_clients_++;
  held_[c];  // (held from now on, even with no subscription)
  const HostSnapshot &hs = *base_;
  if ((size_t)c + 1 < hs.client_off.size())
    for (uint32_t k = hs.client_off[c]; k < hs.client_off[c + 1]; k++) {
      const SubInfo &si = hs.sub_info[hs.client_subs[k]];
      const std::string_view f = st.filters().name(si.filter);
      put(path(f, 0, true), Ent{c, kNone, 0, dollar_skip(f), si});
    }
  if ((size_t)c + 1 < hs.client_shoff.size())
    for (uint32_t k = hs.client_shoff[c]; k < hs.client_shoff[c + 1]; k++) {
      const SubInfo &si = hs.shared_info[hs.client_shared[k]];
      const std::string_view f = st.filters().name(si.filter);
      std::string_view g;
      isolate_particle(f, 1, &g);
      put(path(f, 2, true), Ent{c, token(g, true), 1, 0, si});
    }
}

void FreshOverlay::on_subscribe(const Store &st, std::string_view filter, const SubRec &rec) {
  std::unique_lock<std::shared_mutex> w(rw_);
  version_ = st.version();
  if (!active_) return;
  const Store::Footprint &fp = st.last_footprint();
  touch(st, rec.client);
  const SubInfo si{rec.filter, rec.client, rec.ident, rec.qos, rec.no_local, rec.rap, rec.rh};
  if (fp.shared) {  // stored at levels >= 2 under group = level 1 (topics.go:306-318)
    std::string_view g;
    isolate_particle(filter, 1, &g);
    put(path(filter, 2, true), Ent{rec.client, token(g, true), 1, 0, si});
  } else {
    put(path(filter, 0, true), Ent{rec.client, kNone, 0, dollar_skip(filter), si});
  }
  last_mut_[rec.client] = version_;
}

void FreshOverlay::on_unsubscribe(const Store &st, std::string_view filter) {
  std::unique_lock<std::shared_mutex> w(rw_);
  version_ = st.version();
  if (!active_) return;
  const Store::Footprint &fp = st.last_footprint();
  if (fp.client == kNone) return;  // a client never seen: nothing of it changes
  touch(st, fp.client);
  // the node the store looked at: levels from 2 only for a case-sensitive
  // "$SHARE" prefix (topics.go:330); the shared record dropped when level 0
  // EqualFolds "$SHARE" (:337-341)
  const int d = filter.substr(0, 6) == "$SHARE" ? 2 : 0;
  const uint32_t n = path(filter, d, false);
  if (n != kNone) {
    if (fp.shared) {
      std::string_view g;
      isolate_particle(filter, 1, &g);
      const uint32_t gt = token(g, false);
      if (gt != kNone) drop(n, fp.client, 1, gt);
    } else {
      drop(n, fp.client, 0, kNone);
    }
  }
  last_mut_[fp.client] = version_;
}

void FreshOverlay::on_version(const Store &st) {
  std::unique_lock<std::shared_mutex> w(rw_);
  version_ = st.version();
}

void FreshOverlay::on_install(std::shared_ptr<const HostSnapshot> hs, const Store &st) {
  std::unique_lock<std::shared_mutex> w(rw_);
  version_ = st.version();
  if (!hs || (hs->client_off.empty() && !hs->sub_info.empty()) ||
      (hs->client_shoff.empty() && !hs->shared_info.empty())) {  // (no client index: nothing to start from)
    active_ = false;
    return;
  }
  // results on the snapshot published before this one are still corrected;
  // the clients only older results would need are dropped
  floor_ = active_ && base_ ? base_->version : hs->version;
  for (auto it = held_.begin(); it != held_.end();) {
    const uint32_t c = it->first;
    if (last_mut_[c] > floor_) {
      ++it;
      continue;
    }
    for (uint32_t node : it->second) {
      auto &es = nodes_[node].ents;
      es.erase(std::remove_if(es.begin(), es.end(), [c](const Ent &e) { return e.client == c; }), es.end());
    }
    last_mut_[c] = 0;
    n_clients_--;
    it = held_.erase(it);
  }
  // the trie keeps every path it ever held: start over once it is mostly empty
  size_t live = 0;
  for (const auto &kv : held_) live += kv.second.size();
  if (nodes_.size() > 4096 && nodes_.size() > 16 * (live + 64)) {
    std::vector<Ent> keep;
    for (const auto &kv : held_)
      for (uint32_t node : kv.second)
        for (const Ent &e : nodes_[node].ents)
          if (e.client == kv.first) keep.push_back(e);
    nodes_.assign(1, Node());
    kids_.clear();
    for (auto &kv : held_) kv.second.clear();
    for (const Ent &e : keep) {
      const std::string_view f = st.filters().name(e.info.filter);
      put(e.shared ? path(f, 2, true) : path(f, 0, true), e);
    }
  }
  base_ = std::move(hs);
  active_ = true;
}

int FreshOverlay::Reader::status(uint64_t vs) const {
  if (!o_.active_) return 0;
  if (vs < o_.floor_) return -1;
  return o_.version_ > vs ? 1 : 0;
}

void FreshOverlay::gather(uint32_t node, std::string_view topic, uint64_t vs, bool with_shared, Match *m,
                          std::unordered_map<uint32_t, uint32_t> *row_of) const {
  for (const Ent &e : nodes_[node].ents) {
    if (!(e.client < last_mut_.size() && last_mut_[e.client] > vs)) continue;  // its snapshot rows stand
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
// level, gather at every visited node, the parent-"#" probe after a literal
void FreshOverlay::scan(std::string_view topic, int d, uint32_t node, uint64_t vs, Match *m,
                        std::unordered_map<uint32_t, uint32_t> *row_of) const {
  std::string_view key;
  const bool has_next = isolate_particle(topic, d, &key);
  const std::string_view keys[3] = {key, "+", "#"};
  for (int k = 0; k < 3; k++) {
    uint32_t tok = kNone;
    const uint64_t h = fnv(keys[k]);
    auto it = tok_head_.find(h);
    if (it != tok_head_.end())
      for (uint32_t id = it->second; id != kNone; id = tok_next_[id])
        if (tok_str_[id] == keys[k]) {
          tok = id;
          break;
        }
    if (tok == kNone) continue;
    const uint32_t p = child(node, tok);
    if (p == kNone) continue;
    gather(p, topic, vs, true, m, row_of);
    if (keys[k] != "#" && keys[k] != "+" && hash_tok_ >= 0) {
      const uint32_t wc = child(p, (uint32_t)hash_tok_);
      if (wc != kNone) gather(wc, topic, vs, false, m, row_of);
    }
    if (has_next) scan(topic, d + 1, p, vs, m, row_of);
  }
}

void FreshOverlay::Reader::match(std::string_view topic, uint64_t vs, Match *out) const {
  out->version = o_.version_;
  out->rows.clear();
  out->subs.clear();
  out->shared.clear();
  if (topic.empty()) return;  // (topics.go:498)
  std::unordered_map<uint32_t, uint32_t> row_of;
  o_.scan(topic, 0, 0, vs, out, &row_of);
}

}  // namespace mqm
