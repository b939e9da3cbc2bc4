// maxmq_amd/csrc/store.cpp — host-authoritative store (see store.h).
#include "store.h"

#include <algorithm>
#include <cstddef>
#include <cstring>

#include "keys.h"

namespace mqm {

static inline uint64_t edge_id(uint32_t parent, uint32_t tok) { return ((uint64_t)parent << 32) | tok; }

bool isolate_particle(std::string_view s, int d, std::string_view *out) {
  if (d < 0) {
    *out = std::string_view();
    return false;
  }
  size_t start = 0;
  for (int i = 0; i < d; i++) {
    size_t p = s.find('/', start);
    if (p == std::string_view::npos) {  // d past the last level: the last level, no next
      *out = s.substr(start);
      return false;
    }
    start = p + 1;
  }
  size_t p = s.find('/', start);
  if (p == std::string_view::npos) {
    *out = s.substr(start);
    return false;
  }
  *out = s.substr(start, p - start);
  return true;
}

bool equal_fold_share(std::string_view s) {
  static const char want[6] = {'$', 's', 'h', 'a', 'r', 'e'};
  size_t i = 0;
  for (char w : want) {
    if (i >= s.size()) return false;
    unsigned char x = (unsigned char)s[i];
    if (w == 's' && x == 0xC5 && i + 1 < s.size() && (unsigned char)s[i + 1] == 0xBF) {  // U+017F
      i += 2;
      continue;
    }
    if (x >= 'A' && x <= 'Z') x = (unsigned char)(x - 'A' + 'a');
    if (x != (unsigned char)w) return false;
    i++;
  }
  return i == s.size();
}

bool is_shared_filter(std::string_view f) {
  std::string_view p;
  isolate_particle(f, 0, &p);
  return equal_fold_share(p);
}

bool is_valid_filter(std::string_view f, bool for_publish) {
  if (!for_publish && f.empty()) return false;  // [MQTT-4.7.3-1]
  if (for_publish) {
    if (f.size() >= 4) {  // EqualFold(filter[0:4], "$SYS"): 4 bytes, ASCII fold
      static const char sys[4] = {'$', 's', 'y', 's'};
      bool eq = true;
      for (int i = 0; i < 4; i++) {
        unsigned char x = (unsigned char)f[i];
        if (x >= 'A' && x <= 'Z') x = (unsigned char)(x - 'A' + 'a');
        eq = eq && x == (unsigned char)sys[i];
      }
      if (eq) return false;
    }
    if (f.find('+') != std::string_view::npos || f.find('#') != std::string_view::npos) return false;
  }
  size_t h = f.find('#');
  if (h != std::string_view::npos && h != f.size() - 1) return false;  // [MQTT-4.7.1-2]
  std::string_view prefix;
  bool has_next = isolate_particle(f, 0, &prefix);
  if (!has_next && equal_fold_share(prefix)) return false;  // [MQTT-4.8.2-1]
  if (has_next && equal_fold_share(prefix)) {
    std::string_view group;
    if (!isolate_particle(f, 1, &group)) return false;
    if (group.find('+') != std::string_view::npos || group.find('#') != std::string_view::npos) return false;
  }
  return true;
}

static uint64_t hash_sv(std::string_view s) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (s.size() * 0xff51afd7ed558ccdull);
  size_t i = 0;
  for (; i + 8 <= s.size(); i += 8) {
    uint64_t w;
    memcpy(&w, s.data() + i, 8);
    h = fmix64(h ^ w) * 0x87c37b91114253d5ull;
  }
  uint64_t w = 0;
  memcpy(&w, s.data() + i, s.size() - i);
  return fmix64(h ^ w ^ 0x4cf5ad432745937full);
}

// slot holding s, or the empty slot where it would go
uint64_t Interner::slot_of(std::string_view s, uint64_t h) const {
  const uint64_t mask = table_.size() - 1;
  const uint64_t tag = h >> 32;
  for (uint64_t i = h & mask;; i = (i + 1) & mask) {
    const uint64_t e = table_[i];
    if (e == 0) return i;
    if ((e >> 32) == tag && name((uint32_t)(e & 0xFFFFFFFFu) - 1) == s) return i;
  }
}

void Interner::grow() {
  std::vector<uint64_t> old;
  old.swap(table_);
  table_.assign(old.empty() ? 1024 : old.size() * 2, 0);
  const uint64_t mask = table_.size() - 1;
  for (uint64_t e : old) {
    if (!e) continue;
    uint64_t i = hash_sv(name((uint32_t)(e & 0xFFFFFFFFu) - 1)) & mask;
    while (table_[i]) i = (i + 1) & mask;
    table_[i] = e;
  }
}

uint32_t Interner::intern(std::string_view s) {
  if ((size() + 1) * 2 > table_.size()) grow();
  const uint64_t h = hash_sv(s);
  const uint64_t i = slot_of(s, h);
  if (table_[i]) return (uint32_t)(table_[i] & 0xFFFFFFFFu) - 1;
  const uint32_t id = size();
  arena_.insert(arena_.end(), s.begin(), s.end());
  offs_.push_back(arena_.size());
  table_[i] = ((h >> 32) << 32) | (uint64_t)(id + 1);
  return id;
}

uint32_t Interner::find(std::string_view s) const {
  if (table_.empty()) return kNone;
  const uint64_t i = slot_of(s, hash_sv(s));
  return table_[i] ? (uint32_t)(table_[i] & 0xFFFFFFFFu) - 1 : kNone;
}

Store::Store() {
  plus_tok_ = tokens_.intern("+");
  hash_tok_ = tokens_.intern("#");
  nodes_.emplace_back();  // root (NewTopicsIndex, topics.go:291-299)
  nodes_[0].live = true;
  nodes_[0].key = tokens_.intern("");
}

uint32_t EdgeMap::find(uint64_t key) const {
  if (!n_) return kNone;
  for (uint64_t i = mix(key) & mask_;; i = (i + 1) & mask_) {
    if (keys_[i] == key) return vals_[i];
    if (keys_[i] == ~0ull) return kNone;
  }
}

void EdgeMap::grow() {
  std::vector<uint64_t> ok;
  std::vector<uint32_t> ov;
  ok.swap(keys_);
  ov.swap(vals_);
  const uint64_t cap = ok.empty() ? 1024 : ok.size() * 2;
  keys_.assign(cap, ~0ull);
  vals_.assign(cap, 0);
  mask_ = cap - 1;
  for (uint64_t j = 0; j < ok.size(); j++) {
    if (ok[j] == ~0ull) continue;
    uint64_t i = mix(ok[j]) & mask_;
    while (keys_[i] != ~0ull) i = (i + 1) & mask_;
    keys_[i] = ok[j];
    vals_[i] = ov[j];
  }
}

void EdgeMap::insert(uint64_t key, uint32_t val) {
  if ((n_ + 1) * 2 > keys_.size()) grow();  // load <= 0.5
  uint64_t i = mix(key) & mask_;
  while (keys_[i] != ~0ull) i = (i + 1) & mask_;
  keys_[i] = key;
  vals_[i] = val;
  n_++;
}

void EdgeMap::erase(uint64_t key) {
  if (!n_) return;
  uint64_t i = mix(key) & mask_;
  while (keys_[i] != key) {
    if (keys_[i] == ~0ull) return;
    i = (i + 1) & mask_;
  }
  // backward shift: pull later entries of the cluster into the hole when
  // their home slot does not lie cyclically in (hole, j]
  for (uint64_t j = (i + 1) & mask_;; j = (j + 1) & mask_) {
    if (keys_[j] == ~0ull) break;
    const uint64_t home = mix(keys_[j]) & mask_;
    if (((j - home) & mask_) >= ((j - i) & mask_)) {
      keys_[i] = keys_[j];
      vals_[i] = vals_[j];
      i = j;
    }
  }
  keys_[i] = ~0ull;
  n_--;
}

uint32_t Store::child(uint32_t parent, uint32_t tok) const { return children_.find(edge_id(parent, tok)); }

uint32_t Store::new_node(uint32_t parent, uint32_t tok) {
  uint32_t id;
  if (!free_.empty()) {
    id = free_.back();
    free_.pop_back();
    nodes_[id] = HNode();
  } else {
    id = (uint32_t)nodes_.size();
    nodes_.emplace_back();
  }
  HNode &n = nodes_[id];
  n.live = true;
  n.key = tok;
  n.parent = parent;
  HNode &p = nodes_[parent];
  n.depth = p.depth + 1;
  n.next_sibling = p.first_child;
  if (p.first_child != kNone) nodes_[p.first_child].prev_sibling = id;
  p.first_child = id;
  p.n_children++;
  for (uint32_t a = parent; a != kNone; a = nodes_[a].parent) nodes_[a].subtree++;
  structure_version_++;
  children_.insert(edge_id(parent, tok), id);
  return id;
}

void Store::unlink(uint32_t id) {
  HNode &n = nodes_[id];
  HNode &p = nodes_[n.parent];
  if (n.prev_sibling != kNone)
    nodes_[n.prev_sibling].next_sibling = n.next_sibling;
  else
    p.first_child = n.next_sibling;
  if (n.next_sibling != kNone) nodes_[n.next_sibling].prev_sibling = n.prev_sibling;
  p.n_children--;
  for (uint32_t a = n.parent; a != kNone; a = nodes_[a].parent) nodes_[a].subtree -= n.subtree;  // (a leaf: 1)
  structure_version_++;
  children_.erase(edge_id(n.parent, n.key));
  n = HNode();
  free_.push_back(id);
}

uint32_t Store::set_path(std::string_view s, int d) {
  bool has_next = true;
  uint32_t n = 0;
  while (has_next) {
    std::string_view key;
    has_next = isolate_particle(s, d, &key);
    d++;
    uint32_t tok = tokens_.intern(key);
    uint32_t c = child(n, tok);
    if (c == kNone) c = new_node(n, tok);
    n = c;
  }
  return n;
}

uint32_t Store::seek_path(std::string_view s, int d) const {
  bool has_next = true;
  uint32_t n = 0;
  while (has_next) {
    std::string_view key;
    has_next = isolate_particle(s, d, &key);
    d++;
    uint32_t tok = tokens_.find(key);
    if (tok == kNone) return kNone;
    n = child(n, tok);
    if (n == kNone) return kNone;
  }
  return n;
}

void Store::trim(uint32_t id) {
  while (nodes_[id].parent != kNone && !nodes_[id].retain_path &&
         nodes_[id].n_children + nodes_[id].subs.size() + nodes_[id].shared.size() == 0) {
    uint32_t parent = nodes_[id].parent;
    unlink(id);
    id = parent;
  }
}

bool Store::subscribe(std::string_view client, std::string_view filter, uint8_t qos, uint8_t no_local, uint8_t rap,
                      uint8_t rh, int32_t ident) {
  const uint64_t mark0 = shape_mark();
  last_ = Footprint();
  SubRec rec;
  rec.client = clients_.intern(client);
  rec.filter = filters_.intern(filter);
  rec.ident = ident;
  rec.qos = qos;
  rec.no_local = no_local;
  rec.rap = rap;
  rec.rh = rh;
  version_.v.fetch_add(1, std::memory_order_release);
  std::string_view prefix;
  isolate_particle(filter, 0, &prefix);
  if (equal_fold_share(prefix)) {
    std::string_view group;
    isolate_particle(filter, 1, &group);
    uint32_t gtok = tokens_.intern(group);
    uint32_t n = set_path(filter, 2);
    last_ = Footprint{n, rec.client, rec.filter, gtok, true, shape_mark() != mark0};
    for (auto &s : nodes_[n].shared)
      if (s.group == gtok && s.sub.client == rec.client) {
        s.sub = rec;
        return false;
      }
    nodes_[n].shared.push_back(SharedRec{gtok, rec});
    return true;
  }
  uint32_t n = set_path(filter, 0);
  last_ = Footprint{n, rec.client, rec.filter, 0xFFFFFFFFu, false, shape_mark() != mark0};
  auto &subs = nodes_[n].subs;
  // hub nodes can hold many subscribers: keep them sorted by client
  auto it = std::lower_bound(subs.begin(), subs.end(), rec.client,
                             [](const SubRec &a, uint32_t c) { return a.client < c; });
  if (it != subs.end() && it->client == rec.client) {
    *it = rec;
    return false;
  }
  subs.insert(it, rec);
  return true;
}

bool Store::unsubscribe(std::string_view filter, std::string_view client) {
  int d = filter.substr(0, 6) == "$SHARE" ? 2 : 0;  // strings.HasPrefix: case-sensitive (topics.go:330)
  last_ = Footprint();
  uint32_t n = seek_path(filter, d);
  if (n == kNone) return false;
  const uint64_t mark0 = shape_mark();
  version_.v.fetch_add(1, std::memory_order_release);
  uint32_t cid = clients_.find(client);
  std::string_view prefix;
  isolate_particle(filter, 0, &prefix);
  Footprint fp{n, cid, kNone, kNone, false, false};
  if (equal_fold_share(prefix)) {
    std::string_view group;
    isolate_particle(filter, 1, &group);
    fp.shared = true;
    fp.group = tokens_.find(group);
  }
  drop_sub(fp);
  trim(n);
  fp.structural = shape_mark() != mark0;
  last_ = fp;
  return true;  // true whenever the node exists (topics.go:347-348)
}

// the list change of an unsubscribe at its node (unsubscribe, unsubscribe_at)
void Store::drop_sub(const Footprint &fp) {
  const uint32_t n = fp.node, cid = fp.client;
  if (fp.shared) {
    auto &sh = nodes_[n].shared;
    for (size_t i = 0; i < sh.size(); i++)
      if (sh[i].group == fp.group && sh[i].sub.client == cid) {
        sh.erase(sh.begin() + (std::ptrdiff_t)i);
        break;
      }
  } else if (cid != kNone) {
    auto &subs = nodes_[n].subs;
    auto it = std::lower_bound(subs.begin(), subs.end(), cid,
                               [](const SubRec &a, uint32_t c) { return a.client < c; });
    if (it != subs.end() && it->client == cid) subs.erase(it);
  }
}

bool Store::subscribe_at(const Footprint &fp, uint8_t qos, uint8_t no_local, uint8_t rap, uint8_t rh,
                         int32_t ident) {
  SubRec rec;
  rec.client = fp.client;
  rec.filter = fp.filter;
  rec.ident = ident;
  rec.qos = qos;
  rec.no_local = no_local;
  rec.rap = rap;
  rec.rh = rh;
  version_.v.fetch_add(1, std::memory_order_release);
  last_ = fp;
  const uint32_t n = fp.node;
  if (fp.shared) {
    for (auto &s : nodes_[n].shared)
      if (s.group == fp.group && s.sub.client == rec.client) {
        s.sub = rec;
        return false;
      }
    nodes_[n].shared.push_back(SharedRec{fp.group, rec});
    return true;
  }
  auto &subs = nodes_[n].subs;
  auto it = std::lower_bound(subs.begin(), subs.end(), rec.client,
                             [](const SubRec &a, uint32_t c) { return a.client < c; });
  if (it != subs.end() && it->client == rec.client) {
    *it = rec;
    return false;
  }
  subs.insert(it, rec);
  return true;
}

void Store::unsubscribe_at(const Footprint &fp) {
  version_.v.fetch_add(1, std::memory_order_release);
  last_ = fp;
  drop_sub(fp);
  trim(fp.node);  // (removes nothing: the call was not structural)
}

int64_t Store::retain_message(std::string_view topic, uint64_t msg_ref, uint32_t payload_len, bool retain_flag) {
  version_.v.fetch_add(1, std::memory_order_release);
  uint32_t n = set_path(topic, 0);
  std::string key(topic);
  if (payload_len > 0) {
    nodes_[n].retain_path = !topic.empty();  // retainPath = pk.TopicName
    nodes_[n].ret_ref = msg_ref;
    retained_[key] = RetainedRec{msg_ref, payload_len, retain_flag};
    return 1;
  }
  int64_t out = 0;
  auto it = retained_.find(key);
  if (it != retained_.end() && it->second.payload_len > 0 && it->second.retain_flag) out = -1;
  nodes_[n].retain_path = false;
  if (it != retained_.end()) retained_.erase(it);
  trim(n);
  return out;
}

}  // namespace mqm
