// maxmq_amd/csrc/flatten.cpp — host store -> GPU-resident CSR level-trie.
//
// Node ids are assigned in DFS preorder with children ordered
// (literals..., '+', '#') — the probe order of scanSubscribers
// (vendor/.../mqtt/v2/topics.go:503) — so rank = 2*node+slot orders hits
// exactly as the reference walk emits them (snapshot.h).
#include "flatten.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <unordered_map>

#include "../../include/mqmatch.h"

namespace mqm {

static uint64_t next_pow2(uint64_t x) {
  uint64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

int flatten(const Store &st, HostSnapshot *out) {
  const auto &nodes = st.nodes();
  const uint32_t plus_tok = st.plus_token(), hash_tok = st.hash_token();
  HostSnapshot &hs = *out;
  hs = HostSnapshot();

  // 1. preorder ids
  std::vector<uint32_t> order;
  std::vector<uint32_t> new_id(nodes.size(), kNone);
  order.reserve(nodes.size());
  std::vector<uint32_t> stack{st.root()};
  std::vector<uint32_t> lits;
  while (!stack.empty()) {
    uint32_t n = stack.back();
    stack.pop_back();
    new_id[n] = (uint32_t)order.size();
    order.push_back(n);
    uint32_t pc = st.child(n, plus_tok), hc = st.child(n, hash_tok);
    if (hc != kNone) stack.push_back(hc);  // LIFO: '#' visited last
    if (pc != kNone) stack.push_back(pc);
    lits.clear();
    for (uint32_t c = nodes[n].first_child; c != kNone; c = nodes[c].next_sibling)
      if (c != pc && c != hc) lits.push_back(c);
    for (auto it = lits.rbegin(); it != lits.rend(); ++it) stack.push_back(*it);
  }
  const uint64_t nn = order.size();
  if (nn >= (1ull << 31)) return MQM_ELIMIT;

  // 2. descriptors, subscription ranges, flags
  hs.nodes.resize(nn);
  std::vector<uint8_t> flags(nn, 0);
  uint64_t n_literal_edges = 0;
  for (uint64_t i = 0; i < nn; i++) {
    const HNode &h = nodes[order[i]];
    NodeDesc &d = hs.nodes[i];
    uint32_t pc = st.child(order[i], plus_tok), hc = st.child(order[i], hash_tok);
    d.plus = pc == kNone ? kNone : new_id[pc];
    d.hash = hc == kNone ? kNone : new_id[hc];
    n_literal_edges += h.n_children - (pc != kNone) - (hc != kNone);
    if (hs.subs.size() + h.subs.size() > kMaxSubs) return MQM_ELIMIT;
    d.sub_off = (uint32_t)hs.subs.size();
    d.sub_cnt = (uint32_t)h.subs.size();
    for (const SubRec &s : h.subs) {  // sorted by client (store.cpp)
      hs.subs.push_back(SubEnt{s.client, (uint32_t)s.qos | ((uint32_t)(s.no_local & 1) << 2) |
                                             ((uint32_t)(s.rap & 1) << 3) | ((uint32_t)(s.rh & 3) << 4)});
      hs.sub_info.push_back(SubInfo{s.filter, s.client, s.ident, s.qos, s.no_local, s.rap, s.rh});
    }
    if (h.shared.size() > kShCntMask) return MQM_ELIMIT;
    d.sh_off = (uint32_t)hs.shared_info.size();
    for (const SharedRec &s : h.shared)
      hs.shared_info.push_back(
          SubInfo{s.sub.filter, s.sub.client, s.sub.ident, s.sub.qos, s.sub.no_local, s.sub.rap, s.sub.rh});
    uint8_t f = h.n_children ? (uint8_t)kFlagHasChildren : (uint8_t)0;
    if (i > 0) {
      const uint32_t parent_new = new_id[h.parent];
      if (parent_new == 0) {  // root child: Filter[0] of every sub stored below it
        const std::string_view k = st.tokens().name(h.key);
        if (!k.empty() && (k[0] == '+' || k[0] == '#')) f |= kFlagDollarWild;
      } else {
        f |= flags[parent_new] & kFlagDollarWild;
      }
    }
    flags[i] = f;
    d.sh_cnt_flags = (uint32_t)h.shared.size() | ((uint32_t)f << 24);
    hs.height = std::max(hs.height, h.depth);
  }
  for (uint64_t i = 0; i < nn; i++) {
    NodeDesc &d = hs.nodes[i];
    if (d.hash != kNone) {
      d.hsub_off = hs.nodes[d.hash].sub_off;
      d.hsub_cnt = hs.nodes[d.hash].sub_cnt;
    } else {
      d.hsub_off = 0;
      d.hsub_cnt = 0;
    }
  }

  // 3. literal edges -> open-addressed table of 128-B buckets (load <= 0.5)
  const uint64_t buckets = next_pow2(std::max<uint64_t>(n_literal_edges, 1));
  hs.bucket_mask = buckets - 1;
  hs.n_edges = n_literal_edges;
  EdgeEntry empty;
  memset(&empty, 0, sizeof(empty));
  empty.parent = kNone;
  empty.child = kNone;
  hs.edges.assign(buckets * kEdgesPerBucket, empty);
  const uint64_t n_slots = buckets * kEdgesPerBucket;
  std::unordered_map<uint32_t, uint32_t> pool_off;
  for (uint64_t i = 0; i < nn; i++) {
    const uint32_t pc = hs.nodes[i].plus, hc = hs.nodes[i].hash;
    for (uint32_t c = nodes[order[i]].first_child; c != kNone; c = nodes[c].next_sibling) {
      const uint32_t cn = new_id[c];
      if (cn == pc || cn == hc) continue;
      const std::string_view tok = st.tokens().name(nodes[c].key);
      Key k = make_key([&](uint32_t j) { return (uint8_t)tok[j]; }, (uint32_t)tok.size());
      EdgeEntry e;
      e.k0 = k.k0;
      e.k1 = k.k1;
      e.parent = (uint32_t)i;
      e.child = cn;
      e.tok_off = 0;
      e.tok_len = (uint32_t)tok.size();
      if (key_is_long(k)) {
        auto it = pool_off.find(nodes[c].key);
        if (it == pool_off.end()) {
          if (hs.tok_pool.size() + tok.size() > 0xFFFFFFFFull) return MQM_ELIMIT;
          it = pool_off.emplace(nodes[c].key, (uint32_t)hs.tok_pool.size()).first;
          hs.tok_pool.insert(hs.tok_pool.end(), tok.begin(), tok.end());
        }
        e.tok_off = it->second;
      }
      e.desc = hs.nodes[cn];
      uint64_t slot = (edge_hash((uint32_t)i, k) & hs.bucket_mask) * kEdgesPerBucket;
      while (hs.edges[slot].parent != kNone) slot = (slot + 1) & (n_slots - 1);
      hs.edges[slot] = e;
    }
  }
  if (hs.tok_pool.empty()) hs.tok_pool.push_back(0);
  if (hs.subs.empty()) hs.subs.push_back(SubEnt{0, 0});
  return MQM_OK;
}

GpuSnapshot::~GpuSnapshot() {
  for (void *b : buffers)
    if (b) (void)hipFree(b);
}

int upload(std::shared_ptr<const HostSnapshot> hs, int device, std::unique_ptr<GpuSnapshot> *out) {
  if (hipSetDevice(device) != hipSuccess) return MQM_EHIP;
  auto g = std::make_unique<GpuSnapshot>();
  const void *src[4] = {hs->nodes.data(), hs->edges.data(), hs->subs.data(), hs->tok_pool.data()};
  const size_t sz[4] = {hs->nodes.size() * sizeof(NodeDesc), hs->edges.size() * sizeof(EdgeEntry),
                        hs->subs.size() * sizeof(SubEnt), hs->tok_pool.size()};
  for (int i = 0; i < 4; i++) {
    if (hipMalloc(&g->buffers[i], sz[i] ? sz[i] : 16) != hipSuccess) return MQM_ENOMEM;
    if (sz[i] && hipMemcpy(g->buffers[i], src[i], sz[i], hipMemcpyHostToDevice) != hipSuccess) return MQM_EHIP;
    g->device_bytes += sz[i];
  }
  g->dev.nodes = (const NodeDesc *)g->buffers[0];
  g->dev.edges = (const EdgeEntry *)g->buffers[1];
  g->dev.subs = (const SubEnt *)g->buffers[2];
  g->dev.tok_pool = (const uint8_t *)g->buffers[3];
  g->dev.bucket_mask = hs->bucket_mask;
  g->dev.n_nodes = (uint32_t)hs->nodes.size();
  g->dev.n_subs = (uint32_t)hs->sub_info.size();
  g->dev.n_shared = (uint32_t)hs->shared_info.size();
  g->dev.height = hs->height;
  g->host = std::move(hs);
  *out = std::move(g);
  return MQM_OK;
}

}  // namespace mqm
