// maxmq_amd/csrc/flatten.cpp — host store -> GPU-resident CSR level-trie.
//
// Node ids are assigned in DFS preorder with children ordered
// (literals..., '+', '#') — the probe order of scanSubscribers
// (vendor/.../mqtt/v2/topics.go:503) — so rank = 2*node+slot orders hits
// exactly as the reference walk emits them (snapshot.h).
#include "flatten.h"
#include "builder.h"
#include "match.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>

#include "../../include/mqmatch.h"

namespace mqm {

namespace {
std::atomic<uint32_t> g_build_threads{0};  // mqm_build_threads (0: the default)
}  // namespace

std::atomic<int> g_servers{0};  // live per-publish servers (serve_count)

uint32_t build_threads() {
  const uint32_t set = g_build_threads.load(std::memory_order_relaxed);
  if (set) return set;
  static const int env = [] {
    const char *e = getenv("MQM_BUILD_THREADS");
    return e ? atoi(e) : 0;
  }();
  if (env > 0) return (uint32_t)env;
  const uint32_t hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  // a per-publish server's callers share the CPUs with the rebuild, which runs
  // back to back under churn (its CPU share is its thread count): 16 / 4 / 2
  // flatten threads give 0.79-0.82 / 0.85-1.00 / 0.93-1.10M served calls/s
  // at a visibility lag of 4-5 / 7-8 / 11-13 s (r05af-r05ai, 64 callers,
  // 100k mutations/s, C3)
  return g_servers.load(std::memory_order_relaxed) > 0 ? std::min(hw, 2u) : hw;
}

void serve_count(int delta) { g_servers.fetch_add(delta, std::memory_order_relaxed); }

void set_build_threads(uint32_t n) { g_build_threads.store(n, std::memory_order_relaxed); }

namespace {
// run f(t) for t in [0, n) on up to build_threads() host threads (default 16,
// the box's CPU share)
template <class F>
void parallel_for(uint32_t n, F &&f) {
  const uint32_t nt = std::min(build_threads(), n);
  if (nt <= 1) {
    for (uint32_t t = 0; t < n; t++) f(t);
    return;
  }
  std::vector<std::thread> th;
  for (uint32_t w = 0; w < nt; w++)
    th.emplace_back([&, w] {
      for (uint32_t t = w; t < n; t += nt) f(t);
    });
  for (auto &x : th) x.join();
}

// the flatten's loops walk one array in order and read another at the
// positions it holds (store ids <-> preorder ids): prefetching a few
// iterations ahead keeps several of those misses in flight per thread
constexpr uint64_t kAhead = 8;
inline void prefetch_node(const HNode *h) {
  __builtin_prefetch(h);
  __builtin_prefetch(reinterpret_cast<const char *>(h) + 64);  // (96 B: may span two lines)
}

// MQM_FLATTEN_TRACE=1: per-phase wall time to stderr
struct PhaseTimer {
  bool on = getenv("MQM_FLATTEN_TRACE") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void mark(const char *what) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "[flatten] %-10s %8.1f ms\n", what, std::chrono::duration<double, std::milli>(now - t).count());
    t = now;
  }
};
}  // namespace

// kMetaMulti (snapshot.h).  Levels of a filter are the keys on its node's
// path; two filters of one client can be gathered for the same topic only if
// the levels both have are pairwise equal or wildcards (a topic level cannot
// equal two different literals), so a subscription whose client has no such
// partner — and which the parent-'#' probe cannot emit twice — is solo.
// A multi subscription's partners (its client's level-compatible
// subscriptions) go to `part` (old sids, by `poff`), for the merge by
// resolution (snapshot.h: pinfo); a subscription whose merge needs the hash
// table instead gets kPHeavy (client with more than kMaxPairwise
// subscriptions, more than kMaxPartners partners, or the old '#' marking).
static constexpr uint32_t kMaxPairwise = 64;  // clients with more subscriptions: all multi
static constexpr uint32_t kPHeavy = 0xFFFFu;

struct Partners {
  std::vector<uint16_t> cnt;   // by old sid: 0 solo, 1..kMaxPartners partners, kPHeavy
  std::vector<uint64_t> off;   // by old sid: start in `part`
  std::vector<uint32_t> part;  // partner old sids
};

// (par / kd: every node's parent, and its token and depth, by preorder id —
// the pairwise level checks climb these: a parent sits just before its
// subtree, so a climb mostly stays in lines already read, where the node
// array by store id was a miss per level)
template <class ParVec>
static void mark_multi(const Store &st, HostSnapshot &hs, Partners &pt, const ParVec &par,
                       const std::vector<uint2, NoInitAlloc<uint2>> &kd) {
  PhaseTimer ph;
  const uint32_t plus_tok = st.plus_token(), hash_tok = st.hash_token();
  const uint64_t nsub = hs.sub_info.size();
  std::vector<uint32_t, NoInitAlloc<uint32_t>> sub_node(nsub);  // (every range is written: ranges tile the subs)
  const uint64_t nn = hs.nodes.size();
  parallel_for(256, [&](uint32_t c) {
    for (uint64_t i = nn * c / 256; i < nn * (c + 1) / 256; i++)
      for (uint32_t j = 0; j < hs.nodes[i].sub_cnt; j++) sub_node[hs.nodes[i].sub_off + j] = (uint32_t)i;
  });
  ph.mark("m:subnode");
  const uint32_t nc = st.clients().size();
  // the subscriptions by client, each client's in sid order (cstart[c] ..
  // cstart[c + 1]): a counting sort by client-range bin with per-chunk counts,
  // then each bin by client (the serial pass took 0.3 s at C3)
  std::vector<uint32_t> cstart(nc + 2, 0);
  U32Vec by_client(nsub);
  {
    constexpr uint32_t kB = 256, kS = 256;
    const uint32_t bw = nc / kB + 1;
    std::vector<uint64_t> cnt((size_t)kS * kB, 0), blo(kB + 1, 0);
    auto srange = [&](uint32_t c, uint64_t *lo, uint64_t *hi) {
      *lo = nsub * c / kS;
      *hi = nsub * (c + 1) / kS;
    };
    parallel_for(kS, [&](uint32_t c) {
      uint64_t lo, hi;
      srange(c, &lo, &hi);
      for (uint64_t x = lo; x < hi; x++) cnt[(size_t)c * kB + hs.subs[x].client / bw]++;
    });
    uint64_t run = 0;
    for (uint32_t b = 0; b < kB; b++) {
      blo[b] = run;
      for (uint32_t c = 0; c < kS; c++) {
        const uint64_t v = cnt[(size_t)c * kB + b];
        cnt[(size_t)c * kB + b] = run;
        run += v;
      }
    }
    blo[kB] = run;
    U32Vec tmp(nsub);  // sids by bin, sid order within
    parallel_for(kS, [&](uint32_t c) {
      uint64_t lo, hi;
      srange(c, &lo, &hi);
      for (uint64_t x = lo; x < hi; x++) tmp[cnt[(size_t)c * kB + hs.subs[x].client / bw]++] = (uint32_t)x;
    });
    parallel_for(kB, [&](uint32_t b) {
      const uint32_t clo = std::min<uint64_t>((uint64_t)b * bw, nc), chi = std::min<uint64_t>((uint64_t)(b + 1) * bw, nc);
      for (uint64_t j = blo[b]; j < blo[b + 1]; j++) cstart[hs.subs[tmp[j]].client + 1]++;
      uint64_t r = blo[b];
      for (uint32_t c = clo; c < chi; c++) {
        const uint32_t v = cstart[c + 1];
        cstart[c + 1] = (uint32_t)r;  // (a cursor first, then client c's end)
        r += v;
      }
      for (uint64_t j = blo[b]; j < blo[b + 1]; j++) by_client[cstart[hs.subs[tmp[j]].client + 1]++] = tmp[j];
    });
    // cstart[c + 1] is now client c's end = client c + 1's start
  }
  ph.mark("m:byclient");
  auto wild = [&](uint32_t tok) { return tok == plus_tok || tok == hash_tok; };
  // (read at every flatten: a test compares both markings in one process)
  const bool hash_multi = getenv("MQM_HASH_MULTI") && atoi(getenv("MQM_HASH_MULTI")) != 0;
  auto compatible = [&](uint32_t a, uint32_t b) {
    while (kd[a].y > kd[b].y) a = par[a];
    while (kd[b].y > kd[a].y) b = par[b];
    for (; a != b; a = par[a], b = par[b]) {  // common ancestor: same levels above
      const uint32_t ka = kd[a].x, kb = kd[b].x;
      if (ka != kb && !wild(ka) && !wild(kb)) return false;
    }
    return true;
  };
  pt.cnt.assign(nsub, 0);
  // clients are independent: chunks of them in parallel (each sub belongs to one client)
  constexpr uint32_t kChunks = 64;
  std::vector<uint64_t> solo(kChunks, 0);
  auto client_range = [&](uint32_t ch, uint32_t *c_lo, uint32_t *c_hi) {
    *c_lo = (uint32_t)((uint64_t)nc * ch / kChunks);
    *c_hi = (uint32_t)((uint64_t)nc * (ch + 1) / kChunks);
  };
  parallel_for(kChunks, [&](uint32_t ch) {
    uint32_t c_lo, c_hi;
    client_range(ch, &c_lo, &c_hi);
    for (uint32_t c = c_lo; c < c_hi; c++) {
      const uint32_t lo = cstart[c], hi = cstart[c + 1];
      for (uint32_t x = lo; x < hi; x++) {
        const uint32_t sx = by_client[x], nx = sub_node[sx], px = par[nx];
        // the parent probe emits a '#' node's subscriptions after a literal hit on its
        // parent; the walks skip the own visit of such a node (kFlagParentLit), so
        // it is emitted once per topic.  MQM_HASH_MULTI=1 (A/B): treat them as multi.
        const bool heavy = hi - lo > kMaxPairwise ||
                           (hash_multi && kd[nx].x == hash_tok && px != 0 && !wild(kd[px].x));
        uint32_t pc = 0;
        if (!heavy)
          for (uint32_t y = lo; y < hi; y++) pc += y != x && compatible(nx, sub_node[by_client[y]]);
        const bool multi = heavy || pc > 0;
        pt.cnt[sx] = heavy || pc > kMaxPartners ? (uint16_t)kPHeavy : (uint16_t)pc;
        if (multi) hs.subs[sx].word |= kMetaMulti;
        else solo[ch]++;
      }
    }
  });
  for (uint64_t v : solo) hs.n_solo += v;
  ph.mark("m:mark");
  pt.off.assign(nsub + 1, 0);
  for (uint64_t sx = 0; sx < nsub; sx++) pt.off[sx + 1] = pt.off[sx] + (pt.cnt[sx] == kPHeavy ? 0 : pt.cnt[sx]);
  pt.part.resize(pt.off[nsub]);
  parallel_for(kChunks, [&](uint32_t ch) {
    uint32_t c_lo, c_hi;
    client_range(ch, &c_lo, &c_hi);
    for (uint32_t c = c_lo; c < c_hi; c++) {
      const uint32_t lo = cstart[c], hi = cstart[c + 1];
      for (uint32_t x = lo; x < hi; x++) {
        const uint32_t sx = by_client[x];
        if (pt.cnt[sx] == 0 || pt.cnt[sx] == kPHeavy) continue;
        uint64_t w = pt.off[sx];
        for (uint32_t y = lo; y < hi; y++)
          if (y != x && compatible(sub_node[sx], sub_node[by_client[y]])) pt.part[w++] = by_client[y];
      }
    }
  });
}

// DeviceRetained arrays (snapshot.h) over the preorder ids
static void build_retained(const Store &st, const U32Vec &order, const U32Vec &new_id,
                           HostSnapshot &hs) {
  const auto &nodes = st.nodes();
  const uint64_t nn = order.size();
  std::vector<uint32_t> parent(nn, kNone);
  for (uint64_t i = 1; i < nn; i++) parent[i] = new_id[nodes[order[i]].parent];
  hs.subtree.assign(nn, 1);
  for (uint64_t i = nn - 1; i >= 1; i--) hs.subtree[parent[i]] += hs.subtree[i];
  hs.child_off.assign(nn + 1, 0);
  for (uint64_t i = 1; i < nn; i++) hs.child_off[parent[i] + 1]++;
  for (uint64_t i = 0; i < nn; i++) hs.child_off[i + 1] += hs.child_off[i];
  hs.child_ids.resize(nn ? nn - 1 : 0);
  {
    std::vector<uint32_t> cur(hs.child_off.begin(), hs.child_off.end() - 1);
    for (uint64_t i = 1; i < nn; i++) hs.child_ids[cur[parent[i]]++] = (uint32_t)i;  // increasing ids
  }
  const uint32_t sys_tok = st.tokens().find("$SYS");
  const uint32_t sys = sys_tok == kNone ? kNone : st.child(st.root(), sys_tok);
  hs.sys_child = sys == kNone ? kNone : new_id[sys];
  hs.cum.assign(nn + 1, 0);
  hs.refs.clear();
  hs.rch_off.assign(nn + 1, 0);
  for (uint64_t i = 0; i < nn; i++) {
    const HNode &h = nodes[order[i]];
    hs.cum[i + 1] = hs.cum[i] + (h.retain_path ? 1u : 0u);
    if (h.retain_path) {
      hs.refs.push_back(h.ret_ref);
      if (i > 0 && (uint32_t)i != hs.sys_child) hs.rch_off[parent[i] + 1]++;
    }
  }
  for (uint64_t i = 0; i < nn; i++) hs.rch_off[i + 1] += hs.rch_off[i];
  hs.rch_refs.resize(hs.rch_off[nn]);
  {
    std::vector<uint32_t> cur(hs.rch_off.begin(), hs.rch_off.end() - 1);
    for (uint64_t i = 1; i < nn; i++)
      if (nodes[order[i]].retain_path && (uint32_t)i != hs.sys_child)
        hs.rch_refs[cur[parent[i]]++] = nodes[order[i]].ret_ref;
  }
  auto it = st.retained().find(std::string());
  hs.has_empty = it != st.retained().end();
  hs.refs.push_back(hs.has_empty ? it->second.msg_ref : 0);
}


// The reverse walk's literal-edge index (DeviceRetained::inv / groups) from
// the staged literal edges (parent preorder order): stable partition of the
// edges into 256 buckets by their (token, child depth) group, a stable sort
// by group within each bucket (edges of one group stay in parent order: at a
// fixed depth, preorder orders children like their parents), then one table
// slot per group.  Depends on nothing but the store: digests are reproducible.
template <class Staged>
static void build_reverse_index(const Store &st, const U32Vec &order, const Staged &staged,
                                HostSnapshot &hs) {
  const auto &nodes = st.nodes();
  const uint64_t ne = staged.size();
  hs.rinv.clear();
  hs.rgroups.clear();
  if (ne == 0 || ne >= kNone || hs.height >= (1u << 16)) return;  // no index: the walk probes children
  constexpr uint32_t kB = 256, kC = 64;
  auto gkey = [&](uint64_t e) {  // token id << 16 | child depth
    const uint32_t c = order[staged[e].child];
    return ((uint64_t)nodes[c].key << 16) | nodes[c].depth;
  };
  auto bucket = [](uint64_t g) { return (uint32_t)((g * 0x9E3779B97F4A7C15ull) >> 56); };
  std::vector<uint64_t> cnt((uint64_t)kC * kB, 0);
  parallel_for(kC, [&](uint32_t c) {
    const uint64_t lo = ne * c / kC, hi = ne * (c + 1) / kC;
    for (uint64_t e = lo; e < hi; e++) cnt[(uint64_t)c * kB + bucket(gkey(e))]++;
  });
  std::vector<uint64_t> bstart(kB + 1, 0);
  {
    uint64_t run = 0;
    for (uint32_t b = 0; b < kB; b++) {
      bstart[b] = run;
      for (uint32_t c = 0; c < kC; c++) {
        const uint64_t v = cnt[(uint64_t)c * kB + b];
        cnt[(uint64_t)c * kB + b] = run;
        run += v;
      }
    }
    bstart[kB] = run;
  }
  struct GE {
    uint64_t g;
    uint32_t e, parent;  // a group's edges by parent preorder (retained.hip inv_lower)
  };
  std::vector<GE, NoInitAlloc<GE>> tmp(ne);
  parallel_for(kC, [&](uint32_t c) {
    const uint64_t lo = ne * c / kC, hi = ne * (c + 1) / kC;
    for (uint64_t e = lo; e < hi; e++) {
      const uint64_t g = gkey(e);
      tmp[cnt[(uint64_t)c * kB + bucket(g)]++] = GE{g, (uint32_t)e, staged[e].parent};
    }
  });
  hs.rinv.resize(ne);
  std::vector<std::vector<RevGroup>> bg(kB);
  parallel_for(kB, [&](uint32_t b) {
    // (a parent has one child per key: (g, parent) is unique)
    std::sort(tmp.begin() + bstart[b], tmp.begin() + bstart[b + 1],
              [](const GE &x, const GE &y) { return x.g != y.g ? x.g < y.g : x.parent < y.parent; });
    for (uint64_t j = bstart[b]; j < bstart[b + 1]; j++) {
      const auto &ed = staged[tmp[j].e];
      hs.rinv[j] = uint2{ed.parent, ed.child};
      if (j == bstart[b] || tmp[j].g != tmp[j - 1].g) {
        RevGroup r;
        r.k0 = ed.k0;
        r.k1 = ed.k1;
        r.depth_len = (uint32_t)(tmp[j].g & 0xFFFFu) | (ed.tok_len << 16);
        r.tok_off = ed.tok_off;
        r.start = (uint32_t)j;
        r.count = 0;
        bg[b].push_back(r);
      }
      bg[b].back().count++;
    }
  });
  uint64_t ng = 0;
  for (auto &v : bg) ng += v.size();
  const uint64_t nslots = 2 * ng + 1;
  RevGroup empty;
  memset(&empty, 0, sizeof(empty));
  hs.rgroups.assign(nslots, empty);
  for (auto &v : bg)
    for (const RevGroup &r : v) {
      const Key k{r.k0, r.k1};
      uint64_t slot = bucket_of(edge_hash(r.depth_len & 0xFFFFu, k), nslots);
      while (hs.rgroups[slot].count != 0) slot = slot + 1 == nslots ? 0 : slot + 1;
      hs.rgroups[slot] = r;
    }
}

void insert_edges_host(HostSnapshot &hs, const EdgeVec &staged) {
  // (b) stable partition by home slot into kEdgeParts contiguous slot ranges;
  // (c) linear-probing insertion per partition in edge order, in parallel;
  // (d) edges whose probe runs past their partition's end, serially in
  // partition order (snapshot.h: the layout edges.hip reproduces)
  constexpr uint32_t kChunks = 64, P = kEdgeParts;
  const uint64_t ne = staged.size(), n_slots = hs.n_buckets * kEdgesPerBucket;
  std::vector<uint64_t, NoInitAlloc<uint64_t>> home(ne);
  std::vector<uint64_t> cnt((uint64_t)kChunks * P, 0);  // [chunk][part]
  parallel_for(kChunks, [&](uint32_t c) {
    const uint64_t lo = ne * c / kChunks, hi = ne * (c + 1) / kChunks;
    for (uint64_t e = lo; e < hi; e++) {
      home[e] = edge_home(staged[e], hs.n_buckets);
      cnt[(uint64_t)c * P + edge_part_of(home[e], n_slots)]++;
    }
  });
  std::vector<uint64_t> pstart(P + 1, 0);
  {
    uint64_t run = 0;
    for (uint32_t p = 0; p < P; p++) {
      pstart[p] = run;
      for (uint32_t c = 0; c < kChunks; c++) {
        const uint64_t v = cnt[(uint64_t)c * P + p];
        cnt[(uint64_t)c * P + p] = run;
        run += v;
      }
    }
    pstart[P] = run;
  }
  std::vector<uint32_t, NoInitAlloc<uint32_t>> by_part(ne);
  parallel_for(kChunks, [&](uint32_t c) {
    const uint64_t lo = ne * c / kChunks, hi = ne * (c + 1) / kChunks;
    for (uint64_t e = lo; e < hi; e++) by_part[cnt[(uint64_t)c * P + edge_part_of(home[e], n_slots)]++] = (uint32_t)e;
  });
  EdgeEntry empty;
  memset(&empty, 0, sizeof(empty));
  empty.parent = kNone;
  empty.child = kNone;
  hs.edges.resize(n_slots);
  std::vector<std::vector<uint32_t>> spill(P);
  parallel_for(P, [&](uint32_t p) {
    const uint64_t lo = edge_part_lo(p, n_slots), hi = edge_part_lo(p + 1, n_slots);
    std::fill(hs.edges.begin() + lo, hs.edges.begin() + hi, empty);
    for (uint64_t j = pstart[p]; j < pstart[p + 1]; j++) {
      const uint32_t e = by_part[j];
      uint64_t slot = home[e];
      while (slot < hi && hs.edges[slot].parent != kNone) slot++;
      if (slot == hi)
        spill[p].push_back(e);
      else
        hs.edges[slot] = staged[e];
    }
  });
  for (uint32_t p = 0; p < P; p++)
    for (uint32_t e : spill[p]) {
      uint64_t slot = home[e];
      while (hs.edges[slot].parent != kNone) slot = slot + 1 == n_slots ? 0 : slot + 1;
      hs.edges[slot] = staged[e];
    }
}

int flatten(const Store &st, HostSnapshot *out, bool host_edges, FlattenCache *cache) {
  PhaseTimer pt;
  const auto &nodes = st.nodes();
  const uint32_t plus_tok = st.plus_token(), hash_tok = st.hash_token();
  HostSnapshot &hs = *out;
  hs = HostSnapshot();
  // the trie's shape as the cache saw it: its preorder and edge list stand
  const bool reuse = cache && cache->valid && cache->structure == st.structure_version() &&
                     cache->n_tokens == st.tokens().size() && cache->host_edges == host_edges &&
                     st.retained_len() == 0 && cache->new_id.size() == nodes.size();
  FlattenCache local;
  FlattenCache &pre = cache ? *cache : local;  // (its arrays are rewritten when the shape is not kept)
  if (cache && !reuse) cache->valid = false;
  U32Vec &new_id = pre.new_id, &order = pre.order, &pc_of = pre.pc_of, &hc_of = pre.hc_of,
                        &nlit = pre.nlit;
  // literal children by parent (store ids), as offsets + list, in store-id
  // order; set below when the shape is not kept, read by the preorder and the
  // edge staging
  using Kids = FlatKids;
  auto &kid = pre.kid;            // by store id (one 16-B read per node for the preorder)
  auto &lch = pre.lch, &kch = pre.kch;  // (kch: lch's token ids)
  if (!reuse) {
  // 0. every node's children from one pass over the node array (the store's
  //    sibling links cost a dependent cache miss per child: the preorder's
  //    chase took 6.5 s on 4 threads at C3).  A node's '+' / '#' child goes to
  //    kid[].pc / .hc, its literal children to its range of lch in store-id order:
  //    a counting sort of the (parent, child) pairs — by parent range into
  //    kPBins bins (per-chunk counts, no atomics: an atomic per child cost a
  //    second at C3), then each bin by parent with the bin's counters in cache;
  //    the pairs of a bin stay in child order, so no range needs sorting.
  const uint32_t n_store = (uint32_t)nodes.size();
  kid.resize(n_store);
  constexpr uint32_t kSChunks = 256, kPBins = 256;
  const uint32_t bin_w = n_store / kPBins + 1;  // parents per bin
  auto schunk = [&](uint32_t c, uint32_t *lo, uint32_t *hi) {
    *lo = (uint32_t)((uint64_t)n_store * c / kSChunks);
    *hi = (uint32_t)((uint64_t)n_store * (c + 1) / kSChunks);
  };
  auto &lpar = pre.lpar, &ktok = pre.ktok;  // a literal child's parent (else kNone), every node's token
  lpar.resize(n_store);
  ktok.resize(n_store);
  std::vector<uint64_t> bcnt((size_t)kSChunks * kPBins, 0);  // [chunk][bin]
  parallel_for(kSChunks, [&](uint32_t c) {
    uint32_t lo, hi;
    schunk(c, &lo, &hi);
    for (uint32_t n = lo; n < hi; n++) kid[n] = Kids{0, 0, kNone, kNone};
  });
  pt.mark("c:init");
  parallel_for(kSChunks, [&](uint32_t c) {
    uint32_t lo, hi;
    schunk(c, &lo, &hi);
    uint64_t *cnt = &bcnt[(size_t)c * kPBins];
    for (uint32_t n = lo; n < hi; n++) {
      const HNode &h = nodes[n];
      ktok[n] = h.key;
      lpar[n] = kNone;
      if (h.parent == kNone) continue;  // the root, a free slot
      if (h.key == plus_tok)
        kid[h.parent].pc = n;
      else if (h.key == hash_tok)
        kid[h.parent].hc = n;
      else {
        lpar[n] = h.parent;
        cnt[h.parent / bin_w]++;
      }
    }
  });
  pt.mark("c:count");
  std::vector<uint64_t> bin_lo(kPBins + 1, 0);
  {
    uint64_t run = 0;
    for (uint32_t b = 0; b < kPBins; b++) {
      bin_lo[b] = run;
      for (uint32_t c = 0; c < kSChunks; c++) {
        const uint64_t v = bcnt[(size_t)c * kPBins + b];
        bcnt[(size_t)c * kPBins + b] = run;
        run += v;
      }
    }
    bin_lo[kPBins] = run;
  }
  const uint64_t n_lit = bin_lo[kPBins];
  std::vector<uint2, NoInitAlloc<uint2>> pairs(n_lit);  // (parent, child), by bin, child order within
  parallel_for(kSChunks, [&](uint32_t c) {
    uint32_t lo, hi;
    schunk(c, &lo, &hi);
    uint64_t *off = &bcnt[(size_t)c * kPBins];
    for (uint32_t n = lo; n < hi; n++)
      if (lpar[n] != kNone) pairs[off[lpar[n] / bin_w]++] = make_uint2(lpar[n], n);
  });
  pt.mark("c:place");
  lch.resize(n_lit);
  kch.resize(n_lit);
  parallel_for(kPBins, [&](uint32_t b) {
    const uint32_t plo = std::min<uint64_t>((uint64_t)b * bin_w, n_store),
                   phi = std::min<uint64_t>((uint64_t)(b + 1) * bin_w, n_store);
    for (uint64_t k = bin_lo[b]; k < bin_lo[b + 1]; k++) kid[pairs[k].x].cnt++;
    uint64_t run = bin_lo[b];
    for (uint32_t p = plo; p < phi; p++) {
      kid[p].off = (uint32_t)run;
      run += kid[p].cnt;
      kid[p].cnt = 0;  // (counts again as the cursor below)
    }
    for (uint64_t k = bin_lo[b]; k < bin_lo[b + 1]; k++) {
      Kids &d = kid[pairs[k].x];
      const uint32_t q = d.off + d.cnt++;
      lch[q] = pairs[k].y;
      kch[q] = ktok[pairs[k].y];
    }
  });
  pt.mark("p:children");
  // 1. preorder ids.  Visiting order at a node: literal children by store id,
  //    then '+', then '#'.  The root and its children are numbered serially;
  //    the subtrees rooted at depth 2 are counted (HNode::subtree), then
  //    numbered at their preorder base, in parallel.
  new_id.resize(nodes.size());  // (kNone everywhere first: free slots keep it)
  parallel_for(64, [&](uint32_t c) {
    std::fill(new_id.begin() + nodes.size() * c / 64, new_id.begin() + nodes.size() * (c + 1) / 64, kNone);
  });
  // children of n in visiting order, pushed for a LIFO visit
  // (each child's record and id slot are prefetched as it is pushed: the
  // DFS pops it soon after)
  auto push_children = [&](std::vector<uint32_t> &stack, uint32_t n) {
    const Kids d = kid[n];
    auto push = [&](uint32_t c) {
      __builtin_prefetch(&kid[c]);
      __builtin_prefetch(&new_id[c], 1);
      stack.push_back(c);
    };
    if (d.hc != kNone) push(d.hc);  // LIFO: '#' visited last
    if (d.pc != kNone) push(d.pc);
    for (uint32_t k = d.off + d.cnt; k > d.off; k--) push(lch[k - 1]);
  };
  struct Item {
    uint32_t node;
    bool task;  // subtree numbered in parallel
    uint64_t size;
  };
  std::vector<Item> seq;  // the top levels in preorder, subtrees as placeholders
  {
    std::vector<uint32_t> top;
    push_children(top, st.root());
    std::reverse(top.begin(), top.end());  // visit order
    size_t n_seq = 1 + top.size();
    for (uint32_t r : top) n_seq += kid[r].cnt + (kid[r].pc != kNone) + (kid[r].hc != kNone);
    seq.reserve(n_seq);
    seq.push_back(Item{st.root(), false, 1});
    for (uint32_t r : top) {
      seq.push_back(Item{r, false, 1});
      const Kids d = kid[r];  // visit order: literals, '+', '#'
      for (uint32_t k = d.off; k < d.off + d.cnt; k++) seq.push_back(Item{lch[k], true, 0});
      if (d.pc != kNone) seq.push_back(Item{d.pc, true, 0});
      if (d.hc != kNone) seq.push_back(Item{d.hc, true, 0});
    }
  }
  pt.mark("p:top");
  // subtree sizes: the store keeps them (HNode::subtree)
  const uint32_t n_items = (uint32_t)seq.size();
  parallel_for(64, [&](uint32_t w) {
    for (uint32_t j = w; j < n_items; j += 64)
      if (seq[j].task) seq[j].size = nodes[seq[j].node].subtree;
  });
  std::vector<uint64_t> base(n_items);
  uint64_t total = 0;
  for (uint32_t j = 0; j < n_items; j++) {
    base[j] = total;
    total += seq[j].size;
  }
  if (total >= (1ull << 30)) return MQM_ELIMIT;  // k_walk packs node id << 2 | item kind
  // (every entry is written by the numbering below)
  order.resize(total);
  pc_of.resize(total);
  hc_of.resize(total);
  nlit.resize(total);
  std::atomic<bool> size_bad{false};
  // number every item: a top node itself, a subtree by DFS from its base
  parallel_for(64, [&](uint32_t w) {
    std::vector<uint32_t> stack;
    for (uint32_t j = w; j < n_items; j += 64) {
      uint64_t id = base[j];
      stack.assign(1, seq[j].node);
      while (!stack.empty()) {
        const uint32_t n = stack.back();
        stack.pop_back();
        if (id >= base[j] + seq[j].size) break;  // (flagged below: no write past the item's range)
        new_id[n] = (uint32_t)id;
        order[id] = n;
        const Kids d = kid[n];
        pc_of[id] = d.pc;
        hc_of[id] = d.hc;
        nlit[id] = d.cnt;
        id++;
        if (seq[j].task) push_children(stack, n);
      }
      if (id != base[j] + seq[j].size || !stack.empty()) size_bad.store(true, std::memory_order_relaxed);
    }
  });
  if (size_bad.load()) return MQM_EINVAL;  // (the store's subtree counts are off: never seen)
  if (pt.on) {
    uint64_t mx = 0;
    for (auto &x : seq) mx = std::max(mx, x.size);
    fprintf(stderr, "[flatten] nodes %zu items %u largest subtree %zu\n", order.size(), n_items, (size_t)mx);
  }
  }  // (!reuse)
  const uint64_t nn = order.size();
  pt.mark(reuse ? "preorder (kept)" : "preorder");

  // 2. descriptors, subscription ranges, flags — in parallel over preorder
  //    chunks: (A) counts, child ids and own flags per node, (prefix sums over
  //    chunks), (B) ranges filled at their prefix offsets, (C) the `$` flag
  //    inherited down the preorder (a parent precedes its children).  The
  //    layout equals that of one serial pass.
  hs.nodes.resize(nn);
  std::vector<uint8_t> flags(nn, 0);
  std::vector<uint32_t, NoInitAlloc<uint32_t>> par_new(nn);  // (set for every node below; kNone at the root)
  par_new[0] = kNone;
  std::vector<uint2, NoInitAlloc<uint2>> kd_pre(nn);  // token, depth by preorder id (mark_multi)
  constexpr uint32_t kNChunks = 256;
  std::vector<uint64_t> sub_base(kNChunks + 1, 0), sh_base(kNChunks + 1, 0), lit_c(kNChunks, 0);
  std::vector<uint32_t> height_c(kNChunks, 0);
  std::vector<uint8_t> too_many_shared(kNChunks, 0);
  auto chunk_lo = [&](uint32_t c) { return nn * c / kNChunks; };
  auto chain_start = [&](uint64_t i) { return i == 0 || nodes[order[i]].key != hash_tok; };
  pt.mark("n:init");
  parallel_for(kNChunks, [&](uint32_t c) {
    uint64_t subs_n = 0, sh_n = 0, lit = 0;
    uint32_t height = 0;
    const uint64_t i_end = chunk_lo(c + 1);
    for (uint64_t i = chunk_lo(c); i < i_end; i++) {
      if (i + kAhead < i_end) prefetch_node(&nodes[order[i + kAhead]]);
      const HNode &h = nodes[order[i]];
      NodeDesc &d = hs.nodes[i];
      kd_pre[i] = make_uint2(h.key, h.depth);
      const uint32_t pc = pc_of[i], hc = hc_of[i];
      d.plus = pc == kNone ? kNone : new_id[pc];
      d.hash = hc == kNone ? kNone : new_id[hc];
      lit += nlit[i];
      // subscription ranges: a node's, then its '#' child's, then that one's
      // '#' child's ... back to back (NodeDesc::hsub_cnt); counted at the chain start
      if (chain_start(i))
        for (uint32_t sn = order[i];;) {
          subs_n += nodes[sn].subs.size();
          sn = hc_of[new_id[sn]];
          if (sn == kNone) break;
        }
      if (h.shared.size() > kShCntMask) too_many_shared[c] = 1;
      sh_n += h.shared.size();
      uint8_t f = h.n_children ? (uint8_t)kFlagHasChildren : (uint8_t)0;
      if (nlit[i]) f |= kFlagHasLiteral;
      if (i > 0) {
        par_new[i] = new_id[h.parent];
        if (h.key == hash_tok && par_new[i] != 0 && nodes[h.parent].key != hash_tok &&
            nodes[h.parent].key != plus_tok)
          f |= kFlagParentLit;
        if (par_new[i] == 0) {  // root child: Filter[0] of every sub stored below it
          const std::string_view k = st.tokens().name(h.key);
          if (!k.empty() && (k[0] == '+' || k[0] == '#')) f |= kFlagDollarWild;
        }
      }
      flags[i] = f;
      d.sh_cnt_flags = (uint32_t)std::min<uint64_t>(h.shared.size(), kShCntMask);
      height = std::max(height, h.depth);
    }
    sub_base[c + 1] = subs_n;
    sh_base[c + 1] = sh_n;
    lit_c[c] = lit;
    height_c[c] = height;
  });
  pt.mark("n:count");
  uint64_t n_literal_edges = 0;
  for (uint32_t c = 0; c < kNChunks; c++) {
    if (too_many_shared[c]) return MQM_ELIMIT;
    sub_base[c + 1] += sub_base[c];
    sh_base[c + 1] += sh_base[c];
    n_literal_edges += lit_c[c];
    hs.height = std::max(hs.height, height_c[c]);
  }
  if (sub_base[kNChunks] > kMaxSubs) return MQM_ELIMIT;
  if (sh_base[kNChunks] > kMaxSubs) return MQM_ELIMIT;  // shared ids fit 28 bits (mqm_gather_shards_shared)
  hs.subs.resize(sub_base[kNChunks]);
  hs.sub_info.resize(sub_base[kNChunks]);
  hs.shared_info.resize(sh_base[kNChunks]);
  pt.mark("n:alloc");
  parallel_for(kNChunks, [&](uint32_t c) {
    uint64_t so = sub_base[c], ho = sh_base[c];
    const uint64_t i_end = chunk_lo(c + 1);
    for (uint64_t i = chunk_lo(c); i < i_end; i++) {
      if (i + 2 * kAhead < i_end) prefetch_node(&nodes[order[i + 2 * kAhead]]);
      if (i + kAhead < i_end) __builtin_prefetch(nodes[order[i + kAhead]].subs.data());
      if (chain_start(i))
        for (uint32_t k = (uint32_t)i, sn = order[i];;) {
          const auto &subs = nodes[sn].subs;
          hs.nodes[k].sub_off = (uint32_t)so;
          hs.nodes[k].sub_cnt = (uint32_t)subs.size();
          for (const SubRec &x : subs) {
            hs.subs[so] = SubEnt{x.client, ((uint32_t)x.qos & 3u) | ((uint32_t)(x.no_local & 1) << 2) |
                                              ((uint32_t)(x.rap & 1) << 3) | ((uint32_t)(x.rh & 3) << 4) |
                                              (x.ident > 0 ? kMetaIdent : 0u)};
            hs.sub_info[so++] = SubInfo{x.filter, x.client, x.ident, x.qos, x.no_local, x.rap, x.rh};
          }
          sn = hc_of[k];
          if (sn == kNone) break;
          k = new_id[sn];
        }
      hs.nodes[i].sh_off = (uint32_t)ho;
      for (const SharedRec &x : nodes[order[i]].shared)
        hs.shared_info[ho++] =
            SubInfo{x.sub.filter, x.sub.client, x.sub.ident, x.sub.qos, x.sub.no_local, x.sub.rap, x.sub.rh};
    }
  });
  pt.mark("n:fill");
  for (uint64_t i = 1; i < nn; i++) {
    if (par_new[i] != 0) flags[i] |= flags[par_new[i]] & kFlagDollarWild;
  }
  for (uint64_t i = 0; i < nn; i++) hs.nodes[i].sh_cnt_flags |= (uint32_t)flags[i] << 24;
  pt.mark("nodes");
  Partners partners;
  mark_multi(st, hs, partners, par_new, kd_pre);
  pt.mark("multi");
  if (st.retained_len() > 0) build_retained(st, order, new_id, hs);
  pt.mark("retained");
  // every range: solo entries first, then multi (stable); count the multi ones
  // (nodes are independent: in parallel over preorder chunks)
  constexpr uint32_t kRChunks = 256;
  auto rchunk = [&](uint32_t c, uint64_t *lo, uint64_t *hi) {
    *lo = nn * c / kRChunks;
    *hi = nn * (c + 1) / kRChunks;
  };
  U32Vec own_multi(nn, 0);
  U32Vec new_sid(hs.subs.size());
  parallel_for(kRChunks, [&](uint32_t c) {
    uint64_t lo, hi;
    rchunk(c, &lo, &hi);
    std::vector<SubEnt> se;
    std::vector<SubInfo> si;
    for (uint64_t i = lo; i < hi; i++) {
      const uint32_t off = hs.nodes[i].sub_off, cnt = hs.nodes[i].sub_cnt;
      se.clear();
      si.clear();
      for (int pass = 0; pass < 2; pass++)
        for (uint32_t j = off; j < off + cnt; j++)
          if (((hs.subs[j].word & kMetaMulti) != 0) == (pass == 1)) {
            new_sid[j] = off + (uint32_t)se.size();
            se.push_back(hs.subs[j]);
            si.push_back(hs.sub_info[j]);
            own_multi[i] += pass;
          }
      std::copy(se.begin(), se.end(), hs.subs.begin() + off);
      std::copy(si.begin(), si.end(), hs.sub_info.begin() + off);
    }
  });
  // the multi subscriptions' partner lists in final sids (snapshot.h: pinfo)
  {
    const uint64_t nsub = hs.subs.size();
    hs.pinfo.assign(nsub, make_uint2(0, 0));
    hs.partners.clear();
    std::vector<uint8_t> heavy_at(nsub, 0);
    // a partner is known by the multi-tail start of its node's range (where
    // the walk's multi part of that range starts, whichever probe gathered it)
    U32Vec tail_of(nsub, 0);
    parallel_for(kRChunks, [&](uint32_t c) {
      uint64_t lo, hi;
      rchunk(c, &lo, &hi);
      for (uint64_t i = lo; i < hi; i++) {
        const uint32_t off = hs.nodes[i].sub_off, cnt = hs.nodes[i].sub_cnt;
        for (uint32_t j = off + cnt - own_multi[i]; j < off + cnt; j++) tail_of[j] = off + cnt - own_multi[i];
      }
    });
    auto pkey = [&](uint32_t old) {
      const uint32_t p = new_sid[old], m = hs.subs[p].word;  // build-time meta (snapshot.h): qos[1:0], nl[2]
      return tail_of[p] | (m & 3u) << 28 | ((m >> 2) & 1u) << 30;
    };
    // lists of more than two partners, at offsets in entry order (counted,
    // prefix-summed, filled in parallel: the layout of one serial pass)
    constexpr uint32_t kPChunks = 256;
    std::vector<uint64_t> list_base(kPChunks + 1, 0);
    auto pchunk = [&](uint32_t c, uint64_t *lo, uint64_t *hi) {
      *lo = nsub * c / kPChunks;
      *hi = nsub * (c + 1) / kPChunks;
    };
    parallel_for(kPChunks, [&](uint32_t c) {
      uint64_t lo, hi, t = 0;
      pchunk(c, &lo, &hi);
      for (uint64_t x = lo; x < hi; x++) {
        const uint16_t k = partners.cnt[x];
        if (k > 2 && k != kPHeavy) t += k;
      }
      list_base[c + 1] = t;
    });
    for (uint32_t c = 0; c < kPChunks; c++) list_base[c + 1] += list_base[c];
    hs.partners.resize(list_base[kPChunks]);
    parallel_for(kPChunks, [&](uint32_t c) {
      uint64_t lo, hi;
      pchunk(c, &lo, &hi);
      uint64_t w = list_base[c];
      for (uint64_t x = lo; x < hi; x++) {
        const uint16_t k = partners.cnt[x];
        if (k == 0) continue;
        const uint32_t nx = new_sid[x];
        if (k == kPHeavy) {
          hs.pinfo[nx] = make_uint2(kNone, kPInfoHeavy);
          heavy_at[nx] = 1;
        } else if (k <= 2) {  // inline: the partner's key | QoS << 28 | NoLocal << 30
          const uint64_t o = partners.off[x];
          hs.pinfo[nx] = make_uint2(pkey(partners.part[o]), k == 2 ? pkey(partners.part[o + 1]) : kNone);
        } else {
          hs.pinfo[nx] = make_uint2((uint32_t)w, kPInfoList | k);
          for (uint64_t o = partners.off[x]; o < partners.off[x + 1]; o++) hs.partners[w++] = pkey(partners.part[o]);
        }
      }
    });
    // a node whose range (multi tail) holds a heavy entry: its topics merge by hash table
    parallel_for(kRChunks, [&](uint32_t c) {
      uint64_t lo, hi;
      rchunk(c, &lo, &hi);
      for (uint64_t i = lo; i < hi; i++) {
        const uint32_t off = hs.nodes[i].sub_off, cnt = hs.nodes[i].sub_cnt;
        for (uint32_t j = off + cnt - own_multi[i]; j < off + cnt; j++)
          if (heavy_at[j]) {
            flags[i] |= kFlagHeavyOwn;
            break;
          }
      }
    });
  }
  // a '#' child that is a leaf without shared subscriptions, read before the
  // pass below adds flag bits (kFlagHashLeaf)
  std::vector<uint8_t> hash_leaf(nn, 0);
  parallel_for(kRChunks, [&](uint32_t c) {
    uint64_t lo, hi;
    rchunk(c, &lo, &hi);
    for (uint64_t i = lo; i < hi; i++) {
      const NodeDesc &h = hs.nodes[i];
      hash_leaf[i] = !((h.sh_cnt_flags >> 24) & kFlagHasChildren) && (h.sh_cnt_flags & kShCntMask) == 0;
    }
  });
  parallel_for(kRChunks, [&](uint32_t c) {
    uint64_t lo, hi;
    rchunk(c, &lo, &hi);
    for (uint64_t i = lo; i < hi; i++) {
      NodeDesc &d = hs.nodes[i];
      const uint32_t hm = d.hash != kNone ? own_multi[d.hash] : 0;
      d.hsub_cnt = d.hash != kNone ? hs.nodes[d.hash].sub_cnt : 0;
      d.multi = std::min<uint32_t>(own_multi[i], 0xFFFF) | (std::min<uint32_t>(hm, 0xFFFF) << 16);
      if (own_multi[i] >= 0xFFFF || hm >= 0xFFFF) d.sh_cnt_flags |= (uint32_t)kFlagMultiSat << 24;
      d.sh_cnt_flags |= (uint32_t)(flags[i] & kFlagHeavyOwn) << 24;
      if (d.hash != kNone && (flags[d.hash] & kFlagHeavyOwn)) d.sh_cnt_flags |= (uint32_t)kFlagHeavyHash << 24;
      if (i > 0 && d.hash != kNone && hash_leaf[d.hash])  // root: its '#' child is dollar-wild, unlike the root itself
        d.sh_cnt_flags |= (uint32_t)kFlagHashLeaf << 24;
    }
  });

  // the device word (snapshot.h): the entry's own delivery, ident flag on top
  // (and the host copy of DeviceSnapshot::words: the runs form's deliveries)
  hs.words.resize(hs.subs.size());
  parallel_for(64, [&](uint32_t c) {
    const uint64_t n = hs.subs.size(), lo = n * c / 64, hi = n * (c + 1) / 64;
    for (uint64_t j = lo; j < hi; j++) {
      const uint32_t m = hs.subs[j].word;
      hs.subs[j].word = (uint32_t)j | ((m & 3u) << 28) | (((m >> 2) & 1u) << 30) | ((m & kMetaIdent) ? kWordIdent : 0u);
      hs.words[j] = hs.subs[j].word & kPackedMask;
    }
  });
  pt.mark("ranges");
  // 3. literal edges -> open-addressed table of 128-B buckets, linear probing
  //    at load factor `load`: a probe chain
  //    that leaves its home entry costs another dependent HBM round trip, and
  //    a wavefront waits for its longest chain (measured on C3: k_walk 9.5 /
  //    10.9 / 16.5 / 71 ms at load 0.15 / 0.26 / 0.5 / 0.8 in round 1; with the
  //    edge filter 6.44 / 6.79 / 7.49 ms at 0.12 / 0.2 / 0.35).  Default 0.12
  //    up to 64M edges (18.5 GB at C3), 0.2 beyond (the table's host copy and
  //    upload grow with it: config 5 has 79M edges)
  const double load = n_literal_edges <= (64ull << 20) ? 0.12 : 0.2;
  const uint64_t buckets =
      std::max<uint64_t>(1, (uint64_t)((double)n_literal_edges / (load * kEdgesPerBucket)) + 1);
  hs.n_buckets = buckets;
  hs.n_edges = n_literal_edges;
  if (n_literal_edges >= kNone || buckets * kEdgesPerBucket >= (1ull << 50)) return MQM_ELIMIT;
  // long tokens (> kInlineMax bytes) go to the pool in token-id order
  const Interner &toks = st.tokens();
  std::vector<uint32_t> pool_off(toks.size(), kNone);
  for (uint32_t t = 0; t < toks.size(); t++) {
    const std::string_view tok = toks.name(t);
    if (tok.size() <= kInlineMax) continue;
    if (hs.tok_pool.size() + tok.size() > 0xFFFFFFFFull) return MQM_ELIMIT;
    pool_off[t] = (uint32_t)hs.tok_pool.size();
    hs.tok_pool.insert(hs.tok_pool.end(), tok.begin(), tok.end());
  }
  // (a) every literal edge in (parent store id, child store id) order, in parallel
  //     over node ranges; the table is then built from this list on the host
  //     (insert_edges_host) or on the device at upload (edges.hip, the same
  //     bytes: the layout depends on kEdgeParts only, not on the thread count,
  //     so digests are reproducible)
  constexpr uint32_t kChunks = 64;
  if (reuse) {
    // the same edges in the same order: only the inline child descriptors change
    if (!pre.staged || pre.staged->size() != n_literal_edges) {
      cache->valid = false;
      return MQM_EINVAL;  // (the shape moved without its version: never seen)
    }
    EdgeVec &staged = *pre.staged;
    parallel_for(kChunks, [&](uint32_t c) {
      const uint64_t lo = n_literal_edges * c / kChunks, hi = n_literal_edges * (c + 1) / kChunks;
      for (uint64_t e = lo; e < hi; e++) staged[e].desc = hs.nodes[staged[e].child];
    });
    hs.bloom = pre.bloom;
    cache->reuses++;
  } else {
    // by parent store id, then child store id (the children lists): the
    // position of an edge is its place in lch
    if (lch.size() != n_literal_edges) return MQM_EINVAL;  // (every live node is reached: never seen)
    // (the previous build's list, once no snapshot holds it: upload drops it)
    if (pre.staged && pre.staged.use_count() == 1)
      pre.staged->resize(n_literal_edges);
    else
      pre.staged = std::make_shared<EdgeVec>(n_literal_edges);
    EdgeVec &staged = *pre.staged;
    const uint32_t n_store = (uint32_t)nodes.size();
    constexpr uint32_t kPChunks = 256;
    parallel_for(kPChunks, [&](uint32_t c) {
      const uint32_t lo = (uint32_t)((uint64_t)n_store * c / kPChunks),
                     hi = (uint32_t)((uint64_t)n_store * (c + 1) / kPChunks);
      const uint64_t q_end = hi < n_store ? kid[hi].off : lch.size();
      for (uint32_t p = lo; p < hi; p++) {
        const Kids d = kid[p];
        if (d.cnt == 0) continue;
        const uint32_t pi = new_id[p];
        for (uint32_t q = d.off; q < d.off + d.cnt; q++) {
          if (q + 2 * kAhead < q_end) __builtin_prefetch(&new_id[lch[q + 2 * kAhead]]);
          if (q + kAhead < q_end) __builtin_prefetch(&hs.nodes[new_id[lch[q + kAhead]]]);
          const uint32_t cn = new_id[lch[q]];
          const std::string_view tok = toks.name(kch[q]);
          Key k = make_key([&](uint32_t j) { return (uint8_t)tok[j]; }, (uint32_t)tok.size());
          EdgeEntry &e = staged[q];
          e.k0 = k.k0;
          e.k1 = k.k1;
          e.parent = pi;
          e.child = cn;
          e.tok_off = key_is_long(k) ? pool_off[kch[q]] : 0;
          e.tok_len = (uint32_t)tok.size();
          e.desc = hs.nodes[cn];
        }
      }
    });
    pt.mark("e:list");
    // the edge-existence filter: >= 16 bits per edge, a power of two of words
    // (env MQM_NO_BLOOM=1: none, for A/B runs); OR is order-free, so the
    // parallel fill is deterministic
    hs.bloom.clear();
    if (n_literal_edges && !getenv("MQM_NO_BLOOM")) {
      uint64_t bits = 4096;
      while (bits < 16 * n_literal_edges) bits <<= 1;
      hs.bloom.assign(bits / 64, 0);
      const uint64_t mask = bits / 64 - 1;
      parallel_for(kChunks, [&](uint32_t c) {
        const uint64_t lo = n_literal_edges * c / kChunks, hi = n_literal_edges * (c + 1) / kChunks;
        // 64 edges at a time: their words are prefetched for writing first, so
        // the atomics (each drains the store buffer) find their lines in cache
        for (uint64_t e0 = lo; e0 < hi; e0 += 64) {
          const uint32_t m = (uint32_t)std::min<uint64_t>(64, hi - e0);
          uint64_t w[64], bb[64];
          for (uint32_t j = 0; j < m; j++) {
            const EdgeEntry &x = staged[e0 + j];
            const uint64_t h = edge_hash(x.parent, Key{x.k0, x.k1});
            w[j] = bloom_word(h, mask);
            bb[j] = bloom_bits(h);
            __builtin_prefetch(&hs.bloom[w[j]], 1);
          }
          for (uint32_t j = 0; j < m; j++) __atomic_fetch_or(&hs.bloom[w[j]], bb[j], __ATOMIC_RELAXED);
        }
      });
    }

  }
  pt.mark("e:stage");
  if (st.retained_len() > 0) {
    build_reverse_index(st, order, *pre.staged, hs);
    pt.mark("rev-index");
  }
  if (host_edges) {
    insert_edges_host(hs, *pre.staged);
    pt.mark("e:insert");
  } else {
    hs.staged = pre.staged;
  }
  if (cache && !reuse) {  // keep this build's shape for the next one
    // (order, new_id, pc_of, hc_of, nlit and staged were built in place)
    cache->bloom = hs.bloom;
    cache->structure = st.structure_version();
    cache->n_tokens = st.tokens().size();
    cache->host_edges = host_edges;
    cache->valid = st.retained_len() == 0;
  }
  if (hs.tok_pool.empty()) hs.tok_pool.push_back(0);
  if (hs.subs.empty()) hs.subs.push_back(SubEnt{0, 0});
  return MQM_OK;
}

// counting sorts of the sids by client (sids ascending within a client)
void build_client_index(HostSnapshot &hs) {
  auto by_client = [](const std::vector<SubInfo> &info, std::vector<uint32_t> &off, std::vector<uint32_t> &ids) {
    uint32_t nc = 0;
    for (const SubInfo &x : info) nc = std::max(nc, x.client + 1);
    off.assign((size_t)nc + 1, 0);
    for (const SubInfo &x : info) off[x.client + 1]++;
    for (uint32_t c = 0; c < nc; c++) off[c + 1] += off[c];
    ids.resize(info.size());
    std::vector<uint32_t> cur(off.begin(), off.end() - 1);
    for (uint32_t sid = 0; sid < (uint32_t)info.size(); sid++) ids[cur[info[sid].client]++] = sid;
  };
  by_client(hs.sub_info, hs.client_off, hs.client_subs);
  by_client(hs.shared_info, hs.client_shoff, hs.client_shared);
}

namespace {
// host -> device in pieces of kUploadChunk: one long DMA of gigabytes held the
// per-publish server's polls of its ring (reads of host memory, whose data
// crosses PCIe in the same direction) for up to 230 ms (r05k); between pieces
// they get through
constexpr size_t kUploadChunk = 32ull << 20;
hipError_t upload_copy(void *dst, const void *src, size_t n, hipStream_t st) {
  for (size_t o = 0; o < n; o += kUploadChunk) {
    const hipError_t e = hipMemcpyAsync((char *)dst + o, (const char *)src + o, std::min(kUploadChunk, n - o),
                                        hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}
}  // namespace

namespace {
// Snapshot buffers come from the device's stream-ordered pool and go back with
// hipFreeAsync on a stream of their own: hipFree (and hipFreeAsync of
// hipMalloc'd memory) waits until every kernel on the device has finished —
// including the per-publish server, which runs as long as calls arrive
// (tools/free_probe.hip on the box: 1000 ms, the spinner's whole run, against
// 0.0 ms for a pool free).  The pool keeps what is freed (release threshold:
// max), so a rebuild reuses the previous snapshot's memory without mapping it
// again.
struct Reclaim {
  std::mutex mu;
  hipStream_t st[64] = {};
};
Reclaim &reclaim() {
  static Reclaim r;
  return r;
}
hipStream_t reclaim_stream(int device) {
  if (device < 0 || device >= 64) return nullptr;
  Reclaim &r = reclaim();
  std::lock_guard<std::mutex> g(r.mu);
  if (!r.st[device]) {
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(device);
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess) {
      r.st[device] = s;
      hipMemPool_t pool;
      if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess) {
        uint64_t keep = ~0ull;
        (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
      }
    }
    (void)hipSetDevice(cur);
  }
  return r.st[device];
}
}  // namespace

// MQM_SNAP_POOL=1 (A/B, unsafe): snapshot buffers from the stream-ordered
// pool, freed with hipFreeAsync.  Measured wrong on the box: served results
// under churn missed the newest subscriptions (tests/test_gpu_serve_churn.py,
// r05o-r05r), and tools/reuse_probe.hip saw a kernel on another stream read
// pool memory that a synchronised host -> device copy had refilled without the
// new data (r05s).  Snapshot buffers are hipMalloc'd and recycled in place
// (below); nothing in the library takes pool memory any more.
static bool snap_pool() {
  static const bool v = getenv("MQM_SNAP_POOL") && atoi(getenv("MQM_SNAP_POOL")) != 0;
  return v;
}

// Snapshot buffers are recycled, not freed (the default since round 6): a
// destroyed snapshot's buffers go to a per-device free list and the next
// upload takes the smallest one that fits (a rebuild's arrays are within a
// few percent of the last one's).  Refilling a kept hipMalloc buffer in place
// is read correctly by kernels on other streams (tools/reuse_probe.hip r05u,
// tools/l2_probe.hip r06b); and no hipFree — which waits for the per-publish
// server — runs at all while the free list stays under kRecycleCap.  Above
// it, the largest spare buffers go to the index layer's reaper
// (retire_device_buffers), which stops the servers before freeing.  (Round 5
// found recycling correct only with a 2-s reuse quarantine; the cause was not
// the recycled buffers but the device edge build's temporaries from the
// stream-ordered pool, which served the build a previous build's staged edges
// now and then — the reaper's hipFree between builds had hidden it.  With the
// temporaries in a kept scratch region, edges.hip, served churn results equal
// the oracle at every version with no quarantine: r06d, 3 of 3 runs, against
// 3 of 3 failing with the pool temporaries.)  MQM_SNAP_RECYCLE=0: hipMalloc /
// hipFree per snapshot through the reaper (round 5's default).
namespace {
constexpr size_t kRecycleCap = 96ull << 30;  // spare bytes kept per device
struct Spare {
  void *p;
  int64_t since_ns;  // retired at (a spare is taken only after kQuarantineNs)
};
struct Recycler {
  std::mutex mu;
  std::multimap<size_t, Spare> spare[64];  // capacity -> buffer
  size_t bytes[64] = {};
};
int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
// MQM_RECYCLE_QUARANTINE_MS: a retired buffer is reused only after this long
// (default 0; round 5's workaround was 2000)
const int64_t kQuarantineNs = [] {
  const char *e = getenv("MQM_RECYCLE_QUARANTINE_MS");
  return (int64_t)(e ? atoi(e) : 0) * 1000000;
}();
// MQM_SNAP_RECYCLE=0: hipFree each snapshot on the reaper instead of recycling
bool snap_recycle() {
  static const bool v = !getenv("MQM_SNAP_RECYCLE") || atoi(getenv("MQM_SNAP_RECYCLE")) != 0;
  return v;
}
Recycler &recycler() {
  static auto *r = new Recycler;  // (never destroyed: snapshots may die during static destruction)
  return *r;
}
// a buffer of at least n bytes: a spare one of capacity in [n, 1.25 n], else a
// new one with 1/16 headroom (the next rebuild's array may be a little larger)
hipError_t recycled_alloc(int device, void **p, size_t n, size_t *cap) {
  if (device >= 0 && device < 64) {
    Recycler &r = recycler();
    std::lock_guard<std::mutex> g(r.mu);
    const int64_t now = now_ns();
    for (auto it = r.spare[device].lower_bound(n); it != r.spare[device].end() && it->first <= n + n / 4; ++it) {
      if (now - it->second.since_ns < kQuarantineNs) continue;
      *p = it->second.p;
      *cap = it->first;
      r.bytes[device] -= it->first;
      r.spare[device].erase(it);
      return hipSuccess;
    }
  }
  const size_t want = n + n / 16;
  *cap = want;
  return hipMalloc(p, want);
}
void recycled_free(int device, std::vector<std::pair<void *, size_t>> &held) {
  if (held.empty()) return;
  if (device < 0 || device >= 64) {
    std::vector<void *> v;
    for (auto &x : held) v.push_back(x.first);
    retire_device_buffers(device, std::move(v));
    return;
  }
  std::vector<void *> excess;
  {
    Recycler &r = recycler();
    std::lock_guard<std::mutex> g(r.mu);
    const int64_t now = now_ns();
    for (auto &x : held) {
      r.spare[device].emplace(x.second, Spare{x.first, now});
      r.bytes[device] += x.second;
    }
    while (r.bytes[device] > kRecycleCap && !r.spare[device].empty()) {
      auto it = std::prev(r.spare[device].end());
      excess.push_back(it->second.p);
      r.bytes[device] -= it->first;
      r.spare[device].erase(it);
    }
  }
  if (!excess.empty()) retire_device_buffers(device, std::move(excess));
}
}  // namespace

bool host_edges_forced() {
  static const bool v = getenv("MQM_HOST_EDGES") && atoi(getenv("MQM_HOST_EDGES")) != 0;
  return v;
}

// MQM_SNAP_VERIFY=1 (diagnostic): after an upload, read the device arrays
// back and compare them with the host arrays (the edge table: a host build of
// the same staged edges, by digest); mismatches go to stderr
static bool snap_verify() {
  static const bool v = getenv("MQM_SNAP_VERIFY") && atoi(getenv("MQM_SNAP_VERIFY")) != 0;
  return v;
}

// MQM_SNAP_STAMP=1 (diagnostic): stamp the snapshot's version into its
// buffers as the upload's last step (snapshot.h DeviceSnapshot::stamp)
static bool snap_stamp() {
  static const bool v = getenv("MQM_SNAP_STAMP") && atoi(getenv("MQM_SNAP_STAMP")) != 0;
  return v;
}

GpuSnapshot::~GpuSnapshot() {
  // (every reader holds this snapshot until its work is done: the server
  // until it is halted, a batch until its stream is synchronised, a queued
  // context until its next call — so nothing on the device reads these now)
  if (snap_pool()) {
    const hipStream_t rs = reclaim_stream(device);
    for (auto &x : held) (void)hipFreeAsync(x.first, rs);
  } else if (snap_recycle()) {
    recycled_free(device, held);
  } else if (!held.empty()) {
    std::vector<void *> v;
    for (auto &x : held) v.push_back(x.first);
    retire_device_buffers(device, std::move(v));
  }
}


int upload(std::shared_ptr<HostSnapshot> hs, int device, hipStream_t stream, std::unique_ptr<GpuSnapshot> *out) {
  auto g = std::make_unique<GpuSnapshot>();
  if (device >= 0) {
    g->device = device;
    if (snap_pool()) (void)reclaim_stream(device);  // (creates it, sets the pool's release threshold)
  }
  auto dalloc = [&](void **p, size_t n) {
    size_t cap = n;
    const hipError_t e = snap_pool()      ? hipMallocAsync(p, n, stream)
                         : snap_recycle() ? recycled_alloc(device, p, n, &cap)
                                          : hipMalloc(p, n);
    if (e == hipSuccess) g->held.emplace_back(*p, cap);
    return e;
  };
  if (device < 0) {  // host-only index: no device copy
    g->host = std::move(hs);
    *out = std::move(g);
    return MQM_OK;
  }
  if (hipSetDevice(device) != hipSuccess) return MQM_EHIP;
  const bool ret = !hs->cum.empty();
  const void *src[GpuSnapshot::kNumBuffers] = {hs->nodes.data(),     hs->edges.data(),     hs->subs.data(),
                                               hs->tok_pool.data(),  hs->subtree.data(),   hs->child_off.data(),
                                               hs->child_ids.data(), hs->cum.data(),       hs->refs.data(),
                                               hs->rch_off.data(),   hs->rch_refs.data(),  hs->rinv.data(),
                                               hs->rgroups.data()};
  // the table is built on the device from the staged edges (flatten's
  // host_edges = false) unless the host built it
  const bool dev_edges = hs->edges.empty();
  const uint64_t n_slots = hs->n_buckets * kEdgesPerBucket;
  if (dev_edges && (!hs->staged || hs->staged->size() != hs->n_edges)) return MQM_EINVAL;
  const size_t sz[GpuSnapshot::kNumBuffers] = {
      hs->nodes.size() * sizeof(NodeDesc), n_slots * sizeof(EdgeEntry), hs->subs.size() * sizeof(SubEnt),
      hs->tok_pool.size(),                 hs->subtree.size() * 4,                hs->child_off.size() * 4,
      hs->child_ids.size() * 4,            hs->cum.size() * 4,                    hs->refs.size() * 8,
      hs->rch_off.size() * 4,              hs->rch_refs.size() * 8,               hs->rinv.size() * 8,
      hs->rgroups.size() * sizeof(RevGroup)};
  // stamps (MQM_SNAP_STAMP=1) sit 64 B past the data of nodes / subs / words
  // (walk_step reads up to 64 B past the last descriptor), 8-B aligned
  const bool stamped = snap_stamp();
  auto stamp_at = [](size_t n) { return ((n + 7) & ~size_t(7)) + 64; };
  for (int i = 0; i < GpuSnapshot::kNumBuffers; i++) {
    if (i >= 4 && !ret) break;
    // +64 B: walk_step reads 64 B at any node descriptor (the last one included)
    const size_t extra = stamped && (i == 0 || i == 2) ? stamp_at(sz[i] ? sz[i] : 16) + 8 - (sz[i] ? sz[i] : 16) : 64;
    if (dalloc(&g->buffers[i], (sz[i] ? sz[i] : 16) + extra) != hipSuccess) return MQM_ENOMEM;
    if (sz[i] && !(i == 1 && dev_edges) &&
        upload_copy(g->buffers[i], src[i], sz[i], stream) != hipSuccess)
      return MQM_EHIP;
    g->device_bytes += sz[i];
  }
  if (dev_edges) {  // edges.hip; a run-past overflow (never seen) falls back to the host build
    const uint64_t ne = hs->staged->size();
    uint64_t sum = 0;
    const int rc = build_edges_device(hs->staged->data(), ne, hs->n_buckets, (EdgeEntry *)g->buffers[1], stream, &sum);
    if (rc < 0) return MQM_EHIP;
    if (rc == 1) {
      insert_edges_host(*hs, *hs->staged);
      if (upload_copy(g->buffers[1], hs->edges.data(), sz[1], stream) != hipSuccess)
        return MQM_EHIP;
    } else {
      hs->edges_digest = edges_digest_final(sum, n_slots);
      if (snap_verify()) {  // the same table built on the host, compared slot by slot
        HostSnapshot tmp;
        tmp.n_buckets = hs->n_buckets;
        insert_edges_host(tmp, *hs->staged);
        std::vector<EdgeEntry> dev(n_slots);
        if (hipMemcpyAsync(dev.data(), g->buffers[1], n_slots * sizeof(EdgeEntry), hipMemcpyDeviceToHost, stream) !=
                hipSuccess ||
            hipStreamSynchronize(stream) != hipSuccess)
          return MQM_EHIP;
        uint64_t bad = 0, first = ~0ull;
        for (uint64_t i = 0; i < n_slots; i++)
          if (memcmp(&dev[i], &tmp.edges[i], sizeof(EdgeEntry)) != 0 && bad++ == 0) first = i;
        const uint64_t dg = edges_digest_of(tmp);
        if (bad || dg != hs->edges_digest)
          fprintf(stderr, "mqmatch verify: version %llu edge table: %llu of %llu slots differ from the host build "
                  "(first %llu), digest %s\n", (unsigned long long)hs->version, (unsigned long long)bad,
                  (unsigned long long)n_slots, (unsigned long long)first, dg == hs->edges_digest ? "equal" : "differs");
      }
    }
    hs->staged.reset();  // (the builder's FlattenCache may keep it for the next build)
  }
  // the packed delivery of every subscription entry (snapshot.h: words)
  const uint64_t n_sub_ents = hs->subs.size();
  if (dalloc(&g->words, stamped ? stamp_at(n_sub_ents * 4) + 8 : n_sub_ents * 4 + 64) != hipSuccess)
    return MQM_ENOMEM;
  if (derive_words((const SubEnt *)g->buffers[2], (uint32_t *)g->words, n_sub_ents, stream)) return MQM_EHIP;
  if (!hs->bloom.empty()) {
    const size_t bb = hs->bloom.size() * 8;
    if (dalloc(&g->bloom, bb) != hipSuccess) return MQM_ENOMEM;
    if (upload_copy(g->bloom, hs->bloom.data(), bb, stream) != hipSuccess) return MQM_EHIP;
    g->device_bytes += bb;
  }
  g->device_bytes += n_sub_ents * 4;
  {  // Identifier > 0, one bit per entry (DeviceSnapshot::ident_bits)
    const uint64_t nw = (n_sub_ents + 31) / 32;
    if (dalloc(&g->ident_bits, nw * 4 + 64) != hipSuccess) return MQM_ENOMEM;
    if (derive_ident_bits((const SubEnt *)g->buffers[2], (uint32_t *)g->ident_bits, n_sub_ents, stream))
      return MQM_EHIP;
    g->device_bytes += nw * 4;
  }
  if (slots_enabled()) {  // paired node slots (snapshot.h DeviceSnapshot::slots; MQM_SLOTS=1)
    const uint64_t nn = hs->nodes.size();
    if (dalloc(&g->slots, nn * 2 * sizeof(NodeDesc) + 64) != hipSuccess) return MQM_ENOMEM;
    if (derive_slots((const NodeDesc *)g->buffers[0], (NodeDesc *)g->slots, nn, stream)) return MQM_EHIP;
    g->device_bytes += nn * 2 * sizeof(NodeDesc);
  }
  {  // partners of the multi entries (merge by resolution)
    const size_t pb = hs->pinfo.size() * sizeof(uint2), qb = hs->partners.size() * 4;
    if (dalloc(&g->pinfo, pb + 64) != hipSuccess || dalloc(&g->partners, qb + 64) != hipSuccess)
      return MQM_ENOMEM;
    if (pb && upload_copy(g->pinfo, hs->pinfo.data(), pb, stream) != hipSuccess)
      return MQM_EHIP;
    if (qb && upload_copy(g->partners, hs->partners.data(), qb, stream) != hipSuccess)
      return MQM_EHIP;
    g->device_bytes += pb + qb;
  }
  if (ret) {  // node flags, one byte per node, for the reverse walk
    const uint64_t nn = hs->nodes.size();
    if (dalloc(&g->nflags, nn + 64) != hipSuccess) return MQM_ENOMEM;
    if (derive_node_flags((const NodeDesc *)g->buffers[0], (uint8_t *)g->nflags, nn, stream)) return MQM_EHIP;
    g->device_bytes += nn;
  }
  if (snap_verify()) {  // the uploaded and derived arrays, read back
    if (hipStreamSynchronize(stream) != hipSuccess) return MQM_EHIP;
    auto check = [&](const char *what, const void *dptr, const void *host, size_t n) {
      if (!n) return;
      std::vector<uint8_t> b(n);
      if (hipMemcpy(b.data(), dptr, n, hipMemcpyDeviceToHost) != hipSuccess) return;
      if (memcmp(b.data(), host, n) != 0) {
        size_t k = 0;
        while (k < n && b[k] == ((const uint8_t *)host)[k]) k++;
        fprintf(stderr, "mqmatch verify: version %llu %s differs from the host array at byte %zu of %zu\n",
                (unsigned long long)hs->version, what, k, n);
      }
    };
    check("nodes", g->buffers[0], hs->nodes.data(), hs->nodes.size() * sizeof(NodeDesc));
    check("subs", g->buffers[2], hs->subs.data(), hs->subs.size() * sizeof(SubEnt));
    check("tok_pool", g->buffers[3], hs->tok_pool.data(), hs->tok_pool.size());
    if (!hs->bloom.empty()) check("bloom", g->bloom, hs->bloom.data(), hs->bloom.size() * 8);
    check("pinfo", g->pinfo, hs->pinfo.data(), hs->pinfo.size() * sizeof(uint2));
    check("partners", g->partners, hs->partners.data(), hs->partners.size() * 4);
    {
      std::vector<uint32_t> w(n_sub_ents);
      for (uint64_t i = 0; i < n_sub_ents; i++) w[i] = hs->subs[i].word & kPackedMask;
      check("words", g->words, w.data(), n_sub_ents * 4);
    }
  }
  if (stamped) {  // last: every buffer above is complete on the stream before its stamp
    void *own = nullptr;
    if (dalloc(&own, 64) != hipSuccess) return MQM_ENOMEM;
    g->stamp_host = hs->version;
    unsigned long long *at[4] = {
        (unsigned long long *)((char *)g->buffers[0] + stamp_at(sz[0] ? sz[0] : 16)),
        (unsigned long long *)((char *)g->buffers[2] + stamp_at(sz[2] ? sz[2] : 16)),
        (unsigned long long *)((char *)g->words + stamp_at(n_sub_ents * 4)), (unsigned long long *)own};
    for (int i = 0; i < 4; i++) {
      if (hipMemcpyAsync(at[i], &g->stamp_host, 8, hipMemcpyHostToDevice, stream) != hipSuccess) return MQM_EHIP;
      g->dev.stamp[i] = at[i];
    }
  }
  g->dev.version = hs->version;
  if (hipStreamSynchronize(stream) != hipSuccess) return MQM_EHIP;
  // the device holds the edge table now: keep its digest, release the host copy
  if (!hs->edges.empty()) {
    hs->edges_digest = edges_digest_of(*hs);
    decltype(hs->edges)().swap(hs->edges);
  }
  if (ret) {
    g->has_retained = true;
    g->ret.nflags = (const uint8_t *)g->nflags;
    g->ret.subtree = (const uint32_t *)g->buffers[4];
    g->ret.child_off = (const uint32_t *)g->buffers[5];
    g->ret.child_ids = (const uint32_t *)g->buffers[6];
    g->ret.cum = (const uint32_t *)g->buffers[7];
    g->ret.refs = (const uint64_t *)g->buffers[8];
    g->ret.rch_off = (const uint32_t *)g->buffers[9];
    g->ret.rch_refs = (const uint64_t *)g->buffers[10];
    g->ret.inv = (const uint2 *)g->buffers[11];
    g->ret.groups = (const RevGroup *)g->buffers[12];
    g->ret.n_gslots = hs->rgroups.size();
    g->ret.n_ret = hs->refs.size() - 1;
    g->ret.n_nodes = (uint32_t)hs->nodes.size();
    g->ret.sys_child = hs->sys_child;
    g->ret.has_empty = hs->has_empty ? 1u : 0u;
  }
  g->dev.nodes = (const NodeDesc *)g->buffers[0];
  g->dev.slots = (const NodeDesc *)g->slots;
  g->dev.edges = (const EdgeEntry *)g->buffers[1];
  g->dev.subs = (const SubEnt *)g->buffers[2];
  g->dev.words = (const uint32_t *)g->words;
  g->dev.ident_bits = (const uint32_t *)g->ident_bits;
  g->dev.pinfo = (const uint2 *)g->pinfo;
  g->dev.partners = (const uint32_t *)g->partners;
  g->dev.bloom = (const uint64_t *)g->bloom;
  g->dev.bloom_mask = g->bloom ? hs->bloom.size() - 1 : 0;
  g->dev.tok_pool = (const uint8_t *)g->buffers[3];
  g->dev.n_buckets = hs->n_buckets;
  g->dev.n_nodes = (uint32_t)hs->nodes.size();
  g->dev.n_subs = (uint32_t)hs->sub_info.size();
  g->dev.n_shared = (uint32_t)hs->shared_info.size();
  g->dev.height = hs->height;
  g->host = std::move(hs);
  *out = std::move(g);
  return MQM_OK;
}

}  // namespace mqm
