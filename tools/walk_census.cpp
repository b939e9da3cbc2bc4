// tools/walk_census.cpp — what the batch walk (match.hip k_walk) loads per
// topic, counted on the host over the real snapshot layout (analysis tooling,
// not product code).  Generates an mqgen workload, builds the store and the
// snapshot exactly as the library does (store.cpp, flatten.cpp), then replays
// the walk's level-synchronous item lists for a sample of topics and counts
// the loads by kind: literal probes (after the edge filter), '+' child
// descriptors, '#' child descriptors — and how many '+' children are leaves
// whose whole gather fits in the parent (no children, no shared or multi
// entries, no heavy flag): the loads a "'+' leaf folded into its parent"
// layout would not issue.
//
// build: make -C tools census     run: tools/_build/walk_census [config] [filters] [topics]
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../maxmq_amd/csrc/flatten.h"
#include "../maxmq_amd/csrc/keys.h"
#include "../maxmq_amd/csrc/store.h"
#include "mqgen.h"

using namespace mqm;

namespace {

const EdgeEntry *probe(const HostSnapshot &hs, uint32_t parent, const Key &k) {
  const uint64_t nslots = hs.n_buckets * kEdgesPerBucket;
  uint64_t slot = bucket_of(edge_hash(parent, k), hs.n_buckets) * kEdgesPerBucket;
  for (;;) {
    const EdgeEntry &e = hs.edges[slot];
    if (e.parent == kNone) return nullptr;
    if (e.parent == parent && e.k0 == k.k0 && e.k1 == k.k1) return &e;  // (long keys: hash match suffices here)
    slot = slot + 1 == nslots ? 0 : slot + 1;
  }
}

bool bloom_pass(const HostSnapshot &hs, uint32_t parent, const Key &k) {
  if (hs.bloom.empty()) return true;
  const uint64_t h = edge_hash(parent, k);
  const uint64_t w = hs.bloom[bloom_word(h, hs.bloom.size() - 1)], b = bloom_bits(h);
  return (w & b) == b;
}

}  // namespace

int main(int argc, char **argv) {
  const int config = argc > 1 ? atoi(argv[1]) : 3;
  mqgen_params p;
  mqgen_default_params(config, &p);
  if (argc > 2) p.n_filters = strtoull(argv[2], nullptr, 10);
  if (argc > 3) p.n_topics = strtoull(argv[3], nullptr, 10);
  mqgen_workload w;
  if (mqgen_generate(&p, &w) != 0) return 1;
  Store st;
  for (uint64_t i = 0; i < w.filters.n; i++) {
    const std::string_view c(w.clients.bytes + w.clients.offs[i], w.clients.offs[i + 1] - w.clients.offs[i]);
    const std::string_view f(w.filters.bytes + w.filters.offs[i], w.filters.offs[i + 1] - w.filters.offs[i]);
    st.subscribe(c, f, w.qos[i], w.no_local[i], w.rap[i], w.rh[i], w.ident[i]);
  }
  HostSnapshot hs;
  if (flatten(st, &hs) != 0) return 2;
  uint64_t n_lit = 0, n_plus = 0, n_plus_leaf = 0, n_plus_leaf_empty = 0, n_hash = 0, n_topics = 0;
  uint64_t n_lit_filtered = 0;
  uint64_t part_hist[8] = {}, entry_hist[8] = {};  // solo parts by length: count, entries
  uint64_t n_plus_after_wild = 0, n_plus_after_root = 0;  // '+' items pushed by a node reached through '+' / '#'
  uint64_t n_plus_free = 0;  // paired slots: '+' items whose descriptor came with the parent's slot
  const bool slots = getenv("CENSUS_SLOTS") != nullptr;
  std::vector<uint32_t> cur, nxt;  // item: id << 2 | kind (0 literal probe of id, 1 '+' node id, 2 '#' node id)
  for (uint64_t t = 0; t < w.topics.n; t++) {
    const char *tb = w.topics.bytes + w.topics.offs[t];
    const uint32_t len = (uint32_t)(w.topics.offs[t + 1] - w.topics.offs[t]);
    std::vector<Key> keys;
    uint32_t st0 = 0;
    for (uint32_t i = 0; i <= len; i++)
      if (i == len || tb[i] == '/') {
        keys.push_back(make_key([&](uint32_t j) { return (uint8_t)tb[st0 + j]; }, i - st0));
        st0 = i + 1;
      }
    if (len == 0) continue;
    n_topics++;
    const NodeDesc &root = hs.nodes[0];
    cur.clear();
    if ((root.sh_cnt_flags >> 24) & kFlagHasLiteral) cur.push_back(0u << 2 | 0);
    if (root.plus != kNone) cur.push_back(root.plus << 2 | 1);
    if (root.hash != kNone) cur.push_back(root.hash << 2 | 2);
    for (size_t d = 0; d < keys.size() && !cur.empty() && d < 16; d++) {
      const bool has_next = d + 1 < keys.size();
      nxt.clear();
      for (uint32_t it : cur) {
        const uint32_t kind = it & 3, id = it >> 2;
        NodeDesc dc;
        uint32_t c;
        if (kind == 0) {
          n_lit++;
          const EdgeEntry *e = probe(hs, id, keys[d]);
          if (!e) continue;
          c = e->child;
          dc = e->desc;
        } else {
          if (kind == 3) n_plus_free++;
          if (kind == 1) {
            n_plus++;
            const NodeDesc &pd = hs.nodes[id];
            const uint32_t fl = pd.sh_cnt_flags >> 24;
            if (!(fl & kFlagHasChildren) && (pd.sh_cnt_flags & kShCntMask) == 0 && (pd.multi & 0xFFFFu) == 0 &&
                !(fl & kFlagHeavyOwn)) {
              n_plus_leaf++;
              if (pd.sub_cnt == 0) n_plus_leaf_empty++;
            }
          } else {
            n_hash++;
          }
          c = id;
          dc = hs.nodes[id];
        }
        const uint32_t fl = dc.sh_cnt_flags >> 24;
        {  // the solo part this visit gathers (approximate: the '#' double-gather rules aside)
          const uint32_t solo = dc.sub_cnt - std::min<uint32_t>(dc.sub_cnt, dc.multi & 0xFFFFu);
          if (solo && !(kind == 2 && (fl & kFlagParentLit))) {
            int b = 0;
            while (b < 7 && solo >= (16u << (2 * b))) b++;  // <16, <64, <256, <1K, <4K, <16K, <64K, more
            part_hist[b]++;
            entry_hist[b] += solo;
          }
          // the '#' child's range: the next level's '#' probe when the topic
          // continues, else the parent-'#' probe after a literal (topics.go:503-509)
          if (dc.hash != kNone && (has_next || kind == 0)) {
            const uint32_t hs_solo = dc.hsub_cnt - std::min<uint32_t>(dc.hsub_cnt, dc.multi >> 16);
            if (hs_solo) {
              int b = 0;
              while (b < 7 && hs_solo >= (16u << (2 * b))) b++;
              part_hist[b]++;
              entry_hist[b] += hs_solo;
            }
          }
        }
        if (!(has_next && (fl & kFlagHasChildren))) continue;
        if ((fl & kFlagHasLiteral) && d + 1 < 16) {
          if (bloom_pass(hs, c, keys[d + 1]))
            nxt.push_back(c << 2 | 0);
          else
            n_lit_filtered++;
        }
        if (dc.plus != kNone) {
          // paired node slots: a node LOADED from the node array (kind 1 or 2)
          // brings its '+' child's descriptor in the same 64-B slot -> kind 3 (free)
          const bool free_plus = slots && (kind == 1 || kind == 2);
          nxt.push_back(dc.plus << 2 | (free_plus ? 3u : 1u));
          if (kind != 0) n_plus_after_wild++;  // parent's descriptor came from a node load, not an edge probe
          else if (it == (0u << 2 | 0) && d == 0) n_plus_after_root++;
        }
        if (dc.hash != kNone && !(fl & kFlagHashLeaf)) nxt.push_back(dc.hash << 2 | 2);
      }
      std::swap(cur, nxt);
    }
  }
  const double n = (double)n_topics;
  printf("{\"config\": %d, \"filters\": %llu, \"topics\": %llu, \"nodes\": %zu, \"per_topic\": {\"literal_probes\": %.3f, "
         "\"filtered_probes\": %.3f, \"plus_loads\": %.3f, \"plus_leaf_foldable\": %.3f, \"plus_leaf_empty\": %.3f, "
         "\"hash_loads\": %.3f}}\n",
         config, (unsigned long long)p.n_filters, (unsigned long long)n_topics, hs.nodes.size(), n_lit / n,
         n_lit_filtered / n, n_plus / n, n_plus_leaf / n, n_plus_leaf_empty / n, n_hash / n);
  printf("'+' items pushed by a node whose descriptor came from a '+'/'#' node load: %.3f per topic\n",
         n_plus_after_wild / n);
  if (slots) printf("paired slots: '+' loads %.3f + free '+' items %.3f per topic\n", n_plus / n, n_plus_free / n);
  const char *bn[8] = {"<16", "<64", "<256", "<1K", "<4K", "<16K", "<64K", ">=64K"};
  uint64_t te = 0;
  for (int b = 0; b < 8; b++) te += entry_hist[b];
  printf("solo parts by length (per topic: parts, entries, share of entries)\n");
  for (int b = 0; b < 8; b++)
    printf("  %-6s %8.3f %10.2f %6.3f\n", bn[b], part_hist[b] / n, entry_hist[b] / n, te ? (double)entry_hist[b] / te : 0.0);
  mqgen_free(&w);
  return 0;
}
