// tests/harness/fresh_test.cpp — the fresh overlay (maxmq_amd/csrc/fresh.h) on
// the CPU, against the C oracle (oracle/mochi_ref.c), under sanitizers.
// Test infrastructure: built by tests/harness/Makefile twice (ASan+UBSan and
// TSan, the overlay's and the store's sources compiled in), run by
// tests/test_capi_host.py without a GPU.
//
// The overlay is driven exactly as capi.cpp drives it (mutation hooks under
// one mutating thread, snapshots published late as the background builder
// does, mqm_fresh_policy off and on, now and then a snapshot without the
// by-client index), with snapshots built here from the
// store's own lists (HostSnapshot's sub_info / shared_info and the by-client
// index; no device, no flatten).  Checked, for every call:
//   * status: -1 below the floor (the snapshot before the published one), 0
//     when nothing is newer or the overlay has not started (no snapshot yet,
//     or on again and no snapshot with every mutation made while off), else 1;
//   * touched(c, vs) == "c's last mutation is newer than vs" for every client;
//   * the corrected rows: for every touched client, the oracle's current
//     delivery (client, QoS max, NoLocal or, first-merged filter, Identifier,
//     RetainAsPublished, RetainHandling: topics.go:493-538, packets.go:250-270),
//     its Identifiers and its shared candidates; nothing for any other client.
// Phase 1 checks every call single-threaded.  Phase 2 runs 4 reader threads
// (Reader, status, match, touched) against the mutating thread and the
// applier, then checks the quiescent overlay as phase 1 does — the left-right
// copies must have lost no operation.
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <random>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "../../maxmq_amd/csrc/fresh.h"
#include "../../oracle/mochi_ref.h"

using namespace mqm;

namespace {

std::atomic<int> failures{0};
#define CHECK(cond, ...)                                \
  do {                                                  \
    if (!(cond)) {                                      \
      if (failures++ < 20) {                            \
        fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
        fprintf(stderr, __VA_ARGS__);                   \
        fputc('\n', stderr);                            \
      }                                                 \
    }                                                   \
  } while (0)

// the snapshot of the store as it is now (what flatten + build_client_index
// give the overlay: sub_info / shared_info and their by-client index)
std::shared_ptr<HostSnapshot> snapshot_of(const Store &st) {
  auto hs = std::make_shared<HostSnapshot>();
  const auto &nodes = st.nodes();
  for (size_t i = 0; i < nodes.size(); i++) {
    const HNode &n = nodes[i];
    if (!n.live) continue;
    for (const SubRec &r : n.subs) hs->sub_info.push_back(SubInfo{r.filter, r.client, r.ident, r.qos, r.no_local, r.rap, r.rh});
    for (const SharedRec &s : n.shared)
      hs->shared_info.push_back(SubInfo{s.sub.filter, s.sub.client, s.sub.ident, s.sub.qos, s.sub.no_local, s.sub.rap, s.sub.rh});
  }
  const uint32_t nc = st.clients().size();
  auto by_client = [nc](const std::vector<SubInfo> &info, std::vector<uint32_t> &off, std::vector<uint32_t> &ids) {
    off.assign(nc + 1, 0);
    for (const SubInfo &s : info) off[s.client + 1]++;
    for (uint32_t c = 0; c < nc; c++) off[c + 1] += off[c];
    std::vector<uint32_t> cur(off.begin(), off.end() - 1);
    ids.resize(info.size());
    for (uint32_t k = 0; k < info.size(); k++) ids[cur[info[k].client]++] = k;
  };
  by_client(hs->sub_info, hs->client_off, hs->client_subs);
  by_client(hs->shared_info, hs->client_shoff, hs->client_shared);
  hs->nodes.resize(nodes.size());
  hs->version = st.version();
  return hs;
}

// one delivery or shared candidate, by names (the oracle interns its own ids)
using Row = std::tuple<std::string, std::string, int, int, int, int, int>;  // client, filter, qos, nl, ident, rap, rh
using Cand = std::tuple<std::string, std::string, int>;                     // filter, client, qos

struct World {
  Store st;
  oref *orc = oref_new();
  std::unique_ptr<FreshOverlay> ov = std::make_unique<FreshOverlay>();
  std::mt19937_64 rng;
  std::vector<uint64_t> lastmut;  // by store client id: the version after its last mutation
  std::shared_ptr<HostSnapshot> published, previous, pending;
  bool enabled = true, active = false;
  uint64_t floor = 0;  // what the overlay must report (phase 1 checks)
  uint64_t wait = 0;   // a snapshot that starts the overlay has this version or newer
  std::shared_ptr<HostSnapshot> base;  // the snapshot the overlay started from / last took
  int n_clients = 12;

  explicit World(uint64_t seed) : rng(seed) {}
  ~World() {
    ov.reset();
    oref_free(orc);
  }
  int pick(int n) { return (int)(rng() % (uint64_t)n); }
  std::string level(bool filter) {
    static const char *lv[] = {"a", "b", "c", "$SYS", "", "+"};
    return lv[pick(filter ? 6 : 5)];
  }
  std::string topic() {
    std::string t = level(false);
    for (int d = pick(4); d > 0; d--) t += "/" + level(false);
    return t;
  }
  std::string filter() {
    std::string f = level(true);
    for (int d = pick(4); d > 0; d--) f += "/" + level(true);
    if (pick(5) == 0) f += "/#";
    if (pick(7) == 0) f = "#";
    if (pick(7) == 0) f = std::string("$SHARE/g") + char('0' + pick(2)) + "/" + f;
    return f;
  }
  void stamp(uint32_t c) {
    if (c >= lastmut.size()) lastmut.resize(c + 1, 0);
    lastmut[c] = st.version();
  }
  // one Subscribe or Unsubscribe, hooked as capi.cpp hooks it (mqm_subscribe,
  // mqm_unsubscribe)
  void mutate() {
    const std::string c = "k" + std::to_string(pick(n_clients)), f = filter();
    if (pick(10) < 6) {
      const uint8_t qos = pick(3), nl = pick(2), rap = pick(2), rh = pick(3);
      const int32_t ident = pick(3) == 0 ? 0 : 1 + pick(9);
      const bool r1 = st.subscribe(c, f, qos, nl, rap, rh, ident);
      const int r2 = oref_subscribe(orc, c.data(), c.size(), f.data(), f.size(), qos, nl, rap, rh, ident);
      CHECK(r1 == (r2 != 0), "subscribe %s %s: store %d oracle %d", c.c_str(), f.c_str(), r1, r2);
      const Store::Footprint &fp = st.last_footprint();
      ov->on_subscribe(st, f, SubRec{fp.client, fp.filter, ident, qos, nl, rap, rh});
      stamp(fp.client);
    } else {
      const bool r1 = st.unsubscribe(f, c);
      const int r2 = oref_unsubscribe(orc, f.data(), f.size(), c.data(), c.size());
      CHECK(r1 == (r2 != 0), "unsubscribe %s %s: store %d oracle %d", c.c_str(), f.c_str(), r1, r2);
      if (r1) {
        ov->on_unsubscribe(st, f);
        if (st.last_footprint().client != 0xFFFFFFFFu) stamp(st.last_footprint().client);
      }
    }
  }
  // the background builder: a snapshot taken now, published a few mutations
  // later (capi.cpp install -> FreshOverlay::on_install)
  void publish_step() {
    if (!pending && pick(12) == 0) {
      pending = snapshot_of(st);
      // (now and then one without the by-client index: the overlay stops, and
      // starts again at the next snapshot that has one)
      if (pick(15) == 0 && !pending->sub_info.empty()) pending->client_off.clear();
    }
    if (pending && pick(6) == 0) {
      previous = published;
      published = std::move(pending);
      if (enabled) {
        offer(published);
        ov->on_install(published, st);
      }
    }
  }
  // what on_install(hs) must do: start the overlay (floor = hs), move the
  // floor to the snapshot it took before, or nothing (hs older than wait)
  void offer(const std::shared_ptr<HostSnapshot> &hs) {
    if (hs->client_off.empty() && !hs->sub_info.empty()) {
      active = false;
      base = nullptr;
      return;
    }
    if (!active) {
      if (hs->version < wait) return;
      active = true;
      floor = hs->version;
    } else {
      floor = base->version;
    }
    base = hs;
  }
  // mqm_fresh_policy (rare)
  void policy_step() {
    if (pick(400) != 0) return;
    enabled = !enabled;
    if (!enabled) {
      active = false;
      ov->set_enabled(false, nullptr, st);
    } else if (published) {
      wait = st.version();
      offer(published);
      ov->set_enabled(true, published, st);
    } else {
      wait = st.version();
      ov->set_enabled(true, nullptr, st);
    }
  }

  // the oracle's deliveries and shared candidates for one topic, by names
  void oracle(const std::string &t, std::map<std::string, Row> *rows, std::vector<Cand> *cands) {
    uint64_t offs[2] = {0, t.size()};
    uint32_t dc = 0, sc = 0;
    oref_stats stats;
    oref_match_counts(orc, t.data(), offs, 1, 1, &dc, &sc, &stats);
    std::vector<oref_delivery> d(dc + 1);
    std::vector<oref_shared> s(sc + 1);
    uint64_t doff[2] = {0, dc}, soff[2] = {0, sc};
    oref_match_fill(orc, t.data(), offs, 1, 1, doff, d.data(), soff, s.data());
    char a[512], b[512];
    for (uint32_t i = 0; i < dc; i++) {
      const uint32_t la = oref_client_name(orc, d[i].client, a, sizeof a);
      const uint32_t lb = oref_filter_name(orc, d[i].first_filter, b, sizeof b);
      (*rows)[std::string(a, la)] = Row{std::string(a, la), std::string(b, lb), d[i].qos, d[i].no_local,
                                        d[i].first_ident, d[i].rap, d[i].rh};
    }
    for (uint32_t i = 0; i < sc; i++) {
      const uint32_t la = oref_client_name(orc, s[i].client, a, sizeof a);
      const uint32_t lb = oref_filter_name(orc, s[i].filter, b, sizeof b);
      cands->push_back(Cand{std::string(b, lb), std::string(a, la), s[i].qos});
    }
  }

  // one call on snapshot version vs, checked (the calling thread's writes applied)
  void check(const std::string &t, uint64_t vs) {
    ov->await_own_writes();
    FreshOverlay::Match m;
    int status;
    std::vector<uint8_t> touched(st.clients().size(), 0);
    {
      FreshOverlay::Reader rd(*ov);
      status = rd.status(vs);
      if (status == 1) {
        rd.match(t, vs, &m);
        for (uint32_t c = 0; c < touched.size(); c++) touched[c] = rd.touched(c, vs);
      }
    }
    int want = 0;
    if (active) want = vs < floor ? -1 : st.version() > vs ? 1 : 0;
    CHECK(status == want, "topic '%s' vs %llu: status %d, want %d (floor %llu version %llu active %d)", t.c_str(),
          (unsigned long long)vs, status, want, (unsigned long long)floor, (unsigned long long)st.version(),
          (int)active);
    if (status != 1 || want != 1) return;
    CHECK(m.version == st.version(), "match version %llu, store %llu", (unsigned long long)m.version,
          (unsigned long long)st.version());
    for (uint32_t c = 0; c < touched.size(); c++) {
      const bool w = c < lastmut.size() && lastmut[c] > vs;
      CHECK((bool)touched[c] == w, "client %u touched %d, want %d (vs %llu)", c, touched[c], (int)w,
            (unsigned long long)vs);
    }
    std::map<std::string, Row> want_rows, got_rows;
    std::vector<Cand> want_c, got_c;
    oracle(t, &want_rows, &want_c);
    for (const auto &r : m.rows) {
      const std::string cn(st.clients().name(r.client));
      CHECK(r.client < touched.size() && touched[r.client], "row of untouched client %s", cn.c_str());
      CHECK(r.first < m.subs.size() && m.subs[r.first].client == r.client, "row %s: bad first", cn.c_str());
      if (r.first >= m.subs.size()) continue;
      const SubInfo &si = m.subs[r.first].info;
      CHECK(!got_rows.count(cn), "client %s twice", cn.c_str());
      got_rows[cn] = Row{cn, std::string(st.filters().name(si.filter)), r.qos, r.no_local, si.ident, si.rap, si.rh};
    }
    for (const auto &kv : want_rows) {
      const uint32_t c = st.clients().find(kv.first);
      if (c != 0xFFFFFFFFu && c < touched.size() && touched[c]) {
        auto it = got_rows.find(kv.first);
        if (it != got_rows.end() && !(it->second == kv.second) && failures.load() < 6) {
          const Row &x = kv.second, &y = it->second;
          fprintf(stderr, "  want %s %s q%d nl%d id%d rap%d rh%d / got %s q%d nl%d id%d rap%d rh%d\n", std::get<0>(x).c_str(),
                  std::get<1>(x).c_str(), std::get<2>(x), std::get<3>(x), std::get<4>(x), std::get<5>(x), std::get<6>(x),
                  std::get<1>(y).c_str(), std::get<2>(y), std::get<3>(y), std::get<4>(y), std::get<5>(y), std::get<6>(y));
        }
        CHECK(it != got_rows.end() && it->second == kv.second, "topic '%s' vs %llu client %s: row %s", t.c_str(),
              (unsigned long long)vs, kv.first.c_str(), it == got_rows.end() ? "missing" : "differs");
      }
    }
    for (const auto &kv : got_rows)
      CHECK(want_rows.count(kv.first), "topic '%s': client %s matched by the overlay, not by the oracle", t.c_str(),
            kv.first.c_str());
    for (const SubInfo &si : m.shared) {
      CHECK(si.client < touched.size() && touched[si.client], "shared candidate of an untouched client");
      got_c.push_back(Cand{std::string(st.filters().name(si.filter)), std::string(st.clients().name(si.client)), si.qos});
    }
    std::vector<Cand> keep;
    for (const Cand &c : want_c) {
      const uint32_t id = st.clients().find(std::get<1>(c));
      if (id != 0xFFFFFFFFu && id < touched.size() && touched[id]) keep.push_back(c);
    }
    std::sort(keep.begin(), keep.end());
    std::sort(got_c.begin(), got_c.end());
    CHECK(keep == got_c, "topic '%s' vs %llu: shared candidates %zu, want %zu", t.c_str(), (unsigned long long)vs,
          got_c.size(), keep.size());
    if (keep != got_c && failures.load() < 4) {
      for (const Cand &c : keep) fprintf(stderr, "  want %s %s %d\n", std::get<0>(c).c_str(), std::get<1>(c).c_str(), std::get<2>(c));
      for (const Cand &c : got_c) fprintf(stderr, "  got  %s %s %d\n", std::get<0>(c).c_str(), std::get<1>(c).c_str(), std::get<2>(c));
    }
    // Subscription.Identifiers of the touched clients' deliveries
    // (packets.go:250-258): {first.Filter: first.Identifier} and every other
    // gathered subscription with an Identifier > 0 — capi.cpp freshen lists
    // the gathered entries with one, the first comes with its row
    using Ident = std::tuple<std::string, std::string, int>;  // client, filter, ident
    std::vector<Ident> want_i, got_i;
    {
      uint64_t offs[2] = {0, t.size()};
      uint32_t ic = 0;
      oref_match_ident_counts(orc, t.data(), offs, 1, 1, &ic);
      std::vector<oref_ident> iv(ic + 1);
      uint64_t ioff[2] = {0, ic};
      oref_match_ident_fill(orc, t.data(), offs, 1, 1, ioff, iv.data());
      char a[512], b[512];
      for (uint32_t i = 0; i < ic; i++) {
        const std::string cn(a, oref_client_name(orc, iv[i].client, a, sizeof a));
        const uint32_t id = st.clients().find(cn);
        if (id == 0xFFFFFFFFu || id >= touched.size() || !touched[id]) continue;
        want_i.push_back(Ident{cn, std::string(b, oref_filter_name(orc, iv[i].filter, b, sizeof b)), iv[i].ident});
      }
    }
    auto ident_of = [&](const FreshOverlay::Gathered &g) {
      return Ident{std::string(st.clients().name(g.client)), std::string(st.filters().name(g.info.filter)), g.info.ident};
    };
    for (const auto &r : m.rows)
      if (r.first < m.subs.size()) got_i.push_back(ident_of(m.subs[r.first]));
    for (const auto &g : m.subs)
      if (g.info.ident > 0) got_i.push_back(ident_of(g));
    std::sort(want_i.begin(), want_i.end());
    std::sort(got_i.begin(), got_i.end());
    got_i.erase(std::unique(got_i.begin(), got_i.end()), got_i.end());
    CHECK(want_i == got_i, "topic '%s' vs %llu: identifiers %zu, want %zu", t.c_str(), (unsigned long long)vs,
          got_i.size(), want_i.size());
  }
  void check_round() {
    for (int k = 0; k < 3; k++) {
      const std::string t = topic();
      if (published) check(t, published->version);
      if (previous) check(t, previous->version);
    }
  }
};

// phase 1: every call checked, single-threaded
void phase1(uint64_t seed, int steps) {
  World w(seed);
  for (int i = 0; i < 40; i++) w.mutate();
  w.published = snapshot_of(w.st);  // (the first commit, synchronous)
  w.offer(w.published);
  w.ov->on_install(w.published, w.st);
  for (int i = 0; i < steps; i++) {
    w.mutate();
    w.publish_step();
    w.policy_step();
    w.check_round();
  }
}

// phase 1b: the first snapshot published late (async first commit): the
// clients mutated since it was built are loaded from the store at the start
void phase1_late_first(uint64_t seed) {
  World w(seed);
  for (int i = 0; i < 30; i++) w.mutate();
  auto first = snapshot_of(w.st);
  for (int i = 0; i < 30; i++) w.mutate();  // not followed: no snapshot yet
  w.published = first;
  w.offer(first);
  w.ov->on_install(first, w.st);
  for (int i = 0; i < 400; i++) {
    w.mutate();
    w.publish_step();
    w.check_round();
  }
}

// phase 2: readers against the mutating thread and the applier, then the
// quiescent overlay checked
void phase2(uint64_t seed, int steps) {
  World w(seed);
  w.n_clients = 64;
  for (int i = 0; i < 200; i++) w.mutate();
  w.published = snapshot_of(w.st);
  w.offer(w.published);
  w.ov->on_install(w.published, w.st);
  std::atomic<bool> stop{false};
  std::atomic<uint64_t> pub_version{w.published->version}, reads{0};
  std::vector<std::thread> readers;
  for (int r = 0; r < 4; r++)
    readers.emplace_back([&, r] {
      std::mt19937_64 rng(seed * 131 + r);
      static const char *tp[] = {"a", "a/b", "b/c/a", "$SYS/a", "a//c", "c/c/c/c", "", "b"};
      FreshOverlay::Match m;
      while (!stop.load(std::memory_order_acquire)) {
        const uint64_t vs = pub_version.load(std::memory_order_acquire);
        const char *t = tp[rng() % 8];
        w.ov->await_own_writes();
        FreshOverlay::Reader rd(*w.ov);
        if (rd.status(vs) == 1) {
          m.rows.clear();
          m.subs.clear();
          m.shared.clear();
          rd.match(t, vs, &m);
          for (const auto &row : m.rows) CHECK(rd.touched(row.client, vs), "row of an untouched client (reader %d)", r);
        }
        reads.fetch_add(1, std::memory_order_relaxed);
      }
    });
  std::thread mut([&] {
    for (int i = 0; i < steps; i++) {
      w.mutate();
      w.publish_step();
      if (w.published) pub_version.store(w.published->version, std::memory_order_release);
    }
    w.ov->await_own_writes();
  });
  mut.join();
  stop.store(true, std::memory_order_release);
  for (auto &t : readers) t.join();
  // quiescent: every operation applied (the mutator's own wait is bounded)
  CHECK(w.ov->await_all(20000), "the applier did not catch up");
  for (int k = 0; k < 200; k++) {
    const std::string t = w.topic();
    if (w.published) w.check(t, w.published->version);
    if (w.previous) w.check(t, w.previous->version);
  }
  const FreshOverlay::Stats s = w.ov->stats();
  printf("phase2 seed %llu: %llu reads, %llu ops, %llu rounds\n", (unsigned long long)seed,
         (unsigned long long)reads.load(), (unsigned long long)s.ops, (unsigned long long)s.rounds);
}

}  // namespace

int main(int argc, char **argv) {
  const int steps = argc > 1 ? atoi(argv[1]) : 3000;
  for (uint64_t seed = 1; seed <= 3; seed++) phase1(seed, steps);
  phase1_late_first(11);
  for (uint64_t seed = 21; seed <= 22; seed++) phase2(seed, 4 * steps);
  if (failures) {
    fprintf(stderr, "%d failures\n", failures.load());
    return 1;
  }
  printf("fresh_test ok\n");
  return 0;
}
