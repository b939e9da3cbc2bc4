// tools/mqgen.cpp — deterministic synthetic MQTT workload generator.
// Bench/test infrastructure (see mqgen.h); never linked into libmqmatch.
#include "mqgen.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() {  // splitmix64
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double uniform() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
  uint64_t below(uint64_t n) { return n ? (uint64_t)(uniform() * (double)n) % n : 0; }
};

uint64_t mix(uint64_t a, uint64_t b) {
  uint64_t z = a * 0x9E3779B97F4A7C15ull ^ (b + 0x632BE59BD9B4E019ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// inverse-CDF Zipf sampler over ranks 0..n-1
struct Zipf {
  std::vector<double> cdf;
  Zipf() = default;
  Zipf(uint64_t n, double s) {
    cdf.resize(n);
    double acc = 0;
    for (uint64_t k = 0; k < n; k++) {
      acc += 1.0 / std::pow((double)(k + 1), s);
      cdf[k] = acc;
    }
    for (auto &c : cdf) c /= acc;
  }
  uint64_t draw(Rng &r) const {
    double u = r.uniform();
    auto it = std::lower_bound(cdf.begin(), cdf.end(), u);
    uint64_t k = (uint64_t)(it - cdf.begin());
    return k < cdf.size() ? k : cdf.size() - 1;
  }
};

struct Vocab {
  std::vector<std::vector<std::string>> tok;  // per depth
  std::vector<Zipf> z;
};

std::string make_token(uint64_t seed, uint32_t d, uint64_t k) {
  static const char *digits = "0123456789abcdefghijklmnopqrstuvwxyz";
  uint64_t h = mix(seed ^ ((uint64_t)d << 40), k);
  uint32_t len = 3 + (uint32_t)(h % 8);
  std::string s;
  uint64_t x = mix(h, 0x5EED);
  for (uint32_t i = 0; i < len; i++) {
    s.push_back(digits[x % 36]);
    x /= 36;
    if (x == 0) x = mix(h, i + 1);
  }
  // never emit a token that collides with the wildcard/sys words
  if (d == 0 && (s == "$SYS" || s == "$share" || s == "$SHARE")) s += "x";
  return s;
}

struct Builder {
  std::vector<char> bytes;
  std::vector<uint64_t> offs{0};
  void push(const std::string &s) {
    bytes.insert(bytes.end(), s.begin(), s.end());
    offs.push_back(bytes.size());
  }
  void emit(mqgen_strings *o) {
    o->n = offs.size() - 1;
    o->bytes = (char *)malloc(bytes.size() ? bytes.size() : 1);
    if (!bytes.empty()) memcpy(o->bytes, bytes.data(), bytes.size());
    o->offs = (uint64_t *)malloc(sizeof(uint64_t) * offs.size());
    memcpy(o->offs, offs.data(), sizeof(uint64_t) * offs.size());
  }
};

}  // namespace

extern "C" void mqgen_default_params(int config, mqgen_params *p) {
  memset(p, 0, sizeof(*p));
  p->seed = 0x4D510000ull + (uint64_t)config;
  p->p_shared = 0.0;
  p->p_dollar_topic = 0.01;
  p->p_instantiate = 0.5;
  p->token_zipf_s = 1.0;
  p->topic_zipf_s = 0.0;
  const uint32_t v[8] = {64, 1024, 4096, 8192, 8192, 8192, 8192, 8192};
  for (int i = 0; i < 8; i++) p->vocab[i] = v[i];
  // filter depth weights: deep filters dominate (MQTT device/tenant trees);
  // shallow filters exist but are rare because of the every-depth gather quirk.
  for (int i = 0; i < 32; i++) p->depth_w[i] = 1.0;
  p->depth_w[0] = 0.0002;
  p->depth_w[1] = 0.004;
  switch (config) {
    case 1:
      p->n_filters = 10000;
      p->n_topics = 100000;
      p->max_depth = 6;
      p->p_plus = 0.20;
      p->p_hash = 0.05;
      for (int i = 0; i < 8; i++) p->vocab[i] = std::max<uint32_t>(4, v[i] / 4);
      break;
    case 2:
      p->n_filters = 1000000;
      p->n_topics = 10000000;
      p->max_depth = 8;
      p->p_plus = 0.20;
      p->p_hash = 0.05;
      break;
    case 3:
      p->n_filters = 10000000;
      p->n_topics = 10000000;
      p->max_depth = 8;
      p->p_plus = 0.40;
      p->p_hash = 0.10;
      p->topic_zipf_s = 1.2;
      p->token_zipf_s = 0.8;
      p->vocab[0] = 4096;
      p->vocab[1] = 16384;
      for (int i = 2; i < 8; i++) p->vocab[i] = 65536;
      break;
    case 4:
      p->n_filters = 100000000;
      p->n_topics = 10000000;
      p->max_depth = 8;
      p->p_plus = 0.20;
      p->p_hash = 0.05;
      p->vocab[0] = 1024;
      p->vocab[1] = 16384;
      for (int i = 2; i < 8; i++) p->vocab[i] = 65536;
      break;
    default:  // 5: shared subscriptions + retained reverse match
      p->n_filters = 1000000;
      p->n_topics = 1000000;
      p->max_depth = 8;
      p->p_plus = 0.20;
      p->p_hash = 0.05;
      p->p_shared = 0.05;
      break;
  }
  for (uint32_t i = p->max_depth; i < 32; i++) p->depth_w[i] = 0.0;
}

extern "C" int mqgen_generate(const mqgen_params *p, mqgen_workload *out) {
  memset(out, 0, sizeof(*out));
  if (p->max_depth < 1 || p->max_depth > 32) return -1;
  Rng rng(p->seed);
  const uint32_t md = p->max_depth;
  Vocab voc;
  voc.tok.resize(md);
  voc.z.resize(md);
  for (uint32_t d = 0; d < md; d++) {
    uint32_t n = p->vocab[d < 8 ? d : 7];
    if (n < 1) n = 1;
    voc.tok[d].resize(n);
    for (uint32_t k = 0; k < n; k++) voc.tok[d][k] = make_token(p->seed, d, k);
    voc.z[d] = Zipf(n, p->token_zipf_s);
  }
  // depth distribution
  std::vector<double> dcdf(md);
  double acc = 0;
  for (uint32_t i = 0; i < md; i++) dcdf[i] = (acc += p->depth_w[i]);
  for (auto &c : dcdf) c /= acc;
  auto draw_depth = [&](Rng &r) {
    double u = r.uniform();
    uint32_t m = (uint32_t)(std::lower_bound(dcdf.begin(), dcdf.end(), u) - dcdf.begin()) + 1;
    return m > md ? md : m;
  };
  const uint64_t nclients = p->n_clients ? p->n_clients : (p->n_filters + 3) / 4;

  Builder fb, cb, tb;
  // every filter's RNG state at its start: a topic instantiating filter fi
  // regenerates its levels (the first draws of the filter) instead of every
  // filter's levels being kept (100M filters would hold ~20 GB of strings)
  std::vector<uint64_t> fstate(p->n_filters);
  const bool all = p->client_lo == 0 && p->client_hi == 0;
  std::vector<uint32_t> cid;
  std::vector<uint8_t> qos, nl, rap, rh;
  std::vector<int32_t> ident;
  if (all) {
    cid.reserve(p->n_filters);
    qos.reserve(p->n_filters);
    nl.reserve(p->n_filters);
    rap.reserve(p->n_filters);
    rh.reserve(p->n_filters);
    ident.reserve(p->n_filters);
  }
  static const std::string kPlus = "+", kHash = "#";
  std::vector<const std::string *> lv;  // levels as pointers into the vocabulary
  auto filter_levels = [&](Rng &r, uint64_t i, std::vector<const std::string *> &out) {
    out.clear();
    if (i < p->n_root_hash) {
      out.push_back(&kHash);
      return;
    }
    uint32_t m = draw_depth(r);
    for (uint32_t d = 0; d < m; d++) out.push_back(&voc.tok[d][voc.z[d].draw(r)]);
    if (m >= 2 && r.uniform() < p->p_plus) {  // a depth-1 "+" would match every topic
      int nplus = (m >= 4 && r.uniform() < p->p_plus) ? 2 : 1;  // "a/+/+"-style filters only when deep
      for (int k = 0; k < nplus; k++) {
        // level 0 becomes '+' rarely (a root '+' matches every topic)
        uint32_t d = (m > 1 && r.uniform() > 0.02) ? 1 + (uint32_t)r.below(m - 1) : 0;
        out[d] = &kPlus;
      }
    }
    if (m >= 2 && r.uniform() < p->p_hash) out[m - 1] = &kHash;
  };
  std::string f;
  for (uint64_t i = 0; i < p->n_filters; i++) {
    fstate[i] = rng.s;
    filter_levels(rng, i, lv);
    bool shared = rng.uniform() < p->p_shared;
    const uint64_t group = shared ? rng.below(16) : 0;
    uint32_t c = (uint32_t)rng.below(nclients);
    const uint8_t q = (uint8_t)rng.below(3);
    const int32_t id = rng.uniform() < 0.5 ? 0 : (int32_t)(1 + rng.below((1u << 28) - 2));
    const uint8_t n_l = (!shared && rng.uniform() < 0.1) ? 1 : 0;
    const uint8_t ra = rng.uniform() < 0.5 ? 1 : 0;
    const uint8_t r_h = (uint8_t)rng.below(3);
    if (!all && (c < p->client_lo || c >= p->client_hi)) continue;
    f.clear();
    if (shared) f = "$SHARE/g" + std::to_string(group) + "/";
    for (size_t d = 0; d < lv.size(); d++) {
      if (d) f.push_back('/');
      f += *lv[d];
    }
    fb.push(f);
    cid.push_back(c);
    cb.push("client-" + std::to_string(c));
    qos.push_back(q);
    ident.push_back(id);
    nl.push_back(n_l);
    rap.push_back(ra);
    rh.push_back(r_h);
  }
  Zipf fz;
  if (p->topic_zipf_s > 0 && p->n_filters) fz = Zipf(p->n_filters, p->topic_zipf_s);
  std::string t;
  std::vector<std::string> tl;  // a topic's levels
  std::vector<const std::string *> fl;
  for (uint64_t i = 0; i < p->n_topics; i++) {
    tl.clear();
    if (p->n_filters && rng.uniform() < p->p_instantiate) {
      uint64_t fi = p->topic_zipf_s > 0 ? fz.draw(rng) : rng.below(p->n_filters);
      Rng fr(fstate[fi]);
      filter_levels(fr, fi, fl);
      for (size_t d = 0; d < fl.size() && tl.size() < md; d++) {
        if (fl[d] == &kPlus) {
          tl.push_back(voc.tok[d][voc.z[d].draw(rng)]);
        } else if (fl[d] == &kHash) {
          uint32_t extra = (uint32_t)rng.below(3);
          for (uint32_t k = 0; k < extra && tl.size() < md; k++) {
            uint32_t dd = (uint32_t)tl.size();
            tl.push_back(voc.tok[dd][voc.z[dd].draw(rng)]);
          }
        } else {
          tl.push_back(*fl[d]);
        }
      }
      if (tl.empty()) tl.push_back(voc.tok[0][voc.z[0].draw(rng)]);
    } else {
      uint32_t m = draw_depth(rng);
      for (uint32_t d = 0; d < m; d++) tl.push_back(voc.tok[d][voc.z[d].draw(rng)]);
    }
    if (rng.uniform() < p->p_dollar_topic) tl[0] = rng.uniform() < 0.5 ? "$SYS" : "$dev" + tl[0];
    t.clear();
    for (size_t d = 0; d < tl.size(); d++) {
      if (d) t.push_back('/');
      t += tl[d];
    }
    tb.push(t);
  }
  fb.emit(&out->filters);
  cb.emit(&out->clients);
  tb.emit(&out->topics);
  auto dup = [](const void *src, size_t n) {
    void *d = malloc(n ? n : 1);
    if (n) memcpy(d, src, n);
    return d;
  };
  out->client_ids = (uint32_t *)dup(cid.data(), cid.size() * 4);
  out->qos = (uint8_t *)dup(qos.data(), qos.size());
  out->no_local = (uint8_t *)dup(nl.data(), nl.size());
  out->rap = (uint8_t *)dup(rap.data(), rap.size());
  out->rh = (uint8_t *)dup(rh.data(), rh.size());
  out->ident = (int32_t *)dup(ident.data(), ident.size() * 4);
  return 0;
}

extern "C" void mqgen_free(mqgen_workload *w) {
  if (!w) return;
  mqgen_strings *s[3] = {&w->filters, &w->clients, &w->topics};
  for (auto *x : s) {
    free(x->bytes);
    free(x->offs);
  }
  free(w->client_ids);
  free(w->qos);
  free(w->no_local);
  free(w->rap);
  free(w->rh);
  free(w->ident);
  memset(w, 0, sizeof(*w));
}
