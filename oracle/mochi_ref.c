/*
 * oracle/mochi_ref.c — TEST INFRASTRUCTURE ONLY (see mochi_ref.h header).
 *
 * Plain-C restatement of mochi-co/mqtt v2.2.12 `TopicsIndex`
 * (vendor/github.com/mochi-co/mqtt/v2/topics.go) as vendored by gsalomao/maxmq.
 * Every function names the reference lines it restates.  The structure is the
 * reference's on purpose (per-node hash maps keyed by level string, recursive
 * scan over {key, "+", "#"}, gather at every visited node, per-client merge),
 * because this file is both the parity checker and the CPU baseline.
 *
 * Not shipped: the product path (maxmq_amd/csrc) is independent code.
 */
#include "mochi_ref.h"

#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* small utilities                                                           */
/* ------------------------------------------------------------------------ */

static uint64_t hash_bytes(const char *p, uint32_t n) {
  /* FNV-1a 64 with a final avalanche; only used for the oracle's own maps */
  uint64_t h = 0xcbf29ce484222325ull;
  for (uint32_t i = 0; i < n; i++) {
    h ^= (uint8_t)p[i];
    h *= 0x100000001b3ull;
  }
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  return h;
}

static char *dup_bytes(const char *p, uint32_t n) {
  char *r = (char *)malloc(n ? n : 1);
  if (n) memcpy(r, p, n);
  return r;
}

static int eq_bytes(const char *a, uint32_t an, const char *b, uint32_t bn) {
  return an == bn && (an == 0 || memcmp(a, b, an) == 0);
}

/* strings.EqualFold(level, "$SHARE") (topics.go:309,340,582).  Go folds by
 * Unicode simple case folding, under which the only non-ASCII rune equal to a
 * letter of "$SHARE" is U+017F (LATIN SMALL LETTER LONG S, UTF-8 C5 BF) ~ 's'. */
static int equal_fold_share(const char *a, uint32_t an) {
  static const char want[6] = {'$', 's', 'h', 'a', 'r', 'e'};
  uint32_t i = 0;
  for (int k = 0; k < 6; k++) {
    if (i >= an) return 0;
    unsigned char x = (unsigned char)a[i];
    if (want[k] == 's' && x == 0xC5 && i + 1 < an && (unsigned char)a[i + 1] == 0xBF) {
      i += 2;
      continue;
    }
    if (x >= 'A' && x <= 'Z') x = (unsigned char)(x - 'A' + 'a');
    if (x != (unsigned char)want[k]) return 0;
    i++;
  }
  return i == an;
}

/* ------------------------------------------------------------------------ */
/* string-keyed map (open addressing, linear probing, backward-shift delete) */
/* ------------------------------------------------------------------------ */

typedef struct {
  char *k;
  uint32_t kn;
  uint32_t used;
  uint64_t h;
  void *v;
} sslot;

typedef struct {
  sslot *s;
  uint32_t cap; /* power of two or 0 */
  uint32_t n;
} smap;

static void smap_grow(smap *m);

static sslot *smap_find(const smap *m, const char *k, uint32_t kn, uint64_t h) {
  if (!m->cap) return NULL;
  uint32_t mask = m->cap - 1;
  for (uint32_t i = (uint32_t)h & mask;; i = (i + 1) & mask) {
    sslot *s = &m->s[i];
    if (!s->used) return NULL;
    if (s->h == h && eq_bytes(s->k, s->kn, k, kn)) return s;
  }
}

static void *smap_get(const smap *m, const char *k, uint32_t kn) {
  sslot *s = smap_find(m, k, kn, hash_bytes(k, kn));
  return s ? s->v : NULL;
}

static void smap_put(smap *m, const char *k, uint32_t kn, void *v) {
  uint64_t h = hash_bytes(k, kn);
  sslot *s = smap_find(m, k, kn, h);
  if (s) {
    s->v = v;
    return;
  }
  if ((m->n + 1) * 2 > m->cap) smap_grow(m);
  uint32_t mask = m->cap - 1;
  uint32_t i = (uint32_t)h & mask;
  while (m->s[i].used) i = (i + 1) & mask;
  m->s[i].k = dup_bytes(k, kn);
  m->s[i].kn = kn;
  m->s[i].h = h;
  m->s[i].v = v;
  m->s[i].used = 1;
  m->n++;
}

static void smap_grow(smap *m) {
  uint32_t nc = m->cap ? m->cap * 2 : 4;
  sslot *old = m->s;
  uint32_t oc = m->cap;
  m->s = (sslot *)calloc(nc, sizeof(sslot));
  m->cap = nc;
  for (uint32_t i = 0; i < oc; i++) {
    if (!old[i].used) continue;
    uint32_t j = (uint32_t)old[i].h & (nc - 1);
    while (m->s[j].used) j = (j + 1) & (nc - 1);
    m->s[j] = old[i];
  }
  free(old);
}

/* delete returns the removed value (or NULL) */
static void *smap_del(smap *m, const char *k, uint32_t kn) {
  uint64_t h = hash_bytes(k, kn);
  sslot *s = smap_find(m, k, kn, h);
  if (!s) return NULL;
  void *v = s->v;
  free(s->k);
  uint32_t mask = m->cap - 1;
  uint32_t i = (uint32_t)(s - m->s);
  m->s[i].used = 0;
  /* backward-shift deletion keeps probe chains intact */
  uint32_t j = i;
  for (;;) {
    j = (j + 1) & mask;
    if (!m->s[j].used) break;
    uint32_t home = (uint32_t)m->s[j].h & mask;
    /* can slot j move to i?  yes if home is not in (i, j] cyclically */
    int move = (i <= j) ? (home <= i || home > j) : (home <= i && home > j);
    if (move) {
      m->s[i] = m->s[j];
      m->s[j].used = 0;
      i = j;
    }
  }
  m->n--;
  return v;
}

static void smap_free(smap *m) {
  for (uint32_t i = 0; i < m->cap; i++)
    if (m->s[i].used) free(m->s[i].k);
  free(m->s);
  m->s = NULL;
  m->cap = m->n = 0;
}

/* ------------------------------------------------------------------------ */
/* client-keyed subscription map: packets.Subscription by client id          */
/* ------------------------------------------------------------------------ */

typedef struct {
  uint32_t filter; /* Subscription.Filter (interned) */
  int32_t ident;   /* Subscription.Identifier        */
  uint8_t qos, no_local, rap, rh;
} sub_t;

typedef struct {
  uint32_t client;
  uint32_t used;
  sub_t sub;
} cslot;

typedef struct {
  cslot *s;
  uint32_t cap, n;
} cmap;

static uint32_t hash_u32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

static cslot *cmap_find(const cmap *m, uint32_t c) {
  if (!m->cap) return NULL;
  uint32_t mask = m->cap - 1;
  for (uint32_t i = hash_u32(c) & mask;; i = (i + 1) & mask) {
    if (!m->s[i].used) return NULL;
    if (m->s[i].client == c) return &m->s[i];
  }
}

static void cmap_grow(cmap *m) {
  uint32_t nc = m->cap ? m->cap * 2 : 4;
  cslot *old = m->s;
  uint32_t oc = m->cap;
  m->s = (cslot *)calloc(nc, sizeof(cslot));
  m->cap = nc;
  for (uint32_t i = 0; i < oc; i++) {
    if (!old[i].used) continue;
    uint32_t j = hash_u32(old[i].client) & (nc - 1);
    while (m->s[j].used) j = (j + 1) & (nc - 1);
    m->s[j] = old[i];
  }
  free(old);
}

static void cmap_put(cmap *m, uint32_t c, const sub_t *v) {
  cslot *s = cmap_find(m, c);
  if (s) {
    s->sub = *v;
    return;
  }
  if ((m->n + 1) * 2 > m->cap) cmap_grow(m);
  uint32_t mask = m->cap - 1;
  uint32_t i = hash_u32(c) & mask;
  while (m->s[i].used) i = (i + 1) & mask;
  m->s[i].client = c;
  m->s[i].sub = *v;
  m->s[i].used = 1;
  m->n++;
}

static void cmap_del(cmap *m, uint32_t c) {
  cslot *s = cmap_find(m, c);
  if (!s) return;
  uint32_t mask = m->cap - 1;
  uint32_t i = (uint32_t)(s - m->s);
  m->s[i].used = 0;
  uint32_t j = i;
  for (;;) {
    j = (j + 1) & mask;
    if (!m->s[j].used) break;
    uint32_t home = hash_u32(m->s[j].client) & mask;
    int move = (i <= j) ? (home <= i || home > j) : (home <= i && home > j);
    if (move) {
      m->s[i] = m->s[j];
      m->s[j].used = 0;
      i = j;
    }
  }
  m->n--;
}

/* ------------------------------------------------------------------------ */
/* intern tables (dense ids in first-appearance order)                       */
/* ------------------------------------------------------------------------ */

typedef struct {
  smap ids; /* value = id + 1 */
  char **names;
  uint32_t *lens;
  uint32_t n, cap;
} interner;

static uint32_t intern(interner *t, const char *s, uint32_t n) {
  void *v = smap_get(&t->ids, s, n);
  if (v) return (uint32_t)((uintptr_t)v - 1);
  if (t->n == t->cap) {
    t->cap = t->cap ? t->cap * 2 : 64;
    t->names = (char **)realloc(t->names, sizeof(char *) * t->cap);
    t->lens = (uint32_t *)realloc(t->lens, sizeof(uint32_t) * t->cap);
  }
  uint32_t id = t->n++;
  t->names[id] = dup_bytes(s, n);
  t->lens[id] = n;
  smap_put(&t->ids, s, n, (void *)(uintptr_t)(id + 1));
  return id;
}

/* lookup without inserting; returns UINT32_MAX if absent */
static uint32_t intern_find(const interner *t, const char *s, uint32_t n) {
  void *v = smap_get(&t->ids, s, n);
  return v ? (uint32_t)((uintptr_t)v - 1) : UINT32_MAX;
}

static void interner_free(interner *t) {
  for (uint32_t i = 0; i < t->n; i++) free(t->names[i]);
  free(t->names);
  free(t->lens);
  smap_free(&t->ids);
}

/* ------------------------------------------------------------------------ */
/* the trie: `particle` (topics.go:627-646)                                  */
/* ------------------------------------------------------------------------ */

typedef struct particle {
  char *key;
  uint32_t klen;
  struct particle *parent;
  smap particles;      /* key -> particle*                         */
  cmap subscriptions;  /* client -> Subscription                   */
  smap shared;         /* group -> cmap* (client -> Subscription)  */
  uint32_t shared_len; /* SharedSubscriptions.Len()                */
  char *retain_path;   /* retainPath ("" == none)                  */
  uint32_t rplen;
} particle;

typedef struct {
  uint64_t msg_ref;
  uint32_t payload_len;
  uint8_t retain_flag;
} retained_t;

struct oref {
  particle *root;
  smap retained; /* topic -> retained_t* (packets.Packets) */
  interner clients;
  interner filters;
};

static particle *new_particle(const char *key, uint32_t klen, particle *parent) {
  particle *p = (particle *)calloc(1, sizeof(particle));
  p->key = dup_bytes(key, klen);
  p->klen = klen;
  p->parent = parent;
  p->retain_path = dup_bytes("", 0);
  p->rplen = 0;
  return p;
}

static void free_particle(particle *p) {
  for (uint32_t i = 0; i < p->particles.cap; i++)
    if (p->particles.s[i].used) free_particle((particle *)p->particles.s[i].v);
  smap_free(&p->particles);
  free(p->subscriptions.s);
  for (uint32_t i = 0; i < p->shared.cap; i++)
    if (p->shared.s[i].used) {
      cmap *g = (cmap *)p->shared.s[i].v;
      free(g->s);
      free(g);
    }
  smap_free(&p->shared);
  free(p->retain_path);
  free(p->key);
  free(p);
}

oref *oref_new(void) {
  oref *x = (oref *)calloc(1, sizeof(oref));
  x->root = new_particle("", 0, NULL); /* NewTopicsIndex (topics.go:291-299) */
  return x;
}

void oref_free(oref *x) {
  if (!x) return;
  free_particle(x->root);
  for (uint32_t i = 0; i < x->retained.cap; i++)
    if (x->retained.s[i].used) free(x->retained.s[i].v);
  smap_free(&x->retained);
  interner_free(&x->clients);
  interner_free(&x->filters);
  free(x);
}

/* isolateParticle (topics.go:558-577).  Restated literally, including its
 * re-scan from the start of the string on every call (O(d) per call). */
int oref_isolate_particle(const char *s, uint32_t slen, int d, uint32_t *start, uint32_t *len) {
  uint32_t base = 0; /* `filter` is the suffix s[base:] */
  int end = 0;
  int has_next = 0;
  *start = 0;
  *len = 0;
  for (int i = 0; end > -1 && i <= d; i++) {
    const char *f = s + base;
    uint32_t fl = slen - base;
    const char *q = (const char *)memchr(f, '/', fl);
    end = q ? (int)(q - f) : -1;
    if (d > -1 && i == d && end > -1) {
      has_next = 1;
      *start = base;
      *len = (uint32_t)end;
    } else if (end > -1) {
      has_next = 0;
      base += (uint32_t)end + 1;
    } else {
      has_next = 0;
      *start = base;
      *len = fl;
    }
  }
  return has_next;
}

static int is_share_prefix_level0(const char *f, uint32_t fl) {
  uint32_t st, ln;
  oref_isolate_particle(f, fl, 0, &st, &ln);
  return equal_fold_share(f + st, ln);
}

/* set (topics.go:380-397) */
static particle *trie_set(oref *x, const char *topic, uint32_t tlen, int d) {
  int has_next = 1;
  particle *n = x->root;
  while (has_next) {
    uint32_t st, ln;
    has_next = oref_isolate_particle(topic, tlen, d, &st, &ln);
    d++;
    particle *p = (particle *)smap_get(&n->particles, topic + st, ln);
    if (!p) {
      p = new_particle(topic + st, ln, n);
      smap_put(&n->particles, topic + st, ln, p);
    }
    n = p;
  }
  return n;
}

/* seek (topics.go:400-414) */
static particle *trie_seek(oref *x, const char *filter, uint32_t flen, int d) {
  int has_next = 1;
  particle *n = x->root;
  while (has_next) {
    uint32_t st, ln;
    has_next = oref_isolate_particle(filter, flen, d, &st, &ln);
    n = (particle *)smap_get(&n->particles, filter + st, ln);
    d++;
    if (!n) return NULL;
  }
  return n;
}

/* trim (topics.go:417-423) */
static void trim(particle *n) {
  while (n->parent && n->rplen == 0 && n->particles.n + n->subscriptions.n + n->shared_len == 0) {
    particle *parent = n->parent;
    particle *p = (particle *)smap_del(&parent->particles, n->key, n->klen);
    if (p) free_particle(p);
    n = parent;
  }
}

/* TopicsIndex.Subscribe (topics.go:303-321) */
int oref_subscribe(oref *x, const char *client, uint32_t clen, const char *filter, uint32_t flen,
                   uint8_t qos, uint8_t no_local, uint8_t rap, uint8_t rh, int32_t ident) {
  uint32_t cid = intern(&x->clients, client, clen);
  sub_t s;
  s.filter = intern(&x->filters, filter, flen);
  s.ident = ident;
  s.qos = qos;
  s.no_local = no_local;
  s.rap = rap;
  s.rh = rh;
  int existed;
  if (is_share_prefix_level0(filter, flen)) {
    uint32_t gst, gln;
    oref_isolate_particle(filter, flen, 1, &gst, &gln);
    particle *n = trie_set(x, filter, flen, 2);
    cmap *g = (cmap *)smap_get(&n->shared, filter + gst, gln);
    existed = g && cmap_find(g, cid) != NULL;
    /* SharedSubscriptions.Add (topics.go:122-129) */
    if (!g) {
      g = (cmap *)calloc(1, sizeof(cmap));
      smap_put(&n->shared, filter + gst, gln, g);
    }
    if (!existed) n->shared_len++;
    cmap_put(g, cid, &s);
  } else {
    particle *n = trie_set(x, filter, flen, 0);
    existed = cmap_find(&n->subscriptions, cid) != NULL;
    cmap_put(&n->subscriptions, cid, &s);
  }
  return !existed;
}

void oref_subscribe_many(oref *x, uint64_t n, const char *cbytes, const uint64_t *coffs, const char *fbytes,
                         const uint64_t *foffs, const uint8_t *qos, const uint8_t *no_local, const uint8_t *rap,
                         const uint8_t *rh, const int32_t *ident) {
  for (uint64_t i = 0; i < n; i++)
    oref_subscribe(x, cbytes + coffs[i], (uint32_t)(coffs[i + 1] - coffs[i]), fbytes + foffs[i],
                   (uint32_t)(foffs[i + 1] - foffs[i]), qos[i], no_local[i], rap[i], rh[i], ident[i]);
}

/* TopicsIndex.Unsubscribe (topics.go:325-349) */
int oref_unsubscribe(oref *x, const char *filter, uint32_t flen, const char *client, uint32_t clen) {
  int d = 0;
  if (flen >= 6 && memcmp(filter, "$SHARE", 6) == 0) d = 2; /* strings.HasPrefix: case-sensitive */
  particle *p = trie_seek(x, filter, flen, d);
  if (!p) return 0;
  uint32_t cid = intern_find(&x->clients, client, clen);
  if (is_share_prefix_level0(filter, flen)) {
    uint32_t gst, gln;
    oref_isolate_particle(filter, flen, 1, &gst, &gln);
    /* SharedSubscriptions.Delete (topics.go:132-139) */
    cmap *g = (cmap *)smap_get(&p->shared, filter + gst, gln);
    if (g) {
      if (cid != UINT32_MAX && cmap_find(g, cid)) {
        cmap_del(g, cid);
        p->shared_len--;
      }
      if (g->n == 0) {
        smap_del(&p->shared, filter + gst, gln);
        free(g->s);
        free(g);
      }
    }
  } else if (cid != UINT32_MAX) {
    cmap_del(&p->subscriptions, cid);
  }
  trim(p);
  return 1;
}

/* TopicsIndex.RetainMessage (topics.go:354-377) */
int64_t oref_retain(oref *x, const char *topic, uint32_t tlen, uint64_t msg_ref, uint32_t payload_len,
                    uint8_t retain_flag) {
  particle *n = trie_set(x, topic, tlen, 0);
  if (payload_len > 0) {
    free(n->retain_path);
    n->retain_path = dup_bytes(topic, tlen);
    n->rplen = tlen;
    retained_t *r = (retained_t *)smap_get(&x->retained, topic, tlen);
    if (!r) {
      r = (retained_t *)malloc(sizeof(retained_t));
      smap_put(&x->retained, topic, tlen, r);
    }
    r->msg_ref = msg_ref;
    r->payload_len = payload_len;
    r->retain_flag = retain_flag;
    return 1;
  }
  int64_t out = 0;
  retained_t *r = (retained_t *)smap_get(&x->retained, topic, tlen);
  if (r && r->payload_len > 0 && r->retain_flag) out = -1;
  free(n->retain_path);
  n->retain_path = dup_bytes("", 0);
  n->rplen = 0;
  r = (retained_t *)smap_del(&x->retained, topic, tlen);
  free(r);
  trim(n);
  return out;
}

void oref_retain_many(oref *x, uint64_t n, const char *bytes, const uint64_t *offs, const uint64_t *msg_refs,
                      uint32_t payload_len) {
  for (uint64_t i = 0; i < n; i++)
    oref_retain(x, bytes + offs[i], (uint32_t)(offs[i + 1] - offs[i]), msg_refs[i], payload_len, 1);
}

uint32_t oref_num_clients(const oref *x) { return x->clients.n; }
uint32_t oref_num_filters(const oref *x) { return x->filters.n; }
uint64_t oref_retained_len(const oref *x) { return x->retained.n; }

static uint32_t copy_name(const interner *t, uint32_t id, char *buf, uint32_t cap) {
  if (id >= t->n) return 0;
  uint32_t l = t->lens[id];
  if (buf && cap) memcpy(buf, t->names[id], l < cap ? l : cap);
  return l;
}
uint32_t oref_filter_name(const oref *x, uint32_t id, char *buf, uint32_t cap) {
  return copy_name(&x->filters, id, buf, cap);
}
uint32_t oref_client_name(const oref *x, uint32_t id, char *buf, uint32_t cap) {
  return copy_name(&x->clients, id, buf, cap);
}

/* ------------------------------------------------------------------------ */
/* Subscribers (topics.go:484-555) with per-thread merge scratch             */
/* ------------------------------------------------------------------------ */

typedef struct {
  /* the result map `Subscribers.Subscriptions`, as dense arrays by client */
  uint32_t *stamp;
  sub_t *merged;
  uint32_t *touched;
  uint32_t ntouched, cap_touched;
  uint32_t gen;
  /* `Subscribers.Shared`: (filter, client, qos) list, deduped at the end */
  oref_shared *sh;
  uint32_t nsh, cap_sh;
  /* Identifiers (packets.go:250-258): every gathered (client, filter, id>0),
   * plus the first-merged pair per client; sorted and deduped at the end */
  oref_ident *id;
  uint32_t nid, cap_id;
  int want_ids;
  oref_stats st;
} scratch;

static void scratch_init(scratch *s, uint32_t nclients) {
  memset(s, 0, sizeof(*s));
  s->stamp = (uint32_t *)calloc(nclients ? nclients : 1, sizeof(uint32_t));
  s->merged = (sub_t *)malloc(sizeof(sub_t) * (nclients ? nclients : 1));
}

static void scratch_free(scratch *s) {
  free(s->stamp);
  free(s->merged);
  free(s->touched);
  free(s->sh);
  free(s->id);
}

static void push_ident(scratch *s, uint32_t client, uint32_t filter, int32_t ident) {
  if (s->nid == s->cap_id) {
    s->cap_id = s->cap_id ? s->cap_id * 2 : 256;
    s->id = (oref_ident *)realloc(s->id, sizeof(oref_ident) * s->cap_id);
  }
  oref_ident *o = &s->id[s->nid++];
  o->client = client;
  o->filter = filter;
  o->ident = ident;
}

/* gatherSubscriptions (topics.go:521-538) with Subscription.Merge
 * (packets.go:250-270): first-seen fields kept, QoS = max, NoLocal |=. */
static void gather_subscriptions(const oref *x, const char *topic, const particle *p, scratch *s) {
  for (uint32_t i = 0; i < p->subscriptions.cap; i++) {
    const cslot *cs = &p->subscriptions.s[i];
    if (!cs->used) continue;
    const sub_t *sub = &cs->sub;
    uint32_t fl = x->filters.lens[sub->filter];
    const char *f = x->filters.names[sub->filter];
    s->st.gathered++;
    if (fl > 0 && topic[0] == '$' && (f[0] == '+' || f[0] == '#')) continue; /* [MQTT-4.7.1-1/2] */
    uint32_t c = cs->client;
    /* Merge: Identifiers[n.Filter] = n.Identifier when n.Identifier > 0 (:257-259) */
    if (s->want_ids && sub->ident > 0) push_ident(s, c, sub->filter, sub->ident);
    if (s->stamp[c] != s->gen) {
      s->stamp[c] = s->gen;
      s->merged[c] = *sub;
      if (s->ntouched == s->cap_touched) {
        s->cap_touched = s->cap_touched ? s->cap_touched * 2 : 256;
        s->touched = (uint32_t *)realloc(s->touched, sizeof(uint32_t) * s->cap_touched);
      }
      s->touched[s->ntouched++] = c;
    } else {
      sub_t *m = &s->merged[c];
      if (sub->qos > m->qos) m->qos = sub->qos;
      if (sub->no_local) m->no_local = 1;
    }
  }
}

/* gatherSharedSubscriptions (topics.go:541-555) */
static void gather_shared(const particle *p, scratch *s) {
  for (uint32_t i = 0; i < p->shared.cap; i++) {
    if (!p->shared.s[i].used) continue;
    const cmap *g = (const cmap *)p->shared.s[i].v;
    for (uint32_t j = 0; j < g->cap; j++) {
      if (!g->s[j].used) continue;
      s->st.gathered++;
      if (s->nsh == s->cap_sh) {
        s->cap_sh = s->cap_sh ? s->cap_sh * 2 : 64;
        s->sh = (oref_shared *)realloc(s->sh, sizeof(oref_shared) * s->cap_sh);
      }
      oref_shared *o = &s->sh[s->nsh++];
      o->filter = g->s[j].sub.filter;
      o->client = g->s[j].client;
      o->qos = g->s[j].sub.qos;
      o->pad[0] = o->pad[1] = o->pad[2] = 0;
    }
  }
}

/* scanSubscribers (topics.go:493-518), restated literally: the slice
 * {key, "+", "#"} is walked even when key itself is "+" or "#". */
static void scan_subscribers(const oref *x, const char *topic, uint32_t tlen, int d, const particle *n,
                             scratch *s) {
  if (tlen == 0) return;
  uint32_t st, ln;
  int has_next = oref_isolate_particle(topic, tlen, d, &st, &ln);
  const char *keys[3] = {topic + st, "+", "#"};
  uint32_t klens[3] = {ln, 1, 1};
  for (int k = 0; k < 3; k++) {
    s->st.probes++;
    const particle *p = (const particle *)smap_get(&n->particles, keys[k], klens[k]);
    if (!p) continue;
    s->st.visits++;
    gather_subscriptions(x, topic, p, s);
    gather_shared(p, s);
    const int literal = !eq_bytes(keys[k], klens[k], "#", 1) && !eq_bytes(keys[k], klens[k], "+", 1);
    if (literal) {
      s->st.probes++;
      const particle *w = (const particle *)smap_get(&p->particles, "#", 1);
      if (w) {
        s->st.visits++;
        gather_subscriptions(x, topic, w, s);
      }
    }
    if (has_next) scan_subscribers(x, topic, tlen, d + 1, p, s);
  }
}

static int cmp_u32(const void *a, const void *b) {
  uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
  return (x > y) - (x < y);
}

static int cmp_ident(const void *a, const void *b) {
  const oref_ident *x = (const oref_ident *)a, *y = (const oref_ident *)b;
  if (x->client != y->client) return (x->client > y->client) - (x->client < y->client);
  return (x->filter > y->filter) - (x->filter < y->filter);
}

static int cmp_shared(const void *a, const void *b) {
  const oref_shared *x = (const oref_shared *)a, *y = (const oref_shared *)b;
  if (x->filter != y->filter) return (x->filter > y->filter) - (x->filter < y->filter);
  return (x->client > y->client) - (x->client < y->client);
}

/* one Subscribers(topic) call; leaves sorted, unique results in scratch */
static void subscribers_one(const oref *x, const char *topic, uint32_t tlen, scratch *s) {
  s->gen++;
  if (s->gen == 0) { /* stamp wrap */
    memset(s->stamp, 0, sizeof(uint32_t) * (x->clients.n ? x->clients.n : 1));
    s->gen = 1;
  }
  s->ntouched = 0;
  s->nsh = 0;
  s->nid = 0;
  s->st.topics++;
  s->st.topic_bytes += tlen;
  scan_subscribers(x, topic, tlen, 0, x->root, s);
  if (s->ntouched > 1) qsort(s->touched, s->ntouched, sizeof(uint32_t), cmp_u32);
  if (s->nsh > 1) {
    qsort(s->sh, s->nsh, sizeof(oref_shared), cmp_shared);
    uint32_t w = 1;
    for (uint32_t i = 1; i < s->nsh; i++)
      if (s->sh[i].filter != s->sh[w - 1].filter || s->sh[i].client != s->sh[w - 1].client) s->sh[w++] = s->sh[i];
    s->nsh = w;
  }
  s->st.deliveries += s->ntouched;
  s->st.shared += s->nsh;
  if (s->want_ids) {
    /* the first-merged subscription's pair, kept even when its id is 0
     * (Identifiers = {s.Filter: s.Identifier}, packets.go:251-255) */
    for (uint32_t k = 0; k < s->ntouched; k++) {
      const sub_t *m = &s->merged[s->touched[k]];
      push_ident(s, s->touched[k], m->filter, m->ident);
    }
    if (s->nid > 1) {
      qsort(s->id, s->nid, sizeof(oref_ident), cmp_ident);
      uint32_t w = 1;
      for (uint32_t i = 1; i < s->nid; i++)
        if (s->id[i].client != s->id[w - 1].client || s->id[i].filter != s->id[w - 1].filter) s->id[w++] = s->id[i];
      s->nid = w;
    }
  }
}

/* ------------------------------------------------------------------------ */
/* batch drivers (threads split the batch into contiguous chunks)            */
/* ------------------------------------------------------------------------ */

typedef struct {
  oref *x;
  const char *bytes;
  const uint64_t *offs;
  uint32_t lo, hi;
  int fill;
  uint32_t *dcount, *scount;
  const uint64_t *doffs, *soffs;
  oref_delivery *dout;
  oref_shared *sout;
  int ids;               /* 1: identifiers counts, 2: identifiers fill */
  uint32_t *icount;
  const uint64_t *ioffs;
  oref_ident *iout;
  oref_stats st;
} job_t;

static void *match_worker(void *arg) {
  job_t *j = (job_t *)arg;
  scratch s;
  scratch_init(&s, j->x->clients.n);
  s.want_ids = j->ids != 0;
  for (uint32_t i = j->lo; i < j->hi; i++) {
    const char *t = j->bytes + j->offs[i];
    uint32_t tl = (uint32_t)(j->offs[i + 1] - j->offs[i]);
    subscribers_one(j->x, t, tl, &s);
    if (j->ids == 1) {
      j->icount[i] = s.nid;
      continue;
    }
    if (j->ids == 2) {
      if (s.nid) memcpy(j->iout + j->ioffs[i], s.id, sizeof(oref_ident) * s.nid);
      continue;
    }
    if (!j->fill) {
      j->dcount[i] = s.ntouched;
      j->scount[i] = s.nsh;
      continue;
    }
    oref_delivery *o = j->dout + j->doffs[i];
    for (uint32_t k = 0; k < s.ntouched; k++) {
      uint32_t c = s.touched[k];
      const sub_t *m = &s.merged[c];
      o[k].client = c;
      o[k].first_filter = m->filter;
      o[k].first_ident = m->ident;
      o[k].qos = m->qos;
      o[k].no_local = m->no_local;
      o[k].rap = m->rap;
      o[k].rh = m->rh;
    }
    if (s.nsh) memcpy(j->sout + j->soffs[i], s.sh, sizeof(oref_shared) * s.nsh);
  }
  j->st = s.st;
  scratch_free(&s);
  return NULL;
}

static void run_jobs(job_t *proto, uint32_t n, int nthreads, void *(*fn)(void *), oref_stats *stats) {
  if (nthreads < 1) nthreads = 1;
  if ((uint32_t)nthreads > n) nthreads = n ? (int)n : 1;
  job_t *jobs = (job_t *)calloc((size_t)nthreads, sizeof(job_t));
  pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = *proto;
    jobs[t].lo = (uint32_t)((uint64_t)n * (uint64_t)t / (uint64_t)nthreads);
    jobs[t].hi = (uint32_t)((uint64_t)n * (uint64_t)(t + 1) / (uint64_t)nthreads);
    if (nthreads == 1)
      fn(&jobs[t]);
    else
      pthread_create(&th[t], NULL, fn, &jobs[t]);
  }
  if (nthreads > 1)
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  if (stats) {
    memset(stats, 0, sizeof(*stats));
    for (int t = 0; t < nthreads; t++) {
      stats->topics += jobs[t].st.topics;
      stats->topic_bytes += jobs[t].st.topic_bytes;
      stats->probes += jobs[t].st.probes;
      stats->visits += jobs[t].st.visits;
      stats->gathered += jobs[t].st.gathered;
      stats->deliveries += jobs[t].st.deliveries;
      stats->shared += jobs[t].st.shared;
    }
  }
  free(jobs);
  free(th);
}

int oref_match_counts(oref *x, const char *bytes, const uint64_t *offs, uint32_t n, int nthreads,
                      uint32_t *dcount, uint32_t *scount, oref_stats *stats) {
  job_t p;
  memset(&p, 0, sizeof(p));
  p.x = x;
  p.bytes = bytes;
  p.offs = offs;
  p.dcount = dcount;
  p.scount = scount;
  run_jobs(&p, n, nthreads, match_worker, stats);
  return 0;
}

int oref_match_fill(oref *x, const char *bytes, const uint64_t *offs, uint32_t n, int nthreads,
                    const uint64_t *doffs, oref_delivery *dout, const uint64_t *soffs, oref_shared *sout) {
  job_t p;
  memset(&p, 0, sizeof(p));
  p.x = x;
  p.bytes = bytes;
  p.offs = offs;
  p.fill = 1;
  p.doffs = doffs;
  p.dout = dout;
  p.soffs = soffs;
  p.sout = sout;
  run_jobs(&p, n, nthreads, match_worker, NULL);
  return 0;
}

int oref_match_ident_counts(oref *x, const char *bytes, const uint64_t *offs, uint32_t n, int nthreads,
                            uint32_t *icount) {
  job_t p;
  memset(&p, 0, sizeof(p));
  p.x = x;
  p.bytes = bytes;
  p.offs = offs;
  p.ids = 1;
  p.icount = icount;
  run_jobs(&p, n, nthreads, match_worker, NULL);
  return 0;
}

int oref_match_ident_fill(oref *x, const char *bytes, const uint64_t *offs, uint32_t n, int nthreads,
                          const uint64_t *ioffs, oref_ident *iout) {
  job_t p;
  memset(&p, 0, sizeof(p));
  p.x = x;
  p.bytes = bytes;
  p.offs = offs;
  p.ids = 2;
  p.ioffs = ioffs;
  p.iout = iout;
  run_jobs(&p, n, nthreads, match_worker, NULL);
  return 0;
}

/* ------------------------------------------------------------------------ */
/* Messages / scanMessages (topics.go:426-480)                               */
/* ------------------------------------------------------------------------ */

typedef struct {
  uint64_t *v;
  uint32_t n, cap;
} u64vec;

static void push_u64(u64vec *v, uint64_t x) {
  if (v->n == v->cap) {
    v->cap = v->cap ? v->cap * 2 : 64;
    v->v = (uint64_t *)realloc(v->v, sizeof(uint64_t) * v->cap);
  }
  v->v[v->n++] = x;
}

static void retained_get(const oref *x, const char *t, uint32_t tl, u64vec *out) {
  const retained_t *r = (const retained_t *)smap_get(&x->retained, t, tl);
  if (r) push_u64(out, r->msg_ref);
}

static void scan_messages(const oref *x, const char *filter, uint32_t flen, int d, const particle *n,
                          u64vec *out) {
  if (!n) n = x->root;
  if (flen == 0 || x->retained.n == 0) return;
  if (!memchr(filter, '#', flen) && !memchr(filter, '+', flen)) {
    retained_get(x, filter, flen, out);
    return;
  }
  uint32_t st, ln;
  int has_next = oref_isolate_particle(filter, flen, d, &st, &ln);
  const char *key = filter + st;
  const int is_plus = eq_bytes(key, ln, "+", 1), is_hash = eq_bytes(key, ln, "#", 1);
  if (is_plus || is_hash || d == -1) {
    for (uint32_t i = 0; i < n->particles.cap; i++) {
      if (!n->particles.s[i].used) continue;
      const particle *adj = (const particle *)n->particles.s[i].v;
      if (d == 0 && eq_bytes(adj->key, adj->klen, "$SYS", 4)) continue;
      if (!has_next && adj->rplen != 0) retained_get(x, adj->retain_path, adj->rplen, out);
      if (has_next || (d >= 0 && is_hash)) scan_messages(x, filter, flen, d + 1, adj, out);
    }
    return;
  }
  const particle *p = (const particle *)smap_get(&n->particles, key, ln);
  if (p) {
    if (has_next) {
      scan_messages(x, filter, flen, d + 1, p, out);
      return;
    }
    retained_get(x, p->retain_path, p->rplen, out);
  }
}

static int cmp_u64(const void *a, const void *b) {
  uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
  return (x > y) - (x < y);
}

typedef struct {
  oref *x;
  const char *bytes;
  const uint64_t *offs;
  uint32_t lo, hi;
  uint32_t *count;
  const uint64_t *moffs;
  uint64_t *out;
} mjob_t;

static void *messages_worker(void *arg) {
  mjob_t *j = (mjob_t *)arg;
  u64vec v = {0, 0, 0};
  for (uint32_t i = j->lo; i < j->hi; i++) {
    v.n = 0;
    scan_messages(j->x, j->bytes + j->offs[i], (uint32_t)(j->offs[i + 1] - j->offs[i]), 0, NULL, &v);
    qsort(v.v, v.n, sizeof(uint64_t), cmp_u64);
    if (j->out)
      memcpy(j->out + j->moffs[i], v.v, sizeof(uint64_t) * v.n);
    else
      j->count[i] = v.n;
  }
  free(v.v);
  return NULL;
}

static int run_messages(oref *x, const char *bytes, const uint64_t *offs, uint32_t n, int nthreads,
                        uint32_t *count, const uint64_t *moffs, uint64_t *out) {
  if (nthreads < 1) nthreads = 1;
  if ((uint32_t)nthreads > n) nthreads = n ? (int)n : 1;
  mjob_t *jobs = (mjob_t *)calloc((size_t)nthreads, sizeof(mjob_t));
  pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) {
    jobs[t].x = x;
    jobs[t].bytes = bytes;
    jobs[t].offs = offs;
    jobs[t].count = count;
    jobs[t].moffs = moffs;
    jobs[t].out = out;
    jobs[t].lo = (uint32_t)((uint64_t)n * (uint64_t)t / (uint64_t)nthreads);
    jobs[t].hi = (uint32_t)((uint64_t)n * (uint64_t)(t + 1) / (uint64_t)nthreads);
    pthread_create(&th[t], NULL, messages_worker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(jobs);
  free(th);
  return 0;
}

int oref_messages_counts(oref *x, const char *bytes, const uint64_t *offs, uint32_t n, int nthreads,
                         uint32_t *count) {
  return run_messages(x, bytes, offs, n, nthreads, count, NULL, NULL);
}

int oref_messages_fill(oref *x, const char *bytes, const uint64_t *offs, uint32_t n, int nthreads,
                       const uint64_t *moffs, uint64_t *out) {
  return run_messages(x, bytes, offs, n, nthreads, NULL, moffs, out);
}
