/*
 * tests/harness/shim_harness.c — the Go shim's call sequence
 * in C, from several threads at once, against one index.
 *
 * Test infrastructure (built on the CPU by tests/harness/Makefile, run on the
 * GPU by tests/test_gpu_shim.py).  It links only include/mqmatch.h's ABI —
 * exactly what the cgo binding would call — and renders every result the way
 * the shim builds `*Subscribers` (topics.go:247-252): per delivery the merged
 * packets.Subscription (client, Qos, NoLocal, Filter, Identifier,
 * RetainAsPublished, RetainHandling, Identifiers map: packets.go:250-270) and
 * per topic the `Shared` map's (filter, client) pairs (topics.go:541-555).
 *
 *   shim_harness IN OUT THREADS
 *   IN : "n_subs n_topics\n", n_subs lines "client\tfilter\tqos\tnl\trap\trh\tident\n",
 *        n_topics lines "topic\n"
 *   OUT: "N i is_new" per Subscribe, then per topic (in topic order):
 *        "D t client qos nl filter ident rap rh f1=i1,f2=i2,..." and "H t filter client"
 *
 * Reader threads interleave the two call shapes the shim uses: odd threads
 * call mqm_subscribers (one Subscribers(topic) per call, server.go:776), even
 * threads call mqm_match_batch over small batches (the batching collector,
 * INTEGRATION.md).  Exit status 0 when every call returned MQM_OK.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mqmatch.h"

typedef struct {
  char *p;
  size_t n, cap;
} Buf;

static void buf_put(Buf *b, const char *s, size_t n) {
  if (b->n + n + 1 > b->cap) {
    b->cap = (b->n + n + 1) * 2;
    b->p = realloc(b->p, b->cap);
    if (!b->p) abort();
  }
  memcpy(b->p + b->n, s, n);
  b->n += n;
  b->p[b->n] = 0;
}

static void buf_fmt(Buf *b, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
#include <stdarg.h>
static void buf_fmt(Buf *b, const char *fmt, ...) {
  char tmp[1024];
  va_list ap;
  va_start(ap, fmt);
  int n = vsnprintf(tmp, sizeof tmp, fmt, ap);
  va_end(ap);
  if (n < 0) abort();
  if ((size_t)n >= sizeof tmp) n = sizeof tmp - 1;
  buf_put(b, tmp, (size_t)n);
}

static mqm_index *H;
static char **topics;
static size_t *topic_len;
static uint32_t n_topics;
static Buf *out_of;  /* per topic */
static int n_threads;
static volatile int failed;

static void name_of(int is_client, uint32_t id, char *buf, size_t cap) {
  size_t len = 0;
  int rc = is_client ? mqm_client_name(H, id, buf, cap - 1, &len) : mqm_filter_name(H, id, buf, cap - 1, &len);
  if (rc != MQM_OK) {
    failed = 1;
    len = 0;
  }
  buf[len < cap - 1 ? len : cap - 1] = 0;
}

typedef struct {
  char f[256];
  int32_t id;
} IdPair;

static int cmp_pair(const void *a, const void *b) { return strcmp(((const IdPair *)a)->f, ((const IdPair *)b)->f); }

/* render topic k of result r as topic t */
static void render(mqm_result *r, uint32_t k, uint32_t t) {
  Buf *b = &out_of[t];
  const uint64_t *off = mqm_result_offsets(r);
  const mqm_delivery *d = mqm_result_deliveries(r);
  const uint64_t *ioff = NULL;
  const uint32_t *isid = NULL;
  if (mqm_result_identifiers(r, &ioff, &isid) != MQM_OK) {
    failed = 1;
    return;
  }
  for (uint64_t j = off[k]; j < off[k + 1]; j++) {
    mqm_sub_info first;
    if (mqm_result_sub_info(r, MQM_DELIVERY_SUB(d[j].packed), &first) != MQM_OK) {
      failed = 1;
      return;
    }
    char cl[256];
    name_of(1, d[j].client, cl, sizeof cl);
    /* Identifiers map: {first.Filter: first.Identifier} + the client's other
     * gathered subscriptions with Identifier > 0 (packets.go:250-259) */
    IdPair *ids = malloc(sizeof(IdPair) * (1 + ioff[k + 1] - ioff[k]));
    size_t ni = 0;
    name_of(0, first.filter, ids[0].f, sizeof ids[0].f);
    ids[0].id = first.identifier;
    ni = 1;
    for (uint64_t q = ioff[k]; q < ioff[k + 1]; q++) {
      mqm_sub_info s;
      if (mqm_result_sub_info(r, isid[q], &s) != MQM_OK) {
        failed = 1;
        break;
      }
      if (s.client != d[j].client) continue;
      name_of(0, s.filter, ids[ni].f, sizeof ids[ni].f);
      ids[ni].id = s.identifier;
      int dup = 0;
      for (size_t z = 0; z < ni; z++)
        if (!strcmp(ids[z].f, ids[ni].f)) {
          ids[z].id = s.identifier;  /* a later map assignment keeps its key */
          dup = 1;
        }
      if (!dup) ni++;
    }
    qsort(ids, ni, sizeof(IdPair), cmp_pair);
    char fn[256];
    name_of(0, first.filter, fn, sizeof fn);
    buf_fmt(b, "D %u %s %u %u %s %d %u %u ", t, cl, MQM_DELIVERY_QOS(d[j].packed), MQM_DELIVERY_NOLOCAL(d[j].packed),
            fn, first.identifier, first.retain_as_published, first.retain_handling);
    for (size_t z = 0; z < ni; z++) buf_fmt(b, "%s%s=%d", z ? "," : "", ids[z].f, ids[z].id);
    buf_put(b, "\n", 1);
    free(ids);
  }
  const uint64_t *soff = mqm_result_shared_offsets(r);
  const uint32_t *sh = mqm_result_shared(r);
  for (uint64_t j = soff[k]; j < soff[k + 1]; j++) {
    mqm_sub_info s;
    if (mqm_result_shared_info(r, sh[j], &s) != MQM_OK) {
      failed = 1;
      return;
    }
    char fn[256], cl[256];
    name_of(0, s.filter, fn, sizeof fn);
    name_of(1, s.client, cl, sizeof cl);
    buf_fmt(b, "H %u %s %s\n", t, fn, cl);
  }
}

enum { kBatch = 61 };

static void *reader(void *arg) {
  const int id = (int)(intptr_t)arg;
  if (id & 1) {  /* Subscribers(topic), one call per publish */
    for (uint32_t t = (uint32_t)id; t < n_topics; t += (uint32_t)n_threads) {
      mqm_result *r = NULL;
      if (mqm_subscribers(H, topics[t], topic_len[t], &r) != MQM_OK || mqm_result_num_topics(r) != 1) {
        failed = 1;
        if (r) mqm_result_free(r);
        continue;
      }
      render(r, 0, t);
      mqm_result_free(r);
    }
  } else {  /* a collector's batches: window w of kBatch topics goes to even thread w % n_even */
    const uint32_t n_even = (uint32_t)(n_threads + 1) / 2, e = (uint32_t)id / 2;
    uint64_t offs[kBatch + 1];
    char *bytes = NULL;
    size_t cap = 0;
    for (uint32_t t0 = e * kBatch; t0 < n_topics; t0 += n_even * kBatch) {
      /* the window's topics, minus those the odd threads own */
      uint32_t ts[kBatch], n = 0;
      size_t need = 0;
      for (uint32_t t = t0; t < t0 + kBatch && t < n_topics; t++)
        if (((t % (uint32_t)n_threads) & 1) == 0) ts[n++] = t, need += topic_len[t];
      if (need + 1 > cap) {
        cap = (need + 1) * 2;
        bytes = realloc(bytes, cap);
      }
      offs[0] = 0;
      for (uint32_t i = 0; i < n; i++) {
        memcpy(bytes + offs[i], topics[ts[i]], topic_len[ts[i]]);
        offs[i + 1] = offs[i] + topic_len[ts[i]];
      }
      mqm_result *r = NULL;
      if (mqm_match_batch(H, bytes, offs, n, &r) != MQM_OK || mqm_result_num_topics(r) != n) {
        failed = 1;
        if (r) mqm_result_free(r);
        continue;
      }
      for (uint32_t i = 0; i < n; i++) render(r, i, ts[i]);
      mqm_result_free(r);
    }
    free(bytes);
  }
  return NULL;
}

static char *next_field(char **s) {
  char *p = *s, *q = strchr(p, '\t');
  if (q) {
    *q = 0;
    *s = q + 1;
  } else {
    *s = p + strlen(p);
  }
  return p;
}

int main(int argc, char **argv) {
  if (argc != 4 && argc != 5) {
    fprintf(stderr, "usage: %s IN OUT THREADS [batching]\n", argv[0]);
    return 2;
  }
  n_threads = atoi(argv[3]);
  if (n_threads < 1 || n_threads > 64) return 2;
  FILE *in = fopen(argv[1], "rb");
  FILE *out = fopen(argv[2], "wb");
  if (!in || !out) return 2;
  unsigned long ns = 0, nt = 0;
  if (fscanf(in, "%lu %lu\n", &ns, &nt) != 2) return 2;
  mqm_config cfg = {0, MQM_CFG_AUTOCOMMIT | MQM_CFG_IDENTIFIERS};
  /* "batching": the shim's per-connection Subscribers calls go through the
   * library's collector (MQM_CFG_BATCHING), as a broker with many
   * connections would run it */
  if (argc == 5 && strcmp(argv[4], "batching") == 0) cfg.flags |= MQM_CFG_BATCHING;
  if (mqm_create(&cfg, &H) != MQM_OK) {
    fprintf(stderr, "mqm_create failed\n");
    return 3;
  }
  char *line = NULL;
  size_t lcap = 0;
  ssize_t len;
  for (unsigned long i = 0; i < ns; i++) {
    if ((len = getline(&line, &lcap, in)) < 0) return 2;
    if (len && line[len - 1] == '\n') line[--len] = 0;
    char *s = line;
    char *client = next_field(&s), *filter = next_field(&s);
    mqm_subscription sub;
    sub.qos = (uint8_t)atoi(next_field(&s));
    sub.no_local = (uint8_t)atoi(next_field(&s));
    sub.retain_as_published = (uint8_t)atoi(next_field(&s));
    sub.retain_handling = (uint8_t)atoi(next_field(&s));
    sub.identifier = atoi(next_field(&s));
    int is_new = 0;
    if (mqm_subscribe(H, client, strlen(client), filter, strlen(filter), &sub, &is_new) != MQM_OK) failed = 1;
    fprintf(out, "N %lu %d\n", i, is_new);
  }
  n_topics = (uint32_t)nt;
  topics = calloc(nt + 1, sizeof(char *));
  topic_len = calloc(nt + 1, sizeof(size_t));
  out_of = calloc(nt + 1, sizeof(Buf));
  for (unsigned long i = 0; i < nt; i++) {
    if ((len = getline(&line, &lcap, in)) < 0) return 2;
    if (len && line[len - 1] == '\n') line[--len] = 0;
    topics[i] = strndup(line, (size_t)len);
    topic_len[i] = (size_t)len;
  }
  free(line);
  /* the first match commits (AUTOCOMMIT); every later reader shares that snapshot */
  pthread_t th[64];
  for (int i = 0; i < n_threads; i++) pthread_create(&th[i], NULL, reader, (void *)(intptr_t)i);
  for (int i = 0; i < n_threads; i++) pthread_join(th[i], NULL);
  for (uint32_t t = 0; t < n_topics; t++)
    if (out_of[t].n) fwrite(out_of[t].p, 1, out_of[t].n, out);
  fclose(out);
  mqm_destroy(H);
  if (failed) fprintf(stderr, "a call failed\n");
  return failed ? 1 : 0;
}
