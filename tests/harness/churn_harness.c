/*
 * tests/harness/churn_harness.c — Subscribers(topic) from many threads while
 * another thread keeps subscribing and unsubscribing, against one index with
 * the per-publish server on (MQM_CFG_SERVE).
 *
 * Test infrastructure (built on the CPU by tests/harness/Makefile, run on the
 * GPU by tests/test_gpu_serve_churn.py).  It links only include/mqmatch.h's
 * ABI.  The reference runs Subscribe (server.go:1013 -> topics.go:303-321,
 * under the trie's root mutex) concurrently with Subscribers
 * (server.go:776, one goroutine per connection, listeners/tcp.go:83); here
 * every result reports the snapshot version it was matched on
 * (mqm_result_snapshot_version), and the test compares it with the oracle
 * replayed up to exactly that version.
 *
 *   churn_harness IN OUT THREADS CALLS MODE OP_US
 *   IN  : "n_base n_ops n_topics\n"; n_base lines
 *         "client\tfilter\tqos\tnl\trap\trh\tident"; n_ops lines
 *         "S\tclient\tfilter\tqos\tnl\trap\trh\tident" or "U\tfilter\tclient";
 *         n_topics lines "topic"
 *   MODE: "autocommit" (AUTOCOMMIT | IDENTIFIERS | SERVE: every call commits
 *         the mutations before it, read-your-writes) or "async"
 *         (ASYNC_COMMIT | IDENTIFIERS | SERVE, rebuilt in the background by
 *         mqm_commit_policy(64 ops, 2 ms): calls match the newest published
 *         snapshot) or "fresh" (async + MQM_CFG_FRESH: calls return the
 *         store's current subscriptions less at most the last millisecond of
 *         mutations under load; the test checks that bound from the times)
 *   OP_US: microseconds the mutator sleeps between operations
 *   OUT : "B version" (after the base subscriptions), "V j version us" after
 *         operation j (us: microseconds since the start, after the call
 *         returned), then per call "C thread call topic version us" (us: when
 *         the call started) followed by
 *         that result's rendered lines (shim_harness.c's format:
 *         "D t client qos nl filter ident rap rh f1=i1,..." / "H t filter client")
 * Reader thread r makes CALLS calls on topics (r * 7919 + c * 104729) mod
 * n_topics.  A reader in "autocommit" mode also checks read-your-writes: the
 * version of a result is at least the store version it read before the call.
 * Exit status 0 when every call returned MQM_OK and every check held.
 */
#include <pthread.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

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
static uint32_t n_topics, n_calls;
static int n_threads, autocommit, fresh;
static volatile int failed;
static Buf *out_of;  /* per reader thread */

static void fail(const char *what) {
  fprintf(stderr, "churn_harness: %s\n", what);
  failed = 1;
}

static void name_of(int is_client, uint32_t id, char *buf, size_t cap) {
  size_t len = 0;
  int rc = is_client ? mqm_client_name(H, id, buf, cap - 1, &len) : mqm_filter_name(H, id, buf, cap - 1, &len);
  if (rc != MQM_OK) {
    fail("name lookup");
    len = 0;
  }
  buf[len < cap - 1 ? len : cap - 1] = 0;
}

typedef struct {
  char f[256];
  int32_t id;
} IdPair;

static int cmp_pair(const void *a, const void *b) { return strcmp(((const IdPair *)a)->f, ((const IdPair *)b)->f); }

/* topic 0 of single-topic result r, rendered as topic t (shim_harness.c) */
static void render(Buf *b, mqm_result *r, uint32_t t) {
  const uint64_t *off = mqm_result_offsets(r);
  const mqm_delivery *d = mqm_result_deliveries(r);
  const uint64_t *ioff = NULL;
  const uint32_t *isid = NULL;
  if (mqm_result_identifiers(r, &ioff, &isid) != MQM_OK) {
    fail("mqm_result_identifiers");
    return;
  }
  for (uint64_t j = off[0]; j < off[1]; j++) {
    mqm_sub_info first;
    if (mqm_result_sub_info(r, MQM_DELIVERY_SUB(d[j].packed), &first) != MQM_OK) {
      fail("mqm_result_sub_info");
      return;
    }
    char cl[256];
    name_of(1, d[j].client, cl, sizeof cl);
    IdPair *ids = malloc(sizeof(IdPair) * (1 + ioff[1] - ioff[0]));
    size_t ni = 0;
    name_of(0, first.filter, ids[0].f, sizeof ids[0].f);
    ids[0].id = first.identifier;
    ni = 1;
    for (uint64_t q = ioff[0]; q < ioff[1]; q++) {
      mqm_sub_info s;
      if (mqm_result_sub_info(r, isid[q], &s) != MQM_OK) {
        fail("mqm_result_sub_info (ident)");
        break;
      }
      if (s.client != d[j].client) continue;
      name_of(0, s.filter, ids[ni].f, sizeof ids[ni].f);
      ids[ni].id = s.identifier;
      int dup = 0;
      for (size_t z = 0; z < ni; z++)
        if (!strcmp(ids[z].f, ids[ni].f)) {
          ids[z].id = s.identifier;
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
  for (uint64_t j = soff[0]; j < soff[1]; j++) {
    mqm_sub_info s;
    if (mqm_result_shared_info(r, sh[j], &s) != MQM_OK) {
      fail("mqm_result_shared_info");
      return;
    }
    char fn[256], cl[256];
    name_of(0, s.filter, fn, sizeof fn);
    name_of(1, s.client, cl, sizeof cl);
    buf_fmt(b, "H %u %s %s\n", t, fn, cl);
  }
}

static struct timespec t_start;
static uint64_t now_us(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (uint64_t)(t.tv_sec - t_start.tv_sec) * 1000000u + (uint64_t)((t.tv_nsec - t_start.tv_nsec) / 1000);
}

static uint64_t store_version(void) {
  mqm_commit_state st;
  if (mqm_commit_state_get(H, &st) != MQM_OK) fail("mqm_commit_state_get");
  return st.store_version;
}

static void *reader(void *arg) {
  const int id = (int)(intptr_t)arg;
  Buf *b = &out_of[id];
  for (uint32_t c = 0; c < n_calls; c++) {
    const uint32_t t = (uint32_t)(((uint64_t)id * 7919u + (uint64_t)c * 104729u) % n_topics);
    const uint64_t t_call = now_us();
    const uint64_t before = autocommit ? store_version() : 0;
    mqm_result *r = NULL;
    if (mqm_subscribers(H, topics[t], topic_len[t], &r) != MQM_OK || mqm_result_num_topics(r) != 1) {
      fail("mqm_subscribers");
      if (r) mqm_result_free(r);
      continue;
    }
    const uint64_t v = mqm_result_snapshot_version(r);
    if (autocommit && v < before) {
      char msg[128];
      snprintf(msg, sizeof msg, "read-your-writes: result version %llu < store version %llu before the call",
               (unsigned long long)v, (unsigned long long)before);
      fail(msg);
    }
    buf_fmt(b, "C %d %u %u %llu %llu\n", id, c, t, (unsigned long long)v, (unsigned long long)t_call);
    render(b, r, t);
    mqm_result_free(r);
  }
  return NULL;
}

typedef struct {
  char kind;
  char *a, *b;  /* S: client, filter; U: filter, client */
  mqm_subscription sub;
} Op;

static Op *ops;
static uint32_t n_ops;
static unsigned op_us;
static Buf mut_out;

static void *mutator(void *arg) {
  (void)arg;
  for (uint32_t j = 0; j < n_ops; j++) {
    int x = 0;
    int rc = ops[j].kind == 'S'
                 ? mqm_subscribe(H, ops[j].a, strlen(ops[j].a), ops[j].b, strlen(ops[j].b), &ops[j].sub, &x)
                 : mqm_unsubscribe(H, ops[j].a, strlen(ops[j].a), ops[j].b, strlen(ops[j].b), &x);
    if (rc != MQM_OK) fail("mutation");
    buf_fmt(&mut_out, "V %u %llu %llu\n", j, (unsigned long long)store_version(), (unsigned long long)now_us());
    if (op_us) {
      struct timespec ts = {op_us / 1000000u, (long)(op_us % 1000000u) * 1000L};
      nanosleep(&ts, NULL);
    }
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

static void read_sub(char **s, mqm_subscription *sub) {
  sub->qos = (uint8_t)atoi(next_field(s));
  sub->no_local = (uint8_t)atoi(next_field(s));
  sub->retain_as_published = (uint8_t)atoi(next_field(s));
  sub->retain_handling = (uint8_t)atoi(next_field(s));
  sub->identifier = atoi(next_field(s));
}

int main(int argc, char **argv) {
  if (argc != 7) {
    fprintf(stderr, "usage: %s IN OUT THREADS CALLS MODE OP_US\n", argv[0]);
    return 2;
  }
  n_threads = atoi(argv[3]);
  n_calls = (uint32_t)atoi(argv[4]);
  autocommit = strcmp(argv[5], "autocommit") == 0;
  fresh = strcmp(argv[5], "fresh") == 0;
  op_us = (unsigned)atoi(argv[6]);
  if (n_threads < 1 || n_threads > 128 || (!autocommit && !fresh && strcmp(argv[5], "async") != 0)) return 2;
  FILE *in = fopen(argv[1], "rb");
  FILE *out = fopen(argv[2], "wb");
  if (!in || !out) return 2;
  unsigned long nb = 0, no = 0, nt = 0;
  if (fscanf(in, "%lu %lu %lu\n", &nb, &no, &nt) != 3 || nt == 0) return 2;
  mqm_config cfg = {0, MQM_CFG_IDENTIFIERS | MQM_CFG_SERVE |
                           (autocommit ? MQM_CFG_AUTOCOMMIT : MQM_CFG_ASYNC_COMMIT) | (fresh ? MQM_CFG_FRESH : 0u)};
  if (mqm_create(&cfg, &H) != MQM_OK) {
    fprintf(stderr, "mqm_create failed\n");
    return 3;
  }
  if (!autocommit && mqm_commit_policy(H, 64, 2) != MQM_OK) return 3;
  char *line = NULL;
  size_t lcap = 0;
  ssize_t len;
  for (unsigned long i = 0; i < nb; i++) {
    if ((len = getline(&line, &lcap, in)) < 0) return 2;
    if (len && line[len - 1] == '\n') line[--len] = 0;
    char *s = line;
    char *client = next_field(&s), *filter = next_field(&s);
    mqm_subscription sub;
    read_sub(&s, &sub);
    int is_new = 0;
    if (mqm_subscribe(H, client, strlen(client), filter, strlen(filter), &sub, &is_new) != MQM_OK) fail("subscribe");
  }
  if (mqm_commit(H) != MQM_OK) fail("mqm_commit");
  fprintf(out, "B %llu\n", (unsigned long long)store_version());
  n_ops = (uint32_t)no;
  ops = calloc(no + 1, sizeof(Op));
  for (unsigned long j = 0; j < no; j++) {
    if ((len = getline(&line, &lcap, in)) < 0) return 2;
    if (len && line[len - 1] == '\n') line[--len] = 0;
    char *s = line;
    ops[j].kind = next_field(&s)[0];
    ops[j].a = strdup(next_field(&s));
    ops[j].b = strdup(next_field(&s));
    if (ops[j].kind == 'S') read_sub(&s, &ops[j].sub);
  }
  n_topics = (uint32_t)nt;
  topics = calloc(nt + 1, sizeof(char *));
  topic_len = calloc(nt + 1, sizeof(size_t));
  for (unsigned long i = 0; i < nt; i++) {
    if ((len = getline(&line, &lcap, in)) < 0) return 2;
    if (len && line[len - 1] == '\n') line[--len] = 0;
    topics[i] = strndup(line, (size_t)len);
    topic_len[i] = (size_t)len;
  }
  free(line);
  out_of = calloc((size_t)n_threads, sizeof(Buf));
  clock_gettime(CLOCK_MONOTONIC, &t_start);
  pthread_t th[128], mt;
  pthread_create(&mt, NULL, mutator, NULL);
  for (int i = 0; i < n_threads; i++) pthread_create(&th[i], NULL, reader, (void *)(intptr_t)i);
  for (int i = 0; i < n_threads; i++) pthread_join(th[i], NULL);
  pthread_join(mt, NULL);
  mqm_serve_counters sc;
  if (mqm_serve_counters_get(H, &sc) != MQM_OK) fail("mqm_serve_counters_get");
  fprintf(out, "S %llu %llu %llu %llu %llu %llu %llu %llu\n", (unsigned long long)sc.served,
          (unsigned long long)sc.fallbacks, (unsigned long long)sc.launches, (unsigned long long)sc.stale,
          (unsigned long long)sc.forced, (unsigned long long)sc.slot_timeouts, (unsigned long long)sc.result_timeouts,
          (unsigned long long)sc.skipped_slots);
  uint64_t st_checks = 0, st_cached = 0, st_memory = 0;
  if (mqm_debug_stamp_counts(&st_checks, &st_cached, &st_memory) == MQM_OK)
    fprintf(stderr, "stamp checks %llu, stale cached %llu, stale in memory %llu\n", (unsigned long long)st_checks,
            (unsigned long long)st_cached, (unsigned long long)st_memory);
  if (mut_out.n) fwrite(mut_out.p, 1, mut_out.n, out);
  for (int i = 0; i < n_threads; i++)
    if (out_of[i].n) fwrite(out_of[i].p, 1, out_of[i].n, out);
  fclose(out);
  mqm_destroy(H);
  if (failed) fprintf(stderr, "a call or check failed\n");
  return failed ? 1 : 0;
}
