/*
 * oracle/mochi_ref.h — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference's subscription/retained topic index
 * (`TopicsIndex`, vendored mochi-co/mqtt v2.2.12 under
 * /root/reference/vendor/github.com/mochi-co/mqtt/v2/topics.go:284-699, and
 * `Subscription.Merge`, .../packets/packets.go:248-270).
 *
 * It is the CHECKER for the HIP product path and the CPU baseline timed by
 * bench.py ("kind": "port").  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product library
 * (libmqmatch.so) never links or calls it.
 *
 * Parity pinning: the reference is Go and no Go toolchain exists in this
 * image or on the GPU box, so the reference cannot be executed.  This
 * restatement is pinned by (1) the known-answer table derived by hand from
 * topics.go (tests/golden/kat_*.json), (2) the reference's own
 * system-test routing fixtures (tests/system/mqtt_test.go:84-253), and (3) a
 * second, independent pure-Python restatement (oracle/mochi_ref.py) that the
 * CPU test-suite cross-checks against this one on random workloads.  Beyond
 * those, parity is "unpinned by an executable reference" (DESIGN.md §Oracle).
 *
 * Identity contract shared with the product: client ids and filter ids are
 * dense u32s assigned in order of first appearance in Subscribe calls.
 */
#ifndef MOCHI_REF_H
#define MOCHI_REF_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oref oref;

typedef struct {
  uint32_t client;        /* interned client id                                 */
  uint32_t first_filter;  /* filter id of the first-merged subscription (M3)     */
  int32_t first_ident;    /* Identifier of that subscription                     */
  uint8_t qos;            /* max QoS over matched subs (M1)                       */
  uint8_t no_local;       /* OR over matched subs (M2)                            */
  uint8_t rap;            /* RetainAsPublished of the first                       */
  uint8_t rh;             /* RetainHandling of the first                          */
} oref_delivery;

typedef struct {
  uint32_t filter;        /* full shared filter string id ($SHARE/g/...)          */
  uint32_t client;
  uint8_t qos;
  uint8_t pad[3];
} oref_shared;

/* one entry of a delivery's Subscription.Identifiers map (packets.go:250-258) */
typedef struct {
  uint32_t client;        /* the delivery's client                                */
  uint32_t filter;        /* map key: Subscription.Filter (interned)              */
  int32_t ident;          /* map value: Subscription.Identifier                   */
} oref_ident;

typedef struct {
  uint64_t topics;        /* N: topics matched                                    */
  uint64_t topic_bytes;   /* T                                                    */
  uint64_t probes;        /* P: child probes (3 per expanded level + 1 '#' per literal hit) */
  uint64_t visits;        /* V: probe hits                                        */
  uint64_t gathered;      /* S: subscription entries gathered (non-shared + shared) */
  uint64_t deliveries;    /* D: non-shared (topic, client) pairs after merge      */
  uint64_t shared;        /* shared (topic, filter, client) candidates            */
} oref_stats;

oref *oref_new(void);
void oref_free(oref *x);

/* TopicsIndex.Subscribe (topics.go:303-321).  Returns 1 if new, 0 if it
 * replaced an existing subscription of the same client at the same node. */
int oref_subscribe(oref *x, const char *client, uint32_t clen, const char *filter, uint32_t flen,
                   uint8_t qos, uint8_t no_local, uint8_t rap, uint8_t rh, int32_t ident);
/* n Subscribe calls in order (string i = bytes[offs[i] .. offs[i+1])) */
void oref_subscribe_many(oref *x, uint64_t n, const char *cbytes, const uint64_t *coffs, const char *fbytes,
                         const uint64_t *foffs, const uint8_t *qos, const uint8_t *no_local, const uint8_t *rap,
                         const uint8_t *rh, const int32_t *ident);
/* TopicsIndex.Unsubscribe (topics.go:325-349). */
int oref_unsubscribe(oref *x, const char *filter, uint32_t flen, const char *client, uint32_t clen);
/* TopicsIndex.RetainMessage (topics.go:354-377).  msg_ref identifies the
 * caller's packet; payload_len==0 deletes. */
int64_t oref_retain(oref *x, const char *topic, uint32_t tlen, uint64_t msg_ref, uint32_t payload_len,
                    uint8_t retain_flag);

/* n RetainMessage calls in order (topic i = bytes[offs[i] .. offs[i+1])) */
void oref_retain_many(oref *x, uint64_t n, const char *bytes, const uint64_t *offs, const uint64_t *msg_refs,
                      uint32_t payload_len);

uint32_t oref_num_clients(const oref *x);
uint32_t oref_num_filters(const oref *x);
/* copies the interned string (no NUL) into buf; returns its length */
uint32_t oref_filter_name(const oref *x, uint32_t id, char *buf, uint32_t cap);
uint32_t oref_client_name(const oref *x, uint32_t id, char *buf, uint32_t cap);
uint64_t oref_retained_len(const oref *x);

/* Subscribers() over a batch: topic i is bytes[offs[i] .. offs[i+1]).
 * Phase 1: per-topic counts (deliveries, shared candidates). */
int oref_match_counts(oref *x, const char *bytes, const uint64_t *offs, uint32_t n, int nthreads,
                      uint32_t *dcount, uint32_t *scount, oref_stats *stats);
/* Phase 2: fill at caller-provided exclusive offsets.  Deliveries are sorted
 * by client id, shared candidates by (filter, client). */
int oref_match_fill(oref *x, const char *bytes, const uint64_t *offs, uint32_t n, int nthreads,
                    const uint64_t *doffs, oref_delivery *dout, const uint64_t *soffs, oref_shared *sout);

/* Subscription.Identifiers of every delivery (rule M3): per topic, the
 * (client, filter, ident) entries of all its deliveries' maps, sorted by
 * (client, filter).  A map holds {first.Filter: first.Identifier} (even when
 * 0) and {n.Filter: n.Identifier} for every other gathered subscription n of
 * the client with n.Identifier > 0.  Phase 1 counts, phase 2 fills. */
int oref_match_ident_counts(oref *x, const char *bytes, const uint64_t *offs, uint32_t n, int nthreads,
                            uint32_t *icount);
int oref_match_ident_fill(oref *x, const char *bytes, const uint64_t *offs, uint32_t n, int nthreads,
                          const uint64_t *ioffs, oref_ident *iout);

/* Messages() over a batch of filters (topics.go:426-480): msg_refs per filter,
 * sorted ascending (the reference's order is map iteration order). */
int oref_messages_counts(oref *x, const char *bytes, const uint64_t *offs, uint32_t n, int nthreads,
                         uint32_t *count);
int oref_messages_fill(oref *x, const char *bytes, const uint64_t *offs, uint32_t n, int nthreads,
                       const uint64_t *moffs, uint64_t *out);

/* isolateParticle (topics.go:558-577), exported for the known-answer tests.
 * Writes the particle byte range into start and len and returns hasNext. */
int oref_isolate_particle(const char *s, uint32_t slen, int d, uint32_t *start, uint32_t *len);

#ifdef __cplusplus
}
#endif
#endif
