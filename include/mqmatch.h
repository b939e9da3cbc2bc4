/*
 * mqmatch.h — C ABI of the MI355X-native MQTT publish-routing matcher.
 *
 * Drop-in boundary for mochi-co/mqtt v2.2.12 `TopicsIndex` as vendored by
 * gsalomao/maxmq (reference paths below are relative to
 * vendor/github.com/mochi-co/mqtt/v2/).  The reference exposes a concrete Go
 * type reached through `Server.Topics *TopicsIndex` (server.go:111, created at
 * server.go:149); a cgo shim implements that type's method set over these
 * functions.
 *
 * Conventions
 *   - Every function returns an int status (MQM_OK == 0, < 0 on error) and
 *     never aborts across the ABI.  Boolean/int64 results of the reference
 *     methods come back through out-parameters.
 *   - Strings are (pointer, length) byte ranges, borrowed for the call.
 *   - Client ids and filter ids are dense uint32 values assigned in order of
 *     first appearance in mqm_subscribe (stable for the index's lifetime).
 *   - Mutations go to the host-authoritative store; matching reads the last
 *     committed GPU snapshot (mqm_commit).  With MQM_CFG_AUTOCOMMIT a match
 *     first commits pending mutations, giving the reference's
 *     read-your-writes visibility (topics.go takes no snapshot at all).
 *   - The match path runs on the GPU only.  There is no CPU fallback: without
 *     a usable HIP device mqm_create fails with MQM_ENODEV.
 *   - Threading (the reference calls Subscribers() concurrently from every
 *     connection goroutine, listeners/tcp.go:83): mutations and commits
 *     serialise on the index mutex (topics.go:304,326,355 take the root
 *     mutex).  The host-path matches (mqm_match_batch, mqm_subscribers,
 *     mqm_messages_batch, mqm_messages_one) may be called from any number of
 *     threads at once: each borrows its own workspace and HIP stream and reads
 *     the published snapshot without holding the mutex (a commit that
 *     publishes a new snapshot does not wait for them).  The device-result
 *     calls (mqm_match_device, mqm_dense_device, mqm_identifiers_device,
 *     mqm_messages_device) share one library-owned result area per index and
 *     serialise on it.
 */
#ifndef MQMATCH_H
#define MQMATCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MQM_OK 0
#define MQM_EINVAL -1  /* bad handle / argument                               */
#define MQM_ENOMEM -2  /* host or device allocation failed                      */
#define MQM_EHIP -3    /* HIP runtime error                                     */
#define MQM_ELIMIT -4  /* a documented capacity limit was exceeded              */
#define MQM_ENODEV -5  /* no HIP device                                         */

#define MQM_CFG_AUTOCOMMIT 1u
/* mqm_match_batch also returns Identifiers support (mqm_result_identifiers) */
#define MQM_CFG_IDENTIFIERS 2u
/* MQM_CFG_ASYNC_COMMIT: every mutation is also appended to a delta log; a
 * commit hands the log to a background builder thread that replays it into a
 * shadow store, flattens it and uploads the new snapshot on its own HIP stream
 * (the back buffer) while matches keep reading the front buffer.  Matches
 * publish a finished back buffer at their start (no wait).  mqm_commit keeps
 * its synchronous meaning (submit, wait, publish).  See mqm_commit_async. */
#define MQM_CFG_ASYNC_COMMIT 4u
/* MQM_CFG_BATCHING: mqm_subscribers calls from concurrent threads (the
 * reference's one-goroutine-per-connection Subscribers(topic) calls,
 * listeners/tcp.go:83, server.go:776) are gathered by a collector thread into
 * one mqm_match_batch; each caller gets its own single-topic result.  Calls
 * arriving while a batch runs form the next batch (no added latency when
 * idle; mqm_batching_policy can add a linger).  Results are identical. */
#define MQM_CFG_BATCHING 8u
/* MQM_CFG_SERVE: mqm_subscribers calls go to a persistent GPU server instead
 * (the per-publish call shape with no kernel launch and no stream
 * synchronisation per call): the caller writes its topic into a ring slot in
 * pinned host memory, one of the server's resident workgroups claims it, runs
 * the small-batch path's per-topic match straight into the slot and flags it
 * done; the caller spins on that flag.  The server occupies `grid` CUs while
 * it runs and exits after `idle_us` without a call (relaunched on the next);
 * mqm_serve_policy sets both (default 32 workgroups, 20000 us).  Topics or
 * results past a slot's capacities take the batch path.  Results are
 * identical.  Takes precedence over MQM_CFG_BATCHING. */
#define MQM_CFG_SERVE 16u
/* MQM_CFG_FRESH (with MQM_CFG_ASYNC_COMMIT): mqm_subscribers returns the
 * store's current subscriptions, as the reference's live trie does
 * (topics.go:303-321, 484-518), without waiting for a rebuild: a result
 * matched on the published snapshot is corrected on the host for the clients
 * a mutation touched since that snapshot (their rows dropped, then recomputed
 * from their current subscriptions by the reference's scan and merge), and
 * mqm_result_snapshot_version reports the store version the result reflects.
 * Corrected results carry subscription ids past the snapshot's; resolve them
 * with mqm_result_sub_info / mqm_result_shared_info as usual.  Batch calls
 * (mqm_match_batch*, mqm_match_device) keep the snapshot's view.  Costs: each
 * publish builds a by-client index of the snapshot; each mutation updates the
 * overlay under the index mutex; a call on a stale snapshot adds a host scan
 * of the touched clients' subscriptions.  Corrections start with the first
 * publish; the clients mutated after that snapshot was built are then read
 * from the store once (one pass over its nodes, under the index mutex). */
#define MQM_CFG_FRESH 32u
/* device value for a host-only index: the store and its mutation API work,
 * mqm_commit / mqm_match_* return MQM_ENODEV (there is no CPU match path). */
#define MQM_DEVICE_NONE (-1)

typedef struct mqm_index mqm_index;   /* replaces *TopicsIndex               */
typedef struct mqm_result mqm_result; /* one batch's host-side match result   */
typedef struct mqm_messages mqm_messages; /* one batch's retained-message result */

typedef struct {
  int device;     /* HIP device ordinal, or MQM_DEVICE_NONE                    */
  uint32_t flags; /* MQM_CFG_*                                                 */
} mqm_config;

/* packets.Subscription fields the index reads (packets/packets.go:168-178) */
typedef struct {
  uint8_t qos;                 /* 0..2 (SubscribeDecode enforces, :953)        */
  uint8_t no_local;            /* MQTT 5 No Local                              */
  uint8_t retain_as_published; /* MQTT 5 RAP                                   */
  uint8_t retain_handling;     /* MQTT 5 RH (0..2)                             */
  int32_t identifier;          /* subscription identifier (0 = none)          */
} mqm_subscription;

/* One merged non-shared delivery (topics.go:531-536 + packets.go:250-270).
 *   client   : interned client id
 *   packed   : first_sub (bits 0..27) | qos << 28 (2 bits) | no_local << 30
 *              first_sub names the first-merged subscription; resolve it with
 *              mqm_result_sub_info. */
typedef struct {
  uint32_t client;
  uint32_t packed;
} mqm_delivery;

#define MQM_DELIVERY_SUB(p) ((p) & 0x0FFFFFFFu)
#define MQM_DELIVERY_QOS(p) (((p) >> 28) & 3u)
#define MQM_DELIVERY_NOLOCAL(p) (((p) >> 30) & 1u)

typedef struct {
  uint32_t filter;             /* filter id                                    */
  uint32_t client;             /* client id                                    */
  int32_t identifier;
  uint8_t qos, no_local, retain_as_published, retain_handling;
} mqm_sub_info;

/* Device-resident result of mqm_match_device (library-owned; valid until the
 * next mqm_match_device / mqm_messages_device call on the same index).  Topic t's deliveries are
 * deliveries[starts[t] .. starts[t] + counts[t]) and its shared candidates
 * shared[shared_starts[t] .. + shared_counts[t]).  Segments are in topic
 * order but may leave gaps (a topic reserves its raw-entry count before
 * deduplication); mqm_match_batch / mqm_dense_device return the dense form.
 * A device delivery is 4 bytes, the `packed` word of mqm_delivery
 * (first_sub | qos << 28 | no_local << 30): the delivery's client is the
 * client of its first-merged subscription (mqm_result_sub_info(...).client,
 * or the dense form, which carries it). */
typedef struct {
  uint32_t n_topics;
  uint64_t n_deliveries;          /* sum of counts                              */
  uint64_t n_shared;              /* sum of shared_counts                       */
  const uint64_t *starts;         /* device, n_topics                           */
  const uint32_t *counts;         /* device, n_topics                           */
  const uint32_t *deliveries;     /* device: packed (MQM_DELIVERY_SUB/QOS/NOLOCAL) */
  const uint64_t *shared_starts;  /* device, n_topics                           */
  const uint32_t *shared_counts;  /* device, n_topics                           */
  const uint32_t *shared;         /* device: shared-subscription ids            */
  uint32_t n_fallback;            /* topics routed through the unbounded path   */
  uint32_t n_big;                 /* topics deduplicated by the workgroup tier  */
  uint32_t fallback_why[5];       /* why topics took the unbounded path: frontier,
                                     hits, cached levels, shared hits, raw entries */
  uint32_t n_merge_small;         /* topics whose <= 24 multi entries an 8-lane group merged */
  uint32_t n_merge_wave;          /* topics whose <= 192 multi entries a wavefront merged */
  uint64_t n_solo_ranges;         /* solo copy ranges (hits with solo entries)    */
  uint32_t n_tier2, n_tier3;      /* topics the workgroup merge passed to its 2nd / 3rd tier */
  uint64_t multi_entries[3];      /* multi entries merged by the workgroup tiers 1 / 2 / 3 */
  uint32_t n_part;                /* tier-3 topics merged in client-hash partitions (> 3072 multi entries) */
  uint32_t n_resolve;             /* topics merged by resolution (partner lists, no table) */
  uint64_t n_solo;                /* solo entries: deliveries copied as they stand */
} mqm_device_result;

/* ---- lifecycle: NewTopicsIndex (topics.go:291-299) ---------------------- */
int mqm_create(const mqm_config *cfg, mqm_index **out);
int mqm_destroy(mqm_index *h);

/* ---- mutation ----------------------------------------------------------- */
/* TopicsIndex.Subscribe (topics.go:303-321): *is_new = !existed.  MQM_EINVAL
 * (nothing stored) for qos > 2 or retain_handling > 3: the snapshot packs them
 * in 2 bits each (the broker never passes more: packets.go:953). */
int mqm_subscribe(mqm_index *h, const char *client, size_t client_len, const char *filter, size_t filter_len,
                  const mqm_subscription *sub, int *is_new);
/* bulk form of the above for store reload (server.go:1377-1393); is_new may be
 * NULL.  Any record out of range: MQM_EINVAL and none is applied. */
int mqm_subscribe_many(mqm_index *h, size_t n, const char *client_bytes, const uint64_t *client_offs,
                       const char *filter_bytes, const uint64_t *filter_offs, const mqm_subscription *subs,
                       uint8_t *is_new);
/* TopicsIndex.Unsubscribe (topics.go:325-349): *existed = the reference's bool */
int mqm_unsubscribe(mqm_index *h, const char *filter, size_t filter_len, const char *client, size_t client_len,
                    int *existed);
/* Server.loadSubscriptions (server.go:1377-1393) over persisted records: json
 * holds storage.Subscription JSON records (hooks/storage/storage.go:151-161)
 * as a JSON array or as concatenated / newline-separated objects; each is
 * decoded with encoding/json's rules (case-insensitive keys, unknown keys
 * skipped, null = zero value) and Subscribed in order.  *n_loaded = records
 * applied, *n_new = how many Subscribe calls returned true.  MQM_EINVAL at
 * the first record encoding/json rejects, MQM_ELIMIT at one outside what the
 * snapshot stores (qos > 2, retain_handling > 3, identifier outside int32);
 * the records before it stay applied. */
int mqm_load_subscriptions_json(mqm_index *h, const char *json, size_t len, uint64_t *n_loaded, uint64_t *n_new);
/* n Unsubscribe calls in order (UnsubscribeClient at session expiry,
 * server.go:1109-1129); existed may be NULL */
int mqm_unsubscribe_many(mqm_index *h, size_t n, const char *filter_bytes, const uint64_t *filter_offs,
                         const char *client_bytes, const uint64_t *client_offs, uint8_t *existed);
/* TopicsIndex.RetainMessage (topics.go:354-377); message_ref is the caller's
 * handle for the packet; payload_len == 0 deletes.  *result = 1 / 0 / -1. */
int mqm_retain_message(mqm_index *h, const char *topic, size_t topic_len, uint64_t message_ref,
                       uint32_t payload_len, int retain_flag, int64_t *result);
/* n RetainMessage calls in order (retained-store reload, server.go:1430-1434);
 * retain_flags NULL = all set; results may be NULL */
int mqm_retain_many(mqm_index *h, size_t n, const char *topic_bytes, const uint64_t *topic_offs,
                    const uint64_t *message_refs, const uint32_t *payload_lens, const uint8_t *retain_flags,
                    int64_t *results);
/* Retained.Len() (packets.go:103) */
int mqm_retained_len(mqm_index *h, uint64_t *out);

/* publish the current store as the snapshot matches read, and wait for it.
 * A host-only index (MQM_DEVICE_NONE) builds the host side only (stats and
 * digest; matching still returns MQM_ENODEV). */
int mqm_commit(mqm_index *h);

/* ---- incremental commits (MQM_CFG_ASYNC_COMMIT; MQM_EINVAL otherwise) ------
 * The reference has no snapshot: a Subscribe is visible to the next
 * Subscribers call (topics.go:303-321, 484-518).  Here visibility starts when
 * the snapshot holding the mutation is published; mqm_commit, or
 * MQM_CFG_AUTOCOMMIT on a match, gives back read-your-writes. */
/* hand the mutations logged since the last submit to the builder; returns at
 * once.  Logs submitted while a build runs are coalesced into the next one. */
int mqm_commit_async(mqm_index *h);
/* publish the newest finished build, if any (*published = 1); wait != 0 first
 * waits until every submitted log is built.  Returns the first build error. */
int mqm_commit_poll(mqm_index *h, int wait, int *published);
/* periodic rebuild: submit automatically once max_ops mutations are logged or
 * the oldest logged one is max_ms old (checked at mutations and matches;
 * 0 disables a bound) */
int mqm_commit_policy(mqm_index *h, uint64_t max_ops, uint32_t max_ms);
typedef struct {
  uint64_t store_version;    /* mutations applied to the authoritative store   */
  uint64_t snapshot_version; /* store version the published snapshot reflects  */
  uint64_t pending_ops;      /* logged, not yet submitted                       */
  uint64_t builds;           /* snapshots published by the builder             */
  uint64_t last_build_ops;   /* delta-log entries folded into the last one      */
  double last_build_ms;      /* its replay + flatten + upload time              */
  int32_t has_snapshot, building;
} mqm_commit_state;
int mqm_commit_state_get(mqm_index *h, mqm_commit_state *out);
/* the last published build's phases (ms[5]): delta-log replay, flatten,
 * upload (ms), then the host threads a flatten runs on, then 1 if the build
 * kept the previous build's trie shape (preorder and edge list: no node was
 * created or removed since) */
int mqm_build_phases_ms(mqm_index *h, double *ms);
/* host threads for every flatten of this process (0: MQM_BUILD_THREADS, else
 * min(16, hardware threads), and at most 2 while a per-publish server
 * (MQM_CFG_SERVE) lives: a background build shares the CPUs with its callers,
 * DESIGN §9) */
int mqm_build_threads(uint32_t n);
/* 64-bit digest of the published snapshot's arrays: replicas and rebuilds of
 * the same store state have equal digests */
int mqm_snapshot_digest(mqm_index *h, uint64_t *out);
/* Fault injection for tests (async indexes only): the next `count` background
 * builds fail at `stage` — 1: part-way through the delta-log replay (as a
 * bad_alloc while interning would), 2: flatten, 3: upload.  A failed build is
 * reported by the next commit; the commit after it rebuilds (after a failed
 * replay, from a full copy of the authoritative store), so a failure never
 * leaves a stale snapshot published as current. */
int mqm_debug_fault(mqm_index *h, int stage, int count);

/* ---- forward match: TopicsIndex.Subscribers (topics.go:484-555) --------- */
/* Host in / host out.  Topic i is bytes[offsets[i] .. offsets[i+1]). */
int mqm_match_batch(mqm_index *h, const char *topic_bytes, const uint64_t *topic_offsets, uint32_t n_topics,
                    mqm_result **out);
/* The same with 4-byte deliveries: the result carries the packed words
 * (mqm_result_packed; mqm_result_deliveries is NULL).  A delivery's client is
 * its first-merged subscription's (mqm_result_sub_info(...).client, which a
 * caller resolving the Subscription fields reads anyway), so nothing is lost
 * and the device-to-host copy halves (the host path is PCIe-bound). */
int mqm_match_batch_packed(mqm_index *h, const char *topic_bytes, const uint64_t *topic_offsets, uint32_t n_topics,
                           mqm_result **out);
/* The runs form: the PCIe-bound host path without a 4-byte transfer per
 * delivery.  ~90 % of deliveries are solo entries (a subscription whose
 * client meets no other of its subscriptions in the topic is its client's
 * merged delivery as it stands, packets.go:250-270), and a gathered node's
 * solo entries are one contiguous run of the snapshot's packed-word table —
 * which the host built and keeps.  So a topic's deliveries are its runs,
 * words[run.off .. run.off + run.count) for runs[run_offsets[t] ..
 * run_offsets[t+1]) (mqm_result_runs), then its merged winners,
 * packed[offsets[t] .. offsets[t+1]) (mqm_result_offsets / _packed).
 * mqm_result_expand writes the plain packed rows of a topic range (e.g. one
 * range per consumer thread).  Only 8 B per run and 4 B per winner cross
 * PCIe.  Replaces Subscribers (topics.go:484-555) like mqm_match_batch; the
 * same sets, same Identifiers support. */
typedef struct {
  uint32_t off, count;
} mqm_run;
int mqm_match_batch_runs(mqm_index *h, const char *topic_bytes, const uint64_t *topic_offsets, uint32_t n_topics,
                         mqm_result **out);
/* single-topic convenience == Subscribers(topic) (batched across concurrent
 * callers with MQM_CFG_BATCHING) */
int mqm_subscribers(mqm_index *h, const char *topic, size_t topic_len, mqm_result **out);
/* MQM_CFG_BATCHING: at most max_batch topics per gathered batch (0 = 8192),
 * and how long the collector waits for more after the first (microseconds,
 * default 0); on an index created without the flag it turns batching on.
 * Statistics: batches run and topics they carried (MQM_EINVAL while batching
 * is off).  Both MQM_EINVAL on a host-only index.  Safe to call while other
 * threads are inside mqm_subscribers: the collector is published atomically,
 * and calls already past that point finish on the direct path. */
int mqm_batching_policy(mqm_index *h, uint32_t max_batch, uint32_t linger_us);
/* MQM_CFG_SERVE: the server's workgroups and idle timeout (applied at its
 * next launch; on an index created without the flag it turns serving on);
 * statistics: calls served in the ring, calls that took the batch path, server
 * launches.  MQM_EINVAL on a host-only index (or for stats while off). */
int mqm_serve_policy(mqm_index *h, uint32_t grid, uint32_t idle_us);
/* MQM_CFG_FRESH indexes: correct_calls = 0 makes mqm_subscribers return the
 * snapshot's view again and drops the overlay (mutations cost nothing extra;
 * A/B and measurement), 1 starts it again: at once when the published
 * snapshot holds every mutation, else at the first publish that does
 * (mqm_commit_async then mqm_commit_poll(wait) gives one); until then calls
 * return the snapshot's view, reporting its version.
 * Statistics (out[9]): clients held, overlay operations applied, applier
 * rounds, calls corrected, nanoseconds spent in the corrections' read
 * sections, the part of them in the overlay's scan, then the largest age of a
 * batch when the applier took it, the longest round and the longest wait for
 * a copy no call was in (ns).
 * MQM_EINVAL on an index created without the flag. */
int mqm_fresh_policy(mqm_index *h, int correct_calls);
int mqm_fresh_stats(mqm_index *h, uint64_t *out);
/* (grid is capped at half the device's CUs: a server under steady traffic
 * never idles out, and batch-path calls need the rest of the device) */
int mqm_serve_stats(mqm_index *h, uint64_t *served, uint64_t *fallbacks, uint64_t *launches);
/* the served path's safety nets, counted since the server started (a healthy
 * run has forced == slot_timeouts == result_timeouts == 0):
 *   served / fallbacks / launches: as mqm_serve_stats;
 *   stale: results whose snapshot's host copy was no longer kept (decoded
 *     again on the batch path: correct, slower);
 *   forced: relaunches because a posted request sat unserved for 1 s (a
 *     request number skipped by a counter restart, or a workgroup waiting on a
 *     request never posted);
 *   slot_timeouts: callers that found their ring slot still taken after 10 s
 *     (returned MQM_EHIP without posting);
 *   result_timeouts: callers that posted and saw no result for 10 s (returned
 *     MQM_EHIP; the slot goes to its next owner when the late result lands);
 *   skipped_slots: ring slots handed on past a ticket whose caller gave up
 *     before posting (slot_timeouts) */
typedef struct mqm_serve_counters {
  uint64_t served, fallbacks, launches, stale, forced, slot_timeouts, result_timeouts, skipped_slots;
} mqm_serve_counters;
int mqm_serve_counters_get(mqm_index *h, mqm_serve_counters *out);
/* diagnostics, MQM_SNAP_STAMP=1 (set before the first snapshot is uploaded):
 * every snapshot's version is stamped into its device buffers as the upload's
 * last step, and the per-publish kernels (server and small-batch path) compare
 * the stamps with the version they were launched for, per call.  Process-wide
 * counts: checks made, stamps found stale through the caches, stale in memory
 * (a buffer refilled for another snapshot while a reader ran on it). */
int mqm_debug_stamp_counts(uint64_t *checks, uint64_t *stale_cached, uint64_t *stale_memory);
/* mean device time per served call (us[4]): claim to published result, then
 * its phases: topic staged + level keys, trie walk, emission + publish */
int mqm_serve_device_us(mqm_index *h, double *us);
/* mean host time per served call since the previous call of this function
 * (us[4]; reads and resets): entry to request posted (snapshot check + slot
 * wait + topic copy), posted to result seen (device time + detection +
 * wake-up), result seen to return (result block built); then the share of
 * calls that slept on the completion poller instead of spinning */
int mqm_serve_host_us(mqm_index *h, double *us);
/* the longest served call per host phase since the previous call of this
 * function (us[8]; reads and resets): front buffer, server check / relaunch,
 * slot wait + post, result wait, result block, batch-path fallback; then the
 * number of calls over 10 ms, then 0 */
int mqm_serve_host_max_us(mqm_index *h, double *us);
int mqm_batching_stats(mqm_index *h, uint64_t *batches, uint64_t *topics);
/* single-topic calls on the direct path (no collector, no server: the
 * small-batch kernel per call) since the previous call of this function
 * (us[9]; reads and resets): mean time per phase — front buffer (commit check),
 * context from the pool, launch + wait for the kernel, result block — then the
 * maximum of each phase, then the number of calls */
int mqm_direct_host_us(mqm_index *h, double *us);
/* host-path calls through the batch pipeline (mqm_match_batch / _packed /
 * _runs, the SURVEY §8(d) end-to-end form) since the previous call of this
 * function (us[6]; reads and resets): mean time per phase — front buffer and
 * context, topics H2D (after the context's previous work), match (walk to
 * merges, collected), runs / identifiers / densify, result D2H + stream
 * synchronisation — then the number of calls */
int mqm_batch_host_us(mqm_index *h, double *us);
/* Device in / device out on `hip_stream` (hipStream_t, NULL = default stream). */
/* on != 0: every device match (mqm_match_device, queued contexts) computes
 * the Identifiers lists beside its merges (a second stream forked after the
 * walk), so a following mqm_identifiers_device only collects them; for a
 * caller that wants them after every batch.  Host-path matches of an
 * MQM_CFG_IDENTIFIERS index always do. */
int mqm_identifiers_early(mqm_index *h, int on);
int mqm_match_device(mqm_index *h, const uint8_t *d_topic_bytes, const uint64_t *d_topic_offsets,
                     uint32_t n_topics, void *hip_stream, mqm_device_result *out);

/* ---- queued device matching (steady state) ------------------------------
 * mqm_match_device waits for its batch.  A broker streaming batches through
 * the GPU keeps several in flight instead: each caller-owned context holds one
 * batch's pipeline state and results; mqm_match_device_async queues the whole
 * pipeline on hip_stream and returns without waiting (no host read-back
 * before the end: the outputs are sized from the context's earlier batches),
 * mqm_match_ctx_wait waits for it and returns its result (device buffers owned
 * by the context, valid until its next call).  A batch that outgrows the
 * buffers the earlier ones sized is run again inside mqm_match_ctx_wait, sized
 * exactly (mqm_match_ctx_stats counts those), so the topic buffers must stay
 * valid until the wait returns.  One batch in flight per context (a second
 * async call before the wait: MQM_EINVAL); contexts are independent, so
 * batches on different contexts and streams overlap.  The snapshot a batch
 * reads is the published one when it was queued.  A context reads its index:
 * destroy every context before the index (mqm_destroy returns MQM_EINVAL
 * while any is alive and leaves the index intact). */
typedef struct mqm_match_ctx mqm_match_ctx;
int mqm_match_ctx_create(mqm_index *h, mqm_match_ctx **out);
int mqm_match_ctx_destroy(mqm_match_ctx *ctx);
int mqm_match_device_async(mqm_match_ctx *ctx, const uint8_t *d_topic_bytes, const uint64_t *d_topic_offsets,
                           uint32_t n_topics, void *hip_stream);
int mqm_match_ctx_wait(mqm_match_ctx *ctx, mqm_device_result *out);
int mqm_match_ctx_stats(mqm_match_ctx *ctx, uint64_t *requeued);

/* ---- Subscription.Identifiers (packets.go:250-259, rule M3) -------------- */
/* Merge gives every delivery an Identifiers map: {first.Filter:
 * first.Identifier} (kept even when 0) plus {n.Filter: n.Identifier} for
 * every other subscription n of the client gathered for the topic with
 * n.Identifier > 0 (server.go:805-810 turns it into the PUBLISH's
 * subscription identifiers).  This pass returns, per topic, sids of gathered
 * non-shared subscriptions with Identifier > 0: at least every such
 * subscription of a client with more than one subscription in the topic's
 * gather (a subscription gathered twice — a '#' node reached by the parent
 * probe and by '#' — may repeat).  A client with one gathered subscription
 * gets the map {filter(first): ident(first)} alone, so its sid adds nothing
 * and the batch pipeline does not list it (the per-publish paths may).  The
 * map of delivery (topic, client) is {filter(first): ident(first)} plus
 * {filter(s): ident(s)} for the listed s whose client is that client
 * (resolve with mqm_result_sub_info).  Device form: for the last
 * mqm_match_device call on the index, whose topic buffers must still hold the
 * batch, against the snapshot that call read; MQM_EINVAL if there was none. */
typedef struct {
  uint32_t n_topics;
  uint64_t n_idents;
  const uint64_t *offsets; /* device, n_topics + 1 (exclusive prefix)          */
  const uint32_t *sids;    /* device: subscription ids                         */
} mqm_device_identifiers;
int mqm_identifiers_device(mqm_index *h, void *hip_stream, mqm_device_identifiers *out);
/* host form, filled by mqm_match_batch on an index created with
 * MQM_CFG_IDENTIFIERS (MQM_EINVAL otherwise); arrays owned by the result */
int mqm_result_identifiers(const mqm_result *r, const uint64_t **offsets, const uint32_t **sids);

/* ---- dense device form of the last mqm_match_device result --------------- */
/* Topic t's deliveries are deliveries[offsets[t] .. offsets[t+1]) (no gaps);
 * same for shared.  Library-owned, valid until the next device-result call on
 * the index; MQM_EINVAL if there was no device match.  Queued on hip_stream
 * after the match. */
typedef struct {
  uint32_t n_topics;
  uint64_t n_deliveries, n_shared;
  const uint64_t *offsets;        /* device, n_topics + 1                       */
  const mqm_delivery *deliveries; /* device                                     */
  const uint64_t *shared_offsets; /* device, n_topics + 1                       */
  const uint32_t *shared;         /* device                                     */
} mqm_device_dense;
int mqm_dense_device(mqm_index *h, void *hip_stream, mqm_device_dense *out);

/* ---- subscriber-sharded node result (server.go:1232 caller) --- */
/* Each of n_shards indexes (one per GPU) holds the subscriptions of a
 * contiguous client range; Subscription.Merge (packets.go:250-270) is per
 * client, so the shards' per-topic delivery sets are disjoint and final.
 * After the shards' dense CSRs (mqm_dense_device) have been gathered onto one
 * device (RCCL send/recv, maxmq_amd/shard.py), this lays them out as one
 * dense CSR: topic t = shard 0's segment, shard 1's, ...; client ids go
 * through each shard's client_map (shard client id -> node client id; NULL
 * keeps them).  packed.first_sub stays shard-local (resolve it on the
 * shard's index).  d_out_offsets: n_topics + 1; d_out: the sum of the
 * shards' delivery counts.  Synchronises hip_stream; MQM_EINVAL if a client
 * id fell outside its shard's map or n_shards is 0 or > 16. */
typedef struct {
  const uint64_t *offsets;        /* device, n_topics + 1                       */
  const mqm_delivery *deliveries; /* device                                     */
  const uint32_t *client_map;     /* device, n_map entries, or NULL             */
  uint32_t n_map;
} mqm_shard_part;
int mqm_gather_shards(uint32_t n_topics, uint32_t n_shards, const mqm_shard_part *parts, void *hip_stream,
                      uint64_t *d_out_offsets, mqm_delivery *d_out);
/* The shared-subscription candidates of the same shards (gatherSharedSubscriptions,
 * topics.go:541-555): a shared subscription belongs to its client's shard, so
 * the shards' candidate sets are disjoint too.  Each part is a shard's dense
 * shared CSR (mqm_device_dense.shared_offsets / .shared); topic t's node-wide
 * candidates are shard 0's, then shard 1's, ..., each entry
 * MQM_SHARD_SHARED(shard, id) with the shard-local shared id (resolve it on
 * that shard's index).  d_out_offsets: n_topics + 1; d_out: the sum of the
 * shards' candidate counts.  Synchronises hip_stream; MQM_EINVAL if an id
 * does not fit 28 bits or n_shards is 0 or > 16. */
typedef struct {
  const uint64_t *offsets; /* device, n_topics + 1                              */
  const uint32_t *shared;  /* device: shard-local shared-subscription ids       */
} mqm_shard_shared_part;
#define MQM_SHARD_SHARED(shard, id) (((uint32_t)(shard) << 28) | (uint32_t)(id))
#define MQM_SHARED_SHARD(v) ((v) >> 28)
#define MQM_SHARED_ID(v) ((v) & 0x0FFFFFFFu)
int mqm_gather_shards_shared(uint32_t n_topics, uint32_t n_shards, const mqm_shard_shared_part *parts,
                             void *hip_stream, uint64_t *d_out_offsets, uint32_t *d_out);

/* ---- reverse match: TopicsIndex.Messages (topics.go:426-480) ------------ */
/* The message refs retained under each filter (the message_ref given to
 * mqm_retain_message).  Within a filter the order is unspecified (the
 * reference returns Go map iteration order).  Filter i is
 * bytes[offsets[i] .. offsets[i+1]); the reference's callers pass one filter
 * per SUBSCRIBE topic (server.go:870-885). */
int mqm_messages_batch(mqm_index *h, const char *filter_bytes, const uint64_t *filter_offsets, uint32_t n_filters,
                       mqm_messages **out);
/* single-filter convenience == Messages(filter) */
int mqm_messages_one(mqm_index *h, const char *filter, size_t filter_len, mqm_messages **out);
uint32_t mqm_messages_num_filters(const mqm_messages *m);
const uint64_t *mqm_messages_offsets(const mqm_messages *m); /* n + 1 */
const uint64_t *mqm_messages_refs(const mqm_messages *m);
void mqm_messages_free(mqm_messages *m);

/* Device in / device out (library-owned; valid until the next call on the index). */
typedef struct {
  uint32_t n_filters;
  uint64_t n_refs;
  const uint64_t *offsets; /* device, n_filters + 1 */
  const uint64_t *refs;    /* device */
  uint64_t n_ranges;       /* emitted ranges (roofline bookkeeping)      */
  uint64_t n_items;        /* (filter, trie node) steps of the reference's recursion, all levels */
  uint64_t n_skipped;      /* ... of those, children the literal-edge index jumped over (not loaded) */
} mqm_device_messages;
int mqm_messages_device(mqm_index *h, const uint8_t *d_filter_bytes, const uint64_t *d_filter_offsets,
                        uint32_t n_filters, void *hip_stream, mqm_device_messages *out);

/* ---- result accessors --------------------------------------------------- */
uint32_t mqm_result_num_topics(const mqm_result *r);
/* the store version (mqm_commit_state.store_version) of the snapshot the
 * result was matched on: every mutation counted up to that version is in the
 * result, none after it.  The reference matches its live trie
 * (topics.go:484-518); a drop-in caller that needs to know which mutations a
 * result reflects reads this.  0 for NULL. */
uint64_t mqm_result_snapshot_version(const mqm_result *r); /* (MQM_CFG_FRESH: the store version it reflects) */
const uint64_t *mqm_result_offsets(const mqm_result *r);          /* n + 1          */
const mqm_delivery *mqm_result_deliveries(const mqm_result *r); /* NULL for a packed result */
const uint32_t *mqm_result_packed(const mqm_result *r);         /* packed words (mqm_match_batch_packed;
                                                                   the runs form: merged winners only) */
/* the runs form's solo runs and the snapshot's packed-word table they index
 * (owned by the result's snapshot); MQM_EINVAL for any other result */
int mqm_result_runs(const mqm_result *r, const uint64_t **run_offsets, const mqm_run **runs, const uint32_t **words,
                    uint64_t *n_words);
/* topics [t0, t1) of a packed or runs-form result as plain packed rows:
 * offsets[0 .. t1 - t0] (relative to dst), dst the rows back to back (NULL:
 * offsets only, to size dst).  Thread-safe on disjoint ranges. */
int mqm_result_expand(const mqm_result *r, uint32_t t0, uint32_t t1, uint64_t *offsets, uint32_t *dst);
const uint64_t *mqm_result_shared_offsets(const mqm_result *r);   /* n + 1          */
const uint32_t *mqm_result_shared(const mqm_result *r);           /* shared sub ids */
/* resolve a delivery's first_sub / a shared sub id (snapshot-relative) */
int mqm_result_sub_info(const mqm_result *r, uint32_t sub, mqm_sub_info *out);
int mqm_result_shared_info(const mqm_result *r, uint32_t shared_sub, mqm_sub_info *out);
/* batch forms: resolve n ids at once (shared != 0 selects the shared table) */
int mqm_result_sub_infos(const mqm_result *r, int shared, const uint32_t *subs, size_t n, mqm_sub_info *out);
void mqm_result_free(mqm_result *r);

/* ---- names -------------------------------------------------------------- */
/* copy up to cap bytes of the name into buf; *len = full length */
int mqm_client_name(mqm_index *h, uint32_t client, char *buf, size_t cap, size_t *len);
int mqm_filter_name(mqm_index *h, uint32_t filter, char *buf, size_t cap, size_t *len);
int mqm_num_clients(mqm_index *h, uint32_t *out);

/* ---- admission helpers (topics.go:580-624) ------------------------------ */
int mqm_is_valid_filter(const char *filter, size_t len, int for_publish); /* IsValidFilter  */
int mqm_is_shared_filter(const char *filter, size_t len);                  /* IsSharedFilter */

/* ---- stats for the roofline (per committed snapshot) -------------------- */
typedef struct {
  uint64_t nodes, edges, edge_buckets, subs, shared, height;
  uint64_t device_bytes; /* HBM bytes held by the current snapshot */
  uint64_t solo_subs;    /* subscriptions that skip the per-topic merge (snapshot.h kMetaMulti) */
} mqm_snapshot_stats;
int mqm_snapshot_stats_get(mqm_index *h, mqm_snapshot_stats *out);

/* ---- kernel timing (HIP events on the launch stream) --------------------- */
typedef struct {
  uint64_t calls;           /* match calls while enabled                        */
  uint64_t fallback_topics; /* topics that took the unbounded path              */
  double walk_ms;           /* k_walk: tokenize + walk + hit records              */
  double dedupe_ms;         /* k_small + k_big + DFS phases 1-2                   */
  double total_ms;          /* first to last kernel of each call (incl. scans and
                               the one host sync that sizes the outputs), summed  */
} mqm_profile;
int mqm_profile_enable(mqm_index *h, int on); /* resets the accumulators */
int mqm_profile_read(mqm_index *h, mqm_profile *out);

const char *mqm_version(void);

#ifdef __cplusplus
}
#endif
#endif /* MQMATCH_H */
