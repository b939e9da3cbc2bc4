// maxmq_amd/csrc/match.h — batch match pipeline over a DeviceSnapshot.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <unordered_map>

#include "snapshot.h"

namespace mqm {

// ---- small-batch path (fast.hip) --------------------------------------------
// device counters of one k_fast launch; the last workgroup resets them
struct FastCtl {
  unsigned long long dcur, hcur, icur;  // delivery / shared-candidate / identifier slots reserved
  unsigned int flags, done;
};
enum : uint32_t { kFastFallback = 1u, kFastOverflow = 2u };
// topic t's result: deliveries dout[dbase .. + dcount), shared hout[hbase ..
// + hcount), Identifiers support iout[ibase .. + icount) (the sids of its
// gathered non-shared subscriptions with Identifier > 0, kWordIdent)
struct FastRec {
  uint32_t dbase, dcount, hbase, hcount, ibase, icount;
};
struct FastStatus {  // written by the last workgroup (pinned)
  unsigned long long d_total, h_total, i_total;
  unsigned int flags, done;
};
// pinned, device-mapped host blocks of one context (grown, never shrunk)
struct FastArena {
  char *in_bytes = nullptr;
  uint64_t *in_offs = nullptr;
  FastRec *recs = nullptr;
  uint64_t *dout = nullptr;  // {client, packed} deliveries (mqm_delivery)
  uint32_t *hout = nullptr;  // shared-subscription ids
  uint32_t *iout = nullptr;  // identifier sids (MQM_CFG_IDENTIFIERS)
  FastStatus *status = nullptr;
  size_t in_cap = 0, offs_cap = 0, rec_cap = 0, dout_cap = 0, hout_cap = 0, iout_cap = 0, status_cap = 0;
  FastCtl *ctl = nullptr;  // device
  uint32_t grid = 0;       // resident k_fast workgroups
  // the call's completion: a blocking-sync event (the waiting caller sleeps in
  // the driver instead of spinning: 64 direct callers spinning in
  // hipStreamSynchronize on a 16-CPU quota starve the ones whose results are
  // ready — MQM_SPIN_SYNC=1 keeps the stream synchronisation, for A/B)
  hipEvent_t done_ev = nullptr;
  ~FastArena();
};
struct FastOutput {
  uint32_t n_topics = 0;
  uint64_t n_slots = 0, n_shared_slots = 0;  // reserved (raw-entry upper bounds)
  const FastRec *recs = nullptr;             // pinned host, n_topics
  const uint64_t *dout = nullptr;            // pinned host
  const uint32_t *hout = nullptr;            // pinned host
  const uint32_t *iout = nullptr;            // pinned host (want_ids)
};

// Grow-only device buffers reused across batches (no allocation in steady state).
struct Workspace {
  enum Slot {
    kSCount, kHCount, kDCount, kDStart, kHStart, kCls, kDfsList, kRecs, kCounters, kDOut, kHOut,
    kDense, kDenseShared, kDenseOffs, kDenseHOffs, kScanTmp, kRawCnt, kTabOff, kTabSize, kTable,
    kInBytes, kInOffs, kListS, kICount, kIStart, kIOut, kNSolo, kDescStart, kDesc, kWin, kMCount, kRunCount, kRunOffs, kRuns, kListW, kListT1, kListT2, kListT3, kListP, kListH, kListRS, kListR,
    kIMStart, kIScratch, kScanTmp2,
    // reverse match (retained.hip)
    kROffs, kRNLev, kRWild, kRLOff, kRFCount, kRFCur, kRLevels, kRNCount, kRNOff, kRItemF0, kRItemN0, kRItemF1,
    kRItemN1, kRChild, kRECount, kREOff, kREmit, kRPos, kRChunks, kRCOff, kROut, kRInBytes, kRInOffs, kNumSlots
  };
  struct Buf {
    void *p = nullptr;
    size_t cap = 0;
  };
  Buf bufs[kNumSlots];
  void *host_pinned = nullptr;
  uint32_t max_blocks = 2048;  // walk-kernel grid cap (grid-stride beyond)
  // reverse match (retained.hip): list capacities carried from call to call
  // (grown when a call's device counters report an overflow)
  uint64_t rev_item_cap = 0, rev_emit_cap = 0, rev_task_cap = 0, rev_out_cap = 0, rev_ltask_cap = 0;
  std::unordered_map<const void *, uint32_t> resident;  // kernel -> resident blocks on the device
  // why the last batch's DFS topics left the bounded path:
  // frontier, hits, cached levels, shared hits, raw entries
  uint32_t why[5] = {0, 0, 0, 0, 0};
  // the batch pipeline's queued calls (match_enqueue / match_collect): every
  // output buffer sized by an earlier call (caps_known), the DFS list capacity
  // a queued call assumes, the call in flight, and how many queued calls had
  // to be run again exact
  bool caps_known = false, pending = false, pend_exact = false;
  uint32_t dfs_cap = 0;
  // merge / shared lists (bit per list, match.hip kList*) that had topics in the
  // last collected call: a queued call launches only their kernels (an empty
  // list's persistent grid still queues behind the solo copy), and a call
  // whose topics land in a list it did not launch is run again, exact
  uint32_t lists_seen = ~0u, pend_launched = ~0u;
  uint64_t requeued = 0;
  // the last match_device call (identifiers_device works on its records)
  bool last_valid = false;
  uint32_t last_n = 0, last_n_dfs = 0;
  // the runs form (mqm_match_batch_runs): solo parts stay runs of `words`
  // (runs_device lists them), dout holds the merged winners only
  bool runs = false, last_runs = false;
  const uint8_t *last_bytes = nullptr;
  const uint64_t *last_offs = nullptr;
  // Identifiers computed beside the match (mqm_identifiers_early, and every
  // host-path call of an MQM_CFG_IDENTIFIERS index): after the walk, k_ident
  // and its scans run on `side` while the merges and the solo copy run on the
  // call's stream, joined before the call's read-back; identifiers_device then
  // only collects.  ident_cap: the scratch / iout capacity (grown from the
  // multi entries a call reported)
  bool ident_early = false, ident_ready = false;
  // ident_fused: the last enqueued call listed Identifiers in its merges
  // (match.hip ident_base; the default form of ident_early, MQM_IDENT_FUSED=0
  // for the side-stream pass); its totals come back with the call's counters
  bool ident_fused = false;
  uint64_t ident_cap = 0;
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;

  // the small-batch path's pinned blocks (fast.hip)
  FastArena fast;

  // optional kernel timing (mqm_profile_*): events on the launch stream
  bool profile = false;
  hipEvent_t ev[4] = {};  // 0 start, 1 walk done, 2 dedupe start, 3 end
  uint64_t prof_calls = 0, prof_fallback_topics = 0;
  double prof_walk_ms = 0, prof_dedupe_ms = 0, prof_total_ms = 0;
  void reset_profile() {
    prof_calls = prof_fallback_topics = 0;
    prof_walk_ms = prof_dedupe_ms = prof_total_ms = 0;
  }

  // Buffers are hipMalloc'd and grown by replacement: the old one is retired
  // through the reaper (retire_device_buffers) after this workspace's own
  // queued work (`cur`) and its previous calls (`last_use`) — never freed
  // under a running kernel, and no stream-ordered pool memory (its reuse
  // served stale data: DESIGN §9, round 6).
  hipStream_t cur = nullptr;     // stream of the call in progress (begin())
  hipEvent_t last_use = nullptr; // recorded by end() after every call's work
  bool used = false;
  void begin(hipStream_t st) { cur = st; }
  int end(hipStream_t st);       // record last_use on st
  int drain();                   // wait for every queued use of the buffers
  int reserve(void **p, size_t *cap, size_t need);
  int get(Slot s, size_t need) { return reserve(&bufs[s].p, &bufs[s].cap, need); }
  // like get(), but a reallocation keeps the first `used` bytes (copied on `st`)
  int grow_keep(Slot s, size_t used, size_t need, hipStream_t st);
  // 256 B of pinned host memory for small read-backs (nullptr on failure)
  uint64_t *pinned_u64();
  void *ptr(Slot s) const { return bufs[s].p; }
  ~Workspace();
};

// Per-topic segments (starts/counts; see mqm_device_result).
struct MatchOutput {
  uint32_t n_topics = 0;
  uint64_t n_deliveries = 0, n_shared = 0;
  const uint64_t *starts = nullptr;      // device, n
  const uint32_t *counts = nullptr;      // device, n
  const uint32_t *deliveries = nullptr;  // device, packed (snapshot.h: sid | qos << 28 | no_local << 30)
  const uint64_t *shared_starts = nullptr;
  const uint32_t *shared_counts = nullptr;
  const uint32_t *shared = nullptr;
  uint32_t n_fallback = 0;  // topics on the unbounded DFS path
  uint32_t n_big = 0;       // topics whose multi entries the workgroup tier merged
  uint32_t n_tier2 = 0, n_tier3 = 0;  // ... of those, passed on to its second / third tier
  uint32_t n_merge_small = 0, n_merge_wave = 0;  // topics merged by k_merge_small / k_merge
  uint64_t n_solo_ranges = 0;                     // solo parts (copy descriptors / runs: hits with solo entries)
  uint64_t multi_entries[3] = {0, 0, 0};  // multi entries merged by the three workgroup tiers
  uint32_t n_part = 0;                    // ... of the third tier's topics, merged in client-hash partitions
  uint32_t n_resolve = 0;                 // topics merged by resolution (k_resolve: no table)
  uint64_t n_solo = 0;                    // solo entries: deliveries copied as they stand
  bool exact = false;                     // sized by its own read-back (the first call of a workspace, or a re-run)
};

// MQM_SLOTS=1: the snapshot carries DeviceSnapshot::slots and the batch walk
// uses them (off by default: measured slower)
bool slots_enabled();
// slots[2i] = nodes[i], slots[2i + 1] = nodes[nodes[i].plus] or zeros (snapshot upload, on `st`)
int derive_slots(const NodeDesc *nodes, NodeDesc *slots, uint64_t n, hipStream_t st);
// bits[i / 32] bit i % 32 = subs[i].word & kWordIdent (snapshot upload, on `st`)
int derive_ident_bits(const SubEnt *subs, uint32_t *bits, uint64_t n, hipStream_t st);
// words[i] = subs[i].word & kPackedMask for i < n (snapshot upload, on `st`)
int derive_words(const SubEnt *subs, uint32_t *words, uint64_t n, hipStream_t st);
// nflags[i] = nodes[i].sh_cnt_flags >> 24 for i < n (snapshot upload, on `st`)
int derive_node_flags(const NodeDesc *nodes, uint8_t *nflags, uint64_t n, hipStream_t st);

// Runs walk -> scan -> dedupe (small / big / DFS) on `st` and waits for it;
// returns 0 or a negative MQM_E* code.
int match_device(const DeviceSnapshot &s, Workspace &ws, const uint8_t *d_bytes, const uint64_t *d_offs,
                 uint32_t n, hipStream_t st, MatchOutput *out);
// The same in two halves: queue the whole pipeline on `st` (exact: size the
// outputs by a read-back after the walk; otherwise from earlier calls, no
// host sync), then wait and read its counters.  match_collect returns 1 when
// the queued call outgrew the buffers earlier calls sized (run it again with
// exact = true; the inputs must still hold the batch).
int match_enqueue(const DeviceSnapshot &s, Workspace &ws, const uint8_t *d_bytes, const uint64_t *d_offs, uint32_t n,
                  hipStream_t st, bool exact);
int match_collect(Workspace &ws, hipStream_t st, MatchOutput *out);

// Small batches (the per-publish call shape): one kernel over host topics
// (bytes[offs[0] .. offs[n])), results in the workspace's pinned blocks, valid
// until the next call on `ws`.  Synchronises `st`.  Returns 0, 1 when a topic
// is past a capacity of this path (the caller runs the batch pipeline), or a
// negative MQM_E* code.
constexpr uint32_t kFastMaxTopics = 4096;
int match_small(const DeviceSnapshot &s, Workspace &ws, const char *bytes, const uint64_t *offs, uint32_t n,
                hipStream_t st, FastOutput *out, bool want_ids = false);

// ---- the per-publish server (fast.hip k_serve) -------------------------------
// A persistent kernel of `grid` workgroups serves single-topic Subscribers
// calls posted to a ring of slots in pinned, coherent host memory: the caller
// writes the topic into slot k % kServeSlots and then seq = k + 1 (with the
// length); an idle workgroup takes the next request number k from a device
// counter, waits for that slot's seq, runs the small-batch path's per-topic
// body (fast_topic) straight into the slot and publishes done = k + 1.  No
// launch and no stream synchronisation per call.  Every workgroup exits on
// `stop`, or after idle_us without a request, returning its number (the host
// relaunches on the next call; unserved requests wait in the ring).
constexpr uint32_t kServeSlots = 256;
constexpr uint32_t kServeTopic = 1024;  // topic bytes a slot holds (the small-batch path's kFStage)
constexpr uint32_t kServeD = 4096, kServeH = 512, kServeI = 4096;  // result capacities per slot
enum : uint32_t { kServeOk = 0, kServeFallback = 1 };
constexpr int kServeSeqBits = 48;  // ServeSlot::seq: request number + 1 below, the topic length above
constexpr unsigned long long kServeSeqMask = (1ull << kServeSeqBits) - 1;
constexpr uint32_t kServeHead = 48;  // topic bytes in the slot's first 64-B line, with seq and chk
struct alignas(64) ServeSlot {
  // line 0, read by the polling workgroup in one 64-B load: the request word,
  // a check word and the topic's first kServeHead bytes
  unsigned long long seq;   // host: (k + 1) | len << kServeSeqBits once request k's topic is in place
  uint32_t chk, pad0;       // host: serve_check(seq, the head bytes): a read of line 0 that tore fails it
  char topic[kServeTopic];  // topic bytes (0 .. kServeHead - 1 in line 0)
  uint32_t len, status;     // topic length; kServe* (fallback: the caller runs the batch pipeline)
  uint32_t dcount, hcount, icount, pad;
  unsigned long long ver;              // the snapshot version the result was matched on (HostSnapshot::version)
  unsigned long long t_claim, t_done;  // device clock (s_memrealtime, 100 MHz): claimed, published
  unsigned long long t_phase[2];       // ... topic staged and keys built, trie walked
  uint64_t dout[kServeD];   // {client, packed} deliveries
  uint32_t hout[kServeH];   // shared-subscription ids
  uint32_t iout[kServeI];   // identifier sids (want_ids)
};
static_assert(offsetof(ServeSlot, topic) + kServeHead == 64, "ServeSlot line 0");
// the check word of line 0 (host and device): a mix of the request word and
// the kServeHead topic bytes as 6 little-endian words
MQM_HD uint32_t serve_check(unsigned long long seq, const unsigned long long *head) {
  unsigned long long x = seq * 0x9E3779B97F4A7C15ull;
  for (int i = 0; i < (int)(kServeHead / 8); i++) {
    x = (x ^ head[i]) * 0xD6E8FEB86659FD93ull;
    x ^= x >> 32;
  }
  return (uint32_t)(x >> 29);
}
struct ServeQueue {
  unsigned long long stop;    // host: 1 = every workgroup exits
  unsigned long long exited;  // device: the launch generation whose last workgroup has exited
  unsigned long long pad[6];
  // device: done[i] = k + 1 once request k's result (slot i = k % kServeSlots)
  // is complete — one contiguous 2-KB array, so the host's completion poller
  // scans 32 cache lines rather than a line (and a page) per slot
  unsigned long long done[kServeSlots];
  ServeSlot slot[kServeSlots];
};
// launch the server on `st` (q: host-mapped; ctr: two device counters, set by
// the host before every launch: ctr[0] the oldest request not yet served, ctr[1]
// = 0 the workgroups that have exited).  `ver` is written into every slot the
// launch serves (the snapshot's version), `gen` into q->exited by the launch's
// last workgroup to exit; request numbers below `seen` (the highest number an
// earlier launch handed out) are skipped when their slot's done word shows
// them served.
// MQM_SNAP_STAMP=1 diagnostics of the per-publish kernels: checks made,
// stamps found stale through the caches, stale in memory (out[3])
int stamp_counts(uint64_t *out);
int serve_launch(const DeviceSnapshot &s, ServeQueue *q, unsigned long long *ctr, uint32_t grid, uint32_t idle_us,
                 bool want_ids, uint64_t ver, uint64_t gen, uint64_t seen, hipStream_t st);

// Identifiers support for the last match_device call on `ws` (its topic
// buffers must still hold the batch): per topic, the sids of the gathered
// non-shared subscriptions with Identifier > 0 (mqm_device_identifiers).
struct IdentOutput {
  uint32_t n_topics = 0;
  uint64_t n_idents = 0;
  const uint64_t *offsets = nullptr;  // device, n + 1
  const uint32_t *sids = nullptr;     // device
};
int identifiers_device(const DeviceSnapshot &s, Workspace &ws, hipStream_t st, IdentOutput *out);

// The runs form of the last match_device call on `ws` (made with ws.runs):
// topic t's solo deliveries are words[run.x .. run.x + run.y) for its runs
// runs[offsets[t] .. offsets[t+1]); its merged winners are the MatchOutput's
// segments (dcount = winners only).  Device pointers, valid until the next call.
struct RunsOutput {
  uint32_t n_topics = 0;
  uint64_t n_runs = 0;
  const uint64_t *offsets = nullptr;   // n + 1
  const uint2 *runs = nullptr;         // (words offset, count)
  const uint32_t *solo_counts = nullptr;  // per topic: its runs' total
};
int runs_device(Workspace &ws, hipStream_t st, const MatchOutput &m, RunsOutput *out);

// Dense CSR of a MatchOutput (offsets n+1, entries back to back) on `st`.
struct DenseOutput {
  const uint64_t *offsets = nullptr, *deliveries = nullptr, *shared_offsets = nullptr;
  const uint32_t *shared = nullptr;
};
// (clients resolved through the snapshot the match read; packed: the 4-B
// packed words only, `deliveries` then points at uint32_t)
int densify(const DeviceSnapshot &s, Workspace &ws, const MatchOutput &m, hipStream_t st, DenseOutput *out,
            bool packed = false);

// A host-path call's result parts from device buffers into its pinned host
// block (device views), by one kernel on `st` instead of a DMA copy per part
// (MQM_D2H_KERNEL, capi.cpp).  Parts: 4-B multiples, 16-B aligned ends.
struct CopyOut {
  static constexpr int kMax = 8;
  const void *src[kMax];
  void *dst[kMax];
  uint64_t bytes[kMax];
  int n = 0;
};
int copy_out_device(const CopyOut &c, hipStream_t st);

}  // namespace mqm
