// maxmq_amd/csrc/fast.hip — the per-publish path: TopicsIndex.Subscribers
// (vendor/github.com/mochi-co/mqtt/v2/topics.go:484-555) for small batches in
// ONE kernel launch, reading the topics from and writing the results to pinned
// host memory.
//
// The reference calls Subscribers(topic) once per PUBLISH, from one goroutine
// per connection (server.go:776, listeners/tcp.go:83).  The batch pipeline
// (match.hip) is built for 10M-topic batches: ~25 launches and host read-backs
// that cost ~150 us whatever the batch size.  Here a workgroup per topic does
// the whole Subscribers call:
//   1. stage the topic's bytes (read straight from pinned host memory) in LDS,
//      find the '/' separators (isolateParticle, topics.go:558-577) and build
//      the 128-bit level keys (keys.h);
//   2. walk the trie level-synchronously — every frontier node's literal edge
//      probe and '+' / '#' child loads in flight together (device.h
//      walk_step), with exactly the batch walk's rules: gather at every
//      visited node, the parent-'#' probe after a literal level only
//      (topics.go:503-513), the `$` rule as the per-node kFlagDollarWild flag
//      (topics.go:527); hit ranges and shared ranges collected in LDS;
//   3. emit: solo entries (kMetaMulti clear: a client's only entry) copied as
//      is; multi entries merged per client in an LDS hash table — QoS max,
//      NoLocal OR, the first-merged subscription = the lowest hit rank
//      (Subscription.Merge, packets.go:250-270) — in client-hash partitions
//      of at most kFPartCap entries, so any number of them fits; shared
//      candidates (gatherSharedSubscriptions, topics.go:541-555) listed;
//      results written as dense {client, packed} deliveries into a pinned
//      block at a range reserved with one atomic per topic.
// The last workgroup to finish publishes the totals and flags to the host and
// resets the device counters for the next call, so a call is: copy the topics
// into a pinned block, one launch, one stream synchronisation.
// A topic past a capacity (topic > kFStage bytes, > kFLevels levels, a level
// with > kFItems load items, > kFHits hits, > kFSh shared hits, a saturated
// multi count) flags the batch; the caller then runs the batch pipeline,
// which has no limits.  Nothing runs on the CPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "device.h"
#include "match.h"

namespace mqm {

namespace {

constexpr int kFT = 256;             // threads per topic (one workgroup)
constexpr int kFWaves = kFT / 64;
constexpr uint32_t kFStage = 1024;   // topic bytes staged in LDS
constexpr uint32_t kFLevels = 32;
constexpr uint32_t kFItems = 768;    // load items per level (<= 3 per frontier node)
constexpr uint32_t kFHits = 384;     // non-shared hit ranges per topic
constexpr uint32_t kFSh = 128;       // shared hit ranges per topic
constexpr uint32_t kFSlots = 2048;   // merge table slots
constexpr uint32_t kFPartCap = 1536; // multi entries per merge pass (load <= 0.75 on average)
constexpr uint32_t kFFill = kFSlots * 7 / 8;
constexpr uint32_t kFRangeMax = 1u << 24;

enum : uint32_t { kFItemLit = 0, kFItemPlus = 1, kFItemHash = 2 };

struct alignas(16) FastLds {
  unsigned long long tkb[kFSlots], tfirst[kFSlots];
  uint32_t hoff[kFHits], hcnt[kFHits], hmu[kFHits], hrank[kFHits];
  uint32_t spre[kFHits + 1], mpre[kFHits + 1];
  uint32_t shoff[kFSh], shcnt[kFSh], shpre[kFSh + 1];
  uint32_t item[2][kFItems];
  uint64_t key0[kFLevels], key1[kFLevels];
  uint16_t sep[kFLevels];
  alignas(8) uint8_t stage[kFStage];
  uint32_t nitems[3], nh, nsh, fail, nsep, fill, nid, wsum[kFWaves];  // item counts of levels d mod 3
  unsigned long long dbase, hbase, ibase;
};

__device__ __forceinline__ uint64_t f_lanemask_lt(int lane) { return (1ull << lane) - 1ull; }

__device__ __forceinline__ void f_wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint32_t f_qos_bits(uint32_t word) {
  return (1u << ((word >> 28) & 3)) | (((word >> 30) & 1) << 3);
}

// per-topic merge table (as match.hip's MergeTable): kb = (client + 1) << 32 |
// QoS one-hot | NoLocal, first = min(rank << 32 | sid)
__device__ __forceinline__ void f_insert(FastLds &L, uint32_t mask, uint32_t lg, uint32_t client, uint32_t word,
                                         uint32_t rank) {
  uint32_t sl = (uint32_t)(((uint64_t)(client * 2654435769u) << lg) >> 32);
  const unsigned long long key = (unsigned long long)(client + 1u) << 32, kb = key | f_qos_bits(word);
  for (;;) {
    const unsigned long long prev = atomicCAS(&L.tkb[sl], 0ull, kb);
    if (prev == 0) break;
    if ((prev >> 32) == (key >> 32)) {
      if ((prev | kb) != prev) atomicOr(&L.tkb[sl], kb);
      break;
    }
    sl = (sl + 1) & mask;
  }
  atomicMin(&L.tfirst[sl], ((unsigned long long)rank << 32) | (word & kWordSidMask));
}

// a client -> partition hash independent of the table slot's
__device__ __forceinline__ uint32_t f_partition(uint32_t client, uint32_t P) {
  uint32_t h = client * 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return (uint32_t)(((uint64_t)h * P) >> 32);
}

// largest h < nh with pre[h] <= x (pre[0] = 0, nondecreasing)
__device__ __forceinline__ uint32_t f_search(const uint32_t *pre, uint32_t nh, uint32_t x) {
  uint32_t lo = 0, hi = nh;  // invariant: pre[lo] <= x, answer in [lo, hi)
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (pre[mid] <= x)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

// exclusive prefix of v[0 .. n) into pre[0 .. n] by one wave (64 per step;
// pre may be v: a step reads its 64 values before writing them)
__device__ __forceinline__ void f_prefix(const uint32_t *v, uint32_t *pre, uint32_t n, int lane) {
  uint32_t run = 0;
  for (uint32_t b = 0; b < n; b += 64) {
    const uint32_t i = b + lane;
    const uint32_t x = i < n ? v[i] : 0;
    uint32_t inc = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t u = __shfl_up(inc, d, 64);
      if (lane >= d) inc += u;
    }
    if (i < n) pre[i] = run + inc - x;
    run += __shfl(inc, 63, 64);
  }
  if (lane == 0) pre[n] = run;
}

// ---------------------------------------------------------------------------
// One topic's Subscribers by one workgroup: topic bytes (host-mapped) ->
// the sink's result blocks.  Sink: reserve(L, raw entries, shared) -> false
// when its blocks cannot take them (it records why; L.dbase / hbase / ibase
// otherwise), fallback() (a capacity of this path: the batch pipeline has
// none), done(L, deliveries, shared); dout / hout / iout its blocks (iout
// nullptr: no Identifiers support).  Called by every thread of the block.
// ---------------------------------------------------------------------------
template <class Sink>
__device__ __forceinline__ void fast_topic(const DeviceSnapshot &s, FastLds &L, const uint8_t *__restrict__ topic,
                                           uint32_t len, Sink &sink, uint32_t pre = 0) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // the root's descriptor: its load is in flight with the topic's (a PCIe
  // read when the topic is in host memory)
  NodeDesc root{};
  if (tid == 0) root = load_desc(s.nodes);
  if (tid == 0) {
    L.fail = len > kFStage ? 1u : 0u;
    L.nh = L.nsh = 0;
    L.nitems[0] = L.nitems[1] = L.nitems[2] = 0;
  }
  __syncthreads();
  const bool staged = len <= kFStage;
  if (staged)  // (the first `pre` bytes: in LDS already, from the request's line)
    for (uint32_t i = pre + tid; i < len; i += kFT) L.stage[i] = topic[i];
  __syncthreads();
  // ---- 1. separators and level keys ---------------------------------------
  if (wid == 0 && staged) {
    uint32_t nsep = 0;
    for (uint32_t base = 0; base < len; base += 64) {
      const uint32_t p = base + lane;
      const bool sep = p < len && L.stage[p] == '/';
      const uint64_t m = __ballot(sep);
      if (sep) {
        const uint32_t idx = nsep + __popcll(m & f_lanemask_lt(lane));
        if (idx < kFLevels) L.sep[idx] = (uint16_t)p;
      }
      nsep += __popcll(m);
    }
    if (lane == 0) {
      L.nsep = nsep;
      if (nsep >= kFLevels) L.fail = 1;
    }
  }
  __syncthreads();
  const uint32_t nsep = staged ? L.nsep : 0;
  const uint32_t nlev = (len == 0 || L.fail) ? 0 : nsep + 1;
  const bool dollar = len > 0 && staged && L.stage[0] == '$';
  if ((uint32_t)tid < nlev) {
    const uint32_t st = tid == 0 ? 0 : L.sep[tid - 1] + 1u;
    const uint32_t en = (uint32_t)tid < nsep ? L.sep[tid] : len;
    const Key k = make_key([&](uint32_t i) { return L.stage[st + i]; }, en - st);
    L.key0[tid] = k.k0;
    L.key1[tid] = k.k1;
  }
  if (tid == 0 && nlev > 0) {  // level 0's items: the root's literal probe, '+' and '#' children
    uint32_t k = 0;
    if ((root.sh_cnt_flags >> 24) & kFlagHasLiteral) L.item[0][k++] = (0u << 2) | kFItemLit;
    if (root.plus != kNone) L.item[0][k++] = (root.plus << 2) | kFItemPlus;
    if (root.hash != kNone) L.item[0][k++] = (root.hash << 2) | kFItemHash;
    L.nitems[0] = k;
  }
  __syncthreads();
  if (tid == 0) sink.stamp(0);  // staged, keys built
  // ---- 2. level-synchronous walk -------------------------------------------
  int cur = 0;  // item lists alternate; their counts rotate over three words, so
                // the count two levels ahead is cleared during this level and one
                // barrier per level suffices
  for (uint32_t d = 0; d < nlev; d++) {
    const uint32_t ni = L.nitems[d % 3];
    if (tid == 0) L.nitems[(d + 2) % 3] = 0;  // (last read at level d - 1)
    if (ni == 0 || L.fail) break;  // block-uniform (read after a barrier)
    const uint64_t k0 = L.key0[d], k1 = L.key1[d];
    const bool has_next = d + 1 < nlev;
    // a topic level "+" / "#": its literal probe is the wildcard's (the
    // reference visits that child twice, with no parent probe)
    const bool lit_is_wild = (k1 == (1ull << 56)) && (k0 == '+' || k0 == '#');
    const uint32_t tst = d == 0 ? 0 : L.sep[d - 1] + 1u;
    const uint32_t tln = (d < nsep ? L.sep[d] : len) - tst;
    for (uint32_t base = 0; base < ni; base += kFT) {
      const uint32_t it = base + tid;
      const bool live = it < ni;
      const uint32_t iw = live ? L.item[cur][it] : 0;
      const uint32_t kind = iw & 3u, id = iw >> 2;
      const bool lit = kind == kFItemLit;
      NodeDesc dc;
      const uint32_t c = walk_step(s, live && lit && !lit_is_wild, live && !lit, id, id, k0, k1,
                                   L.stage + tst, tln, &dc);
      if (c == kNone) continue;
      const uint32_t fl = dc.sh_cnt_flags >> 24;
      const bool skip_dollar = dollar && (fl & kFlagDollarWild);      // topics.go:527
      // a '#' node after a literal parent: gathered by the parent probe (kFlagParentLit)
      const uint32_t c_own = skip_dollar || (fl & kFlagParentLit) ? 0 : dc.sub_cnt;
      const uint32_t c_par = lit && !skip_dollar ? dc.hsub_cnt : 0;  // topics.go:507-509
      const uint32_t c_sh = dc.sh_cnt_flags & kShCntMask;
      if (((c_own | c_par) && (fl & kFlagMultiSat)) || c_own > kFRangeMax || c_par > kFRangeMax)
        atomicOr(&L.fail, 1u);
      if (c_own) {
        const uint32_t h = atomicAdd(&L.nh, 1u);
        if (h < kFHits) {
          L.hoff[h] = dc.sub_off, L.hcnt[h] = c_own, L.hmu[h] = dc.multi & 0xFFFFu, L.hrank[h] = 2 * c;
        } else {
          atomicOr(&L.fail, 1u);
        }
      }
      if (c_par) {  // the '#' child's range follows this node's (snapshot.h)
        const uint32_t h = atomicAdd(&L.nh, 1u);
        if (h < kFHits) {
          L.hoff[h] = dc.sub_off + dc.sub_cnt, L.hcnt[h] = c_par, L.hmu[h] = dc.multi >> 16, L.hrank[h] = 2 * c + 1;
        } else {
          atomicOr(&L.fail, 1u);
        }
      }
      if (c_sh) {
        const uint32_t h = atomicAdd(&L.nsh, 1u);
        if (h < kFSh) {
          L.shoff[h] = dc.sh_off, L.shcnt[h] = c_sh;
        } else {
          atomicOr(&L.fail, 1u);
        }
      }
      if (has_next && (fl & kFlagHasChildren)) {
        const bool has_lit = fl & kFlagHasLiteral;
        const uint32_t k = (has_lit ? 1u : 0u) + (dc.plus != kNone ? 1u : 0u) + (dc.hash != kNone ? 1u : 0u);
        const uint32_t at = k ? atomicAdd(&L.nitems[(d + 1) % 3], k) : 0;
        if (at + k > kFItems) {
          atomicOr(&L.fail, 1u);
        } else {
          uint32_t j = at;
          if (has_lit) L.item[cur ^ 1][j++] = (c << 2) | kFItemLit;
          if (dc.plus != kNone) L.item[cur ^ 1][j++] = (dc.plus << 2) | kFItemPlus;
          if (dc.hash != kNone) L.item[cur ^ 1][j++] = (dc.hash << 2) | kFItemHash;
        }
      }
    }
    __syncthreads();
    cur ^= 1;
  }
  if (L.fail) {  // block-uniform: the batch takes the pipeline without limits
    if (tid == 0) sink.fallback();
    __syncthreads();
    return;
  }
  if (tid == 0) sink.stamp(1);  // walked
  // ---- 3. emission -----------------------------------------------------------
  // prefixes of the hits' solo counts, multi counts and the shared counts
  // (one wave each, in place)
  const uint32_t nh = L.nh, nsh = L.nsh;
  if (wid == 0) {
    for (uint32_t i = lane; i < nh; i += 64) L.spre[i] = L.hcnt[i] - L.hmu[i];
    f_wave_lds_sync();
    f_prefix(L.spre, L.spre, nh, lane);
  } else if (wid == 1) {
    for (uint32_t i = lane; i < nh; i += 64) L.mpre[i] = L.hmu[i];
    f_wave_lds_sync();
    f_prefix(L.mpre, L.mpre, nh, lane);
  } else if (wid == 2) {
    f_prefix(L.shcnt, L.shpre, nsh, lane);
  }
  __syncthreads();
  const uint32_t Ss = L.spre[nh], Ms = L.mpre[nh], H = L.shpre[nsh];
  if (tid == 0) {
    L.nid = 0;
    L.fail = sink.reserve(L, (unsigned long long)Ss + Ms, H) ? 0u : 1u;  // sets L.dbase / hbase / ibase
  }
  __syncthreads();
  if (L.fail) {  // (the sink has recorded why: grow and run again, or the pipeline)
    __syncthreads();
    return;
  }
  uint64_t *const dout = sink.dout;
  uint32_t *const hout = sink.hout;
  uint32_t *const iout = sink.iout;
  const uint64_t db = L.dbase, hb = L.hbase, ib = L.ibase;
  // solo entries: each its client's merged delivery as is
  for (uint32_t q = tid; q < Ss; q += kFT) {
    const uint32_t h = f_search(L.spre, nh, q);
    const uint32_t sid = L.hoff[h] + (q - L.spre[h]);
    const uint2 e = *reinterpret_cast<const uint2 *>(s.subs + sid);
    dout[db + q] = (uint64_t)e.x | ((uint64_t)(e.y & kPackedMask) << 32);
    if (iout && (e.y & kWordIdent)) iout[ib + atomicAdd(&L.nid, 1u)] = sid;  // packets.go:257-259
  }
  // shared candidates
  for (uint32_t j = tid; j < H; j += kFT) {
    const uint32_t h = f_search(L.shpre, nsh, j);
    hout[hb + j] = L.shoff[h] + (j - L.shpre[h]);
  }
  // multi entries: the per-client merge, in client-hash partitions
  uint32_t W = 0;
  const uint32_t P = Ms ? (Ms + kFPartCap - 1) / kFPartCap : 0;
  const uint32_t per = P ? (Ms + P - 1) / P : 0;
  uint32_t lg = 6;
  while ((1u << lg) < 2 * per && (1u << lg) < kFSlots) lg++;
  const uint32_t mask = (1u << lg) - 1;
  for (uint32_t p = 0; p < P; p++) {
    __syncthreads();  // the previous pass's winners are read
    for (uint32_t j = tid; j <= mask; j += kFT) {
      L.tkb[j] = 0;
      L.tfirst[j] = ~0ull;
    }
    if (tid == 0) L.fill = 0;
    __syncthreads();
    for (uint32_t q = tid; q < Ms; q += kFT) {
      const uint32_t h = f_search(L.mpre, nh, q);
      const uint32_t sid = L.hoff[h] + (L.hcnt[h] - L.hmu[h]) + (q - L.mpre[h]);
      const uint2 e = *reinterpret_cast<const uint2 *>(s.subs + sid);
      if (P > 1 && f_partition(e.x, P) != p) continue;
      if (iout && (e.y & kWordIdent)) iout[ib + atomicAdd(&L.nid, 1u)] = sid;
      if (atomicAdd(&L.fill, 1u) >= (P > 1 ? kFFill : mask)) {  // an unlucky partition: never spin
        atomicOr(&L.fail, 1u);
        continue;
      }
      f_insert(L, mask, lg, e.x, e.y, L.hrank[h]);
    }
    __syncthreads();
    // winners in slot order: wave w scans its quarter of the table twice
    const uint32_t slots = mask + 1, q4 = (slots + kFWaves - 1) / kFWaves;
    const uint32_t lo = wid * q4, hi = min(slots, lo + q4);
    uint32_t cnt = 0;
    for (uint32_t j0 = lo; j0 < hi; j0 += 64) {
      const uint32_t j = j0 + lane;
      cnt += __popcll(__ballot(j < hi && L.tkb[j] != 0));
    }
    if (lane == 0) L.wsum[wid] = cnt;
    __syncthreads();
    uint32_t w = W, tot = W;
    for (int k = 0; k < kFWaves; k++) {
      if (k < wid) w += L.wsum[k];
      tot += L.wsum[k];
    }
    for (uint32_t j0 = lo; j0 < hi; j0 += 64) {
      const uint32_t j = j0 + lane;
      const bool occ = j < hi && L.tkb[j] != 0;
      const uint64_t m = __ballot(occ);
      if (occ) {
        const unsigned long long kb = L.tkb[j];
        const uint32_t v = (uint32_t)kb;
        const uint32_t packed = ((uint32_t)L.tfirst[j] & kWordSidMask) | ((31u - __builtin_clz(v & 7u)) << 28) |
                                (((v >> 3) & 1u) << 30);
        dout[db + Ss + w + __popcll(m & f_lanemask_lt(lane))] = (uint64_t)((kb >> 32) - 1) | ((uint64_t)packed << 32);
      }
      w += __popcll(m);
    }
    W = tot;
  }
  __syncthreads();
  if (tid == 0) {
    if (L.fail)
      sink.fallback();
    else
      sink.done(L, Ss + W, H);
  }
  __syncthreads();
}

// the batch form's sink: ranges of the pinned result blocks reserved with one
// atomic per topic, a FastRec per topic, flags for the host
struct BatchSink {
  FastCtl *ctl;
  FastRec *recs;
  uint32_t t;
  uint64_t *dout;
  uint64_t dcap;
  uint32_t *hout;
  uint64_t hcap;
  uint32_t *iout;
  uint64_t icap;
  __device__ bool reserve(FastLds &L, unsigned long long need, uint32_t H) {
    const unsigned long long db = need ? atomicAdd(&ctl->dcur, need) : 0ull;
    const unsigned long long hb = H ? atomicAdd(&ctl->hcur, (unsigned long long)H) : 0ull;
    // identifiers: at most one per gathered entry
    const unsigned long long ib = (iout && need) ? atomicAdd(&ctl->icur, need) : 0ull;
    const bool ovf = db + need > dcap || hb + H > hcap || (iout && ib + need > icap);
    // FastRec keeps 32-bit offsets: a batch whose results pass 2^32 entries
    // takes the batch pipeline (64-bit segments) instead of growing the blocks
    const bool wide = db + need > 0xFFFFFFFFull || hb + H > 0xFFFFFFFFull || ib + need > 0xFFFFFFFFull;
    if (wide)
      atomicOr(&ctl->flags, kFastFallback);
    else if (ovf)
      atomicOr(&ctl->flags, kFastOverflow);  // the host grows the blocks to the reported totals, runs again
    L.dbase = db;
    L.hbase = hb;
    L.ibase = ib;
    if (ovf || wide) recs[t] = FastRec{0, 0, 0, 0, 0, 0};
    return !(ovf || wide);
  }
  __device__ void fallback() {
    atomicOr(&ctl->flags, kFastFallback);
    recs[t] = FastRec{0, 0, 0, 0, 0, 0};
  }
  __device__ void done(FastLds &L, uint32_t d, uint32_t h) {
    recs[t] = FastRec{(uint32_t)L.dbase, d, (uint32_t)L.hbase, h, (uint32_t)L.ibase, L.nid};
  }
  __device__ void stamp(int) {}
};

// MQM_SNAP_STAMP=1: [0] checks, [1] stale through the caches, [2] stale in
// memory (device.h stamp_mismatch), for mqm_debug_stamp_counts
__device__ unsigned long long g_stamp[3];

__device__ __noinline__ void check_stamps(const DeviceSnapshot &s, const char *where, unsigned long long job) {
  unsigned long long c = 0, m = 0;
  const uint32_t bad = stamp_mismatch(s, &c, &m);
  atomicAdd(&g_stamp[0], 1ull);
  if (!bad) return;
  unsigned long long n = 0;
  if (bad & 1) n = atomicAdd(&g_stamp[1], 1ull);
  if (bad & 2) n = atomicAdd(&g_stamp[2], 1ull);
  if (n < 8)
    printf("mqmatch stamp: %s job %llu: snapshot version %llu, cached stamp %llu, memory stamp %llu (bad %u)\n", where,
           job, (unsigned long long)s.version, c, m, bad);
}

__global__ __launch_bounds__(kFT) void k_fast(DeviceSnapshot s, const uint8_t *__restrict__ tb,
                                              const uint64_t *__restrict__ to, uint32_t n, FastCtl *ctl,
                                              FastRec *__restrict__ recs, uint64_t *__restrict__ dout, uint64_t dcap,
                                              uint32_t *__restrict__ hout, uint64_t hcap, uint32_t *__restrict__ iout,
                                              uint64_t icap, FastStatus *status) {
  __shared__ FastLds L;
  const int tid = threadIdx.x;
  for (uint32_t t = blockIdx.x; t < n; t += gridDim.x) {
    BatchSink sink{ctl, recs, t, dout, dcap, hout, hcap, iout, icap};
    if (s.stamp[0] && tid == 0) check_stamps(s, "k_fast", t);
    fast_topic(s, L, tb + to[t], (uint32_t)(to[t + 1] - to[t]), sink);
  }
  // the last workgroup to finish publishes the totals and resets the counters;
  // every workgroup's host writes are made visible (system scope) before its
  // ticket, so a host that sees `done` sees every result
  __syncthreads();
  if (tid == 0) {
    __threadfence_system();
    const unsigned int ticket = atomicAdd(&ctl->done, 1u);
    if (ticket == gridDim.x - 1) {
      __threadfence();
      const unsigned long long dt = atomicAdd(&ctl->dcur, 0ull), ht = atomicAdd(&ctl->hcur, 0ull),
                               it = atomicAdd(&ctl->icur, 0ull);
      const unsigned int fl = atomicOr(&ctl->flags, 0u);
      status->d_total = dt;
      status->h_total = ht;
      status->i_total = it;
      status->flags = fl;
      __threadfence_system();
      __hip_atomic_store(&status->done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      atomicExch(&ctl->dcur, 0ull);
      atomicExch(&ctl->hcur, 0ull);
      atomicExch(&ctl->icur, 0ull);
      atomicExch(&ctl->flags, 0u);
      atomicExch(&ctl->done, 0u);
      __threadfence_system();
    }
  }
}

// ---------------------------------------------------------------------------
// k_serve: the per-publish server (match.h ServeQueue).  Lane 0 of an idle
// workgroup takes the next request number from the device counter and polls
// that request's slot (system-scope loads of host memory, with a growing
// s_sleep between polls); the workgroup runs fast_topic into the slot and
// publishes done after a system fence.  Exit: the host's stop word, or
// idle_us without a request (s_memrealtime, 100 MHz).
// ---------------------------------------------------------------------------
struct ServeSink {
  ServeSlot *slot;
  unsigned long long *done_word;  // the slot's word of ServeQueue::done
  uint64_t *dout;
  uint32_t *hout;
  uint32_t *iout;
  unsigned long long k;
  unsigned long long ver;  // the launch's snapshot version, reported with every result
  __device__ bool reserve(FastLds &L, unsigned long long need, uint32_t H) {
    L.dbase = L.hbase = L.ibase = 0;
    if (need > kServeD || H > kServeH || (iout && need > kServeI)) {  // too big for a slot: the pipeline
      fallback();
      return false;
    }
    return true;
  }
  __device__ void publish(uint32_t status, uint32_t d, uint32_t h, uint32_t i) {
    slot->status = status;
    slot->dcount = d;
    slot->hcount = h;
    slot->icount = i;
    slot->ver = ver;
    slot->t_done = __builtin_amdgcn_s_memrealtime();
    __threadfence_system();  // the result reaches host memory before done
    __hip_atomic_store(done_word, k + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __device__ void fallback() { publish(kServeFallback, 0, 0, 0); }
  __device__ void stamp(int i) { slot->t_phase[i] = __builtin_amdgcn_s_memrealtime(); }
  __device__ void done(FastLds &L, uint32_t d, uint32_t h) { publish(kServeOk, d, h, L.nid); }
};

__global__ __launch_bounds__(kFT) void k_serve(DeviceSnapshot s, ServeQueue *q, unsigned long long *ctr,
                                               uint64_t idle_ticks, int want_ids, unsigned long long ver,
                                               unsigned long long gen, unsigned long long seen) {
  unsigned long long *claimed = ctr;  // ctr[1]: workgroups of this launch that have exited
  __shared__ FastLds L;
  __shared__ unsigned long long job;
  __shared__ uint32_t job_len;
  __shared__ int quit;
  const int tid = threadIdx.x, lane = tid & 63;
  for (;;) {
    if (tid < 64) {  // wave 0
      // take the next request number first (a device atomic: workgroups wait
      // on distinct requests in parallel, instead of queueing behind one PCIe
      // poll per claim), then wait for its topic
      // (a number below `seen` was handed out by an earlier launch, which may
      // have served it: the counter restarts at the oldest unserved request,
      // and the requests after it that are done are skipped, not served twice
      // into a slot whose caller may be reading it)
      unsigned long long c;
      for (;;) {
        unsigned int clo = 0, chi = 0, served = 0;
        if (lane == 0) {
          const unsigned long long c0 = atomicAdd(claimed, 1ull);
          clo = (unsigned int)c0, chi = (unsigned int)(c0 >> 32);
          if (c0 < seen)
            served = __hip_atomic_load(&q->done[c0 % kServeSlots], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= c0 + 1;
        }
        c = ((unsigned long long)__shfl(chi, 0, 64) << 32) | __shfl(clo, 0, 64);
        if (!__shfl(served, 0, 64)) break;
      }
      const unsigned long long *line = reinterpret_cast<const unsigned long long *>(&q->slot[c % kServeSlots]);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      uint32_t nap = 1;
      bool got = false;
      for (;;) {
        // line 0 in one instruction: the request word, the check word and
        // the topic's first kServeHead bytes (lanes 2 .. 7)
        unsigned long long w = 0;
        if (lane < 8) w = __hip_atomic_load(line + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const unsigned long long seq =
            ((unsigned long long)__shfl((unsigned int)(w >> 32), 0, 64) << 32) | __shfl((unsigned int)w, 0, 64);
        if ((seq & kServeSeqMask) == c + 1) {  // request c is posted
          unsigned long long head[kServeHead / 8];
#pragma unroll
          for (int i = 0; i < (int)(kServeHead / 8); i++)
            head[i] = ((unsigned long long)__shfl((unsigned int)(w >> 32), 2 + i, 64) << 32) |
                      __shfl((unsigned int)w, 2 + i, 64);
          const uint32_t chk = __shfl((unsigned int)w, 1, 64);
          if (chk == serve_check(seq, head)) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the topic's later bytes: written before seq
            if (lane >= 2 && lane < 8) *reinterpret_cast<unsigned long long *>(&L.stage[8 * (lane - 2)]) = w;
            if (lane == 0) {
              job = c;
              job_len = (uint32_t)(seq >> kServeSeqBits);
            }
            got = true;
            break;
          }
          continue;  // a read that tore (line 0 caught mid-write): read it again
        }
        // stop: the host resets the counter to its first unserved request
        // before the next launch (Server::ensure)
        if (__hip_atomic_load(&q->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
        // idle: give the number back — possible only while it is the last one
        // taken, so idle workgroups leave newest first and no posted request
        // is left without a waiter while the kernel runs
        if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) {
          unsigned int back = 0;
          if (lane == 0) back = atomicCAS(claimed, c + 1, c) == c + 1 ? 1u : 0u;
          if (__shfl(back, 0, 64)) break;
        }
        // back off: ~0.1 us while requests flow, up to ~0.4 us when idle (a
        // poll is one PCIe read of the slot's line 0)
        for (uint32_t z = 0; z < nap; z++) __builtin_amdgcn_s_sleep(4);
        nap = nap < 4 ? nap + 1 : nap;
      }
      if (lane == 0) quit = got ? 0 : 1;
    }
    __syncthreads();
    if (quit) {
      // the launch's last workgroup out tells the host (q->exited = gen): a
      // caller that posts after it relaunches at once instead of waiting for
      // its liveness check
      if (tid == 0 && atomicAdd(ctr + 1, 1ull) == (unsigned long long)gridDim.x - 1) {
        __threadfence_system();
        __hip_atomic_store(&q->exited, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      break;
    }
    ServeSlot *slot = &q->slot[job % kServeSlots];
    if (tid == 0) slot->t_claim = __builtin_amdgcn_s_memrealtime();
    if (s.stamp[0] && tid == 0) {
      if (ver != s.version) printf("mqmatch stamp: k_serve launched for version %llu on snapshot %llu\n", ver,
                                   (unsigned long long)s.version);
      check_stamps(s, "k_serve", job);
    }
    ServeSink sink{slot, &q->done[job % kServeSlots], slot->dout, slot->hout, want_ids ? slot->iout : nullptr, job,
                   ver};
    fast_topic(s, L, reinterpret_cast<const uint8_t *>(slot->topic), min(job_len, kServeTopic + 1), sink, kServeHead);
    __syncthreads();
  }
}

#define HIP_TRY(x)                                                                                        \
  do {                                                                                                    \
    hipError_t e_ = (x);                                                                                  \
    if (e_ != hipSuccess) {                                                                               \
      fprintf(stderr, "mqmatch: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
      return -3;                                                                                          \
    }                                                                                                     \
  } while (0)

// a pinned, device-mapped host block of at least `need` bytes (grown, never
// shrunk); coherent (fine-grained: the kernel's writes reach host memory as
// they are made) only for the status word the host polls — inputs and
// results stay cached (coarse-grained), read after the stream synchronisation
int pinned_grow(void **p, size_t *cap, size_t need, bool coherent = false) {
  if (*p && *cap >= need) return 0;
  if (*p) (void)hipHostFree(*p);
  *p = nullptr;
  *cap = 0;
  const size_t n = std::max<size_t>(need + need / 4, 4096);
  if (hipHostMalloc(p, n, hipHostMallocMapped | (coherent ? hipHostMallocCoherent : 0)) != hipSuccess) {
    *p = nullptr;
    return -2;
  }
  *cap = n;
  return 0;
}

}  // namespace

static bool spin_sync() {
  static const bool v = getenv("MQM_SPIN_SYNC") && atoi(getenv("MQM_SPIN_SYNC")) != 0;
  return v;
}

FastArena::~FastArena() {
  if (done_ev) (void)hipEventDestroy(done_ev);
  for (void *p : {(void *)in_bytes, (void *)in_offs, (void *)recs, (void *)dout, (void *)hout, (void *)iout,
                  (void *)status})
    if (p) (void)hipHostFree(p);
  if (ctl) (void)hipFree(ctl);
}

int stamp_counts(uint64_t *out) {
  unsigned long long v[3] = {};
  HIP_TRY(hipMemcpyFromSymbol(v, HIP_SYMBOL(g_stamp), sizeof(v), 0, hipMemcpyDeviceToHost));
  for (int i = 0; i < 3; i++) out[i] = v[i];
  return 0;
}

int serve_launch(const DeviceSnapshot &s, ServeQueue *q, unsigned long long *ctr, uint32_t grid, uint32_t idle_us,
                 bool want_ids, uint64_t ver, uint64_t gen, uint64_t seen, hipStream_t st) {
  const uint64_t idle_ticks = (uint64_t)idle_us * 100;  // s_memrealtime: 100 MHz
  hipLaunchKernelGGL(k_serve, dim3(std::max<uint32_t>(1, grid)), dim3(kFT), 0, st, s, q, ctr, idle_ticks,
                     want_ids ? 1 : 0, (unsigned long long)ver, (unsigned long long)gen, (unsigned long long)seen);
  HIP_TRY(hipGetLastError());
  return 0;
}

int match_small(const DeviceSnapshot &s, Workspace &ws, const char *bytes, const uint64_t *offs, uint32_t n,
                hipStream_t st, FastOutput *out, bool want_ids) {
  FastArena &a = ws.fast;
  const uint64_t base = offs[0], nbytes = offs[n] - base;
  if (!a.ctl) {
    if (hipMalloc(&a.ctl, sizeof(FastCtl)) != hipSuccess) {
      a.ctl = nullptr;
      return -2;
    }
    HIP_TRY(hipMemsetAsync(a.ctl, 0, sizeof(FastCtl), st));
  }
  if (!a.grid) {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_fast, kFT, 0) != hipSuccess || per < 1)
      per = 1, cus = 256;
    a.grid = (uint32_t)(per * cus);
  }
  if (pinned_grow((void **)&a.in_bytes, &a.in_cap, nbytes + 16) ||
      pinned_grow((void **)&a.in_offs, &a.offs_cap, sizeof(uint64_t) * (n + 1)) ||
      pinned_grow((void **)&a.recs, &a.rec_cap, sizeof(FastRec) * (n + 1)) ||
      pinned_grow((void **)&a.status, &a.status_cap, sizeof(FastStatus), true))
    return -2;
  if (!a.dout && (pinned_grow((void **)&a.dout, &a.dout_cap, sizeof(uint64_t) * (1u << 16)) ||
                  pinned_grow((void **)&a.hout, &a.hout_cap, sizeof(uint32_t) * (1u << 12))))
    return -2;
  if (want_ids && !a.iout && pinned_grow((void **)&a.iout, &a.iout_cap, sizeof(uint32_t) * (1u << 16))) return -2;
  // the previous call on this workspace has been waited for (its results read)
  if (nbytes) memcpy(a.in_bytes, bytes + base, nbytes);
  for (uint32_t i = 0; i <= n; i++) a.in_offs[i] = offs[i] - base;
  for (int attempt = 0; attempt < 3; attempt++) {
    a.status->done = 0;
    const uint32_t grid = std::max<uint32_t>(1, std::min<uint32_t>(n, a.grid));
    hipLaunchKernelGGL(k_fast, dim3(grid), dim3(kFT), 0, st, s, (const uint8_t *)a.in_bytes, a.in_offs, n, a.ctl,
                       a.recs, a.dout, a.dout_cap / sizeof(uint64_t), a.hout, a.hout_cap / sizeof(uint32_t),
                       want_ids ? a.iout : nullptr, a.iout_cap / sizeof(uint32_t), a.status);
    HIP_TRY(hipGetLastError());
    if (spin_sync()) {
      HIP_TRY(hipStreamSynchronize(st));
    } else {
      if (!a.done_ev) HIP_TRY(hipEventCreateWithFlags(&a.done_ev, hipEventBlockingSync | hipEventDisableTiming));
      HIP_TRY(hipEventRecord(a.done_ev, st));
      HIP_TRY(hipEventSynchronize(a.done_ev));
    }
    FastStatus stt;
    memcpy(&stt, (const void *)a.status, sizeof(stt));  // after the stream synchronisation
    if (!stt.done) {
      // the last workgroup never reset the counters: clear them, so the next
      // call on this context starts from zero instead of failing the same way
      (void)hipMemsetAsync(a.ctl, 0, sizeof(FastCtl), st);
      (void)hipStreamSynchronize(st);
      return -3;
    }
    if (stt.flags & kFastFallback) return 1;  // the caller runs the batch pipeline
    if (!(stt.flags & kFastOverflow)) {
      out->n_topics = n;
      out->n_slots = stt.d_total;
      out->n_shared_slots = stt.h_total;
      out->recs = a.recs;
      out->dout = a.dout;
      out->hout = a.hout;
      out->iout = want_ids ? a.iout : nullptr;
      return 0;
    }
    // a result block was too small: grow them to the totals this attempt reported
    if (pinned_grow((void **)&a.dout, &a.dout_cap, sizeof(uint64_t) * (stt.d_total + 1)) ||
        pinned_grow((void **)&a.hout, &a.hout_cap, sizeof(uint32_t) * (stt.h_total + 1)) ||
        (want_ids && pinned_grow((void **)&a.iout, &a.iout_cap, sizeof(uint32_t) * (stt.i_total + 1))))
      return -2;
  }
  return 1;
}

}  // namespace mqm
