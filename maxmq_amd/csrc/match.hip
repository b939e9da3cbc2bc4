// maxmq_amd/csrc/match.hip — gfx950 kernels for TopicsIndex.Subscribers
// (vendor/github.com/mochi-co/mqtt/v2/topics.go:484-555) over a batch of
// publish topics, against the GPU-resident CSR level-trie (snapshot.h).
//
// One pass over the trie per topic, then deduplication sized to the topic:
//   k_walk    a 4-lane group per topic, 16 topics per wavefront.
//     1. tokenize : the group scans the topic kStage bytes at a time and
//                   ballots the '/' positions; lane k builds the 128-bit keys
//                   of levels k, k + 4, ...
//     2. walk     : level-synchronous over the frontier; each frontier node
//                   enqueues only the loads it needs (literal edge probe,
//                   checked against the edge filter when pushed / '+' child /
//                   '#' child), so a level costs one dependent memory round
//                   trip (the literal child's descriptor is inline in its
//                   edge entry; a wildcard child's 64-B node slot carries its
//                   own '+' child's descriptor, which waits in LDS for the
//                   next level: that '+' item costs no load).  Hits are
//                   compacted with ballot + popcount
//                   and written to the topic's record: solo parts (off,
//                   count), multi parts (off, count, rank = 2 * node + slot,
//                   the reference's emission order, snapshot.h), shared
//                   ranges; S (raw entries) and H (shared candidates) counted.
//   scans     S and H -> each topic's segment start (S bounds its
//             deliveries, so every later kernel writes final positions).
//   solo copy k_desc turns the records' solo parts into copy descriptors in
//             topic order; k_longcopy moves the long parts (>= 256 entries)
//             a wavefront each with 16-B stores, k_winmap / k_wincopy copy the
//             other solo entries (~90 % of the deliveries are solo: an entry
//             whose client meets no other of its subscriptions in the topic is
//             its client's merged delivery as it stands) in fixed windows of
//             the output space, skipping the long parts' gaps.  (Round 4
//             measured the copy fused into k_walk from LDS-held parts: 15.2
//             / 17.5 ms per C3 batch at 4 / 3 waves per SIMD against 14.4 ms
//             this way — the walk's register budget leaves too few loads in
//             flight for a streaming copy; profiles/r04/r04f.)
//   k_route   topics with multi entries -> merge lists by their count Ms.
//   merges    k_resolve (partner lists, no table), k_merge_small / k_merge /
//             k_multi<N> / k_multi_part (LDS hash tables keyed by client):
//             Subscription.Merge (packets.go:250-270), winners after the
//             topic's solo deliveries.  k_shared writes shared candidates.
//   k_dfs<P>  the unbounded path for topics past a capacity (frontier, hits,
//             cached levels, shared hits, raw entries): wave-cooperative DFS
//             with an LDS stack and a global-memory dedupe table, writing to
//             a tail region after the reserved segments.
// Nothing runs on the CPU.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "device.h"
#include "flatten.h"
#include "match.h"

// MQM_WALK_STATS=1: count the walk's literal probes, the ones that found no
// child, and the wildcard-child descriptor loads (printed per batch;
// instrumentation build, `make variant VFLAGS=-DMQM_WALK_STATS=1`)
#ifndef MQM_WALK_STATS
#define MQM_WALK_STATS 0
#endif

namespace mqm {

namespace {

constexpr int kWave = 64;
constexpr int kWalkWaves = 4;            // wavefronts per k_walk block
constexpr int kWalkG = 4;                // k_walk lanes per topic (C3, round 2: 4 / 8 / 16 lanes 7.9 / 8.8 / 11.0 ms)
constexpr int kLMax = 16;                // levels cached per topic (deeper topics: DFS path)
constexpr int kHCap = 64;                // non-shared hits per topic (hit_of: 6 search steps)
constexpr int kShCap = 16;               // shared hits per topic
constexpr int kStage = 64;               // topic bytes staged in LDS (one round trip)
constexpr int kICap = 48;                // load items per level (<= 3 per frontier node; more -> DFS path)
// record of a topic, written while walking (kRecStrideAlloc words, 64-B
// aligned).  A hit range subs[off, off + c) holds solo entries, then multi
// ones (snapshot.h); the two parts are listed apart, each where its reader
// wants it, so a topic writes (and its readers read) only the parts it has:
//   from the start: [2i] off, [2i + 1] count of the i-th solo part (i <
//            nsolo[t]): k_desc's copy descriptors (and the runs form's runs)
//   [kRecSh + 2i] off, [kRecSh + 1 + 2i] cnt of shared hit i (i < nsh)
//   the tail, in 16-B units counted back from the record's end (rec_tail):
//     unit 0      header: nm | nsh << 8, Ssolo, M, nsolo (written only when M > 0,
//                 H > 0 or in the runs form: its readers)
//     unit 1 + h  multi part h (h < nm): moff, mcount, rank of its hit, 0 —
//                 multi entries subs[moff, moff + mcount); the merges copy
//                 the tail into LDS as header at word 0, part h at 4 + 4h,
//                 and turn mcount into the prefix mpre (rec_prefix)
constexpr int kRecHit = 4;
constexpr int kRecLds = 4 + kRecHit * kHCap;          // 260: header + multi parts (the merges' LDS copy)
constexpr int kRecSh = 2 * kHCap;                     // 128: shared pairs
constexpr int kRecTail = kRecSh + 2 * kShCap;         // 160: the tail area starts at or after this
constexpr int kRecStrideAlloc = 432;                  // words per topic: 1728 B = 27 x 64 B
// raw entries per hit range on the bounded path (keeps the per-lane sums of a
// topic's 64 hits inside 32 bits); emission itself has no per-topic size
// limit (the solo copy loops; partitioned merge of any number of multi entries)
constexpr uint32_t kSMax = 1u << 24;
constexpr int kEmitWaves = 4;
constexpr int kSmallLanes = 8;           // k_merge_small: lanes per topic
constexpr uint32_t kSmallHits = 15;      // k_merge_small: at most this many hits (one 64-word record prefetch)
constexpr uint32_t kSmallMultiS = 3 * kSmallLanes;  //   and multi entries
constexpr int kSmallSlots = 256;         // k_merge table slots (per wave)
constexpr int kSmallMulti = 192;         // multi entries it holds (load <= 0.75)
constexpr int kBigThreads = 256;
constexpr int kPartCap = 2048;           // k_multi_part: multi entries per client partition (expected)
constexpr uint32_t kNoWhy = 0xFFFFFFFFu;

static_assert(kRecStrideAlloc % 16 == 0 && kRecStrideAlloc >= kRecTail + kRecLds, "64-B aligned records");
static_assert(kSmallMulti * 4 <= kSmallSlots * 3, "k_emit table load factor");
static_assert(kSmallMulti % kWave == 0, "register tiles");
static_assert(kLMax % kWalkG == 0, "levels per lane");

// a load item of the walk: the literal-child probe of a frontier node (pushed
// only when the edge filter says the next level's key may be a child of it),
// or the descriptor load of its '+' / '#' child
enum : uint32_t { kItemLit = 0, kItemPlus = 1, kItemHash = 2, kItemPlusKnown = 3 };
// kItemPlusKnown: a '+' child whose descriptor came with its parent's node
// slot (DeviceSnapshot::slots) — no load; the descriptor waits in the topic's
// LDS (TopicLds::pdesc, kPK per level, by rank among the level's such items;
// a parent past kPK pushes a plain kItemPlus)
constexpr int kPK = 2;

// topic class (cls): Done = no entries and no shared candidates; Bounded (+
// FewHits when nh <= kSmallHits, for k_route) = emitted from its record; Dfs
// kClsHeavy: a gathered multi range holds an entry the merge by resolution
// cannot take (kFlagHeavyOwn / kFlagHeavyHash): the topic merges by hash table
enum : uint8_t { kClsDone = 0, kClsBounded = 1, kClsDfs = 2, kClsFewHits = 4, kClsHeavy = 8 };
enum : uint32_t { kWhyFrontier = 0, kWhyHits = 1, kWhyLevels = 2, kWhyShared = 3, kWhyEntries = 4 };

struct Counters {              // zeroed before every batch
  unsigned long long dtail;    // DFS deliveries: next free entry after the scanned segments
  unsigned long long htail;    // DFS shared candidates: likewise
  unsigned int n_dfs;          // topics appended to the DFS list
  unsigned int walk_next;      // k_walk<.., kChunk>: the next topic to hand out
  unsigned int why[5];         // DFS routing reasons (kWhy*)
  // merge lists (k_route), in kList* order
  unsigned int n_small;        // k_merge_small: 0 < Ms <= kSmallMultiS, nh <= kSmallHits
  unsigned int n_wmerge;       // k_merge: other topics with Ms <= kSmallMulti
  unsigned int n_t1;           // k_multi<1024>: kSmallMulti < Ms <= 768
  unsigned int n_t2;           // k_multi<2048>: 768 < Ms <= 1536
  unsigned int n_t3;           // k_multi<4096>: 1536 < Ms <= 3072
  unsigned int n_part;         // k_multi_part: Ms > 3072
  unsigned int n_shlist;       // k_shared: topics with shared candidates
  unsigned int n_res_small;    // k_resolve<8>: no heavy entry, Ms <= kSmallMultiS, nh <= kSmallHits
  unsigned int n_res;          // k_resolve<64>: other topics with multi entries and no heavy entry
  unsigned int res_next;       // k_resolve<.., kChunk>: the next list entry to hand out
  unsigned long long m_sum[3]; // multi entries of the k_multi<1024> / <2048> / <4096> + k_multi_part lists
  unsigned int oob;            // a store fell outside its output buffer (queued calls: buffers sized
                               //   from an earlier call were too small; the call is re-run)
  unsigned int cap_ovf;        // queued calls: the DFS lists / table / tails did not fit (re-run)
  // what the call needed (k_totals / k_dfs_prep): the next call's capacities
  unsigned long long s_total, h_total, n_desc;  // raw-entry slots, shared slots, solo parts (descriptors)
  unsigned long long n_solo;                    // solo entries the walk copied
  unsigned long long tab_total, dfs_raw, dfs_h; // DFS: dedupe table, raw entries, shared candidates
  unsigned long long d_sum, h_sum;              // deliveries, shared candidates (after dedupe)
  // Identifiers listed by the merges (Outputs::iscratch): total listed, total
  // multi entries (the scratch areas' extent), a scratch area or the packed
  // list past its capacity (then identifiers_device runs its own pass)
  unsigned long long i_total, i_multi, i_ovf;
#if MQM_WALK_STATS
  unsigned long long st_probe, st_miss, st_desc;
#endif
};

struct Outputs {
  uint32_t *hcount, *dcount;
  uint32_t *mcount;           // multi entries per topic (Ms; 0 for DFS topics)
  uint32_t *scount;           // raw entries per topic (the segment; runs form: the multi entries only)
  uint32_t *nsolo;            // solo parts per topic (k_desc's descriptors; 0 in the runs form)
  uint64_t *dstart, *hstart;  // n + 1 (exclusive scans; DFS topics overwritten)
  uint8_t *cls;
  uint32_t *dfs_list;
  uint32_t *recs;  // kRecStrideAlloc words per topic
  Counters *ctr;
  uint32_t *dout;  // packed deliveries (snapshot.h)
  uint32_t *hout;
  // identifiers pass (identifiers_device): per-topic counts, starts, sids
  uint32_t *icount;
  uint64_t *istart;
  uint32_t *iout;
  // Identifiers listed by the merges themselves (nullptr: not listed): each
  // merge writes the sids of a topic's multi entries with Identifier > 0 to
  // iscratch[imstart[t] ..) (imstart: the scan of mcount, so a topic's area
  // holds all its multi entries) and their count to icount[t]; capacity icap
  uint64_t *imstart;
  uint32_t *iscratch;
  uint64_t icap;
  // capacities of dout / hout in entries: every store is checked against them
  // (a wrong offset becomes a reported error, never an out-of-bounds write)
  uint64_t dcap, hcap;
  uint32_t dfs_cap;  // DFS topics raw_cnt / raw_h / tab_off hold
  // runs form (runs_device, mqm_match_batch_runs): no solo copy; every solo
  // part stays in the record as a run of `words`, the segment and the
  // header's solo count cover only the merge's winners
  uint32_t runs;
};

constexpr int kTopicWords = (2 * kLMax + 8 * kICap + kStage) / 4 + 2 * kPK * 8;
struct TopicLds {              // k_walk context of one topic (one lane group)
  uint16_t sep[kLMax];         // position of the '/' ending level k (topics > 64 KiB: DFS path)
  uint32_t item[2][kICap];     // the level's load items: node id << 2 | kind (kItem*)
  uint8_t stage[kStage];       // the topic's first kStage bytes
  uint32_t pdesc[2][kPK][8];   // kItemPlusKnown descriptors: [level parity][rank among the level's such items]
  uint32_t pad[kTopicWords % 2 ? 2 : 1];  // odd dword stride: the groups of a wave reading the
                               //   same field hit different banks (a 128-dword stride put all
                               //   16 groups on one bank: SQ_LDS_BANK_CONFLICT 3x the LDS cycles)
};
static_assert(kStage % 16 == 0 && kICap >= 3, "walk context");
static_assert((sizeof(TopicLds) / 4) % 2 == 1, "bank-skewed topic contexts");

__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint64_t lanemask_lt(int lane) { return (1ull << lane) - 1ull; }

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
  const uint32_t lo = __shfl((uint32_t)v, src, 64), hi = __shfl((uint32_t)(v >> 32), src, 64);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t table_slot(uint32_t client, uint32_t lg) {
  return (uint32_t)(((uint64_t)(client * 2654435769u) << lg) >> 32);
}

// Counters::oob bits: which check failed (reported when an exact call fails)
enum : unsigned int { kOobDesc = 1u, kOobStore = 2u, kOobShared = 4u, kOobHeavy = 8u, kOobPart = 16u, kOobDfs = 32u };

// a checked store: out[i] = v if i < cap, else flag the batch as failed
template <class T>
__device__ __forceinline__ void put_checked(T *out, uint64_t i, uint64_t cap, T v, unsigned int *oob,
                                            unsigned int bit = kOobStore) {
  if (i < cap)
    out[i] = v;
  else
    atomicOr(oob, bit);
}


__device__ __forceinline__ uint32_t pack_delivery(uint32_t sid, uint32_t qos, uint32_t nl) {
  return sid | (qos << 28) | (nl << 30);
}

// QoS one-hot (bits 0..2) | NoLocal (bit 3) of a SubEnt word: OR-merged, max
// QoS = top set bit
__device__ __forceinline__ uint32_t qos_bits(uint32_t word) {
  return (1u << ((word >> 28) & 3)) | (((word >> 30) & 1) << 3);
}



// the multi part h holding multi entry x (prefix field kFieldMpre): the
// largest h < nh with field(h) <= x (field(0) = 0).  Hits with none of those
// entries tie with their successor, so the largest such h is the one that
// holds x.  Branch-free binary search over the prefixes in LDS: 6 dependent
// reads for nh <= 64 (round 1 counted over every hit per entry: ~nh reads and
// 2 nh VALU ops per entry, which made emission issue-bound on big topics).
enum : int { kFieldOff = 0, kFieldMpre = 1, kFieldRank = 2 };
static_assert(kHCap <= 64, "hit_of searches 6 levels");
template <int kField>
__device__ __forceinline__ uint32_t hit_of(const uint32_t *rec, uint32_t nh, uint32_t x) {
  uint32_t h = 0;
#pragma unroll
  for (uint32_t step = 32; step > 0; step >>= 1) {
    const uint32_t c = h + step;
    const uint32_t v = rec[4 + kRecHit * (c < nh ? c : 0) + kField];
    h = ((c < nh) & (v <= x)) ? c : h;  // bitwise: no branch around the read
  }
  return h;
}

__device__ __forceinline__ uint32_t rec_at(const uint32_t *rec, uint32_t h, int field) {
  return rec[4 + kRecHit * h + field];
}

// per-topic merge table in LDS (linear probing): kb = (client + 1) << 32 |
// the QoS one-hot | NoLocal of the client's entries OR-folded, first = rank
// << 32 | sid of its first-merged subscription by a 64-bit atomicMin —
// exactly Subscription.Merge (packets.go:250-270): max QoS, NoLocal OR,
// every other field from the first subscription in the reference's emission
// order.  A client's first entry claims its slot with key and bits in one
// 64-bit CAS; only a repeated client pays an OR.  The winners are read off
// the table afterwards (one delivery per occupied slot).
struct MergeTable {
  unsigned long long *kb, *first;
};

__device__ __forceinline__ void mt_clear(MergeTable t, uint32_t j) {
  t.kb[j] = 0;
  t.first[j] = ~0ull;
}

__device__ __forceinline__ bool mt_occupied(MergeTable t, uint32_t j) { return t.kb[j] != 0; }

__device__ __forceinline__ void mt_insert(MergeTable t, uint32_t mask, uint32_t lg, uint32_t client, uint32_t word,
                                          uint32_t rank) {
  uint32_t sl = table_slot(client, lg);
  const unsigned long long key = (unsigned long long)(client + 1u) << 32, kb = key | qos_bits(word);
  for (;;) {
    const unsigned long long prev = atomicCAS(&t.kb[sl], 0ull, kb);
    if (prev == 0) break;
    if ((prev >> 32) == (key >> 32)) {
      if ((prev | kb) != prev) atomicOr(&t.kb[sl], kb);
      break;
    }
    sl = (sl + 1) & mask;
  }
  atomicMin(&t.first[sl], ((unsigned long long)rank << 32) | (word & kWordSidMask));
}

__device__ __forceinline__ uint32_t mt_delivery(MergeTable t, uint32_t j) {
  const uint32_t v = (uint32_t)t.kb[j];
  return pack_delivery((uint32_t)t.first[j] & kWordSidMask, 31u - __builtin_clz(v & 7u), (v >> 3) & 1u);
}

// ---------------------------------------------------------------------------
// k_walk: tokenize + walk, a kG-lane group per topic.  Level keys and the
// running hit counts live in registers (lane k holds the keys of levels k,
// k + kG, ...); LDS holds only the separators, the frontier and the first
// bytes of the topic, so many topics stay in flight per CU.  Hits go straight
// to the topic's record with their rank.
// ---------------------------------------------------------------------------
// A record's multi parts carry their entry counts (field kFieldMpre, as k_walk
// wrote them); the merges turn them into exclusive prefixes in their LDS copy
// (hit_of searches those).  A group of kL aligned lanes (kL <= 64, a power of
// two) converts parts 0 .. nh - 1.
template <int kL, int kCap = kHCap>
__device__ __forceinline__ void rec_prefix(uint32_t *rec, uint32_t nh, int gl) {
  constexpr int kP = (kCap + kL - 1) / kL;
  uint32_t mc[kP], ms = 0;
#pragma unroll
  for (int p = 0; p < kP; p++) {
    const uint32_t h = gl * kP + p;
    mc[p] = h < nh ? rec[4 + kRecHit * h + kFieldMpre] : 0;
    ms += mc[p];
  }
  uint32_t mi = ms;
#pragma unroll
  for (int d = 1; d < kL; d <<= 1) {
    const uint32_t um = __shfl_up(mi, d, kL);
    if (gl >= d) mi += um;
  }
  mi -= ms;
#pragma unroll
  for (int p = 0; p < kP; p++) {
    const uint32_t h = gl * kP + p;
    if (h < nh) rec[4 + kRecHit * h + kFieldMpre] = mi;
    mi += mc[p];
  }
}

// 16-B unit u of topic t's record tail is rec_tail(recs, t)[-u] (0 = header,
// 1 + h = multi part h)
__device__ __forceinline__ const uint4 *rec_tail(const uint32_t *recs, uint32_t t) {
  return reinterpret_cast<const uint4 *>(recs + ((uint64_t)t + 1) * kRecStrideAlloc) - 1;
}

// ---- Identifiers listed by the merges (Outputs::iscratch; packets.go:257-259)
// A merge reads every multi entry of its topic anyway, so it lists the ones
// whose Identifier is > 0 as it goes, in entry order (the order k_ident used:
// part by part), instead of a pass of its own over the records (k_ident: 3.6
// ms on C3, r05z).  A solo entry is its client's only one in the topic, so its
// map is its first pair, which its delivery already names (see k_ident).
// The topic's scratch base, or ~0 when listing is off or its area would pass
// the capacity (flagged: identifiers_device then runs the separate pass).
__device__ __forceinline__ uint64_t ident_base(const Outputs &o, uint32_t t, uint32_t M, bool leader) {
  if (!o.iscratch) return ~0ull;
  const uint64_t ib = o.imstart[t];
  if (ib + M > o.icap) {  // (one atomic once the flag is up, not one per topic)
    if (leader && !__hip_atomic_load(&o.ctr->i_ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      atomicOr(&o.ctr->i_ovf, 1ull);
    return ~0ull;
  }
  return ib;
}
// a kE-lane group lists the entries with `has` set at ib + nid .. in lane order
template <int kE>
__device__ __forceinline__ void ident_put(const Outputs &o, uint64_t ib, bool has, uint32_t sid, int gbase,
                                          uint64_t glt, uint32_t &nid) {
  constexpr uint64_t kGMask = kE == 64 ? ~0ull : (1ull << kE) - 1ull;
  const uint64_t m = (__ballot(has) >> gbase) & kGMask;
  if (has) o.iscratch[ib + nid + __popcll(m & glt)] = sid;
  nid += (uint32_t)__popcll(m);
}


template <int kG, int kChunk = 0, bool kSlots = true>
__global__ __launch_bounds__(kWave *kWalkWaves) __attribute__((amdgpu_waves_per_eu(4))) void k_walk(DeviceSnapshot s, const uint8_t *__restrict__ tbytes,
                                                           const uint64_t *__restrict__ toffs, uint32_t n,
                                                           Outputs o) {
  constexpr int kGroups = kWave / kG;
  constexpr int kLPer = (kLMax + kG - 1) / kG;  // level keys held per lane
  constexpr uint32_t kGMask = (1u << kG) - 1u;
  static_assert(kLMax % kG == 0 || kG > kLMax, "levels per lane");
  __shared__ TopicLds lds_all[kWalkWaves * kGroups];
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / kG, gl = lane & (kG - 1), gbase = g * kG;
  TopicLds &L = lds_all[(threadIdx.x / kWave) * kGroups + g];
  const uint32_t gmask_lt = (1u << gl) - 1u;
  const uint64_t stride = (uint64_t)gridDim.x * kWalkWaves * kGroups;
  const NodeDesc root = load_desc(s.nodes);
  // the root's '+' child (every topic visits it at level 0): its descriptor is
  // the second half of the root's slot, kept in LDS for the block (copied
  // into each topic's pdesc at its start; not a register across the loop)
  __shared__ uint32_t root_plus[8];
  if (kSlots && threadIdx.x < 8) root_plus[threadIdx.x] = reinterpret_cast<const uint32_t *>(s.slots + 1)[threadIdx.x];
  __syncthreads();
  uint32_t n_parts = 0; // solo parts of this lane's topics (Counters::n_desc; group leaders)
  uint32_t n_solo = 0;  // solo entries of this lane's topics (Counters::n_solo; group leaders, flushed before 2^32)

  // kChunk > 0: a wavefront takes kChunk steps of kGroups topics at a time
  // from a device counter (a wave that drew deep topics takes fewer), else
  // a fixed stride
  uint64_t c_end = 0;
  auto take = [&](uint64_t cur) -> uint64_t {
    if (cur + kGroups < c_end) return cur + kGroups;
    unsigned int v = 0;
    if (lane == 0) v = atomicAdd(&o.ctr->walk_next, (unsigned)(kChunk * kGroups));
    v = __builtin_amdgcn_readfirstlane(v);  // (scalar: the walk is at its VGPR budget)
    c_end = (uint64_t)v + kChunk * kGroups;
    return v;
  };
  uint64_t tb = kChunk ? take(~0ull - kGroups) : ((uint64_t)blockIdx.x * kWalkWaves + threadIdx.x / kWave) * kGroups;
  uint64_t nx_off = 0, nx_end = 0;  // the next topic's byte range, one topic ahead
  if (tb + g < n) {
    nx_off = toffs[tb + g];
    nx_end = toffs[tb + g + 1];
  }
  for (uint64_t tb_next; tb < n; tb = tb_next) {
    tb_next = kChunk ? take(tb) : tb + stride;
    const bool active = tb + g < n;
    const uint32_t t = active ? (uint32_t)(tb + g) : n;  // (inactive lanes never use t)
    const uint32_t len = active ? (uint32_t)(nx_end - nx_off) : 0;
    const uint8_t *tp = tbytes + (active ? nx_off : 0);
    if (tb_next + g < n) {
      nx_off = toffs[tb_next + g];
      nx_end = toffs[tb_next + g + 1];
    }
    uint32_t why = kNoWhy;

    // ---- 1. tokenize ------------------------------------------------------
    // lane gl takes the chunk's bytes [16 gl, 16 gl + 16) as 5 aligned dword
    // loads (clamped into the topic's last dword), one round trip; 16 byte
    // loads per lane cost the address unit 16 instructions per chunk (TA busy
    // 0.69 in the walk, r04ay).  Separators: counted per lane, placed in order
    // through the group's prefix.  The first chunk is kept in LDS for the key
    // build below.
    static_assert(kStage == 16 * kG, "16 bytes per lane per chunk");
    uint32_t nsep = 0;
    bool dollar = false;
    for (uint32_t base = 0; base < len && nsep < (uint32_t)kLMax; base += kStage) {
      const uint32_t p0 = base + 16 * gl;
      const uint64_t first = reinterpret_cast<uint64_t>(len ? tp + p0 : o.cls);
      const uint64_t lastw = reinterpret_cast<uint64_t>(len ? tp + len - 1 : o.cls) & ~3ull;
      const uint64_t a0 = first & ~3ull;
      const uint32_t r = (uint32_t)(first & 3u);
      uint32_t w[5];
#pragma unroll
      for (int k = 0; k < 5; k++) w[k] = *reinterpret_cast<const uint32_t *>(min(a0 + 4 * k, lastw));
      uint32_t b4[4];  // the lane's 16 bytes, little-endian words, shifted by r
#pragma unroll
      for (int k = 0; k < 4; k++) b4[k] = align_byte(w[k + 1], w[k], r);
      // bytes at or past len read as 0 (never a separator)
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t pk = p0 + 4 * k;
        if (pk >= len) b4[k] = 0;
        else if (pk + 4 > len) b4[k] &= 0xFFFFFFFFu >> (8 * (pk + 4 - len));
      }
      if (base == 0) {
#pragma unroll
        for (int k = 0; k < 4; k++) reinterpret_cast<uint32_t *>(L.stage)[4 * gl + k] = b4[k];
        dollar = (__shfl(b4[0], gbase, 64) & 0xFFu) == '$';
      }
      const uint32_t sm = slash_mask16(b4);  // the lane's '/' bytes (keys.h)
      const uint32_t cnt = __popc(sm);
      uint32_t pre = cnt;  // inclusive prefix over the group's lanes
#pragma unroll
      for (int d = 1; d < kG; d <<= 1) {
        const uint32_t v = __shfl_up(pre, d, kG);
        if (gl >= d) pre += v;
      }
      uint32_t idx = nsep + pre - cnt;
      for (uint32_t m = sm; m; m &= m - 1, idx++)
        if (idx < (uint32_t)kLMax) L.sep[idx] = (uint16_t)(p0 + __builtin_ctz(m));
      nsep += __shfl(pre, gbase + kG - 1, 64);
    }
    // levels known: 0 .. nlev-1, with nlev capped at kLMax + 1
    const uint32_t nlev = len == 0 ? 0 : (nsep >= (uint32_t)kLMax ? kLMax + 1 : nsep + 1);
    wave_lds_sync();
    uint64_t my_k0[kLPer], my_k1[kLPer];  // lane gl: the keys of levels gl, gl + kG, ...
#pragma unroll
    for (int j = 0; j < kLPer; j++) {
      const uint32_t lv = gl + j * kG;
      my_k0[j] = my_k1[j] = 0;
      if (lv < nlev && lv < (uint32_t)kLMax) {
        const uint32_t st = lv == 0 ? 0 : L.sep[lv - 1] + 1;
        const uint32_t en = (lv < nsep) ? L.sep[lv] : len;
        Key k = en <= (uint32_t)kStage ? make_key([&](uint32_t i) { return L.stage[st + i]; }, en - st)
                                       : make_key([&](uint32_t i) { return tp[st + i]; }, en - st);
        my_k0[j] = k.k0;
        my_k1[j] = k.k1;
      }
    }
    // level 0's items: the root's literal probe, '+' (its descriptor known:
    // the root's slot) and '#' children
    if (gl == 0) {
      uint32_t k = 0;
      if ((root.sh_cnt_flags >> 24) & kFlagHasLiteral) L.item[0][k++] = (0u << 2) | kItemLit;
      if (root.plus != kNone) L.item[0][k++] = (root.plus << 2) | (kSlots ? kItemPlusKnown : kItemPlus);
      if (root.hash != kNone) L.item[0][k++] = (root.hash << 2) | kItemHash;
    }
    if (kSlots && root.plus != kNone) {  // (lanes gl copy words gl, gl + kG, ...)
#pragma unroll
      for (int w = 0; w < 8; w += kG) L.pdesc[0][0][w + gl] = root_plus[w + gl];
    }
    const uint32_t root_items = (((root.sh_cnt_flags >> 24) & kFlagHasLiteral) ? 1u : 0u) +
                                (root.plus != kNone ? 1u : 0u) + (root.hash != kNone ? 1u : 0u);
    wave_lds_sync();

    // ---- 2. walk ----------------------------------------------------------
    // Level-synchronous over compact item lists: a node pushed to the next
    // level enqueues only the loads it needs (its literal probe if it has a
    // literal child, its '+' child, its '#' child unless kFlagHashLeaf lets
    // the '#' child's gather be recorded at push time: partKey '#' of the
    // next level, topics.go:503-505, rank 2 * '#' child).
    uint32_t *rec = o.recs + (uint64_t)(active ? t : 0) * kRecStrideAlloc;
    uint4 *tail = reinterpret_cast<uint4 *>(rec + kRecStrideAlloc) - 1;  // unit u at tail[-u]
    if (len > 0xFFFFu) why = kWhyLevels;  // separators are kept as 16-bit positions
    uint32_t ni = nlev > 0 && why == kNoWhy ? root_items : 0, nh = 0, nsh = 0, nq = 0, nm = 0;
    uint32_t ls = 0, lm = 0, lh = 0;  // this lane's solo / multi / shared entries
    bool heavy = false;                // a gathered multi range with a heavy entry (kClsHeavy)
    int cur = 0;
    for (uint32_t d = 0; d < nlev && ni > 0; d++) {
      if (d >= (uint32_t)kLMax) {
        why = kWhyLevels;
        break;
      }
      uint64_t s0 = my_k0[0], s1 = my_k1[0];
#pragma unroll
      for (int j = 1; j < kLPer; j++)
        if (d / kG == (uint32_t)j) s0 = my_k0[j], s1 = my_k1[j];
      const uint64_t k0 = shfl64(s0, gbase + (int)(d % kG)), k1 = shfl64(s1, gbase + (int)(d % kG));
      const bool has_next = d + 1 < nlev;
      // key == "+" / "#": the literal probe IS the wildcard probe (the
      // reference visits that child twice; no parent probe: topics.go:507)
      const bool lit_is_wild = (k1 == (1ull << 56)) && (k0 == '+' || k0 == '#');
      // the next level's key, for the filter check of the literal items this
      // level pushes (d + 1 < kLMax; the walk leaves at kLMax otherwise)
      uint64_t n0 = my_k0[0], n1 = my_k1[0];
#pragma unroll
      for (int j = 1; j < kLPer; j++)
        if ((d + 1) / kG == (uint32_t)j) n0 = my_k0[j], n1 = my_k1[j];
      const uint64_t nk0 = shfl64(n0, gbase + (int)((d + 1) % kG)), nk1 = shfl64(n1, gbase + (int)((d + 1) % kG));
      const bool next_wild = (nk1 == (1ull << 56)) && (nk0 == '+' || nk0 == '#');
      const uint32_t tst = d == 0 ? 0 : L.sep[d - 1] + 1;
      const uint32_t tln = ((d < nsep) ? L.sep[d] : len) - tst;
      uint32_t nnext = 0;
      uint32_t k3r = 0, k3w = 0;  // kItemPlusKnown items read at this level / carried to the next (group-uniform)
      for (uint32_t base = 0; base < ni; base += kG) {
        const uint32_t it = base + gl;
        const bool live = it < ni;
        const uint32_t iw = L.item[cur][live ? it : 0];
        const uint32_t kind = iw & 3u, id = iw >> 2;
        const bool lit = kind == kItemLit;
        const bool known = live && kind == kItemPlusKnown;
        const uint32_t m3 = (uint32_t)(__ballot(known) >> gbase) & kGMask;
        const uint32_t r3 = k3r + __popc(m3 & gmask_lt);
        k3r += __popc(m3);
        // a node loaded from its slot brings its '+' child's descriptor: when
        // that child is pushed, the descriptor goes to the next level in LDS
        // (the first kPK such per level) right at the load (the walk is at its
        // VGPR budget)
        const bool slot_load = live && !lit && !known;
        bool pk = false;
        NodeDesc dc;
        uint32_t c = !kSlots ? walk_step(s, live && lit && !lit_is_wild, slot_load, id, id, k0, k1, tp + tst, tln, &dc)
                             : walk_step_slot(s, live && lit && !lit_is_wild, slot_load, id, id, k0, k1, tp + tst, tln, &dc,
                                    [&](bool ld, const uint4 &a0, const uint4 &a1, const uint4 &p0, const uint4 &p1) {
                                      // (pushed: has_next and children; x.plus = a0.x, flags = a1.w >> 24)
                                      const bool want3 = ld && has_next && ((a1.w >> 24) & kFlagHasChildren) &&
                                                         a0.x != kNone;
                                      const uint32_t mw = (uint32_t)(__ballot(want3) >> gbase) & kGMask;
                                      const uint32_t w3 = k3w + __popc(mw & gmask_lt);
                                      pk = want3 && w3 < (uint32_t)kPK;
                                      k3w += __popc(mw);
                                      if (pk) {
                                        uint32_t *q = L.pdesc[(d + 1) & 1][w3];
                                        q[0] = p0.x, q[1] = p0.y, q[2] = p0.z, q[3] = p0.w;
                                        q[4] = p1.x, q[5] = p1.y, q[6] = p1.z, q[7] = p1.w;
                                      }
                                    });
        if (known) {
          const uint32_t *q = L.pdesc[d & 1][r3];
          dc = NodeDesc{q[0], q[1], q[2], q[3], q[4], q[5], q[6], q[7]};
          c = id;
        }
        const bool found = c != kNone;
#if MQM_WALK_STATS
        {
          const bool pr = live && lit && !lit_is_wild;
          const uint32_t mp = (uint32_t)(__ballot(pr) >> gbase) & kGMask;
          const uint32_t mm = (uint32_t)(__ballot(pr && !found) >> gbase) & kGMask;
          const uint32_t md = (uint32_t)(__ballot(slot_load) >> gbase) & kGMask;
          if (gl == 0) {
            atomicAdd(&o.ctr->st_probe, (unsigned long long)__popc(mp));
            atomicAdd(&o.ctr->st_miss, (unsigned long long)__popc(mm));
            atomicAdd(&o.ctr->st_desc, (unsigned long long)__popc(md));
          }
        }
#endif
        const uint32_t fl = found ? dc.sh_cnt_flags >> 24 : 0;
        const bool skip_dollar = dollar && (fl & kFlagDollarWild);  // topics.go:527
        // (a '#' node after a literal parent: its parent probe gathered it, kFlagParentLit)
        const uint32_t c_own = found && !skip_dollar && !(fl & kFlagParentLit) ? dc.sub_cnt : 0;
        const uint32_t c_par = found && lit && !skip_dollar ? dc.hsub_cnt : 0;  // topics.go:507-509
        const uint32_t c_sh = found ? dc.sh_cnt_flags & kShCntMask : 0;
        const bool push = found && has_next && (fl & kFlagHasChildren);
        const bool leaf = push && (fl & kFlagHashLeaf);
        // the '#' child's gather at the next level ('$' flag = this node's); after
        // a literal hit c_par gathered the same range (kFlagParentLit)
        const uint32_t c_hl = leaf && !skip_dollar && !lit ? dc.hsub_cnt : 0;
        // the pushed literal probe's filter word, loaded now: its round trip
        // overlaps this level's record writes, and a negative (or a '+' / '#'
        // next level, whose literal probe is the wildcard's) drops the item
        const bool chk = push && (fl & kFlagHasLiteral) && s.bloom && d + 1 < (uint32_t)kLMax && !next_wild;
        const uint64_t nh2 = chk ? edge_hash(c, Key{nk0, nk1}) : 0;
        const uint64_t bw = chk ? s.bloom[bloom_word(nh2, s.bloom_mask)] : 0;
        const uint64_t bb = bloom_bits(nh2);
        const uint32_t m_own = (uint32_t)(__ballot(c_own > 0) >> gbase) & kGMask;
        const uint32_t m_par = (uint32_t)(__ballot(c_par > 0) >> gbase) & kGMask;
        const uint32_t m_hl = (uint32_t)(__ballot(c_hl > 0) >> gbase) & kGMask;
        const uint32_t m_sh = (uint32_t)(__ballot(c_sh > 0) >> gbase) & kGMask;
        const uint32_t n_own = __popc(m_own), n_par = __popc(m_par), n_hl = __popc(m_hl);
        if (nh + n_own + n_par + n_hl > (uint32_t)kHCap) why = kWhyHits;
        if (nsh + __popc(m_sh) > (uint32_t)kShCap) why = kWhyShared;
        // a saturated multi count, or a range past the bounded path's entries
        // (also keeps the per-lane sums below from overflowing)
        if ((uint32_t)(__ballot(((c_own | c_par | c_hl) && (fl & kFlagMultiSat)) ||
                                max(c_own, max(c_par, c_hl)) > kSMax) >> gbase) & kGMask)
          why = kWhyEntries;
        if (why != kNoWhy) break;
        // solo / multi split of the ranges (multi entries sit at the end of a
        // range; the '#' child's range follows its parent's, snapshot.h): the
        // multi parts go to the record's tail with their hit's rank
        const uint32_t mu_own = c_own ? (dc.multi & 0xFFFFu) : 0, mu_par = c_par ? (dc.multi >> 16) : 0;
        const uint32_t mu_hl = c_hl ? (dc.multi >> 16) : 0;
        heavy |= (mu_own && (fl & kFlagHeavyOwn)) || ((mu_par | mu_hl) && (fl & kFlagHeavyHash));
        const uint32_t hoff = dc.sub_off + dc.sub_cnt;
        const uint32_t x_own = (uint32_t)(__ballot(mu_own > 0) >> gbase) & kGMask;
        const uint32_t x_par = (uint32_t)(__ballot(mu_par > 0) >> gbase) & kGMask;
        const uint32_t x_hl = (uint32_t)(__ballot(mu_hl > 0) >> gbase) & kGMask;
        if (active && mu_own)
          tail[-(int)(1 + nm + __popc(x_own & gmask_lt))] = make_uint4(dc.sub_off + c_own - mu_own, mu_own, 2 * c, 0);
        if (active && mu_par)
          tail[-(int)(1 + nm + __popc(x_own) + __popc(x_par & gmask_lt))] =
              make_uint4(hoff + c_par - mu_par, mu_par, 2 * c + 1, 0);
        if (active && mu_hl)
          tail[-(int)(1 + nm + __popc(x_own) + __popc(x_par) + __popc(x_hl & gmask_lt))] =
              make_uint4(hoff + c_hl - mu_hl, mu_hl, 2 * dc.hash, 0);
        nm += __popc(x_own) + __popc(x_par) + __popc(x_hl);
        if (active && c_sh) {
          const uint32_t i = nsh + __popc(m_sh & gmask_lt);
          *reinterpret_cast<uint2 *>(rec + kRecSh + 2 * i) = make_uint2(dc.sh_off, c_sh);
        }
        // the solo parts, as (off, solo count) pairs from the record's start
        const uint32_t q_own = (uint32_t)(__ballot(c_own > mu_own) >> gbase) & kGMask;
        const uint32_t q_par = (uint32_t)(__ballot(c_par > mu_par) >> gbase) & kGMask;
        const uint32_t q_hl = (uint32_t)(__ballot(c_hl > mu_hl) >> gbase) & kGMask;
        if (active && c_own > mu_own)
          *reinterpret_cast<uint2 *>(rec + 2 * (nq + __popc(q_own & gmask_lt))) =
              make_uint2(dc.sub_off, c_own - mu_own);
        if (active && c_par > mu_par)
          *reinterpret_cast<uint2 *>(rec + 2 * (nq + __popc(q_own) + __popc(q_par & gmask_lt))) =
              make_uint2(hoff, c_par - mu_par);
        if (active && c_hl > mu_hl)
          *reinterpret_cast<uint2 *>(rec + 2 * (nq + __popc(q_own) + __popc(q_par) + __popc(q_hl & gmask_lt))) =
              make_uint2(hoff, c_hl - mu_hl);
        nq += __popc(q_own) + __popc(q_par) + __popc(q_hl);
        // the next level's items (after the record writes: the frontier cap
        // needs the filter's answer; a topic leaving here goes to the DFS path)
        // (at d + 1 == kLMax the item is kept: the next level routes the topic to
        // the DFS path; without a filter, every literal item unless the next
        // level is '+' / '#')
        const bool lit_next = (fl & kFlagHasLiteral) &&
                              (d + 1 >= (uint32_t)kLMax || (s.bloom ? (chk && (bw & bb) == bb) : !next_wild));
        const uint32_t n_items = push ? ((lit_next ? 1u : 0u) + (dc.plus != kNone ? 1u : 0u) +
                                         (dc.hash != kNone && !leaf ? 1u : 0u))
                                      : 0u;
        const uint32_t m_i0 = (uint32_t)(__ballot(n_items & 1u) >> gbase) & kGMask;
        const uint32_t m_i1 = (uint32_t)(__ballot(n_items & 2u) >> gbase) & kGMask;
        const uint32_t t_items = __popc(m_i0) + 2 * __popc(m_i1);
        if (nnext + t_items > (uint32_t)kICap) {
          why = kWhyFrontier;
          break;
        }
        if (push) {
          uint32_t *nx = &L.item[cur ^ 1][nnext + __popc(m_i0 & gmask_lt) + 2 * __popc(m_i1 & gmask_lt)];
          uint32_t k = 0;
          if (lit_next) nx[k++] = (c << 2) | kItemLit;
          if (dc.plus != kNone) nx[k++] = (dc.plus << 2) | (pk ? kItemPlusKnown : kItemPlus);
          if (dc.hash != kNone && !leaf) nx[k++] = (dc.hash << 2) | kItemHash;
        }
        nh += n_own + n_par + n_hl;
        nsh += __popc(m_sh);
        nnext += t_items;
        ls += c_own - mu_own + c_par - mu_par + c_hl - mu_hl;
        lm += mu_own + mu_par + mu_hl;
        lh += c_sh;
      }
      wave_lds_sync();
      if (why != kNoWhy) break;
      cur ^= 1;
      ni = nnext;
    }
#pragma unroll
    for (int m = kG / 2; m > 0; m >>= 1) {  // group totals
      ls += __shfl_xor(ls, m, 64);
      lm += __shfl_xor(lm, m, 64);
      lh += __shfl_xor(lh, m, 64);
    }
    const uint32_t Ss = ls, Ms = lm, H = lh;
    const uint32_t S = Ss + Ms;
    const bool any_heavy = ((__ballot(heavy) >> gbase) & kGMask) != 0;
    if (why == kNoWhy && S > kSMax) why = kWhyEntries;
    if (active && gl == 0) {
      const bool dfs = why != kNoWhy;
      // the header: read by the merges (Ms > 0), k_shared (H > 0) and the
      // runs form's run listing; k_ident takes nq from nsolo and nm = 0 from
      // Ms == 0 otherwise — most topics skip this 16-B write (a sector of its own)
      if (!dfs && (Ms || H || o.runs)) tail[0] = make_uint4(nm | (nsh << 8), o.runs ? 0u : Ss, Ms, nq);
      o.cls[t] = dfs ? kClsDfs
                     : (S == 0 && H == 0) ? kClsDone
                                          : (kClsBounded | (nm <= kSmallHits ? kClsFewHits : 0) | (any_heavy ? kClsHeavy : 0));
      o.nsolo[t] = dfs || o.runs ? 0 : nq;  // (runs form: no solo copy; the parts stay in the record)
      o.scount[t] = dfs ? 0 : o.runs ? Ms : S;  // the segment: raw entries (runs form: the winners' only)
      if (!dfs) {
        if (n_solo + Ss < n_solo) atomicAdd(&o.ctr->n_solo, (unsigned long long)n_solo), n_solo = 0;
        n_solo += Ss;
        n_parts += nq;
      }
      o.hcount[t] = dfs ? 0 : H;
      o.mcount[t] = dfs ? 0 : Ms;
      o.dcount[t] = 0;
      if (dfs) {
        o.dfs_list[atomicAdd(&o.ctr->n_dfs, 1u)] = t;
        atomicAdd(&o.ctr->why[why], 1u);
      }
    }
    wave_lds_sync();
  }
  if (n_solo) atomicAdd(&o.ctr->n_solo, (unsigned long long)n_solo);  // (group leaders)
  if (n_parts) atomicAdd(&o.ctr->n_desc, (unsigned long long)n_parts);
}


// ---------------------------------------------------------------------------
// Emission of the topics with multi entries.  A topic's deliveries are
// written at dstart[t] (the walk's reservation of its raw-entry count S, an
// upper bound): first its solo entries (the walk copied them), then the
// winners of the merge of its multi entries, compacted.  dcount[t] = Ss +
// winners.  Merges by the topic's multi count Ms (k_route lists):
// k_resolve<8|64> (by resolution, no table), k_merge_small (8 lanes per
// topic, Ms <= 24, <= 15 hits), k_merge (a wavefront, Ms <= 192),
// k_multi<1024|2048|4096>, k_multi_part.  The table merge: an LDS hash table
// keyed by client — atomicOr folds QoS (one-hot) and NoLocal, a 64-bit
// atomicMin keeps the lowest (hit rank, sid): exactly Subscription.Merge
// (packets.go:250-270) with the first-merged subscription's fields.
// ---------------------------------------------------------------------------

// multi entry q of a topic: subs index and multi part
__device__ __forceinline__ uint32_t multi_sid(const uint32_t *rec, uint32_t nh, uint32_t q, uint32_t *hit) {
  const uint32_t h = hit_of<kFieldMpre>(rec, nh, q);
  *hit = h;
  return rec_at(rec, h, kFieldOff) + (q - rec_at(rec, h, kFieldMpre));
}

__device__ __forceinline__ SubEnt load_sub(const DeviceSnapshot &s, uint32_t sid) {
  const uint2 v = *reinterpret_cast<const uint2 *>(s.subs + sid);
  return SubEnt{v.x, v.y};
}

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// ---- k_desc: solo parts -> copy descriptors ----------------------------------
// A wavefront per 64 consecutive topics.  Their descriptors are one contiguous
// range of desc (desc_start is the exclusive scan of nsolo), so lane k writes
// descriptor k of the range (coalesced 16-B stores): its topic by a 6-step
// search over the wave's prefix of solo-part counts in LDS, its output
// position by a segmented scan of the part sizes (running per-topic position
// carried in LDS across 64-part steps).  Also dcount of topics without multi
// entries (the merges write the others').  Round 1 ran a thread per topic:
// scattered 16-B stores wrote 2.8x the descriptor bytes.
struct alignas(8) DescLds {
  unsigned long long run[kWave];  // next output position of each topic's solo part
  uint32_t pre[kWave + 1];        // exclusive prefix of the topics' solo-part counts
};

// a long solo part's descriptor keeps its length with this flag: the window
// copy reads it as empty (a gap), k_longcopy finds it by the flag
constexpr uint32_t kDescLong = 0x80000000u;

// kCopy (MQM_DESC_COPY=1, A/B): no descriptors — the wave copies the step's
// 64 parts itself, 4 parts at a time, each by the whole wavefront (lanes over
// its entries: no position -> descriptor search, no k_winmap / k_wincopy)
template <bool kCopy = false>
__global__ __launch_bounds__(256) void k_desc(DeviceSnapshot s, Outputs o, uint32_t n,
                                              const uint64_t *__restrict__ desc_start, uint4 *__restrict__ desc,
                                              uint64_t desc_cap, uint32_t long_min) {
  __shared__ DescLds lds_all[4];
  const int lane = threadIdx.x & (kWave - 1);
  DescLds &L = lds_all[threadIdx.x / kWave];
  const uint32_t nw = gridDim.x * (blockDim.x / kWave);
  for (uint32_t w = blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave; (uint64_t)w * kWave < n; w += nw) {
    const uint32_t t0 = w * kWave, t = t0 + lane;
    uint32_t q = 0;
    uint64_t db = 0;
    if (t < n) {
      const uint8_t cls = o.cls[t];
      if (cls & kClsBounded) {
        q = o.nsolo[t];
        db = o.dstart[t];
        if (o.mcount[t] == 0) o.dcount[t] = o.scount[t];
      }
    }
    uint32_t inc = q;  // inclusive scan of q over the wave
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      const uint32_t v = __shfl_up(inc, d, kWave);
      if (lane >= d) inc += v;
    }
    const uint32_t Q = __shfl(inc, kWave - 1, kWave);
    if (Q == 0) continue;  // wave-uniform
    L.pre[lane] = inc - q;
    if (lane == 0) L.pre[kWave] = Q;
    L.run[lane] = db;
    const uint64_t pb = desc_start[t0];
    wave_lds_sync();
    for (uint32_t k0 = 0; k0 < Q; k0 += kWave) {
      const uint32_t k = k0 + lane;
      const bool valid = k < Q;
      uint32_t j = 0;  // the topic holding part k: the largest j with pre[j] <= k
#pragma unroll
      for (uint32_t step = 32; step > 0; step >>= 1) j = L.pre[j + step] <= k ? j + step : j;  // j + step <= 63
      uint2 part = make_uint2(0, 0);
      if (valid) part = *reinterpret_cast<const uint2 *>(o.recs + (uint64_t)(t0 + j) * kRecStrideAlloc + 2 * (k - L.pre[j]));
      const uint32_t seg = valid ? j : kWave;  // invalid lanes: a segment of their own, size 0
      uint32_t si = part.y;
#pragma unroll
      for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t v = __shfl_up(si, d, kWave);
        const uint32_t sj = __shfl_up(seg, d, kWave);
        if (lane >= d && sj == seg) si += v;
      }
      const uint64_t at = valid ? L.run[j] + (si - part.y) : 0;
      const bool seg_end = __shfl_down(seg, 1, kWave) != seg || lane == kWave - 1;
      // a long part is flagged (kDescLong): k_longcopy moves it, the window
      // copy sees a gap at its place (parts are < 2^24 entries, kSMax)
      const bool lng = valid && part.y >= long_min;
      wave_lds_sync();
      if (valid) {
        if (!kCopy)
          put_checked(desc, pb + k, desc_cap,
                      make_uint4(part.x, part.y | (lng ? kDescLong : 0u), (uint32_t)at, (uint32_t)(at >> 32)),
                      &o.ctr->oob);
        if (seg_end) L.run[j] += si;
      }
      if (kCopy) {
        uint64_t vm = __ballot(valid && part.y > 0);
        while (vm) {  // (wave-uniform)
          uint32_t src[4], len[4];
          uint64_t dst[4];
          uint32_t mx = 0;
#pragma unroll
          for (int i = 0; i < 4; i++) {
            len[i] = 0, src[i] = 0, dst[i] = 0;
            if (vm) {
              const int l = __builtin_ctzll(vm);
              vm &= vm - 1;
              src[i] = __shfl(part.x, l, 64);
              len[i] = __shfl(part.y, l, 64);
              dst[i] = shfl64(at, l);
              mx = max(mx, len[i]);
            }
          }
          for (uint32_t r0 = 0; r0 < mx; r0 += kWave) {
            const uint32_t jj = r0 + lane;
            uint32_t v[4];
#pragma unroll
            for (int i = 0; i < 4; i++) v[i] = jj < len[i] ? s.words[src[i] + jj] : 0u;
#pragma unroll
            for (int i = 0; i < 4; i++)
              if (jj < len[i]) put_checked(o.dout, dst[i] + jj, o.dcap, v[i], &o.ctr->oob);
          }
        }
      }
      wave_lds_sync();
    }
  }
}

// window w of the output space [w * kWin, (w + 1) * kWin) -> the descriptor
// holding (or, in a gap, preceding) its first position; windows before the
// first descriptor map to it
constexpr uint32_t kWin = 4096;
// (counts read on the device: nd = solo descriptors, clamped to their buffer;
// total = solo output positions; windows past win_cap flag the call)
__global__ __launch_bounds__(256) void k_winmap(const uint4 *__restrict__ desc, const uint64_t *__restrict__ nd_ptr,
                                                uint64_t desc_cap, const uint64_t *__restrict__ total_ptr,
                                                uint32_t *__restrict__ win, uint64_t win_cap, unsigned int *oob) {
  const uint64_t nd = min(*nd_ptr, desc_cap), total = *total_ptr;
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nd; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 a = desc[j];
    const uint64_t d = a.z | ((uint64_t)a.w << 32);
    uint64_t e = total;
    if (j + 1 < nd) {
      const uint4 b = desc[j + 1];
      e = b.z | ((uint64_t)b.w << 32);
    }
    const uint64_t lo = j == 0 ? 0 : (d + kWin - 1) / kWin, hi = (e + kWin - 1) / kWin;
    if (hi > win_cap) atomicOr(oob, 1u);
    for (uint64_t w = lo; w < hi && w < win_cap; w++) win[w] = (uint32_t)j;
  }
}

// ---- k_wincopy: the solo deliveries, a wavefront per output window ----------
// Loads 64 descriptors from the window's first one (one coalesced 16-B load
// per lane), clips them to the window in LDS, then moves kCU entries per lane
// and step: position q -> its descriptor by a 6-step search over the clipped
// starts -> words[src + q - start] -> dout[q] (the word IS the packed
// delivery: a 4-B copy, lane-consecutive loads and stores).  More than 64
// descriptors in a window (many tiny topics): the next 64, from where the
// previous batch ended.
constexpr int kCU = 16;  // entries per lane per step
// position -> descriptor through a per-64-position block index (the last
// descriptor starting at or before each block, one search per block and
// descriptor batch), then a search inside the block's few descriptors —
// usually none or one step instead of six per entry
struct alignas(16) WinLds {
  uint32_t st[kWave], en[kWave], src[kWave];
  uint32_t blk[kWin / kWave];
};

// kVec (MQM_WINCOPY_VEC=1, A/B): each lane moves 4 consecutive positions at
// a time — one 16-B load and one 16-B store when one descriptor covers all
// four (a quarter of the memory instructions), position by position at part
// boundaries
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// kNT (default; MQM_NT_STORE=0 off): the scalar path's stores non-temporal, so the
// result stream does not evict the hub ranges the copy re-reads from L2
template <bool kVec = false, bool kNT = false>
__global__ __launch_bounds__(kWave *kEmitWaves) __attribute__((amdgpu_waves_per_eu(8))) void k_wincopy(
    DeviceSnapshot s, const uint4 *__restrict__ desc, const uint64_t *__restrict__ nd_ptr, uint64_t desc_cap,
    const uint32_t *__restrict__ win, uint64_t win_cap, const uint64_t *__restrict__ total_ptr,
    uint32_t *__restrict__ out, uint64_t cap, unsigned int *oob) {
  __shared__ WinLds lds_all[kEmitWaves];
  const uint64_t nd = min(*nd_ptr, desc_cap), total = *total_ptr;
  const uint64_t nwin = min((total + kWin - 1) / kWin, win_cap);
  const int lane = threadIdx.x & (kWave - 1);
  WinLds &L = lds_all[threadIdx.x / kWave];
  // words through a buffer descriptor: 32-bit offsets, bounds-checked reads
  const __amdgpu_buffer_rsrc_t words =
      __builtin_amdgcn_make_buffer_rsrc((void *)s.words, (short)0, (int)(s.n_subs * 4u + 64u), 0x00020000);
  const uint64_t nw = (uint64_t)gridDim.x * kEmitWaves;
  for (uint64_t w = (uint64_t)blockIdx.x * kEmitWaves + threadIdx.x / kWave; w < nwin; w += nw) {
    const uint64_t g0 = w * kWin, g1 = min(g0 + kWin, total);
    uint64_t j = win[w];
    uint64_t pos = g0;
    while (pos < g1 && j < nd) {
      const uint64_t jj = j + lane;
      uint4 d = make_uint4(0, 0, 0xFFFFFFFFu, 0xFFFFFFFFu);
      if (jj < nd) d = desc[jj];
      const uint64_t dst = d.z | ((uint64_t)d.w << 32);
      const uint64_t dend = jj < nd ? dst + ((d.y & kDescLong) ? 0u : d.y) : ~0ull;  // (a long part: a gap)
      uint64_t a = dst > pos ? dst : pos, b = dend < g1 ? dend : g1;
      if (b < a) b = a;
      if (a > g1) a = b = g1;
      // positions handled by this batch: up to the end of its last descriptor
      const uint64_t last_end = shfl64(dend, kWave - 1);
      const uint64_t bend = j + kWave < nd ? (last_end < g1 ? (last_end > pos ? last_end : pos) : g1) : g1;
      L.st[lane] = (uint32_t)(a - g0);
      L.en[lane] = (uint32_t)(b - g0);
      L.src[lane] = d.x + (uint32_t)(a - dst);
      wave_lds_sync();
      {  // block lane (positions lane * 64 ..): the last descriptor starting at or before its start
        static_assert(kWin / kWave == kWave, "one block per lane");
        const uint32_t q = (uint32_t)lane * kWave;
        uint32_t k = 0;
#pragma unroll
        for (uint32_t step = 32; step > 0; step >>= 1) k = L.st[k + step] <= q ? k + step : k;
        L.blk[lane] = k;
      }
      wave_lds_sync();
      const uint32_t q0 = (uint32_t)(pos - g0), q1 = (uint32_t)(bend - g0);
      auto desc_of = [&](uint32_t q) {  // the last descriptor starting at or before q (q < kWin)
        const uint32_t bq = q / kWave;
        uint32_t k = L.blk[bq], left = (bq + 1 < kWin / kWave ? L.blk[bq + 1] : kWave - 1) - k;
        while (left > 0) {
          const uint32_t half = (left + 1) / 2;
          if (L.st[k + half] <= q) {
            k += half;
            left -= half;
          } else {
            left = half - 1;
          }
        }
        return k;
      };
      if (kVec) {
        constexpr int kU = 4;  // units of 4 positions per lane per step
        for (uint32_t base = q0 & ~3u; base < q1; base += kWave * 4 * kU) {
          uint32_t qa[kU], sa[kU];
          bool full[kU];
#pragma unroll
          for (int u = 0; u < kU; u++) {
            const uint32_t q = base + (u * kWave + lane) * 4;
            const uint32_t k = desc_of(min(q, (uint32_t)kWin - 1));
            full[u] = q >= q0 && q + 4 <= q1 && q >= L.st[k] && q + 4 <= L.en[k];
            qa[u] = q;
            sa[u] = full[u] ? L.src[k] + (q - L.st[k]) : 0u;
          }
          u32x4 vv[kU];
#pragma unroll
          for (int u = 0; u < kU; u++) vv[u] = __builtin_amdgcn_raw_buffer_load_b128(words, (int)(sa[u] * 4u), 0, 0);
#pragma unroll
          for (int u = 0; u < kU; u++) {
            const uint32_t q = qa[u];
            if (full[u]) {
              const uint64_t p = g0 + q;
              if (p + 4 <= cap)
                *reinterpret_cast<uint4 *>(out + p) = make_uint4(vv[u].x, vv[u].y, vv[u].z, vv[u].w);
              else
                atomicOr(oob, kOobStore);
              continue;
            }
            for (uint32_t r = 0; r < 4; r++) {  // a part boundary or the batch's ends inside the unit
              const uint32_t qr = q + r;
              if (qr < q0 || qr >= q1) continue;
              const uint32_t k = desc_of(qr);
              if (qr < L.st[k] || qr >= L.en[k]) continue;
              const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(words, (int)((L.src[k] + (qr - L.st[k])) * 4u), 0, 0);
              const uint64_t p = g0 + qr;
              if (p < cap)
                out[p] = v;
              else
                atomicOr(oob, kOobStore);
            }
          }
        }
      }
      for (uint32_t base = q0; !kVec && base < q1; base += kWave * kCU) {
        uint32_t sa[kCU];
        bool in[kCU];
#pragma unroll
        for (int u = 0; u < kCU; u++) {
          const uint32_t q = base + u * kWave + lane;
          // the last descriptor starting at or before q: within [blk[b], blk[b + 1]]
          const uint32_t bq = min(q, (uint32_t)kWin - 1) / kWave;
          uint32_t k = L.blk[bq], left = (bq + 1 < kWin / kWave ? L.blk[bq + 1] : kWave - 1) - k;
          while (left > 0) {
            const uint32_t half = (left + 1) / 2;
            if (L.st[k + half] <= q) {
              k += half;
              left -= half;
            } else {
              left = half - 1;
            }
          }
          in[u] = q < q1 && q >= L.st[k] && q < L.en[k];
          sa[u] = in[u] ? L.src[k] + (q - L.st[k]) : 0u;
        }
        uint32_t v[kCU];
#pragma unroll
        for (int u = 0; u < kCU; u++) v[u] = __builtin_amdgcn_raw_buffer_load_b32(words, (int)(sa[u] * 4u), 0, 0);
#pragma unroll
        for (int u = 0; u < kCU; u++) {
          if (!in[u]) continue;
          const uint64_t p = g0 + base + u * kWave + lane;
          if (p < cap) {
            if (kNT)
              __builtin_nontemporal_store(v[u], out + p);
            else
              out[p] = v[u];
          } else {
            atomicOr(oob, kOobStore);
          }
        }
      }
      wave_lds_sync();
      pos = bend;
      j += kWave;
    }
  }
}

// ---- k_longcopy: the long solo parts, a wavefront per part ------------------
// A solo part is a run of `words` copied as it stands (its entries are their
// clients' deliveries).  The window copy above pays a descriptor search and a
// 4-B load and store per entry; a part of >= long_min entries (C3: 0.16 parts
// of >= 256 entries per topic hold 61 % of the solo entries, tools/walk_census)
// is instead moved by one wavefront with 16-B stores aligned on the output
// (the 4-word units inside the part) and 16-B loads at the matching source
// offset (dword-aligned: `words` and `dout` shift by different amounts), its
// first and last partial units word by word.  4 units per lane in flight.
__global__ __launch_bounds__(kWave *kEmitWaves) void k_longcopy(DeviceSnapshot s, const uint4 *__restrict__ desc,
                                                              const uint64_t *__restrict__ nd_ptr, uint64_t desc_cap,
                                                              uint32_t *__restrict__ out, uint64_t cap,
                                                              unsigned int *oob) {
  const uint64_t nd = min(*nd_ptr, desc_cap);
  const int lane = threadIdx.x & (kWave - 1);
  const __amdgpu_buffer_rsrc_t words =
      __builtin_amdgcn_make_buffer_rsrc((void *)s.words, (short)0, (int)(s.n_subs * 4u + 64u), 0x00020000);
  const uint64_t nw = (uint64_t)gridDim.x * kEmitWaves;
  constexpr int kU = 4;
  // 64 descriptors per wave step (one coalesced load), then the flagged ones,
  // each by the whole wavefront
  for (uint64_t j0 = ((uint64_t)blockIdx.x * kEmitWaves + threadIdx.x / kWave) * kWave; j0 < nd; j0 += nw * kWave) {
    uint4 mine = make_uint4(0, 0, 0, 0);
    if (j0 + lane < nd) mine = desc[j0 + lane];
    uint64_t lm = __ballot((mine.y & kDescLong) != 0);
   while (lm) {
    const int src_lane = __builtin_ctzll(lm);
    lm &= lm - 1;
    const uint4 d = make_uint4(__shfl(mine.x, src_lane, 64), __shfl(mine.y, src_lane, 64) & ~kDescLong,
                               __shfl(mine.z, src_lane, 64), __shfl(mine.w, src_lane, 64));
    const uint64_t dst = d.z | ((uint64_t)d.w << 32), e = dst + d.y, a = dst & ~3ull;
    const uint64_t units = (e - a + 3) >> 2;
    const uint32_t src = d.x;
    for (uint64_t u0 = 0; u0 < units; u0 += (uint64_t)kWave * kU) {
      uint4 v[kU];
      bool full[kU];
#pragma unroll
      for (int k = 0; k < kU; k++) {
        const uint64_t unit = u0 + (uint64_t)k * kWave + lane, w0 = a + 4 * unit;
        full[k] = unit < units && w0 >= dst && w0 + 4 <= e;
        if (full[k]) {
          const auto x = __builtin_amdgcn_raw_buffer_load_b128(words, (int)(4u * (src + (uint32_t)(w0 - dst))), 0, 0);
          v[k] = make_uint4(x[0], x[1], x[2], x[3]);
        }
      }
#pragma unroll
      for (int k = 0; k < kU; k++) {
        const uint64_t unit = u0 + (uint64_t)k * kWave + lane, w0 = a + 4 * unit;
        if (unit >= units) continue;
        if (full[k]) {
          if (w0 + 4 <= cap)
            *reinterpret_cast<uint4 *>(out + w0) = v[k];
          else
            atomicOr(oob, kOobStore);
        } else {  // the part's first or last unit: the words inside it
#pragma unroll
          for (int z = 0; z < 4; z++) {
            const uint64_t p = w0 + z;
            if (p < dst || p >= e) continue;
            const uint32_t x = __builtin_amdgcn_raw_buffer_load_b32(words, (int)(4u * (src + (uint32_t)(p - dst))), 0, 0);
            put_checked(out, p, cap, x, oob);
          }
        }
      }
    }
   }
  }
}

// ---- k_shared: shared candidates (gatherSharedSubscriptions, topics.go:541-555)
// a 16-lane group per topic with H > 0: its shared hits are id ranges
constexpr int kHL = 16;
__global__ __launch_bounds__(256) void k_shared(Outputs o, const uint32_t *__restrict__ list,
                                                const unsigned int *__restrict__ count) {
  const int lane = threadIdx.x & (kWave - 1), g = lane / kHL, gl = lane % kHL;
  const uint32_t nl = *count, stride = gridDim.x * (blockDim.x / kHL);
  for (uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) / kHL; i < nl; i += stride) {
    (void)g;
    const uint32_t t = list[i];
    const uint32_t *grec = o.recs + (uint64_t)t * kRecStrideAlloc;
    const uint32_t nsh = (rec_tail(o.recs, t)[0].x >> 8) & 0xFFu;
    const uint64_t hb = o.hstart[t];
    uint32_t w = 0;
    for (uint32_t j = 0; j < nsh; j++) {
      const uint32_t so = grec[kRecSh + 2 * j], c = grec[kRecSh + 1 + 2 * j];
      for (uint32_t j2 = gl; j2 < c; j2 += kHL) put_checked(o.hout, hb + w + j2, o.hcap, so + j2, &o.ctr->oob, kOobShared);
      w += c;
    }
  }
}

__global__ __launch_bounds__(256) void k_nflags(const NodeDesc *__restrict__ nodes, uint8_t *__restrict__ f,
                                                uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    f[i] = (uint8_t)(nodes[i].sh_cnt_flags >> 24);
}

// word w of DeviceSnapshot::ident_bits: entries 32w .. 32w + 31
__global__ __launch_bounds__(256) void k_ident_bits(const SubEnt *__restrict__ subs, uint32_t *__restrict__ bits,
                                                    uint64_t n) {
  const uint64_t nw = (n + 31) / 32;
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t b = 0;
    for (uint32_t k = 0; k < 32 && w * 32 + k < n; k++) b |= ((subs[w * 32 + k].word & kWordIdent) ? 1u : 0u) << k;
    bits[w] = b;
  }
}

// slot i = {node i, its '+' child (zeros without one)} (snapshot.h DeviceSnapshot::slots)
__global__ __launch_bounds__(256) void k_slots(const NodeDesc *__restrict__ nodes, NodeDesc *__restrict__ slots,
                                               uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const NodeDesc d = load_desc(nodes + i);
    NodeDesc p{kNone, kNone, 0, 0, 0, 0, 0, 0};
    if (d.plus != kNone && d.plus < n) p = load_desc(nodes + d.plus);
    slots[2 * i] = d;
    slots[2 * i + 1] = p;
  }
}

__global__ __launch_bounds__(256) void k_words(const SubEnt *__restrict__ subs, uint32_t *__restrict__ words,
                                               uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    words[i] = subs[i].word & kPackedMask;
}

// Merge kMPer multi entries per lane of a kE-lane group in a table of
// (1 << lg) <= kSlots slots and write the winners at out[db + D ..); returns
// the new D (group-uniform).  Entries past M are inert.
template <int kE, int kMPer>
__device__ __forceinline__ uint32_t merge_multi(MergeTable tb, uint32_t kSlots, const uint32_t (&mcl)[kMPer],
                                                const uint32_t (&mw)[kMPer], const uint32_t (&mrk)[kMPer],
                                                uint32_t M, int gl, int gbase, uint32_t *out, uint64_t db,
                                                uint32_t D, uint64_t cap, unsigned int *oob) {
  constexpr uint64_t kGMask = kE == 64 ? ~0ull : (1ull << kE) - 1ull;
  const uint64_t glt = (1ull << gl) - 1ull;
  uint32_t lg = 5;
  while ((1u << lg) < 2 * M && (1u << lg) < kSlots) lg++;
  const uint32_t mask = (1u << lg) - 1;
  for (uint32_t j = gl; j <= mask; j += kE) mt_clear(tb, j);
  wave_lds_sync();
#pragma unroll
  for (int k = 0; k < kMPer; k++)
    if (gl + k * kE < M) mt_insert(tb, mask, lg, mcl[k], mw[k], mrk[k]);
  wave_lds_sync();
  for (uint32_t j0 = 0; j0 <= mask; j0 += kE) {  // one delivery per occupied slot, slot order
    const uint32_t j = j0 + gl;
    const bool occ = j <= mask && mt_occupied(tb, j);
    const uint64_t m = (__ballot(occ) >> gbase) & kGMask;
    if (occ) put_checked(out, db + D + __popcll(m & glt), cap, mt_delivery(tb, j), oob);
    D += __popcll(m);
  }
  return D;
}

// ---- k_merge_small ------------------------------------------------------------
// kSmallLanes lanes per topic (8 topics per wavefront) for topics with 0 < Ms
// <= kSmallMultiS and <= kSmallHits hits: the whole record (header + hits =
// 64 words) is prefetched one topic ahead and its list entry two ahead, so a
// topic costs one dependent round trip (its multi entries) after its record
// arrives.
constexpr int kSE = kSmallLanes;
constexpr int kSGroups = kWave / kSE;
constexpr int kSRecPer = 64 / kSE;  // record words prefetched per lane
static_assert(4 + kRecHit * kSmallHits <= 64 && kSRecPer % 4 == 0, "small-class record prefetch");

constexpr int kSmallTab = 32;  // k_merge_small table slots (<= kSmallMultiS entries: load <= 0.75)
static_assert(kSmallMultiS * 4 <= kSmallTab * 3, "k_merge_small table load factor");
struct alignas(8) SmallLds {
  unsigned long long tfirst[kSmallTab], tkb[kSmallTab];
  uint32_t rec[64];
  uint32_t pad[2];  // 194-dword stride: the 8 groups' contexts start 2 banks apart
};
static_assert(sizeof(SmallLds) % 256 == 8, "bank-skewed group contexts");

// kIdent: the merges list Identifiers (Outputs::iscratch); a variant of its
// own, so the plain merges keep their registers (k_merge 72 VGPRs, 7 waves /
// SIMD; with the listing compiled in: 82, 5 — r06f, 1.08 -> 1.26 ms on C3)
template <int kOcc, bool kIdent = false>
__global__ __launch_bounds__(kWave *kEmitWaves) __attribute__((amdgpu_waves_per_eu(kOcc))) void k_merge_small(
    DeviceSnapshot s, Outputs o, const uint32_t *__restrict__ list, const unsigned int *__restrict__ count) {
  constexpr int kMPer = kSmallMultiS / kSE, kRecPer = kSRecPer;
  __shared__ SmallLds lds_all[kEmitWaves * kSGroups];
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / kSE, gl = lane % kSE, gbase = g * kSE;
  SmallLds &L = lds_all[(threadIdx.x / kWave) * kSGroups + g];
  const uint32_t ngroups = gridDim.x * kEmitWaves * kSGroups;
  const uint32_t nl = *count;
  uint32_t i = (blockIdx.x * kEmitWaves + threadIdx.x / kWave) * kSGroups + g;
  uint32_t n_rw[kRecPer];
  uint64_t n_db = 0;
  auto fetch = [&](uint32_t u) {
    n_db = o.dstart[u];
    const uint4 *r = rec_tail(o.recs, u);  // units gl * kRecPer / 4 ..: header, multi parts
#pragma unroll
    for (int v = 0; v < kRecPer / 4; v++) {
      const uint4 x = r[-(gl * (kRecPer / 4) + v)];
      n_rw[4 * v] = x.x, n_rw[4 * v + 1] = x.y, n_rw[4 * v + 2] = x.z, n_rw[4 * v + 3] = x.w;
    }
  };
  uint32_t t_nxt = i < nl ? list[i] : 0;
  uint32_t t_nn = i + ngroups < nl ? list[i + ngroups] : 0;
  if (i < nl) fetch(t_nxt);
  for (; i < nl; i += ngroups) {
    const uint32_t t = t_nxt;
    const uint64_t db = n_db;
#pragma unroll
    for (int j = 0; j < kRecPer; j++) L.rec[gl * kRecPer + j] = n_rw[j];
    t_nxt = t_nn;
    if (i + ngroups < nl) fetch(t_nxt);
    t_nn = i + 2 * ngroups < nl ? list[i + 2 * ngroups] : 0;
    wave_lds_sync();
    const uint32_t nh = L.rec[0] & 0xFFu, Ss = L.rec[1], M = L.rec[2];
    const uint64_t ib = kIdent ? ident_base(o, t, M, gl == 0) : ~0ull;
    rec_prefix<kSE, kSmallHits>(L.rec, nh, gl);
    wave_lds_sync();
    uint32_t mcl[kMPer], mw[kMPer], mrk[kMPer];
#pragma unroll
    for (int k = 0; k < kMPer; k++) {
      const uint32_t q = gl + k * kSE;
      uint32_t h;
      const uint32_t sid = multi_sid(L.rec, nh, q < M ? q : 0, &h);
      mrk[k] = rec_at(L.rec, h, kFieldRank);
      const SubEnt e = load_sub(s, sid);
      mcl[k] = e.client;
      mw[k] = e.word;
    }
    uint32_t im = 0;  // (kIdent) bit k: entry k's Identifier is > 0 — one register across the merge
    if constexpr (kIdent) {
#pragma unroll
      for (int k = 0; k < kMPer; k++) im |= (mw[k] & kWordIdent) ? 1u << k : 0u;
    }
    const uint32_t D = merge_multi<kSE, kMPer>(MergeTable{L.tkb, L.tfirst}, kSmallTab, mcl, mw, mrk, M, gl,
                                               gbase, o.dout, db, Ss, o.dcap, &o.ctr->oob);
    if (gl == 0) o.dcount[t] = D;
    if constexpr (kIdent) {  // (wave-uniform: every group runs the ballots; sids again from the record in LDS)
      uint32_t nid = 0;
      const uint64_t glt = (1ull << gl) - 1ull;
#pragma unroll
      for (int k = 0; k < kMPer; k++) {
        const uint32_t q = gl + k * kSE;
        uint32_t h;
        const uint32_t sid = multi_sid(L.rec, nh, q < M ? q : 0, &h);
        ident_put<kSE>(o, ib, ib != ~0ull && q < M && ((im >> k) & 1u), sid, gbase, glt, nid);
      }
      if (gl == 0 && ib != ~0ull) o.icount[t] = nid;
    }
    wave_lds_sync();
  }
}

// ---- k_merge: a wavefront per topic with kSmallMultiS < Ms <= kSmallMulti (or
// more than kSmallHits hits) ----------------------------------------------------
struct alignas(16) MergeLds {
  unsigned long long tfirst[kSmallSlots], tkb[kSmallSlots];
  uint32_t rec[kRecLds];
};

template <bool kIdent = false>
__global__ __launch_bounds__(kWave *kEmitWaves) void k_merge(DeviceSnapshot s, Outputs o,
                                                            const uint32_t *__restrict__ list,
                                                            const unsigned int *__restrict__ count) {
  constexpr int kMPer = kSmallMulti / kWave;
  __shared__ MergeLds lds_all[kEmitWaves];
  const int lane = threadIdx.x & (kWave - 1);
  MergeLds &L = lds_all[threadIdx.x / kWave];
  const uint32_t nw = gridDim.x * kEmitWaves, nl = *count;
  uint32_t i = blockIdx.x * kEmitWaves + threadIdx.x / kWave;
  uint32_t n_t = 0;
  uint4 n_rw = make_uint4(0, 0, 0, 0);
  uint64_t n_db = 0;
  auto fetch = [&](uint32_t k) {
    n_t = list[k];
    n_db = o.dstart[n_t];
    if (lane < 16) n_rw = rec_tail(o.recs, n_t)[-lane];  // header + the first 15 multi parts
  };
  if (i < nl) fetch(i);
  for (; i < nl; i += nw) {
    const uint32_t t = n_t;
    const uint64_t db = n_db;
    uint4 *rec4 = reinterpret_cast<uint4 *>(L.rec);
    if (lane < 16) rec4[lane] = n_rw;
    if (i + nw < nl) fetch(i + nw);
    wave_lds_sync();
    const uint32_t nh = L.rec[0] & 0xFFu, Ss = L.rec[1], M = L.rec[2];
    const uint64_t ib = kIdent ? ident_base(o, t, M, lane == 0) : ~0ull;
    const uint4 *gt = rec_tail(o.recs, t);
    for (uint32_t u = 16 + lane; u < 1 + nh; u += kWave) rec4[u] = gt[-(int)u];
    wave_lds_sync();
    rec_prefix<kWave>(L.rec, nh, lane);
    wave_lds_sync();
    uint32_t mcl[kMPer], mw[kMPer], mrk[kMPer];
#pragma unroll
    for (int k = 0; k < kMPer; k++) {
      const uint32_t q = lane + k * kWave;
      uint32_t h;
      const uint32_t sid = multi_sid(L.rec, nh, q < M ? q : 0, &h);
      mrk[k] = rec_at(L.rec, h, kFieldRank);
      const SubEnt e = load_sub(s, sid);
      mcl[k] = e.client;
      mw[k] = e.word;
    }
    uint32_t im = 0;  // (kIdent) bit k: entry k's Identifier is > 0
    if constexpr (kIdent) {
#pragma unroll
      for (int k = 0; k < kMPer; k++) im |= (mw[k] & kWordIdent) ? 1u << k : 0u;
    }
    const uint32_t D =
        merge_multi<kWave, kMPer>(MergeTable{L.tkb, L.tfirst}, kSmallSlots, mcl, mw, mrk, M, lane, 0,
                                  o.dout, db, Ss, o.dcap, &o.ctr->oob);
    if (lane == 0) o.dcount[t] = D;
    if constexpr (kIdent) {
      if (ib != ~0ull) {  // (wave-uniform)
        uint32_t nid = 0;
#pragma unroll
        for (int k = 0; k < kMPer; k++) {
          const uint32_t q = lane + k * kWave;
          uint32_t h;
          const uint32_t sid = multi_sid(L.rec, nh, q < M ? q : 0, &h);
          ident_put<kWave>(o, ib, q < M && ((im >> k) & 1u), sid, 0, lanemask_lt(lane), nid);
        }
        if (lane == 0) o.icount[t] = nid;
      }
    }
    wave_lds_sync();
  }
}

// ---------------------------------------------------------------------------
// Workgroup merges (256 threads per topic) for big-class topics with more
// multi entries than k_merge's wave table holds, routed by size (k_route):
//   k_multi<kSlots>  M <= kSlots * 3 / 4 in one LDS table;
//   k_multi_part     any M: the topic's clients split into P = ceil(M /
//                    kPartCap) hash partitions merged one after another in a
//                    4096-slot table (each pass reads all M entries and keeps
//                    its partition's; a client's entries share a partition).
// Winners are written after the topic's solo deliveries (k_wincopy writes those)
// in table-slot order: each wave scans a quarter of the table twice (count,
// then write at its prefix), so the layout is deterministic.
// ---------------------------------------------------------------------------
// k_multi's table: >= 2 slots per entry

struct alignas(16) MultiLds {
  uint32_t rec[kRecLds];
  uint32_t wsum[kBigThreads / kWave];
};

// the block's record of topic t, with prefixes (all threads; ends synced)
// The next topic of a workgroup's list is fetched while the current one is
// merged (its list entry, segment start and record tail in registers: one
// 16-B unit per thread), so a topic's record never costs a round trip of
// its own.
static_assert(kRecLds / 4 <= kBigThreads, "one record unit per thread");
struct NextTopic {
  uint32_t t = 0;
  uint64_t db = 0;
  uint4 unit = make_uint4(0, 0, 0, 0);
  __device__ __forceinline__ void fetch(Outputs o, const uint32_t *list, uint32_t bi, uint32_t nb) {
    if (bi >= nb) return;
    t = list[bi];
    db = o.dstart[t];
    if (threadIdx.x < (uint32_t)kRecLds / 4) unit = rec_tail(o.recs, t)[-(int)threadIdx.x];
  }
};

__device__ __forceinline__ void block_record(const NextTopic &nx, uint32_t *rec) {
  const int tid = threadIdx.x;
  if (tid < kRecLds / 4) reinterpret_cast<uint4 *>(rec)[tid] = nx.unit;
  __syncthreads();
  const uint32_t nh = rec[0] & 0xFFu;
  __syncthreads();
  if (tid < kWave) rec_prefix<kWave>(rec, nh, tid);
  __syncthreads();
}

// winners of the table [0, nslots) at out[db + D ..); returns the new D
__device__ __forceinline__ uint32_t block_winners(MergeTable tb, uint32_t nslots, uint32_t *wsum, Outputs o, uint64_t db,
                                                  uint32_t D) {
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  constexpr int kW = kBigThreads / kWave;
  const uint32_t per = (nslots + kW - 1) / kW, lo = wid * per, hi = min(nslots, lo + per);
  uint32_t c = 0;
  for (uint32_t j0 = lo; j0 < hi; j0 += kWave) {
    const uint32_t j = j0 + lane;
    c += __popcll(__ballot(j < hi && mt_occupied(tb, j)));
  }
  if (lane == 0) wsum[wid] = c;
  __syncthreads();
  uint32_t w = D, total = D;
  for (int k = 0; k < kW; k++) {
    if (k < wid) w += wsum[k];
    total += wsum[k];
  }
  for (uint32_t j0 = lo; j0 < hi; j0 += kWave) {
    const uint32_t j = j0 + lane;
    const bool occ = j < hi && mt_occupied(tb, j);
    const uint64_t m = __ballot(occ);
    if (occ) put_checked(o.dout, db + w + __popcll(m & lanemask_lt(lane)), o.dcap, mt_delivery(tb, j), &o.ctr->oob);
    w += __popcll(m);
  }
  __syncthreads();
  return total;
}

// the workgroup merges' Identifiers listing (Outputs::iscratch): a pass over
// the topic's multi entries after its merge, 256 at a time, placed in entry
// order by a block prefix of the waves' ballots (wsum: the winners' scratch)
__device__ __forceinline__ void block_ident(const DeviceSnapshot &s, Outputs o, uint32_t t, uint32_t nh, uint32_t M,
                                            const uint32_t *rec, uint32_t *wsum) {
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  constexpr int kW = kBigThreads / kWave;
  const uint64_t ib = ident_base(o, t, M, tid == 0);
  if (ib == ~0ull) return;  // (block-uniform)
  uint32_t nid = 0;
  for (uint32_t q0 = 0; q0 < M; q0 += kBigThreads) {
    const uint32_t q = q0 + tid;
    uint32_t h, sid = 0;
    bool has = false;
    if (q < M) {
      sid = multi_sid(rec, nh, q, &h);
      has = (s.ident_bits[sid >> 5] >> (sid & 31)) & 1u;
    }
    const uint64_t m = __ballot(has);
    if (lane == 0) wsum[wid] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t w = nid, tot = 0;
    for (int k = 0; k < kW; k++) {
      if (k < wid) w += wsum[k];
      tot += wsum[k];
    }
    if (has) o.iscratch[ib + w + __popcll(m & lanemask_lt(lane))] = sid;
    nid += tot;
    __syncthreads();
  }
  if (tid == 0) o.icount[t] = nid;
}

template <int kSlots>
__global__ __launch_bounds__(kBigThreads) void k_multi(DeviceSnapshot s, Outputs o, const uint32_t *__restrict__ list,
                                                      const unsigned int *__restrict__ count) {
  __shared__ unsigned long long tfirst[kSlots], tkb[kSlots];
  __shared__ MultiLds L;
  const MergeTable tb{tkb, tfirst};
  const int tid = threadIdx.x;
  const uint32_t nb = *count;
  NextTopic nx;
  nx.fetch(o, list, blockIdx.x, nb);
  for (uint32_t bi = blockIdx.x; bi < nb; bi += gridDim.x) {
    const uint32_t t = nx.t;
    const uint64_t db = nx.db;
    block_record(nx, L.rec);
    nx.fetch(o, list, bi + gridDim.x, nb);
    const uint32_t nh = L.rec[0] & 0xFFu, Ss = L.rec[1], M = L.rec[2];
    uint32_t lg = 6;
    const uint32_t need = 2 * M;
    while ((1u << lg) < need && (1u << lg) < (uint32_t)kSlots) lg++;
    const uint32_t mask = (1u << lg) - 1;
    for (uint32_t i = tid; i <= mask; i += kBigThreads) mt_clear(tb, i);
    __syncthreads();
    for (uint32_t q = tid; q < M; q += kBigThreads) {  // (a hit-by-hit loop measured slower: idle lanes on small hits)
      uint32_t h;
      const uint32_t sid = multi_sid(L.rec, nh, q, &h);
      const SubEnt e = load_sub(s, sid);
      mt_insert(tb, mask, lg, e.client, e.word, rec_at(L.rec, h, kFieldRank));
    }
    __syncthreads();
    const uint32_t D = block_winners(tb, mask + 1, L.wsum, o, db, Ss);
    if (tid == 0) o.dcount[t] = D;
    if (o.iscratch) block_ident(s, o, t, nh, M, L.rec, L.wsum);
  }
}

// client -> partition: a hash independent of table_slot's (which takes the
// top bits of client * 2654435769: a partition must spread over the table)
__device__ __forceinline__ uint32_t partition_of(uint32_t client, uint32_t P) {
  uint32_t h = client * 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return (uint32_t)(((uint64_t)h * P) >> 32);
}

__global__ __launch_bounds__(kBigThreads) void k_multi_part(DeviceSnapshot s, Outputs o,
                                                           const uint32_t *__restrict__ list,
                                                           const unsigned int *__restrict__ count) {
  constexpr uint32_t kSlots = 4096, kFill = kSlots * 7 / 8;
  __shared__ unsigned long long tfirst[kSlots], tkb[kSlots];
  __shared__ MultiLds L;
  __shared__ uint32_t fill;
  const MergeTable tb{tkb, tfirst};
  const int tid = threadIdx.x;
  const uint32_t nb = *count;
  NextTopic nx;
  nx.fetch(o, list, blockIdx.x, nb);
  for (uint32_t bi = blockIdx.x; bi < nb; bi += gridDim.x) {
    const uint32_t t = nx.t;
    const uint64_t db = nx.db;
    block_record(nx, L.rec);
    nx.fetch(o, list, bi + gridDim.x, nb);
    const uint32_t nh = L.rec[0] & 0xFFu, Ss = L.rec[1], M = L.rec[2];
    const uint32_t P = (M + kPartCap - 1) / kPartCap;
    uint32_t D = Ss;
    for (uint32_t p = 0; p < P; p++) {
      for (uint32_t i = tid; i < kSlots; i += kBigThreads) mt_clear(tb, i);
      if (tid == 0) fill = 0;
      __syncthreads();
      for (uint32_t q = tid; q < M; q += kBigThreads) {
        uint32_t h;
        const uint32_t sid = multi_sid(L.rec, nh, q, &h);
        const SubEnt e = load_sub(s, sid);
        if (partition_of(e.client, P) != p) continue;
        if (atomicAdd(&fill, 1u) >= kFill) {  // never for a hash of this spread: fail, do not spin
          atomicOr(&o.ctr->oob, kOobPart);
          continue;
        }
        mt_insert(tb, kSlots - 1, 12, e.client, e.word, rec_at(L.rec, h, kFieldRank));
      }
      __syncthreads();
      D = block_winners(tb, kSlots, L.wsum, o, db, D);
    }
    if (tid == 0) o.dcount[t] = D;
    if (o.iscratch) block_ident(s, o, t, nh, M, L.rec, L.wsum);
  }
}



// ---------------------------------------------------------------------------
// k_resolve<kE, kH>: the merge by resolution (snapshot.h: pinfo) for topics
// whose multi entries are all light (no kClsHeavy): kE lanes per topic (8 for
// topics with <= kSmallMultiS entries and <= kSmallHits multi parts, 64
// otherwise), no table, no atomics.  The topic's multi parts (the walk's
// record: multi-tail start, count, hit rank) go into a small LDS hash by
// multi-tail start; every multi entry reads its packed word and its partners
// (each encoded as the multi-tail start of its node's range, which is where a
// gathered partner's part starts, with its QoS / NoLocal bits) and is its
// client's delivery iff no gathered partner has a lower hit rank (the
// reference's emission order; partners sit on other nodes) — the winner folds
// the gathered partners' QoS / NoLocal in: Subscription.Merge
// (packets.go:250-270) without a table.  Winners are written after the
// topic's solo deliveries in entry order (deterministic).
// ---------------------------------------------------------------------------
// Which light topics merge by resolution: those with at least this many multi
// entries (the rest, and every heavy topic, by hash table).  Measured
// (profiles/r03/r03m): resolution wins on wide topics (C4 shard, ~1000 multi
// entries per topic: emission 33.1 -> 23.5 ms) and loses on many small ones
// (C3: 8.1 -> 10.8 ms), so by default it takes the topics past the wave-table
// tier (> 192 entries: r03n, C3 14.35 vs 14.48 ms and C4 shard 28.24 vs 28.80
// ms against a threshold of 769).  Read at every batch (a test compares modes in one process):
// MQM_RESOLVE=1 every light topic, MQM_RESOLVE=0 none,
// MQM_RESOLVE_MIN=m the threshold.
static bool walk_slots() { return slots_enabled(); }
static bool desc_copy_on() {
  static const bool v = getenv("MQM_DESC_COPY") && atoi(getenv("MQM_DESC_COPY")) != 0;
  return v;
}
// MQM_WINCOPY_VEC=1: the window copy moves 4 positions per lane at a time (A/B)
static bool wincopy_vec() {
  static const bool v = getenv("MQM_WINCOPY_VEC") && atoi(getenv("MQM_WINCOPY_VEC")) != 0;
  return v;
}
// the window copy's stores non-temporal, on by default (C3 773-782M vs
// 740-746M topics/s, emission 8.02 -> 7.62 ms, r05ak); MQM_NT_STORE=0 for the
// plain stores
static bool nt_store() {
  static const bool v = !getenv("MQM_NT_STORE") || atoi(getenv("MQM_NT_STORE")) != 0;
  return v;
}
// MQM_LONG_PART=m: solo parts of at least m entries take k_longcopy (A/B; off
// by default: measured slower than the window copy alone, r05e — DESIGN §3)
static uint32_t long_part_min() {
  if (const char *v = getenv("MQM_LONG_PART")) {
    const long x = atol(v);
    return x <= 0 ? 0xFFFFFFFFu : (uint32_t)x;
  }
  return 0xFFFFFFFFu;
}
constexpr uint32_t kResolveMinDefault = 193;
static uint32_t resolve_min() {
  if (const char *v = getenv("MQM_RESOLVE")) return atoi(v) != 0 ? 1u : 0xFFFFFFFFu;
  if (const char *v = getenv("MQM_RESOLVE_MIN")) return (uint32_t)std::max(1L, atol(v));
  return kResolveMinDefault;
}

template <int kH>
struct alignas(16) ResolveLds {
  uint32_t rec[4 + kRecHit * kH];  // header + multi parts (the record's tail, in the walk's order)
  uint32_t key[2 * kH], rank[2 * kH];  // gathered multi parts by multi-tail start + 1 (0: empty) -> hit rank
};

template <int kE, int kH, int kPer, int kChunk = 0, bool kIdent = false>
__global__ __launch_bounds__(kWave *kEmitWaves) __attribute__((amdgpu_waves_per_eu(6))) void k_resolve(DeviceSnapshot s, Outputs o,
                                                               const uint32_t *__restrict__ list,
                                                               const unsigned int *__restrict__ count) {
  constexpr int kGroups = kWave / kE;
  constexpr uint64_t kGMask = kE == 64 ? ~0ull : (1ull << kE) - 1ull;
  constexpr int kUnits = 1 + kH;  // record units (16 B) read per topic
  constexpr uint32_t kT = 2 * kH, kTBits = kH == 64 ? 7 : kH == 32 ? 6 : kH == 16 ? 5 : 4;
  static_assert(kH <= kHCap && kUnits <= kRecStrideAlloc / 4 && (1u << kTBits) == kT, "record tail / table");
  __shared__ ResolveLds<kH> lds_all[kEmitWaves * kGroups];
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / kE, gl = lane % kE, gbase = g * kE;
  const uint64_t glt = (1ull << gl) - 1ull;
  ResolveLds<kH> &L = lds_all[(threadIdx.x / kWave) * kGroups + g];
  const uint32_t ngroups = gridDim.x * kEmitWaves * kGroups, nl = *count;
  auto tslot = [](uint32_t k) { return (k * 2654435769u) >> (32 - kTBits); };
  // the next topic's list entry, segment start and record tail (header + kH
  // parts, unconditionally: inside the record slot) load while this one resolves
  constexpr int kUPer = (kUnits + kE - 1) / kE;
  uint32_t t_n = 0;
  uint64_t db_n = 0;
  uint4 u_n[kUPer];
  auto fetch = [&](uint32_t k) {
    t_n = list[k];
    db_n = o.dstart[t_n];
    const uint4 *gt = rec_tail(o.recs, t_n);
#pragma unroll
    for (int v = 0; v < kUPer; v++)
      if (v * kE + gl < kUnits) u_n[v] = gt[-(v * kE + gl)];
  };
  // kChunk > 0 (a wave per topic only): list entries taken kChunk at a time
  // from a device counter, so a wave that drew wide topics takes fewer;
  // else a fixed stride over the list
  uint32_t c_end = 0;
  auto take = [&](uint32_t cur) -> uint32_t {
    if (cur + 1 < c_end) return cur + 1;
    uint32_t v = 0;
    if (gl == 0) v = atomicAdd(&o.ctr->res_next, (unsigned)kChunk);
    v = __builtin_amdgcn_readfirstlane(v);  // (kChunk: a wave per topic)
    c_end = v + kChunk;
    return v;
  };
  uint32_t i = kChunk ? take(~0u) : (blockIdx.x * kEmitWaves + threadIdx.x / kWave) * kGroups + g;
  if (i < nl) fetch(i);
  for (uint32_t i_next; i < nl; i = i_next) {
    i_next = kChunk ? take(i) : i + ngroups;
    const uint32_t t = t_n;
    const uint64_t db = db_n;
    uint4 *rec4 = reinterpret_cast<uint4 *>(L.rec);
#pragma unroll
    for (int v = 0; v < kUPer; v++)
      if (v * kE + gl < kUnits) rec4[v * kE + gl] = u_n[v];
    for (uint32_t j = gl; j < kT; j += kE) L.key[j] = 0;
    if (i_next < nl) fetch(i_next);
    wave_lds_sync();
    const uint32_t nh = L.rec[0] & 0xFFu, Ss = L.rec[1], M = L.rec[2];
    const uint64_t ib = kIdent ? ident_base(o, t, M, gl == 0) : ~0ull;
    uint32_t nid = 0;
    // the gathered multi parts by their range's multi-tail start (a node's
    // range is gathered at most once per topic: distinct keys)
    for (uint32_t h = gl; h < nh; h += kE) {
      const uint32_t k = rec_at(L.rec, h, kFieldOff) + 1u;
      uint32_t sl = tslot(k);
      while (atomicCAS(&L.key[sl], 0u, k) != 0u) sl = (sl + 1) & (kT - 1);
      L.rank[sl] = rec_at(L.rec, h, kFieldRank);
    }
    wave_lds_sync();
    rec_prefix<kE, kH>(L.rec, nh, gl);  // part counts -> exclusive prefixes (multi_sid)
    wave_lds_sync();
    uint32_t D = 0;
    for (uint32_t q0 = 0; q0 < M; q0 += kE * kPer) {
      uint32_t sid[kPer], rk[kPer], wd[kPer], iw[kIdent ? kPer : 1];
      uint32_t im = 0;  // (kIdent) bit k: entry k's Identifier is > 0
      uint2 pi[kPer];
#pragma unroll
      for (int k = 0; k < kPer; k++) {  // every entry's loads in flight together
        const uint32_t q = q0 + k * kE + gl;
        uint32_t h;
        sid[k] = multi_sid(L.rec, nh, q < M ? q : 0, &h);
        rk[k] = rec_at(L.rec, h, kFieldRank);
        wd[k] = s.words[sid[k]];
        pi[k] = s.pinfo[sid[k]];
        if constexpr (kIdent) iw[k] = s.ident_bits[sid[k] >> 5];  // (1.25 MB at C3: L2)
      }
      if constexpr (kIdent) {
#pragma unroll
        for (int k = 0; k < kPer; k++) im |= ((iw[k] >> (sid[k] & 31)) & 1u) << k;
      }
#pragma unroll
      for (int k = 0; k < kPer; k++) {
        const uint32_t q = q0 + k * kE + gl;
        bool win = q < M;
        uint32_t qb = qos_bits(wd[k]);
        // a partner: its range's multi-tail start | QoS << 28 | NoLocal << 30;
        // gathered iff that range is one of the topic's multi parts (its own
        // node differs from this entry's, so its hit rank does too)
        auto meet = [&](uint32_t pw) {
          const uint32_t key = (pw & kWordSidMask) + 1u;
          uint32_t sl = tslot(key), kk;
          while ((kk = L.key[sl]) != 0u && kk != key) sl = (sl + 1) & (kT - 1);
          if (kk != key) return;
          qb |= qos_bits(pw);
          if (L.rank[sl] < rk[k]) win = false;
        };
        if (win) {
          if (pi[k].y == kPInfoHeavy) {  // routed here by mistake: never expected (kClsHeavy)
            atomicOr(&o.ctr->oob, kOobHeavy);
          } else if (pi[k].y != kNone && (pi[k].y & kPInfoList)) {  // (kNone: one inline partner)
            const uint32_t c = pi[k].y & 0xFFu;
            for (uint32_t j = 0; j < c; j++) meet(s.partners[pi[k].x + j]);
          } else {
            if (pi[k].x != kNone) meet(pi[k].x);
            if (pi[k].y != kNone) meet(pi[k].y);
          }
        }
        const uint64_t m = (__ballot(win) >> gbase) & kGMask;
        if (win)
          put_checked(o.dout, db + Ss + D + __popcll(m & glt), o.dcap,
                      pack_delivery(sid[k], 31u - __builtin_clz(qb & 7u), (qb >> 3) & 1u), &o.ctr->oob);
        D += __popcll(m);
      }
      if constexpr (kIdent) {  // (wave-uniform) the identified entries, in entry order
#pragma unroll
        for (int k = 0; k < kPer; k++) {
          const uint32_t q = q0 + k * kE + gl;
          ident_put<kE>(o, ib, ib != ~0ull && q < M && ((im >> k) & 1u), sid[k], gbase, glt, nid);
        }
      }
    }
    if (gl == 0) o.dcount[t] = Ss + D;
    if (kIdent && gl == 0 && ib != ~0ull) o.icount[t] = nid;
    wave_lds_sync();
  }
}

// ---------------------------------------------------------------------------
// k_dfs<P>: the unbounded path.  P0 counts raw entries / shared candidates;
// P1 inserts into a per-topic global table and writes the shared candidates;
// P2 counts the table's clients and writes the deliveries.  Output goes to
// the tail regions after the scanned segments.
// ---------------------------------------------------------------------------
struct GEnt {                  // global dedupe slot (16 B)
  unsigned long long keybits;  // (client + 1) | bits << 32
  unsigned long long first;    // ~((rank << 32) | sid), atomicMax: the table starts zeroed
};

template <int kPhase>
__global__ __launch_bounds__(kWave) void k_dfs(DeviceSnapshot s, const uint8_t *__restrict__ tbytes,
                                              const uint64_t *__restrict__ toffs, Outputs o,
                                              uint64_t *__restrict__ raw_cnt, uint64_t *__restrict__ raw_h,
                                              const uint64_t *__restrict__ tab_off, GEnt *__restrict__ tab,
                                              uint32_t max_levels) {
  extern __shared__ uint32_t dyn[];
  // layout: sep[max_levels] | key0/key1 (u64 x max_levels each) | stack (4 x u32) x (2*max_levels + 8)
  uint32_t *sep = dyn;
  uint64_t *key0 = reinterpret_cast<uint64_t *>(dyn + ((max_levels + 1) & ~1u));
  uint64_t *key1 = key0 + max_levels;
  uint32_t *stk = reinterpret_cast<uint32_t *>(key1 + max_levels);
  const int lane = threadIdx.x;
  // raw_cnt / raw_h / tab_off hold dfs_cap topics (o.dfs_cap); a longer list
  // (or DFS tails that do not fit) makes k_dfs_prep flag the call for a re-run
  const uint32_t cnt = min(o.ctr->n_dfs, o.dfs_cap);
  if ((kPhase == 1 || kPhase == 2) && o.ctr->cap_ovf) return;
  for (uint32_t i = blockIdx.x; i < cnt; i += gridDim.x) {
    const uint32_t t = o.dfs_list[i];
    const uint64_t off = toffs[t];
    const uint32_t len = (uint32_t)(toffs[t + 1] - off);
    const uint8_t *tp = tbytes + off;
    const uint64_t tsz = (kPhase == 1 || kPhase == 2) ? tab_off[i + 1] - tab_off[i] : 0;
    GEnt *T = (kPhase == 1 || kPhase == 2) ? tab + tab_off[i] : nullptr;

    if (kPhase == 2) {
      uint32_t D = 0;
      for (uint64_t b = 0; b < tsz; b += kWave) {
        const uint64_t j = b + lane;
        D += __popcll(__ballot(j < tsz && (uint32_t)T[j].keybits != 0));
      }
      uint64_t db = 0;
      if (lane == 0 && D) db = atomicAdd(&o.ctr->dtail, (unsigned long long)D);
      db = shfl64(db, 0);
      uint32_t w = 0;
      for (uint64_t b = 0; b < tsz; b += kWave) {
        const uint64_t j = b + lane;
        GEnt gg{0, 0};
        if (j < tsz) gg = T[j];
        const bool occ = (uint32_t)gg.keybits != 0;
        const uint64_t m = __ballot(occ);
        if (occ) {
          const uint32_t bits = (uint32_t)(gg.keybits >> 32);
          put_checked(o.dout, db + w + __popcll(m & lanemask_lt(lane)), o.dcap,
                      pack_delivery((uint32_t)~gg.first & kWordSidMask, 31u - __builtin_clz(bits & 7u),
                                    (bits >> 3) & 1u),
                      &o.ctr->oob, kOobDfs);
        }
        w += __popcll(m);
      }
      if (lane == 0) {
        o.dcount[t] = D;
        o.dstart[t] = db;
      }
      continue;
    }

    // tokenize up to max_levels levels
    uint32_t nsep = 0;
    bool dollar = false;
    for (uint32_t base = 0; base < len && nsep < max_levels; base += kWave) {
      const uint32_t p = base + lane;
      const uint8_t b = p < len ? tp[p] : 0;
      if (base == 0) dollar = __shfl(b, 0, 64) == '$';
      const uint64_t m = __ballot(p < len && b == '/');
      if (b == '/' && p < len) {
        const uint32_t idx = nsep + __popcll(m & lanemask_lt(lane));
        if (idx < max_levels) sep[idx] = p;
      }
      nsep += __popcll(m);
    }
    const uint32_t nlev = len == 0 ? 0 : (nsep >= max_levels ? max_levels + 1 : nsep + 1);
    wave_lds_sync();
    const uint32_t nkeys = nlev < max_levels ? nlev : max_levels;
    for (uint32_t k = lane; k < nkeys; k += kWave) {
      const uint32_t st = k == 0 ? 0 : sep[k - 1] + 1;
      const uint32_t en = (k < nsep) ? sep[k] : len;
      Key kk = make_key([&](uint32_t j) { return tp[st + j]; }, en - st);
      key0[k] = kk.k0;
      key1[k] = kk.k1;
    }
    wave_lds_sync();

    uint64_t S = 0;
    uint32_t H = 0, nid = 0;
    uint64_t hb = 0;
    if (kPhase == 1) {
      const uint32_t hn = (uint32_t)raw_h[i];  // counted by phase 0
      if (lane == 0 && hn) hb = atomicAdd(&o.ctr->htail, (unsigned long long)hn);
      hb = shfl64(hb, 0);
      if (lane == 0) {
        o.hstart[t] = hb;
        o.hcount[t] = hn;
      }
    }
    uint32_t lg = 0;
    if (kPhase == 1)
      while ((1ull << lg) < tsz) lg++;
    // DFS stack of (node, plus, hash, depth); bounded by 2 * height + 1
    int sp = 0;
    if (nlev > 0) {
      if (lane == 0) {
        const NodeDesc r = load_desc(s.nodes);
        stk[0] = 0;
        stk[1] = r.plus;
        stk[2] = r.hash;
        stk[3] = 0;
      }
      sp = 1;
    }
    wave_lds_sync();
    while (sp > 0) {
      sp--;
      const uint32_t node = stk[4 * sp], pl = stk[4 * sp + 1], hs = stk[4 * sp + 2], d = stk[4 * sp + 3];
      wave_lds_sync();
      const uint64_t k0 = key0[d], k1 = key1[d];
      const bool has_next = d + 1 < nlev;
      const bool lit_is_wild = (k1 == (1ull << 56)) && (k0 == '+' || k0 == '#');
      const uint32_t tst = d == 0 ? 0 : sep[d - 1] + 1;
      const uint32_t tln = ((d < nsep) ? sep[d] : len) - tst;
      uint32_t c = kNone;
      NodeDesc dc;
      if (lane == 0 && !lit_is_wild) c = probe_edge(s, node, k0, k1, tp + tst, tln, &dc);
      if (lane == 1 && pl != kNone) {
        c = pl;
        dc = load_desc(s.nodes + c);
      }
      if (lane == 2 && hs != kNone) {
        c = hs;
        dc = load_desc(s.nodes + c);
      }
      for (int src = 0; src < 3; src++) {  // the 3 probe results, wave-uniformly
        const uint32_t cc = __shfl(c, src, 64);
        if (cc == kNone) continue;
        NodeDesc e;
        e.plus = __shfl(dc.plus, src, 64);
        e.hash = __shfl(dc.hash, src, 64);
        e.sub_off = __shfl(dc.sub_off, src, 64);
        e.sub_cnt = __shfl(dc.sub_cnt, src, 64);
        e.multi = __shfl(dc.multi, src, 64);
        e.hsub_cnt = __shfl(dc.hsub_cnt, src, 64);
        e.sh_off = __shfl(dc.sh_off, src, 64);
        e.sh_cnt_flags = __shfl(dc.sh_cnt_flags, src, 64);
        const uint32_t fl = e.sh_cnt_flags >> 24;
        const bool skip_dollar = dollar && (fl & kFlagDollarWild);
        for (int part = 0; part < 2; part++) {
          if (part == 1 && src != 0) break;
          const uint32_t roff = part ? e.sub_off + e.sub_cnt : e.sub_off;  // '#' child's range follows
          // (a '#' node after a literal parent: its parent probe gathered it, kFlagParentLit)
          const uint32_t rcnt = skip_dollar || (part == 0 && (fl & kFlagParentLit)) ? 0 : (part ? e.hsub_cnt : e.sub_cnt);
          const uint32_t rank = 2 * cc + part;
          S += rcnt;
          if (kPhase >= 3) {  // identifiers: the range's entries with Identifier > 0
            for (uint32_t b0 = 0; b0 < rcnt; b0 += kWave) {
              const uint32_t j = b0 + lane;
              const bool has = j < rcnt && (s.subs[roff + j].word & kWordIdent);
              const uint64_t m = __ballot(has);
              if (kPhase == 4 && has) o.iout[o.istart[t] + nid + __popcll(m & lanemask_lt(lane))] = roff + j;
              nid += (uint32_t)__popcll(m);
            }
          }
          if (kPhase == 1) {
            for (uint32_t j = lane; j < rcnt; j += kWave) {
              const uint32_t sid = roff + j;
              const SubEnt se = s.subs[sid];
              uint64_t slot = ((uint64_t)(se.client * 2654435769u) << lg) >> 32;
              for (;;) {
                const unsigned long long prev =
                    atomicCAS(reinterpret_cast<unsigned long long *>(&T[slot].keybits), 0ull,
                              (unsigned long long)(se.client + 1));
                if (prev == 0 || (uint32_t)prev == se.client + 1) break;
                slot = (slot + 1) & (tsz - 1);
              }
              atomicOr(&T[slot].keybits, (unsigned long long)qos_bits(se.word) << 32);
              atomicMax(&T[slot].first, ~(((unsigned long long)rank << 32) | sid));
            }
          }
        }
        const uint32_t shc = e.sh_cnt_flags & kShCntMask;
        if (kPhase == 1)
          for (uint32_t j = lane; j < shc; j += kWave) put_checked(o.hout, hb + H + j, o.hcap, e.sh_off + j, &o.ctr->oob, kOobDfs);
        H += shc;
        if (has_next && (fl & kFlagHasChildren)) {
          if (lane == 0) {
            stk[4 * sp] = cc;
            stk[4 * sp + 1] = e.plus;
            stk[4 * sp + 2] = e.hash;
            stk[4 * sp + 3] = d + 1;
          }
          sp++;
        }
      }
      wave_lds_sync();
    }
    if (lane == 0 && kPhase == 0) {
      raw_cnt[i] = S;
      raw_h[i] = H;
    }
    if (lane == 0 && kPhase == 3) o.icount[t] = nid;
  }
}

// ---------------------------------------------------------------------------
// k_ident: Subscription.Identifiers support (packets.go:250-259).  For every
// bounded topic, the sids of the gathered *multi* entries whose Identifier is
// > 0 (kMetaIdent), part by part from the walk's record, written once into the
// topic's Ms-bounded scratch area (mstart = the scan of mcount) with their
// count; k_ident_pack then moves them to iout at the scan of the counts.  (One
// pass over the records: round 5's count-then-write pair read every record
// and identifier word twice, 3.1 + 3.5 ms on C3.)  A solo entry is its
// client's only subscription in any topic's gather (that is what solo means,
// flatten.cpp), so its delivery's map is its first pair {Filter: Identifier}
// alone, which the host already has from the delivery's first sid: listing it
// would add nothing.  So only the multi parts are read — C3 gathers 233
// entries per topic, almost all solo.  A node gathered twice repeats its
// sids; the map the host builds keeps one key per filter, as the reference's
// does.  DFS topics are handled by k_dfs<3|4> (every entry).
// ---------------------------------------------------------------------------
// (early: beside the match, ident_launch — DFS topics get a count of 0 and a
// scratch area past `cap` raises *ovf instead of writing; the call then runs
// the pass again after the match)
__global__ __launch_bounds__(256) void k_ident(DeviceSnapshot s, Outputs o, uint32_t n,
                                               const uint64_t *__restrict__ mstart, uint32_t *__restrict__ scratch,
                                               uint64_t cap, unsigned long long *ovf) {
  // an 8-lane group per topic: most topics have a few short multi parts, and
  // a wavefront per topic left 56 lanes idle through each topic's dependent
  // loads (C3: 5.5 ms for the two phases, r05d)
  constexpr int kL = 8;
  const int lane = threadIdx.x & (kWave - 1), gl = lane % kL, gbase = lane - gl;
  const uint64_t glt = (1ull << gl) - 1ull;
  const uint32_t groups = gridDim.x * (blockDim.x / kL);
  for (uint32_t t = (blockIdx.x * blockDim.x + threadIdx.x) / kL; t < n; t += groups) {
    const uint8_t cls = o.cls[t];
    if (cls == kClsDfs) {
      if (ovf && gl == 0) o.icount[t] = 0;
      continue;
    }
    uint32_t nid = 0;
    // (the walk writes the record header, which counts the multi parts, for
    // every topic with multi entries)
    uint32_t ms = cls != kClsDone ? o.mcount[t] : 0u;
    const uint64_t ib = ms ? mstart[t] : 0;
    if (ms && ib + ms > cap) {
      if (gl == 0) atomicOr(ovf, 1ull);
      ms = 0;
    }
    if (ms) {
      const uint4 *gt = rec_tail(o.recs, t);
      const uint32_t nm = gt[0].x & 0xFFu;
      for (uint32_t h = 0; h < nm; h++) {  // the multi parts (solo parts: see above)
        const uint4 u = gt[-(int)(1 + h)];
        const uint32_t off = u.x, cnt = u.y;
        for (uint32_t b0 = 0; b0 < cnt; b0 += kL) {
          const uint32_t j = b0 + gl;
          const uint32_t q = off + j;
          const bool has = j < cnt && ((s.ident_bits[q >> 5] >> (q & 31)) & 1u);
          const uint64_t m = (__ballot(has) >> gbase) & ((1ull << kL) - 1ull);
          const uint32_t at = nid + (uint32_t)__popcll(m & glt);
          if (has && at < ms) scratch[ib + at] = q;  // (at < Ms: the multi entries bound the listed ones)
          nid += (uint32_t)__popcll(m);
        }
      }
      nid = min(nid, ms);
    }
    if (gl == 0) o.icount[t] = nid;
  }
}

// a wavefront per 64 topics: their listed sids from the scratch areas to
// iout[istart[t] ..).  The lanes scan the 64 counts, then copy the wave's
// entries 64 at a time (entry -> topic by a 6-step search over the prefix in
// LDS), so loads and stores stay lane-consecutive across topic boundaries
// (8 lanes per topic moved 19 sids per topic at 0.86 TB/s, 1.81 ms on C3,
// r05y).  DFS topics: k_dfs<4> writes theirs.
__global__ __launch_bounds__(256) void k_ident_pack(Outputs o, uint32_t n, const uint64_t *__restrict__ mstart,
                                                    const uint32_t *__restrict__ scratch, uint64_t cap,
                                                    unsigned long long *ovf) {
  __shared__ uint32_t pre_all[4][kWave + 1];
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  uint32_t *pre = pre_all[wid];
  const uint32_t nw = gridDim.x * (blockDim.x / kWave);
  for (uint32_t w = blockIdx.x * (blockDim.x / kWave) + wid; (uint64_t)w * kWave < n; w += nw) {
    const uint32_t t = w * kWave + lane;
    uint32_t c = 0;
    uint64_t src = 0, dst = 0;
    if (t < n && o.cls[t] != kClsDfs) {
      c = o.icount[t];
      src = mstart[t];
      dst = o.istart[t];
    }
    uint32_t inc = c;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      const uint32_t v = __shfl_up(inc, d, kWave);
      if (lane >= d) inc += v;
    }
    const uint32_t total = __shfl(inc, kWave - 1, kWave);
    if (total == 0) continue;  // (wave-uniform)
    pre[lane] = inc - c;
    if (lane == 0) pre[kWave] = total;
    wave_lds_sync();
    for (uint32_t b = 0; b < total; b += kWave) {  // (every lane runs every step: the shuffles)
      const uint32_t e = b + lane;
      const bool ok = e < total;
      uint32_t k = 0;  // the topic holding entry e: the largest k with pre[k] <= e
#pragma unroll
      for (uint32_t step = 32; step > 0; step >>= 1) k = pre[k + step] <= e ? k + step : k;
      const uint32_t j = e - pre[k];
      const uint64_t s0 = shfl64(src, (int)k), d0 = shfl64(dst, (int)k);
      if (ok) {
        if (!ovf)
          put_checked(o.iout, d0 + j, cap, scratch[s0 + j], &o.ctr->oob);
        else if (d0 + j < cap)
          o.iout[d0 + j] = scratch[s0 + j];
        else
          atomicOr(ovf, 2ull);
      }
    }
    wave_lds_sync();
  }
}

// ---- the runs form (runs_device): every bounded topic's solo parts, listed
// from its record (the walk wrote them there and copied nothing) ------------
__global__ __launch_bounds__(256) void k_run_count(Outputs o, uint32_t n, uint32_t *__restrict__ nrun) {
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x)
    nrun[t] = (o.cls[t] & kClsBounded) ? rec_tail(o.recs, t)[0].w : 0u;
}

// 8 lanes per topic: its runs (8 B each) to runs[roff[t] ..)
__global__ __launch_bounds__(256) void k_run_copy(Outputs o, uint32_t n, const uint64_t *__restrict__ roff,
                                                  uint2 *__restrict__ runs, uint64_t cap) {
  constexpr int kL = 8;
  const uint32_t gl = threadIdx.x % kL, ng = gridDim.x * (blockDim.x / kL);
  for (uint32_t t = (blockIdx.x * blockDim.x + threadIdx.x) / kL; t < n; t += ng) {
    const uint64_t a = roff[t], c = roff[t + 1] - a;
    const uint2 *rec = reinterpret_cast<const uint2 *>(o.recs + (uint64_t)t * kRecStrideAlloc);
    for (uint32_t j = gl; j < c; j += kL) put_checked(runs, a + j, cap, rec[j], &o.ctr->oob);
  }
}

// DFS sizing on the device (one workgroup): per DFS topic a dedupe table of
// the next power of two >= 2 x its raw entries (>= 64), their offsets, the
// DFS tails' start after the scanned segments, the totals — and the capacity
// check of a queued call (its buffers were sized from an earlier call)
__global__ __launch_bounds__(256) void k_dfs_prep(Counters *ctr, const uint64_t *__restrict__ raw_cnt,
                                                  const uint64_t *__restrict__ raw_h, uint64_t *__restrict__ tab_off,
                                                  uint32_t dfs_cap, uint64_t tab_cap,
                                                  const uint64_t *__restrict__ s_tot_ptr,
                                                  const uint64_t *__restrict__ h_tot_ptr, uint64_t dcap, uint64_t hcap) {
  __shared__ unsigned long long wsum[4], wraw[4], wh[4];
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  const uint32_t nd = ctr->n_dfs, n = min(nd, dfs_cap);
  unsigned long long run = 0, raw = 0, hh = 0;
  for (uint32_t b = 0; b < n; b += 256) {
    const uint32_t i = b + tid;
    unsigned long long sz = 0;
    if (i < n) {
      sz = 64;
      while (sz < 2 * raw_cnt[i]) sz <<= 1;
      raw += raw_cnt[i];
      hh += raw_h[i];
    }
    unsigned long long inc = sz;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      const unsigned long long u = shfl64(inc, max(lane - d, 0));
      if (lane >= d) inc += u;
    }
    if (lane == kWave - 1) wsum[wid] = inc;
    __syncthreads();
    unsigned long long before = run;
    for (int k = 0; k < wid; k++) before += wsum[k];
    if (i < n) tab_off[i] = before + inc - sz;
    for (int k = 0; k < 4; k++) run += wsum[k];
    __syncthreads();
  }
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) {
    raw += shfl64(raw, lane ^ d);
    hh += shfl64(hh, lane ^ d);
  }
  if (lane == 0) wraw[wid] = raw, wh[wid] = hh;
  __syncthreads();
  if (tid == 0) {
    raw = wraw[0] + wraw[1] + wraw[2] + wraw[3];
    hh = wh[0] + wh[1] + wh[2] + wh[3];
    tab_off[n] = run;
    const unsigned long long st = *s_tot_ptr, ht = *h_tot_ptr;
    ctr->dtail = st;
    ctr->htail = ht;
    ctr->tab_total = run;
    ctr->dfs_raw = raw;
    ctr->dfs_h = hh;
    if (nd > dfs_cap || run > tab_cap || st + raw > dcap || ht + hh > hcap) ctr->cap_ovf = 1;
  }
}

__global__ __launch_bounds__(256) void k_zero_tab(unsigned long long *__restrict__ tab, const Counters *ctr,
                                                  uint64_t tab_cap) {
  const uint64_t n = 2 * min((uint64_t)ctr->tab_total, tab_cap);  // GEnt = two 64-bit words
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    tab[i] = 0;
}

// what the call needed, for the host (read back once, at the end)
__global__ void k_totals(Counters *ctr, const uint64_t *__restrict__ dstart, const uint64_t *__restrict__ hstart,
                         const uint64_t *__restrict__ desc_start, uint32_t n) {
  if (threadIdx.x == 0) {
    ctr->s_total = dstart[n];
    ctr->h_total = hstart[n];
    (void)desc_start;  // (n_desc: the walk counts the solo parts, runs form included)
  }
}

// segments -> dense CSR (one wavefront per topic); deliveries resolved to
// {client, packed} (the client of the first-merged subscription), or the
// packed words alone (kPacked: 4 B per delivery, the client being the first
// subscription's)
template <bool kPacked>
__global__ __launch_bounds__(256) void k_densify(DeviceSnapshot s, uint32_t n, const uint32_t *__restrict__ dcount,
                                                const uint64_t *__restrict__ dstart,
                                                const uint64_t *__restrict__ doffs, const uint32_t *__restrict__ dsrc,
                                                void *__restrict__ ddst_v, const uint32_t *__restrict__ hcount,
                                                const uint64_t *__restrict__ hstart,
                                                const uint64_t *__restrict__ hoffs, const uint32_t *__restrict__ hsrc,
                                                uint32_t *__restrict__ hdst) {
  const int lane = threadIdx.x & (kWave - 1);
  const uint32_t nwaves = gridDim.x * (blockDim.x / kWave);
  for (uint32_t t = blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave; t < n; t += nwaves) {
    const uint32_t D = dcount[t], H = hcount[t];
    const uint64_t ds = dstart[t], dd = doffs[t], hs = hstart[t], hd = hoffs[t];
    if (kPacked) {
      uint32_t *ddst = static_cast<uint32_t *>(ddst_v);
      for (uint32_t j = lane; j < D; j += kWave) ddst[dd + j] = dsrc[ds + j];
    } else {
      uint64_t *ddst = static_cast<uint64_t *>(ddst_v);
      for (uint32_t j = lane; j < D; j += kWave) {
        const uint32_t p = dsrc[ds + j];
        ddst[dd + j] = (uint64_t)s.subs[p & kWordSidMask].client | ((uint64_t)p << 32);
      }
    }
    for (uint32_t j = lane; j < H; j += kWave) hdst[hd + j] = hsrc[hs + j];
  }
}

// merge lists in one pass over the topics (replaces one DeviceSelect per
// list): each block counts its chunk's members per list (wave ballots, LDS
// counters), reserves its ranges with one global atomic per list, then
// writes them.  Order within a list is unspecified (lists only schedule
// work; every topic's output position is its own dstart).
enum : int { kLSmall = 0, kLWave, kLT1, kLT2, kLT3, kLPart, kLShared, kLResSmall, kLRes, kNLists };
// k_multi<1024> / <2048> / <4096> capacities (load 0.75); k_multi_part beyond
// (partition passes re-read every entry: a single-pass 4096-slot table is
// cheaper up to its capacity)
constexpr uint32_t kT1Max = 768, kT2Max = 1536, kT3Max = 3072;
struct Lists {
  uint32_t *l[kNLists];
};

// the merge list of a topic with multi entries (by their count m), and the
// shared-candidate list
__device__ __forceinline__ uint32_t route_mask(uint8_t c, uint32_t m, uint32_t h, uint32_t res_min) {
  if (!(c & kClsBounded)) return 0;
  const uint32_t sh = h ? (1u << kLShared) : 0u;
  if (m == 0) return sh;
  if (m >= res_min && !(c & kClsHeavy))  // merge by resolution (k_resolve)
    return sh | (((c & kClsFewHits) && m <= kSmallMultiS) ? (1u << kLResSmall) : (1u << kLRes));
  if ((c & kClsFewHits) && m <= kSmallMultiS) return sh | (1u << kLSmall);
  return sh | (m <= kSmallMulti ? (1u << kLWave)
               : m <= kT1Max  ? (1u << kLT1)
               : m <= kT2Max  ? (1u << kLT2)
               : m <= kT3Max  ? (1u << kLT3)
                              : (1u << kLPart));
}

__global__ __launch_bounds__(256) void k_route(const uint8_t *__restrict__ cls, const uint32_t *__restrict__ mcount,
                                               const uint32_t *__restrict__ hcount, uint32_t n, Lists L,
                                               unsigned int *__restrict__ counts,
                                               unsigned long long *__restrict__ msum, uint32_t res_min) {
  __shared__ unsigned int lc[kNLists], base[kNLists];
  __shared__ unsigned long long ms[3];
  const int tid = threadIdx.x, lane = tid & (kWave - 1);
  if (tid < 3) ms[tid] = 0;
  const uint32_t per = (n + gridDim.x - 1) / gridDim.x;
  const uint32_t lo = blockIdx.x * per, hi = min(n, lo + per);
  if (tid < kNLists) lc[tid] = 0;
  __syncthreads();
  for (uint32_t t0 = lo; t0 < hi; t0 += blockDim.x) {
    const uint32_t t = t0 + tid;
    const uint32_t r = t < hi ? route_mask(cls[t], mcount[t], hcount[t], res_min) : 0;
#pragma unroll
    for (int l = 0; l < kNLists; l++) {
      const uint64_t m = __ballot((r >> l) & 1u);
      if (lane == 0 && m) atomicAdd(&lc[l], (unsigned int)__popcll(m));
    }
    if (r & ((1u << kLT1) | (1u << kLT2) | (1u << kLT3) | (1u << kLPart)))
      atomicAdd(&ms[(r >> kLPart) & 1u || (r >> kLT3) & 1u ? 2 : (r >> kLT2) & 1u ? 1 : 0], (unsigned long long)mcount[t]);
  }
  __syncthreads();
  if (tid < 3 && ms[tid]) atomicAdd(&msum[tid], ms[tid]);
  if (tid < kNLists) {
    base[tid] = lc[tid] ? atomicAdd(&counts[tid], lc[tid]) : 0;
    lc[tid] = 0;
  }
  __syncthreads();
  for (uint32_t t0 = lo; t0 < hi; t0 += blockDim.x) {
    const uint32_t t = t0 + tid;
    const uint32_t r = t < hi ? route_mask(cls[t], mcount[t], hcount[t], res_min) : 0;
#pragma unroll
    for (int l = 0; l < kNLists; l++) {
      const bool in = (r >> l) & 1u;
      const uint64_t m = __ballot(in);
      uint32_t wpos = 0;
      if (lane == 0 && m) wpos = atomicAdd(&lc[l], (unsigned int)__popcll(m));
      wpos = __shfl(wpos, 0, 64);
      if (in) L.l[l][base[l] + wpos + __popcll(m & lanemask_lt(lane))] = t;
    }
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

}  // namespace

// ---------------------------------------------------------------------------
// workspace / orchestration
// ---------------------------------------------------------------------------
int Workspace::end(hipStream_t st) {
  if (!last_use && hipEventCreateWithFlags(&last_use, hipEventDisableTiming) != hipSuccess) {
    last_use = nullptr;
    return -3;
  }
  if (hipEventRecord(last_use, st) != hipSuccess) return -3;
  used = true;
  return 0;
}

int Workspace::drain() {
  if (cur && hipStreamSynchronize(cur) != hipSuccess) return -3;
  if (used && last_use && hipEventSynchronize(last_use) != hipSuccess) return -3;
  return 0;
}

// Workspace memory comes from hipMalloc, and a grown-out buffer goes to the
// index layer's reaper (flatten.h retire_device_buffers: it stops the
// per-publish servers, then hipFree — which waits for every kernel on the
// device).  Round 5 used the stream-ordered pool (hipMallocAsync /
// hipFreeAsync), whose reuse of freed memory served kernels stale contents
// (tools/reuse_probe.hip r05s/r05u; the device edge build's pool temporaries
// made recycled snapshots miss their newest edges, r06d): no pool memory
// anywhere in the library now.
static void retire(void *p) {
  if (!p) return;
  int dev = -1;
  (void)hipGetDevice(&dev);
  retire_device_buffers(dev, {p});
}

int Workspace::reserve(void **p, size_t *cap, size_t need) {
  if (*cap >= need && *p) return 0;
  if (*p) {
    // queued kernels of this call (cur) or of earlier calls (last_use) may
    // still read the old buffer
    if (drain()) return -3;
    retire(*p);
  }
  *p = nullptr;
  size_t n = std::max<size_t>(need, 256);
  n = n + n / 4;
  if (hipMalloc(p, n) != hipSuccess) {
    *p = nullptr;
    *cap = 0;
    return -2;
  }
  *cap = n;
  return 0;
}

int Workspace::grow_keep(Slot s, size_t used_bytes, size_t need, hipStream_t st) {
  Buf &b = bufs[s];
  if (b.cap >= need && b.p) return 0;
  void *p = nullptr;
  size_t cap = 0;
  if (drain()) return -3;
  if (reserve(&p, &cap, need)) return -2;
  if (used_bytes && (hipMemcpyAsync(p, b.p, used_bytes, hipMemcpyDeviceToDevice, st) != hipSuccess ||
                     hipStreamSynchronize(st) != hipSuccess)) {
    retire(p);
    return -3;
  }
  retire(b.p);
  b.p = p;
  b.cap = cap;
  return 0;
}

// pinned scratch: the batch pipeline's Counters at 0, small read-backs at 256
constexpr size_t kPinnedBytes = 512, kPinnedU64 = 256;
uint64_t *Workspace::pinned_u64() {
  if (!host_pinned && hipHostMalloc(&host_pinned, kPinnedBytes, hipHostMallocDefault) != hipSuccess) return nullptr;
  return reinterpret_cast<uint64_t *>(reinterpret_cast<char *>(host_pinned) + kPinnedU64);
}

Workspace::~Workspace() {
  // `cur` may name a caller's stream that no longer exists: wait on our event
  if (used && last_use) (void)hipEventSynchronize(last_use);
  for (auto &b : bufs) retire(b.p);  // (hipFree would wait for a running per-publish server)
  if (last_use) (void)hipEventDestroy(last_use);
  if (host_pinned) (void)hipHostFree(host_pinned);
  for (auto &e : ev)
    if (e) (void)hipEventDestroy(e);
  if (ev_fork) (void)hipEventDestroy(ev_fork);
  if (ev_join) (void)hipEventDestroy(ev_join);
  if (side) (void)hipStreamDestroy(side);
}

static void mark(Workspace &ws, int i, hipStream_t st) {
  if (!ws.profile) return;
  if (!ws.ev[i] && hipEventCreate(&ws.ev[i]) != hipSuccess) {
    ws.profile = false;
    return;
  }
  (void)hipEventRecord(ws.ev[i], st);
}

static float elapsed(Workspace &ws, int a, int b) {
  float ms = 0;
  if (hipEventElapsedTime(&ms, ws.ev[a], ws.ev[b]) != hipSuccess) return 0;
  return ms;
}

// grid = the blocks of `kern` that fit on the device at once (cached per slot)
template <class K>
static uint32_t resident_blocks(Workspace &ws, int, K kern) {
  uint32_t &slot_v = ws.resident[reinterpret_cast<const void *>(kern)];
  if (!slot_v) {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, kBigThreads, 0) != hipSuccess || per < 1)
      per = 2, cus = 256;
    slot_v = (uint32_t)(per * cus);
  }
  return slot_v;
}

// ---------------------------------------------------------------------------
// Launch guard (host side, before every launch that takes an Outputs): every
// array the kernel reads or writes is set, and the workspace buffer behind it
// holds what the kernel indexes for n topics.  A miss returns -1 (MQM_EINVAL)
// and names the kernel and the array — never a launch with a null or short
// array (round 4's r04x fault: k_ident read record headers through a null
// nsolo / mcount / hcount that its launch site had not set).
// ---------------------------------------------------------------------------
enum : uint32_t {
  kOHCount = 1u << 0, kODCount = 1u << 1, kOMCount = 1u << 2, kOSCount = 1u << 3, kONSolo = 1u << 4,
  kODStart = 1u << 5, kOHStart = 1u << 6, kOCls = 1u << 7, kODfsList = 1u << 8, kORecs = 1u << 9,
  kOCtr = 1u << 10, kODOut = 1u << 11, kOHOut = 1u << 12, kOICount = 1u << 13, kOIStart = 1u << 14,
  kOIOut = 1u << 15,
};
// what each kernel family touches (match.hip bodies and the helpers they call)
constexpr uint32_t kNeedWalk = kOHCount | kODCount | kOMCount | kOSCount | kONSolo | kOCls | kODfsList | kORecs | kOCtr;
constexpr uint32_t kNeedMerge = kODCount | kOMCount | kODStart | kORecs | kOCtr | kODOut;
constexpr uint32_t kNeedDesc = kODCount | kOMCount | kOSCount | kONSolo | kODStart | kOCls | kORecs | kOCtr;
constexpr uint32_t kNeedShared = kOHCount | kOHStart | kORecs | kOCtr | kOHOut;
constexpr uint32_t kNeedDfs = kOHCount | kODCount | kODStart | kOHStart | kODfsList | kOCtr | kODOut | kOHOut;
constexpr uint32_t kNeedRuns = kOCls | kORecs | kOCtr;
constexpr uint32_t kNeedIdentIn = kOMCount | kOCls | kORecs | kOCtr | kODfsList;
constexpr uint32_t kNeedIdent = kNeedIdentIn | kOICount | kOIStart;

static int guard_outputs(const Workspace &ws, const Outputs &o, uint32_t need, uint32_t n, const char *kernel) {
  const uint64_t n1 = (uint64_t)n + 1;
  struct F {
    uint32_t bit;
    const void *p;
    uint64_t bytes;
    const char *name;
  } f[] = {{kOHCount, o.hcount, 4 * (uint64_t)n, "hcount"},
           {kODCount, o.dcount, 4 * (uint64_t)n, "dcount"},
           {kOMCount, o.mcount, 4 * (uint64_t)n, "mcount"},
           {kOSCount, o.scount, 4 * (uint64_t)n, "scount"},
           {kONSolo, o.nsolo, 4 * (uint64_t)n, "nsolo"},
           {kODStart, o.dstart, 8 * n1, "dstart"},
           {kOHStart, o.hstart, 8 * n1, "hstart"},
           {kOCls, o.cls, (uint64_t)n, "cls"},
           {kODfsList, o.dfs_list, 4 * (uint64_t)std::min<uint64_t>(o.dfs_cap, n1), "dfs_list"},  // (k_dfs reads min(n_dfs, dfs_cap))
           {kORecs, o.recs, 4 * (uint64_t)kRecStrideAlloc * n, "recs"},
           {kOCtr, o.ctr, sizeof(Counters), "ctr"},
           {kODOut, o.dout, 4 * o.dcap, "dout"},
           {kOHOut, o.hout, 4 * o.hcap, "hout"},
           {kOICount, o.icount, 4 * (uint64_t)n, "icount"},
           {kOIStart, o.istart, 8 * n1, "istart"},
           {kOIOut, o.iout, 0, "iout"}};
  for (const F &x : f) {
    if (!(need & x.bit)) continue;
    if (!x.p) {
      fprintf(stderr, "mqmatch: %s not launched: Outputs::%s is not set\n", kernel, x.name);
      return -1;
    }
    for (const auto &b : ws.bufs)  // an array the workspace owns must hold what the kernel indexes
      if (b.p == x.p && b.cap < x.bytes) {
        fprintf(stderr, "mqmatch: %s not launched: Outputs::%s holds %zu B, the launch indexes %llu B\n", kernel,
                x.name, b.cap, (unsigned long long)x.bytes);
        return -1;
      }
  }
  return 0;
}
#define GUARD(o, need, n, kernel)                                   \
  do {                                                              \
    if (guard_outputs(ws, (o), (need), (n), (kernel)) != 0) return -1; \
  } while (0)

// counts (n) -> exclusive offsets (u64, n + 1).  u32 counts are widened on
// the fly: hipCUB accumulates in the input type, and a batch's raw entries can
// pass 2^32 (config 4 shards gather ~6.8G per 10M topics)
struct Widen {
  __host__ __device__ uint64_t operator()(uint32_t c) const { return c; }
};
template <class T>
static int scan_offsets_it(Workspace &ws, T counts, uint64_t *offs, uint32_t n, hipStream_t st,
                           Workspace::Slot tmp_slot = Workspace::kScanTmp);
static int scan_offsets(Workspace &ws, const uint32_t *counts, uint64_t *offs, uint32_t n, hipStream_t st,
                        Workspace::Slot tmp_slot = Workspace::kScanTmp) {
  return scan_offsets_it(ws, hipcub::TransformInputIterator<uint64_t, Widen, const uint32_t *>(counts, Widen{}), offs,
                         n, st, tmp_slot);
}
template <class T>
static int scan_offsets_it(Workspace &ws, T counts, uint64_t *offs, uint32_t n, hipStream_t st,
                           Workspace::Slot tmp_slot) {
  static_assert(sizeof(typename std::iterator_traits<T>::value_type) == 8, "64-bit accumulation");
  HIP_TRY(hipMemsetAsync(offs, 0, sizeof(uint64_t), st));
  if (n == 0) return 0;
  size_t tmp = 0;
  HIP_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, tmp, counts, offs + 1, n, st));
  if (ws.get(tmp_slot, tmp)) return -2;
  HIP_TRY(hipcub::DeviceScan::InclusiveSum(ws.ptr(tmp_slot), tmp, counts, offs + 1, n, st));
  return 0;
}

// ---------------------------------------------------------------------------
// One batch = match_enqueue (every launch of the pipeline, queued on st) +
// match_collect (wait, read the counters back once).
//   exact  : the first call of a workspace (or after an overflow): one
//            read-back after the walk and the scans sizes every output buffer
//            and picks the merge kernels that have work (and one more for the
//            DFS tails when a topic took that path);
//   queued : every later call: no read-back before the end — the output
//            buffers are the ones earlier calls sized, every kernel reads its
//            count from the device (an empty list costs an empty launch), and
//            every store is checked against its buffer; a call that needed
//            more reports it (Counters::oob / cap_ovf and the sizes it needed)
//            and match_device runs it again, exact.  So consecutive batches
//            queue back to back on a stream, on several streams at once
//            (one workspace each), with no host round trip in between.
// ---------------------------------------------------------------------------
static Counters *pinned_counters(Workspace &ws) {
  if (!ws.pinned_u64()) return nullptr;
  static_assert(sizeof(Counters) <= kPinnedU64, "pinned layout");
  return reinterpret_cast<Counters *>(ws.host_pinned);
}

// The identifiers pass beside the match (Workspace::ident_early): forked
// from `st` after the walk onto ws.side — the walk's records, classes and
// multi counts are final then, and the merges and the solo copy only read
// them — and joined back before the call's read-back (match_enqueue).  Sized
// from the last call's multi entries; a scratch area or list past that
// capacity sets the flag the collect reads, and identifiers_device runs the
// pass again after the match.  Pinned read-backs: total listed, overflow
// flag, total multi entries (hp[8..10]).
static int ident_launch(const DeviceSnapshot &s, Workspace &ws, Outputs o, uint32_t n, hipStream_t st) {
  using W = Workspace;
  if (!ws.side) {
    if (hipStreamCreateWithFlags(&ws.side, hipStreamNonBlocking) != hipSuccess) {
      ws.side = nullptr;
      return -3;
    }
    if (hipEventCreateWithFlags(&ws.ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ws.ev_join, hipEventDisableTiming) != hipSuccess)
      return -3;
  }
  uint64_t *hp = ws.pinned_u64();
  if (!hp) return -2;
  const uint64_t cap = std::max<uint64_t>(ws.ident_cap, 4ull * n + 4096);
  size_t tmp = 0;
  {
    hipcub::TransformInputIterator<uint64_t, Widen, const uint32_t *> it(o.mcount, Widen{});
    HIP_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, tmp, it, (uint64_t *)nullptr, (int)std::max<uint32_t>(n, 1), st));
  }
  // (every buffer sized on the host before the fork: a growth waits for this
  // workspace's queued work, which must not include the side stream's)
  if (ws.get(W::kIMStart, sizeof(uint64_t) * (n + 1)) || ws.get(W::kICount, sizeof(uint32_t) * (n + 1)) ||
      ws.get(W::kIStart, sizeof(uint64_t) * (n + 2)) || ws.get(W::kIScratch, sizeof(uint32_t) * (cap + 1)) ||
      ws.get(W::kIOut, sizeof(uint32_t) * (cap + 1)) || ws.get(W::kScanTmp2, tmp + 16))
    return -2;
  uint64_t *mstart = (uint64_t *)ws.ptr(W::kIMStart);
  uint32_t *scratch = (uint32_t *)ws.ptr(W::kIScratch);
  o.icount = (uint32_t *)ws.ptr(W::kICount);
  o.istart = (uint64_t *)ws.ptr(W::kIStart);
  o.iout = (uint32_t *)ws.ptr(W::kIOut);
  GUARD(o, kNeedIdent | kOIOut, n, "k_ident (early)");
  unsigned long long *ovf = (unsigned long long *)(o.istart + n + 1);
  HIP_TRY(hipEventRecord(ws.ev_fork, st));
  HIP_TRY(hipStreamWaitEvent(ws.side, ws.ev_fork, 0));
  hipStream_t sd = ws.side;
  const int rc = [&]() -> int {  // (work is queued on the side stream from here on)
    HIP_TRY(hipMemsetAsync(ovf, 0, sizeof(uint64_t), sd));
    if (scan_offsets(ws, o.mcount, mstart, n, sd, W::kScanTmp2)) return -3;
    const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>((n + 31) / 32, 8192));
    if (n > 0) {
      hipLaunchKernelGGL(k_ident, dim3(blocks), dim3(256), 0, sd, s, o, n, mstart, scratch, cap, ovf);
      HIP_TRY(hipGetLastError());
    }
    if (scan_offsets(ws, o.icount, o.istart, n, sd, W::kScanTmp2)) return -3;
    if (n > 0) {
      hipLaunchKernelGGL(k_ident_pack, dim3(std::max<uint32_t>(1, std::min<uint32_t>((n + 255) / 256, 16384))),
                         dim3(256), 0, sd, o, n, mstart, scratch, cap, ovf);
      HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipMemcpyAsync(hp + 8, o.istart + n, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, sd));
    HIP_TRY(hipMemcpyAsync(hp + 10, mstart + n, sizeof(uint64_t), hipMemcpyDeviceToHost, sd));
    return 0;
  }();
  // joined in every case: after a failure part-way the side stream may still
  // write kICount / kIStart / kIOut, which the fallback pass after the match
  // (identifiers_device on `st`) writes too
  const hipError_t je = hipEventRecord(ws.ev_join, sd);
  if (rc != 0) {
    if (je == hipSuccess) (void)hipStreamWaitEvent(st, ws.ev_join, 0);
    else (void)hipStreamSynchronize(sd);
    return rc;
  }
  return je == hipSuccess ? 0 : -3;
}

// MQM_IDENT_FUSED=0: Identifiers by the separate pass beside the match
// (ident_launch, round 5) instead of listed by the merges
static bool ident_fused_on() {
  static const bool v = !getenv("MQM_IDENT_FUSED") || atoi(getenv("MQM_IDENT_FUSED")) != 0;
  return v;
}

int match_enqueue(const DeviceSnapshot &s, Workspace &ws, const uint8_t *d_bytes, const uint64_t *d_offs, uint32_t n,
                  hipStream_t st, bool exact) {
  using W = Workspace;
  if (ws.pending) return -1;  // one call in flight per workspace (collect it first)
  const bool fuse_ids = ws.ident_early && !ws.runs && ident_fused_on();
  // queued calls need every output buffer sized by an earlier call (the
  // Identifiers scratch included: its first call reads the multi-entry total back)
  exact = exact || !ws.caps_known || (fuse_ids && ws.ident_cap == 0);
  if (ws.get(W::kSCount, sizeof(uint32_t) * (n + 1)) || ws.get(W::kHCount, sizeof(uint32_t) * (n + 1)) ||
      ws.get(W::kDCount, sizeof(uint32_t) * (n + 1)) || ws.get(W::kDStart, sizeof(uint64_t) * (n + 1)) ||
      ws.get(W::kHStart, sizeof(uint64_t) * (n + 1)) || ws.get(W::kCls, n + 1) ||
      ws.get(W::kDfsList, sizeof(uint32_t) * (n + 2)) || ws.get(W::kMCount, sizeof(uint32_t) * (n + 1)) ||
      ws.get(W::kRecs, sizeof(uint32_t) * kRecStrideAlloc * ((uint64_t)n + 1)) || ws.get(W::kCounters, 256) ||
      ws.get(W::kNSolo, sizeof(uint32_t) * (n + 1)) || ws.get(W::kDescStart, sizeof(uint64_t) * (n + 1)))
    return -2;
  Counters *hc = pinned_counters(ws);
  if (!hc) return -2;

  Outputs o{};
  o.scount = (uint32_t *)ws.ptr(W::kSCount);
  o.hcount = (uint32_t *)ws.ptr(W::kHCount);
  o.dcount = (uint32_t *)ws.ptr(W::kDCount);
  o.dstart = (uint64_t *)ws.ptr(W::kDStart);
  o.hstart = (uint64_t *)ws.ptr(W::kHStart);
  o.cls = (uint8_t *)ws.ptr(W::kCls);
  o.dfs_list = (uint32_t *)ws.ptr(W::kDfsList);
  o.mcount = (uint32_t *)ws.ptr(W::kMCount);
  o.recs = (uint32_t *)ws.ptr(W::kRecs);
  o.ctr = (Counters *)ws.ptr(W::kCounters);
  o.nsolo = (uint32_t *)ws.ptr(W::kNSolo);
  o.runs = ws.runs ? 1u : 0u;
  auto *desc_start = (uint64_t *)ws.ptr(W::kDescStart);
  HIP_TRY(hipMemsetAsync(o.ctr, 0, sizeof(Counters), st));
  mark(ws, 0, st);
  o.dfs_cap = n + 1;  // (the walk lists DFS topics in dfs_list, one per topic at most)
  GUARD(o, kNeedWalk, n, "k_walk");
  if (n > 0) {
    constexpr uint32_t per_block = kWalkWaves * (kWave / kWalkG);
    const uint32_t blocks = std::max<uint32_t>(
        1, std::min<uint32_t>((n + per_block - 1) / per_block, resident_blocks(ws, 0, k_walk<kWalkG>)));
    // topics handed out 4 steps (64 topics) at a time from a device counter:
    // C3 walk 5.76 -> 5.19 ms, C4 shard 6.22 -> 5.57 (r04an, r04ao; 16 at a
    // time 5.37, 1 at a time 7.53: the counter's atomics serialise); the fixed
    // stride for batches whose counter could pass 2^32
    // (MQM_SLOTS=1: the walk over paired node slots; measured slower, r05d: see DESIGN §3)
    if (n >= (1u << 31))
      hipLaunchKernelGGL(k_walk<kWalkG>, dim3(blocks), dim3(kWave * kWalkWaves), 0, st, s, d_bytes, d_offs, n, o);
    else if (walk_slots() && s.slots)
      hipLaunchKernelGGL((k_walk<kWalkG, 4>), dim3(blocks), dim3(kWave * kWalkWaves), 0, st, s, d_bytes, d_offs, n, o);
    else
      hipLaunchKernelGGL((k_walk<kWalkG, 4, false>), dim3(blocks), dim3(kWave * kWalkWaves), 0, st, s, d_bytes, d_offs,
                         n, o);
  }
  HIP_TRY(hipGetLastError());
  mark(ws, 1, st);
  ws.ident_ready = false;
  ws.ident_fused = false;
  if (fuse_ids) {
    // Identifiers listed by the merges: every count starts at 0 (topics
    // without multi entries, DFS topics), each topic's scratch area at the
    // scan of the multi counts; its extent comes back with the exact
    // read-back below and sizes the scratch
    if (ws.get(W::kIMStart, sizeof(uint64_t) * (n + 1)) || ws.get(W::kICount, sizeof(uint32_t) * (n + 1)))
      return -2;
    o.imstart = (uint64_t *)ws.ptr(W::kIMStart);
    o.icount = (uint32_t *)ws.ptr(W::kICount);
    HIP_TRY(hipMemsetAsync(o.icount, 0, sizeof(uint32_t) * (n + 1), st));
    if (scan_offsets(ws, o.mcount, o.imstart, n, st)) return -3;
    HIP_TRY(hipMemcpyAsync(&o.ctr->i_multi, o.imstart + n, sizeof(uint64_t), hipMemcpyDeviceToDevice, st));
  } else if (ws.ident_early && !ws.runs && ident_launch(s, ws, o, n, st) == 0) {
    ws.ident_ready = true;
  }
  // segment starts: exclusive scans of S (raw entries, an upper bound of a
  // topic's deliveries) and H (shared candidates); the solo descriptors'
  // positions: exclusive scan of the solo-part counts
  if (scan_offsets(ws, (const uint32_t *)o.scount, o.dstart, n, st) ||
      scan_offsets(ws, (const uint32_t *)o.hcount, o.hstart, n, st) || scan_offsets(ws, o.nsolo, desc_start, n, st))
    return -3;
  // merge lists
  const W::Slot list_slots[kNLists] = {W::kListS, W::kListW, W::kListT1, W::kListT2, W::kListT3,
                                       W::kListP, W::kListH, W::kListRS, W::kListR};
  Lists lists;
  for (int l = 0; l < kNLists; l++) {
    if (ws.get(list_slots[l], sizeof(uint32_t) * (n + 1))) return -2;
    lists.l[l] = (uint32_t *)ws.ptr(list_slots[l]);
  }
  unsigned int *lcount = &o.ctr->n_small;  // kNLists consecutive counters
  if (n > 0) {
    hipLaunchKernelGGL(k_route, dim3(std::min<uint32_t>((n + 4095) / 4096, 2048)), dim3(256), 0, st, o.cls, o.mcount,
                       o.hcount, n, lists, lcount, o.ctr->m_sum, resolve_min());
    HIP_TRY(hipGetLastError());
  }
  hipLaunchKernelGGL(k_totals, dim3(1), dim3(64), 0, st, o.ctr, o.dstart, o.hstart, desc_start, n);
  HIP_TRY(hipGetLastError());
  if (exact) {  // the one read-back that sizes the outputs
    HIP_TRY(hipMemcpyAsync(hc, o.ctr, sizeof(Counters), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
  }
  // capacity of a buffer in elements (one element kept spare, as the exact sizing does)
  auto cap_of = [&](W::Slot sl, size_t elem) -> uint64_t {
    const size_t c = ws.bufs[sl].cap / elem;
    return c ? c - 1 : 0;
  };

  // DFS topics (a capacity of the walk exceeded): phase 0 counts each one's
  // raw entries, k_dfs_prep sizes their tables and tails on the device
  const bool dfs = !exact || hc->n_dfs > 0;
  const uint32_t max_levels = s.height + 1;
  const size_t fb_lds = sizeof(uint32_t) * (((max_levels + 1) & ~1u) + 4 * (2 * max_levels + 8)) +
                        sizeof(uint64_t) * 2 * max_levels;
  uint64_t *raw_cnt = nullptr, *raw_h = nullptr, *tab_off = nullptr;
  uint32_t dfs_cap = 0;
  if (dfs) {
    dfs_cap = exact ? hc->n_dfs : ws.dfs_cap;
    if (ws.get(W::kRawCnt, sizeof(uint64_t) * 2 * (dfs_cap + 1)) || ws.get(W::kTabOff, sizeof(uint64_t) * (dfs_cap + 2)))
      return -2;
    raw_cnt = (uint64_t *)ws.ptr(W::kRawCnt);
    raw_h = raw_cnt + dfs_cap + 1;
    tab_off = (uint64_t *)ws.ptr(W::kTabOff);
  }
  o.dfs_cap = dfs_cap;
  const uint32_t fb_blocks = exact ? std::max<uint32_t>(1, std::min<uint32_t>(hc->n_dfs, 4096)) : 1024;
  uint64_t dcap, hcap, desc_cap, win_cap, tab_cap = 0;
  if (exact) {
    if (dfs) {
      hipLaunchKernelGGL(k_dfs<0>, dim3(fb_blocks), dim3(kWave), fb_lds, st, s, d_bytes, d_offs, o, raw_cnt, raw_h,
                         nullptr, nullptr, max_levels);
      HIP_TRY(hipGetLastError());
      hipLaunchKernelGGL(k_dfs_prep, dim3(1), dim3(256), 0, st, o.ctr, raw_cnt, raw_h, tab_off, dfs_cap, ~0ull,
                         o.dstart + n, o.hstart + n, ~0ull, ~0ull);
      HIP_TRY(hipGetLastError());
      HIP_TRY(hipMemcpyAsync(hc, o.ctr, sizeof(Counters), hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
    }
    dcap = hc->s_total + hc->dfs_raw;
    hcap = hc->h_total + hc->dfs_h;
    desc_cap = hc->n_desc;
    win_cap = (hc->s_total + kWin - 1) / kWin;
    tab_cap = hc->tab_total;
  } else {  // what the buffers hold
    dcap = cap_of(W::kDOut, sizeof(uint32_t));
    hcap = cap_of(W::kHOut, sizeof(uint32_t));
    desc_cap = cap_of(W::kDesc, sizeof(uint4));
    win_cap = cap_of(W::kWin, sizeof(uint32_t));
    tab_cap = std::max<uint64_t>(cap_of(W::kTable, sizeof(GEnt)), 1u << 16);
  }
  if (ws.get(W::kDOut, sizeof(uint32_t) * (dcap + 1)) || ws.get(W::kHOut, sizeof(uint32_t) * (hcap + 1)) ||
      ws.get(W::kDesc, sizeof(uint4) * (desc_cap + 1)) || ws.get(W::kWin, sizeof(uint32_t) * (win_cap + 1)))
    return -2;
  if (fuse_ids) {  // the scratch and the packed list: at most one sid per multi entry
    const uint64_t icap = exact ? hc->i_multi : std::max<uint64_t>(ws.ident_cap, 4ull * n + 4096);
    if (ws.get(W::kIScratch, sizeof(uint32_t) * (icap + 1)) || ws.get(W::kIOut, sizeof(uint32_t) * (icap + 1)) ||
        ws.get(W::kIStart, sizeof(uint64_t) * (n + 2)))
      return -2;
    o.iscratch = (uint32_t *)ws.ptr(W::kIScratch);
    o.iout = (uint32_t *)ws.ptr(W::kIOut);
    o.istart = (uint64_t *)ws.ptr(W::kIStart);
    o.icap = icap;
  }
  o.dout = (uint32_t *)ws.ptr(W::kDOut);
  o.hout = (uint32_t *)ws.ptr(W::kHOut);
  o.dcap = dcap;
  o.hcap = hcap;
  // every emission kernel below (merges, solo copy, shared candidates, DFS)
  GUARD(o, kNeedMerge | kNeedDesc | kNeedShared, n, "the emission kernels");
  if (dfs) {
    Outputs od = o;
    od.dfs_cap = dfs_cap;
    GUARD(od, kNeedDfs, n, "k_dfs");
  }
  auto *desc = (uint4 *)ws.ptr(W::kDesc);
  auto *win = (uint32_t *)ws.ptr(W::kWin);
  GEnt *tab = nullptr;
  if (dfs) {
    if (ws.get(W::kTable, sizeof(GEnt) * (tab_cap + 1))) return -2;
    tab = (GEnt *)ws.ptr(W::kTable);
    if (!exact) {  // sized on the device, checked against the buffers above
      hipLaunchKernelGGL(k_dfs<0>, dim3(fb_blocks), dim3(kWave), fb_lds, st, s, d_bytes, d_offs, o, raw_cnt, raw_h,
                         nullptr, nullptr, max_levels);
      HIP_TRY(hipGetLastError());
      hipLaunchKernelGGL(k_dfs_prep, dim3(1), dim3(256), 0, st, o.ctr, raw_cnt, raw_h, tab_off, dfs_cap, tab_cap,
                         o.dstart + n, o.hstart + n, dcap, hcap);
      HIP_TRY(hipGetLastError());
    }
    hipLaunchKernelGGL(k_zero_tab, dim3(exact ? (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((tab_cap + 127) / 128, 4096))
                                              : 1024),
                       dim3(256), 0, st, reinterpret_cast<unsigned long long *>(tab), o.ctr, tab_cap);
    HIP_TRY(hipGetLastError());
  }

  mark(ws, 2, st);
  static_assert(kWave * kEmitWaves == kBigThreads, "resident_blocks assumes 256-thread blocks");
  if (n > 0) {
    // a queued call launches the merge / shared kernels of the lists the last
    // collected call had topics in (each reads its count from the device)
    uint32_t launched = 0;
    auto has_list = [&](uint32_t c, int list) {
      const bool l = exact ? c > 0 : ((ws.lists_seen >> list) & 1u) != 0;
      if (l) launched |= 1u << list;
      return l;
    };
    const bool ids = o.iscratch != nullptr;  // (the merges list Identifiers: their kIdent variants)
    const bool l_small = has_list(hc->n_small, kLSmall), l_wave = has_list(hc->n_wmerge, kLWave),
               l_t1 = has_list(hc->n_t1, kLT1), l_t2 = has_list(hc->n_t2, kLT2), l_t3 = has_list(hc->n_t3, kLT3),
               l_part = has_list(hc->n_part, kLPart), l_sh = has_list(hc->n_shlist, kLShared),
               l_rs = has_list(hc->n_res_small, kLResSmall), l_r = has_list(hc->n_res, kLRes);
    ws.pend_launched = launched;
    // persistent grids: the blocks that fit on the device at once
    auto grid = [&](auto kern) { return dim3(std::max<uint32_t>(1, resident_blocks(ws, 0, kern))); };
    // the workgroup merges first, the small-topic merges last (they fill the
    // device better at the end of the stream)
    if (l_r) {
      // 6 entries per lane in flight: C4 shard emission 20.39 ms against 21.64
      // (4, 64 VGPRs) and 21.07 (8, 86 VGPRs, 5 waves/SIMD) — r04z;
      // topics handed out 4 at a time from a device counter: C4 shard emission
      // 19.03 ms against 20.22 with a fixed stride and 19.15 with 16 (r04ae)
      if (n < (1u << 31) && ids)
        hipLaunchKernelGGL((k_resolve<kWave, kHCap, 6, 4, true>), grid((k_resolve<kWave, kHCap, 6, 4, true>)),
                           dim3(kWave * kEmitWaves), 0, st, s, o, lists.l[kLRes], lcount + kLRes);
      else if (n < (1u << 31))
        hipLaunchKernelGGL((k_resolve<kWave, kHCap, 6, 4>), grid((k_resolve<kWave, kHCap, 6, 4>)),
                           dim3(kWave * kEmitWaves), 0, st, s, o, lists.l[kLRes], lcount + kLRes);
      else if (ids)  // (the counter could pass 2^32)
        hipLaunchKernelGGL((k_resolve<kWave, kHCap, 6, 0, true>), grid((k_resolve<kWave, kHCap, 6, 0, true>)),
                           dim3(kWave * kEmitWaves), 0, st, s, o, lists.l[kLRes], lcount + kLRes);
      else
        hipLaunchKernelGGL((k_resolve<kWave, kHCap, 6>), grid((k_resolve<kWave, kHCap, 6>)),
                           dim3(kWave * kEmitWaves), 0, st, s, o, lists.l[kLRes], lcount + kLRes);
      HIP_TRY(hipGetLastError());
    }
    if (l_t1) {
      hipLaunchKernelGGL(k_multi<1024>, grid(k_multi<1024>), dim3(kBigThreads), 0, st, s, o, lists.l[kLT1],
                         lcount + kLT1);
      HIP_TRY(hipGetLastError());
    }
    if (l_t2) {
      hipLaunchKernelGGL(k_multi<2048>, grid(k_multi<2048>), dim3(kBigThreads), 0, st, s, o, lists.l[kLT2],
                         lcount + kLT2);
      HIP_TRY(hipGetLastError());
    }
    if (l_t3) {
      hipLaunchKernelGGL(k_multi<4096>, grid(k_multi<4096>), dim3(kBigThreads), 0, st, s, o, lists.l[kLT3],
                         lcount + kLT3);
      HIP_TRY(hipGetLastError());
    }
    if (l_part) {
      hipLaunchKernelGGL(k_multi_part, grid(k_multi_part), dim3(kBigThreads), 0, st, s, o, lists.l[kLPart],
                         lcount + kLPart);
      HIP_TRY(hipGetLastError());
    }
    if (l_rs) {
      if (ids)
        hipLaunchKernelGGL((k_resolve<kSmallLanes, 16, 3, 0, true>), grid((k_resolve<kSmallLanes, 16, 3, 0, true>)),
                           dim3(kWave * kEmitWaves), 0, st, s, o, lists.l[kLResSmall], lcount + kLResSmall);
      else
        hipLaunchKernelGGL((k_resolve<kSmallLanes, 16, 3>), grid((k_resolve<kSmallLanes, 16, 3>)),
                           dim3(kWave * kEmitWaves), 0, st, s, o, lists.l[kLResSmall], lcount + kLResSmall);
      HIP_TRY(hipGetLastError());
    }
    if (l_small) {
      if (ids)
        hipLaunchKernelGGL((k_merge_small<6, true>), grid(k_merge_small<6, true>), dim3(kWave * kEmitWaves), 0, st, s,
                           o, lists.l[kLSmall], lcount + kLSmall);
      else
        hipLaunchKernelGGL((k_merge_small<6>), grid(k_merge_small<6>), dim3(kWave * kEmitWaves), 0, st, s, o,
                           lists.l[kLSmall], lcount + kLSmall);
      HIP_TRY(hipGetLastError());
    }
    if (l_wave) {
      if (ids)
        hipLaunchKernelGGL(k_merge<true>, grid(k_merge<true>), dim3(kWave * kEmitWaves), 0, st, s, o, lists.l[kLWave],
                           lcount + kLWave);
      else
        hipLaunchKernelGGL(k_merge<false>, grid(k_merge<false>), dim3(kWave * kEmitWaves), 0, st, s, o,
                           lists.l[kLWave], lcount + kLWave);
      HIP_TRY(hipGetLastError());
    }
    // the solo copy (none in the runs form: the solo parts stay runs)
    if (!ws.runs) {
      const uint32_t long_min = long_part_min();
      const bool desc_copy = desc_copy_on();
      if (desc_copy)  // (A/B: the parts copied by k_desc itself; no window copy below)
        hipLaunchKernelGGL(k_desc<true>, dim3(std::min<uint32_t>((n + 255) / 256, 8192)), dim3(256), 0, st, s, o, n,
                           desc_start, desc, desc_cap, 0xFFFFFFFFu);
      else
        hipLaunchKernelGGL(k_desc<false>, dim3(std::min<uint32_t>((n + 255) / 256, 8192)), dim3(256), 0, st, s, o, n,
                           desc_start, desc, desc_cap, long_min);  // a wavefront per 64 topics
      HIP_TRY(hipGetLastError());
      // the long parts (flagged descriptors, 16-B moves) before the window copy of the rest
      if (!desc_copy && long_min != 0xFFFFFFFFu) {
        hipLaunchKernelGGL(k_longcopy, grid(k_longcopy), dim3(kWave * kEmitWaves), 0, st, s, desc, desc_start + n,
                           desc_cap, o.dout, o.dcap, &o.ctr->oob);
        HIP_TRY(hipGetLastError());
      }
      if (!desc_copy && (!exact || hc->n_desc > 0)) {
        const uint64_t nd_grid = exact ? hc->n_desc : desc_cap;
        hipLaunchKernelGGL(k_winmap,
                           dim3((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((nd_grid + 255) / 256, 8192))),
                           dim3(256), 0, st, desc, desc_start + n, desc_cap, o.dstart + n, win, win_cap, &o.ctr->oob);
        HIP_TRY(hipGetLastError());
        if (wincopy_vec())
          hipLaunchKernelGGL(k_wincopy<true>, grid(k_wincopy<true>), dim3(kWave * kEmitWaves), 0, st, s, desc,
                             desc_start + n, desc_cap, win, win_cap, o.dstart + n, o.dout, o.dcap, &o.ctr->oob);
        else if (nt_store())
          hipLaunchKernelGGL((k_wincopy<false, true>), grid(k_wincopy<false, true>), dim3(kWave * kEmitWaves), 0, st,
                             s, desc, desc_start + n, desc_cap, win, win_cap, o.dstart + n, o.dout, o.dcap,
                             &o.ctr->oob);
        else
          hipLaunchKernelGGL(k_wincopy<false>, grid(k_wincopy<false>), dim3(kWave * kEmitWaves), 0, st, s, desc,
                             desc_start + n, desc_cap, win, win_cap, o.dstart + n, o.dout, o.dcap, &o.ctr->oob);
        HIP_TRY(hipGetLastError());
      }
    }
    if (l_sh) {
      const uint32_t nsh = exact ? hc->n_shlist : n;
      hipLaunchKernelGGL(k_shared, dim3(std::min<uint32_t>((nsh + 15) / 16, 8192)), dim3(256), 0, st, o,
                         lists.l[kLShared], lcount + kLShared);
      HIP_TRY(hipGetLastError());
    }
  }
  if (dfs) {
    hipLaunchKernelGGL(k_dfs<1>, dim3(fb_blocks), dim3(kWave), fb_lds, st, s, d_bytes, d_offs, o, raw_cnt, raw_h,
                       tab_off, tab, max_levels);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_dfs<2>, dim3(fb_blocks), dim3(kWave), fb_lds, st, s, d_bytes, d_offs, o, raw_cnt, raw_h,
                       tab_off, tab, max_levels);
    HIP_TRY(hipGetLastError());
  }
  if (fuse_ids) {  // the merges' lists, packed in topic order (DFS topics: identifiers_device)
    if (scan_offsets(ws, o.icount, o.istart, n, st)) return -3;
    if (n > 0) {
      hipLaunchKernelGGL(k_ident_pack, dim3(std::max<uint32_t>(1, std::min<uint32_t>((n + 255) / 256, 16384))),
                         dim3(256), 0, st, o, n, o.imstart, o.iscratch, o.icap, &o.ctr->i_ovf);
      HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipMemcpyAsync(&o.ctr->i_total, o.istart + n, sizeof(uint64_t), hipMemcpyDeviceToDevice, st));
    ws.ident_fused = true;
  }
  mark(ws, 3, st);
  // the identifiers pass beside the match: joined here, so the read-back's
  // synchronisation covers it (and the next call's buffers wait for it)
  if (ws.ident_ready) HIP_TRY(hipStreamWaitEvent(st, ws.ev_join, 0));
  // totals for the caller: sums of the counts, then the one read-back
  {
    size_t tmp = 0;
    hipcub::TransformInputIterator<uint64_t, Widen, const uint32_t *> dc(o.dcount, Widen{}), hc_it(o.hcount, Widen{});
    HIP_TRY(hipcub::DeviceReduce::Sum(nullptr, tmp, dc, &o.ctr->d_sum, n, st));
    if (ws.get(W::kScanTmp, tmp)) return -2;
    HIP_TRY(hipcub::DeviceReduce::Sum(ws.ptr(W::kScanTmp), tmp, dc, &o.ctr->d_sum, n, st));
    HIP_TRY(hipcub::DeviceReduce::Sum(ws.ptr(W::kScanTmp), tmp, hc_it, &o.ctr->h_sum, n, st));
    HIP_TRY(hipMemcpyAsync(hc, o.ctr, sizeof(Counters), hipMemcpyDeviceToHost, st));
  }
  ws.last_valid = false;  // until collected
  ws.last_n = n;
  ws.last_bytes = d_bytes;
  ws.last_offs = d_offs;
  ws.last_runs = ws.runs;
  ws.pend_exact = exact;
  ws.pending = true;
  return 0;
}

int match_collect(Workspace &ws, hipStream_t st, MatchOutput *out) {
  using W = Workspace;
  if (!ws.pending) return -1;
  ws.pending = false;
  HIP_TRY(hipStreamSynchronize(st));
  Counters *hc = pinned_counters(ws);
  const uint32_t n = ws.last_n;
  // the next queued call's DFS capacity: what this one needed, with room
  ws.dfs_cap = std::max<uint32_t>(ws.dfs_cap, std::max<uint32_t>(1024, hc->n_dfs + hc->n_dfs / 4));
  if (hc->oob || hc->cap_ovf) {
    if (ws.pend_exact) {  // sized exactly from this call's own counts: never expected
      fprintf(stderr, "mqmatch: an output store fell outside its buffer (batch rejected; oob %#x, cap_ovf %u)\n",
              hc->oob, hc->cap_ovf);
      return -3;
    }
    return 1;  // outgrew buffers sized by an earlier call: match_device re-runs it, exact
  }
  {
    uint32_t seen = 0;
    const unsigned int c[][2] = {{hc->n_small, kLSmall}, {hc->n_wmerge, kLWave},     {hc->n_t1, kLT1},
                                 {hc->n_t2, kLT2},       {hc->n_t3, kLT3},         {hc->n_part, kLPart},
                                 {hc->n_shlist, kLShared}, {hc->n_res_small, kLResSmall}, {hc->n_res, kLRes}};
    for (const auto &x : c)
      if (x[0]) seen |= 1u << x[1];
    const bool missed = (seen & ~ws.pend_launched) != 0;
    ws.lists_seen = seen;
    if (missed) {  // a queued call had topics in a list whose kernel it did not launch
      if (ws.pend_exact) return -3;
      return 1;
    }
  }
  ws.caps_known = true;
  ws.last_valid = true;
  ws.last_n_dfs = hc->n_dfs;
  if (ws.ident_fused)  // (the next queued call's Identifiers scratch: this one's multi entries, with room)
    ws.ident_cap = std::max<uint64_t>(ws.ident_cap, hc->i_multi + hc->i_multi / 4 + 1024);
  for (int i = 0; i < 5; i++) ws.why[i] = hc->why[i];
#if MQM_WALK_STATS
  fprintf(stderr, "[walk-stats] topics %u literal probes %llu missed %llu wildcard-child loads %llu\n", n,
          hc->st_probe, hc->st_miss, hc->st_desc);
#endif
  if (ws.profile) {
    ws.prof_calls++;
    ws.prof_fallback_topics += hc->n_dfs;
    ws.prof_walk_ms += elapsed(ws, 0, 1);
    ws.prof_dedupe_ms += elapsed(ws, 2, 3);
    ws.prof_total_ms += elapsed(ws, 0, 3);
  }
  out->n_topics = n;
  out->n_deliveries = hc->d_sum;
  out->n_shared = hc->h_sum;
  out->n_big = hc->n_t1 + hc->n_t2 + hc->n_t3 + hc->n_part;
  out->n_tier2 = hc->n_t2;
  out->n_tier3 = hc->n_t3 + hc->n_part;
  for (int i = 0; i < 3; i++) out->multi_entries[i] = hc->m_sum[i];
  out->n_part = hc->n_part;
  out->n_resolve = hc->n_res_small + hc->n_res;
  out->n_solo = hc->n_solo;
  out->n_merge_small = hc->n_small;
  out->n_merge_wave = hc->n_wmerge;
  out->n_solo_ranges = hc->n_desc;
  out->n_fallback = hc->n_dfs;
  out->starts = (const uint64_t *)ws.ptr(W::kDStart);
  out->counts = (const uint32_t *)ws.ptr(W::kDCount);
  out->deliveries = (const uint32_t *)ws.ptr(W::kDOut);
  out->shared_starts = (const uint64_t *)ws.ptr(W::kHStart);
  out->shared_counts = (const uint32_t *)ws.ptr(W::kHCount);
  out->shared = (const uint32_t *)ws.ptr(W::kHOut);
  out->exact = ws.pend_exact;
  return 0;
}

int match_device(const DeviceSnapshot &s, Workspace &ws, const uint8_t *d_bytes, const uint64_t *d_offs,
                 uint32_t n, hipStream_t st, MatchOutput *out) {
  int rc = match_enqueue(s, ws, d_bytes, d_offs, n, st, false);
  if (rc == 0) rc = match_collect(ws, st, out);
  if (rc == 1) {  // a queued call outgrew its buffers: again, sized exactly
    rc = match_enqueue(s, ws, d_bytes, d_offs, n, st, true);
    if (rc == 0) rc = match_collect(ws, st, out);
    if (rc == 0) ws.requeued++;
  }
  return rc;
}

int runs_device(Workspace &ws, hipStream_t st, const MatchOutput &m, RunsOutput *out) {
  using W = Workspace;
  const uint32_t n = ws.last_n;
  if (!ws.last_valid || !ws.last_runs) return -1;
  if (ws.get(W::kRunCount, sizeof(uint32_t) * (n + 1)) || ws.get(W::kRunOffs, sizeof(uint64_t) * (n + 1)) ||
      ws.get(W::kRuns, sizeof(uint2) * (m.n_solo_ranges + 1)))
    return -2;
  Outputs o{};
  o.cls = (uint8_t *)ws.ptr(W::kCls);
  o.recs = (uint32_t *)ws.ptr(W::kRecs);
  o.ctr = (Counters *)ws.ptr(W::kCounters);
  auto *nrun = (uint32_t *)ws.ptr(W::kRunCount);
  auto *roff = (uint64_t *)ws.ptr(W::kRunOffs);
  auto *runs = (uint2 *)ws.ptr(W::kRuns);
  GUARD(o, kNeedRuns, n, "k_run_count / k_run_copy");
  if (!nrun || !roff || !runs) return -1;
  if (n > 0) {
    hipLaunchKernelGGL(k_run_count, dim3(std::min<uint32_t>((n + 255) / 256, 8192)), dim3(256), 0, st, o, n, nrun);
    HIP_TRY(hipGetLastError());
  }
  if (scan_offsets(ws, nrun, roff, n, st)) return -3;
  if (n > 0) {
    // (the walk counted these parts: Counters::n_desc; a mismatch is a checked store)
    hipLaunchKernelGGL(k_run_copy, dim3(std::min<uint32_t>((n + 31) / 32, 8192)), dim3(256), 0, st, o, n, roff, runs,
                       (uint64_t)m.n_solo_ranges);
    HIP_TRY(hipGetLastError());
  }
  out->n_topics = n;
  out->n_runs = m.n_solo_ranges;
  out->offsets = roff;
  out->runs = runs;
  out->solo_counts = (const uint32_t *)ws.ptr(W::kSCount);
  return 0;
}

int identifiers_device(const DeviceSnapshot &s, Workspace &ws, hipStream_t st, IdentOutput *out) {
  using W = Workspace;
  const uint32_t n = ws.last_n;
  if (!ws.last_valid) return -1;
  if (ws.ident_fused) {  // listed by the merges (the collect synchronised the call)
    ws.ident_fused = false;
    const Counters *hc = pinned_counters(ws);
    if (!hc) return -2;
    ws.ident_cap = std::max<uint64_t>(ws.ident_cap, hc->i_multi + hc->i_multi / 4 + 1024);
    if (!hc->i_ovf && ws.last_n_dfs == 0 && !ws.last_runs) {
      out->n_topics = n;
      out->n_idents = hc->i_total;
      out->offsets = (const uint64_t *)ws.ptr(W::kIStart);
      out->sids = (const uint32_t *)ws.ptr(W::kIOut);
      return 0;
    }
    // (a capacity passed, or DFS topics, whose sids k_dfs<3|4> list: the pass below)
  }
  if (ws.ident_ready) {  // computed beside the match (ident_launch; the collect synchronised the join)
    ws.ident_ready = false;
    const uint64_t *hp = ws.pinned_u64();
    const uint64_t total = hp[8], ovf = hp[9], n_multi = hp[10];
    ws.ident_cap = std::max<uint64_t>(ws.ident_cap, n_multi + n_multi / 4 + 1024);
    if (!ovf && ws.last_n_dfs == 0 && !ws.last_runs) {
      out->n_topics = n;
      out->n_idents = total;
      out->offsets = (const uint64_t *)ws.ptr(W::kIStart);
      out->sids = (const uint32_t *)ws.ptr(W::kIOut);
      return 0;
    }
    // (a capacity passed, or DFS topics, whose sids k_dfs<3|4> list: the pass again, below)
  }
  Outputs o{};
  o.cls = (uint8_t *)ws.ptr(W::kCls);
  o.recs = (uint32_t *)ws.ptr(W::kRecs);
  o.dfs_list = (uint32_t *)ws.ptr(W::kDfsList);
  o.dfs_cap = ws.last_n_dfs;  // the whole list (phases 3 / 4 keep no per-topic arrays)
  o.ctr = (Counters *)ws.ptr(W::kCounters);
  o.mcount = (uint32_t *)ws.ptr(W::kMCount);  // (k_ident: the topics with multi parts, k_walk)
  o.runs = ws.last_runs ? 1u : 0u;
  GUARD(o, kNeedIdentIn, n, "k_ident");  // the last match's arrays, before anything is allocated
  if (ws.get(W::kICount, sizeof(uint32_t) * (n + 1)) || ws.get(W::kIStart, sizeof(uint64_t) * (n + 1))) return -2;
  o.icount = (uint32_t *)ws.ptr(W::kICount);
  o.istart = (uint64_t *)ws.ptr(W::kIStart);
  GUARD(o, kNeedIdent, n, "k_ident");
  const uint32_t max_levels = s.height + 1;
  const size_t fb_lds = sizeof(uint32_t) * (((max_levels + 1) & ~1u) + 4 * (2 * max_levels + 8)) +
                        sizeof(uint64_t) * 2 * max_levels;
  const uint32_t fb_blocks = std::max<uint32_t>(1, std::min<uint32_t>(ws.last_n_dfs, 4096));
  const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>((n + 31) / 32, 8192));  // 32 topics per block
  // the topics' scratch areas: the scan of their multi-entry counts
  if (ws.get(W::kIMStart, sizeof(uint64_t) * (n + 1))) return -2;
  uint64_t *mstart = (uint64_t *)ws.ptr(W::kIMStart);
  if (scan_offsets(ws, o.mcount, mstart, n, st)) return -3;
  uint64_t *hp = ws.pinned_u64();
  if (!hp) return -2;
  HIP_TRY(hipMemcpyAsync(hp, mstart + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  const uint64_t n_multi = hp[0];
  if (ws.get(W::kIScratch, sizeof(uint32_t) * (n_multi + 1))) return -2;
  uint32_t *scratch = (uint32_t *)ws.ptr(W::kIScratch);
  if (n > 0) {
    hipLaunchKernelGGL(k_ident, dim3(blocks), dim3(256), 0, st, s, o, n, mstart, scratch, ~0ull,
                       (unsigned long long *)nullptr);
    HIP_TRY(hipGetLastError());
    if (ws.last_n_dfs) {
      hipLaunchKernelGGL(k_dfs<3>, dim3(fb_blocks), dim3(kWave), fb_lds, st, s, ws.last_bytes, ws.last_offs, o,
                         nullptr, nullptr, nullptr, nullptr, max_levels);
      HIP_TRY(hipGetLastError());
    }
  }
  if (scan_offsets(ws, o.icount, o.istart, n, st)) return -3;
  HIP_TRY(hipMemcpyAsync(hp, o.istart + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  const uint64_t total = hp[0];
  if (ws.get(W::kIOut, sizeof(uint32_t) * (total + 1))) return -2;
  o.iout = (uint32_t *)ws.ptr(W::kIOut);
  GUARD(o, kNeedIdent | kOIOut, n, "k_ident_pack");
  if (n > 0 && total > 0) {
    hipLaunchKernelGGL(k_ident_pack, dim3(std::max<uint32_t>(1, std::min<uint32_t>((n + 255) / 256, 16384))), dim3(256),
                       0, st, o, n, mstart, scratch, total, (unsigned long long *)nullptr);
    HIP_TRY(hipGetLastError());
    if (ws.last_n_dfs) {
      hipLaunchKernelGGL(k_dfs<4>, dim3(fb_blocks), dim3(kWave), fb_lds, st, s, ws.last_bytes, ws.last_offs, o,
                         nullptr, nullptr, nullptr, nullptr, max_levels);
      HIP_TRY(hipGetLastError());
    }
  }
  out->n_topics = n;
  out->n_idents = total;
  out->offsets = o.istart;
  out->sids = o.iout;
  return 0;
}

int derive_node_flags(const NodeDesc *nodes, uint8_t *nflags, uint64_t n, hipStream_t st) {
  if (n)
    hipLaunchKernelGGL(k_nflags, dim3((uint32_t)std::min<uint64_t>((n + 255) / 256, 16384)), dim3(256), 0, st, nodes,
                       nflags, n);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

bool slots_enabled() {
  static const bool v = getenv("MQM_SLOTS") && atoi(getenv("MQM_SLOTS")) != 0;
  return v;
}

int derive_slots(const NodeDesc *nodes, NodeDesc *slots, uint64_t n, hipStream_t st) {
  if (n)
    hipLaunchKernelGGL(k_slots, dim3((uint32_t)std::min<uint64_t>((n + 255) / 256, 16384)), dim3(256), 0, st, nodes,
                       slots, n);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

int derive_ident_bits(const SubEnt *subs, uint32_t *bits, uint64_t n, hipStream_t st) {
  const uint64_t nw = (n + 31) / 32;
  if (nw)
    hipLaunchKernelGGL(k_ident_bits, dim3((uint32_t)std::min<uint64_t>((nw + 255) / 256, 16384)), dim3(256), 0, st,
                       subs, bits, n);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

int derive_words(const SubEnt *subs, uint32_t *words, uint64_t n, hipStream_t st) {
  if (n)
    hipLaunchKernelGGL(k_words, dim3((uint32_t)std::min<uint64_t>((n + 255) / 256, 16384)), dim3(256), 0, st, subs,
                       words, n);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

int densify(const DeviceSnapshot &s, Workspace &ws, const MatchOutput &m, hipStream_t st, DenseOutput *out,
            bool packed) {
  using W = Workspace;
  const uint32_t n = m.n_topics;
  if (ws.get(W::kDenseOffs, sizeof(uint64_t) * (n + 1)) || ws.get(W::kDenseHOffs, sizeof(uint64_t) * (n + 1)) ||
      ws.get(W::kTable, std::max(sizeof(uint64_t) * (m.n_deliveries + 1), sizeof(uint32_t) * (m.n_shared + 1))))
    return -2;
  auto *doffs = (uint64_t *)ws.ptr(W::kDenseOffs);
  auto *hoffs = (uint64_t *)ws.ptr(W::kDenseHOffs);
  if (scan_offsets(ws, m.counts, doffs, n, st) || scan_offsets(ws, m.shared_counts, hoffs, n, st)) return -3;
  // dense deliveries in kTable; dense shared after them in kDenseShared
  if (ws.get(W::kDenseShared, sizeof(uint32_t) * (m.n_shared + 1))) return -2;
  auto *dd = (uint64_t *)ws.ptr(W::kTable);
  auto *hd = (uint32_t *)ws.ptr(W::kDenseShared);
  if (n > 0) {
    if (packed)
      hipLaunchKernelGGL(k_densify<true>, dim3(std::min<uint32_t>((n + 3) / 4, 8192)), dim3(256), 0, st, s, n,
                         m.counts, m.starts, doffs, m.deliveries, (void *)dd, m.shared_counts, m.shared_starts, hoffs,
                         m.shared, hd);
    else
      hipLaunchKernelGGL(k_densify<false>, dim3(std::min<uint32_t>((n + 3) / 4, 8192)), dim3(256), 0, st, s, n,
                         m.counts, m.starts, doffs, m.deliveries, (void *)dd, m.shared_counts, m.shared_starts, hoffs,
                         m.shared, hd);
  }
  HIP_TRY(hipGetLastError());
  out->offsets = doffs;
  out->deliveries = dd;
  out->shared_offsets = hoffs;
  out->shared = hd;
  return 0;
}

// ---- copy-out: a host-path result into pinned host memory, by the CUs -------
// tools/duplex_probe (r06h): a kernel storing to pinned memory moves 54.8 GB/s
// one way; the parts are 16-B aligned, each a multiple of 4 B.  Every lane
// walks every part (at most 8), 16-B units grid-stride, then the 4-B tail.
__global__ __launch_bounds__(256) void k_copy_out(CopyOut c) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x, tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int k = 0; k < c.n; k++) {
    const uint4 *s = static_cast<const uint4 *>(c.src[k]);
    uint4 *d = static_cast<uint4 *>(c.dst[k]);
    const uint64_t n16 = c.bytes[k] / 16;
    uint64_t i = tid;
    for (; i + 3 * stride < n16; i += 4 * stride) {  // 4 loads in flight per lane
      const uint4 a = s[i], b = s[i + stride], e = s[i + 2 * stride], f = s[i + 3 * stride];
      d[i] = a;
      d[i + stride] = b;
      d[i + 2 * stride] = e;
      d[i + 3 * stride] = f;
    }
    for (; i < n16; i += stride) d[i] = s[i];
    const uint64_t t4 = (c.bytes[k] % 16) / 4;
    if (tid < t4)
      static_cast<uint32_t *>(c.dst[k])[n16 * 4 + tid] = static_cast<const uint32_t *>(c.src[k])[n16 * 4 + tid];
  }
}

int copy_out_device(const CopyOut &c, hipStream_t st) {
  if (c.n <= 0) return 0;
  uint64_t total = 0;
  for (int k = 0; k < c.n; k++) {
    if ((c.bytes[k] & 3) || ((uintptr_t)c.src[k] & 15) || ((uintptr_t)c.dst[k] & 15)) return -4;
    total += c.bytes[k];
  }
  static const uint32_t blocks = [] {
    const char *e = getenv("MQM_D2H_KERNEL_BLOCKS");
    const long v = e ? atol(e) : 0;
    return v > 0 && v <= 8192 ? (uint32_t)v : 256u;
  }();
  const uint32_t g = (uint32_t)std::min<uint64_t>(blocks, (total / 16 + 1023) / 1024 + 1);
  hipLaunchKernelGGL(k_copy_out, dim3(g), dim3(256), 0, st, c);
  HIP_TRY(hipGetLastError());
  return 0;
}

}  // namespace mqm
