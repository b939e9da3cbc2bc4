// maxmq_amd/csrc/retained.hip — gfx950 kernels for TopicsIndex.Messages
// (vendor/github.com/mochi-co/mqtt/v2/topics.go:426-480): a batch of
// subscription filters against the retained topics of the snapshot.
//
// The reference recurses per filter (scanMessages).  Here the recursion is
// unrolled level-synchronously over the whole batch, as worklists of
// (filter, node) items in HBM, so wildcard fan-out never overflows a
// per-filter buffer and every level is a balanced launch.  The whole call is
// queued without waiting for the device: every list is appended through
// wave-aggregated atomic counters that live on the device, every kernel is a
// grid-stride loop over a count it reads from device memory, and the host
// reads the counters back once at the end (plus once at the start for the
// filters' level count).  Lists are sized from the previous call; a list that
// would overflow is flagged, and the call is re-queued with the sizes the
// counters report (first call of a workload only).
//   k_flt_levels   a thread per filter: split into levels (isolateParticle,
//                  topics.go:558-577), 128-bit level keys, wildcard flag
//   k_level<d>     a thread per item of level d: the reference's three
//                  cases (topics.go:447-477) —
//                    literal : one edge probe (the forward matcher's table)
//                    '+'/'#' with more levels: every child (minus "$SYS" at
//                             the root, :450) becomes an item of level d+1;
//                             a wavefront writes a big child list together
//                    '+' last : the node's retained children      (:454-460)
//                    '#' last : every retained node below it      (:462, the
//                             recursion keeps isolating the last level)
//                    literal last: the child's retained message, or — only
//                             for wildcard filters — the message retained at
//                             topic "" (Retained.Get(""), :474)
//                  emissions are (filter, list, lo, hi) ranges of message refs:
//                  subtrees are contiguous in preorder (snapshot.h)
//   k_emit_count / k_emit_place / k_task_copy
//                  ranges -> per-filter CSR of message refs: small ranges
//                  copied by their thread, large ones cut into fixed-size
//                  copy tasks so one huge '#' range is spread over many
//                  wavefronts
// Exact filters (no '+'/'#', :440-445) are the literal walk of the same items
// with Retained.Get(filter) semantics (no "" fallback).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "device.h"
#include "retained.h"

namespace mqm {

namespace {

constexpr uint32_t kTaskRefs = 8192;   // refs copied per wavefront task
constexpr uint32_t kSmallEmit = 32;    // emissions up to this size: copied by their own thread
constexpr uint32_t kCoopItems = 64;    // a lane with more next-level items than this: the wave writes them
constexpr uint32_t kLevelBatch = 16;   // levels queued between two looks at the counters
constexpr int kThreads = 256;

struct Level {         // one level of one filter
  uint64_t k0, k1;     // key (keys.h)
  uint32_t start, len; // byte range within the filter
};

enum : uint32_t { kTypeLiteral = 0, kTypePlus = 1, kTypeHash = 2 };

enum : uint32_t { kOvfItems = 1, kOvfEmit = 2, kOvfTasks = 4, kOvfOut = 8, kOvfLTasks = 16 };

// level tasks (MQM_REV_TASKS=1): the long child lists and the literal-edge
// index ranges of a level are cut into chunks of at most kTaskEdges and
// spread over every wavefront of a second launch (k_level_tasks), instead of
// being worked through by the wavefront that found them, lane after lane
constexpr uint32_t kTaskEdges = 1024;
enum : uint32_t { kLTChildren = 0, kLTIndexItems = 1, kLTIndexEmit = 2 };
struct LTask {
  uint32_t f, lo, n, need;  // filter, first child / edge, count, node flags the next level needs
  uint64_t at;              // children: their slots in the next level's list
  uint32_t kind, root;      // kLT*; the level is the root's ("$SYS" dropped)
};

// device-side counters of one call (zeroed at its start); items[d] = items
// appended to level d (d >= 1), the append cursor of that level's list
struct RevCtr {
  unsigned long long n_emit, n_tasks;
  unsigned long long need_items;  // largest level seen (also past the capacity)
  unsigned long long items_total; // items over all levels (statistics)
  unsigned long long skipped;     // items the reference visits that the edge index jumps over
  unsigned int ovf;               // kOvf* bits
  unsigned int pad;
  unsigned long long appended;    // items appended to the lists over all levels (chunk padding excluded)
  unsigned long long n_ltasks;    // level tasks of the current level (reset before each level)
  unsigned long long need_ltasks; // most level tasks any level appended (also past the capacity)
  unsigned long long items[1];    // [levels + 1]
};
// MQM_REV_STATS=1: per level d < kStatLevels, the mix of its items (after the
// counters in the same buffer) — live items, literal probes, children listed
// by wildcard expansions, edges of the literal-edge index's ranges, emissions
constexpr uint32_t kStatLevels = 16, kStatKinds = 5;

__device__ __forceinline__ uint32_t level_type(const Level &l) {
  if (l.k1 != (1ull << 56)) return kTypeLiteral;
  return l.k0 == '+' ? kTypePlus : l.k0 == '#' ? kTypeHash : kTypeLiteral;
}

// per filter: number of levels (0 for ""), wildcard flag (any '+' / '#' byte)
__global__ void k_flt_count(const uint8_t *__restrict__ bytes, const uint64_t *__restrict__ offs, uint32_t n,
                            uint32_t *__restrict__ nlev, uint8_t *__restrict__ wild) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n) return;
  const uint64_t o = offs[f];
  const uint32_t len = (uint32_t)(offs[f + 1] - o);
  uint32_t seps = 0;
  bool w = false;
  for (uint32_t i = 0; i < len; i++) {
    const uint8_t b = bytes[o + i];
    seps += b == '/';
    w |= b == '+' || b == '#';
  }
  nlev[f] = len ? seps + 1 : 0;
  wild[f] = w ? 1 : 0;
}

__global__ void k_flt_fill(const uint8_t *__restrict__ bytes, const uint64_t *__restrict__ offs, uint32_t n,
                           const uint64_t *__restrict__ loff, Level *__restrict__ lv) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n) return;
  const uint64_t o = offs[f];
  const uint32_t len = (uint32_t)(offs[f + 1] - o);
  if (!len) return;
  const uint8_t *p = bytes + o;
  Level *out = lv + loff[f];
  uint32_t st = 0;
  for (uint32_t i = 0; i <= len; i++) {
    if (i < len && p[i] != '/') continue;
    const Key k = make_key([&](uint32_t j) { return p[st + j]; }, i - st);
    Level l;
    l.k0 = k.k0;
    l.k1 = k.k1;
    l.start = st;
    l.len = i - st;
    *out++ = l;
    st = i + 1;
  }
}

// exclusive wave scan of a 64-bit count; *total = the wave's sum
__device__ __forceinline__ uint64_t wave_excl(uint64_t v, uint64_t *total) {
  const int lane = threadIdx.x & 63;
  uint64_t inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t lo = __shfl_up((uint32_t)inc, d, 64), hi = __shfl_up((uint32_t)(inc >> 32), d, 64);
    if (lane >= d) inc += ((uint64_t)hi << 32) | lo;
  }
  const uint32_t tlo = __shfl((uint32_t)inc, 63, 64), thi = __shfl((uint32_t)(inc >> 32), 63, 64);
  *total = ((uint64_t)thi << 32) | tlo;
  return inc - v;
}

// one atomic per wavefront: reserve `v` slots of a list for every lane;
// returns the lane's first slot
__device__ __forceinline__ uint64_t wave_reserve(unsigned long long *ctr, uint64_t v) {
  uint64_t total;
  const uint64_t ex = wave_excl(v, &total);
  unsigned long long base = 0;
  if ((threadIdx.x & 63) == 0 && total) base = atomicAdd(ctr, (unsigned long long)total);
  const uint32_t lo = __shfl((uint32_t)base, 0, 64), hi = __shfl((uint32_t)(base >> 32), 0, 64);
  return (((uint64_t)hi << 32) | lo) + ex;
}

// A wavefront's private chunk of a list: slots [base, base + size) reserved
// with one global atomic and filled in order (wave-uniform state).  One
// atomic per 64 appends on one counter serialised the level kernels: one
// address takes ~88 returning atomics per microsecond (MI355X_MICROARCH,
// dequeue), and C5's levels appended ~2.8M times (r05f rev-stats).  The
// unused tail of a chunk is padded with dead entries (items: node kNone;
// emissions: filter kNone, empty) when the wave takes a new chunk or leaves.
struct WaveChunk {
  uint64_t base = 0, fill = 0, size = 0;
};
constexpr uint64_t kChunkMin = 256, kChunkMax = 2048;

// -> this lane's first slot for its v appends (every lane of the wave calls it)
template <class Pad>
__device__ __forceinline__ uint64_t chunk_take(WaveChunk &c, unsigned long long *ctr, uint64_t v, Pad &&pad,
                                               unsigned long long *need, uint64_t cap, unsigned int *ovf,
                                               unsigned int ovf_bit) {
  uint64_t total;
  const uint64_t ex = wave_excl(v, &total);
  if (total == 0) return 0;
  if (c.fill + total > c.size) {
    if (c.size > c.fill) pad(c.base + c.fill, c.size - c.fill);
    const uint64_t want = max(total, min(kChunkMax, max(kChunkMin, 8 * total)));
    unsigned long long b = 0;
    if ((threadIdx.x & 63) == 0) {
      b = atomicAdd(ctr, (unsigned long long)want);
      if (need) atomicMax(need, b + want);
      if (b + want > cap) atomicOr(ovf, ovf_bit);
    }
    const uint32_t lo = __shfl((uint32_t)b, 0, 64), hi = __shfl((uint32_t)(b >> 32), 0, 64);
    c.base = ((uint64_t)hi << 32) | lo;
    c.fill = 0;
    c.size = want;
  }
  const uint64_t at = c.base + c.fill + ex;
  c.fill += total;
  return at;
}

__device__ __forceinline__ uint64_t bcast64(uint64_t v, int src) {
  const uint32_t lo = __shfl((uint32_t)v, src, 64), hi = __shfl((uint32_t)(v >> 32), src, 64);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ bool retained_node(const DeviceRetained &r, uint32_t c) {
  return r.cum[c + 1] > r.cum[c];
}

// what a node must have for an item of a level of this type to produce
// anything: a literal child (its probe) or any child ('+' / '#')
__device__ __forceinline__ uint32_t need_of(const Level &l, bool wild) {
  return wild && level_type(l) != kTypeLiteral ? kFlagHasChildren : kFlagHasLiteral;
}

// the edge index's group (level key of l, child depth): its edges
// inv[*start, *start + *count); false when no such edge exists
__device__ bool rev_group(const DeviceRetained &r, const uint8_t *tok_pool, const Level &l, const uint8_t *ftok,
                          uint32_t depth, uint32_t *start, uint32_t *count) {
  const Key k{l.k0, l.k1};
  uint64_t slot = bucket_of(edge_hash(depth, k), r.n_gslots);
  for (;;) {
    const RevGroup g = r.groups[slot];
    if (g.count == 0) return false;
    if (g.k0 == k.k0 && g.k1 == k.k1 && (g.depth_len & 0xFFFFu) == depth) {
      bool ok = true;
      if (key_is_long(k)) {  // hashed long token: verify the bytes
        ok = (g.depth_len >> 16) == l.len;
        for (uint32_t i = 0; ok && i < l.len; i++) ok = tok_pool[g.tok_off + i] == ftok[i];
      }
      if (ok) {
        *start = g.start;
        *count = g.count;
        return true;
      }
    }
    slot = slot + 1 == r.n_gslots ? 0 : slot + 1;
  }
}

// first j in [lo, hi) with inv[j].x >= key (parents are sorted within a group)
__device__ __forceinline__ uint32_t inv_lower(const uint2 *inv, uint32_t lo, uint32_t hi, uint32_t key) {
  while (lo < hi) {
    const uint32_t mid = lo + (hi - lo) / 2;
    if (inv[mid].x < key)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

struct LevelArgs {
  DeviceSnapshot s;
  DeviceRetained r;
  const uint8_t *bytes;
  const uint64_t *offs;
  const uint64_t *loff;
  const uint32_t *nlev;
  const uint8_t *wild;
  const Level *lv;
  uint32_t n;                       // filters (the implicit level-0 list: item f = (f, root))
  uint32_t d;
  const uint32_t *item_f, *item_n;  // level d's list (d >= 1)
  uint32_t *next_f, *next_n;        // level d + 1's list
  uint32_t *skip_f, *skip_n;        // level d + 2's list (wildcard + literal through the edge index)
  uint64_t item_cap;                // capacity of each list
  Emit *emit;
  uint64_t emit_cap;
  RevCtr *ctr;
  unsigned long long *st;           // MQM_REV_STATS: the levels' item mix [kStatLevels][kStatKinds], else null
  LTask *ltasks;                    // MQM_REV_TASKS: this level's tasks (nullptr: the wavefront works its own)
  uint64_t ltask_cap;
};

// edge j of a wildcard + literal index range, written at slot `pos` of the
// emissions (the literal is last: c's message, else Retained.Get("") through
// an empty retainPath, topics.go:474) or of level d + 2's list (c, when it can
// continue); anything else writes an empty emission / a dead item
__device__ __forceinline__ void rev_index_edge(const DeviceRetained &r, const LevelArgs &a, bool root, bool emit,
                                               uint32_t f, uint32_t need, uint32_t j, uint64_t pos) {
  const uint2 ed = r.inv[j];
  const uint32_t c = ed.y;
  bool valid = !(root && ed.x == r.sys_child);
  if (emit) {
    Emit em{kNone, 0, 0, 0};
    if (valid) {
      if (retained_node(r, c))
        em = Emit{f, 0, r.cum[c], r.cum[c] + 1};
      else if (r.has_empty)
        em = Emit{f, 0, (uint32_t)r.n_ret, (uint32_t)r.n_ret + 1};
    }
    if (pos < a.emit_cap) a.emit[pos] = em;
  } else {
    valid = valid && (r.nflags[c] & need) != 0;
    if (pos < a.item_cap) {
      a.skip_f[pos] = f;
      a.skip_n[pos] = valid ? c : kNone;
    }
  }
}

// a thread per item of level d; the loop is grid-stride over the level's
// count as the previous launch left it in ctr->items[d]
__global__ __launch_bounds__(kThreads) void k_level(LevelArgs a) {
  const DeviceRetained &r = a.r;
  const int lane = threadIdx.x & 63;
  const uint64_t cnt = a.d == 0 ? a.n : min((uint64_t)a.ctr->items[a.d], a.item_cap);
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  // the wave's chunks of the next level's list, the level after (edge-index
  // jumps) and the emissions; dead-entry padding for their unused tails
  WaveChunk cnext, cskip, cemit;
  uint64_t app = 0, skipped_sum = 0;  // (lane 0 / every lane: flushed once at the end)
  auto pad_items = [&](uint32_t *lf, uint32_t *ln) {
    return [&a, lf, ln, lane](uint64_t pos, uint64_t len) {
      for (uint64_t k = lane; k < len; k += 64)
        if (pos + k < a.item_cap) {
          lf[pos + k] = 0;
          ln[pos + k] = kNone;
        }
    };
  };
  auto pad_next = pad_items(a.next_f, a.next_n);
  auto pad_skip = pad_items(a.skip_f, a.skip_n);
  auto pad_emit = [&](uint64_t pos, uint64_t len) {
    for (uint64_t k = lane; k < len; k += 64)
      if (pos + k < a.emit_cap) a.emit[pos + k] = Emit{kNone, 0, 0, 0};
  };
  // whole wavefronts iterate together (the appends below are wave-collective)
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); base < cnt; base += stride) {
    const uint64_t i = base + lane;
    uint32_t f = 0, p = kNone;
    if (i < cnt) {
      if (a.d == 0) {
        f = (uint32_t)i;
        p = a.nlev[f] ? 0u : kNone;
      } else {
        f = a.item_f[i];
        p = a.item_n[i];
      }
    }
    // outputs of this lane: one next item (literal), a child range (wildcard
    // with more levels), or up to two emissions
    uint32_t nx_one = kNone, ch_lo = 0, ch_hi = 0, ne = 0;
    // what a node of the next level must have to continue (need_of)
    uint32_t need = 0;
    // wildcard + literal through the edge index: edges inv[rg_lo, rg_hi) give
    // the level d + 2 nodes (or, the literal being last, the emissions)
    uint32_t rg_lo = 0, rg_hi = 0, need2 = 0, skipped = 0;
    bool rg_emit = false;
    Emit e0{f, 0, 0, 0}, e1{f, 0, 0, 0};
    if (p != kNone) {
      const uint32_t L = a.nlev[f];
      const Level l = a.lv[a.loff[f] + a.d];
      const bool has_next = a.d + 1 < L;
      const bool wild = a.wild[f] != 0;
      const uint32_t type = wild ? level_type(l) : kTypeLiteral;
      Level l1{};
      if (has_next) {
        l1 = a.lv[a.loff[f] + a.d + 1];
        need = need_of(l1, wild);
      }
      if (type == kTypeLiteral) {  // topics.go:469-477 (and :440-445 for exact filters)
        NodeDesc dc;
        const uint32_t c = probe_edge(a.s, p, l.k0, l.k1, a.bytes + a.offs[f] + l.start, l.len, &dc);
        if (c != kNone) {
          if (has_next) {
            if ((dc.sh_cnt_flags >> 24) & need) nx_one = c;  // else no item of the next level can match
          } else if (retained_node(r, c)) {
            e0 = Emit{f, 0, r.cum[c], r.cum[c] + 1};
            ne = 1;
          } else if (wild && r.has_empty) {  // Retained.Get("") through an empty retainPath
            e0 = Emit{f, 0, (uint32_t)r.n_ret, (uint32_t)r.n_ret + 1};
            ne = 1;
          }
        }
      } else if (has_next && r.n_gslots && level_type(l1) == kTypeLiteral) {
        // '+' / '#', then a literal K: the reference probes K under every
        // child x of p (:449-477); the index lists exactly the x that have a
        // child K — edges of group (K, depth d + 2) whose parent lies in p's
        // subtree (a node of depth d + 1 there is a child of p)
        uint32_t gs, gc;
        if (rev_group(r, a.s.tok_pool, l1, a.bytes + a.offs[f] + l1.start, a.d + 2, &gs, &gc)) {
          rg_lo = inv_lower(r.inv, gs, gs + gc, p + 1);
          rg_hi = inv_lower(r.inv, rg_lo, gs + gc, p + r.subtree[p]);
        }
        rg_emit = a.d + 2 >= L;
        if (!rg_emit) need2 = need_of(a.lv[a.loff[f] + a.d + 2], wild);
        skipped = r.child_off[p + 1] - r.child_off[p] - (a.d == 0 && r.sys_child != kNone ? 1u : 0u);
      } else if (has_next) {  // '+' or '#' followed by more levels: every child (:449-465)
        ch_lo = r.child_off[p];
        ch_hi = r.child_off[p + 1];
      } else if (type == kTypePlus) {  // the retained children (root's list excludes "$SYS")
        e0 = Emit{f, 1, r.rch_off[p], r.rch_off[p + 1]};
        ne = e0.hi > e0.lo;
      } else {  // '#' last: the subtree below p, "$SYS" skipped at the root (:450)
        const uint32_t end = p + r.subtree[p];
        if (a.d == 0 && r.sys_child != kNone) {
          const uint32_t sys = r.sys_child;
          e0 = Emit{f, 0, r.cum[p + 1], r.cum[sys]};
          e1 = Emit{f, 0, r.cum[sys + r.subtree[sys]], r.cum[end]};
          if (e0.hi <= e0.lo) e0 = e1, e1.hi = e1.lo;
          ne = (e0.hi > e0.lo) + (e1.hi > e1.lo);
        } else {
          e0 = Emit{f, 0, r.cum[p + 1], r.cum[end]};
          ne = e0.hi > e0.lo;
        }
      }
    }
    if (a.st && a.d < kStatLevels) {  // the level's item mix (MQM_REV_STATS)
      const bool is_lit = p != kNone && ch_hi == ch_lo && rg_hi == rg_lo && (nx_one != kNone || ne <= 1) &&
                          (a.wild[f] == 0 || level_type(a.lv[a.loff[f] + a.d]) == kTypeLiteral);
      const uint64_t v[5] = {p != kNone ? 1u : 0u, is_lit ? 1u : 0u, ch_hi - ch_lo, rg_hi - rg_lo, ne};
      for (int k = 0; k < 5; k++) {
        uint64_t tot;
        (void)wave_excl(v[k], &tot);
        if (lane == 0 && tot) atomicAdd(&a.st[a.d * kStatKinds + k], (unsigned long long)tot);
      }
    }
    // next-level items: one per literal hit, the child list of a wildcard
    const uint32_t nn = nx_one != kNone ? 1u : ch_hi - ch_lo;
    if (__any(nn != 0)) {
      const uint64_t at = chunk_take(cnext, &a.ctr->items[a.d + 1], nn, pad_next, &a.ctr->need_items, a.item_cap,
                                     &a.ctr->ovf, kOvfItems);
      app += nn;
      // "$SYS" at the root, and every child that cannot continue (node flags),
      // become dead items (kNone): the next level skips them without a read
      const uint32_t skip = a.d == 0 ? r.sys_child : kNone;
      const uint32_t sneed = need;
      if (nx_one != kNone) {
        if (at < a.item_cap) {
          a.next_f[at] = f;
          a.next_n[at] = nx_one;
        }
      } else if (nn <= kCoopItems) {
        for (uint32_t k = 0; k < nn; k++) {
          if (at + k >= a.item_cap) break;
          const uint32_t c = r.child_ids[ch_lo + k];
          a.next_f[at + k] = f;
          a.next_n[at + k] = c == skip || !(r.nflags[c] & sneed) ? kNone : c;
        }
      }
      uint64_t big = __ballot(nx_one == kNone && nn > kCoopItems);
      if (a.ltasks && big) {  // long child lists: chunks for k_level_tasks
        const bool mine = nx_one == kNone && nn > kCoopItems;
        const uint32_t nch = mine ? (nn + kTaskEdges - 1) / kTaskEdges : 0;
        const uint64_t t0 = wave_reserve(&a.ctr->n_ltasks, nch);
        if (lane == 63) atomicMax(&a.ctr->need_ltasks, (unsigned long long)(t0 + nch));
        if (t0 + nch > a.ltask_cap) atomicOr(&a.ctr->ovf, (unsigned)kOvfLTasks);
        for (uint32_t k = 0; k < nch && t0 + k < a.ltask_cap; k++)
          a.ltasks[t0 + k] = LTask{f, ch_lo + k * kTaskEdges, min(kTaskEdges, nn - k * kTaskEdges), need,
                                   at + (uint64_t)k * kTaskEdges, kLTChildren, a.d == 0 ? 1u : 0u};
        big = 0;
      }
      while (big) {  // long child lists: the whole wavefront writes each
        const int src = __builtin_ctzll(big);
        big &= big - 1;
        const uint32_t sf = __shfl(f, src, 64), slo = __shfl(ch_lo, src, 64), snn = __shfl(nn, src, 64);
        const uint32_t bneed = __shfl(need, src, 64);
        const uint64_t sat = bcast64(at, src);
        for (uint32_t k = lane; k < snn; k += 64) {
          if (sat + k >= a.item_cap) break;
          const uint32_t c = r.child_ids[slo + k];
          a.next_f[sat + k] = sf;
          a.next_n[sat + k] = c == skip || !(r.nflags[c] & bneed) ? kNone : c;
        }
      }
    }
    if (__any(ne != 0)) {
      const uint64_t at = chunk_take(cemit, &a.ctr->n_emit, ne, pad_emit, nullptr, a.emit_cap, &a.ctr->ovf,
                                     kOvfEmit);
      if (ne > 0 && at < a.emit_cap) a.emit[at] = e0;
      if (ne > 1 && at + 1 < a.emit_cap) a.emit[at + 1] = e1;
    }
    skipped_sum += skipped;  // statistics: the reference's level d + 1 items
    // index ranges: every edge gets its slot up front (one reservation per
    // lane's range), a wavefront writes each range, 64 edges per step; an
    // edge that yields nothing writes a dead item / an empty emission
    uint64_t rt = __ballot(rg_hi > rg_lo);
    if (rt) {
      const uint32_t rn = rg_hi - rg_lo;
      const uint64_t ra_e = chunk_take(cemit, &a.ctr->n_emit, rg_emit ? rn : 0u, pad_emit, nullptr, a.emit_cap,
                                       &a.ctr->ovf, kOvfEmit);
      const uint64_t ra_s = chunk_take(cskip, &a.ctr->items[a.d + 2], rg_emit ? 0u : rn, pad_skip,
                                       &a.ctr->need_items, a.item_cap, &a.ctr->ovf, kOvfItems);
      app += rg_emit ? 0u : rn;
      const uint64_t ra = rg_emit ? ra_e : ra_s;
      if (a.ltasks) {  // ... or chunks for k_level_tasks
        const uint32_t nch = (rn + kTaskEdges - 1) / kTaskEdges;
        const uint64_t t0 = wave_reserve(&a.ctr->n_ltasks, nch);
        if (lane == 63) atomicMax(&a.ctr->need_ltasks, (unsigned long long)(t0 + nch));
        if (t0 + nch > a.ltask_cap) atomicOr(&a.ctr->ovf, (unsigned)kOvfLTasks);
        for (uint32_t k = 0; k < nch && t0 + k < a.ltask_cap; k++)
          a.ltasks[t0 + k] = LTask{f, rg_lo + k * kTaskEdges, min(kTaskEdges, rn - k * kTaskEdges), need2,
                                   ra + (uint64_t)k * kTaskEdges, rg_emit ? kLTIndexEmit : kLTIndexItems,
                                   a.d == 0 ? 1u : 0u};
        rt = 0;
      }
      while (rt) {
        const int src = __builtin_ctzll(rt);
        rt &= rt - 1;
        const uint32_t sf = __shfl(f, src, 64), slo = __shfl(rg_lo, src, 64), shi = __shfl(rg_hi, src, 64);
        const uint32_t sneed = __shfl(need2, src, 64);
        const bool semit = __shfl((uint32_t)rg_emit, src, 64) != 0;
        const uint64_t sra = bcast64(ra, src);
        for (uint32_t j = slo + lane; j < shi; j += 64)
          rev_index_edge(r, a, a.d == 0, semit, sf, sneed, j, sra + (j - slo));
      }
    }
  }
  if (cnext.size > cnext.fill) pad_next(cnext.base + cnext.fill, cnext.size - cnext.fill);
  if (cskip.size > cskip.fill) pad_skip(cskip.base + cskip.fill, cskip.size - cskip.fill);
  if (cemit.size > cemit.fill) pad_emit(cemit.base + cemit.fill, cemit.size - cemit.fill);
  uint64_t tot;
  (void)wave_excl(skipped_sum, &tot);
  if (lane == 0 && tot) atomicAdd(&a.ctr->skipped, (unsigned long long)tot);
  (void)wave_excl(app, &tot);
  if (lane == 0 && tot) atomicAdd(&a.ctr->appended, (unsigned long long)tot);
}

// k_level_tasks: a wavefront per task of the level (grid-stride), 64
// children / edges per step — the same writes k_level's wavefront loops make
__global__ __launch_bounds__(kThreads) void k_level_tasks(LevelArgs a) {
  const DeviceRetained &r = a.r;
  const int lane = threadIdx.x & 63;
  const uint64_t nt = min((uint64_t)a.ctr->n_ltasks, a.ltask_cap);
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x / 64);
  for (uint64_t t = (uint64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; t < nt; t += nw) {
    const LTask k = a.ltasks[t];
    if (k.kind == kLTChildren) {
      const uint32_t skip = k.root ? r.sys_child : kNone;
      for (uint32_t j = lane; j < k.n; j += 64) {
        if (k.at + j >= a.item_cap) break;
        const uint32_t c = r.child_ids[k.lo + j];
        a.next_f[k.at + j] = k.f;
        a.next_n[k.at + j] = c == skip || !(r.nflags[c] & k.need) ? kNone : c;
      }
      continue;
    }
    const bool semit = k.kind == kLTIndexEmit;
    for (uint32_t j = lane; j < k.n; j += 64) rev_index_edge(r, a, k.root != 0, semit, k.f, k.need, k.lo + j, k.at + j);
  }
}

// Emissions of one filter are mostly adjacent (a wave appends its lanes' in
// order), so a wavefront folds each run of equal filter ids (segmented scan
// over the lanes) and issues one atomic per run.
struct Run {
  uint64_t inc;    // inclusive sum of cnt within the lane's run
  bool last;       // the lane closes its run
  int last_lane;   // lane that closes the lane's run
};

__device__ __forceinline__ Run fold_runs(uint32_t f, uint64_t cnt) {
  const int lane = threadIdx.x & 63;
  const uint32_t pf = __shfl_up(f, 1, 64);
  const bool head = lane == 0 || pf != f;
  const uint64_t heads = __ballot(head);
  const uint64_t le = lane == 63 ? ~0ull : ((1ull << (lane + 1)) - 1);
  const int start = 63 - __builtin_clzll(heads & le);
  uint64_t inc = cnt;
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t lo = __shfl_up((uint32_t)inc, d, 64), hi = __shfl_up((uint32_t)(inc >> 32), d, 64);
    if (lane - d >= start) inc += ((uint64_t)hi << 32) | lo;
  }
  const uint64_t after = heads & ~le;
  Run r;
  r.last_lane = after ? __builtin_ctzll(after) - 1 : 63;
  r.last = r.last_lane == lane;
  r.inc = inc;
  return r;
}

// grid-stride over the emissions the level kernels appended
__global__ __launch_bounds__(kThreads) void k_emit_count(const Emit *__restrict__ e, uint64_t cap, RevCtr *ctr,
                                                        unsigned long long *__restrict__ fcount, uint32_t levels) {
  if (blockIdx.x == 0 && threadIdx.x == 0)  // the level kernels are done: the items appended (no padding)
    ctr->items_total = ctr->appended + ctr->skipped;
  (void)levels;
  const uint64_t ne = min((uint64_t)ctr->n_emit, cap);
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); base < ne; base += stride) {
    const uint64_t i = base + (threadIdx.x & 63);
    const bool ok = i < ne;
    const uint32_t f = ok ? e[i].f : 0xFFFFFFFFu;
    const uint64_t cnt = ok ? e[i].hi - e[i].lo : 0;
    const Run r = fold_runs(f, cnt);
    if (ok && r.last && f != kNone) atomicAdd(&fcount[f], (unsigned long long)r.inc);  // (kNone: chunk padding)
  }
}

struct Task {            // copy list[lo, lo + len) to out[dst ..)
  uint64_t dst;
  uint32_t lo, len_list; // len | list << 31
};

// each emission's place in its filter's segment: small ones copied here by
// the whole wavefront (lanes over the concatenated small emissions of the 64:
// consecutive refs on consecutive lanes — adjacent emissions of one filter are
// adjacent in its segment too; round 5 copied each one on its own lane, 8-B
// accesses strided across the wave: k_emit_place 3.5 ms of 22.1, r05aa),
// large ones cut into kTaskRefs copy tasks
// an output ref: non-temporal (MQM_REV_NT, default on) — the call writes its
// refs once (2,196 per filter at C5: 17.6 GB) and reads none of them back
template <bool kNT>
__device__ __forceinline__ void put_ref(uint64_t *p, uint64_t v) {
  if constexpr (kNT)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

struct EmitLds {
  uint32_t pre[65];           // exclusive prefix of the small emissions' counts
  uint64_t pos[64], src[64];  // output position, source index | list << 63
};
template <bool kNT>
__global__ __launch_bounds__(kThreads) void k_emit_place(const Emit *__restrict__ e, uint64_t cap, RevCtr *ctr,
                                                        const uint64_t *__restrict__ foff,
                                                        unsigned long long *__restrict__ fcur,
                                                        const uint64_t *__restrict__ refs,
                                                        const uint64_t *__restrict__ rch_refs,
                                                        uint64_t *__restrict__ out, uint64_t out_cap,
                                                        Task *__restrict__ tasks, uint64_t task_cap) {
  __shared__ EmitLds lds_all[kThreads / 64];
  EmitLds &L = lds_all[threadIdx.x / 64];
  const uint64_t ne = min((uint64_t)ctr->n_emit, cap);
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const int lane = threadIdx.x & 63;
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); base < ne; base += stride) {
    const uint64_t i = base + lane;
    const bool ok = i < ne;
    const Emit it = ok ? e[i] : Emit{0xFFFFFFFFu, 0, 0, 0};
    const uint64_t cnt = it.hi - it.lo;
    const Run r = fold_runs(it.f, cnt);
    unsigned long long rb = 0;
    if (ok && r.last && it.f != kNone) rb = foff[it.f] + atomicAdd(&fcur[it.f], (unsigned long long)r.inc);
    const uint64_t pos = bcast64(rb, r.last_lane) + (r.inc - cnt);  // run base + the run's entries before this lane
    const bool fits = ok && cnt > 0 && pos + cnt <= out_cap;
    if (ok && cnt > 0 && !fits) atomicOr(&ctr->ovf, (unsigned)kOvfOut);
    // the small ones, together (every lane takes part: wave-uniform loop)
    const uint32_t cs = fits && cnt <= kSmallEmit ? (uint32_t)cnt : 0u;
    uint32_t inc = cs;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t v = __shfl_up(inc, d, 64);
      if (lane >= d) inc += v;
    }
    const uint32_t total = __shfl(inc, 63, 64);
    if (total) {
      L.pre[lane] = inc - cs;
      if (lane == 0) L.pre[64] = total;
      L.pos[lane] = pos;
      L.src[lane] = it.lo | ((uint64_t)it.list << 63);
      __builtin_amdgcn_wave_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      for (uint32_t q = lane; q < total + 63 - (total + 63) % 64; q += 64) {  // (whole-wave steps)
        if (q < total) {
          uint32_t j = 0;  // the emission holding ref q: the largest j with pre[j] <= q
#pragma unroll
          for (uint32_t step = 32; step > 0; step >>= 1) j = L.pre[j + step] <= q ? j + step : j;
          const uint32_t o = q - L.pre[j];
          const uint64_t sw = L.src[j];
          put_ref<kNT>(out + L.pos[j] + o, ((sw >> 63) ? rch_refs : refs)[(sw & ~(1ull << 63)) + o]);
        }
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (!fits || cnt <= kSmallEmit) continue;
    const uint32_t nt = (uint32_t)((cnt + kTaskRefs - 1) / kTaskRefs);
    const unsigned long long t0 = atomicAdd(&ctr->n_tasks, (unsigned long long)nt);
    if (t0 + nt > task_cap) atomicOr(&ctr->ovf, (unsigned)kOvfTasks);
    // every slot below the capacity is written (k_task_copy reads them all)
    for (uint32_t k = 0; k < nt && t0 + k < task_cap; k++) {
      const uint32_t len = (uint32_t)min<uint64_t>(kTaskRefs, cnt - (uint64_t)k * kTaskRefs);
      tasks[t0 + k] = Task{pos + (uint64_t)k * kTaskRefs, it.lo + k * kTaskRefs, len | (it.list << 31)};
    }
  }
}

// a wavefront per copy task, grid-stride over the tasks k_emit_place queued
template <bool kNT>
__global__ __launch_bounds__(kThreads) void k_task_copy(const Task *__restrict__ tasks, uint64_t cap,
                                                       const RevCtr *ctr, const uint64_t *__restrict__ refs,
                                                       const uint64_t *__restrict__ rch_refs,
                                                       uint64_t *__restrict__ out) {
  if (ctr->ovf) return;  // this attempt is discarded (re-queued with larger lists)
  const uint64_t nt = min((uint64_t)ctr->n_tasks, cap);
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x / 64);
  const int lane = threadIdx.x & 63;
  for (uint64_t t = (uint64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; t < nt; t += nw) {
    const Task k = tasks[t];
    const uint32_t len = k.len_list & 0x7FFFFFFFu;
    const uint64_t *src = ((k.len_list >> 31) ? rch_refs : refs) + k.lo;
    uint64_t *dst = out + k.dst;
    uint32_t j = lane;
    for (; j + 192 < len; j += 256) {  // 4 loads in flight per lane
      const uint64_t a = src[j], b = src[j + 64], c = src[j + 128], d = src[j + 192];
      put_ref<kNT>(dst + j, a);
      put_ref<kNT>(dst + j + 64, b);
      put_ref<kNT>(dst + j + 128, c);
      put_ref<kNT>(dst + j + 192, d);
    }
    for (; j < len; j += 64) put_ref<kNT>(dst + j, src[j]);
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

// hipCUB accumulates in the input type: narrower counts are widened on the fly
// so the offsets never wrap at 2^32
template <class T>
struct WidenU64 {
  __host__ __device__ uint64_t operator()(T c) const { return (uint64_t)c; }
};

template <class T>
int scan_u64(Workspace &ws, const T *counts, uint64_t *offs, uint64_t n, hipStream_t st) {
  HIP_TRY(hipMemsetAsync(offs, 0, sizeof(uint64_t), st));
  if (n == 0) return 0;
  hipcub::TransformInputIterator<uint64_t, WidenU64<T>, const T *> in(counts, WidenU64<T>{});
  size_t tmp = 0;
  HIP_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, tmp, in, offs + 1, n, st));
  if (ws.get(Workspace::kScanTmp, tmp)) return -2;
  HIP_TRY(hipcub::DeviceScan::InclusiveSum(ws.ptr(Workspace::kScanTmp), tmp, in, offs + 1, n, st));
  return 0;
}

uint32_t blocks_for(uint64_t n, uint32_t threads = kThreads) {
  return (uint32_t)std::max<uint64_t>(1, (n + threads - 1) / threads);
}

// blocks of a grid-stride kernel: what stays resident on the device
uint32_t resident_grid() {
  static uint32_t g = 0;
  if (!g) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
      cus = 256;
    g = (uint32_t)cus * 8;  // 8 blocks of 256 threads = 32 waves per CU
  }
  return g;
}

size_t ctr_bytes(uint32_t levels) { return sizeof(RevCtr) + sizeof(unsigned long long) * (levels + 1); }

}  // namespace

int messages_device(const DeviceSnapshot &s, const DeviceRetained *r, Workspace &ws, const uint8_t *d_bytes,
                    const uint64_t *d_offs, uint32_t n, hipStream_t st, MessagesOutput *out) {
  using W = Workspace;
  *out = MessagesOutput();
  out->n_filters = n;
  if (ws.get(W::kROffs, sizeof(uint64_t) * (n + 1))) return -2;
  auto *foff = (uint64_t *)ws.ptr(W::kROffs);
  out->offsets = foff;
  if (!r || n == 0) {  // len(Retained) == 0: nothing matches (topics.go:436)
    HIP_TRY(hipMemsetAsync(foff, 0, sizeof(uint64_t) * (n + 1), st));
    HIP_TRY(hipStreamSynchronize(st));
    return 0;
  }
  if (ws.get(W::kRNLev, sizeof(uint32_t) * (n + 1)) || ws.get(W::kRWild, n + 1) ||
      ws.get(W::kRLOff, sizeof(uint64_t) * (n + 1)) || ws.get(W::kRFCount, sizeof(uint64_t) * (n + 1)) ||
      ws.get(W::kRFCur, sizeof(uint64_t) * (n + 1)))
    return -2;
  auto *nlev = (uint32_t *)ws.ptr(W::kRNLev);
  auto *wild = (uint8_t *)ws.ptr(W::kRWild);
  auto *loff = (uint64_t *)ws.ptr(W::kRLOff);
  uint64_t *hp = ws.pinned_u64();
  if (!hp) return -2;

  // the filters' levels: the one read-back before the walk sizes their array
  hipLaunchKernelGGL(k_flt_count, dim3(blocks_for(n)), dim3(kThreads), 0, st, d_bytes, d_offs, n, nlev, wild);
  HIP_TRY(hipGetLastError());
  if (scan_u64(ws, nlev, loff, n, st)) return -3;
  HIP_TRY(hipMemcpyAsync(hp, loff + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  const uint64_t total_levels = hp[0];
  if (ws.get(W::kRLevels, sizeof(Level) * (total_levels + 1))) return -2;
  auto *lv = (Level *)ws.ptr(W::kRLevels);
  hipLaunchKernelGGL(k_flt_fill, dim3(blocks_for(n)), dim3(kThreads), 0, st, d_bytes, d_offs, n, loff, lv);
  HIP_TRY(hipGetLastError());

  // every list starts at its size from the previous call (grown on overflow)
  uint64_t &item_cap = ws.rev_item_cap, &emit_cap = ws.rev_emit_cap, &task_cap = ws.rev_task_cap,
           &out_cap = ws.rev_out_cap, &ltask_cap = ws.rev_ltask_cap;
  static const bool use_ltasks = getenv("MQM_REV_TASKS") && atoi(getenv("MQM_REV_TASKS")) != 0;
  // MQM_REV_CAP0=k (tests): a fresh workspace starts every list at k entries,
  // so the first calls overflow and re-queue at every level
  const char *cap0_env = getenv("MQM_REV_CAP0");
  const uint64_t cap0 = cap0_env ? strtoull(cap0_env, nullptr, 10) : 0;
  if (cap0) {
    if (!item_cap) item_cap = emit_cap = task_cap = out_cap = ltask_cap = cap0;
  } else {
    item_cap = std::max<uint64_t>(item_cap, std::max<uint64_t>(4ull * n, 1u << 16));
    emit_cap = std::max<uint64_t>(emit_cap, std::max<uint64_t>(2ull * n, 1u << 16));
    task_cap = std::max<uint64_t>(task_cap, 1u << 12);
    ltask_cap = std::max<uint64_t>(ltask_cap, std::max<uint64_t>(n, 1u << 16));
    out_cap = std::max<uint64_t>(out_cap, std::max<uint64_t>(4ull * n, 1u << 16));
  }
  const uint32_t grid = resident_grid();
  for (int attempt = 0;; attempt++) {
    if (ws.get(W::kRItemF0, sizeof(uint32_t) * item_cap) || ws.get(W::kRItemN0, sizeof(uint32_t) * item_cap) ||
        ws.get(W::kRItemF1, sizeof(uint32_t) * item_cap) || ws.get(W::kRItemN1, sizeof(uint32_t) * item_cap) ||
        ws.get(W::kRChild, sizeof(uint32_t) * item_cap) || ws.get(W::kRECount, sizeof(uint32_t) * item_cap) ||
        ws.get(W::kREmit, sizeof(Emit) * emit_cap) || ws.get(W::kRChunks, sizeof(Task) * task_cap) ||
        ws.get(W::kROut, sizeof(uint64_t) * out_cap) ||
        (use_ltasks && ws.get(W::kRPos, sizeof(LTask) * ltask_cap)))
      return -2;
    // levels 0 .. height: an item of level d sits on a node of depth d
    const uint32_t max_levels = s.height + 1;
    const size_t st_at = (ctr_bytes(max_levels + 1) + 15) & ~size_t(15);
    const size_t st_bytes = sizeof(unsigned long long) * kStatLevels * kStatKinds;
    if (ws.get(W::kRNCount, st_at + st_bytes)) return -2;
    auto *ctr = (RevCtr *)ws.ptr(W::kRNCount);
    HIP_TRY(hipMemsetAsync(ctr, 0, st_at + st_bytes, st));
    HIP_TRY(hipMemsetAsync(ws.ptr(W::kRFCount), 0, sizeof(uint64_t) * (n + 1), st));
    HIP_TRY(hipMemsetAsync(ws.ptr(W::kRFCur), 0, sizeof(uint64_t) * (n + 1), st));
    LevelArgs a{};
    a.s = s;
    a.r = *r;
    a.bytes = d_bytes;
    a.offs = d_offs;
    a.loff = loff;
    a.nlev = nlev;
    a.wild = wild;
    a.lv = lv;
    a.n = n;
    a.item_cap = item_cap;
    a.emit = (Emit *)ws.ptr(W::kREmit);
    a.emit_cap = emit_cap;
    a.ctr = ctr;
    static const bool rev_stats = getenv("MQM_REV_STATS") && atoi(getenv("MQM_REV_STATS")) != 0;
    a.st = rev_stats ? reinterpret_cast<unsigned long long *>(reinterpret_cast<char *>(ctr) + st_at) : nullptr;
    a.ltasks = use_ltasks ? (LTask *)ws.ptr(W::kRPos) : nullptr;
    a.ltask_cap = use_ltasks ? ltask_cap : 0;
    // level L's list lives in buffer pair L % 3 (a level appends to the next
    // two: wildcard + literal through the edge index jumps one level)
    const W::Slot lf[3] = {W::kRItemF0, W::kRItemF1, W::kRChild}, ln[3] = {W::kRItemN0, W::kRItemN1, W::kRECount};
    for (uint32_t d = 0; d < max_levels; d++) {
      a.d = d;
      a.item_f = (const uint32_t *)ws.ptr(lf[d % 3]);
      a.item_n = (const uint32_t *)ws.ptr(ln[d % 3]);
      a.next_f = (uint32_t *)ws.ptr(lf[(d + 1) % 3]);
      a.next_n = (uint32_t *)ws.ptr(ln[(d + 1) % 3]);
      a.skip_f = (uint32_t *)ws.ptr(lf[(d + 2) % 3]);
      a.skip_n = (uint32_t *)ws.ptr(ln[(d + 2) % 3]);
      const uint32_t g = d == 0 ? std::min<uint32_t>(grid, blocks_for(n)) : grid;
      if (a.ltasks) HIP_TRY(hipMemsetAsync(&ctr->n_ltasks, 0, sizeof(unsigned long long), st));
      hipLaunchKernelGGL(k_level, dim3(g), dim3(kThreads), 0, st, a);
      HIP_TRY(hipGetLastError());
      if (a.ltasks) {
        hipLaunchKernelGGL(k_level_tasks, dim3(grid), dim3(kThreads), 0, st, a);
        HIP_TRY(hipGetLastError());
      }
      // every kLevelBatch levels, stop early once the next two levels are empty
      if ((d + 1) % kLevelBatch == 0 && d + 1 < max_levels) {
        HIP_TRY(hipMemcpyAsync(hp, &ctr->items[d + 1], 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        if (hp[0] == 0 && hp[1] == 0) break;
      }
    }
    // emissions -> per-filter CSR
    auto *fcount = (unsigned long long *)ws.ptr(W::kRFCount);
    hipLaunchKernelGGL(k_emit_count, dim3(grid), dim3(kThreads), 0, st, a.emit, emit_cap, ctr, fcount,
                       max_levels);
    HIP_TRY(hipGetLastError());
    if (scan_u64(ws, (const uint64_t *)fcount, foff, n, st)) return -3;
    auto *refs_out = (uint64_t *)ws.ptr(W::kROut);
    auto *tasks = (Task *)ws.ptr(W::kRChunks);
    static const bool nt_refs = !getenv("MQM_REV_NT") || atoi(getenv("MQM_REV_NT")) != 0;
    hipLaunchKernelGGL(nt_refs ? k_emit_place<true> : k_emit_place<false>, dim3(grid), dim3(kThreads), 0, st, a.emit,
                       emit_cap, ctr, foff, (unsigned long long *)ws.ptr(W::kRFCur), r->refs, r->rch_refs, refs_out,
                       out_cap, tasks, task_cap);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(nt_refs ? k_task_copy<true> : k_task_copy<false>, dim3(grid), dim3(kThreads), 0, st, tasks,
                       task_cap, ctr, r->refs, r->rch_refs, refs_out);
    HIP_TRY(hipGetLastError());
    // the one read-back: sizes and overflow flags
    RevCtr *hc = reinterpret_cast<RevCtr *>(hp);
    static_assert(sizeof(RevCtr) + 8 <= 128, "pinned read-back area");
    HIP_TRY(hipMemcpyAsync(hc, ctr, sizeof(RevCtr), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(hp + 15, foff + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const uint64_t n_refs = hp[15];
    const unsigned ovf = hc->ovf;
    const uint64_t n_emit = hc->n_emit, n_tasks = hc->n_tasks, need_items = hc->need_items,
                   need_ltasks = hc->need_ltasks;
    if (ovf == 0 && a.st) {
      unsigned long long sv[kStatLevels * kStatKinds];
      HIP_TRY(hipMemcpy(sv, a.st, sizeof(sv), hipMemcpyDeviceToHost));
      fprintf(stderr, "[rev-stats] level live literal expand_children index_edges emissions\n");
      for (uint32_t d = 0; d < std::min<uint32_t>(max_levels, kStatLevels); d++)
        fprintf(stderr, "[rev-stats] %u %llu %llu %llu %llu %llu\n", d, sv[d * kStatKinds], sv[d * kStatKinds + 1],
                sv[d * kStatKinds + 2], sv[d * kStatKinds + 3], sv[d * kStatKinds + 4]);
    }
    if (ovf == 0) {
      out->n_refs = n_refs;
      out->refs = refs_out;
      out->n_emissions = n_emit;
      out->n_items = hc->items_total + n;  // level 0 = one item per filter
      out->n_skipped = hc->skipped;
      return 0;
    }
    if (attempt >= 64) return -3;  // (the counters only ever grow: never reached)
    // re-queue with the sizes this attempt needed (its later levels may have
    // been cut short, so another round can still grow them)
    if (ovf & kOvfItems) item_cap = std::max(item_cap, need_items + need_items / 4);
    if (ovf & kOvfEmit) emit_cap = std::max(emit_cap, n_emit + n_emit / 4);
    if (ovf & kOvfTasks) task_cap = std::max(task_cap, n_tasks + n_tasks / 4);
    if (ovf & kOvfOut) out_cap = std::max(out_cap, n_refs + n_refs / 4);
    if (ovf & kOvfLTasks) ltask_cap = std::max(ltask_cap, need_ltasks + need_ltasks / 4);
  }
}

}  // namespace mqm
