// maxmq_amd/csrc/retained.hip — gfx950 kernels for TopicsIndex.Messages
// (vendor/github.com/mochi-co/mqtt/v2/topics.go:426-480): a batch of
// subscription filters against the retained topics of the snapshot.
//
// The reference recurses per filter (scanMessages).  Here the recursion is
// unrolled level-synchronously over the whole batch, as worklists of
// (filter, node) items in HBM, so wildcard fan-out never overflows a
// per-filter buffer and every level is a balanced launch:
//   k_flt_levels   a thread per filter: split into levels (isolateParticle,
//                  topics.go:558-577), 128-bit level keys, wildcard flag
//   k_bfs<count|fill>  a thread per item of level d: the reference's three
//                  cases (topics.go:447-477) —
//                    literal : one edge probe (the forward matcher's table)
//                    '+'/'#' with more levels: every child (minus "$SYS" at
//                             the root, :450) becomes an item of level d+1
//                    '+' last : the node's retained children      (:454-460)
//                    '#' last : every retained node below it      (:462, the
//                             recursion keeps isolating the last level)
//                    literal last: the child's retained message, or — only
//                             for wildcard filters — the message retained at
//                             topic "" (Retained.Get(""), :474)
//                  emissions are (filter, list, lo, hi) ranges of message refs:
//                  subtrees are contiguous in preorder (snapshot.h)
//   k_emit_*       ranges -> per-filter CSR of message refs, copied in
//                  fixed-size chunks so one huge '#' range is spread over
//                  many wavefronts
// Exact filters (no '+'/'#', :440-445) are the literal walk of the same items
// with Retained.Get(filter) semantics (no "" fallback).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "device.h"
#include "retained.h"

namespace mqm {

namespace {

constexpr uint32_t kEmitChunk = 4096;  // refs copied per wavefront task
constexpr uint32_t kSmallEmit = 32;    // emissions up to this size: copied by one thread

struct Level {         // one level of one filter
  uint64_t k0, k1;     // key (keys.h)
  uint32_t start, len; // byte range within the filter
};

enum : uint32_t { kTypeLiteral = 0, kTypePlus = 1, kTypeHash = 2 };

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

struct BfsArgs {
  DeviceSnapshot s;
  DeviceRetained r;
  const uint8_t *bytes;
  const uint64_t *offs;
  const uint64_t *loff;
  const uint32_t *nlev;
  const uint8_t *wild;
  const Level *lv;
  uint32_t d;
  uint64_t n_items;
  const uint32_t *item_f, *item_n;  // items of level d
  uint32_t *child;                  // literal probe result (count pass -> fill pass)
  uint32_t *ncount, *ecount;        // count pass outputs
  const uint64_t *noff, *eoff;      // fill pass: exclusive scans of the above
  uint32_t *next_f, *next_n;        // fill pass: items of level d + 1
  Emit *emit;                       // fill pass: emissions (already offset by the running base)
};

__device__ __forceinline__ bool retained_node(const DeviceRetained &r, uint32_t c) {
  return r.cum[c + 1] > r.cum[c];
}

// kFill == false: count next items / emissions; true: write them
template <bool kFill>
__global__ void k_bfs(BfsArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n_items) return;
  const uint32_t f = a.item_f[i], p = a.item_n[i];
  const uint32_t L = a.nlev[f];
  const Level l = a.lv[a.loff[f] + a.d];
  const bool has_next = a.d + 1 < L;
  const uint32_t type = a.wild[f] ? level_type(l) : kTypeLiteral;
  const DeviceRetained &r = a.r;
  uint32_t nn = 0, ne = 0;
  uint64_t nb = 0, eb = 0;
  if (kFill) {
    nb = a.noff[i];
    eb = a.eoff[i];
  }
  auto emit = [&](uint32_t list, uint32_t lo, uint32_t hi) {
    if (hi <= lo) return;
    if (kFill) a.emit[eb + ne] = Emit{f, list, lo, hi};
    ne++;
  };
  if (type == kTypeLiteral) {  // topics.go:469-477 (and :440-445 for exact filters)
    uint32_t c;
    if (kFill) {
      c = a.child[i];
    } else {
      NodeDesc dc;
      c = probe_edge(a.s, p, l.k0, l.k1, a.bytes + a.offs[f] + l.start, l.len, &dc);
      a.child[i] = c;
    }
    if (c != kNone) {
      if (has_next) {
        if (kFill) {
          a.next_f[nb] = f;
          a.next_n[nb] = c;
        }
        nn = 1;
      } else if (retained_node(r, c)) {
        emit(0, r.cum[c], r.cum[c] + 1);
      } else if (a.wild[f] && r.has_empty) {  // Retained.Get("") through an empty retainPath
        emit(0, (uint32_t)r.n_ret, (uint32_t)r.n_ret + 1);
      }
    }
  } else if (has_next) {  // '+' or '#' followed by more levels: recurse into every child (:449-465)
    const uint32_t skip = a.d == 0 ? r.sys_child : kNone;
    for (uint32_t j = r.child_off[p]; j < r.child_off[p + 1]; j++) {
      const uint32_t c = r.child_ids[j];
      if (c == skip) continue;
      if (kFill) {
        a.next_f[nb + nn] = f;
        a.next_n[nb + nn] = c;
      }
      nn++;
    }
  } else if (type == kTypePlus) {  // the retained children (root's list excludes "$SYS")
    emit(1, r.rch_off[p], r.rch_off[p + 1]);
  } else {  // '#' last: the subtree below p, "$SYS" skipped at the root (:450)
    const uint32_t end = p + r.subtree[p];
    if (a.d == 0 && r.sys_child != kNone) {
      const uint32_t sys = r.sys_child;
      emit(0, r.cum[p + 1], r.cum[sys]);
      emit(0, r.cum[sys + r.subtree[sys]], r.cum[end]);
    } else {
      emit(0, r.cum[p + 1], r.cum[end]);
    }
  }
  if (!kFill) {
    a.ncount[i] = nn;
    a.ecount[i] = ne;
  }
}

__global__ void k_init_items(uint32_t n, const uint32_t *__restrict__ nlev, uint32_t *__restrict__ item_f,
                             uint32_t *__restrict__ item_n, const uint64_t *__restrict__ pos) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n || nlev[f] == 0) return;
  item_f[pos[f]] = f;
  item_n[pos[f]] = 0;
}

__global__ void k_has_levels(uint32_t n, const uint32_t *__restrict__ nlev, uint32_t *__restrict__ flag) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f < n) flag[f] = nlev[f] ? 1u : 0u;
}

// Emissions of one filter are adjacent (every level's items and emissions
// stay in filter order), so a wavefront folds each run of equal filter ids
// (segmented scan over the lanes) and issues one atomic per run.
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

__global__ __launch_bounds__(256) void k_emit_count(uint64_t ne, const Emit *__restrict__ e,
                                                   unsigned long long *__restrict__ fcount) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool ok = i < ne;
  const uint32_t f = ok ? e[i].f : 0xFFFFFFFFu;
  const uint64_t cnt = ok ? e[i].hi - e[i].lo : 0;
  const Run r = fold_runs(f, cnt);
  if (ok && r.last) atomicAdd(&fcount[f], (unsigned long long)r.inc);
}

__global__ __launch_bounds__(256) void k_emit_pos(uint64_t ne, const Emit *__restrict__ e,
                                                 const uint64_t *__restrict__ foff,
                                                 unsigned long long *__restrict__ fcur, uint64_t *__restrict__ pos,
                                                 uint32_t *__restrict__ chunks) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool ok = i < ne;
  const uint32_t f = ok ? e[i].f : 0xFFFFFFFFu;
  const uint64_t cnt = ok ? e[i].hi - e[i].lo : 0;
  const Run r = fold_runs(f, cnt);
  unsigned long long base = 0;
  if (ok && r.last) base = foff[f] + atomicAdd(&fcur[f], (unsigned long long)r.inc);
  const uint32_t blo = __shfl((uint32_t)base, r.last_lane, 64), bhi = __shfl((uint32_t)(base >> 32), r.last_lane, 64);
  const uint32_t tlo = __shfl((uint32_t)r.inc, r.last_lane, 64), thi = __shfl((uint32_t)(r.inc >> 32), r.last_lane, 64);
  if (!ok) return;
  const uint64_t run_base = ((uint64_t)bhi << 32) | blo, run_total = ((uint64_t)thi << 32) | tlo;
  (void)run_total;
  pos[i] = run_base + (r.inc - cnt);
  chunks[i] = cnt > kSmallEmit ? (uint32_t)((cnt + kEmitChunk - 1) / kEmitChunk) : 0u;
}

// emissions of <= kSmallEmit refs: a thread each
__global__ __launch_bounds__(256) void k_emit_small(uint64_t ne, const Emit *__restrict__ e,
                                                   const uint64_t *__restrict__ pos,
                                                   const uint64_t *__restrict__ refs,
                                                   const uint64_t *__restrict__ rch_refs, uint64_t *__restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ne) return;
  const Emit it = e[i];
  const uint32_t cnt = it.hi - it.lo;
  if (cnt > kSmallEmit) return;
  const uint64_t *src = (it.list ? rch_refs : refs) + it.lo;
  uint64_t *dst = out + pos[i];
  for (uint32_t j = 0; j < cnt; j++) dst[j] = src[j];
}

// larger emissions: a wavefront per chunk of kEmitChunk refs
__global__ __launch_bounds__(256) void k_emit_fill(uint64_t ne, uint64_t nchunks, const Emit *__restrict__ e,
                                                  const uint64_t *__restrict__ pos, const uint64_t *__restrict__ coff,
                                                  const uint64_t *__restrict__ refs,
                                                  const uint64_t *__restrict__ rch_refs, uint64_t *__restrict__ out) {
  const int lane = threadIdx.x & 63;
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x / 64);
  for (uint64_t c = (uint64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; c < nchunks; c += nw) {
    uint64_t lo = 0, hi = ne;  // item i with coff[i] <= c < coff[i + 1]
    while (hi - lo > 1) {
      const uint64_t mid = (lo + hi) / 2;
      if (coff[mid] <= c) lo = mid;
      else hi = mid;
    }
    const Emit it = e[lo];
    const uint64_t k0 = (c - coff[lo]) * kEmitChunk;
    const uint64_t cnt = std::min<uint64_t>(kEmitChunk, (uint64_t)(it.hi - it.lo) - k0);
    const uint64_t *src = (it.list ? rch_refs : refs) + it.lo + k0;
    uint64_t *dst = out + pos[lo] + k0;
    for (uint64_t j = lane; j < cnt; j += 64) dst[j] = src[j];
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

uint32_t blocks_for(uint64_t n, uint32_t threads = 256) { return (uint32_t)std::max<uint64_t>(1, (n + threads - 1) / threads); }

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
  auto *fcount = (uint64_t *)ws.ptr(W::kRFCount);
  auto *fcur = (uint64_t *)ws.ptr(W::kRFCur);
  uint64_t *hp = ws.pinned_u64();
  if (!hp) return -2;

  hipLaunchKernelGGL(k_flt_count, dim3(blocks_for(n)), dim3(256), 0, st, d_bytes, d_offs, n, nlev, wild);
  HIP_TRY(hipGetLastError());
  if (scan_u64(ws, nlev, loff, n, st)) return -3;
  HIP_TRY(hipMemcpyAsync(hp, loff + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  const uint64_t total_levels = hp[0];
  if (ws.get(W::kRLevels, sizeof(Level) * (total_levels + 1))) return -2;
  auto *lv = (Level *)ws.ptr(W::kRLevels);
  hipLaunchKernelGGL(k_flt_fill, dim3(blocks_for(n)), dim3(256), 0, st, d_bytes, d_offs, n, loff, lv);
  HIP_TRY(hipGetLastError());

  // level-0 items: (f, root) for every non-empty filter, in filter order
  if (ws.get(W::kRNCount, sizeof(uint32_t) * (n + 1)) || ws.get(W::kRNOff, sizeof(uint64_t) * (n + 2))) return -2;
  {
    auto *flag = (uint32_t *)ws.ptr(W::kRNCount);
    auto *pos = (uint64_t *)ws.ptr(W::kRNOff);
    hipLaunchKernelGGL(k_has_levels, dim3(blocks_for(n)), dim3(256), 0, st, n, nlev, flag);
    if (scan_u64(ws, flag, pos, n, st)) return -3;
    HIP_TRY(hipMemcpyAsync(hp, pos + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (ws.get(W::kRItemF0, sizeof(uint32_t) * (hp[0] + 1)) || ws.get(W::kRItemN0, sizeof(uint32_t) * (hp[0] + 1)))
      return -2;
    hipLaunchKernelGGL(k_init_items, dim3(blocks_for(n)), dim3(256), 0, st, n, nlev, (uint32_t *)ws.ptr(W::kRItemF0),
                       (uint32_t *)ws.ptr(W::kRItemN0), pos);
    HIP_TRY(hipGetLastError());
  }
  uint64_t n_items = hp[0];
  uint64_t n_emit = 0, items_total = 0;
  W::Slot cur_f = W::kRItemF0, cur_n = W::kRItemN0, nxt_f = W::kRItemF1, nxt_n = W::kRItemN1;
  for (uint32_t d = 0; n_items > 0; d++) {
    if (ws.get(W::kRChild, sizeof(uint32_t) * (n_items + 1)) || ws.get(W::kRNCount, sizeof(uint32_t) * (n_items + 1)) ||
        ws.get(W::kRECount, sizeof(uint32_t) * (n_items + 1)) || ws.get(W::kRNOff, sizeof(uint64_t) * (n_items + 1)) ||
        ws.get(W::kREOff, sizeof(uint64_t) * (n_items + 1)))
      return -2;
    BfsArgs a{};
    a.s = s;
    a.r = *r;
    a.bytes = d_bytes;
    a.offs = d_offs;
    a.loff = loff;
    a.nlev = nlev;
    a.wild = wild;
    a.lv = lv;
    a.d = d;
    a.n_items = n_items;
    a.item_f = (const uint32_t *)ws.ptr(cur_f);
    a.item_n = (const uint32_t *)ws.ptr(cur_n);
    a.child = (uint32_t *)ws.ptr(W::kRChild);
    a.ncount = (uint32_t *)ws.ptr(W::kRNCount);
    a.ecount = (uint32_t *)ws.ptr(W::kRECount);
    hipLaunchKernelGGL(k_bfs<false>, dim3(blocks_for(n_items)), dim3(256), 0, st, a);
    HIP_TRY(hipGetLastError());
    auto *noff = (uint64_t *)ws.ptr(W::kRNOff);
    auto *eoff = (uint64_t *)ws.ptr(W::kREOff);
    if (scan_u64(ws, a.ncount, noff, n_items, st) || scan_u64(ws, a.ecount, eoff, n_items, st)) return -3;
    HIP_TRY(hipMemcpyAsync(hp, noff + n_items, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(hp + 1, eoff + n_items, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const uint64_t nn = hp[0], ne = hp[1];
    if (ws.get(nxt_f, sizeof(uint32_t) * (nn + 1)) || ws.get(nxt_n, sizeof(uint32_t) * (nn + 1)) ||
        ws.grow_keep(W::kREmit, sizeof(Emit) * n_emit, sizeof(Emit) * (n_emit + ne + 1), st))
      return -2;
    a.item_f = (const uint32_t *)ws.ptr(cur_f);  // (unchanged slots; pointers re-read after growth)
    a.item_n = (const uint32_t *)ws.ptr(cur_n);
    a.noff = noff;
    a.eoff = eoff;
    a.next_f = (uint32_t *)ws.ptr(nxt_f);
    a.next_n = (uint32_t *)ws.ptr(nxt_n);
    a.emit = (Emit *)ws.ptr(W::kREmit) + n_emit;
    hipLaunchKernelGGL(k_bfs<true>, dim3(blocks_for(n_items)), dim3(256), 0, st, a);
    HIP_TRY(hipGetLastError());
    n_emit += ne;
    items_total += n_items;
    n_items = nn;
    std::swap(cur_f, nxt_f);
    std::swap(cur_n, nxt_n);
  }

  // emissions -> per-filter CSR
  auto *emit = (Emit *)ws.ptr(W::kREmit);
  HIP_TRY(hipMemsetAsync(fcount, 0, sizeof(uint64_t) * (n + 1), st));
  HIP_TRY(hipMemsetAsync(fcur, 0, sizeof(uint64_t) * (n + 1), st));
  if (n_emit)
    hipLaunchKernelGGL(k_emit_count, dim3(blocks_for(n_emit)), dim3(256), 0, st, n_emit, emit,
                       (unsigned long long *)fcount);
  HIP_TRY(hipGetLastError());
  if (scan_u64(ws, fcount, foff, n, st)) return -3;
  if (ws.get(W::kRPos, sizeof(uint64_t) * (n_emit + 1)) || ws.get(W::kRChunks, sizeof(uint32_t) * (n_emit + 1)) ||
      ws.get(W::kRCOff, sizeof(uint64_t) * (n_emit + 1)))
    return -2;
  auto *pos = (uint64_t *)ws.ptr(W::kRPos);
  auto *chunks = (uint32_t *)ws.ptr(W::kRChunks);
  auto *coff = (uint64_t *)ws.ptr(W::kRCOff);
  if (n_emit)
    hipLaunchKernelGGL(k_emit_pos, dim3(blocks_for(n_emit)), dim3(256), 0, st, n_emit, emit, foff,
                       (unsigned long long *)fcur, pos, chunks);
  HIP_TRY(hipGetLastError());
  if (scan_u64(ws, chunks, coff, n_emit, st)) return -3;
  HIP_TRY(hipMemcpyAsync(hp, foff + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(hp + 1, coff + n_emit, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  const uint64_t n_refs = hp[0], nchunks = hp[1];
  if (ws.get(W::kROut, sizeof(uint64_t) * (n_refs + 1))) return -2;
  auto *refs_out = (uint64_t *)ws.ptr(W::kROut);
  if (n_emit)
    hipLaunchKernelGGL(k_emit_small, dim3(blocks_for(n_emit)), dim3(256), 0, st, n_emit, emit, pos, r->refs,
                       r->rch_refs, refs_out);
  HIP_TRY(hipGetLastError());
  if (nchunks)
    hipLaunchKernelGGL(k_emit_fill, dim3((uint32_t)std::min<uint64_t>((nchunks + 3) / 4, 8192)), dim3(256), 0, st,
                       n_emit, nchunks, emit, pos, coff, r->refs, r->rch_refs, refs_out);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(st));
  out->n_refs = n_refs;
  out->refs = refs_out;
  out->n_emissions = n_emit;
  out->n_items = items_total;
  return 0;
}

}  // namespace mqm
