// maxmq_amd/csrc/match.hip — gfx950 kernels for TopicsIndex.Subscribers
// (vendor/github.com/mochi-co/mqtt/v2/topics.go:484-555) over a batch of
// publish topics, against the GPU-resident CSR level-trie (snapshot.h).
//
// One pass over the trie per topic:
//   k_walk    one wavefront per topic (grid-stride).
//     1. tokenize : 64 lanes scan the topic bytes and ballot the '/'
//                   positions; lane k builds level k's 128-bit key (keys.h).
//     2. walk     : level-synchronous over the frontier; each frontier node
//                   fans out to 3 lanes (literal edge probe / '+' child /
//                   '#' child) so a level costs one dependent memory round
//                   trip (the literal child's descriptor is inline in its
//                   edge entry).  Hits and the next frontier are compacted
//                   with ballot + popcount into LDS.
//     3. order    : hits sorted by rank (= the reference's emission order,
//                   snapshot.h) with a 32-lane bitonic network in registers.
//     4. dedupe   : small topics (<= kSMax raw entries) in a per-wave LDS
//                   hash table keyed by client; one atomicOr folds max QoS
//                   (one-hot), NoLocal and the hit's rank (one-hot), i.e.
//                   Subscription.Merge (packets.go:250-270).  The entry whose
//                   hit is its client's lowest rank is the first-merged sub.
//                   Winners are compacted with ballot and written through a
//                   per-wave chunk allocator (no per-topic atomics).
//                   Bigger topics leave their sorted hit list in a record.
//   k_big     one 256-thread workgroup per record: the same dedupe in a
//             64 KiB LDS table shared by 4 waves.
//   k_dfs<P>  the unbounded path for topics that exceed a capacity (frontier,
//             hits, cached levels, raw entries): a wave-cooperative DFS with an
//             LDS stack and a global-memory dedupe table.
//   k_compact raw chunks -> topic-ordered CSR at the scanned offsets.
// Nothing runs on the CPU.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>

#include "match.h"

namespace mqm {

namespace {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kLMax = 16;      // levels cached per topic on the wave path
constexpr int kFCap = 32;      // frontier nodes per level
constexpr int kHCap = 28;      // non-shared hits (rank one-hot uses bits 4..31)
constexpr int kShCap = 32;     // shared hits
constexpr int kTCap = 512;     // per-wave dedupe table slots
constexpr int kSMax = 384;     // raw entries deduplicated per wave (load <= 0.75)
constexpr int kBigThreads = 256;
constexpr int kBigSlots = 8192;   // per-workgroup table: 64 KiB of LDS
constexpr int kBigMax = 6144;     // raw entries deduplicated per workgroup (load <= 0.75)
constexpr int kRecWords = 64;     // big-topic record: t, nh, S, -, off[28], pre[29]
constexpr uint32_t kNoTopic = 0xFFFFFFFFu;
constexpr uint64_t kNoSpace = ~0ull;

static_assert(kSMax * 4 <= kTCap * 3, "wave dedupe table load factor");
static_assert(kBigMax * 4 <= kBigSlots * 3, "workgroup dedupe table load factor");

enum : uint8_t { kTierDone = 0, kTierBig = 1, kTierDfs = 2 };

struct Counters {              // zeroed before every batch
  unsigned long long dpos;     // deliveries bump pointer (entries)
  unsigned long long hpos;     // shared candidates bump pointer
  unsigned long long bpos;     // big-topic records bump pointer
  unsigned long long miss[3];  // entries requested after a buffer ran out (sizes the retry)
  unsigned int n_dfs;          // topics appended to the DFS list
  unsigned int overflow;       // 1: deliveries, 2: shared, 4: records
};

struct Caps {
  uint64_t dcap, hcap, bcap;
  uint32_t dchunk, hchunk, bchunk;
};

struct WaveLds {
  uint64_t key0[kLMax];
  uint64_t key1[kLMax];
  uint32_t sep[kLMax];           // position of the '/' ending level k
  uint32_t front[2][3][kFCap];   // (node, plus, hash) of the frontier
  uint32_t hit_rank[32];
  uint32_t hit_off[32];
  uint32_t hit_pre[33];
  uint32_t sh_off[kShCap];
  uint32_t sh_cnt[kShCap];
  uint32_t tkey[kTCap];
  uint32_t tval[kTCap];
};

__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint64_t lanemask_lt(int lane) { return (1ull << lane) - 1ull; }

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
  const uint32_t lo = __shfl((uint32_t)v, src, 64), hi = __shfl((uint32_t)(v >> 32), src, 64);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ NodeDesc load_desc(const NodeDesc *p) {
  const uint4 *q = reinterpret_cast<const uint4 *>(p);
  uint4 a = q[0], b = q[1];
  NodeDesc d;
  d.plus = a.x;
  d.hash = a.y;
  d.sub_off = a.z;
  d.sub_cnt = a.w;
  d.hsub_off = b.x;
  d.hsub_cnt = b.y;
  d.sh_off = b.z;
  d.sh_cnt_flags = b.w;
  return d;
}

// Literal child lookup: open-addressed edge table, 2 entries per 128-B bucket.
// Long keys (>= 16 bytes) are verified byte-for-byte against the token pool.
__device__ uint32_t probe_edge(const DeviceSnapshot &s, uint32_t parent, uint64_t k0, uint64_t k1,
                               const uint8_t *tok, uint32_t tok_len, NodeDesc *desc) {
  const uint64_t nslots = (s.bucket_mask + 1) * kEdgesPerBucket;
  Key key{k0, k1};
  uint64_t slot = (edge_hash(parent, key) & s.bucket_mask) * kEdgesPerBucket;
  for (;;) {
    const EdgeEntry *e = s.edges + slot;
    const ulonglong2 kk = *reinterpret_cast<const ulonglong2 *>(e);
    const uint4 pc = *reinterpret_cast<const uint4 *>(&e->parent);
    if (pc.x == kNone) return kNone;
    if (pc.x == parent && kk.x == k0 && kk.y == k1) {
      bool ok = true;
      if (key_is_long(key)) {
        ok = pc.w == tok_len;
        for (uint32_t i = 0; ok && i < tok_len; i++) ok = s.tok_pool[pc.z + i] == tok[i];
      }
      if (ok) {
        *desc = load_desc(&e->desc);
        return pc.y;
      }
    }
    slot = (slot + 1) & (nslots - 1);
  }
}

__device__ __forceinline__ uint32_t table_slot(uint32_t client, uint32_t lg) {
  return (uint32_t)(((uint64_t)(client * 2654435769u) << lg) >> 32);
}

__device__ __forceinline__ uint64_t pack_delivery(uint32_t client, uint32_t sid, uint32_t qos, uint32_t nl) {
  return (uint64_t)client | ((uint64_t)(sid | (qos << 28) | (nl << 30)) << 32);
}

__device__ __forceinline__ uint32_t merge_bits(uint32_t h, uint32_t meta) {
  return (1u << (4 + h)) | (1u << (meta & 3)) | (((meta >> 2) & 1) << 3);
}

// hit h with pre[h] <= r < pre[h+1] (pre strictly increasing: empty hits are never recorded)
__device__ __forceinline__ uint32_t find_hit(const uint32_t *pre, uint32_t nh, uint32_t r) {
  uint32_t h = 0;
  for (uint32_t step = 16; step > 0; step >>= 1)
    if (h + step < nh && pre[h + step] <= r) h += step;
  return h;
}

// Per-wave bump allocation from a global counter in chunks (wave-uniform).
// Once the buffer is exhausted the wave only tallies what it still needed.
struct WaveAlloc {
  uint64_t cur = 0, end = 0;
  bool dead = false;
};

__device__ uint64_t wave_alloc(WaveAlloc &a, uint64_t need, unsigned long long *counter, uint64_t cap, uint32_t chunk,
                               Counters *ctr, unsigned int which, int lane) {
  if (need == 0) return 0;
  if (!a.dead && a.cur + need > a.end) {
    const uint64_t grab = need > chunk ? need : chunk;
    uint64_t base = 0;
    if (lane == 0) base = atomicAdd(counter, (unsigned long long)grab);
    base = shfl64(base, 0);
    a.cur = base;
    a.end = base + grab;
    if (a.end > cap) {
      if (lane == 0) atomicOr(&ctr->overflow, 1u << which);
      a.dead = true;
    }
  }
  if (a.dead) {
    if (lane == 0) atomicAdd(&ctr->miss[which], (unsigned long long)need);
    return kNoSpace;
  }
  const uint64_t r = a.cur;
  a.cur += need;
  return r;
}

// Bitonic sort of 32 (rank, off, cnt) triples held by lanes 0..31 (lanes
// 32..63 sort their own copy, harmlessly).  Ascending by rank.
__device__ __forceinline__ void sort32(int lane, uint32_t &rank, uint32_t &off, uint32_t &cnt) {
  for (int k = 2; k <= 32; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      uint32_t r2 = __shfl_xor(rank, j, 64);
      uint32_t o2 = __shfl_xor(off, j, 64);
      uint32_t c2 = __shfl_xor(cnt, j, 64);
      const bool up = (lane & k) == 0;
      const bool lower = (lane & j) == 0;
      const bool take_other = (lower == up) ? (r2 < rank) : (r2 > rank);
      if (take_other) {
        rank = r2;
        off = o2;
        cnt = c2;
      }
    }
  }
}

struct Outputs {
  uint32_t *dcount, *hcount;
  uint64_t *dstart, *hstart;
  uint8_t *tier;
  uint32_t *dfs_list;
  Counters *ctr;
  uint64_t *dbuf;
  uint32_t *hbuf;
  uint32_t *recs;
};

// ---------------------------------------------------------------------------
// k_walk: tokenize + walk + (small topics) dedupe, one wavefront per topic
// ---------------------------------------------------------------------------
// 6 blocks/CU (LDS: 6 x 23 KiB) => 6 waves per SIMD => <= 80 VGPRs
__global__ __launch_bounds__(kWave *kWavesPerBlock, 6) void k_walk(DeviceSnapshot s, const uint8_t *__restrict__ tbytes,
                                                               const uint64_t *__restrict__ toffs, uint32_t n,
                                                               Outputs o, Caps caps) {
  __shared__ WaveLds lds_all[kWavesPerBlock];
  const int lane = threadIdx.x & (kWave - 1);
  const int wib = threadIdx.x / kWave;
  WaveLds &L = lds_all[wib];
  const uint32_t nwaves = gridDim.x * kWavesPerBlock;
  WaveAlloc da, ha, ba;

  for (uint32_t t = blockIdx.x * kWavesPerBlock + wib; t < n; t += nwaves) {
    const uint64_t off = toffs[t];
    const uint32_t len = (uint32_t)(toffs[t + 1] - off);
    const uint8_t *tp = tbytes + off;
    if (len == 0) {  // scanSubscribers returns at once (topics.go:498-500)
      if (lane == 0) {
        o.dcount[t] = 0;
        o.hcount[t] = 0;
        o.dstart[t] = 0;
        o.hstart[t] = 0;
        o.tier[t] = kTierDone;
      }
      continue;
    }
    bool overflow = false;

    // ---- 1. tokenize ------------------------------------------------------
    uint32_t nsep = 0;
    bool dollar = false;
    for (uint32_t base = 0; base < len && nsep < (uint32_t)kLMax; base += kWave) {
      const uint32_t p = base + lane;
      const uint8_t b = p < len ? tp[p] : 0;
      if (base == 0) dollar = __shfl(b, 0, 64) == '$';
      const uint64_t m = __ballot(p < len && b == '/');
      if (b == '/' && p < len) {
        const uint32_t idx = nsep + __popcll(m & lanemask_lt(lane));
        if (idx < (uint32_t)kLMax) L.sep[idx] = p;
      }
      nsep += __popcll(m);
    }
    // levels known: 0 .. nlev-1, with nlev capped at kLMax + 1
    const uint32_t nlev = nsep >= (uint32_t)kLMax ? kLMax + 1 : nsep + 1;
    wave_lds_sync();
    if (lane < kLMax && (uint32_t)lane < nlev) {
      const uint32_t st = lane == 0 ? 0 : L.sep[lane - 1] + 1;
      const uint32_t en = ((uint32_t)lane < nsep) ? L.sep[lane] : len;
      Key k = make_key([&](uint32_t i) { return tp[st + i]; }, en - st);
      L.key0[lane] = k.k0;
      L.key1[lane] = k.k1;
    }
    wave_lds_sync();

    // ---- 2. walk ----------------------------------------------------------
    uint32_t nf = 1, nh = 0, nsh = 0;
    int cur = 0;
    if (lane == 0) {
      const NodeDesc r = load_desc(s.nodes);
      L.front[0][0][0] = 0;
      L.front[0][1][0] = r.plus;
      L.front[0][2][0] = r.hash;
    }
    wave_lds_sync();
    for (uint32_t d = 0; d < nlev && nf > 0 && !overflow; d++) {
      if (d >= (uint32_t)kLMax) {
        overflow = true;
        break;
      }
      const uint64_t k0 = L.key0[d], k1 = L.key1[d];
      const bool has_next = d + 1 < nlev;
      // key == "+" / "#": the literal probe IS the wildcard probe (the
      // reference visits that child twice; no parent probe: topics.go:507)
      const bool lit_is_wild = (k1 == (1ull << 56)) && (k0 == '+' || k0 == '#');
      const uint32_t tst = d == 0 ? 0 : L.sep[d - 1] + 1;
      const uint32_t tln = ((d < nsep) ? L.sep[d] : len) - tst;
      uint32_t nnext = 0;
      for (uint32_t base = 0; base < nf * 3 && !overflow; base += kWave) {
        const uint32_t item = base + lane;
        const uint32_t fi = item / 3, type = item % 3;
        uint32_t c = kNone;
        NodeDesc dc;
        if (item < nf * 3) {
          const uint32_t node = L.front[cur][0][fi];
          if (type == 0) {
            if (!lit_is_wild) c = probe_edge(s, node, k0, k1, tp + tst, tln, &dc);
          } else {
            c = L.front[cur][type][fi];
            if (c != kNone) dc = load_desc(s.nodes + c);
          }
        }
        const bool found = c != kNone;
        const uint32_t fl = found ? dc.sh_cnt_flags >> 24 : 0;
        const bool skip_dollar = dollar && (fl & kFlagDollarWild);  // topics.go:527
        const bool h_own = found && dc.sub_cnt > 0 && !skip_dollar;
        const bool h_par = found && type == 0 && dc.hsub_cnt > 0 && !skip_dollar;  // topics.go:507-509
        const bool h_sh = found && (dc.sh_cnt_flags & kShCntMask) > 0;
        const bool push = found && has_next && (fl & kFlagHasChildren);
        const uint64_t m_own = __ballot(h_own), m_par = __ballot(h_par), m_sh = __ballot(h_sh),
                       m_push = __ballot(push);
        const uint64_t lt = lanemask_lt(lane);
        const uint32_t n_own = __popcll(m_own), n_par = __popcll(m_par);
        if (nh + n_own + n_par > (uint32_t)kHCap || nsh + __popcll(m_sh) > (uint32_t)kShCap ||
            nnext + __popcll(m_push) > (uint32_t)kFCap) {
          overflow = true;
          break;
        }
        if (h_own) {
          const uint32_t i = nh + __popcll(m_own & lt);
          L.hit_rank[i] = 2 * c;
          L.hit_off[i] = dc.sub_off;
          L.hit_pre[i] = dc.sub_cnt;
        }
        if (h_par) {
          const uint32_t i = nh + n_own + __popcll(m_par & lt);
          L.hit_rank[i] = 2 * c + 1;
          L.hit_off[i] = dc.hsub_off;
          L.hit_pre[i] = dc.hsub_cnt;
        }
        if (h_sh) {
          const uint32_t i = nsh + __popcll(m_sh & lt);
          L.sh_off[i] = dc.sh_off;
          L.sh_cnt[i] = dc.sh_cnt_flags & kShCntMask;
        }
        if (push) {
          const uint32_t i = nnext + __popcll(m_push & lt);
          L.front[cur ^ 1][0][i] = c;
          L.front[cur ^ 1][1][i] = dc.plus;
          L.front[cur ^ 1][2][i] = dc.hash;
        }
        nh += n_own + n_par;
        nsh += __popcll(m_sh);
        nnext += __popcll(m_push);
      }
      wave_lds_sync();
      cur ^= 1;
      nf = nnext;
    }

    // ---- 3. order hits by rank, prefix their range sizes -------------------
    uint32_t S = 0;
    if (!overflow) {
      uint32_t rank = 0xFFFFFFFFu, hoff = 0, hcnt = 0;
      if ((uint32_t)(lane & 31) < nh) {
        rank = L.hit_rank[lane & 31];
        hoff = L.hit_off[lane & 31];
        hcnt = L.hit_pre[lane & 31];
      }
      sort32(lane, rank, hoff, hcnt);
      uint32_t inc = hcnt;  // inclusive scan over lanes 0..31
      for (int o2 = 1; o2 < 32; o2 <<= 1) {
        const uint32_t v = __shfl_up(inc, o2, 64);
        if ((lane & 31) >= o2) inc += v;
      }
      S = __shfl(inc, 31, 64);
      wave_lds_sync();
      if (lane < 32) {
        L.hit_rank[lane] = rank;
        L.hit_off[lane] = hoff;
        L.hit_pre[lane + 1] = inc;
      }
      if (lane == 0) L.hit_pre[0] = 0;
      if (S > (uint32_t)kBigMax) overflow = true;
      wave_lds_sync();
    }

    if (overflow) {  // -> unbounded DFS path (it also produces the shared candidates)
      if (lane == 0) {
        o.tier[t] = kTierDfs;
        o.dcount[t] = 0;
        o.hcount[t] = 0;
        o.dfs_list[atomicAdd(&o.ctr->n_dfs, 1u)] = t;
      }
      continue;
    }

    // ---- shared candidates (gatherSharedSubscriptions, topics.go:541-555) ---
    uint32_t H = 0;
    for (uint32_t i = 0; i < nsh; i++) H += L.sh_cnt[i];
    const uint64_t hb = wave_alloc(ha, H, &o.ctr->hpos, caps.hcap, caps.hchunk, o.ctr, 1, lane);
    if (hb != kNoSpace) {
      uint32_t w = 0;
      for (uint32_t i = 0; i < nsh; i++) {
        const uint32_t so = L.sh_off[i], sc = L.sh_cnt[i];
        for (uint32_t j = lane; j < sc; j += kWave) o.hbuf[hb + w + j] = so + j;
        w += sc;
      }
    }
    if (lane == 0) {
      o.hcount[t] = H;
      o.hstart[t] = hb;
    }

    if (S > (uint32_t)kSMax) {  // -> workgroup tier: leave the ordered hit list in a record
      const uint64_t rb = wave_alloc(ba, 1, &o.ctr->bpos, caps.bcap, caps.bchunk, o.ctr, 2, lane);
      if (rb != kNoSpace) {
        uint32_t *rec = o.recs + rb * kRecWords;
        uint32_t v = 0;
        if (lane == 0) v = t;
        else if (lane == 1) v = nh;
        else if (lane == 2) v = S;
        else if (lane >= 4 && lane < 32) v = L.hit_off[lane - 4];
        else if (lane >= 32 && lane <= 60) v = L.hit_pre[lane - 32];
        rec[lane] = v;
      }
      if (lane == 0) {
        o.tier[t] = kTierBig;
        o.dcount[t] = 0;
        o.dstart[t] = 0;
      }
      wave_lds_sync();
      continue;
    }

    // ---- 4. dedupe in the per-wave LDS table --------------------------------
    uint32_t lg = 6;  // load <= 0.5 up to kTCap/2 entries, <= 0.75 above
    while ((1u << lg) < 2 * S && (1u << lg) < (uint32_t)kTCap) lg++;
    const uint32_t tsize = 1u << lg;
    for (uint32_t i = lane; i < tsize; i += kWave) L.tkey[i] = 0, L.tval[i] = 0;
    wave_lds_sync();
    for (uint32_t r = lane; r < S; r += kWave) {
      const uint32_t h = find_hit(L.hit_pre, nh, r);
      const SubEnt e = s.subs[L.hit_off[h] + (r - L.hit_pre[h])];
      uint32_t slot = table_slot(e.client, lg);
      for (;;) {
        const uint32_t prev = atomicCAS(&L.tkey[slot], 0u, e.client + 1);
        if (prev == 0 || prev == e.client + 1) break;
        slot = (slot + 1) & (tsize - 1);
      }
      atomicOr(&L.tval[slot], merge_bits(h, e.meta));
    }
    wave_lds_sync();

    // ---- 5. winners -> deliveries (space for S reserved, D <= S used) -------
    const uint64_t db = wave_alloc(da, S, &o.ctr->dpos, caps.dcap, caps.dchunk, o.ctr, 0, lane);
    uint32_t D = 0;
    for (uint32_t r0 = 0; r0 < S; r0 += kWave) {
      const uint32_t r = r0 + lane;
      bool win = false;
      uint64_t ent = 0;
      if (r < S) {
        const uint32_t h = find_hit(L.hit_pre, nh, r);
        const uint32_t sid = L.hit_off[h] + (r - L.hit_pre[h]);
        const uint32_t client = s.subs[sid].client;
        uint32_t slot = table_slot(client, lg);
        while (L.tkey[slot] != client + 1) slot = (slot + 1) & (tsize - 1);
        const uint32_t v = L.tval[slot];
        win = (uint32_t)__builtin_ctz(v >> 4) == h;
        ent = pack_delivery(client, sid, 31u - __builtin_clz(v & 7u), (v >> 3) & 1u);
      }
      const uint64_t m = __ballot(win);
      if (win && db != kNoSpace) o.dbuf[db + D + __popcll(m & lanemask_lt(lane))] = ent;
      D += __popcll(m);
    }
    if (lane == 0) {
      o.dcount[t] = D;
      o.dstart[t] = db;
      o.tier[t] = kTierDone;
    }
    wave_lds_sync();
  }
}

// ---------------------------------------------------------------------------
// k_big: 256-thread workgroup per big-topic record, 64 KiB LDS dedupe table
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBigThreads) void k_big(DeviceSnapshot s, Outputs o, Caps caps) {
  extern __shared__ uint32_t big_tab[];  // tkey[kBigSlots] | tval[kBigSlots]
  uint32_t *tkey = big_tab, *tval = big_tab + kBigSlots;
  __shared__ uint32_t rec[kRecWords];
  __shared__ uint32_t wsum[kBigThreads / kWave];
  __shared__ unsigned long long blk_base;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  const uint64_t nrec = o.ctr->bpos < caps.bcap ? o.ctr->bpos : caps.bcap;
  uint64_t cur = 0, end = 0;  // block chunk allocator (thread 0)
  bool dead = false;
  for (uint64_t ri = blockIdx.x; ri < nrec; ri += gridDim.x) {
    if (tid < kRecWords) rec[tid] = o.recs[ri * kRecWords + tid];
    __syncthreads();
    const uint32_t t = rec[0];
    if (t == kNoTopic) {  // unused record of some wave's last chunk
      __syncthreads();
      continue;
    }
    const uint32_t nh = rec[1], S = rec[2];
    const uint32_t *hoff = rec + 4, *pre = rec + 32;
    uint32_t lg = 6;
    while ((1u << lg) < 2 * S && (1u << lg) < (uint32_t)kBigSlots) lg++;
    const uint32_t tsize = 1u << lg;
    for (uint32_t i = tid; i < tsize; i += kBigThreads) tkey[i] = 0, tval[i] = 0;
    __syncthreads();
    for (uint32_t r = tid; r < S; r += kBigThreads) {
      const uint32_t h = find_hit(pre, nh, r);
      const SubEnt e = s.subs[hoff[h] + (r - pre[h])];
      uint32_t slot = table_slot(e.client, lg);
      for (;;) {
        const uint32_t prev = atomicCAS(&tkey[slot], 0u, e.client + 1);
        if (prev == 0 || prev == e.client + 1) break;
        slot = (slot + 1) & (tsize - 1);
      }
      atomicOr(&tval[slot], merge_bits(h, e.meta));
    }
    // space for S entries from the block's chunk
    if (tid == 0) {
      if (!dead && cur + S > end) {
        const uint64_t grab = S > caps.dchunk ? S : caps.dchunk;
        cur = atomicAdd(&o.ctr->dpos, (unsigned long long)grab);
        end = cur + grab;
        if (end > caps.dcap) {
          atomicOr(&o.ctr->overflow, 1u);
          dead = true;
        }
      }
      if (dead) atomicAdd(&o.ctr->miss[0], (unsigned long long)S);
      blk_base = dead ? kNoSpace : cur;
      if (!dead) cur += S;
    }
    __syncthreads();
    const uint64_t db = blk_base;
    uint32_t D = 0;
    for (uint32_t r0 = 0; r0 < S; r0 += kBigThreads) {
      const uint32_t r = r0 + tid;
      bool win = false;
      uint64_t ent = 0;
      if (r < S) {
        const uint32_t h = find_hit(pre, nh, r);
        const uint32_t sid = hoff[h] + (r - pre[h]);
        const uint32_t client = s.subs[sid].client;
        uint32_t slot = table_slot(client, lg);
        while (tkey[slot] != client + 1) slot = (slot + 1) & (tsize - 1);
        const uint32_t v = tval[slot];
        win = (uint32_t)__builtin_ctz(v >> 4) == h;
        ent = pack_delivery(client, sid, 31u - __builtin_clz(v & 7u), (v >> 3) & 1u);
      }
      const uint64_t m = __ballot(win);
      if (lane == 0) wsum[wid] = __popcll(m);
      __syncthreads();
      uint32_t before = D;
      for (int w = 0; w < wid; w++) before += wsum[w];
      uint32_t round = 0;
      for (int w = 0; w < kBigThreads / kWave; w++) round += wsum[w];
      if (win && db != kNoSpace) o.dbuf[db + before + __popcll(m & lanemask_lt(lane))] = ent;
      D += round;
      __syncthreads();
    }
    if (tid == 0) {
      o.dcount[t] = D;
      o.dstart[t] = db;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// k_dfs<P>: the unbounded path.  P0 counts raw entries / shared candidates;
// P1 inserts into a per-topic global table and writes the shared candidates;
// P2 counts the table's clients and writes the deliveries.
// ---------------------------------------------------------------------------
struct GEnt {                  // global dedupe slot (16 B)
  unsigned long long keybits;  // (client + 1) | bits << 32
  unsigned long long first;    // ~((rank << 32) | sid), atomicMax: the table starts zeroed
};

template <int kPhase>
__global__ __launch_bounds__(kWave) void k_dfs(DeviceSnapshot s, const uint8_t *__restrict__ tbytes,
                                              const uint64_t *__restrict__ toffs, Outputs o, Caps caps,
                                              uint64_t *__restrict__ raw_cnt, const uint64_t *__restrict__ tab_off,
                                              GEnt *__restrict__ tab, uint32_t max_levels) {
  extern __shared__ uint32_t dyn[];
  // layout: sep[max_levels] | key0/key1 (u64 x max_levels each) | stack (4 x u32) x (2*max_levels + 8)
  uint32_t *sep = dyn;
  uint64_t *key0 = reinterpret_cast<uint64_t *>(dyn + ((max_levels + 1) & ~1u));
  uint64_t *key1 = key0 + max_levels;
  uint32_t *stk = reinterpret_cast<uint32_t *>(key1 + max_levels);
  const int lane = threadIdx.x;
  const uint32_t cnt = o.ctr->n_dfs;
  for (uint32_t i = blockIdx.x; i < cnt; i += gridDim.x) {
    const uint32_t t = o.dfs_list[i];
    const uint64_t off = toffs[t];
    const uint32_t len = (uint32_t)(toffs[t + 1] - off);
    const uint8_t *tp = tbytes + off;
    const uint64_t tsz = kPhase >= 1 ? tab_off[i + 1] - tab_off[i] : 0;
    GEnt *T = kPhase >= 1 ? tab + tab_off[i] : nullptr;

    if (kPhase == 2) {
      uint32_t D = 0;
      for (uint64_t b = 0; b < tsz; b += kWave) {
        const uint64_t j = b + lane;
        D += __popcll(__ballot(j < tsz && (uint32_t)T[j].keybits != 0));
      }
      uint64_t db = 0;
      if (lane == 0 && D) db = atomicAdd(&o.ctr->dpos, (unsigned long long)D);
      db = shfl64(db, 0);
      const bool ok = db + D <= caps.dcap;
      if (!ok && lane == 0) {
        atomicOr(&o.ctr->overflow, 1u);
        atomicAdd(&o.ctr->miss[0], (unsigned long long)D);
      }
      uint32_t w = 0;
      for (uint64_t b = 0; b < tsz; b += kWave) {
        const uint64_t j = b + lane;
        GEnt g{0, 0};
        if (j < tsz) g = T[j];
        const bool occ = (uint32_t)g.keybits != 0;
        const uint64_t m = __ballot(occ);
        if (occ && ok) {
          const uint32_t bits = (uint32_t)(g.keybits >> 32);
          o.dbuf[db + w + __popcll(m & lanemask_lt(lane))] = pack_delivery(
              (uint32_t)g.keybits - 1, (uint32_t)~g.first, 31u - __builtin_clz(bits & 7u), (bits >> 3) & 1u);
        }
        w += __popcll(m);
      }
      if (lane == 0) {
        o.dcount[t] = D;
        o.dstart[t] = ok ? db : kNoSpace;
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
    uint32_t H = 0;
    uint64_t hb = 0;
    bool hok = true;
    if (kPhase == 1) {
      H = o.hcount[t];  // counted by phase 0
      if (lane == 0 && H) hb = atomicAdd(&o.ctr->hpos, (unsigned long long)H);
      hb = shfl64(hb, 0);
      hok = hb + H <= caps.hcap;
      if (!hok && lane == 0) {
        atomicOr(&o.ctr->overflow, 2u);
        atomicAdd(&o.ctr->miss[1], (unsigned long long)H);
      }
      if (lane == 0) o.hstart[t] = hok ? hb : kNoSpace;
      H = 0;
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
        e.hsub_off = __shfl(dc.hsub_off, src, 64);
        e.hsub_cnt = __shfl(dc.hsub_cnt, src, 64);
        e.sh_off = __shfl(dc.sh_off, src, 64);
        e.sh_cnt_flags = __shfl(dc.sh_cnt_flags, src, 64);
        const uint32_t fl = e.sh_cnt_flags >> 24;
        const bool skip_dollar = dollar && (fl & kFlagDollarWild);
        for (int part = 0; part < 2; part++) {
          if (part == 1 && src != 0) break;
          const uint32_t roff = part ? e.hsub_off : e.sub_off;
          const uint32_t rcnt = skip_dollar ? 0 : (part ? e.hsub_cnt : e.sub_cnt);
          const uint32_t rank = 2 * cc + part;
          S += rcnt;
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
              const uint32_t bits = (1u << (se.meta & 3)) | (((se.meta >> 2) & 1) << 3);
              atomicOr(&T[slot].keybits, (unsigned long long)bits << 32);
              atomicMax(&T[slot].first, ~(((unsigned long long)rank << 32) | sid));
            }
          }
        }
        const uint32_t shc = e.sh_cnt_flags & kShCntMask;
        if (kPhase == 1 && hok)
          for (uint32_t j = lane; j < shc; j += kWave) o.hbuf[hb + H + j] = e.sh_off + j;
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
      o.hcount[t] = H;
    }
  }
}

__global__ void k_table_sizes(const uint64_t *__restrict__ raw_cnt, const Counters *__restrict__ ctr,
                              uint64_t *__restrict__ sizes) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ctr->n_dfs) return;
  uint64_t sz = 64;
  while (sz < 2 * raw_cnt[i]) sz <<= 1;
  sizes[i] = sz;
}

// raw chunks -> topic-ordered CSR (one wavefront per topic)
// (a batch whose chunk allocators overflowed is redone: skip what has no space)
__global__ __launch_bounds__(256) void k_compact(uint32_t n, const uint32_t *__restrict__ dcount,
                                                const uint64_t *__restrict__ dstart,
                                                const uint64_t *__restrict__ doffs, const uint64_t *__restrict__ dbuf,
                                                uint64_t *__restrict__ dout, const uint32_t *__restrict__ hcount,
                                                const uint64_t *__restrict__ hstart,
                                                const uint64_t *__restrict__ hoffs, const uint32_t *__restrict__ hbuf,
                                                uint32_t *__restrict__ hout, Caps caps) {
  const int lane = threadIdx.x & (kWave - 1);
  const uint32_t nwaves = gridDim.x * (blockDim.x / kWave);
  for (uint32_t t = blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave; t < n; t += nwaves) {
    const uint32_t D = dcount[t], H = hcount[t];
    if (D) {
      const uint64_t src = dstart[t], dst = doffs[t];
      if (src != kNoSpace && src + D <= caps.dcap && dst + D <= caps.dcap)
        for (uint32_t j = lane; j < D; j += kWave) dout[dst + j] = dbuf[src + j];
    }
    if (H) {
      const uint64_t src = hstart[t], dst = hoffs[t];
      if (src != kNoSpace && src + H <= caps.hcap && dst + H <= caps.hcap)
        for (uint32_t j = lane; j < H; j += kWave) hout[dst + j] = hbuf[src + j];
    }
  }
}

#define HIP_TRY(x)                                                                                  \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) {                                                                         \
      fprintf(stderr, "mqmatch: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
      return -3;                                                                                    \
    }                                                                                               \
  } while (0)

}  // namespace

// ---------------------------------------------------------------------------
// workspace / orchestration
// ---------------------------------------------------------------------------
int Workspace::reserve(void **p, size_t *cap, size_t need) {
  if (*cap >= need && *p) return 0;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  size_t n = std::max<size_t>(need, 256);
  n = n + n / 4;
  if (hipMalloc(p, n) != hipSuccess) {
    *cap = 0;
    return -2;
  }
  *cap = n;
  return 0;
}

Workspace::~Workspace() {
  for (auto &b : bufs)
    if (b.p) (void)hipFree(b.p);
  if (host_pinned) (void)hipHostFree(host_pinned);
  for (auto &e : ev)
    if (e) (void)hipEventDestroy(e);
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

// counts (u32, n) -> exclusive offsets (u64, n + 1)
template <class T>
static int scan_offsets(Workspace &ws, const T *counts, uint64_t *offs, uint32_t n, hipStream_t st) {
  HIP_TRY(hipMemsetAsync(offs, 0, sizeof(uint64_t), st));
  if (n == 0) return 0;
  size_t tmp = 0;
  HIP_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, tmp, counts, offs + 1, n, st));
  if (ws.get(Workspace::kScanTmp, tmp)) return -2;
  HIP_TRY(hipcub::DeviceScan::InclusiveSum(ws.ptr(Workspace::kScanTmp), tmp, counts, offs + 1, n, st));
  return 0;
}

// capacity for a redo: what was handed out before the buffer ran out, what
// was still requested after, and one chunk of slack per wave
static void grow_caps(Workspace &ws, const Counters &c, uint32_t waves, const Caps &caps) {
  if (c.overflow & 1) ws.dcap = (std::min<uint64_t>(c.dpos, ws.dcap) + c.miss[0] + waves * (uint64_t)caps.dchunk) * 5 / 4;
  if (c.overflow & 2) ws.hcap = (std::min<uint64_t>(c.hpos, ws.hcap) + c.miss[1] + waves * (uint64_t)caps.hchunk) * 5 / 4;
  if (c.overflow & 4) ws.bcap = (std::min<uint64_t>(c.bpos, ws.bcap) + c.miss[2] + waves * (uint64_t)caps.bchunk) * 5 / 4;
}

static uint32_t chunk_for(uint64_t cap, uint32_t waves, uint32_t lo, uint32_t hi) {
  uint64_t c = cap / (8ull * waves);
  return (uint32_t)std::max<uint64_t>(lo, std::min<uint64_t>(hi, c));
}

static int match_once(const DeviceSnapshot &s, Workspace &ws, const uint8_t *d_bytes, const uint64_t *d_offs,
                      uint32_t n, hipStream_t st, MatchOutput *out, bool *retry) {
  using W = Workspace;
  *retry = false;
  if (ws.get(W::kDCount, sizeof(uint32_t) * (n + 1)) || ws.get(W::kHCount, sizeof(uint32_t) * (n + 1)) ||
      ws.get(W::kDStart, sizeof(uint64_t) * (n + 1)) || ws.get(W::kHStart, sizeof(uint64_t) * (n + 1)) ||
      ws.get(W::kTier, n + 1) || ws.get(W::kDfsList, sizeof(uint32_t) * (n + 1)) ||
      ws.get(W::kCounters, sizeof(Counters)) || ws.get(W::kDOffs, sizeof(uint64_t) * (n + 1)) ||
      ws.get(W::kHOffs, sizeof(uint64_t) * (n + 1)) || ws.get(W::kDBuf, sizeof(uint64_t) * (ws.dcap + 1)) ||
      ws.get(W::kHBuf, sizeof(uint32_t) * (ws.hcap + 1)) ||
      ws.get(W::kBigRecs, sizeof(uint32_t) * kRecWords * (ws.bcap + 1)) ||
      ws.get(W::kDOut, sizeof(uint64_t) * (ws.dcap + 1)) || ws.get(W::kHOut, sizeof(uint32_t) * (ws.hcap + 1)))
    return -2;
  if (!ws.host_pinned && hipHostMalloc(&ws.host_pinned, 256, hipHostMallocDefault) != hipSuccess) return -2;
  Counters *hc = reinterpret_cast<Counters *>(ws.host_pinned);
  uint64_t *hp = reinterpret_cast<uint64_t *>(reinterpret_cast<char *>(ws.host_pinned) + 128);

  const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>((n + kWavesPerBlock - 1) / kWavesPerBlock,
                                                                   ws.max_blocks));
  const uint32_t waves = blocks * kWavesPerBlock;
  Outputs o;
  o.dcount = (uint32_t *)ws.ptr(W::kDCount);
  o.hcount = (uint32_t *)ws.ptr(W::kHCount);
  o.dstart = (uint64_t *)ws.ptr(W::kDStart);
  o.hstart = (uint64_t *)ws.ptr(W::kHStart);
  o.tier = (uint8_t *)ws.ptr(W::kTier);
  o.dfs_list = (uint32_t *)ws.ptr(W::kDfsList);
  o.ctr = (Counters *)ws.ptr(W::kCounters);
  o.dbuf = (uint64_t *)ws.ptr(W::kDBuf);
  o.hbuf = (uint32_t *)ws.ptr(W::kHBuf);
  o.recs = (uint32_t *)ws.ptr(W::kBigRecs);
  Caps caps;
  caps.dcap = ws.dcap;
  caps.hcap = ws.hcap;
  caps.bcap = ws.bcap;
  caps.dchunk = chunk_for(ws.dcap, waves, 256, 8192);
  caps.hchunk = chunk_for(ws.hcap, waves, 64, 4096);
  caps.bchunk = chunk_for(ws.bcap, waves, 1, 16);

  HIP_TRY(hipMemsetAsync(o.ctr, 0, sizeof(Counters), st));
  HIP_TRY(hipMemsetAsync(o.recs, 0xFF, sizeof(uint32_t) * kRecWords * ws.bcap, st));
  mark(ws, 0, st);
  if (n > 0) hipLaunchKernelGGL(k_walk, dim3(blocks), dim3(kWave * kWavesPerBlock), 0, st, s, d_bytes, d_offs, n, o, caps);
  HIP_TRY(hipGetLastError());
  mark(ws, 1, st);
  HIP_TRY(hipMemcpyAsync(hc, o.ctr, sizeof(Counters), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  const uint32_t n_dfs = hc->n_dfs;
  out->n_fallback = n_dfs;
  out->n_big = (uint32_t)std::min<uint64_t>(hc->bpos, ws.bcap);
  if (hc->overflow) {  // grow to the measured need and redo the batch
    grow_caps(ws, *hc, waves, caps);
    *retry = true;
    return 0;
  }

  // workgroup tier (grid-strides over the records; count read on the device)
  const size_t big_lds = sizeof(uint32_t) * 2 * kBigSlots;
  if (hc->bpos)
    hipLaunchKernelGGL(k_big, dim3(std::min<uint64_t>(hc->bpos, 256 * 2)), dim3(kBigThreads), big_lds, st, s, o,
                       caps);
  HIP_TRY(hipGetLastError());

  if (n_dfs) {
    const uint32_t max_levels = s.height + 1;
    const size_t fb_lds = sizeof(uint32_t) * (((max_levels + 1) & ~1u) + 4 * (2 * max_levels + 8)) +
                          sizeof(uint64_t) * 2 * max_levels;
    const uint32_t fb_blocks = std::max<uint32_t>(1, std::min<uint32_t>(n_dfs, 4096));
    if (ws.get(W::kRawCnt, sizeof(uint64_t) * (n_dfs + 1)) || ws.get(W::kTabOff, sizeof(uint64_t) * (n_dfs + 2)) ||
        ws.get(W::kTabSize, sizeof(uint64_t) * (n_dfs + 1)))
      return -2;
    auto *raw_cnt = (uint64_t *)ws.ptr(W::kRawCnt);
    auto *tab_off = (uint64_t *)ws.ptr(W::kTabOff);
    auto *tab_size = (uint64_t *)ws.ptr(W::kTabSize);
    hipLaunchKernelGGL(k_dfs<0>, dim3(fb_blocks), dim3(kWave), fb_lds, st, s, d_bytes, d_offs, o, caps, raw_cnt,
                       nullptr, nullptr, max_levels);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_table_sizes, dim3((n_dfs + 255) / 256), dim3(256), 0, st, raw_cnt, o.ctr, tab_size);
    HIP_TRY(hipGetLastError());
    if (scan_offsets(ws, tab_size, tab_off, n_dfs, st)) return -3;
    HIP_TRY(hipMemcpyAsync(hp, tab_off + n_dfs, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const uint64_t tab_total = hp[0];
    if (ws.get(W::kTable, sizeof(GEnt) * (tab_total + 1))) return -2;
    GEnt *tab = (GEnt *)ws.ptr(W::kTable);
    HIP_TRY(hipMemsetAsync(tab, 0, sizeof(GEnt) * tab_total, st));
    hipLaunchKernelGGL(k_dfs<1>, dim3(fb_blocks), dim3(kWave), fb_lds, st, s, d_bytes, d_offs, o, caps, raw_cnt,
                       tab_off, tab, max_levels);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_dfs<2>, dim3(fb_blocks), dim3(kWave), fb_lds, st, s, d_bytes, d_offs, o, caps, raw_cnt,
                       tab_off, tab, max_levels);
    HIP_TRY(hipGetLastError());
  }
  mark(ws, 2, st);

  auto *doffs = (uint64_t *)ws.ptr(W::kDOffs);
  auto *hoffs = (uint64_t *)ws.ptr(W::kHOffs);
  if (scan_offsets(ws, o.dcount, doffs, n, st) || scan_offsets(ws, o.hcount, hoffs, n, st)) return -3;
  auto *dout = (uint64_t *)ws.ptr(W::kDOut);
  auto *hout = (uint32_t *)ws.ptr(W::kHOut);
  mark(ws, 3, st);
  if (n > 0)
    hipLaunchKernelGGL(k_compact, dim3(std::min<uint32_t>((n + 3) / 4, 8192)), dim3(256), 0, st, n, o.dcount, o.dstart,
                       doffs, o.dbuf, dout, o.hcount, o.hstart, hoffs, o.hbuf, hout, caps);
  HIP_TRY(hipGetLastError());
  mark(ws, 4, st);
  HIP_TRY(hipMemcpyAsync(hc, o.ctr, sizeof(Counters), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(hp, doffs + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(hp + 1, hoffs + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (hc->overflow) {
    grow_caps(ws, *hc, waves, caps);
    *retry = true;
    return 0;
  }
  if (ws.profile) {
    ws.prof_calls++;
    ws.prof_fallback_topics += n_dfs;
    ws.prof_walk_ms += elapsed(ws, 0, 1);
    ws.prof_big_ms += elapsed(ws, 1, 2);
    ws.prof_compact_ms += elapsed(ws, 3, 4);
    ws.prof_total_ms += elapsed(ws, 0, 4);
  }
  out->n_topics = n;
  out->n_deliveries = hp[0];
  out->n_shared = hp[1];
  out->offsets = doffs;
  out->deliveries = dout;
  out->shared_offsets = hoffs;
  out->shared = hout;
  return 0;
}

int match_device(const DeviceSnapshot &s, Workspace &ws, const uint8_t *d_bytes, const uint64_t *d_offs,
                 uint32_t n, hipStream_t st, MatchOutput *out) {
  if (ws.dcap == 0) ws.dcap = std::max<uint64_t>(1u << 20, 64ull * n);
  if (ws.hcap == 0) ws.hcap = std::max<uint64_t>(1u << 16, 4ull * n);
  if (ws.bcap == 0) ws.bcap = std::max<uint64_t>(1u << 12, n / 4 + 1);
  for (int attempt = 0; attempt < 4; attempt++) {
    bool retry = false;
    int rc = match_once(s, ws, d_bytes, d_offs, n, st, out, &retry);
    if (rc != 0 || !retry) return rc;
  }
  return -4;  // MQM_ELIMIT: capacities kept growing
}

}  // namespace mqm
