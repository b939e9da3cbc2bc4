// maxmq_amd/csrc/edges.hip — the literal-edge table built on the device at
// upload (flatten.h build_edges_device), byte for byte the table
// insert_edges_host (flatten.cpp) builds on the host (snapshot.h: kEdgeParts
// partitions, linear probing that stops at a partition's end, the run-past
// edges placed afterwards in partition order).
//
// Why on the device: the table is the snapshot's largest array (load 0.12:
// 18.5 GB at config 3 for 34.7M edges), and filling it on the host (first
// touch of 18.5 GB, 16 threads), hashing it for the digest and copying it
// over PCIe was most of a rebuild — the rebuild a published snapshot waits
// for under Subscribe/Unsubscribe churn.  Only the staged edges (64 B each,
// 2.2 GB at config 3) cross PCIe now.
//
//   k_edge_empty  every slot empty (HBM-bound store stream)
//   k_edge_keys   each edge's partition (its home slot's) + its index
//   radix sort    stable by partition: edge order within a partition
//   k_edge_insert one thread per partition, in edge order (disjoint slot
//                 ranges: no atomics, no races)
//   k_edge_spill  one wavefront: the run-past edges in partition order
//   k_edge_digest the digest's sum of per-slot terms (builder.h)
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include <mutex>

#include "flatten.h"

namespace mqm {
namespace {

constexpr uint32_t kSpillCap = 256;  // run-past edges kept per partition (more: the host builds the table)

__global__ __launch_bounds__(256) void k_edge_empty(uint4 *__restrict__ t, uint64_t n_slots) {
  const uint64_t n = n_slots * 4;  // 16-B words; word 1 of a slot holds parent, child
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    t[i] = (i & 3) == 1 ? make_uint4(kNone, kNone, 0u, 0u) : make_uint4(0u, 0u, 0u, 0u);
}

__global__ __launch_bounds__(256) void k_edge_keys(const EdgeEntry *__restrict__ staged, uint64_t ne, uint64_t nb,
                                                   uint32_t *__restrict__ part, uint32_t *__restrict__ idx,
                                                   unsigned int *__restrict__ cnt) {
  const uint64_t n_slots = nb * kEdgesPerBucket;
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < ne; e += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t p = edge_part_of(edge_home(staged[e], nb), n_slots);
    part[e] = p;
    idx[e] = (uint32_t)e;
    atomicAdd(&cnt[p], 1u);
  }
}

__device__ __forceinline__ void put_entry(EdgeEntry *t, uint64_t slot, const EdgeEntry *src) {
  const uint4 *s = reinterpret_cast<const uint4 *>(src);
  uint4 *d = reinterpret_cast<uint4 *>(t + slot);
  const uint4 a = s[0], b = s[1], c = s[2], e = s[3];
  d[0] = a;
  d[1] = b;
  d[2] = c;
  d[3] = e;
}

// partition p's edges (sorted[pstart[p] .. pstart[p + 1]), edge order) into
// its slots [edge_part_lo(p), edge_part_lo(p + 1)); an edge whose probe runs
// past the end goes to the partition's run-past list
__global__ __launch_bounds__(256) void k_edge_insert(const EdgeEntry *__restrict__ staged,
                                                     const uint32_t *__restrict__ sorted,
                                                     const uint64_t *__restrict__ pstart, uint64_t nb,
                                                     EdgeEntry *__restrict__ table, uint32_t *__restrict__ spill_cnt,
                                                     uint32_t *__restrict__ spill, unsigned int *ovf) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= kEdgeParts) return;
  const uint64_t n_slots = nb * kEdgesPerBucket, hi = edge_part_lo(p + 1, n_slots);
  uint32_t ns = 0;
  for (uint64_t j = pstart[p]; j < pstart[p + 1]; j++) {
    const uint32_t e = sorted[j];
    uint64_t slot = edge_home(staged[e], nb);
    while (slot < hi && table[slot].parent != kNone) slot++;  // (this thread's own slots)
    if (slot == hi) {
      if (ns < kSpillCap) spill[(uint64_t)p * kSpillCap + ns] = e;
      ns++;
    } else {
      put_entry(table, slot, staged + e);
    }
  }
  spill_cnt[p] = ns;
  if (ns > kSpillCap) atomicOr(ovf, 1u);
}

// one wavefront: the partitions' run-past edges in partition order, probing
// with wrap-around (lane 0 places them; the others find the next partition)
__global__ __launch_bounds__(64) void k_edge_spill(const EdgeEntry *__restrict__ staged,
                                                   const uint32_t *__restrict__ spill_cnt,
                                                   const uint32_t *__restrict__ spill, uint64_t nb,
                                                   EdgeEntry *__restrict__ table) {
  const int lane = threadIdx.x;
  const uint64_t n_slots = nb * kEdgesPerBucket;
  for (uint32_t p0 = 0; p0 < kEdgeParts; p0 += 64) {
    const uint32_t c = min(spill_cnt[p0 + lane], kSpillCap);
    uint64_t m = __ballot(c != 0);
    while (m) {
      const int l = __builtin_ctzll(m);
      m &= m - 1;
      const uint32_t cc = __shfl(c, l, 64);
      if (lane == 0)
        for (uint32_t k = 0; k < cc; k++) {
          const uint32_t e = spill[(uint64_t)(p0 + l) * kSpillCap + k];
          uint64_t slot = edge_home(staged[e], nb);
          while (table[slot].parent != kNone) slot = slot + 1 == n_slots ? 0 : slot + 1;
          put_entry(table, slot, staged + e);
        }
    }
  }
}

__global__ __launch_bounds__(256) void k_edge_digest(const EdgeEntry *__restrict__ t, uint64_t n,
                                                     unsigned long long *sum) {
  uint64_t acc = 0;
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n; s += (uint64_t)gridDim.x * blockDim.x)
    acc += edge_slot_mix(s, t[s]);
  for (int d = 32; d > 0; d >>= 1) {
    const uint32_t lo = __shfl_down((uint32_t)acc, d, 64), hi = __shfl_down((uint32_t)(acc >> 32), d, 64);
    acc += ((uint64_t)hi << 32) | lo;
  }
  if ((threadIdx.x & 63) == 0) atomicAdd(sum, (unsigned long long)acc);
}

struct Widen32 {
  __host__ __device__ uint64_t operator()(unsigned int x) const { return x; }
};

#define EDGE_TRY(x)                      \
  do {                                   \
    if ((x) != hipSuccess) return -1;    \
  } while (0)

uint32_t grid_for(uint64_t n) { return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, 16384)); }

}  // namespace

// The build's device memory: the staged edges and every temporary, carved
// from one region per device that is kept from build to build (grown, never
// shrunk; a grown-out region is freed by the index layer's reaper, which
// stops the per-publish servers first: hipFree waits for every kernel).
// Round 5 took them from the stream-ordered pool (hipMallocAsync /
// hipFreeAsync on the upload stream), whose reuse of freed memory was seen to
// serve stale contents to kernels (tools/reuse_probe.hip, r05s/r05u); with
// snapshot buffers recycled in place — no hipFree between builds — served
// results then missed the newest subscriptions of one snapshot now and then
// (r06a/r06b, tests/test_gpu_serve_churn.py).  MQM_EDGE_POOL=1: the pool.
struct EdgeScratch {
  std::mutex mu;
  char *p = nullptr;
  size_t cap = 0;
};
EdgeScratch &edge_scratch(int dev) {
  static auto *s = new EdgeScratch[64];  // (never destroyed: uploads may run during static destruction)
  return s[dev & 63];
}
bool edge_pool() {
  static const bool v = getenv("MQM_EDGE_POOL") && atoi(getenv("MQM_EDGE_POOL")) != 0;
  return v;
}

int build_edges_device(const EdgeEntry *h_staged, uint64_t ne, uint64_t nb, EdgeEntry *table, hipStream_t st,
                       uint64_t *digest_sum) {
  constexpr uint32_t P = kEdgeParts;
  const uint64_t n_slots = nb * kEdgesPerBucket;
  if (ne >= kNone || n_slots >= (1ull << 50)) return -1;
  int dev = 0;
  EDGE_TRY(hipGetDevice(&dev));
  // sizes of the carved parts (256-B aligned)
  const uint64_t n1 = ne ? ne : 1;
  size_t tsort = 0, tscan = 0;
  {
    uint32_t *np = nullptr;
    uint64_t *pp = nullptr;
    hipcub::TransformInputIterator<uint64_t, Widen32, const unsigned int *> c0((const unsigned int *)np, Widen32{});
    EDGE_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tsort, np, np, np, np, (int)n1, 0, 14, st));
    EDGE_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tscan, c0, pp, (int)P + 1, st));
  }
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  const size_t z_staged = al(ne * sizeof(EdgeEntry) + 64), z4 = al(4 * n1), z_cnt = al(4 * (P + 1) + 4),
               z_pstart = al(8 * (P + 1)), z_spc = al(4 * P), z_spill = al(4 * (uint64_t)P * kSpillCap),
               z_tmp = al(std::max(tsort, tscan) + 16), z_sum = al(8);
  const size_t total = z_staged + 4 * z4 + z_cnt + z_pstart + z_spc + z_spill + z_tmp + z_sum;
  EdgeScratch &sc = edge_scratch(dev);
  std::unique_lock<std::mutex> lk(sc.mu, std::defer_lock);
  char *base = nullptr;
  if (edge_pool()) {
    EDGE_TRY(hipMallocAsync((void **)&base, total, st));
  } else {
    lk.lock();  // (held until the build has synchronised its stream: the region is reused by the next build)
    if (sc.cap < total) {
      if (sc.p) retire_device_buffers(dev, {sc.p});
      sc.p = nullptr;
      sc.cap = 0;
      const size_t want = total + total / 4;
      EDGE_TRY(hipMalloc((void **)&sc.p, want));
      sc.cap = want;
    }
    base = sc.p;
  }
  size_t off = 0;
  auto carve = [&](size_t z) {
    char *q = base + off;
    off += z;
    return q;
  };
  EdgeEntry *d_staged = (EdgeEntry *)carve(z_staged);
  uint32_t *part = (uint32_t *)carve(z4), *idx = (uint32_t *)carve(z4), *part2 = (uint32_t *)carve(z4),
           *idx2 = (uint32_t *)carve(z4);
  unsigned int *cnt = (unsigned int *)carve(z_cnt);  // [P]: 0 (the scan's total); ovf after it
  uint64_t *pstart = (uint64_t *)carve(z_pstart);
  uint32_t *spill_cnt = (uint32_t *)carve(z_spc), *spill = (uint32_t *)carve(z_spill);
  void *tmp = carve(z_tmp);
  unsigned long long *sum = (unsigned long long *)carve(z_sum);
  const int rc = [&]() -> int {
    if (ne) EDGE_TRY(hipMemcpyAsync(d_staged, h_staged, ne * sizeof(EdgeEntry), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_edge_empty, dim3(grid_for(n_slots * 4)), dim3(256), 0, st, (uint4 *)table, n_slots);
    EDGE_TRY(hipGetLastError());
    if (ne) {
      unsigned int *ovf = cnt + P + 1;
      EDGE_TRY(hipMemsetAsync(cnt, 0, 4 * (P + 1) + 4, st));
      hipLaunchKernelGGL(k_edge_keys, dim3(grid_for(ne)), dim3(256), 0, st, d_staged, ne, nb, part, idx, cnt);
      EDGE_TRY(hipGetLastError());
      size_t t1 = tsort;
      EDGE_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, t1, part, part2, idx, idx2, (int)n1, 0, 14, st));
      hipcub::TransformInputIterator<uint64_t, Widen32, const unsigned int *> c64(cnt, Widen32{});
      size_t t2 = tscan;
      EDGE_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, t2, c64, pstart, (int)P + 1, st));
      hipLaunchKernelGGL(k_edge_insert, dim3(P / 256), dim3(256), 0, st, d_staged, idx2, pstart, nb, table, spill_cnt,
                         spill, ovf);
      EDGE_TRY(hipGetLastError());
      unsigned int h_ovf = 0;
      EDGE_TRY(hipMemcpyAsync(&h_ovf, ovf, sizeof(h_ovf), hipMemcpyDeviceToHost, st));
      EDGE_TRY(hipStreamSynchronize(st));
      if (h_ovf) return 1;
      hipLaunchKernelGGL(k_edge_spill, dim3(1), dim3(64), 0, st, d_staged, spill_cnt, spill, nb, table);
      EDGE_TRY(hipGetLastError());
    }
    // the digest's sum of per-slot terms
    EDGE_TRY(hipMemsetAsync(sum, 0, sizeof(unsigned long long), st));
    hipLaunchKernelGGL(k_edge_digest, dim3(grid_for(n_slots)), dim3(256), 0, st, table, n_slots, sum);
    EDGE_TRY(hipGetLastError());
    unsigned long long h = 0;
    EDGE_TRY(hipMemcpyAsync(&h, sum, sizeof(h), hipMemcpyDeviceToHost, st));
    EDGE_TRY(hipStreamSynchronize(st));
    *digest_sum = h;
    return 0;
  }();
  if (edge_pool()) (void)hipFreeAsync(base, st);
  // (an error part-way may leave work queued on the region: wait for it before the next build reuses it)
  if (rc < 0) (void)hipStreamSynchronize(st);
  return rc;
}

}  // namespace mqm
