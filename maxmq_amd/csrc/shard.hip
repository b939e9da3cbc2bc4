// maxmq_amd/csrc/shard.hip — node-wide result of a subscriber-sharded match
// (SURVEY.md §8e).
//
// Rank r of S holds the subscriptions of one contiguous client range; the
// merge rule (packets.go:250-270) is per client, so every shard's per-topic
// delivery set is final and the shards' sets are disjoint.  Topic t's
// node-wide set is shard 0's segment, then shard 1's, ... (concatenation,
// no merge).  The dense per-shard CSRs arrive at the gathering rank over RCCL
// (maxmq_amd/shard.py); this kernel lays them out as one dense CSR and maps
// each shard's interned client ids to node-wide ids.
//
// Node-wide offsets need no scan: every shard's offsets are an exclusive
// prefix of its counts, so out_offsets[t] = sum_r off_r[t].  A wavefront
// copies one topic (all shards), 8 B per lane per step; HBM-bound:
// 16 B per delivery (read + write) + 8 (S + 1) B per topic of offsets.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "shard.h"

namespace mqm {
namespace {

constexpr int kWave = 64;

struct ShardArgs {
  const uint64_t *offsets[kMaxShards];
  const uint64_t *deliveries[kMaxShards];
  const uint32_t *client_map[kMaxShards];  // nullptr: ids kept
  uint32_t n_map[kMaxShards];
};

__global__ __launch_bounds__(256) void k_shard_offsets(uint32_t n, uint32_t S, ShardArgs a,
                                                       uint64_t *__restrict__ out_offs) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t > n) return;
  uint64_t o = 0;
  for (uint32_t r = 0; r < S; r++) o += a.offsets[r][t];
  out_offs[t] = o;
}

__global__ __launch_bounds__(256) void k_shard_gather(uint32_t n, uint32_t S, ShardArgs a,
                                                      const uint64_t *__restrict__ out_offs,
                                                      uint64_t *__restrict__ out, unsigned int *__restrict__ bad) {
  const int lane = threadIdx.x & (kWave - 1);
  const uint32_t waves = gridDim.x * (blockDim.x / kWave);
  for (uint32_t t = blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave; t < n; t += waves) {
    uint64_t w = out_offs[t];
    for (uint32_t r = 0; r < S; r++) {
      const uint64_t b = a.offsets[r][t], e = a.offsets[r][t + 1];
      const uint64_t *src = a.deliveries[r];
      const uint32_t *map = a.client_map[r];
      for (uint64_t j = b + lane; j < e; j += kWave) {
        uint64_t v = src[j];
        if (map) {
          const uint32_t c = (uint32_t)v;  // mqm_delivery.client (low word)
          if (c < a.n_map[r])
            v = (v & 0xFFFFFFFF00000000ull) | map[c];
          else
            atomicOr(bad, 1u);
        }
        out[w + (j - b)] = v;
      }
      w += e - b;
    }
  }
}

// shared candidates: shard r's entry sid becomes r << kShardShift | sid (the
// id stays shard-local: resolve it on shard r's index)
__global__ __launch_bounds__(256) void k_shard_gather_shared(uint32_t n, uint32_t S, ShardArgs a,
                                                             const uint64_t *__restrict__ out_offs,
                                                             uint32_t *__restrict__ out, unsigned int *__restrict__ bad) {
  const int lane = threadIdx.x & (kWave - 1);
  const uint32_t waves = gridDim.x * (blockDim.x / kWave);
  for (uint32_t t = blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave; t < n; t += waves) {
    uint64_t w = out_offs[t];
    for (uint32_t r = 0; r < S; r++) {
      const uint64_t b = a.offsets[r][t], e = a.offsets[r][t + 1];
      const uint32_t *src = reinterpret_cast<const uint32_t *>(a.deliveries[r]);
      for (uint64_t j = b + lane; j < e; j += kWave) {
        const uint32_t v = src[j];
        if (v >> kShardShift) atomicOr(bad, 1u);
        out[w + (j - b)] = (r << kShardShift) | (v & ((1u << kShardShift) - 1));
      }
      w += e - b;
    }
  }
}

}  // namespace

int gather_shards_shared(uint32_t n, uint32_t S, const uint64_t *const *offsets, const uint32_t *const *shared,
                         hipStream_t st, uint64_t *out_offsets, uint32_t *out, unsigned int *d_bad) {
  if (S == 0 || S > (uint32_t)kMaxShards || !out_offsets || !d_bad) return -1;
  ShardArgs a{};
  for (uint32_t r = 0; r < S; r++) {
    if (!offsets[r] || (!shared[r] && n)) return -1;
    a.offsets[r] = offsets[r];
    a.deliveries[r] = reinterpret_cast<const uint64_t *>(shared[r]);
  }
  hipLaunchKernelGGL(k_shard_offsets, dim3(n / 256 + 1), dim3(256), 0, st, n, S, a, out_offsets);
  if (hipGetLastError() != hipSuccess) return -3;
  if (n > 0) {
    const uint32_t blocks = n / 4 + 1 < 16384u ? n / 4 + 1 : 16384u;
    hipLaunchKernelGGL(k_shard_gather_shared, dim3(blocks), dim3(256), 0, st, n, S, a, out_offsets, out, d_bad);
    if (hipGetLastError() != hipSuccess) return -3;
  }
  return 0;
}

int gather_shards(uint32_t n, uint32_t S, const ShardPart *parts, hipStream_t st, uint64_t *out_offsets,
                  uint64_t *out, unsigned int *d_bad) {
  if (S == 0 || S > (uint32_t)kMaxShards || !out_offsets || !d_bad) return -1;
  ShardArgs a{};
  for (uint32_t r = 0; r < S; r++) {
    if (!parts[r].offsets || (!parts[r].deliveries && n)) return -1;
    a.offsets[r] = parts[r].offsets;
    a.deliveries[r] = parts[r].deliveries;
    a.client_map[r] = parts[r].client_map;
    a.n_map[r] = parts[r].n_map;
  }
  hipLaunchKernelGGL(k_shard_offsets, dim3(n / 256 + 1), dim3(256), 0, st, n, S, a, out_offsets);
  if (hipGetLastError() != hipSuccess) return -3;
  if (n > 0) {
    const uint32_t blocks = n / 4 + 1 < 16384u ? n / 4 + 1 : 16384u;
    hipLaunchKernelGGL(k_shard_gather, dim3(blocks), dim3(256), 0, st, n, S, a, out_offsets, out, d_bad);
    if (hipGetLastError() != hipSuccess) return -3;
  }
  return 0;
}

}  // namespace mqm
