// maxmq_amd/csrc/shard.h — node-wide CSR of a subscriber-sharded match
// (shard.hip, mqm_gather_shards).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace mqm {

constexpr int kMaxShards = 16;

struct ShardPart {
  const uint64_t *offsets;     // device, n + 1 (dense CSR of one shard)
  const uint64_t *deliveries;  // device, packed mqm_delivery
  const uint32_t *client_map;  // device, shard client id -> node id (nullptr: identity)
  uint32_t n_map;
};

// out_offsets: n + 1; out: sum of the shards' deliveries.  Client ids outside
// a shard's map set *d_bad (device flag, caller-zeroed).  Returns 0, -1 on bad
// arguments, -3 on a launch error.
int gather_shards(uint32_t n, uint32_t S, const ShardPart *parts, hipStream_t st, uint64_t *out_offsets,
                  uint64_t *out, unsigned int *d_bad);

}  // namespace mqm
