// maxmq_amd/csrc/shard.h — node-wide CSR of a subscriber-sharded match
// (shard.hip, mqm_gather_shards).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace mqm {

constexpr int kMaxShards = 16;
constexpr uint32_t kShardShift = 28;  // node-wide shared candidate = shard << 28 | shard-local shared id

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

// shared candidates of the shards (dense CSRs: offsets n + 1, u32 shared ids)
// -> one node-wide CSR of shard << kShardShift | id; an id >= 2^kShardShift sets *d_bad
int gather_shards_shared(uint32_t n, uint32_t S, const uint64_t *const *offsets, const uint32_t *const *shared,
                         hipStream_t st, uint64_t *out_offsets, uint32_t *out, unsigned int *d_bad);

}  // namespace mqm
