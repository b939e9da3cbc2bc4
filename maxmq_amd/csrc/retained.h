// maxmq_amd/csrc/retained.h — batch reverse match (TopicsIndex.Messages,
// vendor/github.com/mochi-co/mqtt/v2/topics.go:426-480) over a DeviceRetained.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "match.h"
#include "snapshot.h"

namespace mqm {

// one emission: message refs list[lo, hi) (list 0 = DeviceRetained::refs,
// 1 = DeviceRetained::rch_refs) belong to filter f
struct Emit {
  uint32_t f, list, lo, hi;
};

struct MessagesOutput {
  uint32_t n_filters = 0;
  uint64_t n_refs = 0;
  uint64_t n_emissions = 0;
  uint64_t n_items = 0;  // (filter, node) worklist items over all levels
  uint64_t n_skipped = 0;  // ... of those, the reference's items the edge index jumped over (never loaded)
  const uint64_t *offsets = nullptr;  // device, n_filters + 1
  const uint64_t *refs = nullptr;     // device, message refs (order within a filter unspecified)
};

// r == nullptr: nothing is retained.  Returns 0 or a negative MQM_E* code;
// synchronises `st` before returning (the output sizes are read back).
int messages_device(const DeviceSnapshot &s, const DeviceRetained *r, Workspace &ws, const uint8_t *d_bytes,
                    const uint64_t *d_offs, uint32_t n, hipStream_t st, MessagesOutput *out);

}  // namespace mqm
