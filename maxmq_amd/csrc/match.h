// maxmq_amd/csrc/match.h — batch match pipeline over a DeviceSnapshot.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "snapshot.h"

namespace mqm {

// Grow-only device buffers reused across batches (no allocation in steady state).
struct Workspace {
  enum Slot {
    kDCount, kHCount, kStatus, kOvfList, kOvfN, kDOffs, kHOffs, kDOut, kHOut,
    kScanTmp, kRawCnt, kTabOff, kTabSize, kTable, kInBytes, kInOffs, kNumSlots
  };
  struct Buf {
    void *p = nullptr;
    size_t cap = 0;
  };
  Buf bufs[kNumSlots];
  void *host_pinned = nullptr;
  uint32_t max_blocks = 2048;  // main-path grid cap (grid-stride beyond)

  // optional kernel timing (mqm_profile_*): events on the launch stream
  bool profile = false;
  hipEvent_t ev[5] = {};  // 0 start, 1 count done, 2 emit start, 3 emit done, 4 end
  uint64_t prof_calls = 0, prof_fallback_topics = 0;
  double prof_count_ms = 0, prof_emit_ms = 0, prof_between_ms = 0, prof_total_ms = 0;
  void reset_profile() {
    prof_calls = prof_fallback_topics = 0;
    prof_count_ms = prof_emit_ms = prof_between_ms = prof_total_ms = 0;
  }

  static int reserve(void **p, size_t *cap, size_t need);
  int get(Slot s, size_t need) { return reserve(&bufs[s].p, &bufs[s].cap, need); }
  void *ptr(Slot s) const { return bufs[s].p; }
  ~Workspace();
};

struct MatchOutput {
  uint32_t n_topics = 0;
  uint64_t n_deliveries = 0, n_shared = 0;
  const uint64_t *offsets = nullptr;     // device, n + 1
  const uint64_t *deliveries = nullptr;  // device, packed (snapshot.h)
  const uint64_t *shared_offsets = nullptr;
  const uint32_t *shared = nullptr;
  uint32_t n_fallback = 0;
};

// Runs count -> scan -> emit on `st`; returns 0 or a negative MQM_E* code.
int match_device(const DeviceSnapshot &s, Workspace &ws, const uint8_t *d_bytes, const uint64_t *d_offs,
                 uint32_t n, hipStream_t st, MatchOutput *out);

}  // namespace mqm
