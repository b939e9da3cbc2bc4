// tests/harness/guard_test.cpp — the launch guard (match.hip guard_outputs)
// on the CPU: identifiers_device on a workspace whose last match left an array
// missing, or too short for its topics, must return -1 (MQM_EINVAL) before it
// allocates or launches anything (round 4's r04x fault was such a launch).
// Test infrastructure: built by tests/harness/Makefile, run by
// tests/test_capi_host.py without a GPU (no HIP call is reached).
#include <cstdio>
#include <cstring>

#include "../../maxmq_amd/csrc/match.h"

using mqm::Workspace;

static char fake[1 << 20];  // stands in for device buffers: the guard refuses before any use

static int run(Workspace::Slot drop, size_t short_cap) {
  Workspace ws;
  const uint32_t n = 16;
  const Workspace::Slot in[] = {Workspace::kCls,     Workspace::kRecs,   Workspace::kDfsList, Workspace::kCounters,
                                Workspace::kNSolo,   Workspace::kMCount, Workspace::kHCount};
  size_t at = 0;
  for (Workspace::Slot s : in) {
    if (s == drop && !short_cap) continue;
    ws.bufs[s].p = fake + at;
    ws.bufs[s].cap = s == drop ? short_cap : 64 * 1024;
    at += 64 * 1024;
  }
  ws.last_valid = true;
  ws.last_n = n;
  mqm::DeviceSnapshot s{};
  mqm::IdentOutput out{};
  const int rc = mqm::identifiers_device(s, ws, nullptr, &out);
  for (auto &b : ws.bufs) b.p = nullptr;  // nothing of ours for ~Workspace to free
  return rc;
}

int main() {
  int bad = 0;
  struct {
    Workspace::Slot slot;
    size_t cap;
    const char *what;
  } cases[] = {{Workspace::kMCount, 0, "mcount missing"},
               {Workspace::kCounters, 0, "counters missing"},
               {Workspace::kDfsList, 0, "dfs list missing"},
               {Workspace::kCls, 0, "cls missing"},
               {Workspace::kRecs, 0, "recs missing"},
               {Workspace::kMCount, 8, "mcount shorter than 16 topics"},
               {Workspace::kRecs, 4096, "records shorter than 16 topics"}};
  for (const auto &c : cases) {
    const int rc = run(c.slot, c.cap);
    std::printf("%-32s -> %d\n", c.what, rc);
    if (rc != -1) bad++;
  }
  // control: every array present -> past the guard (no GPU here: the first
  // allocation fails with -2).  Skipped where a device exists: the fake
  // buffers must never reach a launch.
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    const int rc = run(Workspace::kNumSlots, 0);
    std::printf("%-32s -> %d\n", "every array present", rc);
    if (rc == -1) bad++;
  }
  std::printf(bad ? "FAIL\n" : "OK\n");
  return bad ? 1 : 0;
}
