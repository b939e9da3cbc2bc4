// tests/harness/slots_test.cpp — the per-publish server's ring-slot ownership
// (maxmq_amd/csrc/serve_slots.h) on the CPU, with the device's done words
// played by this program.  Scenarios: normal turns; a caller that gives up
// after posting (abandon) and its late result; callers that give up before
// posting (slot wait timed out), once and twice in a row, with the previous
// owner finishing normally or by a late result (the slot used to
// stay with the ticket that never posted, and every S-th caller after it
// failed); and the counter restart point (oldest_unserved).  Prints OK.
#include <chrono>
#include <cstdio>
#include <cstdlib>

#include "../../maxmq_amd/csrc/serve_slots.h"

using mqm::SlotOwners;
using namespace std::chrono_literals;

static int fails = 0;
#define CHECK(c)                                              \
  do {                                                        \
    if (!(c)) {                                               \
      printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);     \
      fails++;                                                \
    }                                                         \
  } while (0)

int main() {
  constexpr uint32_t S = 4;
  {  // normal turns: each ticket gets its slot once the previous one released it
    unsigned long long done[S] = {};
    SlotOwners o(S, done);
    for (uint64_t k = 0; k < 12; k++) {
      CHECK(o.wait(k, 10ms));
      done[k % S] = k + 1;
      o.release(k);
    }
    CHECK(!o.wait(16, 1ms) && o.owner(0) == 12);  // not its turn yet
    CHECK(o.oldest_unserved(12) == 12);
  }
  {  // abandon after posting: the slot waits for the late result, then moves on
    unsigned long long done[S] = {};
    SlotOwners o(S, done);
    CHECK(o.wait(1, 10ms));
    o.abandon(1);                  // posted request 1, no result yet
    CHECK(!o.wait(5, 2ms));        // the device may still write slot 1
    CHECK(o.oldest_unserved(6) == 0);  // 0 is unserved (taken, never released here)
    done[1] = 2;                   // the late result lands
    CHECK(o.wait(5, 10ms));
    CHECK(o.abandoned(1) == 0);
  }
  {  // ticket k gives up before posting, then its predecessor finishes
    unsigned long long done[S] = {};
    SlotOwners o(S, done);
    CHECK(o.wait(2, 10ms));        // ticket 2 posts and is slow
    CHECK(!o.wait(6, 1ms));        // ticket 6 times out waiting for slot 2
    o.give_up_unposted(6);
    CHECK(o.slot_timeouts.load() == 1);
    CHECK(o.oldest_unserved(11) == 0);
    done[2] = 3;
    o.release(2);                  // ticket 2 done: the slot skips 6 and goes to 10
    CHECK(o.owner(2) == 10 && o.skipped.load() == 1);
    CHECK(o.wait(10, 10ms));
    done[2] = 11;
    o.release(10);
    CHECK(o.wait(14, 10ms));
    CHECK(o.never_posted_size() == 1);
    CHECK(o.oldest_unserved(15) == 0);  // tickets 0, 1, 3 never ran here
    CHECK(o.never_posted_size() == 0);  // 6 is behind its slot now: pruned
  }
  {  // two give-ups in a row, then the predecessor's late result (it had abandoned)
    unsigned long long done[S] = {};
    SlotOwners o(S, done);
    CHECK(o.wait(3, 10ms));
    o.abandon(3);
    CHECK(!o.wait(7, 1ms));
    o.give_up_unposted(7);
    CHECK(!o.wait(11, 1ms));
    o.give_up_unposted(11);
    // the restart point never waits on a ticket that will not post (7, 11)
    CHECK(o.oldest_unserved(12) == 0);
    done[3] = 4;                   // 3's late result
    CHECK(o.wait(15, 10ms));       // 15 takes the slot past 7 and 11
    CHECK(o.owner(3) == 15 && o.skipped.load() == 2);
  }
  {  // the give-up races the release: the predecessor released to k first
    unsigned long long done[S] = {};
    SlotOwners o(S, done);
    CHECK(o.wait(0, 10ms));
    done[0] = 1;
    o.release(0);                  // slot 0 -> ticket 4 ...
    o.give_up_unposted(4);         // ... which gives up anyway (its wait timed out just before)
    CHECK(o.owner(0) == 8);
    CHECK(o.wait(8, 10ms));
  }
  {  // restart point: a slot whose owner's result is in counts from the next ticket
    unsigned long long done[S] = {};
    SlotOwners o(S, done);
    for (uint64_t k = 0; k < 4; k++) CHECK(o.wait(k, 10ms));
    done[0] = 1;
    done[2] = 3;                   // 0 and 2 served, not yet released; 1 and 3 posted
    CHECK(o.oldest_unserved(4) == 1);
    CHECK(o.oldest_unserved(1) == 1);  // no ticket handed out past 0: nothing to wait for
  }
  if (fails) return 1;
  printf("OK\n");
  return 0;
}
