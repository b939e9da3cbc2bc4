// maxmq_amd/csrc/serve_slots.h — ownership of the per-publish server's ring
// slots (capi.cpp Server, fast.hip k_serve), host side only, so it can be
// unit-tested on the CPU (tests/harness/slots_test.cpp).
//
// A caller takes a ticket k (one host atomic); ticket k uses slot k mod S.  A
// slot's tickets take it in turn: owner[i] is the ticket that may use slot i
// now.  The owner posts its request, waits for done[i] == k + 1 (written by
// the device), reads the result and releases the slot to k + S.  Two ways out
// without a result, and what happens to the slot:
//   * abandon (posted, no result for 10 s): the slot stays with k until the
//     late result lands (done[i] == k + 1) — the device still writes into it —
//     and is then passed on by whichever waiter sees that first;
//   * give_up_unposted (the slot was still taken after 10 s, nothing posted):
//     k never uses or releases the slot, so whoever makes k the owner passes
//     the slot on past it at once (round 5 left the slot with k for good:
//     every S-th caller after it waited 10 s and failed).
// The reference has no such ring: Subscribers() is a function call on the
// publishing goroutine (server.go:776); this is the plumbing of the device
// server that answers it.
#pragma once

#include <atomic>
#include <chrono>
#include <cstdint>
#include <memory>
#include <mutex>
#include <set>
#include <thread>

namespace mqm {

class SlotOwners {
 public:
  // done: the device-written completion words (done[i] = k + 1 once request
  // k's result in slot i is complete)
  SlotOwners(uint32_t n_slots, const unsigned long long *done)
      : S(n_slots), done_(done), owner_(new std::atomic<uint64_t>[n_slots]),
        abandoned_(new std::atomic<uint64_t>[n_slots]) {
    for (uint32_t i = 0; i < S; i++) {
      owner_[i].store(i);
      abandoned_[i].store(0);
    }
  }
  const uint32_t S;

  uint64_t owner(uint32_t i) const { return owner_[i].load(std::memory_order_acquire); }
  uint64_t abandoned(uint32_t i) const { return abandoned_[i].load(std::memory_order_acquire); }
  uint64_t done(uint32_t i) const { return __atomic_load_n(&done_[i], __ATOMIC_ACQUIRE); }

  // wait until ticket k owns slot k mod S; false after `timeout` (the caller
  // then gives up before posting: give_up_unposted)
  bool wait(uint64_t k, std::chrono::nanoseconds timeout) {
    const uint32_t i = (uint32_t)(k % S);
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0;; spin++) {
      const uint64_t f = owner(i);
      if (f == k) return true;
      // the owner f gave up after posting and its late result has landed: the
      // slot passes on (to k, or past tickets that gave up before posting)
      uint64_t ab = f + 1;
      if (f < k && abandoned_[i].load(std::memory_order_acquire) == ab && done(i) == f + 1 &&
          abandoned_[i].compare_exchange_strong(ab, 0, std::memory_order_acq_rel)) {
        hand_on(i, f + S);
        continue;
      }
      if ((spin & 255) == 255 && std::chrono::steady_clock::now() - t0 > timeout) return false;
      std::this_thread::yield();
    }
  }
  // ticket k has read its result: the slot goes to k + S
  void release(uint64_t k) { hand_on((uint32_t)(k % S), k + S); }
  // ticket k posted and gives up waiting for its result
  void abandon(uint64_t k) { abandoned_[k % S].store(k + 1, std::memory_order_release); }
  // ticket k never got its slot (wait timed out) and posts nothing
  void give_up_unposted(uint64_t k) {
    std::lock_guard<std::mutex> g(mu_);
    never_posted_.insert(k);
    n_never_posted_.fetch_add(1, std::memory_order_seq_cst);
    slot_timeouts++;
    skip_locked((uint32_t)(k % S));  // (the previous owner may have released the slot to k meanwhile)
  }
  // the oldest request among tickets < T that may be posted and is not yet
  // served (T if none): the device counter's restart point.  Slot i's oldest
  // unserved ticket is its owner f, or f + S once f's result is in; a ticket
  // that gave up before posting is never served and never waited on.
  uint64_t oldest_unserved(uint64_t T) {
    std::lock_guard<std::mutex> g(mu_);
    uint64_t c = T;
    for (uint32_t i = 0; i < S; i++) {
      const uint64_t f = owner(i);
      if (f >= T) continue;  // no ticket for this slot yet
      const uint64_t u = done(i) >= f + 1 ? f + S : f;
      if (u < T && !never_posted_.count(u)) c = std::min(c, u);
    }
    // tickets the slot has passed no longer matter
    for (auto it = never_posted_.begin(); it != never_posted_.end();)
      it = owner((uint32_t)(*it % S)) > *it ? never_posted_.erase(it) : std::next(it);
    return c;
  }
  size_t never_posted_size() {
    std::lock_guard<std::mutex> g(mu_);
    return never_posted_.size();
  }

  std::atomic<uint64_t> slot_timeouts{0}, skipped{0};

 private:
  // slot i goes to ticket v.  A ticket that gave up before posting never
  // takes or releases the slot, so the releaser passes it on past such
  // tickets (give_up_unposted checks the same from its side: seq_cst on both
  // sides, so at least one sees the other; the fix-up runs under mu_ and is
  // idempotent)
  void hand_on(uint32_t i, uint64_t v) {
    owner_[i].store(v, std::memory_order_seq_cst);
    if (n_never_posted_.load(std::memory_order_seq_cst) == 0) return;
    std::lock_guard<std::mutex> g(mu_);
    skip_locked(i);
  }
  void skip_locked(uint32_t i) {
    uint64_t v = owner_[i].load(std::memory_order_seq_cst);
    bool moved = false;
    while (never_posted_.count(v)) {
      v += S;
      skipped++;
      moved = true;
    }
    if (moved) owner_[i].store(v, std::memory_order_seq_cst);
  }

  const unsigned long long *done_;
  std::unique_ptr<std::atomic<uint64_t>[]> owner_, abandoned_;
  std::mutex mu_;
  std::set<uint64_t> never_posted_;
  std::atomic<uint64_t> n_never_posted_{0};
};

}  // namespace mqm
