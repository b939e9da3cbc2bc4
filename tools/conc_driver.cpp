// tools/conc_driver.cpp — benchmark driver (not product code): the
// reference's per-publish call shape from native threads.  mochi calls
// Subscribers(topic) once per PUBLISH from one goroutine per connection
// (server.go:776, listeners/tcp.go:83, clients.go:331-356); Python threads
// cannot issue calls at that rate (the interpreter lock), so bench.py hands
// the index and the library's entry points to this driver, which runs
// `threads` std::threads each making `calls` mqm_subscribers calls and reading
// every result's delivery count, as a broker would before fanning out.
#include <stdint.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

extern "C" {

typedef int (*subscribers_fn)(void *h, const char *topic, size_t len, void **out);
typedef const uint64_t *(*offsets_fn)(const void *r);
typedef void (*free_fn)(void *r);

struct mqd_api {
  subscribers_fn subscribers;
  offsets_fn offsets;
  free_fn result_free;
};

// -> wall nanoseconds of the timed region (all threads started together), or
// -1 if a call failed; lat_ns[k * calls + j] = call j of thread k; *deliveries
// = the sum of every result's delivery count
int64_t mqd_concurrent(const mqd_api *api, void *h, const char *bytes, const uint64_t *offs, uint32_t n, int threads,
                       int calls, uint64_t *lat_ns, uint64_t *deliveries) {
  std::atomic<int> ready{0}, failed{0};
  std::atomic<bool> go{false};
  std::atomic<uint64_t> dsum{0};
  std::vector<std::thread> ths;
  using clk = std::chrono::steady_clock;
  for (int k = 0; k < threads; k++) {
    ths.emplace_back([&, k] {
      ready++;
      while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
      uint64_t d = 0;
      for (int j = 0; j < calls; j++) {
        const uint32_t t = (uint32_t)(((uint64_t)k * calls + j) % n);
        void *res = nullptr;
        const auto t0 = clk::now();
        const int rc = api->subscribers(h, bytes + offs[t], offs[t + 1] - offs[t], &res);
        if (rc != 0) {
          failed++;
          return;
        }
        d += api->offsets(res)[1];
        lat_ns[(uint64_t)k * calls + j] = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - t0).count();
        api->result_free(res);
      }
      dsum += d;
    });
  }
  while (ready.load() < threads) std::this_thread::yield();
  const auto t0 = clk::now();
  go.store(true, std::memory_order_release);
  for (auto &t : ths) t.join();
  const int64_t ns = std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - t0).count();
  *deliveries = dsum.load();
  return failed.load() ? -1 : ns;
}
}
