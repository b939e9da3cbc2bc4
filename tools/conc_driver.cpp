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

// ---- the host path as a broker drives it (bench.py host_path) -------------
// `threads` native callers claim batches [b * per, (b + 1) * per) of the
// pinned topics in turn, match each (mqm_match_batch_packed or
// mqm_match_batch_runs), then consume the result on the calling thread:
//   consume 0: nothing past the result's arrival in host memory
//   consume 1: read every delivery once (a checksum: what the cgo shim's loop
//              over a topic's subscribers costs before any per-client work)
//   consume 2: expand to plain packed rows (mqm_result_expand) into a buffer
// -> wall nanoseconds (-1 on a failed call); *deliveries and *checksum summed
extern "C" {
typedef int (*batch_fn)(void *h, const char *bytes, const uint64_t *offs, uint32_t n, void **out);
typedef const uint32_t *(*packed_fn)(const void *r);
typedef int (*runs_fn)(const void *r, const uint64_t **ro, const uint32_t **runs, const uint32_t **words,
                       uint64_t *n_words);
typedef int (*expand_fn)(const void *r, uint32_t t0, uint32_t t1, uint64_t *offsets, uint32_t *dst);
struct mqd_host_api {
  batch_fn batch;
  offsets_fn offsets;
  packed_fn packed;
  runs_fn runs;
  expand_fn expand;
  free_fn result_free;
};

int64_t mqd_host_path(const mqd_host_api *api, void *h, const char *bytes, const uint64_t *offs, uint32_t per,
                      uint32_t n_batches, int threads, int consume, uint64_t *deliveries, uint64_t *checksum) {
  std::atomic<uint32_t> next{0};
  std::atomic<int> failed{0};
  std::atomic<uint64_t> dsum{0}, csum{0};
  std::vector<std::thread> ths;
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  for (int k = 0; k < threads; k++) {
    ths.emplace_back([&] {
      std::vector<uint32_t> rows;
      std::vector<uint64_t> roffs(per + 1);
      uint64_t d = 0, c = 0;
      for (;;) {
        const uint32_t b = next.fetch_add(1);
        if (b >= n_batches) break;
        void *res = nullptr;
        if (api->batch(h, bytes, offs + (uint64_t)b * per, per, &res) != 0) {
          failed++;
          break;
        }
        const uint64_t *wo = api->offsets(res);
        const uint32_t *pk = api->packed(res);
        const uint64_t *ro = nullptr;
        const uint32_t *runs = nullptr, *words = nullptr;
        uint64_t nw = 0;
        const bool is_runs = api->runs && api->runs(res, &ro, &runs, &words, &nw) == 0;
        if (consume == 2) {
          api->expand(res, 0, per, roffs.data(), nullptr);
          rows.resize(roffs[per]);
          api->expand(res, 0, per, roffs.data(), rows.data());
          d += roffs[per];
          c += rows.empty() ? 0 : rows[rows.size() / 2];
        } else {
          uint64_t nd = wo[per];
          if (is_runs)
            for (uint64_t k = 0; k < ro[per]; k++) nd += runs[2 * k + 1];
          d += nd;
          if (consume == 1) {
            uint64_t x = 0;
            for (uint32_t t = 0; t < per; t++) {
              if (is_runs)
                for (uint64_t k = ro[t]; k < ro[t + 1]; k++) {
                  const uint32_t *w = words + runs[2 * k];
                  for (uint32_t i = 0; i < runs[2 * k + 1]; i++) x += w[i];
                }
              for (uint64_t i = wo[t]; i < wo[t + 1]; i++) x += pk[i];
            }
            c += x;
          }
        }
        api->result_free(res);
      }
      dsum += d;
      csum += c;
    });
  }
  for (auto &t : ths) t.join();
  const int64_t ns = std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - t0).count();
  *deliveries = dsum.load();
  *checksum = csum.load();
  return failed.load() ? -1 : ns;
}
}
