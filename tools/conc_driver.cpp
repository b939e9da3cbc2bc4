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

// (n_batches calls over the n_distinct batches in the topic buffer, cycling:
// many calls amortise the threads' start and the last calls' tail)
int64_t mqd_host_path(const mqd_host_api *api, void *h, const char *bytes, const uint64_t *offs, uint32_t per,
                      uint32_t n_batches, uint32_t n_distinct, int threads, int consume, uint64_t *deliveries,
                      uint64_t *checksum) {
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
        if (api->batch(h, bytes, offs + (uint64_t)(b % n_distinct) * per, per, &res) != 0) {
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

// ---- per-publish calls while subscriptions change (bench.py serve_churn) --
// `threads` native callers make mqm_subscribers calls for `seconds` while one
// mutator thread runs Subscribe / Unsubscribe at `rate` per second (the
// reference takes both concurrently: Subscribe under the trie's root mutex,
// server.go:1013 / topics.go:303-321, beside one Subscribers goroutine per
// connection, server.go:776).  Mutation k: even k subscribes pair k/2 mod m,
// odd k unsubscribes pair (k/2 + m/2) mod m (about half the pairs present at
// any time).  Recorded: every call's latency (ns, saturated to u32), and per
// sampled call (every `sample`-th) its return time (us since the start) and
// result snapshot version; per mutation its time (us) and the store version
// after it.  -> wall ns, or -1 if a call failed.
extern "C" {
typedef uint64_t (*version_fn)(const void *r);
typedef int (*subscribe_fn)(void *h, const char *c, size_t cl, const char *f, size_t fl, const void *sub, int *is_new);
typedef int (*unsubscribe_fn)(void *h, const char *f, size_t fl, const char *c, size_t cl, int *existed);
typedef int (*state_fn)(void *h, void *state);
struct mqd_churn_api {
  subscribers_fn subscribers;
  offsets_fn offsets;
  free_fn result_free;
  version_fn version;
  subscribe_fn subscribe;
  unsubscribe_fn unsubscribe;
  state_fn state;
};
struct mqd_churn_out {
  uint64_t calls, deliveries, mutations, failed_mutations;
  // the slowest call of each thread: its latency (ns) and return time (us since the start)
  uint64_t slow_ns[256], slow_t_us[256];
  // snapshot publishes the mutator saw (mqm_commit_state builds moving): time (us), builds
  uint64_t n_pub, pub_t_us[256], pub_builds[256];
};

int64_t mqd_serve_churn(const mqd_churn_api *api, void *h, const char *bytes, const uint64_t *offs, uint32_t n,
                        int threads, double seconds, uint32_t cap_per_thread, uint32_t sample, const char *cbytes,
                        const uint64_t *coffs, const char *fbytes, const uint64_t *foffs, uint32_t m, double rate,
                        uint32_t *lat_ns, uint32_t *calls_done, uint32_t *s_t_us, uint64_t *s_ver,
                        uint64_t mut_cap, uint32_t *m_t_us, uint64_t *m_ver, mqd_churn_out *out) {
  std::atomic<int> ready{0}, failed{0};
  std::atomic<bool> go{false}, stop{false};
  std::atomic<uint64_t> dsum{0}, nmut{0}, mfail{0};
  std::vector<std::thread> ths;
  using clk = std::chrono::steady_clock;
  clk::time_point t0;
  const uint32_t per_s = cap_per_thread / (sample ? sample : 1) + 1;
  for (int k = 0; k < threads; k++) {
    ths.emplace_back([&, k] {
      ready++;
      while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
      uint64_t d = 0, slow = 0, slow_t = 0;
      uint32_t j = 0;
      for (; j < cap_per_thread && !stop.load(std::memory_order_relaxed); j++) {
        const uint32_t t = (uint32_t)(((uint64_t)k * 7919u + (uint64_t)j * 104729u) % n);
        void *res = nullptr;
        const auto a = clk::now();
        if (api->subscribers(h, bytes + offs[t], offs[t + 1] - offs[t], &res) != 0) {
          failed++;
          break;
        }
        const auto b = clk::now();
        d += api->offsets(res)[1];
        const uint64_t ns = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count();
        lat_ns[(uint64_t)k * cap_per_thread + j] = ns > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)ns;
        if (ns > slow) {
          slow = ns;
          slow_t = (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(b - t0).count();
        }
        if (sample && j % sample == 0) {
          const uint64_t si = (uint64_t)k * per_s + j / sample;
          s_t_us[si] = (uint32_t)std::chrono::duration_cast<std::chrono::microseconds>(b - t0).count();
          s_ver[si] = api->version(res);
        }
        api->result_free(res);
      }
      calls_done[k] = j;
      dsum += d;
      if (k < 256) {
        out->slow_ns[k] = slow;
        out->slow_t_us[k] = slow_t;
      }
    });
  }
  out->n_pub = 0;
  std::thread mut([&] {
    while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
    if (rate <= 0 || m == 0) return;
    const uint8_t sub[8] = {1, 0, 0, 0, 0, 0, 0, 0};  // mqm_subscription: QoS 1, Identifier 0
    struct {
      uint64_t store_version, snapshot_version, pending_ops, builds, last_build_ops;
      double last_build_ms;
      int32_t has_snapshot, building;
    } st;
    for (uint64_t k = 0; k < mut_cap && !stop.load(std::memory_order_relaxed); k++) {
      if ((k & 63) == 0) {  // pace: mutation k is due at t0 + k / rate
        const auto due = t0 + std::chrono::nanoseconds((int64_t)((double)k * 1e9 / rate));
        while (clk::now() < due && !stop.load(std::memory_order_relaxed))
          std::this_thread::sleep_for(std::chrono::microseconds(50));
      }
      const uint32_t p = (k & 1) ? (uint32_t)((k / 2 + m / 2) % m) : (uint32_t)((k / 2) % m);
      int x = 0;
      const int rc = (k & 1) ? api->unsubscribe(h, fbytes + foffs[p], foffs[p + 1] - foffs[p], cbytes + coffs[p],
                                                coffs[p + 1] - coffs[p], &x)
                             : api->subscribe(h, cbytes + coffs[p], coffs[p + 1] - coffs[p], fbytes + foffs[p],
                                              foffs[p + 1] - foffs[p], sub, &x);
      if (rc != 0) mfail++;
      const uint64_t b0 = k ? st.builds : 0;
      api->state(h, &st);
      m_t_us[k] = (uint32_t)std::chrono::duration_cast<std::chrono::microseconds>(clk::now() - t0).count();
      m_ver[k] = st.store_version;
      if (k && st.builds != b0 && out->n_pub < 256) {
        out->pub_t_us[out->n_pub] = m_t_us[k];
        out->pub_builds[out->n_pub++] = st.builds;
      }
      nmut++;
    }
  });
  while (ready.load() < threads) std::this_thread::yield();
  t0 = clk::now();
  go.store(true, std::memory_order_release);
  std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
  stop.store(true, std::memory_order_release);
  for (auto &t : ths) t.join();
  mut.join();
  const int64_t ns = std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - t0).count();
  uint64_t calls = 0;
  for (int k = 0; k < threads; k++) calls += calls_done[k];
  out->calls = calls;
  out->deliveries = dsum.load();
  out->mutations = nmut.load();
  out->failed_mutations = mfail.load();
  return failed.load() ? -1 : ns;
}
}
