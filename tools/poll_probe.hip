// tools/poll_probe.hip — does a large host -> device copy hold up a kernel
// that polls host memory (the per-publish server, k_serve, polls its ring of
// pinned slots)?  One wavefront polls a host word for up to 4 s and records
// the longest gap between two completed polls (s_memrealtime, 100 MHz); the
// host meanwhile copies 4 GB to the device in one of several ways.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

__global__ void poller(const int *flag, unsigned long long *out, unsigned long long max_ticks) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long last = t0, gap = 0, polls = 0;
  for (;;) {
    const int f = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    if (t - last > gap) gap = t - last;
    last = t;
    polls++;
    if (f || t - t0 > max_ticks) break;
    __builtin_amdgcn_s_sleep(2);
  }
  out[0] = gap;
  out[1] = polls;
}

__global__ __launch_bounds__(256) void fill(uint4 *p, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = make_uint4((uint32_t)i, 0u, 0u, 1u);
}

#define CK(x)                                                  \
  do {                                                         \
    hipError_t e = (x);                                        \
    if (e != hipSuccess) {                                     \
      printf("%s failed: %s\n", #x, hipGetErrorString(e));     \
      return 1;                                                \
    }                                                          \
  } while (0)

int main() {
  const size_t total = 4ull << 30, chunk = 32ull << 20;
  int *flag = nullptr;
  CK(hipHostMalloc((void **)&flag, 64, hipHostMallocMapped | hipHostMallocCoherent));
  unsigned long long *d_out = nullptr, h_out[2];
  CK(hipMalloc((void **)&d_out, 16));
  void *dst = nullptr, *pinned = nullptr;
  CK(hipMalloc(&dst, total));
  std::vector<char> pageable(total, 1);
  CK(hipHostMalloc(&pinned, total, hipHostMallocDefault));
  memset(pinned, 1, total);
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  const char *what[] = {"no copy", "pageable, one 4 GB copy", "pageable, 32 MB pieces queued",
                        "pageable, 32 MB pieces, sync + 200 us between", "pinned, one 4 GB copy",
                        "pinned, 32 MB pieces, sync + 200 us between", "hipMalloc 20 GB + memset",
                        "hipMallocAsync 20 GB + memset (+ free async)", "fill kernel over 16 GB (16384 x 256)",
                        "hipMallocAsync 20 GB again (pool warm)"};
  const size_t big = 20ull << 30;
  void *extra = nullptr;
  for (int mode = 0; mode < 10; mode++) {
    __atomic_store_n(flag, 0, __ATOMIC_SEQ_CST);
    hipLaunchKernelGGL(poller, dim3(1), dim3(64), 0, a, flag, d_out, 400000000ull);
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    const auto t = std::chrono::steady_clock::now();
    const char *src = mode >= 4 ? (const char *)pinned : pageable.data();
    if (mode == 6) {
      CK(hipMalloc(&extra, big));
      CK(hipMemsetAsync(extra, 0, big, b));
    } else if (mode == 7 || mode == 9) {
      void *x = nullptr;
      CK(hipMallocAsync(&x, big, b));
      CK(hipMemsetAsync(x, 0, big, b));
      CK(hipFreeAsync(x, b));
    } else if (mode == 8) {
      hipLaunchKernelGGL(fill, dim3(16384), dim3(256), 0, b, (uint4 *)extra, (uint64_t)(16ull << 30) / 16);
    } else if (mode == 1 || mode == 4) {
      CK(hipMemcpyAsync(dst, src, total, hipMemcpyHostToDevice, b));
    } else if (mode > 0) {
      for (size_t o = 0; o < total; o += chunk) {
        CK(hipMemcpyAsync((char *)dst + o, src + o, chunk, hipMemcpyHostToDevice, b));
        if (mode == 3 || mode == 5) {
          CK(hipStreamSynchronize(b));
          std::this_thread::sleep_for(std::chrono::microseconds(200));
        }
      }
    }
    CK(hipStreamSynchronize(b));
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    __atomic_store_n(flag, 1, __ATOMIC_SEQ_CST);
    CK(hipStreamSynchronize(a));
    CK(hipMemcpy(h_out, d_out, 16, hipMemcpyDeviceToHost));
    printf("%-48s copy %8.1f ms; longest gap between polls %8.3f ms (%llu polls)\n", what[mode], ms,
           h_out[0] / 1e5, h_out[1]);
  }
  if (extra) CK(hipFree(extra));
  printf("OK\n");
  return 0;
}
