// tools/free_probe.hip — does freeing device memory wait for a kernel that
// is still running on another stream?  The per-publish server (k_serve) is a
// kernel that runs as long as requests arrive; a snapshot freed meanwhile
// (hipFree in ~GpuSnapshot) would then wait for it.  A spinner kernel runs on
// stream A until the host sets a flag (or 3 s pass, on the device's clock);
// the host times hipMalloc + hipFree, hipFreeAsync of hipMalloc'd memory,
// and hipMallocAsync + hipFreeAsync, all while the spinner runs.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <thread>

__global__ void spin(volatile int *flag, unsigned long long max_ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0)
    while (__hip_atomic_load((int *)flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0 &&
           __builtin_amdgcn_s_memrealtime() - t0 < max_ticks)
      __builtin_amdgcn_s_sleep(8);
}

static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      printf("%s failed: %s\n", #x, hipGetErrorString(e));                           \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

int main() {
  int *flag = nullptr;
  CK(hipHostMalloc((void **)&flag, 4, hipHostMallocMapped | hipHostMallocCoherent));
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  const size_t sz = 1ull << 30;
  for (int mode = 0; mode < 3; mode++) {
    *flag = 0;
    void *p = nullptr;
    if (mode == 2)
      CK(hipMallocAsync(&p, sz, b));
    else
      CK(hipMalloc(&p, sz));
    CK(hipStreamSynchronize(b));
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, a, flag, 300000000ull);  // 3 s at 100 MHz
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    // release the spinner after 1 s from a helper thread
    std::thread rel([&] {
      std::this_thread::sleep_for(std::chrono::milliseconds(1000));
      __atomic_store_n(flag, 1, __ATOMIC_SEQ_CST);
    });
    const auto t = std::chrono::steady_clock::now();
    if (mode == 0) CK(hipFree(p));
    if (mode == 1) CK(hipFreeAsync(p, b));
    if (mode == 2) CK(hipFreeAsync(p, b));
    const double f = ms_since(t);
    const auto t2 = std::chrono::steady_clock::now();
    CK(hipStreamSynchronize(b));
    const double s = ms_since(t2);
    rel.join();
    CK(hipStreamSynchronize(a));
    const char *what[3] = {"hipMalloc + hipFree", "hipMalloc + hipFreeAsync(b)", "hipMallocAsync + hipFreeAsync(b)"};
    printf("%-36s free call %8.1f ms, then sync(b) %8.1f ms  (spinner released at ~1000 ms)\n", what[mode], f, s);
  }
  // hipMalloc while the spinner runs
  *flag = 0;
  hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, a, flag, 300000000ull);
  std::this_thread::sleep_for(std::chrono::milliseconds(50));
  std::thread rel([&] {
    std::this_thread::sleep_for(std::chrono::milliseconds(1000));
    __atomic_store_n(flag, 1, __ATOMIC_SEQ_CST);
  });
  const auto t = std::chrono::steady_clock::now();
  void *q = nullptr;
  CK(hipMalloc(&q, sz));
  printf("%-36s call %8.1f ms\n", "hipMalloc (spinner running)", ms_since(t));
  rel.join();
  CK(hipStreamSynchronize(a));
  CK(hipFree(q));
  printf("OK\n");
  return 0;
}
