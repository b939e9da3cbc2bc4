// tools/reuse_probe.hip — can a kernel read stale data from device memory
// that the stream-ordered pool handed back out and a host -> device copy
// refilled?  (Round 5: with snapshot buffers from the pool, the served path
// under churn returned results missing the newest subscriptions; with
// hipMalloc / hipFree it did not.)  A kernel reads buffer M (pattern A) on
// stream S; M is freed on stream R, reallocated on stream U (same address
// when the pool reuses it), refilled with pattern B by a host -> device copy
// on U; after synchronising U, a kernel on S counts the words still holding A.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ void count_a(const unsigned *p, size_t n, unsigned a, unsigned long long *out) {
  unsigned long long c = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    c += p[i] == a;
  atomicAdd(out, c);
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
  const size_t n = 64ull << 20, bytes = n * 4;  // 256 MB
  hipStream_t s, r, u;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&r, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&u, hipStreamNonBlocking));
  hipMemPool_t pool;
  CK(hipDeviceGetDefaultMemPool(&pool, 0));
  uint64_t keep = ~0ull;
  CK(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep));
  std::vector<unsigned> a(n, 0xAAAAAAAAu), b(n, 0xBBBBBBBBu);
  unsigned long long *cnt = nullptr, h = 0;
  CK(hipMalloc((void **)&cnt, 8));
  void *keep_buf = nullptr;  // mode 4: one hipMalloc'd buffer refilled in place (no free)
  for (int mode = 0; mode < 6; mode++) {
    // mode 0: pool, copy on U; 1: pool, copy on S (the reading stream);
    // 2: pool, D2D through a fresh staging buffer; 3: hipMalloc / hipFree
    void *m = nullptr;
    if (mode == 3 || mode == 5)
      CK(hipMalloc(&m, bytes));
    else if (mode == 4) {
      if (!keep_buf) CK(hipMalloc(&keep_buf, bytes));
      m = keep_buf;
    } else
      CK(hipMallocAsync(&m, bytes, u));
    CK(hipMemcpyAsync(m, a.data(), bytes, hipMemcpyHostToDevice, u));
    CK(hipStreamSynchronize(u));
    CK(hipMemsetAsync(cnt, 0, 8, s));
    hipLaunchKernelGGL(count_a, dim3(1024), dim3(256), 0, s, (const unsigned *)m, n, 0xAAAAAAAAu, cnt);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(&h, cnt, 8, hipMemcpyDeviceToHost));
    const unsigned long long first = h;
    void *m2 = nullptr;
    if (mode == 4 || mode == 5) {
      m2 = m;  // refilled in place
    } else if (mode == 3) {
      CK(hipFree(m));
      CK(hipMalloc(&m2, bytes));
    } else {
      CK(hipFreeAsync(m, r));
      CK(hipStreamSynchronize(r));
      CK(hipMallocAsync(&m2, bytes, u));
    }
    if (mode == 1) {
      CK(hipStreamSynchronize(u));
      CK(hipMemcpyAsync(m2, b.data(), bytes, hipMemcpyHostToDevice, s));
      CK(hipStreamSynchronize(s));
    } else if (mode == 2) {
      void *stg = nullptr;
      CK(hipMalloc(&stg, bytes));
      CK(hipMemcpy(stg, b.data(), bytes, hipMemcpyHostToDevice));
      CK(hipMemcpyAsync(m2, stg, bytes, hipMemcpyDeviceToDevice, u));
      CK(hipStreamSynchronize(u));
      CK(hipFree(stg));
    } else {
      CK(hipMemcpyAsync(m2, b.data(), bytes, hipMemcpyHostToDevice, u));
      CK(hipStreamSynchronize(u));
    }
    CK(hipMemsetAsync(cnt, 0, 8, s));
    hipLaunchKernelGGL(count_a, dim3(1024), dim3(256), 0, s, (const unsigned *)m2, n, 0xAAAAAAAAu, cnt);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(&h, cnt, 8, hipMemcpyDeviceToHost));
    const char *what[] = {"pool, refill H2D on another stream", "pool, refill H2D on the reading stream",
                          "pool, refill D2D from a fresh buffer", "hipMalloc / hipFree",
                          "one hipMalloc buffer refilled (kept)", "fresh hipMalloc buffer refilled"};
    printf("%-42s same address %d; A words before %llu / %zu, stale A words after refill %llu\n", what[mode],
           m2 == m, first, n, h);
    if (mode == 3 || mode == 5)
      CK(hipFree(m2));
    else if (mode != 4)
      CK(hipFreeAsync(m2, u));
    CK(hipStreamSynchronize(u));
  }
  if (keep_buf) CK(hipFree(keep_buf));
  printf("OK\n");
  return 0;
}
