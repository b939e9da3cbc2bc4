// tools/l2_probe.hip — can a kernel read stale cached lines of a small, hot
// device buffer that was refilled in place for new contents?  (Round 5/6: with
// snapshot buffers recycled in place, MQM_SNAP_RECYCLE=1, served results under
// churn missed the newest subscriptions although every version stamp the
// server read was right; tools/reuse_probe.hip's 256 MB buffers evict every
// L2 between reader and refill, so it cannot see this.)  A 4 MB buffer fits
// the L2s: a reader kernel on stream S warms them, the buffer is refilled by
// one of several writers (stream U unless noted, then U is synchronised), and
// the reader on S counts the words still holding the old pattern.  Each
// writer is tried as is and followed by a cache-flush kernel on U (a
// system-scope fence in workgroups on every XCD).  Measurement infrastructure,
// not product code.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                  \
  do {                                                         \
    hipError_t e = (x);                                        \
    if (e != hipSuccess) {                                     \
      printf("%s failed: %s\n", #x, hipGetErrorString(e));     \
      return 1;                                                \
    }                                                          \
  } while (0)

__global__ void count_eq(const unsigned *p, size_t n, unsigned a, unsigned long long *out) {
  unsigned long long c = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    c += p[i] == a;
  atomicAdd(out, c);
}

__global__ void fill(unsigned *p, size_t n, unsigned v) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}

// one system-scope acquire-release fence per workgroup (writes back and
// invalidates the caches of the XCD it runs on); a grid of many workgroups
// lands on every XCD
__global__ void flush_caches() {
  if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
}

int main() {
  const size_t n = 1u << 20, bytes = n * 4;  // 4 MB
  hipStream_t s, u;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&u, hipStreamNonBlocking));
  unsigned *m = nullptr, *stg = nullptr, *pinned = nullptr;
  unsigned long long *cnt = nullptr, h = 0;
  CK(hipMalloc(&m, bytes));
  CK(hipMalloc(&stg, bytes));
  CK(hipMalloc(&cnt, 8));
  CK(hipHostMalloc(&pinned, bytes, hipHostMallocDefault));
  std::vector<unsigned> pageable(n);
  const char *writers[] = {"H2D pageable on U", "H2D pinned on U", "kernel on U", "D2D copy on U",
                           "kernel on S (the reader's stream)", "H2D pageable on S"};
  unsigned pat = 0x11110000u;
  int fails = 0;
  for (int flush = 0; flush < 2; flush++) {
    for (int w = 0; w < 6; w++) {
      for (int rep = 0; rep < 3; rep++) {
        const unsigned old = ++pat, neu = ++pat;
        // old contents, then the reader warms the caches three times
        hipLaunchKernelGGL(fill, dim3(512), dim3(256), 0, s, m, n, old);
        CK(hipStreamSynchronize(s));
        for (int k = 0; k < 3; k++) {
          CK(hipMemsetAsync(cnt, 0, 8, s));
          hipLaunchKernelGGL(count_eq, dim3(2048), dim3(256), 0, s, (const unsigned *)m, n, old, cnt);
        }
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(&h, cnt, 8, hipMemcpyDeviceToHost));
        const unsigned long long warm = h;
        // the refill
        for (size_t i = 0; i < n; i++) pageable[i] = pinned[i] = neu;
        switch (w) {
          case 0: CK(hipMemcpyAsync(m, pageable.data(), bytes, hipMemcpyHostToDevice, u)); break;
          case 1: CK(hipMemcpyAsync(m, pinned, bytes, hipMemcpyHostToDevice, u)); break;
          case 2: hipLaunchKernelGGL(fill, dim3(512), dim3(256), 0, u, m, n, neu); break;
          case 3:
            hipLaunchKernelGGL(fill, dim3(512), dim3(256), 0, u, stg, n, neu);
            CK(hipMemcpyAsync(m, stg, bytes, hipMemcpyDeviceToDevice, u));
            break;
          case 4: hipLaunchKernelGGL(fill, dim3(512), dim3(256), 0, s, m, n, neu); break;
          case 5: CK(hipMemcpyAsync(m, pageable.data(), bytes, hipMemcpyHostToDevice, s)); break;
        }
        CK(hipGetLastError());
        if (flush) hipLaunchKernelGGL(flush_caches, dim3(4096), dim3(64), 0, w >= 4 ? s : u);
        CK(hipStreamSynchronize(u));
        CK(hipStreamSynchronize(s));
        CK(hipMemsetAsync(cnt, 0, 8, s));
        hipLaunchKernelGGL(count_eq, dim3(2048), dim3(256), 0, s, (const unsigned *)m, n, old, cnt);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(&h, cnt, 8, hipMemcpyDeviceToHost));
        printf("%-36s flush %d rep %d: warm reads %llu of %zu, stale words after the refill %llu\n", writers[w],
               flush, rep, warm / 3, n, h);
        if (h) fails++;
      }
    }
  }
  printf("%s (%d runs with stale words)\n", fails ? "STALE" : "OK", fails);
  CK(hipHostFree(pinned));
  CK(hipFree(cnt));
  CK(hipFree(stg));
  CK(hipFree(m));
  return 0;
}
