// tools/duplex_probe.hip — do host->device and device->host transfers overlap?
//
// The runs-form host path (bench.py `host_path`) moves ~29 MB in and ~108 MB
// out per 500k-topic call; its rate sits at 0.66 of max(in, out) / one-way
// rate and 0.83 of (in + out) / one-way rate, as if the two directions took
// turns.  This probe times, on pinned host memory:
//   h2d / d2h        : hipMemcpyAsync one way, alone
//   both             : both ways at once, each on its own stream
//   kd2h / kh2d      : a kernel storing to / loading from mapped host memory
//                      (the copy done by the CUs over PCIe, no DMA engine)
//   kd2h+h2d, kh2d+d2h: one direction by kernel, the other by DMA, at once
// for each kind of pinned host memory (hipHostMalloc flags, hipHostRegister).
// Every rate is bytes of one direction / wall time of the whole pass.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

// n16 16-B units from src to dst, grid-stride, 4 in flight per lane
__global__ void __launch_bounds__(256) k_copy(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n16) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static const char *kind_name(unsigned f) {
  switch (f) {
    case hipHostMallocDefault: return "default";
    case hipHostMallocMapped: return "mapped";
    case hipHostMallocCoherent: return "coherent";
    case hipHostMallocNonCoherent: return "noncoherent";
    default: return "?";
  }
}

int main(int argc, char **argv) {
  const size_t mb = argc > 1 ? strtoull(argv[1], nullptr, 10) : 128;
  const int reps = argc > 2 ? atoi(argv[2]) : 16;
  const int blocks = argc > 3 ? atoi(argv[3]) : 512;
  const size_t bytes = mb << 20;
  const size_t n16 = bytes / 16;
  void *d_in, *d_out;
  CK(hipMalloc(&d_in, bytes));
  CK(hipMalloc(&d_out, bytes));
  CK(hipMemset(d_in, 3, bytes));
  CK(hipMemset(d_out, 4, bytes));
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  printf("buffer %zu MB, %d reps, copy kernel %d blocks\n", mb, reps, blocks);
  // host memory kinds: hipHostMalloc flags, then malloc + hipHostRegister
  const unsigned kinds[] = {hipHostMallocDefault, hipHostMallocMapped, hipHostMallocCoherent, hipHostMallocNonCoherent,
                            0xFFFFFFFFu};
  for (unsigned kind : kinds) {
    void *h_in, *h_out;
    if (kind == 0xFFFFFFFFu) {
      h_in = aligned_alloc(4096, bytes);
      h_out = aligned_alloc(4096, bytes);
      memset(h_in, 1, bytes);
      memset(h_out, 2, bytes);
      CK(hipHostRegister(h_in, bytes, hipHostRegisterDefault));
      CK(hipHostRegister(h_out, bytes, hipHostRegisterDefault));
    } else {
      CK(hipHostMalloc(&h_in, bytes, kind));
      CK(hipHostMalloc(&h_out, bytes, kind));
      memset(h_in, 1, bytes);
      memset(h_out, 2, bytes);
    }
    void *hd_in, *hd_out;  // device views of the host buffers
    CK(hipHostGetDevicePointer(&hd_in, h_in, 0));
    CK(hipHostGetDevicePointer(&hd_out, h_out, 0));
    printf("-- host memory: %s\n", kind == 0xFFFFFFFFu ? "malloc + hipHostRegister" : kind_name(kind));
    auto run = [&](int k, hipStream_t s) {
      switch (k) {
        case 1: CK(hipMemcpyAsync(d_in, h_in, bytes, hipMemcpyHostToDevice, s)); break;
        case 2: CK(hipMemcpyAsync(h_out, d_out, bytes, hipMemcpyDeviceToHost, s)); break;
        case 3: k_copy<<<blocks, 256, 0, s>>>((const uint4 *)d_out, (uint4 *)hd_out, n16); CK(hipGetLastError()); break;
        case 4: k_copy<<<blocks, 256, 0, s>>>((const uint4 *)hd_in, (uint4 *)d_in, n16); CK(hipGetLastError()); break;
        default: break;
      }
    };
    struct Case {
      const char *name;
      int ka, kb;  // 0 none, 1 h2d, 2 d2h, 3 kd2h, 4 kh2d
    } cases[] = {{"h2d", 1, 0}, {"d2h", 2, 0}, {"both", 1, 2}, {"kd2h", 3, 0},
                 {"kh2d", 4, 0}, {"kd2h+h2d", 3, 1}, {"kh2d+d2h", 4, 2}, {"d2h(again)", 2, 0}};
    for (const Case &c : cases) {
      for (int w = 0; w < 2; w++) {
        run(c.ka, a);
        run(c.kb, b);
      }
      CK(hipDeviceSynchronize());
      const double t0 = now();
      for (int r = 0; r < reps; r++) {
        run(c.ka, a);
        run(c.kb, b);
      }
      CK(hipDeviceSynchronize());
      const double t = now() - t0;
      printf("%-12s %7.2f ms per rep  %6.1f GB/s per direction%s\n", c.name, t / reps * 1e3,
             (double)bytes * reps / t / 1e9, c.kb ? "  (both directions at once)" : "");
    }
    // the kernel copy moved the bytes (the fill finished first: a non-blocking
    // stream does not wait for the null stream)
    CK(hipMemset(d_out, 0x5A, bytes));
    CK(hipDeviceSynchronize());
    run(3, a);
    CK(hipStreamSynchronize(a));
    size_t bad = 0;
    for (size_t i = 0; i < bytes; i += 4099) bad += ((unsigned char *)h_out)[i] != 0x5A;
    printf("kd2h check: %zu bad bytes sampled\n", bad);
    if (kind == 0xFFFFFFFFu) {
      CK(hipHostUnregister(h_in));
      CK(hipHostUnregister(h_out));
      free(h_in);
      free(h_out);
    } else {
      CK(hipHostFree(h_in));
      CK(hipHostFree(h_out));
    }
    if (bad) return 1;
  }
  CK(hipFree(d_in));
  CK(hipFree(d_out));
  return 0;
}
