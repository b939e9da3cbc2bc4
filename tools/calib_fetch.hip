// tools/calib_fetch.hip — calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on
// gfx950 for the access patterns of the match kernels, against known byte
// counts (MI355X_MICROARCH.md §HBM: FETCH_SIZE is calibrated there only for
// 16-B-per-lane coalesced streaming reads; "calibrate on a known byte count in
// your own access pattern").  Measurement infrastructure, not product code.
//
// Every kernel touches a 4 GiB table (far past the 256 MiB Infinity Cache and
// the L2s) so each access is a DRAM fetch; gathers go to distinct random
// lines (a multiplicative permutation of the line index) so no line is
// fetched twice within a launch.
//   k_stream16  : 16 B per lane, coalesced (the guide's reference pattern)
//   k_gather64  : one 64-B entry per lane (4 x 16-B loads), random — the
//                 walk's edge-entry / node-descriptor load (device.h walk_step)
//   k_gather32  : one 32-B descriptor per lane, random (load_desc)
//   k_gather8   : one 8-B entry per lane, random (a lone SubEnt load)
//   k_run256    : 64 lanes read one 512-B run (8 B per lane) at a random
//                 128-B aligned place — a short subscription range
//   k_write16   : 16 B per lane, coalesced stores (the emit's delivery stream)
//   k_write8    : 8 B per lane, coalesced stores
// Prints, per kernel, the algorithmic bytes it moved; divide rocprofv3's
// FETCH_SIZE (KiB) * 1024 or WRITE_SIZE * 1024 by it for the factor.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                            \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

constexpr uint64_t kTable = 4ull << 30;       // bytes
constexpr uint64_t kLines = kTable / 128;     // 128-B lines
constexpr uint64_t kOdd = 0x9E3779B97F4A7C15ull;

__device__ __forceinline__ uint64_t line_of(uint64_t i) { return (i * kOdd) & (kLines - 1); }  // kLines: power of 2

__global__ void k_stream16(const uint4 *__restrict__ t, uint64_t n, uint4 *__restrict__ sink) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = t[i];
    acc.x ^= v.x, acc.y ^= v.y, acc.z ^= v.z, acc.w ^= v.w;
  }
  if ((acc.x & acc.y & acc.z & acc.w) == 0x12345678u) sink[0] = acc;
}

template <int kWords4>  // 16-B loads per lane from one random line
__global__ void k_gather(const uint4 *__restrict__ t, uint64_t n, uint4 *__restrict__ sink) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 *p = t + line_of(i) * 8;
#pragma unroll
    for (int k = 0; k < kWords4; k++) {
      const uint4 v = p[k];
      acc.x ^= v.x, acc.y ^= v.y, acc.z ^= v.z, acc.w ^= v.w;
    }
  }
  if ((acc.x & acc.y & acc.z & acc.w) == 0x12345678u) sink[0] = acc;
}

// kL lanes read one random (kL x 16)-B entry together, 16 B each: one load
// instruction touches 64 / kL lines instead of 64 (the walk's cooperative probe)
template <int kL>
__global__ void k_coop(const uint4 *__restrict__ t, uint64_t n, uint4 *__restrict__ sink) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  const uint64_t g0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / kL, gs = (uint64_t)gridDim.x * blockDim.x / kL;
  const int c = threadIdx.x % kL;
  for (uint64_t i = g0; i < n; i += gs) {
    const uint4 v = t[line_of(i) * 8 + c];
    acc.x ^= v.x, acc.y ^= v.y, acc.z ^= v.z, acc.w ^= v.w;
  }
  if ((acc.x & acc.y & acc.z & acc.w) == 0x12345678u) sink[0] = acc;
}

__global__ void k_gather8(const uint2 *__restrict__ t, uint64_t n, uint4 *__restrict__ sink) {
  uint2 acc = make_uint2(0, 0);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint2 v = t[line_of(i) * 16];
    acc.x ^= v.x, acc.y ^= v.y;
  }
  if ((acc.x & acc.y) == 0x12345678u) sink[0] = make_uint4(acc.x, acc.y, 0, 0);
}

// one wavefront per run: 64 lanes x 8 B = 512 B starting at a random 128-B line
__global__ void k_run256(const uint2 *__restrict__ t, uint64_t runs, uint4 *__restrict__ sink) {
  const int lane = threadIdx.x & 63;
  uint2 acc = make_uint2(0, 0);
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x / 64);
  for (uint64_t r = (uint64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; r < runs; r += nw) {
    const uint64_t line = ((r * kOdd) & (kLines / 4 - 1)) * 4;  // distinct 512-B aligned runs
    const uint2 v = t[line * 16 + lane];
    acc.x ^= v.x, acc.y ^= v.y;
  }
  if ((acc.x & acc.y) == 0x12345678u) sink[0] = make_uint4(acc.x, acc.y, 0, 0);
}

__global__ void k_write16(uint4 *__restrict__ t, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    t[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

__global__ void k_write8(uint2 *__restrict__ t, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    t[i] = make_uint2((uint32_t)i, 1);
}

int main() {
  void *tab = nullptr, *sink = nullptr;
  CHECK(hipMalloc(&tab, kTable));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMemset(tab, 1, kTable));
  const dim3 grid(256 * 8), block(256);
  const uint64_t gathers = 16ull << 20;  // 16M random accesses (< kLines = 32M distinct lines)
  struct Row {
    const char *name;
    double bytes;
  } rows[16];
  int nr = 0;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  auto timed = [&](const char *name, double bytes, auto launch) {
    launch();  // warm (page tables)
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    launch();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    printf("%-11s algorithmic %.0f bytes per launch, %.3f ms, %.1f GB/s\n", name, bytes, ms, bytes / ms / 1e6);
    rows[nr++] = Row{name, bytes};
  };
  const uint4 *t4 = (const uint4 *)tab;
  timed("k_stream16", (double)kTable,
        [&] { hipLaunchKernelGGL(k_stream16, grid, block, 0, 0, t4, kTable / 16, (uint4 *)sink); });
  timed("k_gather64", 64.0 * gathers,
        [&] { hipLaunchKernelGGL(k_gather<4>, grid, block, 0, 0, t4, gathers, (uint4 *)sink); });
  timed("k_gather32", 32.0 * gathers,
        [&] { hipLaunchKernelGGL(k_gather<2>, grid, block, 0, 0, t4, gathers, (uint4 *)sink); });
  timed("k_coop4x16", 64.0 * gathers,
        [&] { hipLaunchKernelGGL(k_coop<4>, grid, block, 0, 0, t4, gathers, (uint4 *)sink); });
  timed("k_coop2x16", 32.0 * gathers,
        [&] { hipLaunchKernelGGL(k_coop<2>, grid, block, 0, 0, t4, gathers, (uint4 *)sink); });
  timed("k_coop8x16", 128.0 * gathers,
        [&] { hipLaunchKernelGGL(k_coop<8>, grid, block, 0, 0, t4, gathers, (uint4 *)sink); });
  timed("k_coop1x16", 16.0 * gathers,
        [&] { hipLaunchKernelGGL(k_coop<1>, grid, block, 0, 0, t4, gathers, (uint4 *)sink); });
  timed("k_gather8", 8.0 * gathers,
        [&] { hipLaunchKernelGGL(k_gather8, grid, block, 0, 0, (const uint2 *)tab, gathers, (uint4 *)sink); });
  const uint64_t runs = 4ull << 20;
  timed("k_run256", 512.0 * runs,
        [&] { hipLaunchKernelGGL(k_run256, grid, block, 0, 0, (const uint2 *)tab, runs, (uint4 *)sink); });
  timed("k_write16", (double)kTable, [&] { hipLaunchKernelGGL(k_write16, grid, block, 0, 0, (uint4 *)tab, kTable / 16); });
  timed("k_write8", (double)kTable, [&] { hipLaunchKernelGGL(k_write8, grid, block, 0, 0, (uint2 *)tab, kTable / 8); });
  CHECK(hipDeviceSynchronize());
  (void)rows;
  CHECK(hipFree(tab));
  CHECK(hipFree(sink));
  return 0;
}
