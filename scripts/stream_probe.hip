// Streaming-bandwidth probe for the BatchNorm elementwise pattern (2 bf16 inputs -> 1 bf16 output,
// 16-B chunks), at ResNet-50 batch-512 tensor sizes.  Variants: grid-stride vs one-pass grids,
// chunks in flight per thread (U), non-temporal loads / stores.  Buffers are rotated over 4 sets
// (> 256 MiB Infinity Cache) so every pass streams from HBM.
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/stream_probe scripts/stream_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k3(const u32x4* __restrict__ a, const u32x4* __restrict__ b, u32x4* __restrict__ y,
                                          int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x; i0 < n; i0 += stride * U) {
    u32x4 ra[U], rb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = min(i0 + u * stride, n - 1);
      ra[u] = NTL ? __builtin_nontemporal_load(a + i) : a[i];
      rb[u] = NTL ? __builtin_nontemporal_load(b + i) : b[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      if (i >= n) break;
      u32x4 r = ra[u] ^ rb[u];
      if (NTS) __builtin_nontemporal_store(r, y + i);
      else y[i] = r;
    }
  }
}

// contiguous per-block ranges: block b streams [b*per, (b+1)*per) with U chunks in flight per thread
template <int U, bool NTL>
__global__ __launch_bounds__(256) void k3c(const u32x4* __restrict__ a, const u32x4* __restrict__ b, u32x4* __restrict__ y,
                                           int64_t n, int64_t per) {
  const int64_t beg = (int64_t)blockIdx.x * per, end = min(n, beg + per);
  for (int64_t i0 = beg + threadIdx.x; i0 < end; i0 += 256 * U) {
    u32x4 ra[U], rb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = min(i0 + u * 256, end - 1);
      ra[u] = NTL ? __builtin_nontemporal_load(a + i) : a[i];
      rb[u] = NTL ? __builtin_nontemporal_load(b + i) : b[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * 256;
      if (i >= end) break;
      y[i] = ra[u] ^ rb[u];
    }
  }
}

// write-heavy probe: read 1 chunk, write W chunks (the pointwise-conv 1:4 pattern)
template <int W, bool NTS>
__global__ __launch_bounds__(256) void kw(const u32x4* __restrict__ a, u32x4* __restrict__ y, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const u32x4 v = a[i];
#pragma unroll
  for (int k = 0; k < W; ++k) {
    const u32x4 r = v + (uint32_t)k;
    if (NTS) __builtin_nontemporal_store(r, y + (int64_t)k * n + i);
    else y[(int64_t)k * n + i] = r;
  }
}
// write-heavy with row-contiguous output: thread i writes W consecutive chunks (one 16*W-byte row)
template <int W>
__global__ __launch_bounds__(256) void kwr(const u32x4* __restrict__ a, u32x4* __restrict__ y, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n * W) return;
  const u32x4 v = a[i / W];
  y[i] = v + (uint32_t)(i % W);
}

int main() {
  const int64_t sizes[] = {(int64_t)512 * 56 * 56 * 64 * 2, (int64_t)512 * 56 * 56 * 256 * 2, (int64_t)512 * 28 * 28 * 128 * 2,
                           (int64_t)512 * 14 * 14 * 1024 * 2};
  const int64_t maxb = sizes[1];
  const int SETS = 4;
  std::vector<u32x4*> bufs(3 * SETS);
  for (auto& p : bufs) {
    if (hipMalloc(&p, maxb) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(p, 1, maxb);
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  {
    const int64_t rb = (int64_t)512 * 56 * 56 * 64 * 2, n = rb / 16;  // 205 MB read, 822 MB written
    for (int rep = 0; rep < 2; ++rep) {
      auto runw = [&](const char* name, auto launch) {
        for (int s = 0; s < SETS; ++s) launch(bufs[3 * s], bufs[3 * s + 2]);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        for (int r = 0; r < 8; ++r)
          for (int s = 0; s < SETS; ++s) launch(bufs[3 * s], bufs[3 * s + 2]);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double us = ms * 1e3 / (8 * SETS);
        printf("1R:4W 205+822 MB  %-28s %8.1f us  %5.2f TB/s\n", name, us, 5.0 * rb / us / 1e6);
      };
      runw("planes W=4", [&](u32x4* a, u32x4* y) { hipLaunchKernelGGL((kw<4, false>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, a, y, n); });
      runw("planes W=4 nts", [&](u32x4* a, u32x4* y) { hipLaunchKernelGGL((kw<4, true>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, a, y, n); });
      runw("rows W=4", [&](u32x4* a, u32x4* y) { hipLaunchKernelGGL((kwr<4>), dim3((unsigned)((4 * n + 255) / 256)), dim3(256), 0, 0, a, y, n); });
      runw("copy-only write 822MB", [&](u32x4* a, u32x4* y) { hipMemsetAsync(y, 0, 4 * rb, 0); });
    }
  }
  for (int64_t bytes : sizes) {
    const int64_t n = bytes / 16;
    auto run = [&](const char* name, auto launch) {
      for (int s = 0; s < SETS; ++s) launch(bufs[3 * s], bufs[3 * s + 1], bufs[3 * s + 2]);
      hipDeviceSynchronize();
      const int reps = 8;
      hipEventRecord(e0);
      for (int r = 0; r < reps; ++r)
        for (int s = 0; s < SETS; ++s) launch(bufs[3 * s], bufs[3 * s + 1], bufs[3 * s + 2]);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 1e3 / (reps * SETS);
      printf("%10.1f MB  %-28s %8.1f us  %5.2f TB/s\n", bytes / 1e6, name, us, 3.0 * bytes / us / 1e6);
    };
#define GS(G, U, NTL, NTS)                                                                                      \
  run("gs g=" #G " U=" #U " ntl=" #NTL " nts=" #NTS, [&](u32x4* a, u32x4* b, u32x4* y) {                       \
    int64_t g = (G) > 0 ? (G) : (n + 256 * (U)-1) / (256 * (U));                                               \
    hipLaunchKernelGGL((k3<U, NTL, NTS>), dim3((unsigned)g), dim3(256), 0, 0, a, b, y, n);                    \
  });
    GS(4096, 4, true, false)
    GS(4096, 4, false, false)
    GS(4096, 4, false, true)
    GS(2048, 4, false, false)
    GS(1024, 8, false, false)
    GS(2048, 8, false, false)
    GS(8192, 2, false, false)
    GS(0, 4, false, false)
    GS(0, 1, false, false)
    GS(0, 2, false, false)
    GS(0, 8, false, false)
#define CB(G, U, NTL)                                                                                \
  run("contig g=" #G " U=" #U " ntl=" #NTL, [&](u32x4* a, u32x4* b, u32x4* y) {                     \
    const int64_t per = ((n + (G)-1) / (G) + 255) / 256 * 256;                                         \
    hipLaunchKernelGGL((k3c<U, NTL>), dim3((unsigned)(G)), dim3(256), 0, 0, a, b, y, n, per);         \
  });
    CB(1024, 4, false)
    CB(2048, 4, false)
    CB(1024, 8, false)
    CB(2048, 4, true)
  }
  return 0;
}
