// Vectorised elementwise kernels (16 B per lane, grid-stride, capped grid):
// casts, ReLU/GELU fwd+bwd, Philox dropout (mask regenerated in backward
// from (seed, offset) -- no mask tensor), residual add, bias-grad column
// sums, NCHW->NHWC input packing, embedding gather / scatter-add.
#include "common.h"
#include <algorithm>

namespace dpe {

constexpr int ET = 256;

DPE_HOST_DEVICE int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

static inline int egrid(int64_t work) {
  int64_t g = (work + ET - 1) / ET;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

#define GRID_STRIDE(i, n) for (int64_t i = blockIdx.x * (int64_t)ET + threadIdx.x; i < (n); i += (int64_t)gridDim.x * ET)

// ------------------------------------------------------------------ casts
__global__ __launch_bounds__(ET) void f32_to_bf16_kernel(const float* __restrict__ x, uint16_t* __restrict__ y, int64_t n) {
  const int64_t n8 = n / 8;
  GRID_STRIDE(i, n8) {
    const f32x4 a = *(const f32x4*)(x + i * 8), b = *(const f32x4*)(x + i * 8 + 4);
    u32x4 r;
    r[0] = pack_bf2(a[0], a[1]); r[1] = pack_bf2(a[2], a[3]);
    r[2] = pack_bf2(b[0], b[1]); r[3] = pack_bf2(b[2], b[3]);
    *(u32x4*)(y + i * 8) = r;
  }
  if (blockIdx.x == 0)
    for (int64_t i = n8 * 8 + threadIdx.x; i < n; i += ET) y[i] = f2bf(x[i]);
}

__global__ __launch_bounds__(ET) void bf16_to_f32_kernel(const uint16_t* __restrict__ x, float* __restrict__ y, int64_t n) {
  const int64_t n8 = n / 8;
  GRID_STRIDE(i, n8) {
    float f[8];
    unpack8(*(const u32x4*)(x + i * 8), f);
    *(f32x4*)(y + i * 8) = f32x4{f[0], f[1], f[2], f[3]};
    *(f32x4*)(y + i * 8 + 4) = f32x4{f[4], f[5], f[6], f[7]};
  }
  if (blockIdx.x == 0)
    for (int64_t i = n8 * 8 + threadIdx.x; i < n; i += ET) y[i] = bf2f(x[i]);
}

// ----------------------------------------------------------- activations
template <typename T> DPE_DEVICE float lf(const T* p, int64_t i);
template <> DPE_DEVICE float lf<float>(const float* p, int64_t i) { return p[i]; }
template <> DPE_DEVICE float lf<uint16_t>(const uint16_t* p, int64_t i) { return bf2f(p[i]); }
template <typename T> DPE_DEVICE void sf(T* p, int64_t i, float v);
template <> DPE_DEVICE void sf<float>(float* p, int64_t i, float v) { p[i] = v; }
template <> DPE_DEVICE void sf<uint16_t>(uint16_t* p, int64_t i, float v) { p[i] = f2bf(v); }

DPE_DEVICE float gelu_f(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
}
DPE_DEVICE float gelu_grad(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float u = k0 * (x + k1 * x * x * x);
  const float t = tanhf(u);
  return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k0 * (1.f + 3.f * k1 * x * x);
}

// op: 0 relu fwd (y=f(x)), 1 relu bwd (dx = dy * (y>0)), 2 gelu fwd, 3 gelu bwd (dx = dy*gelu'(x))
template <typename T>
__global__ __launch_bounds__(ET) void act_kernel(const T* __restrict__ a, const T* __restrict__ b, T* __restrict__ out,
                                                 int64_t n, int op) {
  GRID_STRIDE(i, n) {
    const float x = lf<T>(a, i);
    float r;
    if (op == 0) r = fmaxf(x, 0.f);
    else if (op == 1) r = lf<T>(b, i) > 0.f ? x : 0.f;
    else if (op == 2) r = gelu_f(x);
    else r = x * gelu_grad(lf<T>(b, i));
    sf<T>(out, i, r);
  }
}

// bf16 fast path for the same ops, 8 per lane
__global__ __launch_bounds__(ET) void act_bf16x8_kernel(const uint16_t* __restrict__ a, const uint16_t* __restrict__ b,
                                                        uint16_t* __restrict__ out, int64_t n8, int op) {
  GRID_STRIDE(i, n8) {
    float x[8], y[8];
    unpack8(*(const u32x4*)(a + i * 8), x);
    if (op == 1 || op == 3) unpack8(*(const u32x4*)(b + i * 8), y);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (op == 0) x[e] = fmaxf(x[e], 0.f);
      else if (op == 1) x[e] = y[e] > 0.f ? x[e] : 0.f;
      else if (op == 2) x[e] = gelu_f(x[e]);
      else x[e] = x[e] * gelu_grad(y[e]);
    }
    *(u32x4*)(out + i * 8) = pack8(x);
  }
}

// ---------------------------------------------------------------- dropout
// keep iff u >= p where u = philox(seed, offset + i/4)[i%4] / 2^32 ; scale 1/(1-p)
template <typename T>
__global__ __launch_bounds__(ET) void dropout_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n, float p,
                                                     uint64_t seed, uint64_t offset) {
  const uint32_t thr = (uint32_t)fminf(p * 4294967296.f, 4294967295.f);
  const float scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  const int64_t n4 = (n + 3) / 4;
  GRID_STRIDE(i, n4) {
    const u32x4 r = philox4x32(seed, offset + (uint64_t)i, 0u);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t j = i * 4 + e;
      if (j < n) sf<T>(y, j, (r[e] >= thr) ? lf<T>(x, j) * scale : 0.f);
    }
  }
}

// --------------------------------------------------------------- residual
template <typename T>
__global__ __launch_bounds__(ET) void add_kernel(const T* __restrict__ a, const T* __restrict__ b, T* __restrict__ out,
                                                 int64_t n, float alpha) {
  GRID_STRIDE(i, n) sf<T>(out, i, lf<T>(a, i) + alpha * lf<T>(b, i));
}

// ------------------------------------------------------ bias-grad col-sum
// db[n] (+)= sum_m dy[m][n]; block = 256 threads over 64 columns x 4 row phases
template <typename T>
__global__ __launch_bounds__(ET) void colsum_kernel(const T* __restrict__ dy, int64_t M, int N, int64_t ld, float* __restrict__ db,
                                                    int accumulate) {
  __shared__ float red[4][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int ph = threadIdx.x >> 6;
  float s = 0.f;
  if (col < N)
    for (int64_t m = ph + 4 * (int64_t)blockIdx.y; m < M; m += 4 * (int64_t)gridDim.y) s += lf<T>(dy, m * ld + col);
  red[ph][threadIdx.x & 63] = s;
  __syncthreads();
  if (ph == 0 && col < N) {
    const float t = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    if (gridDim.y == 1 && !accumulate) db[col] = t;
    else atomicAdd(db + col, t);
  }
}

// Vectorised form (N % 8 == 0, ld % 8 == 0): a wave covers 512 columns with
// 16-B loads, 4 waves x gridDim.y blocks split the rows; LDS reduce over the
// waves, then one atomic per column per block.
template <typename T>
__global__ __launch_bounds__(256) void colsum_vec_kernel(const T* __restrict__ dy, int64_t M, int N, int64_t ld,
                                                         float* __restrict__ db, int accumulate) {
  __shared__ float red[4][512];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c8 = blockIdx.x * 512 + lane * 8;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c8 < N) {
    int64_t m = wid + 4 * (int64_t)blockIdx.y;
    const int64_t step = 4 * (int64_t)gridDim.y;
#pragma unroll 4
    for (; m < M; m += step) {
      float f[8];
      if constexpr (sizeof(T) == 2) {
        unpack8(*(const u32x4*)((const uint16_t*)dy + m * ld + c8), f);
      } else {
        const f32x4 a = *(const f32x4*)((const float*)dy + m * ld + c8), b = *(const f32x4*)((const float*)dy + m * ld + c8 + 4);
        f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3]; f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += f[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[wid][lane * 8 + e] = s[e];
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 256) {
    const int col = blockIdx.x * 512 + i;
    if (col < N) {
      const float t = red[0][i] + red[1][i] + red[2][i] + red[3][i];
      if (gridDim.y == 1 && !accumulate) db[col] = t;
      else atomicAdd(db + col, t);
    }
  }
}

// ------------------------------------------------------ input packing
// x NCHW f32 -> y NHWC bf16 with channels padded to Cp (zeros)
__global__ __launch_bounds__(ET) void nchw_to_nhwc_kernel(const float* __restrict__ x, uint16_t* __restrict__ y, int N, int C,
                                                          int HW, int Cp) {
  const int64_t total = (int64_t)N * HW;
  GRID_STRIDE(i, total) {
    const int64_t n = i / HW, hw = i % HW;
    for (int c = 0; c < Cp; ++c) y[i * Cp + c] = c < C ? f2bf(x[(n * C + c) * HW + hw]) : (uint16_t)0;
  }
}

// x NCHW f32 [N,C<=4,H,W] -> space-to-depth NHWC bf16 [N,H/2,W/2,16],
// channel (ay*2+ax)*4+c = x[n][c][2q+ay][2p+ax] (zeros for c >= C).  The 7x7/s2
// stem then runs as a 4x4/s1 conv over 16 channels (K 256 instead of 392, two
// 16-B chunks per tap).
__global__ __launch_bounds__(ET) void nchw_to_s2d_kernel(const float* __restrict__ x, uint16_t* __restrict__ y, int N, int C,
                                                         int H, int W) {
  const int Ho = H / 2, Wo = W / 2;
  const int64_t total = (int64_t)N * Ho * Wo;
  GRID_STRIDE(i, total) {
    const int p = (int)(i % Wo);
    const int64_t t = i / Wo;
    const int q = (int)(t % Ho);
    const int n = (int)(t / Ho);
    // the two horizontal neighbours (ax = 0, 1) of a channel row in one 8-B load (W even)
    float v[16];
#pragma unroll
    for (int ay = 0; ay < 2; ++ay)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float2 t2 = c < C ? *(const float2*)(x + (((int64_t)n * C + c) * H + 2 * q + ay) * W + 2 * p) : float2{0.f, 0.f};
        v[ay * 8 + c] = t2.x;      // j = c + 4 ax + 8 ay
        v[ay * 8 + 4 + c] = t2.y;
      }
    u32x4* o = (u32x4*)(y + i * 16);
    o[0] = pack8(v);
    o[1] = pack8(v + 8);
  }
}

// ------------------------------------------- data-grad filter layout
// wt[c][r][s][k] = w[k][r0 + rs*(Rp-1-r)][s0 + ss*(Sp-1-s)][c], r < Rp, s < Sp.
// With (r0, rs, Rp) = (0, 1, R): the flipped/transposed filter -- the stride-1
// data grad of a conv is a forward conv of dy with it (pad R-1-p), so it runs on
// the forward loaders (K-contiguous filter rows) instead of the transposed ones.
// With a stride > 1, one such filter per output parity holds only the taps that
// reach that parity (phase-decomposed data grad).
// One (r, s) tap per blockIdx.z: a 32x32 tile of the [K][C] slice transposed through LDS (reads of
// w along C and writes of wt along K both 64-B runs; the element-per-thread gather read w with a
// stride of R*S*C elements: 15 us for the 512-channel 3x3 filters).
__global__ __launch_bounds__(256) void conv_w_flipT_kernel(const uint16_t* __restrict__ w, uint16_t* __restrict__ wt, int K,
                                                          int R, int S, int C, int r0, int rs, int Rp, int s0, int ss,
                                                          int Sp) {
  __shared__ uint16_t tile[32][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int c0 = blockIdx.x * 32, k0 = blockIdx.y * 32;
  const int r = (int)blockIdx.z / Sp, s = (int)blockIdx.z % Sp;
  const int rr = r0 + rs * (Rp - 1 - r), sc = s0 + ss * (Sp - 1 - s);
#pragma unroll
  for (int q = 0; q < 32; q += 8) {
    const int k = k0 + q + ty, c = c0 + tx;
    if (k < K && c < C) tile[q + ty][tx] = w[(((int64_t)k * R + rr) * S + sc) * C + c];
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 32; q += 8) {
    const int c = c0 + q + ty, k = k0 + tx;
    if (k < K && c < C) wt[(((int64_t)c * Rp + r) * Sp + s) * K + k] = tile[tx][q + ty];
  }
}

// Several flips in ONE launch (the data grads of a backward pass refresh all their flipped filters at
// once, ops.cpp flipped()): block b belongs to entry e with start[e] <= b < start[e + 1], and runs
// conv_w_flipT_kernel's block (b - start[e]) of that entry.
struct FlipDesc {
  const uint16_t* w;
  uint16_t* wt;
  int K, R, S, C, r0, rs, Rp, s0, ss, Sp;
};
__global__ __launch_bounds__(256) void conv_w_flipT_multi_kernel(const FlipDesc* __restrict__ fd, const int* __restrict__ start,
                                                                int n) {
  __shared__ uint16_t tile[32][33];
  int e = 0;
  while (e + 1 < n && (int)blockIdx.x >= start[e + 1]) ++e;
  const FlipDesc d = fd[e];
  const int lb = (int)blockIdx.x - start[e];
  const int gx = (d.C + 31) / 32, gy = (d.K + 31) / 32;
  const int bx = lb % gx, by = (lb / gx) % gy, bz = lb / (gx * gy);
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int c0 = bx * 32, k0 = by * 32;
  const int r = bz / d.Sp, s = bz % d.Sp;
  const int rr = d.r0 + d.rs * (d.Rp - 1 - r), sc = d.s0 + d.ss * (d.Sp - 1 - s);
#pragma unroll
  for (int q = 0; q < 32; q += 8) {
    const int k = k0 + q + ty, c = c0 + tx;
    if (k < d.K && c < d.C) tile[q + ty][tx] = d.w[(((int64_t)k * d.R + rr) * d.S + sc) * d.C + c];
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 32; q += 8) {
    const int c = c0 + q + ty, k = k0 + tx;
    if (k < d.K && c < d.C) d.wt[(((int64_t)c * d.Rp + r) * d.Sp + s) * d.K + k] = tile[tx][q + ty];
  }
}

// ----------------------------------------------------------- embedding
// out[r][:] = wte[idx[r]][:] (+ wpe[r % T][:]) ; D % 8 == 0, weights bf16, out f32
__global__ __launch_bounds__(ET) void embedding_fwd_kernel(const int64_t* __restrict__ idx, const uint16_t* __restrict__ wte,
                                                           const uint16_t* __restrict__ wpe, float* __restrict__ out,
                                                           int64_t rows, int T, int D) {
  const int CPR = D / 8;
  GRID_STRIDE(i, rows * CPR) {
    const int64_t r = i / CPR;
    const int c8 = (int)(i % CPR) * 8;
    float a[8];
    unpack8(*(const u32x4*)(wte + idx[r] * D + c8), a);
    if (wpe) {
      float b[8];
      unpack8(*(const u32x4*)(wpe + (r % T) * D + c8), b);
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] += b[e];
    }
    *(f32x4*)(out + r * D + c8) = f32x4{a[0], a[1], a[2], a[3]};
    *(f32x4*)(out + r * D + c8 + 4) = f32x4{a[4], a[5], a[6], a[7]};
  }
}

// dwte[idx[r]] += dout[r]; dwpe[r % T] += dout[r]   (fp32 atomics, 256-B wave segments)
__global__ __launch_bounds__(ET) void embedding_bwd_kernel(const int64_t* __restrict__ idx, const float* __restrict__ dout,
                                                           float* __restrict__ dwte, float* __restrict__ dwpe, int64_t rows,
                                                           int T, int D) {
  GRID_STRIDE(i, rows * D) {
    const int64_t r = i / D;
    const int d = (int)(i % D);
    const float g = dout[i];
    atomicAdd(dwte + idx[r] * D + d, g);
    if (dwpe) atomicAdd(dwpe + (r % T) * D + d, g);
  }
}

}  // namespace dpe

using namespace dpe;

extern "C" int dpe_cast_f32_bf16(const float* x, uint16_t* y, int64_t n, hipStream_t st) {
  hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(egrid(n / 8 + 1)), dim3(ET), 0, st, x, y, n);
  return 0;
}
extern "C" int dpe_cast_bf16_f32(const uint16_t* x, float* y, int64_t n, hipStream_t st) {
  hipLaunchKernelGGL(bf16_to_f32_kernel, dim3(egrid(n / 8 + 1)), dim3(ET), 0, st, x, y, n);
  return 0;
}
extern "C" int dpe_act(const void* a, const void* b, void* out, int64_t n, int op, int bf16, hipStream_t st) {
  if (bf16 && n % 8 == 0 && ((uintptr_t)a % 16 == 0) && ((uintptr_t)out % 16 == 0) && (!b || (uintptr_t)b % 16 == 0)) {
    hipLaunchKernelGGL(act_bf16x8_kernel, dim3(egrid(n / 8)), dim3(ET), 0, st, (const uint16_t*)a, (const uint16_t*)b,
                       (uint16_t*)out, n / 8, op);
  } else if (bf16) {
    hipLaunchKernelGGL((act_kernel<uint16_t>), dim3(egrid(n)), dim3(ET), 0, st, (const uint16_t*)a, (const uint16_t*)b,
                       (uint16_t*)out, n, op);
  } else {
    hipLaunchKernelGGL((act_kernel<float>), dim3(egrid(n)), dim3(ET), 0, st, (const float*)a, (const float*)b, (float*)out, n,
                       op);
  }
  return 0;
}
extern "C" int dpe_dropout(const void* x, void* y, int64_t n, float p, uint64_t seed, uint64_t offset, int bf16,
                           hipStream_t st) {
  if (bf16)
    hipLaunchKernelGGL((dropout_kernel<uint16_t>), dim3(egrid((n + 3) / 4)), dim3(ET), 0, st, (const uint16_t*)x, (uint16_t*)y,
                       n, p, seed, offset);
  else
    hipLaunchKernelGGL((dropout_kernel<float>), dim3(egrid((n + 3) / 4)), dim3(ET), 0, st, (const float*)x, (float*)y, n, p,
                       seed, offset);
  return 0;
}
extern "C" int dpe_add(const void* a, const void* b, void* out, int64_t n, float alpha, int bf16, hipStream_t st) {
  if (bf16)
    hipLaunchKernelGGL((add_kernel<uint16_t>), dim3(egrid(n)), dim3(ET), 0, st, (const uint16_t*)a, (const uint16_t*)b,
                       (uint16_t*)out, n, alpha);
  else
    hipLaunchKernelGGL((add_kernel<float>), dim3(egrid(n)), dim3(ET), 0, st, (const float*)a, (const float*)b, (float*)out, n,
                       alpha);
  return 0;
}
extern "C" int dpe_colsum(const void* dy, int64_t M, int N, int64_t ld, float* db, int accumulate, int bf16, hipStream_t st) {
  if (N % 8 == 0 && ld % 8 == 0) {
    const int gx = (N + 511) / 512;
    int64_t gy = std::max<int64_t>(1, std::min<int64_t>((M + 63) / 64, 1024 / gx));
    if (!accumulate && gy > 1) hipMemsetAsync(db, 0, (size_t)N * sizeof(float), st);
    const dim3 grid(gx, (unsigned)gy);
    if (bf16)
      hipLaunchKernelGGL((colsum_vec_kernel<uint16_t>), grid, dim3(256), 0, st, (const uint16_t*)dy, M, N, ld, db, accumulate);
    else
      hipLaunchKernelGGL((colsum_vec_kernel<float>), grid, dim3(256), 0, st, (const float*)dy, M, N, ld, db, accumulate);
    return 0;
  }
  int gy = (int)((M + 255) / 256);
  if (gy > 64) gy = 64;
  if (gy < 1) gy = 1;
  dim3 grid((N + 63) / 64, gy);
  if (bf16)
    hipLaunchKernelGGL((colsum_kernel<uint16_t>), grid, dim3(ET), 0, st, (const uint16_t*)dy, M, N, ld, db, accumulate);
  else
    hipLaunchKernelGGL((colsum_kernel<float>), grid, dim3(ET), 0, st, (const float*)dy, M, N, ld, db, accumulate);
  return 0;
}
extern "C" int dpe_nchw_to_s2d(const float* x, uint16_t* y, int N, int C, int H, int W, hipStream_t st) {
  if (C > 4 || (H & 1) || (W & 1)) return -1;
  hipLaunchKernelGGL(nchw_to_s2d_kernel, dim3(egrid((int64_t)N * (H / 2) * (W / 2))), dim3(ET), 0, st, x, y, N, C, H, W);
  return (int)hipGetLastError();
}

extern "C" int dpe_conv_w_flipT(const uint16_t* w, uint16_t* wt, int K, int R, int S, int C, int r0, int rs, int Rp,
                                int s0, int ss, int Sp, hipStream_t st) {
  if (Rp <= 0 || Sp <= 0 || r0 + rs * (Rp - 1) >= R || s0 + ss * (Sp - 1) >= S) return -1;
  hipLaunchKernelGGL(conv_w_flipT_kernel, dim3((C + 31) / 32, (K + 31) / 32, Rp * Sp), dim3(256), 0, st, w, wt, K, R, S, C, r0,
                     rs, Rp, s0, ss, Sp);
  return (int)hipGetLastError();
}

extern "C" int dpe_flip_desc_bytes() { return (int)sizeof(FlipDesc); }
extern "C" int dpe_flip_blocks(int K, int C, int Rp, int Sp) { return ((C + 31) / 32) * ((K + 31) / 32) * Rp * Sp; }
// desc: n FlipDesc on the device; start: n + 1 block offsets on the device (start[n] = total blocks)
extern "C" int dpe_conv_w_flipT_multi(const void* desc, const int* start, int n, int total_blocks, hipStream_t st) {
  if (n <= 0 || total_blocks <= 0) return 0;
  hipLaunchKernelGGL(conv_w_flipT_multi_kernel, dim3(total_blocks), dim3(256), 0, st, (const FlipDesc*)desc, start, n);
  return (int)hipGetLastError();
}

extern "C" int dpe_nchw_to_nhwc(const float* x, uint16_t* y, int N, int C, int HW, int Cp, hipStream_t st) {
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3(egrid((int64_t)N * HW)), dim3(ET), 0, st, x, y, N, C, HW, Cp);
  return 0;
}
extern "C" int dpe_embedding_fwd(const int64_t* idx, const uint16_t* wte, const uint16_t* wpe, float* out, int64_t rows, int T,
                                 int D, hipStream_t st) {
  if (D % 8) return -1;
  hipLaunchKernelGGL(embedding_fwd_kernel, dim3(egrid(rows * D / 8)), dim3(ET), 0, st, idx, wte, wpe, out, rows, T, D);
  return 0;
}
extern "C" int dpe_embedding_bwd(const int64_t* idx, const float* dout, float* dwte, float* dwpe, int64_t rows, int T, int D,
                                 hipStream_t st) {
  hipLaunchKernelGGL(embedding_bwd_kernel, dim3(egrid(rows * D)), dim3(ET), 0, st, idx, dout, dwte, dwpe, rows, T, D);
  return 0;
}

// CU-occupancy probe: nblocks workgroups that each hold their CU slot (waves, LDS, ~V VGPRs per lane)
// until `stop` becomes non-zero or `ticks` of the 100 MHz wall clock pass -- a stand-in for RCCL's
// channel workgroups sharing the CUs with backward kernels (scripts/hog_probe.py).  Every wave leaves
// at the deadline, so a stop flag that is never set cannot hang the device.
// mode 0: VALU-saturating (worst case); 1: resident but idle; 2: RCCL-like reduce-copy -- each block
// streams its own window of `buf` (dst = src0 + src1 over HOG_WIN floats, the shape of an all-reduce
// channel's inner loop), memory-bound with little VALU.
constexpr int64_t HOG_WIN = 1 << 20;  // floats per block and operand (4 MiB)
template <int V>
__global__ __launch_bounds__(256) void cu_hog_kernel(int64_t ticks, const unsigned* stop, float* sink, int sleepy,
                                                     float* buf) {
  extern __shared__ float lds[];
  const int64_t t0 = wall_clock64();
  float r[V];
#pragma unroll
  for (int i = 0; i < V; ++i) r[i] = (float)(threadIdx.x + i);
  int64_t pos = 0;
  float* const w0 = buf ? buf + (int64_t)blockIdx.x * 3 * HOG_WIN : nullptr;
  while (wall_clock64() - t0 < ticks) {
    if (sleepy == 2 && w0) {
      // 64 KiB per operand per trip: two reads and one write of f32x4 per thread x 16
#pragma unroll 4
      for (int k = 0; k < 16; ++k) {
        const int64_t i = (pos + (int64_t)k * blockDim.x + threadIdx.x) * 4;
        const f32x4 a = *(const f32x4*)(w0 + i), b = *(const f32x4*)(w0 + HOG_WIN + i);
        *(f32x4*)(w0 + 2 * HOG_WIN + i) = a + b;
      }
      pos += 16 * blockDim.x;
      if ((pos + 16 * blockDim.x) * 4 > HOG_WIN) pos = 0;
    } else if (sleepy) {  // resident but idle: slot occupancy only (an RCCL block waiting on its peers)
      __builtin_amdgcn_s_sleep(127);
    } else {       // VALU-saturating: slot occupancy plus issue-cycle contention (worst case)
#pragma unroll 1
      for (int k = 0; k < 16; ++k)
#pragma unroll
        for (int i = 0; i < V; ++i) r[i] = r[i] * 0.999f + 1.f;
    }
    if (stop && __hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) break;
  }
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) acc += r[i];
  if (acc == -1.f) sink[threadIdx.x] = lds[threadIdx.x];  // never true: keeps r / lds live
}
// stop flag for cu_hog: one vector (agent-scope atomic) store, ordered on the caller's stream
__global__ void hog_stop_kernel(unsigned* stop, unsigned v) {
  __hip_atomic_store(stop, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// buf (mode 2): >= nblocks * 3 * HOG_WIN floats
extern "C" int64_t dpe_cu_hog_buf_floats(int nblocks) { return (int64_t)nblocks * 3 * HOG_WIN; }
extern "C" int dpe_cu_hog(int nblocks, int threads, int lds_bytes, double us, int vgprs, const unsigned* stop, float* sink,
                          int sleepy, float* buf, hipStream_t st) {
  if (nblocks <= 0 || threads <= 0 || threads > 256 || us <= 0 || us > 1e6) return -1;  // RCCL-sized: 256 threads
  if (sleepy == 2 && (!buf || threads % 64)) return -1;
  const int64_t t = (int64_t)(us * 100.0);
  if (vgprs <= 16) hipLaunchKernelGGL(cu_hog_kernel<8>, dim3(nblocks), dim3(threads), lds_bytes, st, t, stop, sink, sleepy, buf);
  else if (vgprs <= 64) hipLaunchKernelGGL(cu_hog_kernel<56>, dim3(nblocks), dim3(threads), lds_bytes, st, t, stop, sink, sleepy, buf);
  else if (vgprs <= 128) hipLaunchKernelGGL(cu_hog_kernel<120>, dim3(nblocks), dim3(threads), lds_bytes, st, t, stop, sink, sleepy, buf);
  else hipLaunchKernelGGL(cu_hog_kernel<136>, dim3(nblocks), dim3(threads), lds_bytes, st, t, stop, sink, sleepy, buf);  // RCCL: 140
  return (int)hipGetLastError();
}
extern "C" int dpe_hog_stop(unsigned* stop, unsigned v, hipStream_t st) {
  hipLaunchKernelGGL(hog_stop_kernel, dim3(1), dim3(1), 0, st, stop, v);
  return (int)hipGetLastError();
}
