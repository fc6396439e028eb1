// NHWC pooling: max-pool (with per-element argmax byte for an index-free
// backward gather) and global average pool.  bf16 in/out, 8 channels/lane.
#include <algorithm>

#include "common.h"

namespace dpe {

// coef != nullptr: the input is the PRE-BatchNorm stem output h and each tap is
// relu(h*scale + shift) rounded to bf16 exactly as a materialised BN output
// would be -- the BN+ReLU tensor is never written (stem fusion).
template <bool BNRELU, int KK>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                          uint8_t* __restrict__ idx, int N, int H, int W, int C, int OH,
                                                          int OW, int k_rt, int s, int p, const float* __restrict__ coef) {
  // one 8-channel output chunk per thread over an exact grid, 32-bit index math (the host
  // checks N*OH*OW*C/8 < 2^31).  KK > 0: the window size is a compile-time constant and all
  // KK*KK tap loads are issued before the first use (one load in flight per thread left the
  // stem pool latency-bound).
  const int k = KK > 0 ? KK : k_rt;
  const int CPR = C >> 3;
  const int total = N * OH * OW * CPR;
  // XCD-contiguous block order: an XCD's concurrent blocks cover neighbouring output rows, whose 3x3 / s2
  // windows share input rows in that XCD's L2 (round-robin dispatch spread them over all 8 L2s)
  const int i = xcd_remap(blockIdx.x, gridDim.x) * 256 + threadIdx.x;
  if (i >= total) return;
  const int c8 = (i % CPR) * 8;
  int t = i / CPR;
  const int ow = t % OW; t /= OW;
  const int oh = t % OH;
  const int n = t / OH;
  float sc[8], sh[8];
  if constexpr (BNRELU) {
#pragma unroll
    for (int e = 0; e < 8; ++e) { sc[e] = coef[c8 + e]; sh[e] = coef[C + c8 + e]; }
  }
  float best[8];
  uint8_t bi[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; bi[e] = 0; }
  auto take = [&](const u32x4& raw, int tap) {
    float f[8];
    unpack8(raw, f);
    if constexpr (BNRELU) {
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = bf2f(f2bf(fmaxf(fmaf(f[e], sc[e], sh[e]), 0.f)));
    }
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (f[e] > best[e]) { best[e] = f[e]; bi[e] = (uint8_t)tap; }
  };
  const uint16_t* xn = x + (int64_t)n * H * W * C + c8;
  if constexpr (KK > 0) {
    u32x4 raw[KK * KK];
    bool ok[KK * KK];
#pragma unroll
    for (int r = 0; r < KK; ++r)
#pragma unroll
      for (int q = 0; q < KK; ++q) {
        const int ih = oh * s - p + r, iw = ow * s - p + q;
        ok[r * KK + q] = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
        const int ihc = min(max(ih, 0), H - 1), iwc = min(max(iw, 0), W - 1);
        raw[r * KK + q] = *(const u32x4*)(xn + ((int64_t)ihc * W + iwc) * C);
      }
#pragma unroll
    for (int tp = 0; tp < KK * KK; ++tp)
      if (ok[tp]) take(raw[tp], tp);
  } else {
    for (int r = 0; r < k; ++r) {
      const int ih = oh * s - p + r;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int q = 0; q < k; ++q) {
        const int iw = ow * s - p + q;
        if ((unsigned)iw >= (unsigned)W) continue;
        take(*(const u32x4*)(xn + ((int64_t)ih * W + iw) * C), r * k + q);
      }
    }
  }
  *(u32x4*)(y + (int64_t)i * 8) = pack8(best);
  u32x2 pk;
  pk[0] = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
  pk[1] = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
  *(u32x2*)(idx + (int64_t)i * 8) = pk;
}

// The stem's 3x3 / s2 / p1 max-pool over relu(BN(h)) (C = 8 CPR), VALU-lean: maxpool_fwd_kernel<true, 3>
// spent ~850 VALU instructions per 8-channel output (unpack, fma, max, bf16 round trip, compare, two selects
// per tap and element plus 32-bit index division) -- at 12.8 M outputs that is the whole 276 us it took
// at batch 512 (profiles/resnet50_dispatch_r6.txt: VALU-bound, 4.1 TB/s).  Here each (tap, element) is one
// sortable key: after the bf16 round (RNE, as a materialised BN output) a value's bits shifted to the top
// half compare as a signed int exactly as the float does for every non-negative value, and a negative one
// (ReLU -> 0) compares below 0; the low bits carry 15 - tap, so the running max = max3(best, key, code)
// does the ReLU, the max and the first-tap-wins tie break (the strict '>' scan of the reference kernel) in
// one v_max3_i32.  Same values and argmax bytes as maxpool_fwd_kernel<true, 3> (a -0 maximum is stored as
// +0; a NaN input propagates instead of being clamped to 0 by fmaxf).  Rows: one block covers part of one
// output row (n, oh): the row-tap validity is block-uniform, only the q = 0 / 2 column taps are per lane.
template <int CPR>
__global__ __launch_bounds__(256) void bnrelu_maxpool3_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                              uint8_t* __restrict__ idx, int H, int W, int OH, int OW,
                                                              int nx, const float* __restrict__ coef) {
  constexpr int C = CPR * 8;
  const int rb = xcd_remap(blockIdx.x, gridDim.x);  // XCD-contiguous rows (shared input rows in one L2)
  const int row = rb / nx, xb = rb - row * nx;
  const int n = row / OH, oh = row - n * OH;
  const int j = xb * 256 + (int)threadIdx.x;
  if (j >= OW * CPR) return;
  const int c8 = (j % CPR) * 8, ow = j / CPR;
  float sc[8], sh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { sc[e] = coef[c8 + e]; sh[e] = coef[C + c8 + e]; }
  const uint16_t* xn = x + (int64_t)n * H * W * C + c8;
  const int ih0 = 2 * oh - 1, iw0 = 2 * ow - 1;
  u32x4 raw[9];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int ihc = min(max(ih0 + r, 0), H - 1), iwc = min(max(iw0 + q, 0), W - 1);
      raw[r * 3 + q] = *(const u32x4*)(xn + ((int64_t)ihc * W + iwc) * C);
    }
  int best[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) best[e] = 0;
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    if ((unsigned)(ih0 + r) >= (unsigned)H) continue;  // block-uniform
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      // q = 1 (iw = 2 ow) is always inside the image; q = 0 / 2 per lane
      const bool cok = q == 1 || (unsigned)(iw0 + q) < (unsigned)W;
      const int code = cok ? 15 - (r * 3 + q) : 0;
      const u32x4& v = raw[r * 3 + q];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float lo = fmaf(__uint_as_float(v[k] << 16), sc[2 * k], sh[2 * k]);
        const float hi = fmaf(__uint_as_float(v[k] & 0xffff0000u), sc[2 * k + 1], sh[2 * k + 1]);
        const uint32_t pk = pack_bf2(lo, hi);
        int klo = (int)((pk << 16) | (uint32_t)code), khi = (int)((pk & 0xffff0000u) | (uint32_t)code);
        if (q != 1) {
          klo = cok ? klo : 0;
          khi = cok ? khi : 0;
        }
        best[2 * k] = max(max(best[2 * k], klo), code);
        best[2 * k + 1] = max(max(best[2 * k + 1], khi), code);
      }
    }
  }
  const int64_t o = ((int64_t)row * OW + ow) * C + c8;
  u32x4 out;
  u32x2 ib;
#pragma unroll
  for (int k = 0; k < 4; ++k) out[k] = ((uint32_t)best[2 * k] >> 16) | ((uint32_t)best[2 * k + 1] & 0xffff0000u);
#pragma unroll
  for (int h2 = 0; h2 < 2; ++h2) {
    uint32_t w = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) w |= (((uint32_t)best[4 * h2 + e] & 15u) ^ 15u) << (8 * e);
    ib[h2] = w;
  }
  *(u32x4*)(y + o) = out;
  *(u32x2*)(idx + o) = ib;
}

// d(pool input)[n,h,w,c8..c8+7]: sum of dy over the windows containing (h, w) whose argmax it is
DPE_DEVICE void pool_grad8(const uint16_t* __restrict__ dy, const uint8_t* __restrict__ idx, int n, int h, int w, int c8,
                           int C, int OH, int OW, int k, int s, int p, float* acc) {
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  // oh*s - p <= h <= oh*s - p + k - 1
  const int oh_lo = max(0, (h + p - k + s) / s), oh_hi = min(OH - 1, (h + p) / s);
  const int ow_lo = max(0, (w + p - k + s) / s), ow_hi = min(OW - 1, (w + p) / s);
  for (int oh = oh_lo; oh <= oh_hi; ++oh) {
    const int r = h - (oh * s - p);
    if (r < 0 || r >= k) continue;
    for (int ow = ow_lo; ow <= ow_hi; ++ow) {
      const int q = w - (ow * s - p);
      if (q < 0 || q >= k) continue;
      const int64_t o = (((int64_t)n * OH + oh) * OW + ow) * C + c8;
      const u32x2 pk = *(const u32x2*)(idx + o);
      float g[8];
      unpack8(*(const u32x4*)(dy + o), g);
      const uint8_t want = (uint8_t)(r * k + q);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint8_t b = (uint8_t)((pk[e >> 2] >> ((e & 3) * 8)) & 0xff);
        if (b == want) acc[e] += g[e];
      }
    }
  }
}

// dx[n,h,w,c] = sum over windows (oh,ow) containing (h,w) whose argmax is (h,w)
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const uint16_t* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                          uint16_t* __restrict__ dx, int N, int H, int W, int C, int OH,
                                                          int OW, int k, int s, int p) {
  const int CPR = C >> 3;
  const int64_t total = (int64_t)N * H * W * CPR;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c8 = (int)(i % CPR) * 8;
    int64_t t = i / CPR;
    const int w = (int)(t % W); t /= W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    float acc[8];
    pool_grad8(dy, idx, n, h, w, c8, C, OH, OW, k, s, p, acc);
    *(u32x4*)(dx + i * 8) = pack8(acc);
  }
}

// ---- stem backward: maxpool gather + BN(+ReLU) backward without materialising d(BN output).
// 32-bit index math throughout (the stem tensor has < 2^31 chunks; 64-bit div/mod by a
// runtime divisor is a ~100-instruction software sequence per element).
DPE_DEVICE void pool_grad8_32(const uint16_t* __restrict__ dy, const uint8_t* __restrict__ idx, int n, int h, int w, int c8,
                              int C, int OH, int OW, int k, int s, int p, float* acc) {
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  const int oh_lo = max(0, (h + p - k + s) / s), oh_hi = min(OH - 1, (h + p) / s);
  const int ow_lo = max(0, (w + p - k + s) / s), ow_hi = min(OW - 1, (w + p) / s);
  for (int oh = oh_lo; oh <= oh_hi; ++oh) {
    const int r = h - (oh * s - p);
    for (int ow = ow_lo; ow <= ow_hi; ++ow) {
      const int q = w - (ow * s - p);
      const uint32_t o = ((uint32_t)(n * OH + oh) * OW + ow) * C + c8;
      const u32x2 pk = *(const u32x2*)(idx + o);
      float g[8];
      unpack8(*(const u32x4*)(dy + o), g);
      const uint32_t want = (uint32_t)(r * k + q);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t b = (pk[e >> 2] >> ((e & 3) * 8)) & 0xffu;
        acc[e] += (b == want) ? g[e] : 0.f;
      }
    }
  }
}

// reduce: per-block partials [2][C][nb] of (sum dz, sum dz*(x - mean)), dz = gather * [x*scale+shift > 0]
__global__ __launch_bounds__(256) void maxpool_bn_bwd_reduce_kernel(const uint16_t* __restrict__ dy,
                                                                    const uint8_t* __restrict__ idx,
                                                                    const uint16_t* __restrict__ x,
                                                                    const float* __restrict__ coef, int N, int H, int W,
                                                                    int C, int OH, int OW, int k, int s, int p,
                                                                    int rows_per_block, float* __restrict__ part) {
  const int CPR = C >> 3;
  const int tid = threadIdx.x;
  const int RPI = 256 / CPR;
  const int c = tid % CPR, r = tid / CPR;
  const int M = N * H * W;
  const int rb = blockIdx.x * rows_per_block;
  const int re = min(M, rb + rows_per_block);
  float sm[8], sq[8], mean[8], sc[8], sh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sm[e] = 0.f; sq[e] = 0.f;
    sc[e] = coef[c * 8 + e]; sh[e] = coef[C + c * 8 + e]; mean[e] = coef[2 * C + c * 8 + e];
  }
  if (r < RPI) {
    for (int row = rb + r; row < re; row += RPI) {
      const int w = row % W, t = row / W;
      const int h = t % H, n = t / H;
      float d[8], xv[8];
      unpack8(*(const u32x4*)(x + (size_t)row * C + c * 8), xv);
      pool_grad8_32(dy, idx, n, h, w, c * 8, C, OH, OW, k, s, p, d);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float dz = fmaf(xv[e], sc[e], sh[e]) > 0.f ? d[e] : 0.f;
        sm[e] += dz;
        sq[e] += dz * (xv[e] - mean[e]);
      }
    }
  }
  __shared__ float red[2][256][8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[0][tid][e] = sm[e]; red[1][tid][e] = sq[e]; }
  __syncthreads();
  for (int ch = tid; ch < C; ch += 256) {
    const int cc = ch >> 3, e = ch & 7;
    float a = 0.f, b = 0.f;
    for (int rr = 0; rr < RPI; ++rr) { a += red[0][rr * CPR + cc][e]; b += red[1][rr * CPR + cc][e]; }
    part[(int64_t)ch * gridDim.x + blockIdx.x] = a;
    part[(int64_t)(C + ch) * gridDim.x + blockIdx.x] = b;
  }
}

// apply: dx = a*dz + b*x + c   (bcoef [3][C] from bn_bwd_finalize); one (pixel, 8 channels) per thread
__global__ __launch_bounds__(256) void maxpool_bn_bwd_apply_kernel(const uint16_t* __restrict__ dy,
                                                                   const uint8_t* __restrict__ idx,
                                                                   const uint16_t* __restrict__ x,
                                                                   const float* __restrict__ coef,
                                                                   const float* __restrict__ bcoef,
                                                                   uint16_t* __restrict__ dx, int N, int H, int W, int C,
                                                                   int OH, int OW, int k, int s, int p) {
  const int CPR = C >> 3;
  const int total = N * H * W * CPR;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int c8 = (i % CPR) * 8;
    int t = i / CPR;
    const int w = t % W; t /= W;
    const int h = t % H;
    const int n = t / H;
    float d[8], xv[8], o[8];
    unpack8(*(const u32x4*)(x + (size_t)i * 8), xv);
    pool_grad8_32(dy, idx, n, h, w, c8, C, OH, OW, k, s, p, d);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float dz = fmaf(xv[e], coef[c8 + e], coef[C + c8 + e]) > 0.f ? d[e] : 0.f;
      o[e] = bcoef[c8 + e] * dz + bcoef[C + c8 + e] * xv[e] + bcoef[2 * C + c8 + e];
    }
    *(u32x4*)(dx + (size_t)i * 8) = pack8(o);
  }
}

// ---- quad form for the ResNet stem pool (k = 3, s = 2, p = 1, even H, W; OH = H/2, OW = W/2):
// a thread owns the 2x2 input quad (2i.., 2j..) x 8 channels, which only windows (i|i+1, j|j+1)
// reach -- 4 (dy, argmax) loads serve 4 pixels (instead of 9 for 4 pixels one by one), no loops.
//   pixel (0,0): w00 tap 4 | (0,1): w00 5, w01 3 | (1,0): w00 7, w10 1 | (1,1): w00 8, w01 6, w10 2, w11 0
DPE_DEVICE void pool_grad_quad(const uint16_t* __restrict__ dy, const uint8_t* __restrict__ idx, int n, int i, int j, int c8,
                               int C, int OH, int OW, float (*d)[8]) {
  float g[4][8];
  uint32_t b[4][2];
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const int oi = i + (w >> 1), oj = j + (w & 1);
    const bool v = oi < OH && oj < OW;
    const size_t o = ((size_t)(n * OH + min(oi, OH - 1)) * OW + min(oj, OW - 1)) * C + c8;
    const u32x2 pk = *(const u32x2*)(idx + o);
    unpack8(*(const u32x4*)(dy + o), g[w]);
    b[w][0] = v ? pk[0] : 0xffffffffu;  // 0xff never matches a tap
    b[w][1] = v ? pk[1] : 0xffffffffu;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const uint32_t t0 = (b[0][e >> 2] >> ((e & 3) * 8)) & 0xffu, t1 = (b[1][e >> 2] >> ((e & 3) * 8)) & 0xffu;
    const uint32_t t2 = (b[2][e >> 2] >> ((e & 3) * 8)) & 0xffu, t3 = (b[3][e >> 2] >> ((e & 3) * 8)) & 0xffu;
    d[0][e] = t0 == 4u ? g[0][e] : 0.f;
    d[1][e] = (t0 == 5u ? g[0][e] : 0.f) + (t1 == 3u ? g[1][e] : 0.f);
    d[2][e] = (t0 == 7u ? g[0][e] : 0.f) + (t2 == 1u ? g[2][e] : 0.f);
    d[3][e] = (t0 == 8u ? g[0][e] : 0.f) + (t1 == 6u ? g[1][e] : 0.f) + (t2 == 2u ? g[2][e] : 0.f) +
              (t3 == 0u ? g[3][e] : 0.f);
  }
}

__global__ __launch_bounds__(256) void maxpool_bn_bwd_reduce_quad_kernel(const uint16_t* __restrict__ dy,
                                                                         const uint8_t* __restrict__ idx,
                                                                         const uint16_t* __restrict__ x,
                                                                         const float* __restrict__ coef, int N, int H,
                                                                         int W, int C, int quads_per_block,
                                                                         float* __restrict__ part) {
  const int CPR = C >> 3;
  const int tid = threadIdx.x;
  const int QPI = 256 / CPR;
  const int c = tid % CPR, r = tid / CPR;
  const int OH = H >> 1, OW = W >> 1;
  const int Q = N * OH * OW;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);  // (XCD-contiguous: neighbouring quads share pooled rows in one L2)
  const int qb = lb * quads_per_block;
  const int qe = min(Q, qb + quads_per_block);
  float sm[8], sq[8], mean[8], sc[8], sh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sm[e] = 0.f; sq[e] = 0.f;
    sc[e] = coef[c * 8 + e]; sh[e] = coef[C + c * 8 + e]; mean[e] = coef[2 * C + c * 8 + e];
  }
  if (r < QPI) {
    // U quads per thread per iteration, all of their (dy, argmax, x) loads issued before the first
    // use: one quad at a time left this pass latency-bound (1.08 GB in 357 us)
    constexpr int U = 4;
    for (int q0 = qb + r; q0 < qe; q0 += U * QPI) {
      float d[U][4][8], xv[U][4][8];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int qd = min(q0 + u * QPI, qe - 1);
        const int j = qd % OW, t = qd / OW;
        const int i = t % OH, n = t / OH;
        pool_grad_quad(dy, idx, n, i, j, c * 8, C, OH, OW, d[u]);
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const size_t row = ((size_t)n * H + 2 * i + (v >> 1)) * W + 2 * j + (v & 1);
          unpack8(*(const u32x4*)(x + row * C + c * 8), xv[u][v]);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (q0 + u * QPI >= qe) break;
#pragma unroll
        for (int v = 0; v < 4; ++v)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float dz = fmaf(xv[u][v][e], sc[e], sh[e]) > 0.f ? d[u][v][e] : 0.f;
            sm[e] += dz;
            sq[e] += dz * (xv[u][v][e] - mean[e]);
          }
      }
    }
  }
  __shared__ float red[2][256][8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[0][tid][e] = sm[e]; red[1][tid][e] = sq[e]; }
  __syncthreads();
  for (int ch = tid; ch < C; ch += 256) {
    const int cc = ch >> 3, e = ch & 7;
    float a = 0.f, b2 = 0.f;
    for (int rr = 0; rr < QPI; ++rr) { a += red[0][rr * CPR + cc][e]; b2 += red[1][rr * CPR + cc][e]; }
    part[(int64_t)ch * gridDim.x + lb] = a;
    part[(int64_t)(C + ch) * gridDim.x + lb] = b2;
  }
}

__global__ __launch_bounds__(256) void maxpool_bn_bwd_apply_quad_kernel(const uint16_t* __restrict__ dy,
                                                                        const uint8_t* __restrict__ idx,
                                                                        const uint16_t* __restrict__ x,
                                                                        const float* __restrict__ coef,
                                                                        const float* __restrict__ bcoef,
                                                                        uint16_t* __restrict__ dx, int N, int H, int W,
                                                                        int C) {
  const int CPR = C >> 3;
  const int OH = H >> 1, OW = W >> 1;
  const int total = N * OH * OW * CPR;
  for (int it = blockIdx.x * 256 + threadIdx.x; it < total; it += gridDim.x * 256) {
    const int c8 = (it % CPR) * 8;
    int t = it / CPR;
    const int j = t % OW; t /= OW;
    const int i = t % OH;
    const int n = t / OH;
    float d[4][8];
    pool_grad_quad(dy, idx, n, i, j, c8, C, OH, OW, d);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t off = (((size_t)n * H + 2 * i + (u >> 1)) * W + 2 * j + (u & 1)) * C + c8;
      float xv[8], o[8];
      unpack8(*(const u32x4*)(x + off), xv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float dz = fmaf(xv[e], coef[c8 + e], coef[C + c8 + e]) > 0.f ? d[u][e] : 0.f;
        // (explicit fmaf chain: stem.hip's fused weight grad computes the same dx bit for bit)
        o[e] = fmaf(bcoef[c8 + e], dz, fmaf(bcoef[C + c8 + e], xv[e], bcoef[2 * C + c8 + e]));
      }
      *(u32x4*)(dx + off) = pack8(o);
    }
  }
}

// global average pool: x [N][HW][C] -> y [N][C] (bf16); one thread per (n, 8 channels)
__global__ __launch_bounds__(256) void gavgpool_fwd_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, int N,
                                                           int HW, int C) {
  const int CPR = C >> 3;
  const int64_t total = (int64_t)N * CPR;
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;
  if (i >= total) return;
  const int n = (int)(i / CPR), c8 = (int)(i % CPR) * 8;
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  const uint16_t* base = x + (int64_t)n * HW * C + c8;
  for (int j = 0; j < HW; ++j) {
    float f[8];
    unpack8(*(const u32x4*)(base + (int64_t)j * C), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += f[e];
  }
  const float inv = 1.f / (float)HW;
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] *= inv;
  *(u32x4*)(y + (int64_t)n * C + c8) = pack8(acc);
}

__global__ __launch_bounds__(256) void gavgpool_bwd_kernel(const uint16_t* __restrict__ dy, uint16_t* __restrict__ dx, int N,
                                                           int HW, int C) {
  const int CPR = C >> 3;
  const int64_t total = (int64_t)N * HW * CPR;
  const float inv = 1.f / (float)HW;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c8 = (int)(i % CPR) * 8;
    const int n = (int)(i / ((int64_t)HW * CPR));
    float f[8];
    unpack8(*(const u32x4*)(dy + (int64_t)n * C + c8), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] *= inv;
    *(u32x4*)(dx + i * 8) = pack8(f);
  }
}

}  // namespace dpe

using namespace dpe;

static unsigned exact_grid(int64_t n) { return (unsigned)std::max<int64_t>(1, (n + 255) / 256); }

// 1: the stem max-pool on maxpool_fwd_kernel<true, 3> instead of bnrelu_maxpool3_kernel (test hook: the two
// must agree bit for bit on values and argmax bytes)
static int g_pool_legacy = 0;
extern "C" void dpe_set_pool_legacy(int on) { g_pool_legacy = on; }

static int gs(int64_t n) {
  int64_t g = (n + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

extern "C" int dpe_maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* idx, int N, int H, int W, int C, int OH, int OW,
                               int k, int s, int p, hipStream_t st) {
  if (C % 8 || k * k > 255 || (int64_t)N * OH * OW * C / 8 >= (1ll << 31)) return -1;
  const dim3 g(exact_grid((int64_t)N * OH * OW * C / 8));
  if (k == 3)
    hipLaunchKernelGGL((maxpool_fwd_kernel<false, 3>), g, dim3(256), 0, st, x, y, idx, N, H, W, C, OH, OW, k, s, p, nullptr);
  else
    hipLaunchKernelGGL((maxpool_fwd_kernel<false, 0>), g, dim3(256), 0, st, x, y, idx, N, H, W, C, OH, OW, k, s, p, nullptr);
  return 0;
}

extern "C" int dpe_bnrelu_maxpool_fwd(const uint16_t* h, const float* coef, uint16_t* y, uint8_t* idx, int N, int H, int W,
                                      int C, int OH, int OW, int k, int s, int p, hipStream_t st) {
  if (C % 8 || k * k > 255 || (int64_t)N * OH * OW * C / 8 >= (1ll << 31)) return -1;
  if (k == 3 && s == 2 && p == 1 && C == 64 && OH == (H - 1) / 2 + 1 && OW == (W - 1) / 2 + 1 && !g_pool_legacy) {
    const int nx = (OW * 8 + 255) / 256;
    hipLaunchKernelGGL((bnrelu_maxpool3_kernel<8>), dim3((unsigned)((int64_t)N * OH * nx)), dim3(256), 0, st, h, y, idx, H, W,
                       OH, OW, nx, coef);
    return 0;
  }
  const dim3 g(exact_grid((int64_t)N * OH * OW * C / 8));
  if (k == 3)
    hipLaunchKernelGGL((maxpool_fwd_kernel<true, 3>), g, dim3(256), 0, st, h, y, idx, N, H, W, C, OH, OW, k, s, p, coef);
  else
    hipLaunchKernelGGL((maxpool_fwd_kernel<true, 0>), g, dim3(256), 0, st, h, y, idx, N, H, W, C, OH, OW, k, s, p, coef);
  return 0;
}

extern "C" int dpe_maxpool_bn_bwd_reduce(const uint16_t* dy, const uint8_t* idx, const uint16_t* x, const float* coef, int N,
                                         int H, int W, int C, int OH, int OW, int k, int s, int p, int nb, float* part,
                                         hipStream_t st) {
  if (C % 8 || C / 8 > 256 || (int64_t)N * H * W * C / 8 >= (1ll << 31)) return -1;
  const int64_t M = (int64_t)N * H * W;
  if (k == 3 && s == 2 && p == 1 && H % 2 == 0 && W % 2 == 0 && OH == H / 2 && OW == W / 2) {
    const int64_t Q = M / 4;
    const int qpb = (int)((Q + nb - 1) / nb);
    hipLaunchKernelGGL(maxpool_bn_bwd_reduce_quad_kernel, dim3(nb), dim3(256), 0, st, dy, idx, x, coef, N, H, W, C, qpb, part);
    return 0;
  }
  const int rpb = (int)((M + nb - 1) / nb);
  hipLaunchKernelGGL(maxpool_bn_bwd_reduce_kernel, dim3(nb), dim3(256), 0, st, dy, idx, x, coef, N, H, W, C, OH, OW, k, s, p,
                     rpb, part);
  return 0;
}

extern "C" int dpe_maxpool_bn_bwd_apply(const uint16_t* dy, const uint8_t* idx, const uint16_t* x, const float* coef,
                                        const float* bcoef, uint16_t* dx, int N, int H, int W, int C, int OH, int OW, int k,
                                        int s, int p, hipStream_t st) {
  if (C % 8 || (int64_t)N * H * W * C / 8 >= (1ll << 31)) return -1;
  if (k == 3 && s == 2 && p == 1 && H % 2 == 0 && W % 2 == 0 && OH == H / 2 && OW == W / 2) {
    hipLaunchKernelGGL(maxpool_bn_bwd_apply_quad_kernel, dim3(gs((int64_t)N * OH * OW * C / 8)), dim3(256), 0, st, dy, idx, x,
                       coef, bcoef, dx, N, H, W, C);
    return 0;
  }
  hipLaunchKernelGGL(maxpool_bn_bwd_apply_kernel, dim3(gs((int64_t)N * H * W * C / 8)), dim3(256), 0, st, dy, idx, x, coef,
                     bcoef, dx, N, H, W, C, OH, OW, k, s, p);
  return 0;
}

extern "C" int dpe_maxpool_bwd(const uint16_t* dy, const uint8_t* idx, uint16_t* dx, int N, int H, int W, int C, int OH,
                               int OW, int k, int s, int p, hipStream_t st) {
  if (C % 8) return -1;
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(gs((int64_t)N * H * W * C / 8)), dim3(256), 0, st, dy, idx, dx, N, H, W, C,
                     OH, OW, k, s, p);
  return 0;
}

extern "C" int dpe_gavgpool_fwd(const uint16_t* x, uint16_t* y, int N, int HW, int C, hipStream_t st) {
  if (C % 8) return -1;
  const int64_t total = (int64_t)N * C / 8;
  hipLaunchKernelGGL(gavgpool_fwd_kernel, dim3((int)((total + 255) / 256)), dim3(256), 0, st, x, y, N, HW, C);
  return 0;
}

extern "C" int dpe_gavgpool_bwd(const uint16_t* dy, uint16_t* dx, int N, int HW, int C, hipStream_t st) {
  if (C % 8) return -1;
  hipLaunchKernelGGL(gavgpool_bwd_kernel, dim3(gs((int64_t)N * HW * C / 8)), dim3(256), 0, st, dy, dx, N, HW, C);
  return 0;
}
