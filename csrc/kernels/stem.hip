// ResNet-50 stem convolution over the space-to-depth input: y[n][oh][ow][64] =
// sum_{dy,dx<4} sum_{c<16} xs[n][oh-2+dy][ow-2+dx][c] * w[o][dy][dx][c]  (4x4, stride 1, pad 2/2/1/1,
// the 7x7/s2 conv of ops/functional.py's s2d form), plus the BatchNorm-forward (sum, sum of squares)
// partials of the stored bf16 output.
//
// On the implicit-GEMM tile this shape ran at ~234 TF (519 us at batch 512): K = 256 is only eight
// 32-wide K-steps, the im2col operand re-reads every input pixel 16 times through L2 and each
// 128x64 tile re-reads the whole 32 KiB filter.  Here a block walks consecutive output rows of one
// image:
//   * the filter sits in VGPRs for the whole block (wave (mh, nh): 32 output channels x K = 256
//     as MFMA operands, 64 VGPRs);
//   * the four input rows an output row needs live in a 5-slot LDS ring ([132 pixels][16 ch],
//     zero pixels at both ends); each input row is loaded from HBM once per block (register
//     prefetch two rows ahead, written into the free slot after the row's MFMAs);
//   * an output row (112 pixels x 64 channels) is staged in one of two LDS buffers and stored as
//     whole 16-B chunks of contiguous pixels; BN sums accumulate per thread over the block's rows
//     and are reduced once: one partial column per block ([2][64][blocks]).
// One barrier per output row.  Same K order as the implicit GEMM (two taps per K-step), so the
// output is bitwise identical to it.
#include <cstdlib>

#include "common.h"

namespace dpe {
namespace stem {

constexpr int CO = 64, KK = 8;            // output channels, 32-wide K-steps (K = 256)
constexpr int SLOT_PX = 132;              // ring slot pixels: 2 zero + <= 112 data + zero tail
constexpr int SLOT = SLOT_PX * 32;        // bytes per slot (16 ch bf16 per pixel)
constexpr int NSLOT = 5;
constexpr int OROW = 144;                 // staged output row stride (128 B + 16 pad)
constexpr int OBUF = 112 * OROW;
constexpr int LDS = NSLOT * SLOT + 2 * OBUF;
static_assert(LDS <= 163840 / 3, "three blocks per CU");

DPE_DEVICE u32x4 zero16() { return u32x4{0u, 0u, 0u, 0u}; }

__global__ __launch_bounds__(256, 3) void stem_conv_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                           uint16_t* __restrict__ y, float* __restrict__ stats, int H,
                                                           int W, int parts) {
  __shared__ __attribute__((aligned(16))) char smem[LDS];
  char* const ring = smem;
  char* const obuf = smem + NSLOT * SLOT;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int mh = wid & 1, nh = wid >> 1;  // pixel half (frags 0-3 / 4-6), channel half (32 each)
  const int nfr = mh ? 3 : 4;             // 16-pixel MFMA fragments of this wave (W = 112)
  const int blk = blockIdx.x;
  const int n = blk / parts, part = blk - n * parts;
  const int oh_beg = (int)((int64_t)H * part / parts), oh_end = (int)((int64_t)H * (part + 1) / parts);
  const int lm = lane & 15, kc = lane >> 4;

  // filter fragments: output channel 32 nh + 16 j + lm, K elements 32 kk + 8 kc .. +7
  bf16x8 wf[KK][2];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      wf[kk][j] = __builtin_bit_cast(bf16x8, *(const u32x4*)(w + (32 * nh + 16 * j + lm) * 256 + 32 * kk + 8 * kc));

  // zero the ring (pad pixels stay zero; rows outside the image are written as zeros)
  for (int i = tid; i < NSLOT * SLOT / 16; i += 256) *(u32x4*)(ring + i * 16) = zero16();

  // one input row = W pixels x 32 B = up to 224 16-B chunks: thread t < 2W owns chunk t
  const int64_t img = (int64_t)n * H * W * 16;
  auto load_row = [&](int ih) -> u32x4 {
    if (tid < 2 * W && (unsigned)ih < (unsigned)H) return *(const u32x4*)(x + img + ((int64_t)ih * W) * 16 + tid * 8);
    return zero16();
  };
  auto write_row = [&](int ih, const u32x4& v) {  // input row ih -> slot (ih + 2) % 5, pixel iw + 2
    if (tid < 2 * W) *(u32x4*)(ring + ((ih + 2 + 5 * 4) % NSLOT) * SLOT + 64 + tid * 16) = v;
  };
  __syncthreads();  // ring zeroed before the first rows land
#pragma unroll
  for (int d = -2; d < 2; ++d) write_row(oh_beg + d, load_row(oh_beg + d));
  u32x4 pf0 = load_row(oh_beg + 2), pf1 = load_row(oh_beg + 3);  // rows oh + 2 / oh + 3 of the first iteration
  __syncthreads();

  float s[8], ss[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s[e] = 0.f; ss[e] = 0.f; }
  const int sc = tid & 7;  // this thread's 8-channel chunk in the store phase

  for (int oh = oh_beg; oh < oh_end; ++oh) {
    f32x4 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // K-step kk: filter row dy = kk / 2, taps dx = 2 (kk & 1) + {0, 1}; lane chunk kc -> tap
    // dx0 + kc / 2, channels 8 (kc & 1) .. +7.  Input row oh - 2 + dy sits in slot (oh + dy) % 5.
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const char* sl = ring + ((oh + (kk >> 1)) % NSLOT) * SLOT + ((kk & 1) * 2 + (kc >> 1)) * 32 + (kc & 1) * 16;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (i < nfr) {
          const int ow = (mh * 4 + i) * 16 + lm;
          const bf16x8 af = __builtin_bit_cast(bf16x8, *(const u32x4*)(sl + ow * 32));
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[kk][j], af, acc[i][j], 0, 0, 0);
        }
      }
    }
    // input row oh + 2 into the slot of row oh - 3 (no longer read); prefetch row oh + 4
    write_row(oh + 2, pf0);
    pf0 = pf1;
    pf1 = load_row(oh + 4);
    // stage the output row: acc[i][j][e] = pixel (mh*4+i)*16 + lm, channel 32 nh + 16 j + 4 kc + e
    char* ob = obuf + (oh & 1) * OBUF;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i < nfr) {
        const int ow = (mh * 4 + i) * 16 + lm;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          u32x2 pk;
          pk[0] = pack_bf2(acc[i][j][0], acc[i][j][1]);
          pk[1] = pack_bf2(acc[i][j][2], acc[i][j][3]);
          *(u32x2*)(ob + ow * OROW + (32 * nh + 16 * j + 4 * kc) * 2) = pk;
        }
      }
    }
    __syncthreads();
    // store: thread t -> chunk t & 7 of pixels t / 8 + 32 k (whole 128-B pixel rows per 8 lanes)
    uint16_t* yrow = y + ((int64_t)n * H + oh) * W * CO;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int px = (tid >> 3) + 32 * k;
      if (px < W) {
        const u32x4 v = *(const u32x4*)(ob + px * OROW + sc * 16);
        *(u32x4*)(yrow + px * CO + sc * 8) = v;
        float f[8];
        unpack8(v, f);
#pragma unroll
        for (int e = 0; e < 8; ++e) { s[e] += f[e]; ss[e] = fmaf(f[e], f[e], ss[e]); }
      }
    }
  }
  if (stats) {
    // reduce over the 32 threads of each chunk: lanes sc + 8 t (xor 8, 16, 32), then 4 waves via LDS
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int o = 8; o < 64; o <<= 1) {
        s[e] += __shfl_xor(s[e], o, 64);
        ss[e] += __shfl_xor(ss[e], o, 64);
      }
    __syncthreads();
    float* red = (float*)ring;  // [2][4 waves][64]
    if (lane < 8)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[wid * CO + sc * 8 + e] = s[e];
        red[4 * CO + wid * CO + sc * 8 + e] = ss[e];
      }
    __syncthreads();
    if (tid < CO) {
      const int nb = gridDim.x;
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) { a += red[q * CO + tid]; b += red[4 * CO + q * CO + tid]; }
      stats[(int64_t)tid * nb + blk] = a;
      stats[(int64_t)(CO + tid) * nb + blk] = b;
    }
  }
}


// ------------------------------------------------------------------ weight grad
// dW[o][dy][dx][c] += alpha * sum_{n, oh, ow} dY[n, oh, ow, o] * xs[n, oh - 2 + dy, ow - 2 + dx, c]:
// M = 64, N = 256, K = the 6.4 M output pixels at batch 512.  The im2col weight-grad tile
// (igemm_wgrad_dma 64x256) re-reads every input pixel 16 times through L2 and ran at ~480 TF
// (443 us).  As in the layer-1 weight grad (rowconv.hip), a block walks the output rows of one image
// and keeps that image's whole 64 x 256 gradient in registers: wave w owns filter row dy = w (4 taps
// x 16 channels) for all 64 output channels (4 x 4 accumulator tiles, 64 VGPRs).  Per output row the
// dY row (K = pixels, M = o) and the four input rows (K = pixels shifted by the tap column, N = c)
// are LDS images read with ds_read_b64_tr_b16, each row loaded from HBM once per block; per-image
// partials in accumulator order, summed by wgrad_reduce_kernel.
namespace wg {
constexpr int XROWS = 136;                   // slot pixel rows: 2 zero + W (<= 112) + zeros (K reads <= 130)
constexpr int XSLOT = XROWS * 32;            // 16 channels bf16 per pixel row
constexpr int DSLOT = 128 * 128;             // dY row: 128 pixel rows x 64 channels (>= W zero)
constexpr int LDS = NSLOT * XSLOT + 2 * DSLOT;
constexpr int PART = 64 * 256;
static_assert(LDS <= 163840 / 2, "two blocks per CU");

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// dY image [pixel rows][64 ch]: 16-B chunks XOR-swizzled by row bits 1 and 3 (conflict-free tr reads)
DPE_DEVICE int d_off(int k, int chunk) {
  const int h = (((k >> 1) & 1) | (((k >> 3) & 1) << 1)) << 1;
  return k * 128 + ((chunk ^ h) << 4);
}
// x image [pixel rows][16 ch] (32-B rows): rows with bit 3 set live in the other 128-B half of their
// 256-B bank window, so rows r and r + 8 (read by one half-wave) never share banks, at any shift
DPE_DEVICE int x_off(int k) { return (k * 32) ^ (((k >> 3) & 1) << 7); }

DPE_DEVICE bf16x8 tr2(const char* a1, const char* a2) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a2);
  s16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return __builtin_bit_cast(bf16x8, r);
}
// operand fragments: columns (lane & 15) of c0 .. c0 + 15, K = image rows row0 + 8 (lane >> 4) .. +7
DPE_DEVICE bf16x8 dfrag(const char* img, int row0, int c0) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
  const int k1 = row0 + 8 * g + q, mc = (c0 >> 3) + (pp >> 1), sub = (pp & 1) * 8;
  return tr2(img + d_off(k1, mc) + sub, img + d_off(k1 + 4, mc) + sub);
}
DPE_DEVICE bf16x8 xfrag(const char* img, int row0) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
  const int k1 = row0 + 8 * g + q;
  return tr2(img + x_off(k1) + pp * 8, img + x_off(k1 + 4) + pp * 8);
}

__global__ __launch_bounds__(256, 2) void stem_wgrad_kernel(const uint16_t* __restrict__ x,
                                                            const uint16_t* __restrict__ dy,
                                                            float* __restrict__ part, int H, int W, int halves) {
  __shared__ __attribute__((aligned(16))) char smem[LDS];
  char* const ring = smem;                     // input row ih in slot (ih + 2) % 5
  char* const dbuf = smem + NSLOT * XSLOT;     // dY row oh in slot oh & 1
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // filter row dy = w
  // halves = 2: block b covers output rows [oh0, oh1) = half b & 1 of image b >> 1 (more, shorter blocks:
  // the dispatcher balances them around foreign workgroups -- the CU budget, comm.cpp)
  const int n = (int)blockIdx.x / halves, hb = (int)blockIdx.x % halves;
  const int oh0 = hb * ((H + halves - 1) / halves), oh1 = min(H, oh0 + (H + halves - 1) / halves);
  const int64_t ximg = (int64_t)n * H * W * 16, dimg = (int64_t)n * H * W * 64;
  const int xch = W * 2, dch = W * 8;          // 16-B chunks per row

  for (int i = tid; i < LDS / 16; i += 256) *(u32x4*)(smem + i * 16) = zero16();

  auto loadx = [&](int ih) -> u32x4 {
    if (tid < xch && (unsigned)ih < (unsigned)H) return *(const u32x4*)(x + ximg + (int64_t)ih * W * 16 + tid * 8);
    return zero16();
  };
  auto putx = [&](int ih, const u32x4& v) {  // chunk t -> pixel t / 2 (slot row + 2), half t & 1
    if (tid < xch) *(u32x4*)(ring + ((ih + 2 + 5 * 4) % NSLOT) * XSLOT + x_off((tid >> 1) + 2) + (tid & 1) * 16) = v;
  };
  auto loadd = [&](int oh, u32x4 (&v)[4]) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = tid + 256 * u;
      v[u] = (c < dch && oh < H) ? *(const u32x4*)(dy + dimg + (int64_t)oh * W * 64 + c * 8) : zero16();
    }
  };
  auto putd = [&](int oh, const u32x4 (&v)[4]) {
    char* sl = dbuf + (oh & 1) * DSLOT;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = tid + 256 * u;
      if (c < dch) *(u32x4*)(sl + d_off(c >> 3, c & 7)) = v[u];
    }
  };
  __syncthreads();
  {
#pragma unroll
    for (int d = -2; d < 2; ++d) putx(oh0 + d, loadx(oh0 + d));
    u32x4 t[4];
    loadd(oh0, t);
    putd(oh0, t);
  }
  u32x4 px0 = loadx(oh0 + 2), px1 = loadx(oh0 + 3);  // input rows oh + 2, oh + 3
  u32x4 pd0[4], pd1[4];                              // dY rows oh + 1, oh + 2
  loadd(oh0 + 1, pd0);
  loadd(oh0 + 2, pd1);
  __syncthreads();

  f32x4 acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nks = (W + 31) / 32;

  // one output row; pxA / pdA hold input row oh + 2 / dY row oh + 1 and are refilled in place with
  // rows oh + 4 / oh + 3 (the loop runs two rows per trip with two buffer sets, so a prefetch is
  // first waited on two rows after it was issued -- a register copy between the sets would wait
  // after one)
  auto step = [&](int oh, u32x4& pxA, u32x4 (&pdA)[4]) {
    const char* ds = dbuf + (oh & 1) * DSLOT;
    // input row oh - 2 + w sits in slot (oh + w) % 5; output pixel ow reads slot row ow + dx
    const char* xs = ring + ((oh + w) % NSLOT) * XSLOT;
    for (int ks = 0; ks < nks; ++ks) {
      bf16x8 a[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) a[m] = dfrag(ds, 32 * ks, 16 * m);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bf16x8 b = xfrag(xs, 32 * ks + t);
#pragma unroll
        for (int m = 0; m < 4; ++m) acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a[m], acc[m][t], 0, 0, 0);
      }
    }
    // input row oh + 2 into the slot of row oh - 3, dY row oh + 1 into the slot of row oh - 1
    putx(oh + 2, pxA);
    putd(oh + 1, pdA);
    pxA = loadx(oh + 4);
    loadd(oh + 3, pdA);
    __syncthreads();
  };
  for (int oh = oh0; oh < oh1; oh += 2) {
    step(oh, px0, pd0);
    if (oh + 1 < oh1) step(oh + 1, px1, pd1);
  }
  // acc[m][t][e]: o = 16 m + (lane & 15), c = 4 (lane >> 4) + e, tap (dy = w, dx = t)
  float* pb = part + (int64_t)blockIdx.x * PART;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int t = 0; t < 4; ++t) *(f32x4*)(pb + (((m * 4 + t) * 4 + w) * 64 + lane) * 4) = acc[m][t];
}

// dW [64][4][4][16] += alpha * sum of the partials; grid (PART / 1024, groups), 256 threads
__global__ __launch_bounds__(256) void stem_wgrad_reduce_kernel(const float* __restrict__ part, float* __restrict__ dw,
                                                                int nparts, int per, float alpha) {
  const int q = blockIdx.x * 256 + threadIdx.x;
  const int b0 = blockIdx.y * per, b1 = min(nparts, b0 + per);
  f32x4 s0 = f32x4{0.f, 0.f, 0.f, 0.f}, s1 = s0;
  const f32x4* src = (const f32x4*)part + q;
  int b = b0;
  for (; b + 1 < b1; b += 2) {
    s0 += src[(int64_t)b * (PART / 4)];
    s1 += src[(int64_t)(b + 1) * (PART / 4)];
  }
  if (b < b1) s0 += src[(int64_t)b * (PART / 4)];
  s0 += s1;
  const int lane = q & 63, w = (q >> 6) & 3, mt = q >> 8, t = mt & 3, m = mt >> 2;
  float* d = dw + (16 * m + (lane & 15)) * 256 + (w * 4 + t) * 16 + 4 * (lane >> 4);
#pragma unroll
  for (int e = 0; e < 4; ++e) atomicAdd(d + e, alpha * s0[e]);
}
}  // namespace wg
}  // namespace stem
}  // namespace dpe

// Blocks of the launch for an [N, H, W, 16] s2d input (0: outside the kernel's envelope).
extern "C" int dpe_stem_blocks(int N, int H, int W) {
  if (N <= 0 || H < 3 || W < 97 || W > 112) return 0;  // 7 pixel fragments, 4 + 3 per wave pair
  return N * 3;
}

// y [N, H, W, 64] bf16, stats [2][64][dpe_stem_blocks] or nullptr; w [64][4][4][16] bf16.
extern "C" int dpe_stem_launch(const uint16_t* x, const uint16_t* w, uint16_t* y, float* stats, int N, int H, int W,
                               hipStream_t st) {
  const int nb = dpe_stem_blocks(N, H, W);
  if (nb <= 0) return -1;
  hipLaunchKernelGGL(dpe::stem::stem_conv_kernel, dim3(nb), dim3(256), 0, st, x, w, y, stats, H, W, 3);
  return (int)hipGetLastError();
}

extern "C" int dpe_cu_reserve();  // comm.cpp

// Blocks per image of the stem weight grad: 2 (half-image blocks) while a CU budget is in force
// (collectives in flight: two dispatch rounds balance around their workgroups), else 1.
static int stem_wgrad_halves(int H) {
  static const bool on = [] { const char* e = getenv("DPE_STEM_HALVES"); return !(e && e[0] == '0'); }();
  return (on && dpe_cu_reserve() > 0 && H >= 8) ? 2 : 1;
}

// Scratch floats of the stem weight-grad launch (per-block partials), 0: outside the envelope.
extern "C" int64_t dpe_stem_wgrad_scratch(int N, int H, int W) {
  if (N <= 0 || H < 2 || W < 1 || W > 112) return 0;
  return (int64_t)N * stem_wgrad_halves(H) * dpe::stem::wg::PART;
}

// dw [64][4][4][16] (+)= alpha * filter gradient of the s2d stem conv, given dY [N, H, W, 64].
extern "C" int dpe_stem_wgrad_launch(const uint16_t* x, const uint16_t* dy, float* dw, float* scratch, int N, int H, int W,
                                     float alpha, hipStream_t st) {
  if (dpe_stem_wgrad_scratch(N, H, W) <= 0 || !scratch) return -1;
  using namespace dpe::stem::wg;
  const int halves = stem_wgrad_halves(H), nparts = N * halves;
  hipLaunchKernelGGL(stem_wgrad_kernel, dim3(nparts), dim3(256), 0, st, x, dy, scratch, H, W, halves);
  const int groups = nparts >= 64 ? 16 : 1;
  const int per = (nparts + groups - 1) / groups;
  hipLaunchKernelGGL(stem_wgrad_reduce_kernel, dim3(PART / 1024, groups), dim3(256), 0, st, scratch, dw, nparts, per,
                     alpha);
  return (int)hipGetLastError();
}
