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
#include <type_traits>

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
  // global loads / stores through buffer resources, issued unconditionally (out-of-range: an offset past
  // the resource), so the compiler's waits stay counted and the row prefetch stays in flight (host:
  // N H W 128 < 0xffffff00)
  const int NI = gridDim.x / parts;
  const __amdgpu_buffer_rsrc_t xr = buf_rsrc(x, (uint32_t)((int64_t)NI * H * W * 32));
  const __amdgpu_buffer_rsrc_t yr = buf_rsrc(y, (uint32_t)((int64_t)NI * H * W * CO * 2));
  auto load_row = [&](int ih) -> u32x4 {
    const bool ok = tid < 2 * W && (unsigned)ih < (unsigned)H;
    return __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? (uint32_t)((img + (int64_t)ih * W * 16 + tid * 8) * 2) : BUF_OOB, 0, 0);
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

  // one output row; pfA holds input row oh + 2 and is refilled with row oh + 4 (two register sets, rows
  // alternate: a prefetch is first used two rows after it was issued)
  auto row = [&](const int oh, u32x4& pfA) {
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
    write_row(oh + 2, pfA);
    pfA = load_row(oh + 4);
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
    lds_barrier();  // (LDS only: __syncthreads would drain the prefetch just issued)
    // store: thread t -> chunk t & 7 of pixels t / 8 + 32 k (whole 128-B pixel rows per 8 lanes)
    const int64_t yrow = ((int64_t)n * H + oh) * W * CO;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int px = (tid >> 3) + 32 * k;
      const u32x4 v = *(const u32x4*)(ob + min(px, 111) * OROW + sc * 16);
      __builtin_amdgcn_raw_buffer_store_b128(v, yr, px < W ? (uint32_t)((yrow + px * CO + sc * 8) * 2) : BUF_OOB, 0, 0);
      if (px < W) {
        float f[8];
        unpack8(v, f);
#pragma unroll
        for (int e = 0; e < 8; ++e) { s[e] += f[e]; ss[e] = fmaf(f[e], f[e], ss[e]); }
      }
    }
  };
  for (int oh = oh_beg;; oh += 2) {  // (one backedge, after the second row: see stem_wgrad_kernel)
    row(oh, pf0);
    if (oh + 1 >= oh_end) break;
    row(oh + 1, pf1);
    if (oh + 2 >= oh_end) break;
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

// FUSED: dY is never materialised.  The stem's forward was h = conv(xs) -> relu(BN(h)) -> 3x3/s2/p1
// max-pool (never stored either, pool.hip); its backward needs dY = dL/dh = a dz + b h + c with
// dz = [h scale + shift > 0] * (pooled gradient gathered through the argmax bytes) and (a, b, c) from the
// BN-backward reduce.  The standalone apply pass (maxpool_bn_bwd_apply_quad: read dy_p, idx, h, write dY
// = 1.95 GB at batch 512) is replaced by computing each dY row here, where it is staged into LDS anyway:
// h rows take the dY rows' register prefetch, and the pooled rows (dy_p, idx) a window needs sit in a
// 2-slot LDS ring (pooled row i covers h rows 2i-1 .. 2i+1: an even row reads one pooled row, an odd row
// two), each loaded from HBM once per block, one pooled row ahead in registers.  The dY values are
// computed exactly as the apply kernel computes them (same window order, same fmaf chain): bitwise the
// same operand.
struct StemBwd {
  const uint16_t* dyp;  // pooled gradient [N][H/2][W/2][64]
  const uint8_t* idx;   // argmax tap per pooled element (same shape)
  const uint16_t* h;    // pre-BN stem output [N][H][W][64]
  const float* coef;    // BN forward [4][64]: scale, shift, mean, invstd
  const float* bcoef;   // BN backward [3][64]: a, b, c
};
constexpr int PW = 56;                          // pooled row pixels (W / 2 <= 56)
constexpr int PDY = PW * 128, PIDX = PW * 64;   // bytes of one pooled dy row / idx row
constexpr int PSLOT = PDY + PIDX;
constexpr int LDS_F = LDS + 2 * PSLOT + 5 * 64 * 4;  // + the 5 x 64 BN coefficients
static_assert(LDS_F <= 163840 / 2, "two blocks per CU (fused)");

template <bool FUSED>
__global__ __launch_bounds__(256, 2) void stem_wgrad_kernel(const uint16_t* __restrict__ x,
                                                            const uint16_t* __restrict__ dy,
                                                            float* __restrict__ part, int H, int W, int halves,
                                                            StemBwd fb) {
  __shared__ __attribute__((aligned(16))) char smem[FUSED ? LDS_F : LDS];
  char* const ring = smem;                     // input row ih in slot (ih + 2) % 5
  char* const dbuf = smem + NSLOT * XSLOT;     // dY row oh in slot oh & 1
  char* const pring = smem + LDS;              // FUSED: pooled row i in slot i & 1 (dy, then idx)
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // filter row dy = w
  // halves = 2: block b covers output rows [oh0, oh1) = half b & 1 of image b >> 1 (more, shorter blocks:
  // the dispatcher balances them around foreign workgroups -- the CU budget, comm.cpp)
  const int n = (int)blockIdx.x / halves, hb = (int)blockIdx.x % halves;
  const int oh0 = hb * ((H + halves - 1) / halves), oh1 = min(H, oh0 + (H + halves - 1) / halves);
  const int64_t ximg = (int64_t)n * H * W * 16, dimg = (int64_t)n * H * W * 64;
  const int xch = W * 2, dch = W * 8;          // 16-B chunks per row

  for (int i = tid; i < LDS / 16; i += 256) *(u32x4*)(smem + i * 16) = zero16();

  // global loads through buffer resources, issued unconditionally (see stem_conv_kernel)
  const int NI = gridDim.x / halves;
  const __amdgpu_buffer_rsrc_t xr = buf_rsrc(x, (uint32_t)((int64_t)NI * H * W * 32));
  const __amdgpu_buffer_rsrc_t dr = buf_rsrc(FUSED ? (const void*)fb.h : (const void*)dy, (uint32_t)((int64_t)NI * H * W * 128));
  auto loadx = [&](int ih) -> u32x4 {
    const bool ok = tid < xch && (unsigned)ih < (unsigned)H;
    return __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? (uint32_t)((ximg + (int64_t)ih * W * 16 + tid * 8) * 2) : BUF_OOB, 0, 0);
  };
  auto putx = [&](int ih, const u32x4& v) {  // chunk t -> pixel t / 2 (slot row + 2), half t & 1
    if (tid < xch) *(u32x4*)(ring + ((ih + 2 + 5 * 4) % NSLOT) * XSLOT + x_off((tid >> 1) + 2) + (tid & 1) * 16) = v;
  };
  // FUSED: v holds the h row (the dY row's pre-BN input), not dY
  const uint16_t* const dsrc = FUSED ? fb.h : dy;
  auto loadd = [&](int oh, u32x4 (&v)[4]) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = tid + 256 * u;
      const bool ok = c < dch && oh < H;
      v[u] = __builtin_amdgcn_raw_buffer_load_b128(dr, ok ? (uint32_t)((dimg + (int64_t)oh * W * 64 + c * 8) * 2) : BUF_OOB, 0, 0);
    }
  };
  // FUSED: pooled row i (dy and argmax bytes) -> registers -> LDS slot i & 1
  const int OH = H >> 1, OW = W >> 1;
  const int64_t pimg = (int64_t)n * OH * OW * 64;
  const int pdch = OW * 8, pich = OW * 4;  // 16-B chunks of a pooled dy / idx row
  const __amdgpu_buffer_rsrc_t pr = buf_rsrc(FUSED ? (const void*)fb.dyp : (const void*)x, FUSED ? (uint32_t)((int64_t)NI * OH * OW * 128) : 0u);
  const __amdgpu_buffer_rsrc_t ir = buf_rsrc(FUSED ? (const void*)fb.idx : (const void*)x, FUSED ? (uint32_t)((int64_t)NI * OH * OW * 64) : 0u);
  auto loadp = [&](int i, u32x4 (&v)[3]) {
    if constexpr (FUSED) {
      const bool ok = i < OH;  // (block-uniform)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int c = tid + 256 * u;
        v[u] = __builtin_amdgcn_raw_buffer_load_b128(pr, (ok && c < pdch) ? (uint32_t)((pimg + (int64_t)i * OW * 64 + c * 8) * 2) : BUF_OOB, 0, 0);
      }
      // an out-of-range pooled row: argmax 0xff never matches a tap (selected after the load: the load
      // itself stays unconditional)
      const u32x4 t = __builtin_amdgcn_raw_buffer_load_b128(ir, (ok && tid < pich) ? (uint32_t)(pimg + (int64_t)i * OW * 64 + tid * 16) : BUF_OOB, 0, 0);
      v[2] = ok ? t : u32x4{~0u, ~0u, ~0u, ~0u};
    }
  };
  auto putp = [&](int i, const u32x4 (&v)[3]) {
    if constexpr (FUSED) {
      char* sl = pring + (i & 1) * PSLOT;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int c = tid + 256 * u;
        if (c < pdch) *(u32x4*)(sl + c * 16) = v[u];
      }
      if (tid < pich) *(u32x4*)(sl + PDY + tid * 16) = v[2];
    }
  };
  // FUSED: [scale | shift | a | b | c] x 64 channels in LDS (read per chunk: no 40 registers held all along)
  float* const pcoef = (float*)(smem + LDS + 2 * PSLOT);
  if constexpr (FUSED) {
    if (tid < 128) pcoef[tid] = fb.coef[tid];
    else pcoef[tid] = fb.bcoef[tid - 128];  // (a, b rows: tid 128 .. 255)
    if (tid < 64) pcoef[256 + tid] = fb.bcoef[128 + tid];
  }
  auto putd = [&](int oh, const u32x4 (&v)[4]) {
    char* sl = dbuf + (oh & 1) * DSLOT;
    // FUSED: this thread's 8 channels are cg = tid % 8 for every chunk (c = tid + 256 u); the pooled rows
    // i0 .. i1 of dY row oh
    const int cg = tid & 7, i0 = oh >> 1, i1 = (oh + 1) >> 1, ni = i1 == i0 ? 1 : 2;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = tid + 256 * u;
      if (c >= dch) continue;
      if constexpr (FUSED) {
        // dY chunk (pixel ow = c / 8, channels 8 (c % 8) ..): the windows (i, j) covering (oh, ow), in the
        // apply kernel's order (row-major), tap 3 (oh - 2i + 1) + (ow - 2j + 1).  Branch-free over the
        // column windows (a duplicate or out-of-range one gets tap 0x100, which no argmax byte equals, and
        // adds +0): every window's LDS reads are issued before the first compare.
        const int ow = c >> 3;
        const int j0 = ow >> 1, j1 = (ow + 1) >> 1;
        u32x4 gv[2][2];
        u32x2 bv[2][2];
        uint32_t tp[2][2];
#pragma unroll
        for (int wi = 0; wi < 2; ++wi) {
          if (wi >= ni) break;  // wave-uniform (oh is)
          const int i = wi ? i1 : i0;
          const char* sl2 = pring + (i & 1) * PSLOT;
#pragma unroll
          for (int wj = 0; wj < 2; ++wj) {
            const int j = wj ? j1 : j0;
            const bool valid = (wj == 0 || j1 != j0) && j < OW;
            const int jj = min(j, OW - 1);
            gv[wi][wj] = *(const u32x4*)(sl2 + (jj * 8 + cg) * 16);
            bv[wi][wj] = *(const u32x2*)(sl2 + PDY + (jj * 64 + cg * 8));
            tp[wi][wj] = valid ? (uint32_t)(3 * (oh - 2 * i + 1) + (ow - 2 * j + 1)) : 0x100u;
          }
        }
        float dz[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) dz[e] = 0.f;
#pragma unroll
        for (int wi = 0; wi < 2; ++wi) {
          if (wi >= ni) break;
#pragma unroll
          for (int wj = 0; wj < 2; ++wj) {
            float g[8];
            unpack8(gv[wi][wj], g);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const uint32_t t = (bv[wi][wj][e >> 2] >> ((e & 3) * 8)) & 0xffu;
              dz[e] += t == tp[wi][wj] ? g[e] : 0.f;
            }
          }
        }
        float hv[8], o[8];
        unpack8(v[u], hv);
        const float* pc = pcoef + cg * 8;
#pragma unroll
        for (int h4 = 0; h4 < 2; ++h4) {  // 4 channels at a time: 20 coefficient registers, not 40
          const f32x4 k0 = *(const f32x4*)(pc + 4 * h4), k1 = *(const f32x4*)(pc + 64 + 4 * h4);
          const f32x4 k2 = *(const f32x4*)(pc + 128 + 4 * h4), k3 = *(const f32x4*)(pc + 192 + 4 * h4);
          const f32x4 k4 = *(const f32x4*)(pc + 256 + 4 * h4);
#pragma unroll
          for (int e4 = 0; e4 < 4; ++e4) {
            const int e = 4 * h4 + e4;
            const float d = fmaf(hv[e], k0[e4], k1[e4]) > 0.f ? dz[e] : 0.f;
            o[e] = fmaf(k2[e4], d, fmaf(k3[e4], hv[e], k4[e4]));
          }
        }
        *(u32x4*)(sl + d_off(c >> 3, c & 7)) = pack8(o);
        __builtin_amdgcn_sched_barrier(0);  // one chunk's temporaries at a time (register pressure)
      } else {
        *(u32x4*)(sl + d_off(c >> 3, c & 7)) = v[u];
      }
    }
  };
  __syncthreads();
  // FUSED pooled-row schedule: dY row oh needs pooled rows oh >> 1 .. (oh + 1) >> 1.  Before the loop the
  // ring holds rows p0 = oh0 >> 1 and p0 + 1; row q + 2 (q = the slot it replaces) is written during the
  // step of the odd dY row 2q + 1... see step() below.
  u32x4 pp[3];
  const int p0 = oh0 >> 1;
  if constexpr (FUSED) {
    u32x4 t[3];
    loadp(p0, t);
    putp(p0, t);
    loadp(p0 + 1, t);
    putp(p0 + 1, t);
    loadp(p0 + 2, pp);
    __syncthreads();
  }
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
  // ODD: oh is odd (the block's first row is even: host check), a compile-time tag so the pooled-row
  // refill below is unconditional code in the odd step (a load under a run-time branch made the
  // compiler's later waits vmcnt(0), draining the row prefetch)
  auto step = [&](int oh, u32x4& pxA, u32x4 (&pdA)[4], auto odd_tag) {
    constexpr bool ODD = decltype(odd_tag)::value;
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
    if constexpr (FUSED) {
      // dY row oh + 1 read pooled rows (oh + 1) >> 1 .. (oh + 2) >> 1.  When oh + 1 is even (= 2q), row q - 1
      // was last read by dY row 2q - 1 (previous step, behind its barrier) and no dY row computed later needs
      // it: pooled row q + 1 (prefetched in pp) goes into its slot now, read first by dY row 2q + 1 (next
      // step, behind this step's barrier).
      if constexpr (ODD) {  // q + 1 > p0 + 1 always holds here: rows p0, p0 + 1 were placed before the loop
        const int q = (oh + 1) >> 1;
        putp(q + 1, pp);
        loadp(q + 2, pp);
      }
    }
    pxA = loadx(oh + 4);
    loadd(oh + 3, pdA);
    lds_barrier();  // (LDS only: __syncthreads would drain the prefetch just issued)
  };
  for (int oh = oh0; oh < oh1; oh += 2) {
    step(oh, px0, pd0, std::false_type{});
    if (oh + 1 < oh1) step(oh + 1, px1, pd1, std::true_type{});
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
  if (N <= 0 || H < 3 || W < 97 || W > 112 || (int64_t)N * H * W * 128 >= 0xffffff00ll) return 0;  // 7 pixel fragments, 4 + 3 per wave pair
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
  if (N <= 0 || H < 2 || W < 1 || W > 112 || (int64_t)N * H * W * 128 >= 0xffffff00ll) return 0;
  return (int64_t)N * stem_wgrad_halves(H) * dpe::stem::wg::PART;
}

// dw [64][4][4][16] (+)= alpha * filter gradient of the s2d stem conv, given dY [N, H, W, 64] -- or, with
// dyp != nullptr, given the stem's pooled gradient: dY = BN-backward(maxpool-backward(dyp)) computed on the
// fly (stem_wgrad_kernel<true>; 3x3 / s2 / p1 pool, even H and W).
extern "C" int dpe_stem_wgrad_launch2(const uint16_t* x, const uint16_t* dy, float* dw, float* scratch, int N, int H, int W,
                                      float alpha, const uint16_t* dyp, const uint8_t* idx, const uint16_t* h,
                                      const float* coef, const float* bcoef, hipStream_t st) {
  if (dpe_stem_wgrad_scratch(N, H, W) <= 0 || !scratch) return -1;
  using namespace dpe::stem::wg;
  const int halves = stem_wgrad_halves(H), nparts = N * halves;
  if (dyp) {
    if ((H & 1) || (W & 1) || W / 2 > PW || !idx || !h || !coef || !bcoef) return -1;
    // the pooled-row schedule assumes the block's first row is even (halves of an even H with an even half)
    if (halves > 1 && (((H + halves - 1) / halves) & 1)) return -1;
    hipLaunchKernelGGL(stem_wgrad_kernel<true>, dim3(nparts), dim3(256), 0, st, x, dy, scratch, H, W, halves,
                       StemBwd{dyp, idx, h, coef, bcoef});
  } else {
    hipLaunchKernelGGL(stem_wgrad_kernel<false>, dim3(nparts), dim3(256), 0, st, x, dy, scratch, H, W, halves,
                       StemBwd{nullptr, nullptr, nullptr, nullptr, nullptr});
  }
  const int groups = nparts >= 64 ? 16 : 1;
  const int per = (nparts + groups - 1) / groups;
  hipLaunchKernelGGL(stem_wgrad_reduce_kernel, dim3(PART / 1024, groups), dim3(256), 0, st, scratch, dw, nparts, per,
                     alpha);
  return (int)hipGetLastError();
}

extern "C" int dpe_stem_wgrad_launch(const uint16_t* x, const uint16_t* dy, float* dw, float* scratch, int N, int H, int W,
                                     float alpha, hipStream_t st) {
  return dpe_stem_wgrad_launch2(x, dy, dw, scratch, N, H, W, alpha, nullptr, nullptr, nullptr, nullptr, nullptr, st);
}
