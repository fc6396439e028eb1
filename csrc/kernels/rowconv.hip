// 3x3 / stride 1 / pad 1 convolution with 64 input and 64 output channels (ResNet-50 layer 1:
// the bottleneck conv2 forward and its stride-1 data grad, run as a forward conv of dy with the
// flipped filter), walking output rows.
//
// On the implicit-GEMM tiles these ran at ~500 TF (229 us forward at batch 512) with the L2 ~91 %
// busy: the im2col operand re-reads every input pixel once per tap (9x) and every tile re-reads the
// 72 KiB filter (profiles/pmc_conv3_r2.txt).  A tile-local halo in LDS (the filter in LDS too)
// measured slower: > 80 KiB per block left one block per CU with no overlap (docs/perf_notes.md).
// Here, as in the stem kernel (stem.hip):
//   * a block owns a contiguous range of the N*H output rows (one segment per image it touches; one
//     block per resident slot, rows_grid below); wave (mh, nh) holds output channels
//     32 nh .. +31 of the filter in VGPRs (18 K-steps x 2 fragments, 144 VGPRs) for the whole block;
//   * the three input rows an output row needs sit in a 4-slot LDS ring ([W + 2][64 ch], 16-B
//     chunks XOR-swizzled by pixel, zero pixels at both ends); each input row is read from HBM once
//     per block (register prefetch two rows ahead, written into the free slot after the MFMAs);
//   * the output row is staged in one of two LDS buffers and stored as 16-B chunks of contiguous
//     pixels; the epilogue is the shared one's EPI_BF16 (BN-forward sums of the stored output) or
//     EPI_BF16_BNB (sum dz, sum dz*(x - mean) with the ReLU recomputed from the pre-BN input and its
//     coefficients), accumulated per thread and reduced once per block ([2][64][blocks]).
// One barrier per output row.  Same K order as the implicit GEMM (tap-major, 32-channel halves), so
// the stored output is bitwise identical to it.
#include <algorithm>

#include "common.h"

namespace dpe {
namespace rowconv {

constexpr int CO = 64, KS = 18;           // channels, 32-wide K-steps (9 taps x 2 halves)
constexpr int SLOT_PX = 66;               // ring slot pixels: zero + <= 64 data + zero
constexpr int SLOT = SLOT_PX * 128;
constexpr int NSLOT = 4;
constexpr int OROW = 144;                 // staged output pixel stride (128 B + 16 pad)
constexpr int OBUF = 64 * OROW;
constexpr int LDS = NSLOT * SLOT + 2 * OBUF;
static_assert(LDS <= 163840 / 2, "two blocks per CU");

DPE_DEVICE u32x4 zero16() { return u32x4{0u, 0u, 0u, 0u}; }
// relu(v * scale + shift) of 8 channels: the BatchNorm+ReLU of the producing conv's output applied
// on load (same arithmetic as bn_apply, so the operand is bitwise the tensor bn_apply would store)
DPE_DEVICE u32x4 bnrelu8(const u32x4& v, const float* sc, const float* sh) {
  float f[8];
  unpack8(v, f);
#pragma unroll
  for (int e = 0; e < 8; ++e) f[e] = fmaxf(fmaf(f[e], sc[e], sh[e]), 0.f);
  return pack8(f);
}
DPE_DEVICE int pix_off(int sp, int chunk) { return sp * 128 + ((chunk ^ (sp & 7)) << 4); }

struct RowArgs {
  const uint16_t* x;      // [N][H][W][64] bf16
  const uint16_t* w;      // [64][3][3][64] bf16 (K-contiguous)
  uint16_t* y;            // [N][H][W][64] bf16
  float* stats;           // [2][64][blocks] or nullptr
  const uint16_t* st_x;   // BNB: pre-BN input [N][H][W][64]
  const float* st_coef;   // BNB: [4][64] scale, shift, mean, invstd
  int N, H, W;
  const float* in_coef;   // INBN: x is the pre-BN tensor; the operand is relu(x * in_coef[c] + in_coef[64 + c])
};

template <bool BNB, bool INBN = false>
__global__ __launch_bounds__(256, 2) void conv3x3_rows_kernel(RowArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[LDS];
  char* const ring = smem;
  char* const obuf = smem + NSLOT * SLOT;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int mh = wid & 1, nh = wid >> 1;  // pixels 32 mh .. +31, channels 32 nh .. +31
  const int H = p.H, W = p.W;
  const int blk = blockIdx.x;
  const int lm = lane & 15, kc = lane >> 4;

  // filter fragments: output channel 32 nh + 16 j + lm, K elements 32 ks + 8 kc .. +7
  bf16x8 wf[KS][2];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      wf[ks][j] = __builtin_bit_cast(bf16x8, *(const u32x4*)(p.w + (32 * nh + 16 * j + lm) * 576 + 32 * ks + 8 * kc));

  for (int i = tid; i < NSLOT * SLOT / 16; i += 256) *(u32x4*)(ring + i * 16) = zero16();

  // one input row = W pixels x 8 chunks (<= 512): thread t owns chunks t and t + 256
  int n = 0;
  int64_t img = 0;
  const int nch = W * 8;
  // every global load / store through a buffer resource, issued unconditionally (out-of-range rows and
  // chunks: an offset past the resource -> zeros / dropped), so the compiler's waits stay counted and the
  // row prefetch stays in flight (the host checks N H W 64 2 < 0xffffff00)
  const uint32_t xbytes = (uint32_t)((int64_t)p.N * H * W * CO * 2);
  const __amdgpu_buffer_rsrc_t xr = buf_rsrc(p.x, xbytes), yr = buf_rsrc(p.y, xbytes);
  const __amdgpu_buffer_rsrc_t sxr = buf_rsrc(p.st_x, BNB ? xbytes : 0u);
  auto load_row = [&](int ih, u32x4 (&v)[2]) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = tid + 256 * u;
      const bool ok = c < nch && (unsigned)ih < (unsigned)H;
      v[u] = __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? (uint32_t)((img + (int64_t)ih * W * 64 + c * 8) * 2) : BUF_OOB, 0, 0);
    }
  };
  // INBN: this thread's input channels are 8 (tid & 7) .. +7 for every row (256 % 8 == 0)
  float isc[INBN ? 8 : 1], ish[INBN ? 8 : 1];
  if constexpr (INBN) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      isc[e] = p.in_coef[(tid & 7) * 8 + e];
      ish[e] = p.in_coef[CO + (tid & 7) * 8 + e];
    }
  }
  auto write_row = [&](int ih, const u32x4 (&v)[2]) {  // input row ih -> slot (ih + 1) % 4, pixel iw + 1
    char* sl = ring + ((ih + 1 + 4 * NSLOT) % NSLOT) * SLOT;
    const bool inr = (unsigned)ih < (unsigned)H;  // padding rows stay zero (not relu(shift))
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = tid + 256 * u;
      if (c < nch) {
        u32x4 val = v[u];
        if constexpr (INBN) {
          if (inr) val = bnrelu8(val, isc, ish);
        }
        *(u32x4*)(sl + pix_off((c >> 3) + 1, c & 7)) = val;
      }
    }
  };
  // store-phase channel chunk of this thread and its BN coefficients
  const int sc = tid & 7;
  float s[8], ss[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    s[e] = 0.f;
    ss[e] = 0.f;
  }
  // BNB: [scale | shift | mean] x 64 channels in LDS, read per stored chunk (24 registers held across
  // the row loop spilled beside the filter fragments and the two prefetch sets)
  __shared__ __attribute__((aligned(16))) float bcs[BNB ? 3 * CO : 4];
  if constexpr (BNB)
    if (tid < 3 * CO) bcs[tid] = p.st_coef[tid];
  // this wave's pixel fragments: 32 mh + 16 i + lm (rows >= W compute on zero pixels, never stored)
  const int nfr = min(2, max(0, (W - 32 * mh + 15) / 16));

  // The block owns output rows [r0, r1) of the N*H rows (image-major), one segment per image it
  // touches; the ring's zero pixels persist, every data pixel of a slot is rewritten per row.
  const int64_t T = (int64_t)p.N * H;
  int64_t r0 = T * blk / gridDim.x;
  const int64_t r1 = T * (blk + 1) / gridDim.x;
  for (; r0 < r1;) {
  n = (int)(r0 / H);
  img = (int64_t)n * H * W * 64;
  const int oh_beg = (int)(r0 - (int64_t)n * H);
  const int oh_end = (int)min<int64_t>(H, oh_beg + (r1 - r0));
  r0 += oh_end - oh_beg;
  __syncthreads();  // the previous segment's last stores have read the output buffers
  {
    u32x4 t0[2], t1[2], t2[2];
    load_row(oh_beg - 1, t0);
    load_row(oh_beg, t1);
    load_row(oh_beg + 1, t2);
    write_row(oh_beg - 1, t0);
    write_row(oh_beg, t1);
    write_row(oh_beg + 1, t2);
  }
  u32x4 pf0[2], pf1[2];  // input rows oh + 2, oh + 3 (two sets: a prefetch is first used two rows later)
  load_row(oh_beg + 2, pf0);
  load_row(oh_beg + 3, pf1);
  __syncthreads();

  auto row = [&](const int oh, u32x4 (&pfA)[2]) {
    // the store phase's pre-BN input (BNB) first: its latency overlaps the MFMAs, and it is older than
    // this row's prefetch, so waiting for it leaves the prefetch in flight
    const int64_t rowoff = ((int64_t)n * H + oh) * W * CO;
    u32x4 xv[2];
    uint32_t bo[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int px = (tid >> 3) + 32 * k;
      bo[k] = px < W ? (uint32_t)((rowoff + px * CO + sc * 8) * 2) : BUF_OOB;
      if constexpr (BNB) xv[k] = __builtin_amdgcn_raw_buffer_load_b128(sxr, bo[k], 0, 0);
    }
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // K-step ks: tap t = ks / 2 (r = t / 3, s = t % 3), channel half ks & 1; input row
    // oh - 1 + r in slot (oh + r) % 4, pixel ow + s
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int t = ks >> 1, r = t / 3, s_ = t - 3 * (t / 3), hf = ks & 1;
      const char* sl = ring + ((oh + r) % NSLOT) * SLOT;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if (i < nfr) {
          const int sp = 32 * mh + 16 * i + lm + s_;
          const bf16x8 af = __builtin_bit_cast(bf16x8, *(const u32x4*)(sl + pix_off(sp, hf * 4 + kc)));
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ks][j], af, acc[i][j], 0, 0, 0);
        }
      }
    }
    // input row oh + 2 into the slot of row oh - 2 (free); prefetch row oh + 4 into the same registers
    write_row(oh + 2, pfA);
    load_row(oh + 4, pfA);
    // stage: acc[i][j][e] = pixel 32 mh + 16 i + lm, channel 32 nh + 16 j + 4 kc + e
    char* ob = obuf + (oh & 1) * OBUF;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (i < nfr) {
        const int ow = 32 * mh + 16 * i + lm;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          u32x2 pk;
          pk[0] = pack_bf2(acc[i][j][0], acc[i][j][1]);
          pk[1] = pack_bf2(acc[i][j][2], acc[i][j][3]);
          *(u32x2*)(ob + ow * OROW + (32 * nh + 16 * j + 4 * kc) * 2) = pk;
        }
      }
    }
    lds_barrier();
    // store: thread t -> chunk t & 7 of pixels t / 8 and t / 8 + 32
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int px = (tid >> 3) + 32 * k;
      const u32x4 v = *(const u32x4*)(ob + px * OROW + sc * 16);
      __builtin_amdgcn_raw_buffer_store_b128(v, yr, bo[k], 0, 0);
      if (p.stats && px < W) {
        float f[8];
        unpack8(v, f);
        if constexpr (BNB) {  // (sum dz, sum dz * (x - mean)), dz = f * relu'(x * scale + shift)
          float xf[8];
          unpack8(xv[k], xf);
#pragma unroll
          for (int h4 = 0; h4 < 2; ++h4) {
            const f32x4 k0 = *(const f32x4*)(bcs + sc * 8 + 4 * h4), k1 = *(const f32x4*)(bcs + CO + sc * 8 + 4 * h4);
            const f32x4 k2 = *(const f32x4*)(bcs + 2 * CO + sc * 8 + 4 * h4);
#pragma unroll
            for (int e4 = 0; e4 < 4; ++e4) {
              const int e = 4 * h4 + e4;
              const float dz = fmaf(xf[e], k0[e4], k1[e4]) > 0.f ? f[e] : 0.f;
              s[e] += dz;
              ss[e] += dz * (xf[e] - k2[e4]);
            }
          }
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) { s[e] += f[e]; ss[e] = fmaf(f[e], f[e], ss[e]); }
        }
      }
    }
  };
  // the loop's only backedge follows the second row (a conditional second row before a shared latch
  // merged two paths with different load counts: the compiler's waits became vmcnt(0)); oh_beg < oh_end
  for (int oh = oh_beg;; oh += 2) {
    row(oh, pf0);
    if (oh + 1 >= oh_end) break;
    row(oh + 1, pf1);
    if (oh + 2 >= oh_end) break;
  }
  }  // segments
  if (p.stats) {
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
      p.stats[(int64_t)tid * nb + blk] = a;
      p.stats[(int64_t)(CO + tid) * nb + blk] = b;
    }
  }
}


// ------------------------------------------------------------------ weight grad
// dW[co][r][s][ci] += alpha * sum_{n, oh, ow} dy[n, oh, ow, co] * x[n, oh + r - 1, ow + s - 1, ci]
// for the same 64 -> 64 3x3 / stride-1 / pad-1 layer.  As a GEMM this is M = 64, N = 576 (9 taps x
// 64), K = the 1.6 M output pixels at batch 512; the im2col weight-grad tile (igemm_wgrad_dma,
// 64x128) reads every activation once per tap through L2 and ran at ~320 TF (365 us).  Here a
// block walks a contiguous range of output rows (a slot's share of the N*H rows) and keeps the
// whole 64 x 576 gradient of its rows in registers: wave w owns input channels 16 w .. +15 for all 9 taps and all 64 output channels
// (4 x 9 accumulator tiles, 144 VGPRs).  Per output row the dy row (K = pixels, M = co) and the three
// x rows (K = pixels shifted by the tap column, N = ci) are LDS images read with the transposing
// ds_read_b64_tr_b16, so each input row is read from HBM once per block.  The block's gradient is
// stored as one coalesced fp32 partial ([blocks][64 x 576], in accumulator order) and a second
// kernel sums the partials into dW in a fixed order (16 group sums, then their sum).
namespace wg {
constexpr int XSLOT = 66 * 128;              // x row: zero pixel, W (<= 64) pixels, zero pixels
constexpr int DSLOT = 64 * 128;              // dy row: W pixels, zero rows up to 64
constexpr int LDS = NSLOT * XSLOT + 2 * DSLOT;
constexpr int PART = 64 * 576;               // floats of one block's partial

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// [pixel rows][64 ch] image, 16-B chunks XOR-swizzled by bits 1 and 3 of the row: the transposing
// reads below (rows 8g+q and 8g+q+4 of any 32-row window, shifted by 0-2 rows) are conflict-free
DPE_DEVICE int img_off(int k, int chunk) {
  const int h = (((k >> 1) & 1) | (((k >> 3) & 1) << 1)) << 1;
  return k * 128 + ((chunk ^ h) << 4);
}
// MFMA operand fragment: channels c0 .. c0 + 15 (lane & 15), K = image rows row0 + 8 (lane >> 4) .. +7
DPE_DEVICE bf16x8 trfrag(const char* img, int row0, int c0) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
  const int k1 = row0 + 8 * g + q;
  const int mc = (c0 >> 3) + (pp >> 1), sub = (pp & 1) * 8;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + img_off(k1, mc) + sub));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + img_off(k1 + 4, mc) + sub));
  s16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return __builtin_bit_cast(bf16x8, r);
}

template <bool INBN>
__global__ __launch_bounds__(256, 2) void wgrad3x3_rows_kernel(const uint16_t* __restrict__ x,
                                                               const uint16_t* __restrict__ dy,
                                                               float* __restrict__ part, int N, int H, int W,
                                                               const float* __restrict__ in_coef) {
  __shared__ __attribute__((aligned(16))) char smem[LDS];
  char* const ring = smem;                     // x rows: input row ih in slot (ih + 1) % 4
  char* const dbuf = smem + NSLOT * XSLOT;     // dy rows: output row oh in slot oh & 1
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // input channels 16 w .. +15
  int64_t img = 0;
  const int nch = W * 8;

  for (int i = tid; i < LDS / 16; i += 256) *(u32x4*)(smem + i * 16) = zero16();

  // buffer loads issued unconditionally (see conv3x3_rows_kernel)
  const uint32_t tbytes = (uint32_t)((int64_t)N * H * W * 64 * 2);
  const __amdgpu_buffer_rsrc_t xr = buf_rsrc(x, tbytes), dr = buf_rsrc(dy, tbytes);
  auto load = [&](const uint16_t* src, int row, u32x4 (&v)[2]) {
    const __amdgpu_buffer_rsrc_t r = src == x ? xr : dr;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = tid + 256 * u;
      const bool ok = c < nch && (unsigned)row < (unsigned)H;
      v[u] = __builtin_amdgcn_raw_buffer_load_b128(r, ok ? (uint32_t)((img + (int64_t)row * W * 64 + c * 8) * 2) : BUF_OOB, 0, 0);
    }
  };
  auto put = [&](char* sl, int px0, const u32x4 (&v)[2]) {  // chunk c -> pixel row px0 + c / 8
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = tid + 256 * u;
      if (c < nch) *(u32x4*)(sl + img_off(px0 + (c >> 3), c & 7)) = v[u];
    }
  };
  auto xslot = [&](int ih) { return ring + ((ih + 1 + NSLOT) % NSLOT) * XSLOT; };
  // INBN: x rows are the pre-BN tensor; this thread's channels are 8 (tid & 7) .. +7 for every chunk
  float isc[INBN ? 8 : 1], ish[INBN ? 8 : 1];
  if constexpr (INBN) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      isc[e] = in_coef[(tid & 7) * 8 + e];
      ish[e] = in_coef[64 + (tid & 7) * 8 + e];
    }
  }
  auto putx = [&](int ih, u32x4 (&v)[2]) {
    if constexpr (INBN) {
      if ((unsigned)ih < (unsigned)H) {  // padding rows stay zero (not relu(shift))
#pragma unroll
        for (int u = 0; u < 2; ++u) v[u] = bnrelu8(v[u], isc, ish);
      }
    }
    put(xslot(ih), 1, v);
  };
  f32x4 acc[4][9];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nks = W > 32 ? 2 : 1;  // 32-pixel K-steps per row (pixels >= W are zero rows of dy)
  u32x4 px0[2], px1[2], pd0[2], pd1[2];  // prefetch: x rows oh + 2, oh + 3; dy rows oh + 1, oh + 2

  // one output row; pxA / pdA hold x row oh + 2 / dy row oh + 1 and are refilled in place with rows
  // oh + 4 / oh + 3 (two rows per loop trip with two buffer sets: a prefetch is first waited on two
  // rows after it was issued)
  auto step = [&](int oh, u32x4 (&pxA)[2], u32x4 (&pdA)[2]) {
    const char* ds = dbuf + (oh & 1) * DSLOT;
    for (int ks = 0; ks < nks; ++ks) {
      bf16x8 a[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) a[m] = trfrag(ds, 32 * ks, 16 * m);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int r = t / 3, sc = t % 3;
        // x row oh - 1 + r (slot (oh + r) % 4); output pixel ow reads slot pixel ow + sc
        const bf16x8 b = trfrag(ring + ((oh + r) % NSLOT) * XSLOT, 32 * ks + sc, 16 * w);
#pragma unroll
        for (int m = 0; m < 4; ++m) acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a[m], acc[m][t], 0, 0, 0);
      }
    }
    // x row oh + 2 into the slot of row oh - 2, dy row oh + 1 into the slot of row oh - 1 (both free)
    putx(oh + 2, pxA);
    put(dbuf + ((oh + 1) & 1) * DSLOT, 0, pdA);
    load(x, oh + 4, pxA);
    load(dy, oh + 3, pdA);
    lds_barrier();  // (LDS only: __syncthreads would drain the prefetch just issued)
  };
  // The block owns output rows [r0, r1) of the N*H rows (image-major), one segment per image it
  // touches (dy rows outside the segment are never stepped on, so no row is counted twice).
  const int64_t T = (int64_t)N * H;
  int64_t r0 = T * blockIdx.x / gridDim.x;
  const int64_t r1 = T * (blockIdx.x + 1) / gridDim.x;
  while (r0 < r1) {
    const int n = (int)(r0 / H);
    img = (int64_t)n * H * W * 64;
    const int oh_beg = (int)(r0 - (int64_t)n * H);
    const int oh_end = (int)min<int64_t>(H, oh_beg + (r1 - r0));
    r0 += oh_end - oh_beg;
    __syncthreads();  // every wave is done with the previous segment's slots
    {
      u32x4 t0[2], t1[2], t2[2];
      load(x, oh_beg - 1, t0);
      load(x, oh_beg, t1);
      load(dy, oh_beg, t2);
      putx(oh_beg - 1, t0);
      putx(oh_beg, t1);
      put(dbuf + (oh_beg & 1) * DSLOT, 0, t2);
      load(x, oh_beg + 1, t0);
      putx(oh_beg + 1, t0);
    }
    load(x, oh_beg + 2, px0);
    load(x, oh_beg + 3, px1);
    load(dy, oh_beg + 1, pd0);
    load(dy, oh_beg + 2, pd1);
    __syncthreads();
    for (int oh = oh_beg;; oh += 2) {  // (one backedge, after the second step: see conv3x3_rows_kernel)
      step(oh, px0, pd0);
      if (oh + 1 >= oh_end) break;
      step(oh + 1, px1, pd1);
      if (oh + 2 >= oh_end) break;
    }
  }
  // acc[m][t][e]: co = 16 m + (lane & 15), ci = 16 w + 4 (lane >> 4) + e, tap t
  float* pb = part + (int64_t)blockIdx.x * PART;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int t = 0; t < 9; ++t) *(f32x4*)(pb + (((m * 9 + t) * 4 + w) * 64 + lane) * 4) = acc[m][t];
}

// dW [64][3][3][64] += alpha * sum of the block partials, in a fixed order (bitwise reproducible):
// stage 1, grid (PART / 1024, groups): group g sums partials [g * per, (g + 1) * per) into gsum[g]
// (or, with one group, straight into dW); stage 2, grid PART / 1024: dW += alpha * sum_g gsum[g].
// One thread per float4 of accumulator order; every dW element has one writer.
DPE_DEVICE float* dw_elem(float* dw, int q) {
  const int lane = q & 63, w = (q >> 6) & 3, mt = q >> 8, t = mt % 9, m = mt / 9;
  return dw + (16 * m + (lane & 15)) * 576 + t * 64 + 16 * w + 4 * (lane >> 4);
}
__global__ __launch_bounds__(256) void wgrad3x3_rows_reduce_kernel(const float* __restrict__ part, float* __restrict__ gsum,
                                                                   float* __restrict__ dw, int nparts, int per, float alpha) {
  const int q = blockIdx.x * 256 + threadIdx.x;  // float4 index, < PART / 4
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
  if (gridDim.y > 1) {
    ((f32x4*)gsum)[(int64_t)blockIdx.y * (PART / 4) + q] = s0;
    return;
  }
  float* d = dw_elem(dw, q);
#pragma unroll
  for (int e = 0; e < 4; ++e) d[e] += alpha * s0[e];
}
__global__ __launch_bounds__(256) void wgrad3x3_rows_sum_kernel(const float* __restrict__ gsum, float* __restrict__ dw,
                                                                int groups, float alpha) {
  const int q = blockIdx.x * 256 + threadIdx.x;
  f32x4 s = ((const f32x4*)gsum)[q];
  for (int g = 1; g < groups; ++g) s += ((const f32x4*)gsum)[(int64_t)g * (PART / 4) + q];
  float* d = dw_elem(dw, q);
#pragma unroll
  for (int e = 0; e < 4; ++e) d[e] += alpha * s[e];
}
}  // namespace wg
}  // namespace rowconv
}  // namespace dpe

extern "C" int dpe_cu_reserve();  // comm.cpp: slots left to in-flight collectives

namespace {
int rows_slots() {  // resident blocks of the row-walking kernels (2 per CU), minus the CU budget
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
      (void)hipGetLastError();
      n = 256;
    }
    return n > 0 ? n : 256;
  }();
  return max(2, 2 * ncu - dpe_cu_reserve());
}
// One block per resident slot, each owning a contiguous range of the N*H output rows (>= 16 rows):
// a single wave of blocks -- a fixed N*2 grid went from exactly 2 waves to 2 + a sliver when RCCL
// channel blocks held 16 slots (x1.4-1.6, profiles/cu_hog_probe_r3.txt in git history).  While the budget is in force,
// two rounds of half-size blocks instead: a foreign workgroup that fits beside a block still slows its
// CU, and with one round the slowest CU's block set the launch's time (x1.7-1.8 next to 16 VALU-bound
// RCCL-sized workgroups, profiles/cu_hog_probe_r4.txt); with two, the dispatcher hands it fewer.
int rows_grid(int N, int H) {
  const int slots = rows_slots() * (dpe_cu_reserve() > 0 ? 2 : 1);
  return (int)std::max<int64_t>(1, std::min<int64_t>(slots, (int64_t)N * H / 16));
}
}  // namespace

// Blocks of the launch for an [N, H, W, 64] input (0: outside the kernel's envelope).  Depends on the
// CU budget in force: compute it once per launch and pass it to dpe_conv3x3_rows_launch.
extern "C" int dpe_conv3x3_rows_blocks(int N, int H, int W) {
  if (N <= 0 || H < 2 || W < 1 || W > 64 || (int64_t)N * H * W * 128 >= 0xffffff00ll) return 0;
  return rows_grid(N, H);
}

// y = conv3x3(x, w) (stride 1, pad 1, 64 -> 64 channels) on nb blocks (dpe_conv3x3_rows_blocks); bnb:
// stats ([2][64][nb]) are the BN-backward partials of the BN with pre-BN input st_x and coefficients
// st_coef, else the BN-forward sums of y.  in_coef (forward only, not with bnb): x is the pre-BN
// tensor of a BatchNorm+ReLU, applied on load.
extern "C" int dpe_conv3x3_rows_launch(const uint16_t* x, const uint16_t* w, uint16_t* y, float* stats, const uint16_t* st_x,
                                       const float* st_coef, int N, int H, int W, int nb, int bnb, const float* in_coef,
                                       hipStream_t st) {
  if (nb <= 0 || N <= 0 || H < 2 || W < 1 || W > 64 || (bnb && (!stats || !st_x || !st_coef)) || (bnb && in_coef) ||
      (int64_t)N * H * W * 128 >= 0xffffff00ll)
    return -1;
  dpe::rowconv::RowArgs a{x, w, y, stats, st_x, st_coef, N, H, W, in_coef};
  if (bnb) hipLaunchKernelGGL(dpe::rowconv::conv3x3_rows_kernel<true>, dim3(nb), dim3(256), 0, st, a);
  else if (in_coef) hipLaunchKernelGGL((dpe::rowconv::conv3x3_rows_kernel<false, true>), dim3(nb), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(dpe::rowconv::conv3x3_rows_kernel<false>, dim3(nb), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

// Blocks of the weight-grad launch (0: outside the envelope); as dpe_conv3x3_rows_blocks.
extern "C" int dpe_wgrad3x3_rows_blocks(int N, int H, int W) {
  if (N <= 0 || H < 1 || W < 1 || W > 64 || (int64_t)N * H * W * 128 >= 0xffffff00ll) return 0;
  return rows_grid(N, H);
}
namespace {
int rows_groups(int nb) { return nb >= 64 ? 16 : 1; }
}  // namespace

// Scratch floats of the weight-grad launch on nb blocks: the block partials + the group sums.
extern "C" int64_t dpe_wgrad3x3_rows_scratch(int nb) {
  if (nb <= 0) return 0;
  const int groups = rows_groups(nb);
  return (int64_t)(nb + (groups > 1 ? groups : 0)) * dpe::rowconv::wg::PART;
}

// dw (+)= alpha * dW of conv3x3(x) w.r.t. its filter, given dy (64 -> 64, stride 1, pad 1), on nb
// blocks (dpe_wgrad3x3_rows_blocks).  in_coef: x is the pre-BN tensor of a BatchNorm+ReLU ([scale |
// shift] of 64 channels), applied on load.
extern "C" int dpe_wgrad3x3_rows_launch(const uint16_t* x, const uint16_t* dy, float* dw, float* scratch, int N, int H,
                                        int W, int nb, float alpha, const float* in_coef, hipStream_t st) {
  if (nb <= 0 || N <= 0 || H < 1 || W < 1 || W > 64 || !scratch || (int64_t)N * H * W * 128 >= 0xffffff00ll) return -1;
  using namespace dpe::rowconv::wg;
  if (in_coef) hipLaunchKernelGGL(wgrad3x3_rows_kernel<true>, dim3(nb), dim3(256), 0, st, x, dy, scratch, N, H, W, in_coef);
  else hipLaunchKernelGGL(wgrad3x3_rows_kernel<false>, dim3(nb), dim3(256), 0, st, x, dy, scratch, N, H, W, in_coef);
  const int groups = rows_groups(nb);
  const int per = (nb + groups - 1) / groups;
  float* gsum = scratch + (int64_t)nb * PART;
  hipLaunchKernelGGL(wgrad3x3_rows_reduce_kernel, dim3(PART / 1024, groups), dim3(256), 0, st, scratch, gsum, dw, nb, per,
                     alpha);
  if (groups > 1) hipLaunchKernelGGL(wgrad3x3_rows_sum_kernel, dim3(PART / 1024), dim3(256), 0, st, gsum, dw, groups, alpha);
  return (int)hipGetLastError();
}
